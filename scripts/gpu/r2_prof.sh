#!/bin/bash
# GPU-box job: attribution profiles of the SPADE step.
#   convlog — time / TF/s of every conv kernel call of one eager step, per shape;
#   ops    — torch.profiler self device time of every aten op grouped by Python call site
#            (eager step: graph replay hides the ops);
#   trace  — rocprofv3 kernel trace of the steady state (grid sizes identify conv shapes),
#            compressed into gpurun_out/prof/.
# Each GPU step has its own time limit; the script stops at the first fault / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
mkdir -p gpurun_out/prof
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/prof/$name.out" 2> "$ROOT/gpurun_out/prof/$name.err"
  local rc=$?
  echo "[prof] $name rc=$rc"; tail -3 "$ROOT/gpurun_out/prof/$name.out"
  if [ $rc -ne 0 ]; then tail -20 "$ROOT/gpurun_out/prof/$name.err"; exit $rc; fi
}
if [ -n "$CONVLOG" ]; then
  run convlog 600 python bench.py --steps 1 --warmup 3 --conv-log
fi
if [ -n "$OPS" ]; then
  run ops 600 python bench.py --steps 1 --warmup 3 --no-graph --op-profile --op-stack
  run ops_shapes 600 python bench.py --steps 1 --warmup 3 --no-graph --op-profile
fi
if [ -n "$TRACE" ]; then
  cd /tmp && export TMPDIR=/tmp
  rm -rf /tmp/iamd_trace
  run trace 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/iamd_trace -o run -- \
    python3 "$ROOT/bench.py" ${TRACE_ARGS:---steps 2 --warmup 3 --verbose}
  cd "$ROOT"
  f=$(find /tmp/iamd_trace -name '*kernel_trace.csv' | head -1)
  [ -n "$f" ] && gzip -c "$f" > gpurun_out/prof/kernel_trace.csv.gz
  ls -la gpurun_out/prof/
fi
exit 0
