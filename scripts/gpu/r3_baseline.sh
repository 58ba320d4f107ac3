#!/bin/bash
# GPU-box job (round 3): where does the SPADE step go now?
#   bench   — headline number (graph replay, 20 timed steps)
#   ops     — torch.profiler self device time per aten op / autograd Function with the Python
#             call site (eager step), to attribute the elementwise glue
#   trace   — rocprofv3 kernel stats of the steady state (after the profile marker)
# Each GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r3
mkdir -p "$OUT"
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "[r3] $name rc=$rc"; tail -4 "$OUT/$name.out"
  if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.err"; exit $rc; fi
}
if [ -z "$SKIP_BENCH" ]; then
  run bench 600 python bench.py ${BENCH_ARGS:---steps 20 --warmup 6}
fi
if [ -n "$OPS" ]; then
  run ops 600 python bench.py --steps 1 --warmup 3 --no-graph --op-profile --op-stack
fi
if [ -n "$CONVLOG" ]; then
  run convlog 600 python bench.py --steps 1 --warmup 3 --conv-log
fi
if [ -n "$TRACE" ]; then
  cd /tmp && export TMPDIR=/tmp
  rm -rf /tmp/iamd_prof
  run trace 900 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/iamd_prof -o bench -- \
    python3 "$ROOT/bench.py" ${TRACE_ARGS:---steps 3 --warmup 4 --verbose}
  cd "$ROOT"
  python3 scripts/gpu/summarize_kernels.py /tmp/iamd_prof > "$OUT/top_kernels.txt" || true
  head -50 "$OUT/top_kernels.txt"
fi
exit 0
