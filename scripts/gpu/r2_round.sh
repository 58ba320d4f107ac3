#!/bin/bash
# GPU-box job (round 2): kernel tests -> smoke -> 1-GPU bench -> 2-rank share-GPU gloo
# rehearsal of the bench launcher -> rocprofv3 kernel stats. Every GPU step has its own
# time limit; the script stops at the first fault / abort / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
mkdir -p gpurun_out/prof
step() {  # name, timeout, cmd...  (rc 1 = test failures: keep going; anything else: stop)
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[r2] $name rc=$rc"
  tail -6 "$ROOT/gpurun_out/$name.log"
  if [ $rc -ne 0 ] && { [ $rc -ne 1 ] || [ -n "$STRICT" ]; }; then exit $rc; fi
}
if [ -z "$SKIP_TESTS" ]; then
  step pytest_gpu 900 python -u -m pytest ${PYTEST_ARGS:-tests -m gpu} -x -q --timeout 300 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ -z "$SKIP_BENCH" ]; then
  step bench1 900 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5}
fi
if [ -n "$SHARE2" ]; then
  step bench2_share 900 python bench.py --gpus 2 --backend gloo --share-gpu --steps 2 --warmup 1
fi
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  rm -rf /tmp/iamd_prof
  step rocprof 900 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/iamd_prof -o bench -- \
    python3 "$ROOT/bench.py" ${PROF_ARGS:---steps 3 --warmup 3 --verbose}
  cd "$ROOT"
  find /tmp/iamd_prof -name '*stats*.csv' -exec cp {} gpurun_out/prof/ \;
  python3 scripts/gpu/summarize_kernels.py /tmp/iamd_prof > gpurun_out/prof/top_kernels.txt || true
  head -40 gpurun_out/prof/top_kernels.txt
fi
