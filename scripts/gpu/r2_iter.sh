#!/bin/bash
# GPU-box job (round 2 iteration loop): GPU tests (all, or $TESTS), the 1-GPU bench, and the
# per-conv timing log of one eager step. Each GPU step has its own time limit; stop at the first
# fault / abort / timeout (test failures, rc 1, continue so the bench still runs). Test progress
# goes straight to gpurun_out/ (-v, unbuffered) so a slow test never looks like a hang.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/iter
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/iter/$name.out" 2> "gpurun_out/iter/$name.err"
  local rc=$?
  echo "[iter] $name rc=$rc"; tail -4 "gpurun_out/iter/$name.out"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 "gpurun_out/iter/$name.err"; exit $rc; fi
}
if [ -z "$SKIP_TESTS" ]; then
  run tests 900 python -u -m pytest ${TESTS:-tests} -m gpu -v -rf --timeout 170 --timeout-method thread ${KFILTER:+-k "$KFILTER"}
fi
[ -n "$DIST" ] && run dist 500 python -u -m pytest tests/test_distributed_gpu.py -m gpu -v -s -rf --timeout 170 --timeout-method thread
[ -n "$PROBE" ] && run probe 300 python -u $PROBE
[ -z "$SKIP_BENCH" ] && run bench 600 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5}
[ -n "$CONVLOG" ] && run convlog 600 python bench.py --steps 1 --warmup 3 --conv-log
[ -n "$OPSITES" ] && run opsites 600 python scripts/probe/op_sites.py
exit 0
