#!/bin/bash
# GPU-box job (round 3): targeted GPU tests (TESTS=<pytest -k expr>) + optional conv log.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r3
mkdir -p "$OUT"
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "[r3] $name rc=$rc"; tail -6 "$OUT/$name.out"
  if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.err"; exit $rc; fi
}
if [ -n "$TESTS" ]; then
  run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "$TESTS"
fi
if [ -n "$ALLTESTS" ]; then
  run alltests 1100 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
fi
if [ -n "$CONVLOG" ]; then
  run convlog 600 python bench.py --steps 1 --warmup 3 --conv-log
fi
if [ -n "$BENCH" ]; then
  run bench 600 python bench.py ${BENCH_ARGS:---steps 20 --warmup 6}
fi
if [ -n "$PROBE" ]; then
  run probe 600 python $PROBE
fi
exit 0
