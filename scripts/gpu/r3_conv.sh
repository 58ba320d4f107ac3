#!/bin/bash
# GPU-box job (round 3): conv kernel iteration — GPU conv/wgrad tests, k11 A/B probe, k10 probe
# (v1 forced vs auto routing) on the SPADE-step shapes; optional extra probe / bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r3c
mkdir -p "$OUT"
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "[r3c] $name rc=$rc"; tail -${TAILN:-20} "$OUT/$name.out"
  if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.err"; exit $rc; fi
}
run tests 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "${TESTS:-conv or wgrad}"
[ -n "$NOWPROBE" ] || run wprobe 600 python scripts/probe/wgrad_v2_probe.py
[ -n "$NOCPROBE" ] || run cprobe 600 python scripts/probe/conv_v2_probe.py ${CVERS:-1,0}
if [ -n "$BENCH" ]; then
  run bench 600 python bench.py --steps 20 --warmup 6
fi
exit 0
