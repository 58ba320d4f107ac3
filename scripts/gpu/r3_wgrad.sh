#!/bin/bash
# GPU-box job (round 3): k11 v2 weight-gradient kernel — GPU tests, A/B probe vs the round-2
# kernels, correlation fwd/bwd probe, PMC passes (v2 and old) on the SPADE gamma|beta wgrad.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r3w
mkdir -p "$OUT"
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "[r3w] $name rc=$rc"; tail -${TAILN:-14} "$OUT/$name.out"
  if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.err"; exit $rc; fi
}
run tests 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "wgrad"
run wprobe 600 python scripts/probe/wgrad_v2_probe.py
run corr 600 python scripts/probe/corr_bwd_probe.py
if [ -n "$PMC" ]; then
  SHAPES="wgrad 4 128 1024 128 256 5" bash scripts/gpu/r3_pmc.sh > "$OUT/pmc_v2.out" 2>&1 || exit 1
  mkdir -p "$OUT/pmc_v2" && cp -r gpurun_out/r3pmc/* "$OUT/pmc_v2/"
  IMAGINAIRE_AMD_WGRAD_V2=0 SHAPES="wgrad 4 128 1024 128 256 5" bash scripts/gpu/r3_pmc.sh > "$OUT/pmc_old.out" 2>&1 || exit 1
  cat "$OUT/pmc_v2.out" "$OUT/pmc_old.out" | grep -v "^\[pmc\]"
fi
exit 0
