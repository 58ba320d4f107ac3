#!/bin/bash
# GPU-box job (round 6): same-box A/B of bench.py (SPADE) and the graphed recipes, round-6 conv
# routing off vs on.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6ab
mkdir -p "$OUT"
for arm in off on; do
  if [ $arm = off ]; then export IMAGINAIRE_AMD_TAPPACK=0 IMAGINAIRE_AMD_CONV_RW=0; else unset IMAGINAIRE_AMD_TAPPACK IMAGINAIRE_AMD_CONV_RW; fi
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 6 > "$OUT/bench_$arm.log" 2>&1
  rc=$?; echo "[ab2] bench $arm rc=$rc: $(tail -1 $OUT/bench_$arm.log | cut -c1-160)"; [ $rc -eq 0 ] || exit $rc
done
bash scripts/gpu/r6_ab.sh
