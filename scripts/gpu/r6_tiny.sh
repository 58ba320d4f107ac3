#!/bin/bash
# GPU-box job (round 6): finer split-K for tiny conv grids — conv tests, then SPADE bench A/B
# (IMAGINAIRE_AMD_SPLITK_TINY=1 default vs 0), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6tiny; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_conv_rw_gpu.py -x -q -k "conv" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; echo "[tiny] tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for arm in on off on2 off2; do
  v=1; [[ $arm == off* ]] && v=0
  IMAGINAIRE_AMD_SPLITK_TINY=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 6 > $OUT/bench_$arm.log 2>&1
  rc=$?; echo "[tiny] $arm rc=$rc: $(grep '"metric"' $OUT/bench_$arm.log | cut -c60-140)"; [ $rc -eq 0 ] || exit $rc
done
