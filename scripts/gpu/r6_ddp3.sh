#!/bin/bash
# GPU-box job (round 6): DDP / SN zero-copy tests, then plain vs forced one-rank SPADE bench,
# alternating (plain, forced, plain, forced) to average out box drift and autotune choices.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6ddp3; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py tests/test_sn_fused_gpu.py -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/tests.log" 2>&1
rc=$?; echo "[ddp3] tests rc=$rc"; tail -2 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
for arm in plain forced plain2 forced2; do
  extra=""; [[ $arm == forced* ]] && extra="--force-dist"
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 6 $extra > "$OUT/bench_${arm}.log" 2>&1
  rc=$?; echo "[ddp3] bench $arm rc=$rc: $(grep '"metric"' $OUT/bench_${arm}.log | cut -c60-140)"
  [ $rc -eq 0 ] || exit $rc
done
