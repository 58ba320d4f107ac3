#!/bin/bash
# GPU-box job (round 6): sync-BN / DDP tests after the native sync-BN merge, then the SPADE bench
# plain vs forced one-rank distributed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6ddp2
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > "$OUT/tests.log" 2>&1
rc=$?; echo "[ddp2] tests rc=$rc"; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "norm or bn" --timeout 200 \
  --timeout-method thread -p no:cacheprovider > "$OUT/norm_tests.log" 2>&1
rc=$?; echo "[ddp2] norm tests rc=$rc"; tail -3 "$OUT/norm_tests.log"; [ $rc -eq 0 ] || exit $rc
for arm in plain forced; do
  extra=""; [ $arm = forced ] && extra="--force-dist"
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 6 $extra > "$OUT/bench_${arm}.log" 2>&1
  rc=$?; echo "[ddp2] bench $arm rc=$rc: $(grep '"metric"' $OUT/bench_${arm}.log | cut -c60-130)"
  [ $rc -eq 0 ] || exit $rc
done
