#!/bin/bash
# GPU-box job: kernel tests for the conv paths, bench, op-site attribution of the SPADE step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/tap
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -rf --timeout 120 \
  --timeout-method thread -k "${KFILTER:-tapsplit or conv2d_mfma}" > gpurun_out/tap/tests.out 2>&1
rc=$?; echo "[tap] tests rc=$rc"; tail -5 gpurun_out/tap/tests.out
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/tap/bench.out 2> gpurun_out/tap/bench.err
  rc=$?; echo "[tap] bench rc=$rc"; tail -1 gpurun_out/tap/bench.out
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$CONVLOG" ]; then
  timeout -k 10 600 python bench.py --steps 1 --warmup 3 --conv-log > gpurun_out/tap/convlog.out 2> gpurun_out/tap/convlog.err
  rc=$?; echo "[tap] convlog rc=$rc"; head -12 gpurun_out/tap/convlog.out
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$SITES" ]; then
  timeout -k 10 500 python scripts/probe/op_sites.py > gpurun_out/tap/sites.out 2> gpurun_out/tap/sites.err
  rc=$?; echo "[tap] sites rc=$rc"; head -5 gpurun_out/tap/sites.out
fi
exit $rc
