#!/bin/bash
# GPU-box job: conv routing tests, recipe runs with conv logs, SPADE bench (regression check).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "conv2d_mfma or conv_transpose or predict_flow" > gpurun_out/vc_test.log 2>&1
rc=$?; echo "[vc] tests rc=$rc"; tail -3 gpurun_out/vc_test.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu/recipes_round.sh || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/vc_bench.log 2>&1
rc=$?; echo "[vc] bench rc=$rc"; grep '^{' gpurun_out/vc_bench.log; exit $rc
