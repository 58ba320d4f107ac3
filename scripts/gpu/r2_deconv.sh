#!/bin/bash
# GPU-box job: transposed-conv phase path tests + probe, then the recipe runs (conv logs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "conv_transpose_phase or predict_flow" > gpurun_out/deconv_test.log 2>&1
rc=$?; echo "[dc] tests rc=$rc"; tail -3 gpurun_out/deconv_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probe/deconv_probe.py > gpurun_out/deconv_probe.log 2>&1
rc=$?; echo "[dc] probe rc=$rc"; cat gpurun_out/deconv_probe.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu/recipes_round.sh
