#!/bin/bash
# GPU-box job: multi-condition SPADE / norm tests + video parity, then the video recipes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_model_parity_gpu.py -k "multi_condition or fused_norm or vid2vid" \
  > gpurun_out/mod_test.log 2>&1
rc=$?; echo "[mod] tests rc=$rc"; tail -3 gpurun_out/mod_test.log; [ $rc -eq 0 ] || exit $rc
ONLY="${ONLY:-fsvid2vid512 vid2vid512x1024}" bash scripts/gpu/recipes_round.sh
