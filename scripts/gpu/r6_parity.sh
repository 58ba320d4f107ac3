#!/bin/bash
# GPU-box job (round 6): model-level parity gate (with its negative control), the batched
# discriminator bound, then the plain vs forced-distributed kernel profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6par; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests/test_dis_batch_gpu.py tests/test_model_parity_gpu.py -x -v -s \
  --timeout 400 --timeout-method thread -p no:cacheprovider > $OUT/parity.log 2>&1
rc=$?; echo "[par] rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/parity.log | tail -15
exit $rc
