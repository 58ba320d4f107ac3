#!/bin/bash
# GPU-box job (round 6): parity gate with the perturbed-start envelope, rw / tap-pack tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6par2; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests/test_model_parity_gpu.py -v -s --timeout 400 \
  --timeout-method thread -p no:cacheprovider > $OUT/parity.log 2>&1
rc=$?; echo "[par2] rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/parity.log | tail -12
grep -E "grads: " $OUT/parity.log | cut -c1-330
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_conv_rw_gpu.py -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > $OUT/rw.log 2>&1
rc2=$?; echo "[par2] rw rc=$rc2"; tail -2 $OUT/rw.log
exit $(( rc > rc2 ? rc : rc2 ))
