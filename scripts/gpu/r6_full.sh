#!/bin/bash
# GPU-box job (round 6): the GPU test suite in two halves (PART=1 | 2), one pytest process each,
# then (PART=2) smoke() and a short bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6full; mkdir -p $OUT
if [ "${PART:-1}" = 1 ]; then
  FILES="tests/test_kernels_gpu.py tests/test_conv_rw_gpu.py tests/test_sn_fused_gpu.py tests/test_gp_gpu.py tests/test_dis_batch_gpu.py tests/test_spade_dis_semantics_cpu.py"
else
  FILES="tests/test_graph_gpu.py tests/test_graph_families_gpu.py tests/test_determinism_gpu.py tests/test_distributed_gpu.py tests/test_recipe_finite_gpu.py tests/test_model_parity_gpu.py"
fi
timeout -k 10 1050 python -u -m pytest $FILES -m gpu -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/part${PART:-1}.log 2>&1
rc=$?; echo "[full] part ${PART:-1} rc=$rc"; tail -4 $OUT/part${PART:-1}.log
grep -E "^FAILED|^ERROR" $OUT/part${PART:-1}.log | head -20
exit $rc
