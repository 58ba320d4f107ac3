#!/bin/bash
# GPU-box job (round 6): spectral-norm group fix (idle layers keep u / v) — parity gate,
# SN / graph / determinism tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6sn; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests/test_model_parity_gpu.py tests/test_sn_fused_gpu.py \
  tests/test_dis_batch_gpu.py -v -s --timeout 400 --timeout-method thread -p no:cacheprovider \
  > $OUT/parity.log 2>&1
rc=$?; echo "[sn] parity rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/parity.log | tail -14
[ $rc -le 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_graph_gpu.py tests/test_determinism_gpu.py \
  tests/test_conv_rw_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "not packet" > $OUT/graph.log 2>&1
rc2=$?; echo "[sn] graph/det/rw rc=$rc2"; tail -3 $OUT/graph.log
exit $(( rc > rc2 ? rc : rc2 ))
