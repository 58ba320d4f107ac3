#!/bin/bash
# GPU-box job (round 6, first call): graph packet-capture probes, the model-parity gate with its
# negative control, then per-shape conv logs of the recipes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r6a
bash scripts/gpu/r6_graph.sh; rc=$?; echo "[r6a] graph rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_model_parity_gpu.py -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r6a/parity.log 2>&1
rc=$?; echo "[r6a] parity rc=$rc"; tail -5 gpurun_out/r6a/parity.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ -n "$NOCONV" ] && exit 0
bash scripts/gpu/r6_convlog.sh
