#!/bin/bash
# GPU-box job (round 6): the row-window k10 tile — its own tests, then every k10 test of the
# kernel suite (the forward / backward / split-K / poison cases now routed through it).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6rw
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_conv_rw_gpu.py -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider > "$OUT/rw_tests.log" 2>&1
rc=$?; echo "[rw] rw tests rc=$rc"; tail -15 "$OUT/rw_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "conv or deconv or strided" \
  --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/kernel_conv_tests.log" 2>&1
rc=$?; echo "[rw] kernel conv tests rc=$rc"; tail -15 "$OUT/kernel_conv_tests.log"
exit $rc
