#!/bin/bash
# GPU-box job (round 6): row-window + tap-pack tests, the k10 kernel suite, then the MUNIT /
# FUNIT / pix2pixHD recipes (eager conv log + graphed throughput).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6b
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_conv_rw_gpu.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > "$OUT/rw_tests.log" 2>&1
rc=$?; echo "[b] rw tests rc=$rc"; tail -5 "$OUT/rw_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "conv or deconv or strided" \
  --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/kernel_conv_tests.log" 2>&1
rc=$?; echo "[b] kernel conv tests rc=$rc"; tail -5 "$OUT/kernel_conv_tests.log"; [ $rc -eq 0 ] || exit $rc
[ -n "$NORECIPE" ] && exit 0
RECIPES="${ONLY:-munit256 funit256 pix2pixhd512x1024}"
EXTRA=--graph REPS=1 STEPS=${STEPS:-12} ONLY="$RECIPES" bash scripts/gpu/r5_recipes.sh
rc=$?
mkdir -p "$OUT/graph"; cp gpurun_out/r5rec/* "$OUT/graph/" 2>/dev/null
[ $rc -eq 0 ] || exit $rc
[ -n "$NOCONVLOG" ] && exit 0
REPS=1 STEPS=1 CONVLOG=1 ONLY="$RECIPES" bash scripts/gpu/r5_recipes.sh
rc=$?
mkdir -p "$OUT/convlog"; cp gpurun_out/r5rec/* "$OUT/convlog/" 2>/dev/null
exit $rc
