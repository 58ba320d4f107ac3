#!/bin/bash
# GPU-box job (round 6): narrow row-window variant default (IMAGINAIRE_AMD_CONV_RW_SMALL=2) vs
# off (0) on the recipes with Cout = 64 long-filter convs; rw tests first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r6small
timeout -k 10 400 python -u -m pytest tests/test_conv_rw_gpu.py -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r6small/tests.log 2>&1
rc=$?; echo "[small] tests rc=$rc"; tail -2 gpurun_out/r6small/tests.log; [ $rc -eq 0 ] || exit $rc
LIST="${ONLY:-munit256 pix2pixhd512x1024 vid2vid512x1024 fsvid2vid512}"
for arm in on off; do
  v=2; [ $arm = off ] && v=0
  IMAGINAIRE_AMD_CONV_RW_SMALL=$v OUTDIR=gpurun_out/r6small/$arm REPS=1 STEPS=12 EXTRA=--graph \
    ONLY="$LIST" bash scripts/gpu/r5_recipes.sh > gpurun_out/r6small/$arm.log 2>&1
  rc=$?; echo "[small] $arm rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r6small/$arm.log; exit $rc; }
done
python3 - <<'PY'
import json
for arm in ('on', 'off'):
    for l in open('gpurun_out/r6small/%s/recipes.jsonl' % arm):
        r = json.loads(l)
        print(arm, r['family'], r['frames_per_s'], r['frames_per_s_pipelined'], r['losses_finite'])
PY
