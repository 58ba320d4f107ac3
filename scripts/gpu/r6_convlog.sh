#!/bin/bash
# GPU-box job (round 6): per-shape conv logs (eager, one iteration after warm-up) of the
# BASELINE secondary recipes at HEAD, to size the non-row-window (v1) conv work.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
CONVLOG=1 REPS=1 STEPS=${STEPS:-3} ONLY="${ONLY:-munit256 funit256 pix2pixhd512x1024 vid2vid512x1024 fsvid2vid512}" \
  bash scripts/gpu/r5_recipes.sh
rc=$?
mkdir -p gpurun_out/r6conv
cp gpurun_out/r5rec/* gpurun_out/r6conv/ 2>/dev/null
exit $rc
