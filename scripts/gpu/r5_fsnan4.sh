#!/bin/bash
# GPU-box job (round 5): few-shot vid2vid replay NaN — every timed iteration as a replay AND as
# the eager step from the same saved state (--ab-eager), continuing along the eager trajectory.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
NOEAGER=1 EXTRA="--static-batch --ab-eager $EXTRA2" WARM=6 STEPS=${STEPS:-8} bash scripts/gpu/r5_fsnan.sh
rc=$?
grep "^\[ab\]\|flag-probe" gpurun_out/r5fs/fs_k${K:-1}_graph.err | cut -c1-400 | head -120
exit $rc
