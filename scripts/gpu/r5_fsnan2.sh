#!/bin/bash
# GPU-box job (round 5): few-shot vid2vid recipe divergence, second pass: an eager run with
# NaN-poisoned allocations (uninitialised reads show up as NaN), then a graph run with
# in-graph isfinite flags on every leaf module output / output gradient.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
EAGERONLY=1 EXTRA="--poison" WARM=6 STEPS=2 bash scripts/gpu/r5_fsnan.sh || exit $?
mv gpurun_out/r5fs/fs_k1_eager.err gpurun_out/r5fs/fs_k1_poison_eager.err
NOEAGER=1 EXTRA="--flag-probe" WARM=6 STEPS=4 bash scripts/gpu/r5_fsnan.sh
rc=$?
grep "flag-probe" gpurun_out/r5fs/fs_k1_graph.err | head -80
exit $rc
