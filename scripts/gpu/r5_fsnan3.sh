#!/bin/bash
# GPU-box job (round 5): few-shot vid2vid replay NaN, allocation-churn A/B: the same graph run
# with the batches prepared once (--static-batch: nothing allocated between replays) and with
# a fresh clone per iteration (default).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
NOEAGER=1 EXTRA="--static-batch" WARM=6 STEPS=12 bash scripts/gpu/r5_fsnan.sh || exit $?
mv gpurun_out/r5fs/fs_k1_graph.err gpurun_out/r5fs/fs_k1_graph_static.err
NOEAGER=1 WARM=6 STEPS=12 bash scripts/gpu/r5_fsnan.sh
