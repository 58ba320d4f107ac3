#!/bin/bash
# GPU-box job (round 4): scripts/gpu/r4_tests.sh (TGROUPS / PROBES), then, when it succeeded,
# scripts/gpu/r4_iter.sh (BENCH / TRACE / ... flags). Every GPU step inside runs under its own
# time limit; the second script starts only if the first exited 0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/gpu/r4_tests.sh || exit $?
bash scripts/gpu/r4_iter.sh
