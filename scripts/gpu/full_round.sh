#!/bin/bash
# kernel tests + smoke, then rocprofv3-profiled short bench (stops on first fault)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
NO_BENCH=1 bash scripts/gpu/run_round.sh || exit $?
SKIP_PROBE=1 bash scripts/gpu/profile_round.sh
