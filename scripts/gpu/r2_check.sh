#!/bin/bash
# GPU-box job: the full GPU test suite, then the recipe-scale secondary configs (no rocprof) and
# the flagship bench. Stops at the first fault / abort / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/check
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 170 --timeout-method thread \
  > gpurun_out/check/tests.out 2> gpurun_out/check/tests.err
rc=$?
echo "[check] tests rc=$rc"; tail -8 gpurun_out/check/tests.out
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
if [ -z "$SKIP_RECIPES" ]; then
  bash scripts/gpu/recipes_round.sh || exit $?
fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/check/bench.out 2> gpurun_out/check/bench.err
rc=$?
echo "[check] bench rc=$rc"; tail -1 gpurun_out/check/bench.out
exit $rc
