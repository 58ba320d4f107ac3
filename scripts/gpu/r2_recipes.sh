#!/bin/bash
# GPU-box job: secondary BASELINE configs at recipe scale (+ rocprof breakdowns) and the eager
# PyTorch self-baseline of the flagship SPADE step. Stops at the first fault / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/recipes
PROF=1 bash scripts/gpu/recipes_round.sh || exit $?
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --eager > gpurun_out/recipes/bench_eager.out \
  2> gpurun_out/recipes/bench_eager.err
rc=$?
echo "[recipes] bench_eager rc=$rc"; tail -2 gpurun_out/recipes/bench_eager.out
exit $rc
