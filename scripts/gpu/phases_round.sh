#!/bin/bash
# Steady-state evidence: (1) synchronised per-phase timers, (2) rocprofv3 kernel
# trace split at the profile marker (kernel time vs. wall span of the timed steps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 4 --warmup 3 --profile-phases --verbose \
  > gpurun_out/bench_phases.json 2> gpurun_out/bench_phases.err
rc=$?; echo "[phases] rc=$rc"; cat gpurun_out/bench_phases.json; grep "phase" gpurun_out/bench_phases.err
[ $rc -ne 0 ] && { tail -20 gpurun_out/bench_phases.err; exit $rc; }
SKIP_PROBE=1 BENCH_ARGS="--steps 4 --warmup 3 --verbose" bash scripts/gpu/profile_round.sh
