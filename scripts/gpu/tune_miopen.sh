#!/bin/bash
# Exhaustive MIOpen find for every conv problem of the flagship step; the user
# find-db / perf-db land in gpurun_out/miopen_udb (copy to tuning/miopen to ship).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
mkdir -p gpurun_out/miopen_udb
export MIOPEN_USER_DB_PATH=$ROOT/gpurun_out/miopen_udb
export IMAGINAIRE_AMD_MIOPEN_TUNE=1
( while true; do sleep 50; echo "hb $(date +%s) $(ls gpurun_out/miopen_udb | wc -l) files" >> gpurun_out/tune_heartbeat.log; done ) &
HB=$!
timeout -k 10 ${TUNE_TIMEOUT:-1000} python bench.py --steps 2 --warmup 1 --verbose \
  > gpurun_out/tune_bench.json 2> gpurun_out/tune_bench.err
rc=$?
kill $HB
echo "[tune] rc=$rc"; cat gpurun_out/tune_bench.json; ls -la gpurun_out/miopen_udb
exit $rc
