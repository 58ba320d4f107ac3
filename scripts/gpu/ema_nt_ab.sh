#!/bin/bash
# GPU-box job: non-temporal EMA A/B (probe x2 each, EMA tests with the default, bench each way).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/ema_nt; mkdir -p $OUT
set -o pipefail
for nt in 0 1 0 1; do
  IMAGINAIRE_AMD_EMA_NT=$nt timeout -k 10 120 python -u scripts/probe/adam_nt_probe.py >> $OUT/probe.log 2>&1 || exit $?
done
timeout -k 10 300 python -u -m pytest tests -m gpu -q -k "ema or EMA or average or Average" --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || exit $?
for nt in 1 0 1; do
  IMAGINAIRE_AMD_EMA_NT=$nt timeout -k 10 200 python -u bench.py > $OUT/bench_nt$nt.log 2>&1 || exit $?
  echo "EMA_NT=$nt $(tail -1 $OUT/bench_nt$nt.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $OUT/bench_summary.txt
done
grep -v amdgpu.ids $OUT/probe.log; cat $OUT/bench_summary.txt; tail -2 $OUT/tests.log
