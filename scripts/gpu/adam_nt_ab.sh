#!/bin/bash
# GPU-box job: non-temporal Adam A/B (probe x2 each, kernel tests with NT=1, bench each way).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/adam_nt; mkdir -p $OUT
set -o pipefail
for nt in 0 1 0 1; do
  IMAGINAIRE_AMD_ADAM_NT=$nt timeout -k 10 120 python -u scripts/probe/adam_nt_probe.py >> $OUT/probe.log 2>&1 || exit $?
done
IMAGINAIRE_AMD_ADAM_NT=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py -m gpu -q -k "adam or Adam" --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests_nt1.log 2>&1 || exit $?
for nt in 1 0 1; do
  IMAGINAIRE_AMD_ADAM_NT=$nt timeout -k 10 200 python -u bench.py > $OUT/bench_nt$nt.log 2>&1 || exit $?
  echo "NT=$nt $(tail -1 $OUT/bench_nt$nt.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $OUT/bench_summary.txt
done
cat $OUT/probe.log $OUT/bench_summary.txt; tail -2 $OUT/tests_nt1.log
