#!/bin/bash
# GPU-box job (round 5): the whole GPU test suite (stop at the first failure), then bench.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/full5
rm -rf "$OUT"; mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > "$OUT/tests.log" 2>&1; rc=$?; tail -4 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
for f in ${BENCH_SN:-1}; do
  IMAGINAIRE_AMD_SN_FUSED=$f timeout -k 10 300 python -u bench.py --steps 20 --warmup 6 \
    > "$OUT/bench_sn$f.log" 2>&1; rc=$?; tail -1 "$OUT/bench_sn$f.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
