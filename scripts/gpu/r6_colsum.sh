#!/bin/bash
# GPU-box job (round 6): 16-byte-load spectral-norm column sums — SN tests, bench, kernel time.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r6colsum; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_sn_fused_gpu.py tests/test_kernels_gpu.py -q -k "sn or spectral" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; echo "[colsum] tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 6 > $OUT/bench.log 2>&1
rc=$?; echo "[colsum] bench rc=$rc: $(grep '"metric"' $OUT/bench.log | cut -c60-140)"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/iamd_cprof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/iamd_cprof -o bench \
  -- python3 "$ROOT/bench.py" --steps 3 --warmup 4 --verbose > "$OUT/prof_bench.log" 2>&1
rc=$?; echo "[colsum] prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
SUMMARY_ROWS=120 python3 "$ROOT/scripts/gpu/summarize_kernels.py" /tmp/iamd_cprof > "$OUT/kernels.txt"
grep -E "STEADY|total kernel|sn_" "$OUT/kernels.txt" | cut -c1-150
