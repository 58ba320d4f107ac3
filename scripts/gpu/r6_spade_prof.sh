#!/bin/bash
# GPU-box job (round 6): the SPADE headline step at HEAD — bench (graph), per-conv log of one
# eager step, and the rocprofv3 kernel breakdown of the graphed steady state.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r6spade
mkdir -p "$OUT"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 6 > "$OUT/bench.log" 2>&1
rc=$?; echo "[spade] bench rc=$rc: $(grep '"metric"' $OUT/bench.log | cut -c60-140)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 2 --warmup 3 --conv-log > "$OUT/convlog.log" 2>&1
rc=$?; echo "[spade] convlog rc=$rc"; grep -A8 "conv kernels in one" "$OUT/convlog.log" | head -9; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/iamd_sprof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/iamd_sprof -o bench \
  -- python3 "$ROOT/bench.py" --steps 3 --warmup 4 --verbose > "$OUT/prof_bench.log" 2>&1
rc=$?; echo "[spade] prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
SUMMARY_ROWS=120 python3 "$ROOT/scripts/gpu/summarize_kernels.py" /tmp/iamd_sprof > "$OUT/kernels.txt"
head -12 "$OUT/kernels.txt"
