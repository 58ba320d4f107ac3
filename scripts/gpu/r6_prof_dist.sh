#!/bin/bash
# GPU-box job (round 6): rocprofv3 kernel-trace of the SPADE bench, plain vs forced one-rank
# distributed (where the 13 ms/step of the world-1 distributed wrappers go).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r6prof
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for arm in plain forced; do
  extra=""; [ $arm = forced ] && extra="--force-dist"
  rm -rf /tmp/iamd_prof_$arm
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/iamd_prof_$arm \
    -o bench -- python3 "$ROOT/bench.py" --steps 3 --warmup 4 --verbose $extra > "$OUT/bench_$arm.log" 2>&1
  rc=$?; echo "[prof] $arm rc=$rc"; [ $rc -eq 0 ] || exit $rc
  SUMMARY_ROWS=400 python3 "$ROOT/scripts/gpu/summarize_kernels.py" /tmp/iamd_prof_$arm > "$OUT/kernels_$arm.txt" || true
  head -12 "$OUT/kernels_$arm.txt"
done
