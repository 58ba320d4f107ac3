#!/bin/bash
# GPU-box job (round 5): per-kernel steady-state profile of the SPADE bench step with the fused
# spectral-norm conv path off and on.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/snprof
rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for f in ${FUSED:-0 1}; do
  rm -rf /tmp/prof_sn$f
  IMAGINAIRE_AMD_SN_FUSED=$f timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
    -d /tmp/prof_sn$f -o run -- python3 "$ROOT/bench.py" --steps 3 --warmup 4 --verbose > "$OUT/prof$f.log" 2>&1
  rc=$?; echo "[prof] fused=$f rc=$rc"; tail -1 "$OUT/prof$f.log"; [ $rc -eq 0 ] || exit $rc
  (cd "$ROOT" && python3 scripts/gpu/summarize_kernels.py /tmp/prof_sn$f > "$OUT/kernels$f.txt") || exit 1
  head -10 "$OUT/kernels$f.txt"
done
