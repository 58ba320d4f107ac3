#!/bin/bash
# GPU-box job (round 3): per-conv timing of one SPADE step with k10 v4 on and off (same box),
# then the steady-state rocprofv3 kernel breakdown of the default step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r3ab
mkdir -p "$OUT"
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "[r3ab] $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.err"; exit $rc; fi
}
run convlog_v4 400 python bench.py --steps 1 --warmup 3 --conv-log
run convlog_nov4 400 env IMAGINAIRE_AMD_CONV_V4=0 python bench.py --steps 1 --warmup 3 --conv-log
grep -A 8 "conv kernels in one" "$OUT/convlog_v4.err"; grep -A 8 "conv kernels in one" "$OUT/convlog_nov4.err"
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/iamd_prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/iamd_prof -o bench -- \
  python3 "$ROOT/bench.py" --steps 3 --warmup 4 --verbose > "$OUT/trace.out" 2> "$OUT/trace.err"
rc=$?; echo "[r3ab] trace rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/trace.err"; exit $rc; }
cd "$ROOT"
python3 scripts/gpu/summarize_kernels.py /tmp/iamd_prof > "$OUT/top_kernels.txt" || true
head -40 "$OUT/top_kernels.txt"
exit 0
