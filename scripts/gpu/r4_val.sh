#!/bin/bash
# GPU-box job (round 4): new-kernel tests, their probes, then bench + steady-state trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r4v
mkdir -p "$OUT"
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "[r4v] $name rc=$rc"; tail -${TAILN:-12} "$OUT/$name.out"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.err"; exit $rc; fi
}
step tests 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q --timeout 120 \
  --timeout-method thread -k "${TK:-fused_attention or correlation or spectral or sn_ or adam}"
[ -z "$PROBES" ] || step attn 300 python scripts/probe/attn_probe.py
[ -z "$PROBES" ] || [ -n "$NOCORR" ] || step corr 300 python scripts/probe/corr_bwd_probe.py
if [ -n "$FS" ]; then bash scripts/gpu/r4_fs.sh; rc=$?; [ $rc -eq 0 ] || exit $rc; fi
[ -z "$BENCH" ] || step bench 300 python bench.py --steps 30 --warmup 6
if [ -n "$TRACE" ]; then
  cd /tmp && export TMPDIR=/tmp
  rm -rf /tmp/iamd_prof
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/iamd_prof -o bench -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 4 --verbose > "$OUT/trace.out" 2> "$OUT/trace.err"
  rc=$?; echo "[r4v] trace rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/trace.err"; exit $rc; }
  cd "$ROOT"
  python3 scripts/gpu/summarize_kernels.py /tmp/iamd_prof > "$OUT/top_kernels.txt" || true
  head -60 "$OUT/top_kernels.txt"
fi
exit 0
