#!/bin/bash
# GPU-box job (round 3): is the replayed pix2pixHD NaN MIOpen's weight gradient? Graph replay
# with MIOpen deterministic solvers, then with the small convs on k10 / k11 instead of MIOpen.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r3n3
mkdir -p "$OUT"
run() {  # name, cmd...
  local name=$1; shift
  timeout -k 10 240 "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "[r3n3] $name rc=$rc"; grep -E "replay" "$OUT/$name.out"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.err"; exit $rc; fi
}
run det env IAMD_PROBE_DET=1 python -u scripts/probe/graph_nan_probe.py pix2pixHD
run eager_det env IAMD_PROBE_DET=1 IMAGINAIRE_AMD_EAGER=1 python -u scripts/probe/graph_nan_probe.py pix2pixHD
run minblocks env IMAGINAIRE_AMD_MFMA_MIN_BLOCKS=1 IMAGINAIRE_AMD_MFMA_MIN_DGRAD_BLOCKS=1 python -u scripts/probe/graph_nan_probe.py pix2pixHD
exit 0
