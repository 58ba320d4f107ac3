#!/bin/bash
# GPU-box job (round 3): bisect the non-finite G updates of the replayed pix2pixHD graph by
# kernel switch, then the eager poisoned-pool probe. Each step under its own limit; a crash,
# abort or time-out ends the job.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r3n
mkdir -p "$OUT"
FAM=${FAM:-pix2pixHD}
step() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 240 python -u scripts/probe/graph_nan_probe.py $FAM > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "[r3n] $name ($*) rc=$rc"; grep replay "$OUT/$name.out"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.err"; exit $rc; fi
}
step default
step v4off IMAGINAIRE_AMD_CONV_V4=0
step wv2off IMAGINAIRE_AMD_WGRAD_V2=0
step wgrad_miopen IMAGINAIRE_AMD_MFMA_WGRAD=0
step conv_off IMAGINAIRE_AMD_MFMA_CONV=0
timeout -k 10 240 python -u scripts/probe/poison_probe.py $FAM > "$OUT/poison.out" 2> "$OUT/poison.err"
rc=$?; echo "[r3n] poison rc=$rc"; cat "$OUT/poison.out" | grep -E "trial|non-finite"
exit $rc
