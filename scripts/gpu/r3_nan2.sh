#!/bin/bash
# GPU-box job (round 3): stash-probe the replayed pix2pixHD graph (SN backward tensors, then
# every module's activations / output gradients), then the graph with every HIP op off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r3n2
mkdir -p "$OUT"
run() {  # name, cmd...
  local name=$1; shift
  timeout -k 10 240 "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "[r3n2] $name rc=$rc"; grep -E "replay|stashed|non-finite|sigmas" "$OUT/$name.out"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.err"; exit $rc; fi
}
run stash_sn env MODE=sn python -u scripts/probe/graph_stash_probe.py pix2pixHD
run stash_all env MODE=all python -u scripts/probe/graph_stash_probe.py pix2pixHD
run eager_graph env IMAGINAIRE_AMD_EAGER=1 python -u scripts/probe/graph_nan_probe.py pix2pixHD
exit 0
