#!/bin/bash
# GPU-box job (round 6): per-module forward / backward divergence of the vid2vid unit iteration,
# HIP-bf16 vs two PyTorch-bf16 runs (scripts/probe/parity_act_probe.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6act; mkdir -p $OUT
timeout -k 10 600 python -u scripts/probe/parity_act_probe.py vid2vid_street.yaml 2 60 > $OUT/v2v.log 2>&1
rc=$?; echo "[act] rc=$rc"; grep -v Warning $OUT/v2v.log | tail -70 | cut -c1-260
exit $rc
