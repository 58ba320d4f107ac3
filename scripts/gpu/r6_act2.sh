#!/bin/bash
# GPU-box job (round 6): every module record around the first forward divergence of vid2vid.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6act2; mkdir -p $OUT
ACT_DUMP=${ACT_DUMP:-30:60} timeout -k 10 600 python -u scripts/probe/parity_act_probe.py \
  vid2vid_street.yaml 2 5 > $OUT/act.log 2>&1
rc=$?; echo "[act2] rc=$rc"; grep -E "^ +=" $OUT/act.log | cut -c1-240
exit $rc
