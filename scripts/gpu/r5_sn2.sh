#!/bin/bash
# GPU-box job (round 5): pad_channels_cast call sites with the fused SN path off / on, then the
# SN job (tests, bench A/B, profile).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/padsites
for f in 0 1; do
  IMAGINAIRE_AMD_SN_FUSED=$f timeout -k 10 300 python -u scripts/probe/pad_sites_probe.py \
    > gpurun_out/padsites/pad_sites$f.log 2>&1 || exit $?
  head -3 gpurun_out/padsites/pad_sites$f.log
done
[ -z "$SN_JOB" ] || bash scripts/gpu/r5_sn.sh
