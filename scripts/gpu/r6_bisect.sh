#!/bin/bash
# GPU-box job (round 6): which kernel path moves the vid2vid G up-block weight gradients away
# from PyTorch-bf16 (tests/test_model_parity_gpu.py vid2vid) — the parity test under A/B switches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6bis; mkdir -p $OUT
for arm in default IMAGINAIRE_AMD_TAPPACK=0 IMAGINAIRE_AMD_SN_FUSED=0 IMAGINAIRE_AMD_CONV_RW=0 \
    IMAGINAIRE_AMD_SN_DOT_RATIO=0 IMAGINAIRE_AMD_CONV_V=1; do
  envs=""; [ "$arm" != default ] && envs="$arm"
  env $envs timeout -k 10 300 python -u -m pytest tests/test_model_parity_gpu.py -k vid2vid_iteration -x -q -s \
    --timeout 280 --timeout-method thread -p no:cacheprovider > "$OUT/$arm.log" 2>&1
  rc=$?
  echo "[bis] $arm rc=$rc"
  grep -E "G grads:" "$OUT/$arm.log" | cut -c1-400
  grep -E "^E +AssertionError" "$OUT/$arm.log" | cut -c1-300
  [ $rc -le 1 ] || exit $rc
done
exit 0
