#!/bin/bash
# GPU-box job (round 6): SN idle-layer test, graph / determinism / rw tests, then the per-module
# parity probe of vid2vid after the SN group fix.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6sn2; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_sn_fused_gpu.py tests/test_graph_gpu.py \
  tests/test_determinism_gpu.py tests/test_conv_rw_gpu.py -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; echo "[sn2] tests rc=$rc"; tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u scripts/probe/parity_act_probe.py vid2vid_street.yaml 2 40 > $OUT/act.log 2>&1
rc2=$?; echo "[sn2] act rc=$rc2"; grep -v Warning $OUT/act.log | grep -E "^ +#|records|rows" | head -60 | cut -c1-240
exit $rc
