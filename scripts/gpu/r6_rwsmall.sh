#!/bin/bash
# GPU-box job (round 6): row-window tile tests (any segment width), the per-shape probe with the
# narrow variant off / on (IMAGINAIRE_AMD_CONV_RW_SMALL), then MUNIT / FUNIT A/B of the
# any-width segments.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6rwany; mkdir -p $OUT
timeout -k 10 200 python -u scripts/probe/conv_rw_probe.py > $OUT/probe_default.txt 2>&1
rc=$?; echo "[rws] probe default rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/probe_default.txt; exit $rc; }
IMAGINAIRE_AMD_CONV_RW_SMALL=1 timeout -k 10 200 python -u scripts/probe/conv_rw_probe.py > $OUT/probe_small.txt 2>&1
rc=$?; echo "[rws] probe small rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/probe_small.txt; exit $rc; }
paste -d'|' <(cut -c1-100 $OUT/probe_default.txt) <(cut -c47-100 $OUT/probe_small.txt)
IMAGINAIRE_AMD_CONV_RW_SMALL=1 timeout -k 10 400 python -u -m pytest tests/test_conv_rw_gpu.py -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider -k "forward or splitk or lds" > $OUT/tests_small.log 2>&1
rc=$?; echo "[rws] small tests rc=$rc"; tail -2 $OUT/tests_small.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu/r6_rwany.sh
