#!/bin/bash
# GPU-box job (round 6): SPADE bench A/B of the selective backward overlap (weight gradients of
# the small convs on a side stream: IMAGINAIRE_AMD_CONV_BWD_OVERLAP=small[:P]).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6ovl; mkdir -p $OUT
for arm in 0 small small:32768 0b small:2048; do
  v=${arm%b}
  IMAGINAIRE_AMD_CONV_BWD_OVERLAP=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 6 \
    > "$OUT/bench_$arm.log" 2>&1
  rc=$?; echo "[ovl] $arm rc=$rc: $(grep '"metric"' $OUT/bench_$arm.log | cut -c60-135)"
  [ $rc -eq 0 ] || { tail -5 "$OUT/bench_$arm.log"; exit $rc; }
done
