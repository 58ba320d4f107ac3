#!/bin/bash
# GPU-box job (round 3): hipGraph capture of every family's unit-test step, eager vs replayed
# (losses + throughput); DEBUG=1 makes a failed capture raise (IMAGINAIRE_AMD_GRAPH_DEBUG) so
# the stack names the op that breaks it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r3g
mkdir -p $OUT
: > $OUT/results.jsonl
for cfg in ${CFGS:-pix2pixHD munit vid2vid_street fs_vid2vid_face}; do
  for mode in ${MODES:-eager graph}; do
    extra=""; [ $mode = graph ] && extra="--graph"
    env ${DEBUG:+IMAGINAIRE_AMD_GRAPH_DEBUG=1} timeout -k 10 400 python scripts/bench_families.py \
      --config configs/unit_test/$cfg.yaml --steps ${STEPS:-6} --warmup 3 --pool 1 $extra \
      ${SEQ:+--seq-len $SEQ} >> $OUT/results.jsonl 2> $OUT/${cfg}_$mode.err
    rc=$?; echo "[r3g] $cfg $mode rc=$rc"; tail -1 $OUT/results.jsonl | cut -c1-400
    grep "\[graph\]" $OUT/${cfg}_$mode.err | tail -2
    if [ $rc -ne 0 ]; then tail -12 $OUT/${cfg}_$mode.err; [ $rc -eq 1 ] || exit $rc; fi
  done
done
exit 0
