#!/bin/bash
# GPU-box job (round 6): video-recipe graph replay throughput with the runtime's packet-capture
# mode off (package default) vs on (DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 with the capture guard
# overridden) — the price of the workaround on the tens-of-thousands-of-node graphs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6pc; mkdir -p $OUT
: > $OUT/pc.jsonl
V2V="--config configs/unit_test/vid2vid_street.yaml --seq-len 3 --set gen.num_filters=32 \
  gen.max_num_filters=1024 gen.flow.num_filters=32 gen.flow.max_num_filters=1024 \
  gen.flow.multi_spade_combine.embed.num_filters=32 gen.embed.num_filters=32 \
  gen.embed.max_num_filters=1024 dis.image.num_filters=64 dis.image.max_num_filters=512 \
  dis.temporal.num_filters=64 dis.temporal.max_num_filters=512 data.train.batch_size=2 \
  data.train.augmentations.resize_h_w=512,1024 data.val.augmentations.resize_h_w=512,1024"
for arm in off on off2; do
  envs=""
  [ $arm = on ] && envs="DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 IMAGINAIRE_AMD_GRAPH_ALLOW_PACKET_CAPTURE=1"
  env $envs timeout -k 10 500 python scripts/bench_families.py $V2V --steps 8 --warmup 4 --graph \
    > $OUT/v2v_$arm.json 2> $OUT/v2v_$arm.err
  rc=$?; echo "[pc] vid2vid $arm rc=$rc $(cut -c1-200 $OUT/v2v_$arm.json)"
  echo "{\"arm\": \"$arm\", \"rc\": $rc, \"row\": $(cat $OUT/v2v_$arm.json | tail -1 || echo null)}" >> $OUT/pc.jsonl
  [ $rc -le 3 ] || exit $rc
done
exit 0
