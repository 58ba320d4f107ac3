#!/bin/bash
# GPU-box job (round 5): ATen glue of the vid2vid 512x1024 recipe by Python call site (one
# eager iteration under the captured step's routing).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/v2vsites; mkdir -p $OUT
OP_SITES_OPS=${OPS:-copy_,_to_copy,cat,clone,fill_,zero_,contiguous,add,add_,mul,sub,div,where,mean,sum} timeout -k 10 600 \
  python -u scripts/bench_families.py --config configs/unit_test/vid2vid_street.yaml \
  --seq-len 3 --set gen.num_filters=32 gen.max_num_filters=1024 gen.flow.num_filters=32 \
  gen.flow.max_num_filters=1024 gen.flow.multi_spade_combine.embed.num_filters=32 \
  gen.embed.num_filters=32 gen.embed.max_num_filters=1024 dis.image.num_filters=64 \
  dis.image.max_num_filters=512 dis.temporal.num_filters=64 dis.temporal.max_num_filters=512 \
  data.train.batch_size=2 data.train.augmentations.resize_h_w=512,1024 \
  data.val.augmentations.resize_h_w=512,1024 --steps 2 --warmup 2 \
  --ext-sites pad_channels_cast --op-sites > $OUT/v2v.jsonl 2> $OUT/v2v.err; rc=$?; echo "rc=$rc"
exit $rc
