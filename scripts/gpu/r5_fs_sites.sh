#!/bin/bash
# GPU-box job (round 5): where the few-shot vid2vid recipe's glue comes from — extension calls
# (channel pad-casts, phase scatters) and ATen copies / cats by Python call site, one eager
# iteration under the captured step's routing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/fssites; mkdir -p $OUT
K=${K:-1}
OP_SITES_OPS=${OPS:-copy_,_to_copy,cat,clone,fill_,zero_,contiguous,add,add_} timeout -k 10 600 \
  python -u scripts/bench_families.py --config configs/unit_test/fs_vid2vid_face.yaml \
  --seq-len 4 --set gen.num_filters=32 gen.num_downsamples=5 gen.hyper.num_hyper_layers=4 \
  gen.hyper.attention.num_filters=32 gen.flow.num_filters=32 gen.flow.max_num_filters=1024 \
  gen.flow.num_res_blocks=6 gen.flow.multi_spade_combine.embed.num_filters=32 \
  gen.flow.multi_spade_combine.embed.num_downsamples=5 gen.embed.num_filters=32 \
  gen.embed.num_downsamples=5 dis.image.num_filters=32 dis.image.max_num_filters=512 \
  dis.image.num_layers=4 data.initial_few_shot_K=$K data.train.batch_size=3 \
  data.train.augmentations.resize_h_w=512,512 data.val.augmentations.resize_h_w=512,512 \
  --steps 2 --warmup 2 --ext-sites pad_channels_cast,conv_phase_scatter --op-sites \
  > $OUT/k$K.jsonl 2> $OUT/k$K.err; rc=$?; echo "rc=$rc"; grep -n "extension calls\|op self\|aten glue" $OUT/k$K.err | head
exit $rc
