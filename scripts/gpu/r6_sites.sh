#!/bin/bash
# GPU-box job (round 6): ATen glue and pad_cast call sites (scripts/probe/op_sites.py) of the
# few-shot vid2vid K = 2 and vid2vid 512x1024 recipes, one eager iteration each under the
# captured step's routing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6sites; mkdir -p $OUT
export OP_SITES_OPS=${OPS:-copy_,_to_copy,cat,clone,fill_,zero_,zeros,zeros_like,new_zeros,contiguous,add,add_,mul,sub,div,where,mean,sum}
timeout -k 10 500 python -u scripts/bench_families.py --config configs/unit_test/fs_vid2vid_face.yaml \
  --seq-len 4 --set gen.num_filters=32 gen.num_downsamples=5 gen.hyper.num_hyper_layers=4 \
  gen.hyper.attention.num_filters=32 gen.flow.num_filters=32 gen.flow.max_num_filters=1024 \
  gen.flow.num_res_blocks=6 gen.flow.multi_spade_combine.embed.num_filters=32 \
  gen.flow.multi_spade_combine.embed.num_downsamples=5 gen.embed.num_filters=32 \
  gen.embed.num_downsamples=5 dis.image.num_filters=32 dis.image.max_num_filters=512 \
  dis.image.num_layers=4 data.initial_few_shot_K=2 data.train.batch_size=3 \
  data.train.augmentations.resize_h_w=512,512 data.val.augmentations.resize_h_w=512,512 \
  --steps 1 --warmup 2 --ext-sites pad_channels_cast --op-sites > $OUT/fsk2.jsonl 2> $OUT/fsk2.err
rc=$?; echo "[sites] fsk2 rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/fsk2.err; exit $rc; }
timeout -k 10 500 python -u scripts/bench_families.py --config configs/unit_test/vid2vid_street.yaml \
  --seq-len 3 --set gen.num_filters=32 gen.max_num_filters=1024 gen.flow.num_filters=32 \
  gen.flow.max_num_filters=1024 gen.flow.multi_spade_combine.embed.num_filters=32 \
  gen.embed.num_filters=32 gen.embed.max_num_filters=1024 dis.image.num_filters=64 \
  dis.image.max_num_filters=512 dis.temporal.num_filters=64 dis.temporal.max_num_filters=512 \
  data.train.batch_size=2 data.train.augmentations.resize_h_w=512,1024 \
  data.val.augmentations.resize_h_w=512,1024 --steps 1 --warmup 2 \
  --ext-sites pad_channels_cast --op-sites > $OUT/v2v.jsonl 2> $OUT/v2v.err
rc=$?; echo "[sites] v2v rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/v2v.err; exit $rc; }
