#!/bin/bash
# GPU-box job: same-box A/B of the multi-condition SPADE modulation (eager vs k1 'none' mode).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/ab
: > gpurun_out/ab/ab.jsonl
for mode in 0 1 0 1; do
  for cfg in fs vid; do
    if [ $cfg = fs ]; then
      args="--config configs/unit_test/fs_vid2vid_face.yaml --steps 3 --warmup 2 --seq-len 4 --set gen.num_filters=32 gen.num_downsamples=5 gen.hyper.num_hyper_layers=4 gen.hyper.attention.num_filters=32 gen.flow.num_filters=32 gen.flow.max_num_filters=1024 gen.flow.num_res_blocks=6 gen.flow.multi_spade_combine.embed.num_filters=32 gen.flow.multi_spade_combine.embed.num_downsamples=5 gen.embed.num_filters=32 gen.embed.num_downsamples=5 dis.image.num_filters=32 dis.image.max_num_filters=512 dis.image.num_layers=4 data.initial_few_shot_K=1 data.train.batch_size=3 data.train.augmentations.resize_h_w=512,512 data.val.augmentations.resize_h_w=512,512"
    else
      args="--config configs/unit_test/vid2vid_street.yaml --steps 3 --warmup 2 --seq-len 3 --set gen.num_filters=32 gen.max_num_filters=1024 gen.flow.num_filters=32 gen.flow.max_num_filters=1024 gen.flow.multi_spade_combine.embed.num_filters=32 gen.embed.num_filters=32 gen.embed.max_num_filters=1024 dis.image.num_filters=64 dis.image.max_num_filters=512 dis.temporal.num_filters=64 dis.temporal.max_num_filters=512 data.train.batch_size=2 data.train.augmentations.resize_h_w=512,1024 data.val.augmentations.resize_h_w=512,1024"
    fi
    IMAGINAIRE_AMD_SPADE_MULTIMOD=$mode timeout -k 10 300 python scripts/bench_families.py $args \
      > gpurun_out/ab/out.json 2> gpurun_out/ab/${cfg}_$mode.err || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/ab/out.json')); print('[ab] $cfg multimod=$mode', d['frames_per_s'], d['ms_per_iteration'])"
  done
done
