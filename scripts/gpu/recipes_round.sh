#!/bin/bash
# BASELINE.json secondary configs at their recipe scale (reference project configs' model widths,
# batch and crop) on one MI355X, synthetic data: unit-test configs scaled up with --set.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
: > gpurun_out/recipes.jsonl
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" python scripts/bench_families.py "$@" >> gpurun_out/recipes.jsonl \
    2> gpurun_out/recipe_$name.err
  local rc=$?
  echo "[recipes] $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/recipe_$name.err; [ $rc -eq 1 ] || exit $rc; fi
}
# MUNIT afhq_dog2cat ampO1 recipe: 256x256, batch 16
run munit256 400 --config configs/unit_test/munit.yaml --steps 5 --warmup 2 --set \
  gen.num_filters=64 gen.num_filters_mlp=256 gen.num_res_blocks=4 \
  dis.num_filters=32 dis.max_num_filters=512 dis.num_layers=6 trainer.loss_weight.perceptual=0 \
  data.train.batch_size=16 data.train.augmentations.random_crop_h_w=256,256
# vid2vid cityscapes ampO1 recipe: 512x1024, batch 2, 3-frame sequences, FlowNet2 flow loss
run vid2vid512x1024 600 --config configs/unit_test/vid2vid_street.yaml --steps 3 --warmup 2 \
  --seq-len 3 --set gen.num_filters=32 gen.max_num_filters=1024 gen.flow.num_filters=32 \
  gen.flow.max_num_filters=1024 gen.flow.multi_spade_combine.embed.num_filters=32 \
  gen.embed.num_filters=32 gen.embed.max_num_filters=1024 dis.image.num_filters=64 \
  dis.image.max_num_filters=512 dis.temporal.num_filters=64 dis.temporal.max_num_filters=512 \
  data.train.batch_size=2 data.train.augmentations.resize_h_w=512,1024 \
  data.val.augmentations.resize_h_w=512,1024
cat gpurun_out/recipes.jsonl
