#!/bin/bash
# GPU-box job: the BASELINE families with a published (derived) per-node throughput, at their
# recipe scale on one MI355X, synthetic data: pix2pixHD Cityscapes ampO1 (512x1024, batch 2,
# 64-filter global G with 9 res blocks, 2-scale D; reference ~16.5 img/s per 8xV100 node) and
# FUNIT AnimalFaces base64_bs8_class149 (256x256, batch 8; reference ~15.9 pairs/s per node).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/recipes2
: > gpurun_out/recipes2/recipes.jsonl
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" python scripts/bench_families.py "$@" --conv-log \
    >> gpurun_out/recipes2/recipes.jsonl 2> gpurun_out/recipes2/$name.err
  local rc=$?
  echo "[recipes2] $name rc=$rc"; tail -1 gpurun_out/recipes2/recipes.jsonl
  [ $rc -eq 0 ] || { tail -5 gpurun_out/recipes2/$name.err; exit $rc; }
}
run pix2pixhd512x1024 500 --config configs/unit_test/pix2pixHD.yaml --steps 5 --warmup 2 --set \
  gen.global_generator.num_filters=64 gen.global_generator.num_res_blocks=9 \
  dis.num_filters=64 dis.num_discriminators=2 data.train.batch_size=2 trainer.model_average=True \
  trainer.model_average_beta=0.999 trainer.model_average_start_iteration=0 \
  trainer.model_average_batch_norm_estimation_iteration=0 \
  data.train.augmentations.resize_h_w=512,1024 data.val.augmentations.resize_h_w=512,1024
run funit256 500 --config configs/unit_test/funit.yaml --steps 5 --warmup 2 --set \
  gen.num_filters=64 gen.num_filters_mlp=256 gen.style_dims=64 gen.num_downsamples_content=4 \
  gen.num_downsamples_style=5 dis.num_filters=64 dis.max_num_filters=1024 dis.num_layers=6 \
  dis.num_classes=149 data.num_style_classes=149 data.train.batch_size=8 \
  data.train.augmentations.random_crop_h_w=256,256 data.val.augmentations.center_crop_h_w=256,256
exit 0
