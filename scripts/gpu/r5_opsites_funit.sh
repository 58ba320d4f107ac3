#!/bin/bash
# GPU-box job (round 5): ATen glue by Python call site for the FUNIT recipe.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/opsites; mkdir -p $OUT
timeout -k 10 400 python -u scripts/bench_families.py --config configs/unit_test/funit.yaml --set \
  gen.num_filters=64 gen.num_filters_mlp=256 gen.style_dims=64 gen.num_downsamples_content=4 \
  gen.num_downsamples_style=5 dis.num_filters=64 dis.max_num_filters=1024 dis.num_layers=6 \
  dis.num_classes=149 data.num_style_classes=149 data.train.batch_size=8 \
  data.train.augmentations.random_crop_h_w=256,256 data.val.augmentations.center_crop_h_w=256,256 \
  --steps 2 --warmup 3 --op-sites > $OUT/funit2.log 2>&1
