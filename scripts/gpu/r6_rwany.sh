#!/bin/bash
# GPU-box job (round 6): row-window tile with any segment width — its tests, then MUNIT / FUNIT
# recipe A/B against power-of-two segments only (IMAGINAIRE_AMD_CONV_RW_POW2=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6rwany; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_conv_rw_gpu.py -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; echo "[rwany] tests rc=$rc"; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
MUNIT="--config configs/unit_test/munit.yaml --set gen.num_filters=64 gen.num_filters_mlp=256 \
  gen.num_res_blocks=4 dis.num_filters=32 dis.max_num_filters=512 dis.num_layers=6 \
  trainer.loss_weight.perceptual=0 trainer.loss_weight.gp=0 trainer.loss_weight.consistency_reg=0 \
  data.train.batch_size=16 data.train.augmentations.random_crop_h_w=256,256"
FUNIT="--config configs/unit_test/funit.yaml --set gen.num_filters=64 gen.num_filters_mlp=256 \
  gen.style_dims=64 gen.num_downsamples_content=4 gen.num_downsamples_style=5 dis.num_filters=64 \
  dis.max_num_filters=1024 dis.num_layers=6 dis.num_classes=149 data.num_style_classes=149 \
  data.train.batch_size=8 data.train.augmentations.random_crop_h_w=256,256 \
  data.val.augmentations.center_crop_h_w=256,256"
: > $OUT/ab.jsonl
for fam in MUNIT FUNIT; do
  eval "ARGS=\$$fam"
  for arm in any pow2 any2; do
    envs=""; [ $arm = pow2 ] && envs="IMAGINAIRE_AMD_CONV_RW_POW2=1"
    env $envs timeout -k 10 400 python scripts/bench_families.py $ARGS --steps 16 --warmup 4 --graph \
      > $OUT/${fam}_$arm.json 2> $OUT/${fam}_$arm.err
    rc=$?
    echo "{\"family\": \"$fam\", \"arm\": \"$arm\", \"rc\": $rc, \"row\": $(tail -1 $OUT/${fam}_$arm.json)}" >> $OUT/ab.jsonl
    echo "[rwany] $fam $arm rc=$rc $(python3 -c "import json,sys; r=json.loads(open('$OUT/${fam}_$arm.json').read().strip().splitlines()[-1]); print(r['frames_per_s'], r['frames_per_s_pipelined'], r['losses_finite'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
