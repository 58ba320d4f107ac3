#!/bin/bash
# GPU-box job: kernel tests touched by the last changes, then op-site attribution + conv log of
# the vid2vid 512x1024 recipe iteration and the MUNIT recipe conv log.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/sites
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -rf --timeout 120 \
  --timeout-method thread -k "${KFILTER:-multitap or per_sample or conv2d_mfma or pad_nhwc}" \
  > gpurun_out/sites/tests.out 2>&1
rc=$?; echo "[sites] tests rc=$rc"; tail -3 gpurun_out/sites/tests.out
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python scripts/bench_families.py --config configs/unit_test/vid2vid_street.yaml \
  --steps 2 --warmup 2 --seq-len 3 --op-sites --conv-log --set gen.num_filters=32 \
  gen.max_num_filters=1024 gen.flow.num_filters=32 gen.flow.max_num_filters=1024 \
  gen.flow.multi_spade_combine.embed.num_filters=32 gen.embed.num_filters=32 \
  gen.embed.max_num_filters=1024 dis.image.num_filters=64 dis.image.max_num_filters=512 \
  dis.temporal.num_filters=64 dis.temporal.max_num_filters=512 data.train.batch_size=2 \
  data.train.augmentations.resize_h_w=512,1024 data.val.augmentations.resize_h_w=512,1024 \
  > gpurun_out/sites/vid2vid.out 2> gpurun_out/sites/vid2vid.err
rc=$?; echo "[sites] vid2vid rc=$rc"; tail -1 gpurun_out/sites/vid2vid.out
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/bench_families.py --config configs/unit_test/munit.yaml --steps 3 \
  --warmup 2 --conv-log --op-sites --set gen.num_filters=64 gen.num_filters_mlp=256 \
  gen.num_res_blocks=4 dis.num_filters=32 dis.max_num_filters=512 dis.num_layers=6 \
  trainer.loss_weight.perceptual=0 data.train.batch_size=16 \
  data.train.augmentations.random_crop_h_w=256,256 > gpurun_out/sites/munit.out 2> gpurun_out/sites/munit.err
rc=$?; echo "[sites] munit rc=$rc"; tail -1 gpurun_out/sites/munit.out
exit $rc
