#!/bin/bash
# BASELINE.json secondary configs at their recipe scale (reference project configs' model widths,
# batch and crop) on one MI355X, synthetic data: unit-test configs scaled up with --set.
# Each run also prints the per-conv timing log of one extra iteration (stderr) and, with PROF=1,
# runs once more under rocprofv3 --stats for the kernel breakdown.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
mkdir -p gpurun_out/recipes
: > gpurun_out/recipes/recipes.jsonl
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  if [ -n "$ONLY" ] && [[ " $ONLY " != *" $name "* ]]; then return 0; fi
  timeout -k 10 "$t" python scripts/bench_families.py "$@" --conv-log $EXTRA \
    >> gpurun_out/recipes/recipes.jsonl 2> gpurun_out/recipes/$name.err
  local rc=$?
  echo "[recipes] $name rc=$rc"; tail -1 gpurun_out/recipes/recipes.jsonl
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/recipes/$name.err; [ $rc -eq 1 ] || exit $rc; fi
  if [ -n "$PROF" ]; then
    rm -rf /tmp/iamd_rprof
    # absolute config path: the profiled run starts in /tmp
    local args=()
    for a in "$@"; do
      if [[ "$a" == configs/* ]]; then args+=("$ROOT/$a"); else args+=("$a"); fi
    done
    (cd /tmp && TMPDIR=/tmp timeout -k 10 "$t" rocprofv3 --kernel-trace --stats --output-format csv \
      -d /tmp/iamd_rprof -o run -- python3 "$ROOT/scripts/bench_families.py" "${args[@]}" \
      > "$ROOT/gpurun_out/recipes/${name}_prof.log" 2>&1)
    local prc=$?
    echo "[recipes] $name rocprof rc=$prc"
    [ $prc -eq 0 ] || exit $prc
    python3 scripts/gpu/summarize_kernels.py /tmp/iamd_rprof > gpurun_out/recipes/${name}_kernels.txt
    head -25 gpurun_out/recipes/${name}_kernels.txt
  fi
}
# MUNIT afhq_dog2cat ampO1 recipe: 256x256, batch 16 (gp 0 and consistency_reg 0, as the recipe)
run munit256 400 --config configs/unit_test/munit.yaml --steps 5 --warmup 2 --set \
  gen.num_filters=64 gen.num_filters_mlp=256 gen.num_res_blocks=4 \
  dis.num_filters=32 dis.max_num_filters=512 dis.num_layers=6 trainer.loss_weight.perceptual=0 \
  trainer.loss_weight.gp=0 trainer.loss_weight.consistency_reg=0 \
  data.train.batch_size=16 data.train.augmentations.random_crop_h_w=256,256
# vid2vid cityscapes ampO1 recipe: 512x1024, batch 2, 3-frame sequences, FlowNet2 flow loss
run vid2vid512x1024 600 --config configs/unit_test/vid2vid_street.yaml --steps 3 --warmup 2 \
  --seq-len 3 --set gen.num_filters=32 gen.max_num_filters=1024 gen.flow.num_filters=32 \
  gen.flow.max_num_filters=1024 gen.flow.multi_spade_combine.embed.num_filters=32 \
  gen.embed.num_filters=32 gen.embed.max_num_filters=1024 dis.image.num_filters=64 \
  dis.image.max_num_filters=512 dis.temporal.num_filters=64 dis.temporal.max_num_filters=512 \
  data.train.batch_size=2 data.train.augmentations.resize_h_w=512,1024 \
  data.val.augmentations.resize_h_w=512,1024
# fs_vid2vid faceForensics ampO1 recipe: 512x512, batch 3, 1-shot, 4-frame sequences (4 warm-up
# iterations: with 2, one-off first-time work leaked into the timed ones: 26-40 frames/s)
run fsvid2vid512 600 --config configs/unit_test/fs_vid2vid_face.yaml --steps 4 --warmup 4 \
  --seq-len 4 --set gen.num_filters=32 gen.num_downsamples=5 gen.hyper.num_hyper_layers=4 \
  gen.hyper.attention.num_filters=32 gen.flow.num_filters=32 gen.flow.max_num_filters=1024 \
  gen.flow.num_res_blocks=6 gen.flow.multi_spade_combine.embed.num_filters=32 \
  gen.flow.multi_spade_combine.embed.num_downsamples=5 gen.embed.num_filters=32 \
  gen.embed.num_downsamples=5 dis.image.num_filters=32 dis.image.max_num_filters=512 \
  dis.image.num_layers=4 data.initial_few_shot_K=1 data.train.batch_size=3 \
  data.train.augmentations.resize_h_w=512,512 data.val.augmentations.resize_h_w=512,512
cat gpurun_out/recipes/recipes.jsonl
