#!/bin/bash
# GPU-box job (round 5): BASELINE secondary configs at recipe scale (graph: EXTRA=--graph), with
# finite-loss checks (bench_families.py exits 3 on a NaN row), measured with hygiene:
# 20 timed iterations (each synchronised: median / min / max / spread) after 4 warm-up ones,
# in REPS fresh processes (default 2), routing decisions recorded in each jsonl row. The first
# process of each config also prints the conv log; PROF=1 adds a rocprofv3 --stats run whose
# breakdown starts at the steady-state marker bench_families.py emits after warm-up.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=${OUTDIR:-$ROOT/gpurun_out/r5rec}
mkdir -p "$OUT"
OUT=$(cd "$OUT" && pwd)  # (absolute: the profiling runs start from /tmp)
: > "$OUT/recipes.jsonl"
REPS=${REPS:-2}
STEPS=${STEPS:-20}
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  if [ -n "$ONLY" ] && [[ " $ONLY " != *" $name "* ]]; then return 0; fi
  for rep in $(seq 1 "$REPS"); do
    local extra=""
    [ "$rep" = 1 ] && [ -n "$CONVLOG" ] && extra="--conv-log"
    timeout -k 10 "$t" python scripts/bench_families.py "$@" --steps "$STEPS" --warmup 4 $extra $EXTRA \
      >> "$OUT/recipes.jsonl" 2> "$OUT/${name}_$rep.err"
    local rc=$?
    echo "[r5rec] $name rep $rep rc=$rc"; tail -1 "$OUT/recipes.jsonl" | cut -c1-400
    if [ $rc -ne 0 ]; then tail -8 "$OUT/${name}_$rep.err"; exit $rc; fi
  done
  if [ -n "$PROF" ]; then
    rm -rf /tmp/iamd_rprof
    local args=()
    for a in "$@"; do
      if [[ "$a" == configs/* ]]; then args+=("$ROOT/$a"); else args+=("$a"); fi
    done
    (cd /tmp && TMPDIR=/tmp timeout -k 10 "$t" rocprofv3 --kernel-trace --stats --output-format csv \
      -d /tmp/iamd_rprof -o run -- python3 "$ROOT/scripts/bench_families.py" "${args[@]}" \
      --steps 5 --warmup 4 $EXTRA > "$OUT/${name}_prof.log" 2>&1)
    local prc=$?
    echo "[r5rec] $name rocprof rc=$prc"
    [ $prc -eq 0 ] || exit $prc
    python3 scripts/gpu/summarize_kernels.py /tmp/iamd_rprof > "$OUT/${name}_kernels.txt"
    head -25 "$OUT/${name}_kernels.txt"
  fi
}
run munit256 500 --config configs/unit_test/munit.yaml --set \
  gen.num_filters=64 gen.num_filters_mlp=256 gen.num_res_blocks=4 \
  dis.num_filters=32 dis.max_num_filters=512 dis.num_layers=6 trainer.loss_weight.perceptual=0 \
  trainer.loss_weight.gp=0 trainer.loss_weight.consistency_reg=0 \
  data.train.batch_size=16 data.train.augmentations.random_crop_h_w=256,256
run vid2vid512x1024 700 --config configs/unit_test/vid2vid_street.yaml \
  --seq-len 3 --set gen.num_filters=32 gen.max_num_filters=1024 gen.flow.num_filters=32 \
  gen.flow.max_num_filters=1024 gen.flow.multi_spade_combine.embed.num_filters=32 \
  gen.embed.num_filters=32 gen.embed.max_num_filters=1024 dis.image.num_filters=64 \
  dis.image.max_num_filters=512 dis.temporal.num_filters=64 dis.temporal.max_num_filters=512 \
  data.train.batch_size=2 data.train.augmentations.resize_h_w=512,1024 \
  data.val.augmentations.resize_h_w=512,1024
run fsvid2vid512 700 --config configs/unit_test/fs_vid2vid_face.yaml \
  --seq-len 4 --set gen.num_filters=32 gen.num_downsamples=5 gen.hyper.num_hyper_layers=4 \
  gen.hyper.attention.num_filters=32 gen.flow.num_filters=32 gen.flow.max_num_filters=1024 \
  gen.flow.num_res_blocks=6 gen.flow.multi_spade_combine.embed.num_filters=32 \
  gen.flow.multi_spade_combine.embed.num_downsamples=5 gen.embed.num_filters=32 \
  gen.embed.num_downsamples=5 dis.image.num_filters=32 dis.image.max_num_filters=512 \
  dis.image.num_layers=4 data.initial_few_shot_K=1 data.train.batch_size=3 \
  data.train.augmentations.resize_h_w=512,512 data.val.augmentations.resize_h_w=512,512
run fsvid2vid512k2 700 --config configs/unit_test/fs_vid2vid_face.yaml \
  --seq-len 4 --set gen.num_filters=32 gen.num_downsamples=5 gen.hyper.num_hyper_layers=4 \
  gen.hyper.attention.num_filters=32 gen.flow.num_filters=32 gen.flow.max_num_filters=1024 \
  gen.flow.num_res_blocks=6 gen.flow.multi_spade_combine.embed.num_filters=32 \
  gen.flow.multi_spade_combine.embed.num_downsamples=5 gen.embed.num_filters=32 \
  gen.embed.num_downsamples=5 dis.image.num_filters=32 dis.image.max_num_filters=512 \
  dis.image.num_layers=4 data.initial_few_shot_K=2 data.train.batch_size=3 \
  data.train.augmentations.resize_h_w=512,512 data.val.augmentations.resize_h_w=512,512
run pix2pixhd512x1024 600 --config configs/unit_test/pix2pixHD.yaml --set \
  gen.global_generator.num_filters=64 gen.global_generator.num_res_blocks=9 \
  dis.num_filters=64 dis.num_discriminators=2 data.train.batch_size=2 trainer.model_average=True \
  trainer.model_average_beta=0.999 trainer.model_average_start_iteration=0 \
  trainer.model_average_batch_norm_estimation_iteration=0 \
  data.train.augmentations.resize_h_w=512,1024 data.val.augmentations.resize_h_w=512,1024
run funit256 500 --config configs/unit_test/funit.yaml --set \
  gen.num_filters=64 gen.num_filters_mlp=256 gen.style_dims=64 gen.num_downsamples_content=4 \
  gen.num_downsamples_style=5 dis.num_filters=64 dis.max_num_filters=1024 dis.num_layers=6 \
  dis.num_classes=149 data.num_style_classes=149 data.train.batch_size=8 \
  data.train.augmentations.random_crop_h_w=256,256 data.val.augmentations.center_crop_h_w=256,256
exit 0
