#!/bin/bash
# GPU-box job (round 5): localise the few-shot vid2vid recipe divergence.
# Runs the 512x512 recipe (K from $K, default 1) eager and graph-replayed with every
# iteration's D/G losses printed, then graph runs with one round-4 feature switched off each
# ($SWITCHES). Each run stops the script on a crash / timeout; a NaN run (exit 3) continues.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r5fs
mkdir -p "$OUT"
K=${K:-1}
ARGS=(--config "$ROOT/configs/unit_test/fs_vid2vid_face.yaml" --seq-len 4 --print-losses --set
  gen.num_filters=32 gen.num_downsamples=5 gen.hyper.num_hyper_layers=4
  gen.hyper.attention.num_filters=32 gen.flow.num_filters=32 gen.flow.max_num_filters=1024
  gen.flow.num_res_blocks=6 gen.flow.multi_spade_combine.embed.num_filters=32
  gen.flow.multi_spade_combine.embed.num_downsamples=5 gen.embed.num_filters=32
  gen.embed.num_downsamples=5 dis.image.num_filters=32 dis.image.max_num_filters=512
  dis.image.num_layers=4 data.initial_few_shot_K=$K data.train.batch_size=3
  data.train.augmentations.resize_h_w=512,512 data.val.augmentations.resize_h_w=512,512)
: > "$OUT/fs_k$K.jsonl"
run() {  # tag, env..., -- extra args
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 ${T:-400} python scripts/bench_families.py "${ARGS[@]}" \
    --steps ${STEPS:-2} --warmup ${WARM:-6} --allow-nonfinite "$@" $EXTRA \
    >> "$OUT/fs_k$K.jsonl" 2> "$OUT/fs_k${K}_$tag.err"
  local rc=$?
  echo "[r5fs] $tag rc=$rc"
  grep "losses\|diag" "$OUT/fs_k${K}_$tag.err" | cut -c1-900
  [ $rc -eq 0 ] || { tail -15 "$OUT/fs_k${K}_$tag.err"; exit $rc; }
}
[ -z "$NOEAGER" ] && run eager X=1 --
[ -n "$EAGERONLY" ] && exit 0
run graph X=1 -- --graph
for sw in $SWITCHES; do
  run "graph_${sw%%=*}" "$sw" -- --graph
done
exit 0
