#!/bin/bash
# GPU-box job (round 4): few-shot vid2vid 512x512 at recipe widths with K = 2 reference frames
# (the attention runs), graph-replayed: k16 fused attention (default) vs PyTorch SDPA
# (IMAGINAIRE_AMD_FUSED_ATTN_KERNEL=0), then a rocprofv3 --stats pass of the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r4fs
mkdir -p "$OUT"
ARGS=(--config "$ROOT/configs/unit_test/fs_vid2vid_face.yaml" --seq-len 4 --graph --set
  gen.num_filters=32 gen.num_downsamples=5 gen.hyper.num_hyper_layers=4
  gen.hyper.attention.num_filters=32 gen.flow.num_filters=32 gen.flow.max_num_filters=1024
  gen.flow.num_res_blocks=6 gen.flow.multi_spade_combine.embed.num_filters=32
  gen.flow.multi_spade_combine.embed.num_downsamples=5 gen.embed.num_filters=32
  gen.embed.num_downsamples=5 dis.image.num_filters=32 dis.image.max_num_filters=512
  dis.image.num_layers=4 data.initial_few_shot_K=2 data.train.batch_size=3
  data.train.augmentations.resize_h_w=512,512 data.val.augmentations.resize_h_w=512,512)
: > "$OUT/fs_k2.jsonl"
for mode in 1 0 1; do
  IMAGINAIRE_AMD_FUSED_ATTN_KERNEL=$mode timeout -k 10 600 python scripts/bench_families.py \
    "${ARGS[@]}" --steps ${STEPS:-15} --warmup 4 >> "$OUT/fs_k2.jsonl" 2> "$OUT/fs_k2_$mode.err"
  rc=$?; echo "[r4fs] attn kernel=$mode rc=$rc"; tail -1 "$OUT/fs_k2.jsonl" | cut -c1-300
  [ $rc -eq 0 ] || { tail -15 "$OUT/fs_k2_$mode.err"; exit $rc; }
done
if [ -n "$PROF" ]; then
  rm -rf /tmp/iamd_fsprof
  (cd /tmp && TMPDIR=/tmp timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv \
    -d /tmp/iamd_fsprof -o run -- python3 "$ROOT/scripts/bench_families.py" "${ARGS[@]}" \
    --steps 3 --warmup 4 > "$OUT/fs_prof.log" 2>&1)
  rc=$?; echo "[r4fs] rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -15 "$OUT/fs_prof.log"; exit $rc; }
  python3 scripts/gpu/summarize_kernels.py /tmp/iamd_fsprof > "$OUT/fs_k2_kernels.txt"
  head -40 "$OUT/fs_k2_kernels.txt"
  grep -i "attn\|softmax\|gemm\|Cijk\|fmha\|flash" "$OUT/fs_k2_kernels.txt" | head -20
fi
exit 0
