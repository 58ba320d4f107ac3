#!/bin/bash
# GPU-box job (round 6): what does the HIP runtime's graph packet-capture mode break?
# (1) long dependent chains of PyTorch kernels, D2D memcpy nodes and framework HIP kernels,
#     replayed with packet capture on and off; (2) the node kinds / edges of the few-shot
#     vid2vid recipe's captured graph (hipGraphDebugDotPrint).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6graph
mkdir -p "$OUT"
for pc in 1 0; do
  for mode in kernel copy hip; do
    DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc MODE=$mode timeout -k 10 240 python -u \
      scripts/probe/graph_coherence_probe.py ${N:-20000} ${S:-4194304} 3 \
      > "$OUT/coh_pc${pc}_$mode.log" 2>&1
    rc=$?; echo "[coh] pc=$pc mode=$mode rc=$rc: $(tail -1 $OUT/coh_pc${pc}_$mode.log)"
    [ $rc -eq 0 ] || exit $rc
  done
done
[ -n "$NODOT" ] && exit 0
IMAGINAIRE_AMD_GRAPH_DOT=/tmp/fs_graph.dot timeout -k 10 600 python -u scripts/bench_families.py \
  --config configs/unit_test/fs_vid2vid_face.yaml --graph --steps 2 --warmup 3 \
  --seq-len 4 --set gen.num_filters=32 gen.num_downsamples=5 gen.hyper.num_hyper_layers=4 \
  gen.hyper.attention.num_filters=32 gen.flow.num_filters=32 gen.flow.max_num_filters=1024 \
  gen.flow.num_res_blocks=6 gen.flow.multi_spade_combine.embed.num_filters=32 \
  gen.flow.multi_spade_combine.embed.num_downsamples=5 gen.embed.num_filters=32 \
  gen.embed.num_downsamples=5 dis.image.num_filters=32 dis.image.max_num_filters=512 \
  dis.image.num_layers=4 data.initial_few_shot_K=1 data.train.batch_size=3 \
  data.train.augmentations.resize_h_w=512,512 data.val.augmentations.resize_h_w=512,512 \
  > "$OUT/fs_dot.log" 2>&1
rc=$?; echo "[dot] fs rc=$rc"; tail -3 "$OUT/fs_dot.log"
ls -la /tmp/fs_graph.dot* 2>/dev/null
for f in /tmp/fs_graph.dot*; do
  [ -f "$f" ] || continue
  head -c 3000 "$f" > "$OUT/$(basename $f).head.txt"
  python scripts/probe/graph_dot.py "$f" > "$OUT/$(basename $f).summary.txt" 2>&1
  cat "$OUT/$(basename $f).summary.txt" | head -40
done
exit $rc
