#!/bin/bash
# GPU-box job (round 6): (1) MFMA shape probe; (2) the few-shot vid2vid K=1 recipe replayed with
# the runtime's packet capture ON (the round-5 NaN trigger) at HEAD, 8 steps, losses printed;
# (3) the DOT dump of its captured graph (packet capture off) and its node / edge summary.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6graph2
mkdir -p "$OUT"
timeout -k 10 120 ./scripts/probe/native/mfma_shape_probe 20000 > "$OUT/mfma_shape.txt" 2>&1
rc=$?; echo "[g2] mfma rc=$rc"; cat "$OUT/mfma_shape.txt"; [ $rc -eq 0 ] || exit $rc
ARGS=(--config configs/unit_test/fs_vid2vid_face.yaml --graph --seq-len 4 --set gen.num_filters=32
  gen.num_downsamples=5 gen.hyper.num_hyper_layers=4 gen.hyper.attention.num_filters=32
  gen.flow.num_filters=32 gen.flow.max_num_filters=1024 gen.flow.num_res_blocks=6
  gen.flow.multi_spade_combine.embed.num_filters=32 gen.flow.multi_spade_combine.embed.num_downsamples=5
  gen.embed.num_filters=32 gen.embed.num_downsamples=5 dis.image.num_filters=32
  dis.image.max_num_filters=512 dis.image.num_layers=4 data.initial_few_shot_K=1
  data.train.batch_size=3 data.train.augmentations.resize_h_w=512,512
  data.val.augmentations.resize_h_w=512,512)
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 IMAGINAIRE_AMD_GRAPH_ALLOW_PACKET_CAPTURE=1 timeout -k 10 400 \
  python -u scripts/bench_families.py "${ARGS[@]}" --steps 8 --warmup 4 --print-losses \
  --allow-nonfinite > "$OUT/fs_pc1.jsonl" 2> "$OUT/fs_pc1.err"
rc=$?; echo "[g2] fs packet-capture-on rc=$rc"; grep -E "losses|graph\]" "$OUT/fs_pc1.err" | cut -c1-300 | head -20
tail -1 "$OUT/fs_pc1.jsonl" | cut -c1-300; [ $rc -eq 0 ] || exit $rc
IMAGINAIRE_AMD_GRAPH_DOT=/tmp/fs_graph.dot timeout -k 10 400 python -u scripts/bench_families.py \
  "${ARGS[@]}" --steps 2 --warmup 3 > "$OUT/fs_dot.jsonl" 2> "$OUT/fs_dot.err"
rc=$?; echo "[g2] dot rc=$rc"; ls -la /tmp/fs_graph.dot* 2>/dev/null
for f in /tmp/fs_graph.dot*; do
  [ -f "$f" ] || continue
  head -c 4000 "$f" > "$OUT/$(basename $f).head.txt"
  timeout -k 10 300 python scripts/probe/graph_dot.py "$f" > "$OUT/$(basename $f).summary.txt" 2>&1
  head -40 "$OUT/$(basename $f).summary.txt"
done
exit $rc
