#!/bin/bash
# GPU-box job (round 6): memset graph nodes under packet capture (coherence probe, memset modes),
# then the few-shot vid2vid graph's non-kernel node neighbourhoods (DOT dump summary).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6graph3
mkdir -p "$OUT"
for pc in 1 0; do
  for mode in memset memset4; do
    DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc MODE=$mode timeout -k 10 240 python -u \
      scripts/probe/graph_coherence_probe.py ${N:-20000} ${S:-4194304} 3 \
      > "$OUT/coh_pc${pc}_$mode.log" 2>&1
    rc=$?; echo "[coh] pc=$pc mode=$mode rc=$rc: $(tail -1 $OUT/coh_pc${pc}_$mode.log)"
    [ $rc -eq 0 ] || exit $rc
  done
done
IMAGINAIRE_AMD_GRAPH_DOT=/tmp/fs_graph.dot timeout -k 10 400 python -u scripts/bench_families.py \
  --config configs/unit_test/fs_vid2vid_face.yaml --graph --seq-len 4 --steps 1 --warmup 3 --set \
  gen.num_filters=32 gen.num_downsamples=5 gen.hyper.num_hyper_layers=4 gen.hyper.attention.num_filters=32 \
  gen.flow.num_filters=32 gen.flow.max_num_filters=1024 gen.flow.num_res_blocks=6 \
  gen.flow.multi_spade_combine.embed.num_filters=32 gen.flow.multi_spade_combine.embed.num_downsamples=5 \
  gen.embed.num_filters=32 gen.embed.num_downsamples=5 dis.image.num_filters=32 \
  dis.image.max_num_filters=512 dis.image.num_layers=4 data.initial_few_shot_K=1 \
  data.train.batch_size=3 data.train.augmentations.resize_h_w=512,512 \
  data.val.augmentations.resize_h_w=512,512 > "$OUT/fs_dot.jsonl" 2> "$OUT/fs_dot.err"
rc=$?; echo "[g3] dot rc=$rc"
timeout -k 10 300 python scripts/probe/graph_dot.py /tmp/fs_graph.dot > "$OUT/fs_graph.summary.txt" 2>&1
gzip -c /tmp/fs_graph.dot > "$OUT/fs_graph.dot.gz"
sed -n '/non-kernel node neigh/,$p' "$OUT/fs_graph.summary.txt" | head -50
exit $rc
