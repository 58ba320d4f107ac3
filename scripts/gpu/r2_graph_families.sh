#!/bin/bash
# GPU-box job: every family's unit config eager vs hipGraph-replayed (losses + throughput).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/gf
: > gpurun_out/gf/results.jsonl
for cfg in ${CFGS:-munit unit funit coco_funit pix2pixHD vid2vid_street fs_vid2vid_face wc_vid2vid}; do
  for mode in eager graph; do
    extra=""; [ $mode = graph ] && extra="--graph"
    timeout -k 10 300 python scripts/bench_families.py --config configs/unit_test/$cfg.yaml --steps 4 \
      --warmup 3 --pool 1 $extra >> gpurun_out/gf/results.jsonl 2> gpurun_out/gf/${cfg}_$mode.err
    rc=$?; echo "[gf] $cfg $mode rc=$rc"; tail -1 gpurun_out/gf/results.jsonl | cut -c1-300
    grep "\[graph\]" gpurun_out/gf/${cfg}_$mode.err | tail -1
    [ $rc -eq 0 ] || { tail -4 gpurun_out/gf/${cfg}_$mode.err; exit $rc; }
  done
done
