#!/bin/bash
# GPU-box job: one short training run of every family's unit-test config (HIP path).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/fam
: > gpurun_out/fam/families.jsonl
for cfg in spade pix2pixHD munit munit_patch unit funit coco_funit vid2vid_street vid2vid_pose \
           fs_vid2vid_face fs_vid2vid_pose wc_vid2vid; do
  timeout -k 10 300 python scripts/bench_families.py --config configs/unit_test/$cfg.yaml --steps 2 \
    --warmup 1 >> gpurun_out/fam/families.jsonl 2> gpurun_out/fam/$cfg.err
  rc=$?; echo "[fam] $cfg rc=$rc"; tail -1 gpurun_out/fam/families.jsonl | cut -c1-160
  [ $rc -eq 0 ] || { tail -5 gpurun_out/fam/$cfg.err; exit $rc; }
done
