#!/bin/bash
# Every model family's training iteration on the GPU (unit-test configs, synthetic data):
# one JSON line per family into gpurun_out/families.jsonl; stops at the first fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
: > gpurun_out/families.jsonl
for cfg in spade pix2pixHD munit munit_patch unit funit coco_funit vid2vid_street vid2vid_pose fs_vid2vid_face fs_vid2vid_pose wc_vid2vid; do
  extra=""
  case $cfg in vid2vid*|fs_vid2vid*|wc_vid2vid) extra="--seq-len 3";; esac
  timeout -k 10 300 python scripts/bench_families.py --config configs/unit_test/$cfg.yaml \
    --steps 5 --warmup 2 $extra >> gpurun_out/families.jsonl 2> gpurun_out/family_$cfg.err
  rc=$?
  echo "[families] $cfg rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/family_$cfg.err; [ $rc -eq 1 ] || exit $rc; fi
done
cat gpurun_out/families.jsonl
