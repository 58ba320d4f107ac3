#!/bin/bash
# GPU-box job: video-family parity + family iterations, then the vid2vid / fs_vid2vid recipes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/video
timeout -k 10 400 python -u -m pytest tests/test_model_parity_gpu.py -q --timeout 300 \
  --timeout-method thread > gpurun_out/video/parity.out 2>&1
rc=$?; echo "[video] parity rc=$rc"; tail -2 gpurun_out/video/parity.out
[ $rc -eq 0 ] || exit $rc
for cfg in vid2vid_street vid2vid_pose fs_vid2vid_face fs_vid2vid_pose wc_vid2vid; do
  timeout -k 10 300 python scripts/bench_families.py --config configs/unit_test/$cfg.yaml --steps 2 \
    --warmup 1 >> gpurun_out/video/families.jsonl 2> gpurun_out/video/$cfg.err
  rc=$?; echo "[video] $cfg rc=$rc"; tail -1 gpurun_out/video/families.jsonl | cut -c1-200
  [ $rc -eq 0 ] || { tail -5 gpurun_out/video/$cfg.err; exit $rc; }
done
bash scripts/gpu/recipes_round.sh
