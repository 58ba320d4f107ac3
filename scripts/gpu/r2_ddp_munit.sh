#!/bin/bash
# GPU-box job: distributed GPU tests (2-rank gloo SyncBN / DDP, RCCL world-1 DDP), the tap-split
# tests, then the MUNIT recipe (conv log + throughput). Stops at the first fault / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/dm
timeout -k 10 500 python -u -m pytest tests/test_distributed_gpu.py tests/test_kernels_gpu.py -q -rf \
  --timeout 240 --timeout-method thread -k "${KFILTER:-world or rccl or tapsplit}" > gpurun_out/dm/tests.out 2>&1
rc=$?; echo "[dm] tests rc=$rc"; tail -4 gpurun_out/dm/tests.out
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python scripts/bench_families.py --config configs/unit_test/munit.yaml --steps 5 \
  --warmup 2 --conv-log --set gen.num_filters=64 gen.num_filters_mlp=256 gen.num_res_blocks=4 \
  dis.num_filters=32 dis.max_num_filters=512 dis.num_layers=6 trainer.loss_weight.perceptual=0 \
  data.train.batch_size=16 data.train.augmentations.random_crop_h_w=256,256 \
  > gpurun_out/dm/munit.jsonl 2> gpurun_out/dm/munit.err
rc2=$?; echo "[dm] munit rc=$rc2"; tail -1 gpurun_out/dm/munit.jsonl
exit $(( rc > rc2 ? rc : rc2 ))
