#!/bin/bash
# GPU tests + smoke + 1-GPU bench + a 2-rank DDP rehearsal on the single GPU
# (gloo, --share-gpu) to exercise bucketed all-reduce with channels-last grads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
BENCH_ARGS="--steps 10 --warmup 3" bash scripts/gpu/run_round.sh || exit $?
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 2 --warmup 2 \
  --backend gloo --share-gpu > gpurun_out/bench_ddp2.json 2> gpurun_out/bench_ddp2.err
rc=$?; echo "[validate] ddp2 rc=$rc"; cat gpurun_out/bench_ddp2.json; tail -5 gpurun_out/bench_ddp2.err
exit $rc
