#!/bin/bash
# Per-(conv, input shape) GPU time of one SPADE training step (torch.profiler, CUDA activity).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 1 --warmup 3 --conv-profile \
  > gpurun_out/bench_convprof.json 2> gpurun_out/bench_convprof.err
rc=$?; echo "[convprof] rc=$rc"; grep -A62 "conv GPU time" gpurun_out/bench_convprof.err
exit $rc
