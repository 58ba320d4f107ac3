#!/bin/bash
# GPU-box job: new kernel tests, bench (graph), FID throughput (HIP and eager), eager
# self-baseline of the SPADE step. Each step has its own time limit; stop at the first fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
  local rc=$?
  echo "[misc] $name rc=$rc"; tail -3 "gpurun_out/$name.out"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
run ktests 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 200 --timeout-method thread -k "${KTESTS:-k12 or padded}"
run bench 400 python bench.py --steps 20 --warmup 5
[ -n "$FID" ] && run fid 400 python scripts/bench_fid.py
[ -n "$FID" ] && run fid_eager 500 python scripts/bench_fid.py --eager
[ -n "$EAGER" ] && run bench_eager 600 python bench.py --steps 10 --warmup 3 --eager
exit 0
