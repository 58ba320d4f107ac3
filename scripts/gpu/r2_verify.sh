#!/bin/bash
# GPU-box job (round 2, verification batch): model-level HIP-vs-eager parity tests and the new
# kernel backward tests, then the metric's missing halves: eager self-baseline of the SPADE
# step, hipGraph on/off A/B, FID pipeline throughput (HIP and eager). Every GPU step has its own
# time limit; the script stops at the first fault / abort / timeout (test failures: rc 1, go on).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/verify
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/verify/$name.out" 2> "gpurun_out/verify/$name.err"
  local rc=$?
  echo "[verify] $name rc=$rc"; tail -4 "gpurun_out/verify/$name.out"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -20 "gpurun_out/verify/$name.err"; exit $rc; fi
}
if [ -z "$SKIP_TESTS" ]; then
  run tests 600 python -u -m pytest ${TESTS:-tests/test_model_parity_gpu.py tests/test_spade_dis_semantics_cpu.py tests/test_kernels_gpu.py} \
    -m gpu -q -rA --timeout 300 --timeout-method thread ${KFILTER:+-k "$KFILTER"}
fi
[ -n "$NOGRAPH" ] && run bench_nograph 400 python bench.py --steps 10 --warmup 3 --no-graph
[ -n "$EAGER" ] && run bench_eager 600 python bench.py --steps 5 --warmup 2 --eager
[ -n "$FID" ] && run fid 400 python scripts/bench_fid.py
[ -n "$FID" ] && run fid_eager 500 python scripts/bench_fid.py --eager
exit 0
