#!/bin/bash
# GPU-box job (round 5): the fused spectral-norm conv path — numerics tests, the SN / graph /
# recipe GPU tests, then bench.py with the path off and on (same steps), per-kernel profile of
# the fused step (r5_sn_prof.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/sn5
rm -rf "$OUT"; mkdir -p "$OUT"
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_sn_fused_gpu.py tests/test_kernels_gpu.py -k "spectral or sn_ or fused" \
  > "$OUT/tests_sn.log" 2>&1; rc=$?; tail -3 "$OUT/tests_sn.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 $T tests/test_graph_gpu.py tests/test_recipe_finite_gpu.py \
  > "$OUT/tests_graph.log" 2>&1; rc=$?; tail -3 "$OUT/tests_graph.log"; [ $rc -eq 0 ] || exit $rc
for f in 0 1; do
  IMAGINAIRE_AMD_SN_FUSED=$f timeout -k 10 400 python -u bench.py --steps 20 --warmup 6 \
    > "$OUT/bench_sn$f.log" 2>&1; rc=$?; tail -1 "$OUT/bench_sn$f.log"; [ $rc -eq 0 ] || exit $rc
done
FUSED=1 bash "$ROOT/scripts/gpu/r5_sn_prof.sh"
