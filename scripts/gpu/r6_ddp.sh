#!/bin/bash
# GPU-box job (round 6): DDP zero-copy / per-net communicator tests, SN module.weight test, the
# memset-order graph test, then the SPADE bench plain vs forced one-rank distributed (the DDP
# wrapper's overhead at world 1), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6ddp
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py tests/test_sn_fused_gpu.py \
  "tests/test_graph_gpu.py::test_package_default_orders_memset_nodes" -x -v --timeout 200 \
  --timeout-method thread -p no:cacheprovider > "$OUT/tests.log" 2>&1
rc=$?; echo "[ddp] tests rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" "$OUT/tests.log" | tail -14; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for arm in plain forced; do
    extra=""; [ $arm = forced ] && extra="--force-dist"
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 6 $extra > "$OUT/bench_${arm}_$r.log" 2>&1
    rc=$?; echo "[ddp] bench $arm $r rc=$rc: $(tail -1 $OUT/bench_${arm}_$r.log | cut -c1-200)"
    [ $rc -eq 0 ] || exit $rc
  done
done
