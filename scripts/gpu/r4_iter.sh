#!/bin/bash
# GPU-box job (round 4): one build -> measure iteration. Steps chosen by env flags, each under
# its own time limit, stopping at the first failure:
#   TESTS=<pytest -k expr>  WPROBE=1  CPROBE=1  BENCH=1  OPS=1 (torch.profiler op attribution)
#   TRACE=1 (rocprofv3 steady-state kernel breakdown)  PROBE=<script args>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r4i
mkdir -p "$OUT"
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "[r4i] $name rc=$rc"; tail -${TAILN:-20} "$OUT/$name.out"
  if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.err"; exit $rc; fi
}
[ -z "$ALL" ] || run alltests 1100 python -u -m pytest tests -m gpu -x -q --timeout 120 \
  --timeout-method thread
[ -z "$TESTS" ] || run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "$TESTS"
[ -z "$WPROBE" ] || run wprobe 600 python scripts/probe/wgrad_v2_probe.py
[ -z "$CPROBE" ] || run cprobe 600 python scripts/probe/conv_v5_probe.py ${CVERS:-4,5}
[ -z "$PROBE" ] || run probe 600 python $PROBE
[ -z "$BENCH" ] || run bench 600 python bench.py --steps 20 --warmup 6
[ -z "$NOGRAPH" ] || run bench_nograph 600 python bench.py --steps 20 --warmup 6 --no-graph
# AB="VAR=val ...": the same bench again with those variables (same box: a fair A/B), then the
# default once more (order effects)
if [ -n "$AB" ]; then
  run bench_ab 600 env $AB python bench.py --steps 20 --warmup 6
  run bench_again 600 python bench.py --steps 20 --warmup 6
fi
[ -z "$CONVLOG" ] || run convlog 600 python bench.py --steps 1 --warmup 3 --conv-log
[ -z "$GRAPH" ] || run graph 1000 bash scripts/gpu/r3_graph.sh
[ -z "$OPS" ] || TAILN=60 run ops 600 python bench.py --steps 1 --warmup 3 --no-graph --op-profile --op-stack
if [ -n "$TRACE" ]; then
  cd /tmp && export TMPDIR=/tmp
  rm -rf /tmp/iamd_prof
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/iamd_prof -o bench -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 4 --verbose > "$OUT/trace.out" 2> "$OUT/trace.err"
  rc=$?; echo "[r4i] trace rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/trace.err"; exit $rc; }
  cd "$ROOT"
  python3 scripts/gpu/summarize_kernels.py /tmp/iamd_prof > "$OUT/top_kernels.txt" || true
  head -60 "$OUT/top_kernels.txt"
  find /tmp/iamd_prof -name '*kernel_trace.csv' -exec cp {} "$OUT/kernel_trace.csv" \; || true
fi
exit 0
