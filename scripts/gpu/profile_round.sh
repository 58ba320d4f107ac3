#!/bin/bash
# GPU-box job: MIOpen find-cost probe (no-benchmark vs benchmark) + rocprofv3 kernel
# stats of a short bench. Each GPU step under its own timeout; stop on any fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
mkdir -p gpurun_out/prof
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[profile_round] $name rc=$rc"
  tail -12 "$ROOT/gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
if [ -z "$SKIP_PROBE" ]; then
  step probe_nobench 300 python scripts/probe/conv_find_probe.py nobench
  step probe_bench 400 python scripts/probe/conv_find_probe.py bench
fi
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/iamd_prof
step rocprof 900 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/iamd_prof -o bench -- \
  python3 "$ROOT/bench.py" ${BENCH_ARGS:---steps 3 --warmup 2 --verbose}
cd "$ROOT"
# keep only the (small) summary tables; the full trace stays on the box
find /tmp/iamd_prof -name '*stats*.csv' -exec cp {} gpurun_out/prof/ \;
python3 scripts/gpu/summarize_kernels.py /tmp/iamd_prof > gpurun_out/prof/top_kernels.txt || true
head -60 gpurun_out/prof/top_kernels.txt
