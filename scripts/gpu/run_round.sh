#!/bin/bash
# GPU-box job: kernel tests -> smoke -> short bench. Stops on any fault/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
ok_or_stop() {  # rc 0/1 (test failures) continue; anything else (fault, abort, timeout) stops
  local rc=$1 what=$2
  echo "[run_round] $what rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "[run_round] stopping after $what"; exit $rc; fi
}
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest ${PYTEST_ARGS:-tests -m gpu} -x -q > gpurun_out/pytest_gpu.log 2>&1
ok_or_stop $? pytest
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
ok_or_stop $? smoke
tail -2 gpurun_out/smoke.log
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-900} python bench.py ${BENCH_ARGS:---steps 10 --warmup 5} > gpurun_out/bench.json 2> gpurun_out/bench.err
  ok_or_stop $? bench
  cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
fi
