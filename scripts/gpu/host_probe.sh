#!/bin/bash
# Where does a SPADE step spend host time? cProfile of a short bench, then the
# same bench with PyTorch's MIOpen find-and-cache path (benchmark=True) in FAST
# find mode (no exhaustive tuning).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m cProfile -o gpurun_out/bench.cprof bench.py --steps 3 --warmup 2 \
  > gpurun_out/bench_cprof.json 2> gpurun_out/bench_cprof.err
rc=$?; echo "[host_probe] cprof rc=$rc"; cat gpurun_out/bench_cprof.json
[ $rc -ne 0 ] && { tail -20 gpurun_out/bench_cprof.err; exit $rc; }
python - <<'PY' > gpurun_out/cprof_top.txt
import pstats
s = pstats.Stats('gpurun_out/bench.cprof')
s.sort_stats('tottime').print_stats(45)
s.sort_stats('cumulative').print_stats(45)
PY
head -80 gpurun_out/cprof_top.txt
IMAGINAIRE_AMD_MIOPEN_TUNE=1 MIOPEN_FIND_MODE=FAST timeout -k 10 600 python bench.py \
  --steps 5 --warmup 3 > gpurun_out/bench_fastfind.json 2> gpurun_out/bench_fastfind.err
rc=$?; echo "[host_probe] fastfind rc=$rc"; cat gpurun_out/bench_fastfind.json; tail -3 gpurun_out/bench_fastfind.err
exit $rc
