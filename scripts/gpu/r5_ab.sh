#!/bin/bash
# GPU-box job (round 5): bench.py A/B over environment settings, back to back on one box.
#   AB="NAME=VALUE ..." entries separated by ';' (e.g. AB="X=0;X=1"), REPS per setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/ab5; mkdir -p $OUT
IFS=';' read -ra SETS <<< "${AB:-IMAGINAIRE_AMD_SN_FUSED=0;IMAGINAIRE_AMD_SN_FUSED=1}"
for rep in $(seq 1 ${REPS:-1}); do
  for s in "${SETS[@]}"; do
    tag=$(echo "$s" | tr ' =' '__')
    env $s timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 6 > $OUT/$tag.$rep.log 2>&1 || exit 1
    echo "[$s] rep $rep: $(tail -1 $OUT/$tag.$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
