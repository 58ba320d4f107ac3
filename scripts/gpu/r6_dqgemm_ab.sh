#!/bin/bash
# GPU-box job (round 6): few-shot vid2vid K=2 recipe (graph) with the k16 dQ from the stored dS^T
# by one GEMM (IMAGINAIRE_AMD_ATTN_DQ_GEMM=1, default) vs the dQ kernel (0), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6dqab; mkdir -p $OUT
for round in 1 2; do
  for g in 1 0; do
    IMAGINAIRE_AMD_ATTN_DQ_GEMM=$g OUTDIR=$OUT/g${g}_$round ONLY=fsvid2vid512k2 REPS=1 EXTRA=--graph \
      bash scripts/gpu/r5_recipes.sh > $OUT/g${g}_$round.log 2>&1 || { tail -5 $OUT/g${g}_$round.log; exit 1; }
    python3 - "$OUT/g${g}_$round/recipes.jsonl" "$g" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('dq_gemm=%s frames/s %.3f (pipelined %.3f) ms/iter %.2f losses_finite %s' % (
    sys.argv[2], d['frames_per_s'], d.get('frames_per_s_pipelined', float('nan')),
    d['ms_per_iteration'], d.get('losses_finite')))
PY
  done
done
