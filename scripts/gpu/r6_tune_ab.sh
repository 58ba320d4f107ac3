#!/bin/bash
# GPU-box job (round 6): MUNIT / FUNIT recipes (graph) with the k11 wgrad autotuner timing its
# candidates over 3 interleaved rounds (default) vs 1, alternating, and the choices it made.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6tune; mkdir -p $OUT
for round in 1 2; do
  for t in 3 1; do
    IMAGINAIRE_AMD_TUNE_TRIALS=$t OUTDIR=$OUT/t${t}_$round ONLY="munit256 funit256" REPS=1 EXTRA=--graph \
      bash scripts/gpu/r5_recipes.sh > $OUT/t${t}_$round.log 2>&1 || { tail -5 $OUT/t${t}_$round.log; exit 1; }
    python3 - "$OUT/t${t}_$round/recipes.jsonl" "$t" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print('trials=%s %-12s frames/s %.2f (pipelined %.2f) routing %s' % (
        sys.argv[2], d['config'].split('/')[-1], d['frames_per_s'],
        d.get('frames_per_s_pipelined', float('nan')), json.dumps(d.get('routing', {}).get('wgrad'))))
PY
  done
done
