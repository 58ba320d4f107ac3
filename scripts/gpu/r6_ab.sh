#!/bin/bash
# GPU-box job (round 6): same-box A/B of the graphed recipes: every round-6 conv routing off
# (IMAGINAIRE_AMD_TAPPACK=0 IMAGINAIRE_AMD_CONV_RW=0, i.e. the round-5 routing) vs default,
# alternating, REPS times each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6ab
mkdir -p "$OUT"
: > "$OUT/ab.jsonl"
for r in $(seq 1 ${REPS:-1}); do
  for arm in off on; do
    if [ $arm = off ]; then export IMAGINAIRE_AMD_TAPPACK=0 IMAGINAIRE_AMD_CONV_RW=0; else unset IMAGINAIRE_AMD_TAPPACK IMAGINAIRE_AMD_CONV_RW; fi
    EXTRA=--graph REPS=1 STEPS=${STEPS:-12} ONLY="${ONLY:-munit256 funit256 pix2pixhd512x1024}" \
      bash scripts/gpu/r5_recipes.sh > "$OUT/run_${arm}_$r.log" 2>&1
    rc=$?
    python3 - "$arm" >> "$OUT/ab.jsonl" <<'PY'
import json, sys
for l in open('gpurun_out/r5rec/recipes.jsonl'):
    try:
        d = json.loads(l)
    except Exception:
        continue
    print(json.dumps({'arm': sys.argv[1], 'family': d.get('family'), 'samples_per_s': d.get('samples_per_s'),
                      'ms': d.get('median_ms'), 'finite': d.get('losses_finite')}))
PY
    tail -3 "$OUT/ab.jsonl"
    [ $rc -eq 0 ] || exit $rc
  done
done
