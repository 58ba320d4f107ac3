#!/bin/bash
# GPU-box job (round 4): pytest groups (each under its own time limit), then optional probes.
# An ordinary test failure (rc 1) moves on to the next group; a time limit, abort or crash
# (rc >= 124) stops the job.   TGROUPS="expr1;expr2"
# PROBES="python script args;VAR=1 python bench.py ..." (each entry run through env)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r4t
mkdir -p "$OUT"
IFS=";" read -ra GS <<< "${TGROUPS:-}"
i=0
worst=0
for g in "${GS[@]}"; do
  i=$((i+1))
  timeout -k 10 ${TLIM:-900} python -u -m pytest tests -m gpu -q --timeout 170 \
    --timeout-method thread -k "$g" > "$OUT/g$i.out" 2> "$OUT/g$i.err"
  rc=$?
  echo "[r4t] group $i '$g' rc=$rc"; tail -4 "$OUT/g$i.out"
  [ $rc -ge 124 ] && exit $rc
  [ $rc -gt $worst ] && worst=$rc
done
IFS=';' read -ra PS <<< "${PROBES:-}"
j=0
for p in "${PS[@]}"; do
  j=$((j+1))
  # an entry may start with VAR=value words: they are set for that probe only
  timeout -k 10 600 env $p > "$OUT/p$j.out" 2> "$OUT/p$j.err"
  rc=$?
  echo "[r4t] probe $j '$p' rc=$rc"; tail -${TAILN:-30} "$OUT/p$j.out"
  [ $rc -ne 0 ] && { tail -20 "$OUT/p$j.err"; exit $rc; }
done
exit $worst
