#!/bin/bash
# GPU-box job (round 5): PMC passes (one rocprofv3 run per pass) over one conv shape per mode:
# MFMA busy, issue stalls, LDS traffic / conflicts, L2 hits. SHAPE / MODES overridable.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc5
rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SHAPE=${SHAPE:-"4 128 1024 128 256 5"}
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
P2="SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY"
P3="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"
for mode in ${MODES:-wgrad fwd}; do
  echo "$SHAPE" > "$OUT/$mode.shape"
  for pass in 1 2 3; do
    eval "CTRS=\$P$pass"
    rm -rf /tmp/pmc_$mode$pass
    timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d /tmp/pmc_$mode$pass -o run -- \
      python3 "$ROOT/scripts/probe/conv_kernel_driver.py" $mode $SHAPE 10 > "$OUT/${mode}_$pass.log" 2>&1
    rc=$?; echo "[pmc] $mode pass $pass rc=$rc"
    [ $rc -eq 0 ] || exit $rc
    find /tmp/pmc_$mode$pass -name '*counter_collection*.csv' -exec cp {} "$OUT/${mode}_$pass.csv" \;
  done
done
cd "$ROOT" && python3 scripts/gpu/pmc_summarize.py "$OUT" > "$OUT/summary.txt"; cat "$OUT/summary.txt"
