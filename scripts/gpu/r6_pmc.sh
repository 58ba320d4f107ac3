#!/bin/bash
# GPU-box job (round 6): PMC passes (one rocprofv3 run per pass, counters within the per-block
# limits) over the round's k10 / k11 tiles: v5 forward and k11 multi-tap weight gradient on the
# SPADE gamma|beta 5x5 shape, the 3x3 multi-tap weight gradient of the G 512-channel layers, and
# the row-window tile on a PatchGAN 4x4 stride-2 layer and a 7x7 stride-1 layer.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc6
rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
P2="SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY"
P3="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"
# tag mode B Cin Cout H W k stride
SPECS=(
  "v5fwd fwd 4 128 1024 128 256 5 1"
  "mt5wgrad wgrad 4 128 1024 128 256 5 1"
  "mt3wgrad wgrad 4 512 512 128 256 3 1"
  "rws2fwd fwd 8 128 256 128 256 4 2"
  "rw7fwd fwd 4 64 128 128 128 7 1"
)
for spec in "${SPECS[@]}"; do
  set -- $spec
  tag=$1; mode=$2; shift 2
  echo "$mode $*" > "$OUT/$tag.shape"
  for pass in 1 2 3; do
    eval "CTRS=\$P$pass"
    rm -rf /tmp/pmc_$tag$pass
    timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d /tmp/pmc_$tag$pass -o run -- \
      python3 "$ROOT/scripts/probe/conv_kernel_driver.py" $mode $1 $2 $3 $4 $5 $6 10 $7 \
      > "$OUT/${tag}_$pass.log" 2>&1
    rc=$?; echo "[pmc] $tag pass $pass rc=$rc $(grep done "$OUT/${tag}_$pass.log")"
    [ $rc -eq 0 ] || exit $rc
    find /tmp/pmc_$tag$pass -name '*counter_collection*.csv' -exec cp {} "$OUT/${tag}_$pass.csv" \;
  done
done
cd "$ROOT" && python3 scripts/gpu/pmc_summarize.py "$OUT" > "$OUT/summary.txt"; cat "$OUT/summary.txt"
