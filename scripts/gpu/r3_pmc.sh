#!/bin/bash
# GPU-box job (round 3): PMC passes over the hot conv kernels (one rocprofv3 run per pass, each
# under its own time limit): SQ instruction mix / wait breakdown, LDS, MFMA busy, L2 traffic.
#   SHAPES: list of "mode B Cin Cout H W k" (default: the SPADE gamma|beta conv three ways)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r3pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
P2="SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE GRBM_COUNT"
IFS=';' read -ra SH <<< "${SHAPES:-wgrad 4 128 1024 128 256 5;dgrad 4 128 1024 128 256 5;fwd 4 128 1024 128 256 5}"
i=0
for s in "${SH[@]}"; do
  i=$((i+1))
  for pass in 1 2 3; do
    eval "CTRS=\$P$pass"
    rm -rf /tmp/pmc_$i_$pass
    timeout -s KILL 90 rocprofv3 --pmc $CTRS --output-format csv -d /tmp/pmc_${i}_$pass -o run -- \
      python3 "$ROOT/scripts/probe/conv_kernel_driver.py" $s 10 > "$OUT/s${i}_$pass.log" 2>&1
    rc=$?; echo "[pmc] '$s' pass $pass rc=$rc"
    [ $rc -eq 0 ] || { tail -5 "$OUT/s${i}_$pass.log"; exit $rc; }
    find /tmp/pmc_${i}_$pass -name '*counter_collection*.csv' -exec cp {} "$OUT/s${i}_$pass.csv" \;
  done
  echo "$s" > "$OUT/s${i}.shape"
done
cd "$ROOT" && python3 scripts/gpu/pmc_summarize.py "$OUT" > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt" | head -80
exit 0
