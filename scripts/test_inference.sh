#!/bin/bash
# Inference smoke test of every family (reference scripts/test_inference.sh downloads released
# checkpoints + test data). Offline flow: train each unit-test config for 2 iterations from
# synthetic LMDBs (scripts/test_training.sh), then run inference.py on the last checkpoint.
#   bash scripts/test_inference.sh [config ...]
cd "$(dirname "$0")/.."
WORK=${WORK:-dataset/unit_test}
LOG=${LOG:-/tmp/unit_test_inference.log}
CONFIGS=("$@")
[ ${#CONFIGS[@]} -eq 0 ] && CONFIGS=(configs/unit_test/*.yaml)
: > "$LOG"
for cfg in "${CONFIGS[@]}"; do
  name=$(basename "$cfg" .yaml)
  lcfg=$WORK/$name.lmdb.yaml
  if [ ! -f "$lcfg" ]; then
    LOG=$LOG bash scripts/test_training.sh "$cfg" > /dev/null || {
      echo -e "\e[1;31m $name: training [Failure] \e[0m"; exit 1; }
  fi
  ckpt=$(ls -t "$WORK/logs/$name"/*.pt 2>/dev/null | head -n 1)
  args=(--single_gpu --config "$lcfg" --output_dir "$WORK/output/$name")
  [ -n "$ckpt" ] && args+=(--checkpoint "$ckpt")
  if python inference.py "${args[@]}" >> "$LOG" 2>&1; then
    echo -e "\e[1;32m $name [Success] \e[0m"
  else
    echo -e "\e[1;31m $name [Failure] (see $LOG) \e[0m"; exit 1
  fi
done
