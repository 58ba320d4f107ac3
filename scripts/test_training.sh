#!/bin/bash
# End-to-end training unit test of every model family (reference scripts/test_training.sh):
# synthetic raw folders -> build_lmdb.py -> train.py for cfg.max_iter (2) iterations,
# reading real LMDBs through the full BaseDataset op pipeline.
#   bash scripts/test_training.sh [config ...]   (default: every configs/unit_test/*.yaml)
#   LAUNCH="python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1" to use DDP.
cd "$(dirname "$0")/.."
LOG=${LOG:-/tmp/unit_test.log}
WORK=${WORK:-dataset/unit_test}
LAUNCH=${LAUNCH:-python}
CONFIGS=("$@")
[ ${#CONFIGS[@]} -eq 0 ] && CONFIGS=(configs/unit_test/*.yaml)
: > "$LOG"
for cfg in "${CONFIGS[@]}"; do
  name=$(basename "$cfg" .yaml)
  raw=$WORK/raw/$name; lmdb=$WORK/lmdb/$name; lcfg=$WORK/$name.lmdb.yaml
  mkdir -p "$WORK"
  out=$(python scripts/make_unit_test_data.py --config "$cfg" --output_root "$raw" \
        --lmdb_root "$lmdb" --lmdb_config "$lcfg" --max_iter 2 2>>"$LOG") || {
    echo -e "\e[1;31m $name: raw data [Failure] \e[0m"; exit 1; }
  paired=""; [ "$out" = "paired=1" ] && paired="--paired"
  python scripts/build_lmdb.py --config "$lcfg" --data_root "$raw" --output_root "$lmdb" \
    --overwrite $paired >> "$LOG" 2>&1 || { echo -e "\e[1;31m $name: build_lmdb [Failure] \e[0m"; exit 1; }
  if $LAUNCH train.py --single_gpu --config "$lcfg" --logdir "$WORK/logs/$name" >> "$LOG" 2>&1; then
    echo -e "\e[1;32m $name [Success] \e[0m"
  else
    echo -e "\e[1;31m $name [Failure] (see $LOG) \e[0m"; exit 1
  fi
done
