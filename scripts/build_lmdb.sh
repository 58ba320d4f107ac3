#!/bin/bash
# Build train/test LMDBs of one dataset (reference scripts/build_lmdb.sh).
#   bash scripts/build_lmdb.sh <model> <dataset>   e.g. spade cocostuff
# expects dataset/<dataset>_raw/{train,test}; writes dataset/<dataset>/{train,test}.
MODEL=$1
DATASET=$2
CFG=${CFG:-configs/projects/${MODEL}/${DATASET}/ampO1.yaml}
PAIRED=${PAIRED:---paired}
for SPLIT in test train; do
  RAW=dataset/${DATASET}_raw/${SPLIT}
  LMDB=dataset/${DATASET}/${SPLIT}
  echo "${LMDB}"
  python scripts/build_lmdb.py --config "${CFG}" --data_root "${RAW}" --output_root "${LMDB}" \
    --overwrite ${PAIRED} || exit 1
done
