#!/bin/bash
# GPU-box job (round 6): wc-vid2vid at the reference cityscapes recipe's scale (512x1024, batch 1,
# G 32 -> 1024 filters, D 64 -> 512), eager (the renderer keeps host-side state), with a
# rocprofv3 kernel breakdown of the steady state.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r6wc; mkdir -p $OUT
ARGS="--config $ROOT/configs/unit_test/wc_vid2vid.yaml --seq-len 3 --set gen.num_filters=32 \
gen.max_num_filters=1024 gen.flow.num_filters=32 gen.flow.max_num_filters=1024 \
gen.flow.multi_spade_combine.embed.num_filters=32 gen.embed.num_filters=32 \
gen.embed.max_num_filters=1024 dis.image.num_filters=64 dis.image.max_num_filters=512 \
dis.temporal.num_filters=64 dis.temporal.max_num_filters=512 data.train.batch_size=1 \
data.train.augmentations.resize_h_w=512,1024 data.val.augmentations.resize_h_w=512,1024"
timeout -k 10 600 python -u scripts/bench_families.py $ARGS --steps 8 --warmup 3 \
  > $OUT/wc.jsonl 2> $OUT/wc.err || { tail -20 $OUT/wc.err; exit 1; }
tail -1 $OUT/wc.jsonl | cut -c1-600
rm -rf /tmp/iamd_rprof
(cd /tmp && TMPDIR=/tmp timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
  -d /tmp/iamd_rprof -o run -- python3 $ROOT/scripts/bench_families.py $ARGS --steps 3 --warmup 3 \
  --no-pipelined > $OUT/wc_prof.log 2>&1) || { tail -20 $OUT/wc_prof.log; exit 1; }
python3 scripts/gpu/summarize_kernels.py /tmp/iamd_rprof > $OUT/wc_kernels.txt
head -30 $OUT/wc_kernels.txt
