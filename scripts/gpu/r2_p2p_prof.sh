#!/bin/bash
# GPU-box job: kernel breakdown + op-site attribution of the pix2pixHD Cityscapes recipe iteration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
mkdir -p gpurun_out/p2p
ARGS="--config $ROOT/configs/unit_test/pix2pixHD.yaml --steps 3 --warmup 2 --set gen.global_generator.num_filters=64 gen.global_generator.num_res_blocks=9 dis.num_filters=64 dis.num_discriminators=2 data.train.batch_size=2 trainer.model_average=True trainer.model_average_beta=0.999 trainer.model_average_start_iteration=0 trainer.model_average_batch_norm_estimation_iteration=0 data.train.augmentations.resize_h_w=512,1024 data.val.augmentations.resize_h_w=512,1024"
timeout -k 10 300 python scripts/bench_families.py $ARGS --op-sites > gpurun_out/p2p/sites.out 2> gpurun_out/p2p/sites.err
echo "[p2p] sites rc=$?"
cd /tmp && export TMPDIR=/tmp && rm -rf /tmp/p2p_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p2p_prof -o run -- \
  python3 "$ROOT/scripts/bench_families.py" $ARGS > "$ROOT/gpurun_out/p2p/prof.log" 2>&1
rc=$?; echo "[p2p] rocprof rc=$rc"
cd "$ROOT"
python3 scripts/gpu/summarize_kernels.py /tmp/p2p_prof > gpurun_out/p2p/kernels.txt
head -40 gpurun_out/p2p/kernels.txt
exit $rc
