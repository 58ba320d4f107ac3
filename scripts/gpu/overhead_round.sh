#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for args in "nobench nhwc" "nobench nchw" "bench nhwc"; do
  timeout -k 10 400 python scripts/probe/launch_overhead_probe.py $args >> gpurun_out/overhead.log 2>&1
  rc=$?; echo "[overhead] $args rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/overhead.log; exit $rc; }
done
grep -v amdgpu.ids gpurun_out/overhead.log
