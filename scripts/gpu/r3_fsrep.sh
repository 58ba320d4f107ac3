cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r3f
for i in 1 2; do
  timeout -k 10 300 python -u -m pytest tests/test_graph_families_gpu.py -x -q --timeout 200 -k fs_vid2vid -s > gpurun_out/r3f/rep$i.out 2>&1
  echo "rep $i rc=$?"; grep -E "graph \{|eager \{|passed|failed" gpurun_out/r3f/rep$i.out | cut -c1-200
done
