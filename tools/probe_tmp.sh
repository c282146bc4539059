cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
RRT_LIB_PATH=variants/pl/librrt_hip.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_book2.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_b2.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_b2.log; [ $rc -le 1 ] || exit $rc
for r in 1 2; do for v in cur pl; do
RRT_LIB_PATH=variants/$v/librrt_hip.so timeout -k 10 300 python3 tools/scene_probe.py --scenes NW9 NW4 --spp 16 --iters 2 > gpurun_out/probe_$v.log 2>&1 || { tail -5 gpurun_out/probe_$v.log; exit 1; }
echo "$v"; grep '^{' gpurun_out/probe_$v.log | cut -c1-140
done; done
