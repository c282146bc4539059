cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_book2.py tests/test_gpu_book3.py tests/test_gpu_world.py tests/test_abi.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_b2.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_b2.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 tools/scene_probe.py --scenes NW9 NW10 NW8 C2 --spp 16 --iters 2 > gpurun_out/probe_nw9.log 2>&1 || { tail -5 gpurun_out/probe_nw9.log; exit 1; }
grep '^{' gpurun_out/probe_nw9.log | cut -c1-260
