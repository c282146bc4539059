#!/bin/bash
# Round-4 batch 19: texture coordinates divided by 2 pi and pi through Markstein's fma step (both
# kernels): parity of the textured paths, A/B against the IEEE division (variants/dc0) on C4 (f32 +
# f64) and the earth scene.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_book2.py tests/test_gpu_books64.py tests/test_gpu_edges.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4v_parity.log 2>&1 || { tail -30 gpurun_out/r4v_parity.log; exit 1; }
tail -1 gpurun_out/r4v_parity.log
STEPS=3 CONFIG=C4 ROUNDS=3 timeout -k 10 600 bash tools/sweep_env.sh "d:" "k:RRT_LIB_PATH=variants/dc0/librrt_hip.so" || exit 1
BENCH_ARGS="--no-f64" STEPS=3 CONFIG=NW3 ROUNDS=2 timeout -k 10 400 bash tools/sweep_env.sh "d:" "k:RRT_LIB_PATH=variants/dc0/librrt_hip.so" || exit 1
