#!/bin/bash
# Round-4 batch 15: f32 book-1 kernel with 1 / r (all book-1 classes) and Russian roulette's 1 / pr
# (the untextured class) formed on the host: parity suites, same-box A/B against the kernel-side
# divisions (variants/k2: neither; variants/pr0: 1 / r only) on C2, C4, C5, cornell_smoke.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_fullsize.py tests/test_gpu_book2.py tests/test_gpu_book3.py tests/test_gpu_books64.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4r_parity.log 2>&1 || { tail -30 gpurun_out/r4r_parity.log; exit 1; }
tail -1 gpurun_out/r4r_parity.log
export BENCH_ARGS="--no-f64" STEPS=3
CONFIG=C2 ROUNDS=3 timeout -k 10 600 bash tools/sweep_env.sh "d:" "k2:RRT_LIB_PATH=variants/k2/librrt_hip.so" "pr0:RRT_LIB_PATH=variants/pr0/librrt_hip.so" || exit 1
STEPS=2 CONFIG=C4 ROUNDS=2 timeout -k 10 400 bash tools/sweep_env.sh "d:" "k2:RRT_LIB_PATH=variants/k2/librrt_hip.so" || exit 1
STEPS=2 CONFIG=C5 ROUNDS=2 timeout -k 10 400 bash tools/sweep_env.sh "d:" "k2:RRT_LIB_PATH=variants/k2/librrt_hip.so" || exit 1
STEPS=2 CONFIG=NW8 ROUNDS=2 timeout -k 10 400 bash tools/sweep_env.sh "d:" "k2:RRT_LIB_PATH=variants/k2/librrt_hip.so" || exit 1
