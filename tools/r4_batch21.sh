#!/bin/bash
# Round-4 batch 21/22: short square roots (provable domains; then wave-uniform gated in the leaf loops and unit()):
# |p|^2, dielectric 1 - c^2, refraction): exhaustive device check, parity, A/B against the previous
# commit's library (variants/prev) on C2, C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_recip.py tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_fullsize.py tests/test_gpu_book2.py tests/test_gpu_book3.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4x_parity.log 2>&1 || { tail -30 gpurun_out/r4x_parity.log; exit 1; }
tail -1 gpurun_out/r4x_parity.log
export BENCH_ARGS="--no-f64"
STEPS=3 CONFIG=C2 ROUNDS=3 timeout -k 10 600 bash tools/sweep_env.sh "d:" "k:RRT_LIB_PATH=variants/prev/librrt_hip.so" || exit 1
STEPS=2 CONFIG=C5 ROUNDS=2 timeout -k 10 400 bash tools/sweep_env.sh "d:" "k:RRT_LIB_PATH=variants/prev/librrt_hip.so" || exit 1
