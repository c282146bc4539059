#!/bin/bash
# Round-4 batch 20: the f32 kernel's short reciprocal (v_rcp_f32 + one fma Newton step) for unit
# vectors, the ray slopes and RR's 1 / pr: the exhaustive device check, parity suites, A/B against
# the IEEE division (variants/rcp0) on C2, C4, C5, final_scene.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_recip.py tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_fullsize.py tests/test_gpu_book2.py tests/test_gpu_book3.py tests/test_gpu_world.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4w_parity.log 2>&1 || { tail -30 gpurun_out/r4w_parity.log; exit 1; }
tail -1 gpurun_out/r4w_parity.log
export BENCH_ARGS="--no-f64"
STEPS=3 CONFIG=C2 ROUNDS=3 timeout -k 10 600 bash tools/sweep_env.sh "d:" "k:RRT_LIB_PATH=variants/rcp0/librrt_hip.so" || exit 1
for c in C4 C5 NW9; do STEPS=2 CONFIG=$c ROUNDS=2 timeout -k 10 400 bash tools/sweep_env.sh "d:" "k:RRT_LIB_PATH=variants/rcp0/librrt_hip.so" || exit 1; done
