#!/bin/bash
# Round-4 batch 14: dielectric constants formed on the host (1 / eta and both Schlick r0 per
# material: f32 in the material record, f64 in a per-primitive table): parity suites, same-box A/B
# against the kernel-side divisions (variants/dielk) on C2 (both kernels), C5, final_scene, book 3;
# leaf-size bound of the LDS trees on C2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_fullsize.py tests/test_gpu_book2.py tests/test_gpu_book3.py tests/test_gpu_books64.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4q_diel_parity.log 2>&1 || { tail -30 gpurun_out/r4q_diel_parity.log; exit 1; }
tail -1 gpurun_out/r4q_diel_parity.log
V=variants/dielk/librrt_hip.so
STEPS=3 CONFIG=C2 ROUNDS=3 timeout -k 10 600 bash tools/sweep_env.sh "d:" "k:RRT_LIB_PATH=$V" || exit 1
export BENCH_ARGS="--no-f64" STEPS=2
CONFIG=C5 ROUNDS=2 timeout -k 10 400 bash tools/sweep_env.sh "d:" "k:RRT_LIB_PATH=$V" || exit 1
CONFIG=NW9 ROUNDS=2 timeout -k 10 400 bash tools/sweep_env.sh "d:" "k:RRT_LIB_PATH=$V" || exit 1
CONFIG=B3 ROUNDS=2 timeout -k 10 400 bash tools/sweep_env.sh "d:" "k:RRT_LIB_PATH=$V" || exit 1
unset BENCH_ARGS
CONFIG=C2 ROUNDS=2 timeout -k 10 600 bash tools/sweep_env.sh "d:" "l2:RRT_MAX_LEAF=2" "l4:RRT_MAX_LEAF=4" "l5:RRT_MAX_LEAF=5" || exit 1
