#!/bin/bash
# Round-4 batch 11: leaf size of the global-memory trees (RRT_MAX_LEAF_GLOBAL) on C5 (f32 + f64),
# bouncing spheres and final_scene.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp STEPS=2
CONFIG=C5 ROUNDS=2 timeout -k 10 500 bash tools/sweep_env.sh "d:" "l1:RRT_MAX_LEAF_GLOBAL=1" "l2:RRT_MAX_LEAF_GLOBAL=2" || exit 1
export BENCH_ARGS="--no-f64"
CONFIG=NW9 ROUNDS=2 timeout -k 10 500 bash tools/sweep_env.sh "d:" "l1:RRT_MAX_LEAF_GLOBAL=1" "l2:RRT_MAX_LEAF_GLOBAL=2" "l1c01:RRT_MAX_LEAF_GLOBAL=1,RRT_SAH_CT_GLOBAL=0.1" || exit 1
CONFIG=NW1 ROUNDS=2 timeout -k 10 500 bash tools/sweep_env.sh "d:" "l1:RRT_MAX_LEAF_GLOBAL=1" "c2:RRT_SAH_CT_GLOBAL=2" || exit 1
