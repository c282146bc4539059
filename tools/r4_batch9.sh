#!/bin/bash
# Round-4 batch 9: the f32 kernel's SAH node price (RRT_SAH_CT) on the global-memory scenes (C5,
# final_scene) and C2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export BENCH_ARGS="--no-f64" STEPS=2
CONFIG=C5 ROUNDS=2 timeout -k 10 500 bash tools/sweep_env.sh "d:" "c3:RRT_SAH_CT=3" "c15:RRT_SAH_CT=1.5" "c1:RRT_SAH_CT=1" "c05:RRT_SAH_CT=0.5" || exit 1
CONFIG=NW9 ROUNDS=2 timeout -k 10 500 bash tools/sweep_env.sh "d:" "c3:RRT_SAH_CT=3" "c15:RRT_SAH_CT=1.5" "c1:RRT_SAH_CT=1" "c05:RRT_SAH_CT=0.5" || exit 1
CONFIG=C2 ROUNDS=2 timeout -k 10 400 bash tools/sweep_env.sh "d:" "c25:RRT_SAH_CT=2.5" "c175:RRT_SAH_CT=1.75" || exit 1
