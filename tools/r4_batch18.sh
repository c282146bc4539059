#!/bin/bash
# Round-4 batch 18: traversal-exit / leaf-batch thresholds and the L2 launch shape re-swept on the
# round-4 trees (single-primitive leaves from L2, the f64 kernel's price-1.5 LDS tree).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp STEPS=2
CONFIG=C5 ROUNDS=2 timeout -k 10 900 bash tools/sweep_env.sh "d:" "t48l32:RRT_TRAV_FRAC=48,RRT_LEAF_FRAC=32" "t80l48:RRT_TRAV_FRAC=80,RRT_LEAF_FRAC=48" "t64l32:RRT_TRAV_FRAC=64,RRT_LEAF_FRAC=32" "t64l64:RRT_TRAV_FRAC=64,RRT_LEAF_FRAC=64" "gw6:RRT_GLOBAL_WAVES=6" || exit 1
BENCH_ARGS="--no-f64" CONFIG=NW9 ROUNDS=2 timeout -k 10 600 bash tools/sweep_env.sh "d:" "t48l32:RRT_TRAV_FRAC=48,RRT_LEAF_FRAC=32" "t80l48:RRT_TRAV_FRAC=80,RRT_LEAF_FRAC=48" "t64l32:RRT_TRAV_FRAC=64,RRT_LEAF_FRAC=32" "t64l64:RRT_TRAV_FRAC=64,RRT_LEAF_FRAC=64" || exit 1
CONFIG=C2 ROUNDS=2 timeout -k 10 600 bash tools/sweep_env.sh "d:" "t32l32:RRT_TRAV_FRAC=32,RRT_LEAF_FRAC=32" "t72l72:RRT_TRAV_FRAC=72,RRT_LEAF_FRAC=72" "t56l40:RRT_TRAV_FRAC=56,RRT_LEAF_FRAC=40" || exit 1
