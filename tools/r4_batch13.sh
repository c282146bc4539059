#!/bin/bash
# Round-4 batch 13: f32 kernel, LDS-staged scenes with materials read from L2 (RRT_MTL_LDS=0, so the
# per-primitive LDS record is 16 B and the 40-KB scene budget holds a deeper tree): parity of the
# variant, C2 at SAH node prices 2 / 1.5 / 1.25, C4 and cornell_smoke at 2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=variants/mtlg/librrt_hip.so
RRT_LIB_PATH=$V timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_book2.py tests/test_gpu_book3.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4p_mtlg_parity.log 2>&1 || { tail -30 gpurun_out/r4p_mtlg_parity.log; exit 1; }
tail -1 gpurun_out/r4p_mtlg_parity.log
export BENCH_ARGS="--no-f64" STEPS=3
CONFIG=C2 ROUNDS=2 timeout -k 10 600 bash tools/sweep_env.sh "d:" "g2:RRT_LIB_PATH=$V" "g15:RRT_LIB_PATH=$V,RRT_SAH_CT=1.5" "g125:RRT_LIB_PATH=$V,RRT_SAH_CT=1.25" "d15:RRT_SAH_CT=1.5" || exit 1
STEPS=2 CONFIG=C4 ROUNDS=2 timeout -k 10 400 bash tools/sweep_env.sh "d:" "g2:RRT_LIB_PATH=$V" || exit 1
STEPS=2 CONFIG=NW8 ROUNDS=2 timeout -k 10 400 bash tools/sweep_env.sh "d:" "g2:RRT_LIB_PATH=$V" "g15:RRT_LIB_PATH=$V,RRT_SAH_CT=1.5" || exit 1
