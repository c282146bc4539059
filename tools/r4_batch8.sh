#!/bin/bash
# Round-4 batch 8: the f64 kernel's per-placement SAH node prices as defaults (1.5 LDS, 0.5 global):
# books-path parity, a finer price sweep on C2 (LDS) and C5 (global).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_books64.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4m_books64.log 2>&1 || { tail -20 gpurun_out/r4m_books64.log; exit 1; }
tail -1 gpurun_out/r4m_books64.log
CONFIG=C2 ROUNDS=2 timeout -k 10 400 bash tools/sweep_env.sh "d:" "l14:RRT_F64_SAH_CT_LDS=1.4" "l16:RRT_F64_SAH_CT_LDS=1.6" "l2:RRT_F64_SAH_CT_LDS=2" || exit 1
CONFIG=C5 ROUNDS=2 timeout -k 10 500 bash tools/sweep_env.sh "d:" "g025:RRT_F64_SAH_CT_GLOBAL=0.25" "g075:RRT_F64_SAH_CT_GLOBAL=0.75" "g2:RRT_F64_SAH_CT_GLOBAL=2" || exit 1
