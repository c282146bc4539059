#!/bin/bash
# Round-4 batch 7: f64 books kernel with r*r in the widened records and an f64-specific BVH
# (RRT_F64_SAH_CT: the SAH's node price for the f64 kernel, its own LDS fit): parity, A/B against
# the round's previous build, node-price sweep on C2 and C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_books64.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4l_books64.log 2>&1 || { tail -20 gpurun_out/r4l_books64.log; exit 1; }
tail -1 gpurun_out/r4l_books64.log
RRT_F64_SAH_CT=1.5 timeout -k 10 400 python -u -m pytest tests/test_gpu_books64.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4l_books64_ct15.log 2>&1 || { tail -20 gpurun_out/r4l_books64_ct15.log; exit 1; }
tail -1 gpurun_out/r4l_books64_ct15.log
for c in C2 C4; do CONFIG=$c ROUNDS=2 VARIANTS="f64old f64cur" timeout -k 10 300 bash tools/ab_f64.sh || exit 1; done
CONFIG=C2 ROUNDS=2 timeout -k 10 400 bash tools/sweep_env.sh "d:" "ct175:RRT_F64_SAH_CT=1.75" "ct15:RRT_F64_SAH_CT=1.5" "ct125:RRT_F64_SAH_CT=1.25" || exit 1
CONFIG=C5 ROUNDS=2 timeout -k 10 500 bash tools/sweep_env.sh "d:" "ct15:RRT_F64_SAH_CT=1.5" "ct1:RRT_F64_SAH_CT=1" "ct05:RRT_F64_SAH_CT=0.5" || exit 1
