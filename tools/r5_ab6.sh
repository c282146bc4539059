#!/bin/bash
# Round-5 batch 6: the f64 tail share T = S/2 against S/4 (prefix units of S/2 balance the queue's
# drain better on high-spp frames), same-box A/B on C2, C4, C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VARIANTS="prev cur6 tdiv2" CONFIG=C2 ROUNDS=3 timeout -k 10 400 bash tools/ab_f64.sh || exit 1
VARIANTS="prev cur6 tdiv2" CONFIG=C4 ROUNDS=3 timeout -k 10 300 bash tools/ab_f64.sh || exit 1
VARIANTS="prev cur6 tdiv2" CONFIG=C5 ROUNDS=2 timeout -k 10 300 bash tools/ab_f64.sh || exit 1
RRT_LIB_PATH=variants/tdiv2/librrt_hip.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_books64.py -q --timeout 300 --timeout-method thread > gpurun_out/r5g_tdiv2.log 2>&1
tail -1 gpurun_out/r5g_tdiv2.log
