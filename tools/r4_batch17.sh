#!/bin/bash
# Round-4 batch 17: the f64 kernel's Russian-roulette 1 / pr from the host (untextured class):
# books-path parity, A/B against the division (variants/f64pr0) on C2 and C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_books64.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4t_books64.log 2>&1 || { tail -30 gpurun_out/r4t_books64.log; exit 1; }
tail -1 gpurun_out/r4t_books64.log
for c in C2 C5; do CONFIG=$c ROUNDS=2 STEPS=1 timeout -k 10 500 bash tools/sweep_env.sh "d:" "k:RRT_LIB_PATH=variants/f64pr0/librrt_hip.so" || exit 1; done
