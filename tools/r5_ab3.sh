#!/bin/bash
# Round-5 batch 3: the f64 suite on the built library (texel records fixed in the diffuse class,
# tail = S/4, pre-test off, grouped fold), then same-box A/B of the f64 variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_books64.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r5d_books64.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|max \|diff|layouts run|quantisation step" gpurun_out/r5d_books64.log | cut -c1-250
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
VARIANTS="prev cur2 fg1 fg2 s32on bm1 bm2 b2f0" CONFIG=C2 ROUNDS=2 timeout -k 10 800 bash tools/ab_f64.sh || exit 1
VARIANTS="prev cur2 fg1 fg2 b2f0" CONFIG=C4 ROUNDS=1 timeout -k 10 300 bash tools/ab_f64.sh || exit 1
VARIANTS="prev cur2 s32on b2f0" CONFIG=C5 ROUNDS=1 timeout -k 10 300 bash tools/ab_f64.sh || exit 1
export BENCH_ARGS="--no-f64" STEPS=3
CONFIG=C2 ROUNDS=2 timeout -k 10 300 bash tools/sweep_env.sh "prev:RRT_LIB_PATH=variants/prev/librrt_hip.so" "ftail4:RRT_LIB_PATH=variants/ftail4/librrt_hip.so" || exit 1
STEPS=2 CONFIG=C4 ROUNDS=2 timeout -k 10 200 bash tools/sweep_env.sh "prev:RRT_LIB_PATH=variants/prev/librrt_hip.so" "ftail4:RRT_LIB_PATH=variants/ftail4/librrt_hip.so" || exit 1
STEPS=2 CONFIG=C5 ROUNDS=2 timeout -k 10 200 bash tools/sweep_env.sh "prev:RRT_LIB_PATH=variants/prev/librrt_hip.so" "ftail4:RRT_LIB_PATH=variants/ftail4/librrt_hip.so" || exit 1
