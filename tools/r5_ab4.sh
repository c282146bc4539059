#!/bin/bash
# Round-5 batch 4: compact tail storage (nonzero radiances + masks), ABI v10 (f32 tail chunks of
# K/4), and the LDS history ring with 1024-thread blocks (up to 160 KiB of LDS): the f64 suite and
# the f32 parity suite on the built library, the f64 suite on the ring variant, then same-box A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_books64.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r5e_books64.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5e_books64.log | cut -c1-250 | tail -5
if [ $rc -ne 0 ]; then grep -E "max \|diff" gpurun_out/r5e_books64.log | cut -c1-200 | head; exit 1; fi
RRT_LIB_PATH=variants/b1kr4/librrt_hip.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_books64.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r5e_b1kr4.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5e_b1kr4.log | cut -c1-250 | tail -5
if [ $rc -ne 0 ]; then grep -E "max \|diff|Error" gpurun_out/r5e_b1kr4.log | cut -c1-200 | head; exit 1; fi
VARIANTS="prev cur3 b1k b1kr4 b1kr6" CONFIG=C2 ROUNDS=2 timeout -k 10 500 bash tools/ab_f64.sh || exit 1
VARIANTS="prev cur3 b1k b1kr4" CONFIG=C4 ROUNDS=2 timeout -k 10 300 bash tools/ab_f64.sh || exit 1
VARIANTS="prev cur3 b1kr4" CONFIG=C5 ROUNDS=1 timeout -k 10 300 bash tools/ab_f64.sh || exit 1
