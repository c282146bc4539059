#!/bin/bash
# Round-5 batch 5: the f64 rejection loops decided in f32 where provably decisive (integers in the
# band) and the fast in-range reciprocal: the f64 suite on the built library, then same-box A/B on C2, C4, C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_books64.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r5f_books64.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5f_books64.log | cut -c1-250 | tail -5
if [ $rc -ne 0 ]; then grep -E "max \|diff" gpurun_out/r5f_books64.log | cut -c1-200 | head; exit 1; fi
VARIANTS="prev cur5 rej0 frc0" CONFIG=C2 ROUNDS=3 timeout -k 10 500 bash tools/ab_f64.sh || exit 1
VARIANTS="prev cur5 rej0 frc0" CONFIG=C4 ROUNDS=2 timeout -k 10 300 bash tools/ab_f64.sh || exit 1
VARIANTS="prev cur5 rej0 frc0" CONFIG=C5 ROUNDS=2 timeout -k 10 300 bash tools/ab_f64.sh || exit 1
