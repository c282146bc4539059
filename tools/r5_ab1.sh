#!/bin/bash
# Round-5 batch 1: the f64 kernel's f32 sphere pre-test. Parity of the f64 suite on the built
# library, pre-test statistics (variants/s5), same-box A/B of the variants on C2 and C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_books64.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r5b_books64.log 2>&1 || { tail -40 gpurun_out/r5b_books64.log; exit 1; }
grep -E "passed|failed" gpurun_out/r5b_books64.log | tail -1
for c in "C2 --spp 64" "C5 --spp 32"; do
  RRT_LIB_PATH=variants/s5/librrt_hip.so timeout -k 10 120 python3 tools/prof_render.py --f64 --config $c --iters 1 > gpurun_out/st_s5.log 2>&1 || exit 1
  echo "s5 $c: $(tail -n 1 gpurun_out/st_s5.log)"
done
VARIANTS="prev cur hold f32rec norej" CONFIG=C2 ROUNDS=2 timeout -k 10 700 bash tools/ab_f64.sh || exit 1
VARIANTS="prev cur hold f32rec norej" CONFIG=C5 ROUNDS=2 timeout -k 10 700 bash tools/ab_f64.sh || exit 1
