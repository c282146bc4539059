#!/bin/bash
# Round-5 batch 2: the f64 books path bit-exact by construction (back-to-front product, sequential
# sums) + the f32 sphere pre-test: the f64 suite, then same-box A/B of the variants on C2 and C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_books64.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r5c_books64.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|max \|diff|layouts run|quantisation step" gpurun_out/r5c_books64.log | cut -c1-250
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
for c in "C2 --spp 64" "C5 --spp 32"; do
  RRT_LIB_PATH=variants/s5/librrt_hip.so timeout -k 10 120 python3 tools/prof_render.py --f64 --config $c --iters 1 > gpurun_out/st_s5.log 2>&1 || exit 1
  echo "s5 $c: $(tail -n 1 gpurun_out/st_s5.log | cut -c1-200)"
done
VARIANTS="prev cur nos32 b2f0 seq0 tail4 f32rec norej" CONFIG=C2 ROUNDS=2 timeout -k 10 900 bash tools/ab_f64.sh || exit 1
VARIANTS="prev cur nos32 b2f0 seq0 norej" CONFIG=C5 ROUNDS=1 timeout -k 10 700 bash tools/ab_f64.sh || exit 1
