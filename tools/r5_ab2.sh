#!/bin/bash
# Round-5 batch 2: the f64 books path bit-exact by construction (back-to-front product, sequential
# sums) + the f32 sphere pre-test: the f64 suite, the deferred-rejection variant's parity, then
# same-box A/B of the variants on C2 and C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_books64.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r5c_books64.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|max \|diff|layouts run|quantisation step" gpurun_out/r5c_books64.log | cut -c1-250
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
RRT_LIB_PATH=variants/defer2/librrt_hip.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_books64.py -v -s --timeout 300 --timeout-method thread -k "matches_books_path or full_class" > gpurun_out/r5c_defer2.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r5c_defer2.log | cut -c1-200
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
for c in "C2 --spp 64" "C5 --spp 32"; do
  RRT_LIB_PATH=variants/s5/librrt_hip.so timeout -k 10 120 python3 tools/prof_render.py --f64 --config $c --iters 1 > gpurun_out/st_s5.log 2>&1 || exit 1
  echo "s5 $c: $(tail -n 1 gpurun_out/st_s5.log | cut -c1-200)"
done
VARIANTS="prev cur nos32 b2f0 seq0 tail4 f32rec defer1 defer2 defer3 ftail4 norej" CONFIG=C2 ROUNDS=2 timeout -k 10 1100 bash tools/ab_f64.sh || exit 1
VARIANTS="prev cur nos32 b2f0 defer2 ftail4 norej" CONFIG=C5 ROUNDS=1 timeout -k 10 600 bash tools/ab_f64.sh || exit 1
VARIANTS="prev cur defer2 ftail4 norej" CONFIG=C4 ROUNDS=1 timeout -k 10 400 bash tools/ab_f64.sh || exit 1
