#!/bin/bash
# Round-4 batch 4: the f64 kernel's widened LDS sphere records and host-formed constants (parity of
# each build, then a same-box A/B), the wavefront prototype with per-wave unit pools, the medium
# free-flight early exit, the chunk rule K0 = 256 under the GPU parity suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in f64base f64wide f64wcam f64wall; do
  RRT_LIB_PATH=variants/$v/librrt_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_books64.py -q --timeout 200 --timeout-method thread > gpurun_out/r4h_f64_tests_$v.log 2>&1
  echo "$v rc=$? $(tail -1 gpurun_out/r4h_f64_tests_$v.log)"
done > gpurun_out/r4h_f64_isolate.log 2>&1
for c in C2 C5 C4; do CONFIG=$c ROUNDS=2 VARIANTS="f64base f64wide f64wcam f64wall" timeout -k 10 400 bash tools/ab_f64.sh || exit 1; done > gpurun_out/r4h_f64_ab.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_book2.py tests/test_gpu_book3.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4h_parity_book2_tests.log 2>&1 || exit 1
for c in NW9 NW8; do VARIANTS="f64prev medexit" ROUNDS=2 STEPS=3 BENCH_ARGS="--config $c --no-extra" timeout -k 10 300 bash tools/ab.sh || exit 1; done > gpurun_out/r4h_medexit_ab.log 2>&1 || exit 1
RRT_LIB_PATH=variants/wf/librrt_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 100 --timeout-method thread > gpurun_out/r4h_wf_parity.log 2>&1 || exit 1
for c in C2 C4 C5; do
  RRT_LIB_PATH=variants/wf/librrt_hip.so timeout -k 10 200 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-breakdown --no-extra --no-f64 > gpurun_out/r4h_wf_$c.json 2> gpurun_out/r4h_wf_$c.err || exit 1
done
RRT_LIB_PATH=variants/wf/librrt_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4h_wfprof -o run -- python3 tools/prof_render.py --config C2 --spp 64 --iters 1 > gpurun_out/r4h_wfprof.log 2>&1
