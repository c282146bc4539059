#!/bin/bash
# Round-4 batch 2: the wavefront prototype's parity and bench lines, book-2 static-sphere records,
# the hit-center carry (C5), the C3 frame at chunk K = 256.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RRT_LIB_PATH=variants/wf/librrt_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -x -q --timeout 100 --timeout-method thread > gpurun_out/r4f_wf_parity.log 2>&1 || exit 1
for c in C2 C4 C5; do
  RRT_LIB_PATH=variants/wf/librrt_hip.so timeout -k 10 200 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-breakdown --no-extra --no-f64 > gpurun_out/r4f_wf_$c.json 2> gpurun_out/r4f_wf_$c.err || exit 1
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_book2.py tests/test_gpu_book3.py tests/test_gpu_world.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4f_book2_tests.log 2>&1 || exit 1
for c in NW9 NW1 NW8; do VARIANTS="f64rej b2skip" ROUNDS=2 STEPS=3 BENCH_ARGS="--config $c --no-extra" timeout -k 10 300 bash tools/ab.sh || exit 1; done > gpurun_out/r4f_b2skip_ab.log 2>&1 || exit 1
VARIANTS="b2skip carry" ROUNDS=3 STEPS=2 BENCH_ARGS="--config C5 --no-extra" timeout -k 10 300 bash tools/ab.sh > gpurun_out/r4f_carry_ab.log 2>&1 || exit 1
for r in 1 2; do for k in 128 256; do
  RRT_CHUNK=$k timeout -k 10 200 python bench.py --config C3 --steps 1 --warmup 1 --no-cpu-baseline --no-breakdown --no-extra --no-f64 > gpurun_out/r4f_c3_k$k.json 2>/dev/null || exit 1
  echo "r$r K=$k C3 $(python -c "import json;d=json.load(open('gpurun_out/r4f_c3_k$k.json'));print(d['value'],d['kernel_ms_avg'])")"
done; done > gpurun_out/r4f_c3_chunk.log 2>&1
