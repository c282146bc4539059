#!/bin/bash
# Round-4 batch: f64 integer rejection loops (A/B against the rcp build), the wavefront prototype's
# parity and bench lines (variants/wf), and the chunk size K = 256 against 128 (RRT_CHUNK, timing only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_books64.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4e_f64_tests.log 2>&1 || exit 1
for c in C2 C5 C4; do CONFIG=$c ROUNDS=2 VARIANTS="f64rcp f64rej" timeout -k 10 300 bash tools/ab_f64.sh || exit 1; done > gpurun_out/r4e_f64_ab.log 2>&1 || exit 1
for r in 1 2; do for k in 128 256; do for c in C2 C4 C5; do
  RRT_CHUNK=$k timeout -k 10 200 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-breakdown --no-extra --no-f64 > gpurun_out/r4e_k${k}_${c}.json 2>/dev/null || exit 1
  echo "r$r K=$k $c $(python -c "import json;d=json.load(open('gpurun_out/r4e_k${k}_${c}.json'));print(d['value'],d['kernel_ms_avg'])")"
done; done; done > gpurun_out/r4e_chunk_ab.log 2>&1 || exit 1
RRT_LIB_PATH=variants/wf/librrt_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 100 --timeout-method thread > gpurun_out/r4e_wf_parity.log 2>&1 || exit 1
for c in C2 C4 C5; do
  RRT_LIB_PATH=variants/wf/librrt_hip.so timeout -k 10 200 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-breakdown --no-extra --no-f64 > gpurun_out/r4e_wf_$c.json 2> gpurun_out/r4e_wf_$c.err || exit 1
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_book2.py tests/test_gpu_book3.py tests/test_gpu_world.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4e_book2_tests.log 2>&1 || exit 1
for c in NW9 NW1 NW8; do VARIANTS="f64rej b2skip" ROUNDS=2 STEPS=3 BENCH_ARGS="--config $c --no-extra" timeout -k 10 300 bash tools/ab.sh || exit 1; done > gpurun_out/r4e_b2skip_ab.log 2>&1
VARIANTS="b2skip carry" ROUNDS=3 STEPS=2 BENCH_ARGS="--config C5 --no-extra" timeout -k 10 300 bash tools/ab.sh > gpurun_out/r4e_carry_ab.log 2>&1
