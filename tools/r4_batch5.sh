#!/bin/bash
# Round-4 batch 5: the GPU suite on the current library; the wavefront prototype (per-wave unit
# pools): parity, bench lines, kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4i_gpu_suite.log 2>&1 || exit 1
RRT_LIB_PATH=variants/wf/librrt_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -x -q --timeout 100 --timeout-method thread > gpurun_out/r4i_wf_parity.log 2>&1 || exit 1
for c in C2 C4 C5; do
  RRT_LIB_PATH=variants/wf/librrt_hip.so timeout -k 10 200 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-breakdown --no-extra --no-f64 > gpurun_out/r4i_wf_$c.json 2> gpurun_out/r4i_wf_$c.err || exit 1
done
for n in 262144 1048576 2097152; do
  RRT_WF_SLOTS=$n RRT_LIB_PATH=variants/wf/librrt_hip.so timeout -k 10 200 python bench.py --config C2 --spp 64 --steps 2 --warmup 1 --no-cpu-baseline --no-breakdown --no-extra --no-f64 > gpurun_out/r4i_wf_slots$n.json 2>/dev/null || exit 1
  echo "slots $n $(python -c "import json;d=json.load(open('gpurun_out/r4i_wf_slots$n.json'));print(d['value'],'Mrays/s',d['kernel_ms_avg'],'ms')")"
done > gpurun_out/r4i_wf_slots.log 2>&1
RRT_LIB_PATH=variants/wf/librrt_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4i_wfprof -o run --output-format csv -- python3 tools/prof_render.py --config C2 --spp 64 --iters 1 > gpurun_out/r4i_wfprof.log 2>&1
for c in C2 C5; do CONFIG=$c ROUNDS=2 VARIANTS="f64cur f64ra" timeout -k 10 300 bash tools/ab_f64.sh || exit 1; done > gpurun_out/r4i_f64_ra_ab.log 2>&1
RRT_LIB_PATH=variants/node96/librrt_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -x -q --timeout 100 --timeout-method thread > gpurun_out/r4i_node96_parity.log 2>&1 || exit 1
for c in C2 C4; do VARIANTS="f64cur node96" ROUNDS=3 STEPS=3 BENCH_ARGS="--config $c --no-extra" timeout -k 10 400 bash tools/ab.sh || exit 1; done > gpurun_out/r4i_node96_ab.log 2>&1
RRT_LIB_PATH=variants/f64n96/librrt_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_books64.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4i_f64n96_tests.log 2>&1 || exit 1
for c in C2 C4; do CONFIG=$c ROUNDS=2 VARIANTS="f64cur f64n96" timeout -k 10 300 bash tools/ab_f64.sh || exit 1; done > gpurun_out/r4i_f64n96_ab.log 2>&1
