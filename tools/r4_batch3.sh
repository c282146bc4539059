#!/bin/bash
# Round-4 batch 3: where the wavefront prototype's time goes (rocprofv3 kernel stats, one PMC pass
# summed over its dispatches, the slot-pool size), and C2 at chunk K = 256 against 128.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 262144 1048576 2097152 4194304; do
  RRT_WF_SLOTS=$n RRT_LIB_PATH=variants/wf/librrt_hip.so timeout -k 10 200 python bench.py --config C2 --spp 64 --steps 2 --warmup 1 --no-cpu-baseline --no-breakdown --no-extra --no-f64 > gpurun_out/r4g_wf_slots$n.json 2>/dev/null || exit 1
  echo "slots $n $(python -c "import json;d=json.load(open('gpurun_out/r4g_wf_slots$n.json'));print(d['value'],'Mrays/s',d['kernel_ms_avg'],'ms')")"
done > gpurun_out/r4g_wf_slots.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config C2 --spp 64 --steps 2 --warmup 1 --no-cpu-baseline --no-breakdown --no-extra --no-f64 > gpurun_out/r4g_mk_c2_64.json 2>/dev/null || exit 1
RRT_LIB_PATH=variants/wf/librrt_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4g_wfprof -o run -- python3 tools/prof_render.py --config C2 --spp 64 --iters 1 > gpurun_out/r4g_wfprof.log 2>&1 || exit 1
RRT_LIB_PATH=variants/wf/librrt_hip.so timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/r4g_wfpmc -o run -- python3 tools/prof_render.py --config C2 --spp 16 --iters 1 --json gpurun_out/r4g_wfpmc_render.json > gpurun_out/r4g_wfpmc.log 2>&1 || exit 1
for r in 1 2; do for k in 0 256; do
  if [ $k = 0 ]; then unset RRT_CHUNK_FORCE; else export RRT_CHUNK_FORCE=$k; fi
  timeout -k 10 200 python bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline --no-breakdown --no-extra --no-f64 > gpurun_out/r4g_c2_k$k.json 2>/dev/null || exit 1
  echo "r$r K=$k C2 $(python -c "import json;d=json.load(open('gpurun_out/r4g_c2_k$k.json'));print(d['value'],d['kernel_ms_avg'])")"
done; done > gpurun_out/r4g_c2_chunk.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_books64.py tests/test_gpu_multidevice.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4g_f64_tests.log 2>&1 || exit 1
for c in C2 C5 C4; do CONFIG=$c ROUNDS=2 VARIANTS="f64prev f64cam" timeout -k 10 300 bash tools/ab_f64.sh || exit 1; done > gpurun_out/r4g_f64_ab.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_book2.py tests/test_gpu_book3.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4g_book2_tests.log 2>&1 || exit 1
for c in NW9 NW8; do VARIANTS="f64cam medexit" ROUNDS=2 STEPS=3 BENCH_ARGS="--config $c --no-extra" timeout -k 10 300 bash tools/ab.sh || exit 1; done > gpurun_out/r4g_medexit_ab.log 2>&1
