#!/bin/bash
# Round-4 batch 6: f64 books kernel — r*r in the widened sphere records (RRT_F64_R2), the leaf loop
# split on a wave-uniform division mode (RRT_F64_DIV_UNIFORM), the structurizer flag on the f64
# object: books-path parity per variant, same-box A/B (C2, C4, C5), issue PMC of the new build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in f64new f64su; do
  RRT_LIB_PATH=variants/$v/librrt_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_books64.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4k_${v}_books64.log 2>&1 || { tail -20 gpurun_out/r4k_${v}_books64.log; exit 1; }
  tail -1 gpurun_out/r4k_${v}_books64.log
done
for c in C2 C4 C5; do CONFIG=$c ROUNDS=2 VARIANTS="f64old f64r2 f64new f64su" timeout -k 10 500 bash tools/ab_f64.sh || exit 1; done > gpurun_out/r4k_f64_ab.log 2>&1
cat gpurun_out/r4k_f64_ab.log
RRT_LIB_PATH=variants/f64new/librrt_hip.so timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/ti_f64 -o p --output-format csv -- python3 tools/prof_render.py --config C2 --spp 512 --iters 1 --f64 --json gpurun_out/ti_f64.json > gpurun_out/r4k_pmc_f64.log 2>&1 || exit 1
python3 tools/pmc_issue.py gpurun_out/ti_f64 gpurun_out/ti_f64.json gpurun_out/r4k_issue_C2_f64.json && cat gpurun_out/r4k_issue_C2_f64.json
