#!/bin/bash
# VALU instruction mix of the render kernels: two rocprofv3 --pmc passes (8 SQ + 1 GRBM counters
# each, no tracing) per run of tools/prof_render.py, summarised by tools/pmc_mix.py into
# gpurun_out/pmc_mix_<name>.json. RUNS = "name|prof_render args;..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
A="SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 GRBM_GUI_ACTIVE"
B="SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
IFS=';' read -ra LIST <<< "${RUNS:-f64_C2|--f64 --config C2 --spp 64 --iters 1;f32_C2|--config C2 --spp 64 --iters 1}"
for spec in "${LIST[@]}"; do
  name=${spec%%|*}; args=${spec#*|}
  for pass in A B; do
    rm -rf gpurun_out/pmix_${name}_$pass
    timeout -s KILL 120 rocprofv3 --pmc ${!pass} -d gpurun_out/pmix_${name}_$pass -o run --output-format csv \
      -- python3 tools/prof_render.py $args --json gpurun_out/pmix_${name}.json > gpurun_out/pmix_${name}_$pass.log 2>&1
    rc=$?; echo "$name $pass rc=$rc"
    if [ $rc -ne 0 ]; then tail -n 5 gpurun_out/pmix_${name}_$pass.log; exit $rc; fi
  done
  python3 tools/pmc_mix.py gpurun_out/pmix_${name}_A gpurun_out/pmix_${name}_B gpurun_out/pmix_${name}.json gpurun_out/pmc_mix_$name.json || exit 1
done
