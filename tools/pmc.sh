#!/bin/bash
# PMC passes (one rocprofv3 run per counter group; never combined with tracing domains).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS=${PROF_ARGS:---config C2 --spp 64 --iters 2}
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group -d gpurun_out/pmc${PMC_TAG:-}$i -o p --output-format csv -- python3 tools/prof_render.py $ARGS > gpurun_out/pmc${PMC_TAG:-}$i.log 2>&1
  rc=$?
  echo "pass $i ($group) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc${PMC_TAG:-}$i.log; exit $rc; fi
done <<< "${GROUPS_LIST:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH
FETCH_SIZE
WRITE_SIZE TCC_HIT_sum
TCC_MISS_sum TCC_EA0_RDREQ_sum}"
