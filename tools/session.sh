#!/bin/bash
# Combined session: sweep + PMC for two BVH widths.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/sweep.sh || exit $?
for w in 2 4; do
  RRT_BVH_WIDTH=$w PMC_TAG=w$w GROUPS_LIST="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH GRBM_GUI_ACTIVE
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" bash tools/pmc.sh || exit $?
done
python3 tools/pmc_summary.py gpurun_out/pmcw2 gpurun_out/pmcw4
