#!/bin/bash
# PMC instruction-mix passes (separate rocprofv3 runs, no tracing domains) for each
# variants/<name>/librrt_hip.so given, on C2 at ${SPP:-64} spp; summary per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
for v in "$@"; do
  i=0
  while read -r group; do
    [ -z "$group" ] && continue
    # keep only counters this rocprofv3 lists (an unknown name fails the pass)
    group=$(for c in $group; do grep -qw "${c%_sum}" gpurun_out/counters_list.txt && echo -n "$c "; done)
    [ -z "$group" ] && continue
    i=$((i+1))
    RRT_LIB_PATH=variants/$v/librrt_hip.so timeout -s KILL 120 rocprofv3 --pmc $group -d gpurun_out/pmc_${v}_$i -o p --output-format csv -- python3 tools/prof_render.py --config C2 --spp ${SPP:-64} --iters 1 > gpurun_out/pmc_${v}_$i.log 2>&1
    rc=$?
    echo "$v pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_${v}_$i.log; exit $rc; fi
  done <<< "${GROUPS_LIST:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH GRBM_GUI_ACTIVE
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM}"
  python3 tools/pmc_summary.py gpurun_out/pmc_${v}_ | tee gpurun_out/pmc_${v}_summary.txt
done
