#!/bin/bash
# Memory-path PMC of one render launch per workload: three --pmc passes (SQ issue/wait
# counts; L1/L2 hit counts; TA/TD/TCP busy and latency), each its own run. WORKLOADS = config:spp[:width] list.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in ${WORKLOADS:-C2:64 NW9:64:1080}; do
  c=${spec%%:*}; rest=${spec#*:}; s=${rest%%:*}; wa=""
  [ "$rest" != "$s" ] && wa="--width ${rest#*:}"
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -d gpurun_out/lat_$c -o p --output-format csv -- python3 tools/prof_render.py --config $c --spp $s $wa --iters 1 > gpurun_out/lat_$c.log 2>&1 || { echo "lat $c failed"; tail -3 gpurun_out/lat_$c.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum -d gpurun_out/hit_$c -o p --output-format csv -- python3 tools/prof_render.py --config $c --spp $s $wa --iters 1 > gpurun_out/hit_$c.log 2>&1 || { echo "hit $c failed"; tail -3 gpurun_out/hit_$c.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE TCP_TCP_LATENCY_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TOTAL_READ_sum TCP_PENDING_STALL_CYCLES_sum -d gpurun_out/busy_$c -o p --output-format csv -- python3 tools/prof_render.py --config $c --spp $s $wa --iters 1 > gpurun_out/busy_$c.log 2>&1 || { echo "busy $c failed"; tail -3 gpurun_out/busy_$c.log; exit 1; }
  python3 - "$c" <<'PY'
import sys, os
sys.path.insert(0, "tools")
from pmc_issue import per_dispatch
c = sys.argv[1]
a, _ = per_dispatch(f"gpurun_out/lat_{c}")
b, _ = per_dispatch(f"gpurun_out/hit_{c}")
a.update(b)
b, _ = per_dispatch(f"gpurun_out/busy_{c}")
a.update(b)
print(c, {k: f"{v:.4g}" for k, v in sorted(a.items())})
cyc = a["GRBM_GUI_ACTIVE"] / 8  # per XCD
print(c, "TA busy %.1f %%, TD busy %.1f %% per CU; L1 hit %.1f %%; vector loads %.3g; SQ_WAIT_ANY %.3g" % (
      100 * a["TA_TA_BUSY_sum"] / 256 / cyc, 100 * a["TD_TD_BUSY_sum"] / 256 / cyc,
      100 * (1 - a["TCP_TCC_READ_REQ_sum"] / a["TCP_TOTAL_CACHE_ACCESSES_sum"]), a["SQ_INSTS_VMEM_RD"], a["SQ_WAIT_ANY"]))
PY
done
