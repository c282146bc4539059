#!/bin/bash
# Per-phase lane / cycle breakdown of the f32 kernel from the RRT_PHASE_TIMING debug variants
# (tools/build_variants.sh pt1:-DRRT_PHASE_TIMING=1 ... pt8:-DRRT_PHASE_TIMING=8), for each of
# CONFIGS (default C2 C5) at SPP samples; tools/phase_breakdown.py turns the JSONs into the table.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/phase
for c in ${CONFIGS:-C2 C5}; do
  for v in ${VARIANTS:-pt1 pt2 pt3 pt4 pt5 pt6 pt7 pt8}; do
    RRT_LIB_PATH=variants/$v/librrt_hip.so timeout -k 10 120 python3 tools/prof_render.py --config $c --spp ${SPP:-64} --iters 1 --json gpurun_out/phase/${c}_$v.json > gpurun_out/phase/${c}_$v.log 2>&1
    rc=$?
    echo "$c $v rc=$rc: $(tail -n 1 gpurun_out/phase/${c}_$v.log | cut -c1-200)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
