#!/bin/bash
# Phase statistics of the render kernel from the RRT_PHASE_TIMING debug variants
# (tools/build_variants.sh pt1:-DRRT_PHASE_TIMING=1 pt2:-DRRT_PHASE_TIMING=2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-pt1 pt2}; do
  RRT_LIB_PATH=variants/$v/librrt_hip.so timeout -k 10 300 python3 tools/prof_render.py ${PROF_ARGS:---config C2 --spp 64 --iters 1} > gpurun_out/phase_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc: $(tail -n 1 gpurun_out/phase_$v.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
