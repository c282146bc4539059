#!/bin/bash
# Debug-statistics pass (round 5): the f64 kernel's RRT_F64_STATS variants (variants/s1..s4) on C2 and C5,
# and the f32 kernel's RRT_PHASE_TIMING=8 variant (variants/p8: node steps whose stepping lanes all
# visit one node) on C5 and final_scene (NW9). Each line: config, counters (slots 2..4 = the stats).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # variant, args...
  local v=$1; shift
  RRT_LIB_PATH=variants/$v/librrt_hip.so timeout -k 10 120 python3 tools/prof_render.py "$@" > gpurun_out/st_$v.log 2>&1
  local rc=$?
  echo "$v $* rc=$rc: $(tail -n 1 gpurun_out/st_$v.log)"
  return $rc
}
for v in s1 s2 s3 s4; do
  run $v --f64 --config C2 --spp 64 --iters 1 || exit 1
  run $v --f64 --config C5 --spp 32 --iters 1 || exit 1
done
run p8 --config C5 --spp 32 --iters 1 || exit 1
run p8 --config NW9 --spp 16 --iters 1 || exit 1
run p8 --config C2 --spp 32 --iters 1 || exit 1
