#!/bin/bash
# Round-4 batch 12: global-memory scenes in single-primitive leaves — GPU suite, scene table against
# the previous shape (RRT_MAX_LEAF_GLOBAL=3 = node price 2, 3-primitive leaves), C5 f64 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x > gpurun_out/r4o_gpu_suite.log 2>&1 || { tail -30 gpurun_out/r4o_gpu_suite.log; exit 1; }
tail -1 gpurun_out/r4o_gpu_suite.log
for r in 1 2; do
  RRT_MAX_LEAF_GLOBAL=3 timeout -k 10 300 python3 tools/bench_scenes.py > gpurun_out/r4o_scenes_old_$r.jsonl 2> gpurun_out/r4o_scenes_old_$r.txt || exit 1
  timeout -k 10 300 python3 tools/bench_scenes.py > gpurun_out/r4o_scenes_new_$r.jsonl 2> gpurun_out/r4o_scenes_new_$r.txt || exit 1
done
cat gpurun_out/r4o_scenes_old_2.txt gpurun_out/r4o_scenes_new_2.txt
CONFIG=C5 ROUNDS=2 STEPS=2 timeout -k 10 500 bash tools/sweep_env.sh "d:" "old:RRT_MAX_LEAF_GLOBAL=3" || exit 1
