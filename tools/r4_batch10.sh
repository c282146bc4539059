#!/bin/bash
# Round-4 batch 10: global-memory scenes built at SAH node price 0.5 (f32 kernel) — the GPU suite
# (bit-exact parity on the new trees), the scene table at the old price (2) and the new default,
# a finer price sweep on final_scene.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x > gpurun_out/r4n_gpu_suite.log 2>&1 || { tail -30 gpurun_out/r4n_gpu_suite.log; exit 1; }
tail -1 gpurun_out/r4n_gpu_suite.log
for r in 1 2; do
  RRT_SAH_CT_GLOBAL=2 timeout -k 10 300 python3 tools/bench_scenes.py > gpurun_out/r4n_scenes_ct2_$r.jsonl 2> gpurun_out/r4n_scenes_ct2_$r.txt || exit 1
  timeout -k 10 300 python3 tools/bench_scenes.py > gpurun_out/r4n_scenes_new_$r.jsonl 2> gpurun_out/r4n_scenes_new_$r.txt || exit 1
done
cat gpurun_out/r4n_scenes_ct2_1.txt gpurun_out/r4n_scenes_new_1.txt
export BENCH_ARGS="--no-f64" STEPS=2
CONFIG=NW9 ROUNDS=2 timeout -k 10 500 bash tools/sweep_env.sh "d:" "g025:RRT_SAH_CT_GLOBAL=0.25" "g01:RRT_SAH_CT_GLOBAL=0.1" "g075:RRT_SAH_CT_GLOBAL=0.75" "l1:RRT_MAX_LEAF=1" || exit 1
