#!/bin/bash
# Round-4 batch 16: 1 / r from the host for book-2 / book-3 spheres too (motion record's w): parity
# suites, scene table against the kernel-side divisions (variants/k3: no host 1 / r, no host 1 / pr).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_book2.py tests/test_gpu_book3.py tests/test_gpu_world.py tests/test_gpu_cli.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4s_parity.log 2>&1 || { tail -30 gpurun_out/r4s_parity.log; exit 1; }
tail -1 gpurun_out/r4s_parity.log
for r in 1 2; do
  RRT_LIB_PATH=variants/k3/librrt_hip.so timeout -k 10 300 python3 tools/bench_scenes.py > gpurun_out/r4s_scenes_k3_$r.jsonl 2> gpurun_out/r4s_scenes_k3_$r.txt || exit 1
  timeout -k 10 300 python3 tools/bench_scenes.py > gpurun_out/r4s_scenes_new_$r.jsonl 2> gpurun_out/r4s_scenes_new_$r.txt || exit 1
done
paste gpurun_out/r4s_scenes_k3_2.txt gpurun_out/r4s_scenes_new_2.txt | awk -F'  +' '{print}' 
