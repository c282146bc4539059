#!/bin/bash
# Round-end evidence, part B: bench lines for C4, C5 (with their f64_books legs) and final_scene,
# and the scene table. Outputs under gpurun_out/profiles/<TAG>_*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r3z}
mkdir -p gpurun_out/profiles
step() { local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc: $(tail -n 1 gpurun_out/$name.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then exit $rc; fi; }
for c in C4 C5 NW9; do
  step bench_$c 300 python3 bench.py --config $c --no-cpu-baseline --no-extra --no-breakdown
  grep -v "^W20\|amdgpu.ids" gpurun_out/bench_$c.log | tail -n 1 > gpurun_out/profiles/${TAG}_bench_$c.json
done
step scenes 600 python3 tools/bench_scenes.py
grep "^{" gpurun_out/scenes.log > gpurun_out/profiles/${TAG}_scenes.jsonl
