#!/bin/bash
# Round-end evidence on one GPU, every step time-limited, stopping at the first failure:
# the GPU test suite, smoke(), the PMC / rocprof / bench evidence (tools/evidence_r3.sh), bench
# lines for C4, C5 and final_scene, and the scene table. Outputs under gpurun_out/ (profiles/ copies).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r3z}
mkdir -p gpurun_out/profiles
step() { local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc: $(tail -n 1 gpurun_out/$name.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then exit $rc; fi; }
step gpu_suite 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
cp gpurun_out/gpu_suite.log gpurun_out/profiles/${TAG}_gpu_suite.log
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
TAG=$TAG CONFIGS="C2:512 C4:1024 C5:256 NW9:64:1080" bash tools/evidence_r3.sh || exit 1
for c in C4 C5 NW9; do
  step bench_$c 300 python3 bench.py --config $c --no-cpu-baseline --no-extra --no-breakdown  # f64_books on C4 / C5
  grep -v "^W20\|amdgpu.ids" gpurun_out/bench_$c.log | tail -n 1 > gpurun_out/profiles/${TAG}_bench_$c.json
done
step scenes 600 python3 tools/bench_scenes.py
grep "^{" gpurun_out/scenes.log > gpurun_out/profiles/${TAG}_scenes.jsonl
