#!/bin/bash
# Round-end evidence, part A (one gpurun call): GPU suite, smoke(), the PMC / rocprof / bench
# evidence of tools/evidence_r3.sh for C2, C4, C5 and final_scene. Part B: tools/evidence_b.sh.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r3z}
mkdir -p gpurun_out/profiles
step() { local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc: $(tail -n 1 gpurun_out/$name.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then exit $rc; fi; }
step gpu_suite 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
cp gpurun_out/gpu_suite.log gpurun_out/profiles/${TAG}_gpu_suite.log
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
TAG=$TAG CONFIGS="${CONFIGS:-C2:512 C4:1024 C5:256 NW9:64:1080}" bash tools/evidence_r3.sh || exit 1
