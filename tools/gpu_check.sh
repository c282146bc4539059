#!/bin/bash
# One GPU session: parity tests, smoke, short bench. Stops at the first step that faults,
# aborts or times out (exit >= 124 or signal); plain test failures (rc 1) do not stop it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 600 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py ${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline}
if [ -n "${PROFILE:-}" ]; then
  export TMPDIR=/tmp
  step rocprof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
  find gpurun_out/prof -name "*stats*" | head -5
fi
