#!/bin/bash
# Bench every variants/<name>/librrt_hip.so (RRT_MIN_WAVES=6 selects its launch-bounds variant).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for d in variants/*/; do
  n=$(basename $d)
  RRT_LIB_PATH=$d/librrt_hip.so RRT_MIN_WAVES=${MINW:-6} timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-breakdown --no-f64 ${BENCH_ARGS:-} > gpurun_out/var_$n.log 2>&1
  rc=$?
  echo "$n rc=$rc $(python -c "import json;d=json.loads(open('gpurun_out/var_$n.log').read().splitlines()[-1]);print(d['value'],'Mrays/s',d['ms_per_step'],'ms')" 2>/dev/null)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/var_$n.log; exit $rc; fi
done
