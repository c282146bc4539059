#!/bin/bash
# Same-box A/B of every variants/<name>/librrt_hip.so, ROUNDS passes interleaved (C2 bench lines).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
if [ -n "$VARIANTS" ]; then DIRS=$(printf "variants/%s/ " $VARIANTS); else DIRS=$(ls -d variants/*/); fi
for d in $DIRS; do
  n=$(basename $d)
  RRT_LIB_PATH=$d/librrt_hip.so timeout -k 10 300 python bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-breakdown --no-f64 ${BENCH_ARGS:-} > gpurun_out/ab_$n.log 2>&1
  rc=$?
  echo "r$r $n rc=$rc $(python -c "import json;d=json.loads(open('gpurun_out/ab_$n.log').read().splitlines()[-1]);print(d['value'],'Mrays/s',d['ms_per_step'],'ms')" 2>/dev/null)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab_$n.log; exit $rc; fi
done
done
