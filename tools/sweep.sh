#!/bin/bash
# Variant sweep on one GPU: parity subset, then bench lines per env setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -q -x > gpurun_out/sweep_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/sweep_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
for v in ${SWEEP:-"RRT_SCENE_IN_LDS=1" "RRT_SCENE_IN_LDS=0"}; do
  env ${v//,/ } timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-breakdown ${BENCH_ARGS:-} > gpurun_out/sweep_bench.log 2>&1
  rc=$?
  echo "$v rc=$rc $(python -c "import json;d=json.loads(open('gpurun_out/sweep_bench.log').read().splitlines()[-1]);print(d['value'],'Mrays/s',d['ms_per_step'],'ms',d['roofline']['frac'])" 2>/dev/null)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/sweep_bench.log; exit $rc; fi
done
