#!/bin/bash
# Same-box A/B over "name:variant:ENV=V,ENV2=V2" specs (variant = variants/<variant>/librrt_hip.so),
# ROUNDS passes interleaved; one C2 bench line each (value, kernel ms, node visits, sphere tests per ray).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; v=${rest%%:*}; envs=${rest#*:}
  [ "$envs" = "$rest" ] && envs=""
  ( export RRT_LIB_PATH=variants/$v/librrt_hip.so; for kv in ${envs//,/ }; do export "$kv"; done
    timeout -k 10 300 python bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-breakdown --no-f64 --no-extra ${BENCH_ARGS:-} > gpurun_out/ab_$name.log 2>&1 )
  rc=$?
  echo "r$r $name rc=$rc $(python -c "
import json;d=json.loads(open('gpurun_out/ab_$name.log').read().splitlines()[-1]);r=d['rank0_rays_per_launch']
a=d['roofline']['algorithmic_flop_per_launch'];b=d['roofline']['algorithmic_scene_bytes_per_launch']
nv=(23*b-16*a)/(23*56-16*24);st=(b-56*nv)/16
print(d['value'],'Mrays/s',d['kernel_ms_avg'],'ms','nodes/ray %.3f spheres/ray %.3f'%(nv/r,st/r))" 2>/dev/null)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab_$name.log; exit $rc; fi
done
done
