#!/bin/bash
# Same-box sweep of host-side environment knobs: "name:VAR=V,VAR2=V2" specs ("name:" = defaults),
# ROUNDS passes interleaved, bench.py on CONFIG; prints the f32 line value and the f64_books leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
for spec in "$@"; do
  name=${spec%%:*}; kv=${spec#*:}
  ( IFS=','; for a in $kv; do [ -n "$a" ] && export "$a"; done
    timeout -k 10 300 python bench.py --config ${CONFIG:-C2} --steps ${STEPS:-1} --warmup 1 --no-cpu-baseline --no-breakdown --no-extra ${BENCH_ARGS:-} > gpurun_out/se_$name.log 2>&1 )
  rc=$?
  echo "r$r ${CONFIG:-C2} $name ($kv) rc=$rc $(python -c "
import json;d=json.loads(open('gpurun_out/se_$name.log').read().splitlines()[-1]);f=d.get('f64_books') or {}
print(d['value'],'f32 Mrays/s',d['kernel_ms_avg'],'ms |',f.get('value'),'f64 Mrays/s',f.get('ms_per_frame'),'ms | bvh',d['bvh']['n_nodes'],d['bvh']['max_depth'],d['bvh']['max_leaf_size'])" 2>/dev/null)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/se_$name.log; exit $rc; fi
done
done
