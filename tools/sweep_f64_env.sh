#!/bin/bash
# Same-box sweep of the f64 kernel's traversal-exit / leaf-batch thresholds (x/256 of the live
# lanes): "name:TRAV/LEAF" specs, ROUNDS passes interleaved, bench.py's f64_books leg on CONFIG.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
for spec in "$@"; do
  name=${spec%%:*}; tl=${spec#*:}
  ( if [ "$tl" != "default" ]; then export RRT_TRAV_FRAC=${tl%/*} RRT_LEAF_FRAC=${tl#*/}; fi
    timeout -k 10 300 python bench.py --config ${CONFIG:-C2} --steps 1 --warmup 1 --no-cpu-baseline --no-breakdown --no-extra > gpurun_out/sf_$name.log 2>&1 )
  rc=$?
  echo "r$r ${CONFIG:-C2} $name ($tl) rc=$rc $(python -c "import json;d=json.loads(open('gpurun_out/sf_$name.log').read().splitlines()[-1]);f=d['f64_books'];print(f['value'],'f64 Mrays/s',f['ms_per_frame'],'ms')" 2>/dev/null)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/sf_$name.log; exit $rc; fi
done
done
