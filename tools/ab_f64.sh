#!/bin/bash
# Same-box A/B of the f64 books kernel across variants/<name>/librrt_hip.so, ROUNDS passes
# interleaved: bench.py's f64_books leg (CONFIG, default C2) per variant (VARIANTS, default all).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
for n in ${VARIANTS:-$(ls variants)}; do
  d=variants/$n
  RRT_LIB_PATH=$d/librrt_hip.so timeout -k 10 300 python bench.py --config ${CONFIG:-C2} --steps 1 --warmup 1 --no-cpu-baseline --no-breakdown --no-extra > gpurun_out/abf_$n.log 2>&1
  rc=$?
  echo "r$r ${CONFIG:-C2} $n rc=$rc $(python -c "import json;d=json.loads(open('gpurun_out/abf_$n.log').read().splitlines()[-1]);f=d['f64_books'];print(d['value'],'f32 Mrays/s |',f['value'],'f64 Mrays/s',f['ms_per_frame'],'ms')" 2>/dev/null)" | tee -a gpurun_out/ab_f64_summary.log
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/abf_$n.log; exit $rc; fi
done
done
