#!/bin/bash
# Round-2 evidence session on one GPU: PMC HBM passes (FETCH_SIZE / WRITE_SIZE in separate runs,
# TCC hit/miss) for C2 512 spp, C4 1024 spp and C5 256 spp (their configured sizes), rocprofv3
# kernel stats of the C4/C5 bench commands, and the C4/C5 bench lines. Stops at the first failing
# step. TAG names the outputs (profiles/<TAG>_*).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r2}
mkdir -p gpurun_out/profiles
run() { local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -n 2 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi; }
for spec in ${CONFIGS:-C2:512 C4:1024 C5:256}; do
  c=${spec%%:*}; s=${spec##*:}
  run pmc_fetch_$c 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/tf_$c -o p --output-format csv -- python3 tools/prof_render.py --config $c --spp $s --iters 1
  run pmc_write_$c 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/tw_$c -o p --output-format csv -- python3 tools/prof_render.py --config $c --spp $s --iters 1
  run traffic_$c 60 python3 tools/pmc_traffic.py gpurun_out/tf_$c gpurun_out/tw_$c $c 1920 $s profiles/traffic_$c.json
  cp profiles/traffic_$c.json gpurun_out/profiles/traffic_$c.json
done
if [ -z "${SKIP_TCC:-}" ]; then
  run pmc_tcc_C5 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/tcc_C5 -o p --output-format csv -- python3 tools/prof_render.py --config C5 --spp 256 --iters 1
fi
for c in ${BENCH_CONFIGS:-C4 C5}; do
  run kstats_$c 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$c -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-breakdown --no-extra
  run bench_$c 300 python3 bench.py --config $c --steps 3 --warmup 1 --no-breakdown --no-extra --cpu-seconds 8
  tail -n 1 gpurun_out/bench_$c.log > gpurun_out/profiles/${TAG}_bench_$c.json
  cp gpurun_out/prof_${TAG}_$c/run_kernel_stats.csv gpurun_out/profiles/${TAG}_${c}_kernel_stats.csv
done
