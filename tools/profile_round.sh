#!/bin/bash
# Evidence session: PMC traffic passes, rocprof kernel stats of the bench, full bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
TAG=${TAG:-r1}
run() { local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -n 3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi; }
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/traffic_fetch -o p --output-format csv -- python3 tools/prof_render.py --config C2 --spp 512 --iters 1
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/traffic_write -o p --output-format csv -- python3 tools/prof_render.py --config C2 --spp 512 --iters 1
run traffic 60 python3 tools/pmc_traffic.py gpurun_out/traffic_fetch gpurun_out/traffic_write C2 1920 512 profiles/traffic_C2.json
cp profiles/traffic_C2.json gpurun_out/profiles/traffic_C2.json
# C5 (10k spheres, BVH and spheres in HBM/L2, not LDS): SURVEY 8(d)'s HBM run, 64 spp
run pmc_fetch_c5 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/traffic_fetch_c5 -o p --output-format csv -- python3 tools/prof_render.py --config C5 --spp 64 --iters 1
run pmc_write_c5 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/traffic_write_c5 -o p --output-format csv -- python3 tools/prof_render.py --config C5 --spp 64 --iters 1
run pmc_tcc_c5 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/traffic_tcc_c5 -o p --output-format csv -- python3 tools/prof_render.py --config C5 --spp 64 --iters 1
run traffic_c5 60 python3 tools/pmc_traffic.py gpurun_out/traffic_fetch_c5 gpurun_out/traffic_write_c5 C5 1920 64 profiles/traffic_C5.json
cp profiles/traffic_C5.json gpurun_out/profiles/traffic_C5.json
run kstats_c5 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_$TAG -o run --output-format csv -- python3 tools/prof_render.py --config C5 --spp 64 --iters 2
run rocprof_stats 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline
run bench_full 900 python3 bench.py
cp gpurun_out/bench_full.log gpurun_out/profiles/bench_$TAG.json
