#!/bin/bash
# Round-3 evidence on one GPU: the issue-side PMC pass (tools/pmc_issue.py) and the HBM traffic
# passes (FETCH_SIZE / WRITE_SIZE in separate runs) of a full-size launch per config, rocprofv3
# kernel stats of the bench command, the bench line. Stops at the first failing step.
# TAG names the outputs (profiles/<TAG>_*); CONFIGS = config:spp[:width] list (NW9:64:1080);
# STEPS=issue,traffic,stats,bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r3}
STEPS=${STEPS:-issue,traffic,stats,bench}
mkdir -p gpurun_out/profiles
run() { local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -n 2 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi; }
for spec in ${CONFIGS:-C2:512}; do
  c=${spec%%:*}; rest=${spec#*:}; s=${rest%%:*}; w=1920; wa=""
  [ "$rest" != "$s" ] && { w=${rest#*:}; wa="--width $w"; }
  if [[ $STEPS == *issue* ]]; then
    run pmc_issue_$c 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/ti_$c -o p --output-format csv -- python3 tools/prof_render.py --config $c --spp $s $wa --iters 1 --json gpurun_out/ti_$c.json
    run issue_$c 60 python3 tools/pmc_issue.py gpurun_out/ti_$c gpurun_out/ti_$c.json profiles/issue_$c.json
    cp profiles/issue_$c.json gpurun_out/profiles/issue_$c.json
  fi
  if [[ $STEPS == *traffic* ]]; then
    run pmc_fetch_$c 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/tf_$c -o p --output-format csv -- python3 tools/prof_render.py --config $c --spp $s $wa --iters 1
    run pmc_write_$c 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/tw_$c -o p --output-format csv -- python3 tools/prof_render.py --config $c --spp $s $wa --iters 1
    run traffic_$c 60 python3 tools/pmc_traffic.py gpurun_out/tf_$c gpurun_out/tw_$c $c $w $s profiles/traffic_$c.json
    cp profiles/traffic_$c.json gpurun_out/profiles/traffic_$c.json
  fi
done
if [[ $STEPS == *stats* ]]; then
  run kstats 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-breakdown --no-extra --no-f64
  cp gpurun_out/prof_$TAG/run_kernel_stats.csv gpurun_out/profiles/${TAG}_kernel_stats.csv
fi
if [[ $STEPS == *bench* ]]; then
  run bench 600 python3 bench.py ${BENCH_ARGS:-}
  tail -n 1 gpurun_out/bench.log > gpurun_out/profiles/${TAG}_bench_full.json
fi
