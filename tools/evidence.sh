#!/bin/bash
# End-of-round evidence on one GPU, final library: the GPU suite, smoke(), the bench lines (C2
# default with its f64 leg; C4, C5, NW9), rocprofv3 kernel stats of each bench command (the
# rocprof average must agree with the line's kernel_ms_avg) and of the f64 C2 frame, the issue-side
# PMC pass and the HBM traffic passes per config (f32 and the f64 C2 launch). Stops at the first
# failing step. TAG names the outputs (gpurun_out/profiles/<TAG>_*); STEPS=suite,bench,multi,stats,issue,traffic
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r5}
STEPS=${STEPS:-suite,bench,multi,stats,issue,traffic}
mkdir -p gpurun_out/profiles
run() { local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -n 2 "gpurun_out/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi; }
if [[ $STEPS == *suite* ]]; then
  run gpu_suite 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
  cp gpurun_out/gpu_suite.log gpurun_out/profiles/${TAG}_gpu_suite.log
  run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $STEPS == *bench* ]]; then
  run bench 600 python3 bench.py
  tail -n 1 gpurun_out/bench.log > gpurun_out/profiles/${TAG}_bench_full.json
  for c in C4 C5 NW9; do
    run bench_$c 300 python3 bench.py --config $c --no-extra --no-cpu-baseline --no-breakdown
    tail -n 1 gpurun_out/bench_$c.log > gpurun_out/profiles/${TAG}_bench_$c.json
  done
fi
if [[ $STEPS == *multi* ]]; then  # full-size rehearsals of the N > 1 legs on one GPU
  run bench_C3_f64 600 python3 bench.py --config C3 --f64 --steps 2 --warmup 1 --no-cpu-baseline --no-breakdown
  tail -n 1 gpurun_out/bench_C3_f64.log > gpurun_out/profiles/${TAG}_bench_C3_f64.json
  run bench_gpus2_gloo 900 env RRT_BENCH_BACKEND=gloo python3 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline
  tail -n 1 gpurun_out/bench_gpus2_gloo.log > gpurun_out/profiles/${TAG}_bench_gpus2_gloo_rehearsal.json
fi
if [[ $STEPS == *stats* ]]; then
  for c in C2 C4 C5; do
    run kstats_$c 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$c -o run --output-format csv -- python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-breakdown --no-extra --no-f64
    cp gpurun_out/prof_${TAG}_$c/run_kernel_stats.csv gpurun_out/profiles/${TAG}_${c}_kernel_stats.csv
    grep '^{"metric"' gpurun_out/kstats_$c.log | tail -n 1 > gpurun_out/profiles/${TAG}_${c}_kstats_bench.json
  done
  run kstats_C2_f64 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_C2_f64 -o run --output-format csv -- python3 tools/prof_render.py --f64 --config C2 --spp 512 --iters 3 --json gpurun_out/kstats_C2_f64.json
  cp gpurun_out/prof_${TAG}_C2_f64/run_kernel_stats.csv gpurun_out/profiles/${TAG}_C2_f64_kernel_stats.csv
fi
for spec in ${CONFIGS:-C2:512 C4:1024 C5:256 NW9:64:1080 C2f64:512 C4f64:1024 C5f64:256}; do
  c=${spec%%:*}; rest=${spec#*:}; s=${rest%%:*}; w=1920; wa=""; fa=""; cfg=$c; tf=""
  [ "$rest" != "$s" ] && { w=${rest#*:}; wa="--width $w"; }
  [[ $c == *f64 ]] && { cfg=${c%f64}; fa="--f64"; c=${cfg}_f64; tf=f64; }
  if [[ $STEPS == *issue* ]]; then
    run pmc_issue_$c 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/ti_$c -o p --output-format csv -- python3 tools/prof_render.py --config $cfg $fa --spp $s $wa --iters 1 --json gpurun_out/ti_$c.json
    f64dir=""
    if [ -n "$tf" ]; then  # the f64 kernel: its typed f64 instructions weigh 4 issue cycles (tools/pmc_issue.py)
      run pmc_issue64_$c 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE -d gpurun_out/ti64_$c -o p --output-format csv -- python3 tools/prof_render.py --config $cfg $fa --spp $s $wa --iters 1
      f64dir=gpurun_out/ti64_$c
    fi
    run issue_$c 60 python3 tools/pmc_issue.py gpurun_out/ti_$c gpurun_out/ti_$c.json profiles/issue_$c.json $f64dir
    cp profiles/issue_$c.json gpurun_out/profiles/issue_$c.json
  fi
  if [[ $STEPS == *traffic* ]]; then
    run pmc_fetch_$c 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/tf_$c -o p --output-format csv -- python3 tools/prof_render.py --config $cfg $fa --spp $s $wa --iters 1
    run pmc_write_$c 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/tw_$c -o p --output-format csv -- python3 tools/prof_render.py --config $cfg $fa --spp $s $wa --iters 1
    run traffic_$c 60 python3 tools/pmc_traffic.py gpurun_out/tf_$c gpurun_out/tw_$c $cfg $w $s profiles/traffic_$c.json $tf
    cp profiles/traffic_$c.json gpurun_out/profiles/traffic_$c.json
  fi
done
