#!/bin/bash
# GPU-side trace of one path: find the first differing (pixel, sample) with tools/debug_pixel.py,
# build a librrt_hip variant that printf-traces that path (RRT_TRACE_X/Y/S) and run it.
# Usage: [WARMUP="<scene expr>;..."] tools/trace_pixel.sh "<scene expr>"
cd "$(dirname "$0")/.."
set -e
timeout -k 10 300 python3 tools/debug_pixel.py "$1" gpurun_out/trace_target.txt
read X Y S < gpurun_out/trace_target.txt
bash tools/build_variants.sh "trace:-DRRT_TRACE_X=$X -DRRT_TRACE_Y=$Y -DRRT_TRACE_S=$S"
cat > /tmp/trace_run.py <<PY
import sys, numpy as np
sys.path.insert(0, ".")
import rustraytrace_amd as rrt
from rustraytrace_amd.render import build_bvh
from oracle import oracle
import os
for w in os.environ.get("WARMUP", "").split(";"):
    if w and sys.argv[2] == "gpu":
        rrt.render(eval(w, {"rrt": rrt, "np": np}))
sc = eval(sys.argv[1], {"rrt": rrt, "np": np})
if sys.argv[2] == "gpu":
    rrt.render(sc)
else:
    nodes, order, info = build_bvh(sc)
    oracle.render_kbvh(sc, nodes, order, info["width"], rows=($Y, $Y + 1), samples=($S, $S + 1))
PY
RRT_LIB_PATH=variants/trace/librrt_hip.so timeout -k 10 300 python3 /tmp/trace_run.py "$1" gpu > gpurun_out/trace_gpu.txt 2>&1
grep "^K" gpurun_out/trace_gpu.txt | head -60
