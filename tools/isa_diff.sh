#!/bin/bash
# Per-kernel ISA comparison of rrt_kernel.hip between a git revision and the working tree:
# device assembly of both, split per function, instruction lines compared (SAME / DIFF).
#   tools/isa_diff.sh [REV=HEAD]
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
T=$(mktemp -d)
F="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-fast-math -fno-slp-vectorize -mllvm -amdgpu-sched-strategy=iterative-ilp --cuda-device-only -S"
mkdir -p $T/old
for f in rrt_kernel.hip rrt_internal.h rrt_device.h; do git show $REV:rustraytrace_amd/csrc/$f > $T/old/$f; done
/opt/rocm/bin/hipcc $F $T/old/rrt_kernel.hip -o $T/old.s || exit 1
/opt/rocm/bin/hipcc $F rustraytrace_amd/csrc/rrt_kernel.hip -o $T/new.s || exit 1
python3 - $T/old.s $T/new.s <<'PY'
import re, sys
def funcs(path):
    out, cur = {}, None
    for line in open(path):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            cur = m.group(1); out[cur] = []
            continue
        if cur and line.startswith("\t.size\t" + cur):
            cur = None
            continue
        if cur and line.startswith("\t") and not line.startswith("\t.") and not line.startswith("\t;"):
            out[cur].append(line.split(";")[0].strip())
    return out
a, b = funcs(sys.argv[1]), funcs(sys.argv[2])
for k in sorted(set(a) | set(b)):
    s = "SAME" if a.get(k) == b.get(k) else "DIFF"
    print(s, len(a.get(k, [])), len(b.get(k, [])), k[:110])
PY
rm -rf $T
