"""Every compile-time arm left in the kernel sources is the shipped default or compiled here.

rrt_kernel.hip keeps only debug builds (-DRRT_PHASE_TIMING=1..9: per-wave phase statistics,
-DRRT_TRACE_X/Y/S: a printf trace of one path) and numeric tuning knobs (launch shapes, issue
priorities, the work-unit tile). Rejected variants are deleted (DESIGN.md §5 keeps their
measurements). Each non-default arm is type-checked for gfx950 here (hipcc -fsyntax-only
instantiates every kernel template the launch functions reference), so none of them rots.
CPU only: hipcc cross-compiles without a GPU.
"""
import os
import shutil
import subprocess

import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rustraytrace_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

VARIANTS = {
    "phase1": ["-DRRT_PHASE_TIMING=1"],
    "phase2": ["-DRRT_PHASE_TIMING=2"],
    "phase3": ["-DRRT_PHASE_TIMING=3"],
    "phase4": ["-DRRT_PHASE_TIMING=4"],
    "phase5": ["-DRRT_PHASE_TIMING=5"],
    "phase6": ["-DRRT_PHASE_TIMING=6"],
    "phase7": ["-DRRT_PHASE_TIMING=7"],
    "phase8": ["-DRRT_PHASE_TIMING=8"],
    "phase9": ["-DRRT_PHASE_TIMING=9"],
    # the noise texture's generic-pointer reads, rolled corner loop, inlined evaluation; and the
    # debug stand-in that prices the texture
    "noise": ["-DRRT_PERLIN_LDS_PTR=0", "-DRRT_NOISE_UNROLL=0", "-DRRT_NOISE_CALL=0", "-DRRT_DEBUG_NOISE_FIXED=1"],
    # noise textures evaluated per lane only; the wave pass as a call, unrolled, for every count
    "noise_per_lane": ["-DRRT_NOISE_WAVE=0"],
    "noise_wave": ["-DRRT_NOISE_WAVE_CALL=1", "-DRRT_WAVE_NOISE_UNROLL=1", "-DRRT_NOISE_WAVE_MAX=64"],
    "trace": ["-DRRT_TRACE_X=3", "-DRRT_TRACE_Y=4", "-DRRT_TRACE_S=5"],
    # lazy exact roots in the leaf loop (bit-exact, measured and left off: DESIGN.md §4)
    "lazy_root": ["-DRRT_LAZY_ROOT=1", "-DRRT_F64_LAZY=0", "-DRRT_F64_SQRT=0", "-DRRT_F16_ORDERED=0"],
    # the 8-wave class freeing registers (pixel key per path, radiance sum in LDS)
    "lean_8w": ["-DRRT_LEAN_8W=1"],
    # round-6 launch shapes back at their earlier values
    "launch_knobs": ["-DRRT_B1U_WAVES=6", "-DRRT_B1D_WAVES=6", "-DRRT_B3_WAVES=1", "-DRRT_B2_NF_WAVES=5",
                     "-DRRT_B1_GLOBAL_WAVES=6"],
    "knobs": ["-DRRT_BLOCK=256", "-DRRT_WAVES=4", "-DRRT_TILE_W=16", "-DRRT_B2_WAVES=1", "-DRRT_B2_BLOCK=512",
              "-DRRT_PRIO_REFILL=0", "-DRRT_PRIO_NODE=0", "-DRRT_PRIO_LEAF=0", "-DRRT_PRIO_SHADE=0"],
    # rrt_books64.hip: the per-ray reciprocal root division, one class for every scene, f32 nodes in
    # LDS for every LDS scene, launch shape
    "f64_knobs": ["-DRRT_F64_DIVA=0", "-DRRT_F64_CLASSES=0", "-DRRT_F64_BLOCK=256", "-DRRT_F64_WAVES=2"],
    # the f64 kernel's host-formed constants and widened sphere records switched off
    "f64_host": ["-DRRT_F64_CAM64=0", "-DRRT_F64_HOST_INVR=0", "-DRRT_F64_WIDE_SPHERES=0", "-DRRT_F64_R2=0",
                 "-DRRT_F64_DIEL_HOST=0"],
    # the f32 kernel dividing for its dielectric constants, 1 / r and 1 / pr (host-formed by default)
    "diel_kernel": ["-DRRT_DIEL_HOST=0", "-DRRT_INVR_HOST=0", "-DRRT_PR_HOST=0", "-DRRT_DIV_CONST=0", "-DRRT_RCP=0"],
}


@pytest.mark.skipif(not os.path.exists(HIPCC) or shutil.which("make") is None, reason="no hipcc")
@pytest.mark.parametrize("name", sorted(VARIANTS))
def test_kernel_variant_type_checks(name):
    srcs = [f for f in os.listdir(CSRC) if f.endswith(".hip")]
    assert srcs
    for src in srcs:
        cmd = [HIPCC, "--offload-arch=gfx950", "-std=c++17", "-fsyntax-only", "-Wall", "-Wno-unused-function",
               "-Wno-unused-command-line-argument", *VARIANTS[name], os.path.join(CSRC, src)]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, f"{src} [{name}]:\n{r.stderr[-4000:]}"
