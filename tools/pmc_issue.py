"""Issue-side roofline of the render kernel from one rocprofv3 --pmc pass over a full-size launch
(tools/prof_render.py --json): profiles/issue_<config>.json, which bench.py reports beside the FLOP
roofline as roofline.valu_busy / lanes_per_valu / valu_insts_per_ray.

  valu_busy          = VALU issue cycles / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): a wave64 f32 / integer
                       VALU instruction holds a SIMD-32 for 2 cycles, an f64 one for 4 (half the
                       f32 rate: 78.6 against 157.3 TFLOP/s, MI355X_MICROARCH.md constants table);
                       GRBM_GUI_ACTIVE is summed over the 8 XCDs. The f64 instructions come from a
                       second --pmc pass of the typed counters (SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64,
                       <f64_pmc_dir>); without it every instruction counts 2 cycles (exact for the f32
                       kernel, whose f64 share is 0; round 5 reported the f64 kernel that way, 0.555
                       on C2 where the weighted figure is 0.67)
  lanes_per_valu     = SQ_THREAD_CYCLES_VALU / SQ_INSTS_VALU (active lanes per VALU wave-instruction, of 64)
  valu_insts_per_ray = SQ_INSTS_VALU / closest-hit queries of the launch

    python tools/pmc_issue.py <pmc_dir> <render_json> <out_json> [<f64_pmc_dir>]
"""
import csv
import glob
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COUNTERS = ("SQ_INSTS_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT",
            "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_WAVES", "GRBM_GUI_ACTIVE")


def per_dispatch(d, kernel="rrt_render"):
    """Every counter summed over the dispatches of kernels named `kernel` in one render call
    (tools/prof_render.py --iters 1: a frame the f64 kernel renders in several sample passes counts
    all of them; round 5 averaged per dispatch, which divided C4's f64 instructions per ray by 4)."""
    vals = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if kernel not in r["Kernel_Name"]:
                continue
            key = (path, r.get("Dispatch_Id") or r.get("Correlation_Id"))
            vals.setdefault(r["Counter_Name"], {}).setdefault(key, 0.0)
            vals[r["Counter_Name"]][key] += float(r["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {kernel} rows in {d}")
    return {k: sum(v.values()) for k, v in vals.items()}, max(len(v) for v in vals.values())


F64 = ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64")


def valu_cycles(c, f64_counts):
    """Issue cycles of the VALU stream: 2 per wave64 instruction, 4 per f64 one."""
    n64 = sum(f64_counts.get(k, 0.0) for k in F64)
    return 2.0 * (c["SQ_INSTS_VALU"] - n64) + 4.0 * n64, n64


def main(pmc_dir, render_json, out, f64_pmc_dir=None):
    c, n = per_dispatch(pmc_dir)
    f64c = {}
    if f64_pmc_dir:
        f64c, _ = per_dispatch(f64_pmc_dir)
        # the typed pass ran its own launch of the same workload: scale to this pass's VALU count
        scale = c["SQ_INSTS_VALU"] / f64c["SQ_INSTS_VALU"]
        f64c = {k: v * scale for k, v in f64c.items()}
    cyc, n64 = valu_cycles(c, f64c)
    rj = json.load(open(render_json))
    so = os.path.join(ROOT, "rustraytrace_amd", "librrt_hip.so")
    rec = {
        "config": rj["config"], "width": rj["width"], "spp": rj["spp"], "f64": rj.get("f64", False),
        "dispatches": n, "rays_per_launch": rj["rays_per_launch"],
        "counters": {k: c.get(k) for k in COUNTERS},
        "valu_busy": round(cyc / (1024.0 * c["GRBM_GUI_ACTIVE"] / 8.0), 4),
        "valu_busy_2cycle": round(2.0 * c["SQ_INSTS_VALU"] / (1024.0 * c["GRBM_GUI_ACTIVE"] / 8.0), 4),
        "f64_share_of_valu": round(n64 / c["SQ_INSTS_VALU"], 4) if f64_pmc_dir else None,
        "f64_counters": {k: f64c.get(k) for k in F64} if f64_pmc_dir else None,
        "lanes_per_valu": round(c["SQ_THREAD_CYCLES_VALU"] / c["SQ_INSTS_VALU"], 2),
        "valu_insts_per_ray": round(c["SQ_INSTS_VALU"] / rj["rays_per_launch"], 2),
        "salu_per_valu": round(c["SQ_INSTS_SALU"] / c["SQ_INSTS_VALU"], 4),
        "lds_conflict_cycles_per_lds_inst": round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_INSTS_LDS"], 3),
        "lib_sha256": hashlib.sha256(open(so, "rb").read()).hexdigest(),
        "note": "one rocprofv3 --pmc pass (8 SQ + 1 GRBM counters, no tracing) over tools/prof_render.py --iters 1"
                + ("; f64 instructions weighted 4 cycles from a second pass of the typed counters" if f64_pmc_dir else ""),
    }
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main(*sys.argv[1:])
