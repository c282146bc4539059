"""Issue-side roofline of the render kernel from one rocprofv3 --pmc pass over a full-size launch
(tools/prof_render.py --json): profiles/issue_<config>.json, which bench.py reports beside the FLOP
roofline as roofline.valu_busy / lanes_per_valu / valu_insts_per_ray.

  valu_busy          = 2 cycles x SQ_INSTS_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): a wave64 VALU
                       instruction holds a SIMD-32 for 2 cycles (MI355X_MICROARCH.md constants
                       table); GRBM_GUI_ACTIVE is summed over the 8 XCDs
  lanes_per_valu     = SQ_THREAD_CYCLES_VALU / SQ_INSTS_VALU (active lanes per VALU wave-instruction, of 64)
  valu_insts_per_ray = SQ_INSTS_VALU / closest-hit queries of the launch

    python tools/pmc_issue.py <pmc_dir> <render_json> <out_json>
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
    """Per-dispatch averages of every counter over the dispatches of kernels named `kernel`."""
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
    return {k: sum(v.values()) / len(v) for k, v in vals.items()}, max(len(v) for v in vals.values())


def main(pmc_dir, render_json, out):
    c, n = per_dispatch(pmc_dir)
    rj = json.load(open(render_json))
    so = os.path.join(ROOT, "rustraytrace_amd", "librrt_hip.so")
    rec = {
        "config": rj["config"], "width": rj["width"], "spp": rj["spp"], "f64": rj.get("f64", False),
        "dispatches": n, "rays_per_launch": rj["rays_per_launch"],
        "counters": {k: c.get(k) for k in COUNTERS},
        "valu_busy": round(2.0 * c["SQ_INSTS_VALU"] / (1024.0 * c["GRBM_GUI_ACTIVE"] / 8.0), 4),
        "lanes_per_valu": round(c["SQ_THREAD_CYCLES_VALU"] / c["SQ_INSTS_VALU"], 2),
        "valu_insts_per_ray": round(c["SQ_INSTS_VALU"] / rj["rays_per_launch"], 2),
        "salu_per_valu": round(c["SQ_INSTS_SALU"] / c["SQ_INSTS_VALU"], 4),
        "lds_conflict_cycles_per_lds_inst": round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_INSTS_LDS"], 3),
        "lib_sha256": hashlib.sha256(open(so, "rb").read()).hexdigest(),
        "note": "one rocprofv3 --pmc pass (8 SQ + 1 GRBM counters, no tracing) over tools/prof_render.py --iters 1",
    }
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main(*sys.argv[1:])
