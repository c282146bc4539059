"""Summarise tools/pmc_mix.sh's two --pmc passes: per-ray VALU instruction counts by type and the
average SQ_ACTIVE_INST_VALU cycles per VALU wave-instruction (quad-cycles x 4).

    python tools/pmc_mix.py <pass A dir> <pass B dir> <render_json> <out_json>
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_issue import per_dispatch  # noqa: E402


def main(da, db, render_json, out):
    a, _ = per_dispatch(da)
    b, _ = per_dispatch(db)
    rj = json.load(open(render_json))
    rays = rj["rays_per_launch"]
    c = {**b, **a}
    per_ray = {k.replace("SQ_INSTS_VALU_", "").replace("SQ_INSTS_", ""): round(v / rays, 3)
               for k, v in c.items() if k.startswith("SQ_INSTS")}
    typed = sum(v for k, v in c.items() if k.startswith("SQ_INSTS_VALU_") and k != "SQ_INSTS_VALU")
    rec = {"config": rj["config"], "width": rj["width"], "spp": rj["spp"], "f64": rj.get("f64", False),
           "rays_per_launch": rays, "per_ray": per_ray,
           "untyped_valu_per_ray": round((c["SQ_INSTS_VALU"] - typed) / rays, 3),
           "f64_share_of_valu": round(sum(c.get(f"SQ_INSTS_VALU_{t}_F64", 0) for t in ("ADD", "MUL", "FMA", "TRANS"))
                                      / c["SQ_INSTS_VALU"], 4),
           "active_valu_cycles_per_inst": round(4.0 * c["SQ_ACTIVE_INST_VALU"] / c["SQ_INSTS_VALU"], 3),
           "counters": c}
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps({k: v for k, v in rec.items() if k != "counters"}))


if __name__ == "__main__":
    main(*sys.argv[1:])
