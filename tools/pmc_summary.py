"""Summarise rocprofv3 --pmc CSVs: per-dispatch averages of the render kernel's counters."""
import collections
import csv
import glob
import sys


def summarise(prefix):
    agg = collections.defaultdict(float)
    nd = {}
    for path in sorted(glob.glob(f"{prefix}*/p_counter_collection.csv")):
        for r in csv.DictReader(open(path)):
            if "rrt_render" not in r["Kernel_Name"]:
                continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            nd.setdefault(r["Counter_Name"], set()).add((path, r["Dispatch_Id"]))
    out = {k: v / len(nd[k]) for k, v in agg.items()}
    if "SQ_THREAD_CYCLES_VALU" in out and "SQ_INSTS_VALU" in out:
        out["lanes_per_valu_inst"] = out["SQ_THREAD_CYCLES_VALU"] / out["SQ_INSTS_VALU"]
    if "SQ_WAVE_CYCLES" in out and "SQ_ACTIVE_INST_ANY" in out:
        out["active_frac"] = out["SQ_ACTIVE_INST_ANY"] / out["SQ_WAVE_CYCLES"]
        out["wait_inst_frac"] = out.get("SQ_WAIT_INST_ANY", 0) / out["SQ_WAVE_CYCLES"]
        out["wait_any_frac"] = out.get("SQ_WAIT_ANY", 0) / out["SQ_WAVE_CYCLES"]
    return out


if __name__ == "__main__":
    for pre in sys.argv[1:]:
        print(pre, {k: f"{v:.4g}" for k, v in sorted(summarise(pre).items())})
