"""Turn two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs, as MI355X_MICROARCH.md
§HBM prescribes) over one full-size render launch into profiles/traffic_<config>.json, which
bench.py reports as roofline.traffic (HBM bytes per launch).

FETCH_SIZE / WRITE_SIZE are in KiB and count the L2's memory-side requests. gfx950 caveat:
FETCH_SIZE reads half the bytes of a wide 16-B/lane streaming read; this kernel's reads are
L2-resident scene gathers and its only streaming traffic is the accum write, so the raw
values are reported alongside the corrected upper bound (2 x FETCH_SIZE + WRITE_SIZE).
    python tools/pmc_traffic.py <fetch_dir> <write_dir> <config> <width> <spp> <out_json> [f64]
The f64 books kernel's launch (trailing argument `f64`): rrt_render64, with its in-order tail fold
(rrt_fold_samples64) reported as the combine step.
"""
import csv
import glob
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counter(d, name, kernel="rrt_render"):
    """Sum of `name` over the dispatches whose kernel name contains `kernel` in one render call
    (tools/prof_render.py --iters 1; rocprofv3 writes one row per dispatch and counter, values summed
    over the row's dimensions): a frame the f64 kernel renders in several sample passes (C4's 1024
    samples: 4 dispatches) counts all of them. Round 5 averaged per dispatch, which reported a quarter
    of C4's f64 frame."""
    per = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == name:
                key = (path, r.get("Dispatch_Id") or r.get("Correlation_Id") or len(per))
                per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    vals = list(per.values())
    if not vals:
        if kernel != "rrt_render":
            return 0.0, 0
        raise SystemExit(f"no {name} rows in {d}")
    return sum(vals), len(vals)


def main(fetch_dir, write_dir, config, width, spp, out, f64=""):
    f64 = f64 == "f64"
    fetch_kib, n1 = counter(fetch_dir, "FETCH_SIZE")
    write_kib, n2 = counter(write_dir, "WRITE_SIZE")
    combine = "rrt_fold_samples64" if f64 else "rrt_combine_chunks"
    cf_kib, nc = counter(fetch_dir, "FETCH_SIZE", combine)
    cw_kib, _ = counter(write_dir, "WRITE_SIZE", combine)
    so = os.path.join(ROOT, "rustraytrace_amd", "librrt_hip.so")
    rec = {
        "config": config,
        "f64": f64,
        "width": int(width),
        "spp": int(spp),
        "dispatches": [n1, n2],
        "fetch_size_kib": fetch_kib,
        "write_size_kib": write_kib,
        "hbm_bytes_per_launch": int((fetch_kib + write_kib) * 1024),
        "hbm_bytes_per_launch_fetch_corrected": int((2 * fetch_kib + write_kib) * 1024),
        "combine_dispatches": nc,
        "combine_fetch_size_kib": cf_kib,
        "combine_write_size_kib": cw_kib,
        "lib_sha256": hashlib.sha256(open(so, "rb").read()).hexdigest(),
        "note": "separate --pmc passes FETCH_SIZE / WRITE_SIZE on tools/prof_render.py --iters 1 (one render call: "
                "the sum over its render dispatches)",
    }
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main(*sys.argv[1:])
