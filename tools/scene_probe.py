"""Per-scene work profile of the render kernel on one GPU: HIP-event kernel time over --iters
launches (after one warm-up), rays, and the instrumented twin kernel's per-launch work counts
(node visits, box tests, primitive tests per ray). One JSON line per scene.

    python tools/scene_probe.py --scenes NW9 C5 --spp 16 [--width 1080] [--iters 2]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make_scene(name, spp, width):
    import numpy as np

    import rustraytrace_amd as rrt

    if "-" in name:  # experiment variants of a scene: NW9-nofog (no r >= 1000 sphere medium),
        # NW9-nonoise (noise Lambertians as plain ones), NW9-nomedia
        base, mod = name.split("-", 1)
        sc = make_scene(base, spp, width)
        if mod in ("nofog", "nomedia") and sc.media is not None:
            keep = [m for m in sc.media if mod == "nofog" and not (m["boundary_kind"] == 0 and m["sphere"][3] >= 1000)]
            sc.media = np.array(keep, dtype=sc.media.dtype) if keep else None
        if mod == "nonoise":
            sc.materials["kind"][sc.materials["kind"] == 6] = 0
        return sc

    if name.startswith("C"):
        kw = dict(samples_per_pixel=spp)
        if width:
            kw["image_width"] = width
        return rrt.config_scene(name, **kw)
    if name.startswith("NW"):
        n = int(name[2:])
        kw = dict(image_width=width or 1080, samples_per_pixel=spp)
        if n != 9:
            kw["max_depth"] = 50
        return rrt.next_week_scene(n, kw)
    if name == "B3":
        return rrt.rest_of_your_life_scene(dict(image_width=width or 1080, samples_per_pixel=spp, max_depth=50))
    raise SystemExit(f"unknown scene {name}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", nargs="+", default=["NW9"])
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--iters", type=int, default=2)
    a = ap.parse_args()
    import torch

    import rustraytrace_amd as rrt

    for name in a.scenes:
        sc = make_scene(name, a.spp, a.width)
        ds = rrt.DeviceScene(sc)
        tile = ds.tile(16, 0, 1, 0, sc.spp)
        buf = torch.empty((sc.height, sc.width, 4), dtype=torch.float32, device="cuda:0")
        stream = torch.cuda.current_stream()
        ds.render_tile_async(tile, buf.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        ds.reset_counters()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record(stream)
        for _ in range(a.iters):
            ds.render_tile_async(tile, buf.data_ptr(), stream.cuda_stream)
        t1.record(stream)
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / a.iters
        raw = ds.counters()
        rays = raw["rays"] // a.iters
        w = ds.count_work(tile)
        r = max(1, w["rays"])
        print(json.dumps({
            "scene": name, "width": sc.width, "height": sc.height, "spp": sc.spp, "max_depth": sc.max_depth,
            "kernel_ms": round(ms, 3), "rays": rays, "grays_s": round(rays / ms / 1e6, 3),
            "rays_per_path": round(w["rays"] / max(1, w["paths"]), 3),
            "nodes_per_ray": round(w["node_visits"] / r, 3), "prim_tests_per_ray": round(w["sphere_tests"] / r, 3),
            "bvh": ds.bvh_info(), "raw_counters": raw,
        }), flush=True)
        ds.close()


if __name__ == "__main__":
    main()
