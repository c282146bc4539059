"""Render a config a few times through the device API (a short, fixed workload for rocprofv3)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--f64", action="store_true", help="the f64 books kernel (RRT_FLAG_F64)")
    ap.add_argument("--json", default=None, help="write {config, width, spp, rays_per_launch, ...} here")
    a = ap.parse_args()
    import torch

    import rustraytrace_amd as rrt

    kw = dict(samples_per_pixel=a.spp)
    if a.width:
        kw["image_width"] = a.width
    scene = rrt.named_scene(a.config, **kw)
    ds = rrt.DeviceScene(scene, f64=a.f64)
    tile = ds.tile(16, 0, 1, 0, scene.spp)
    buf = torch.empty((scene.height, scene.width, 4), dtype=torch.float32, device="cuda:0")
    for _ in range(a.iters):
        ds.render_tile_async(tile, buf.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ctr = ds.counters()
    print(a.config, scene.width, scene.height, scene.spp, ctr, ds.bvh_info())
    if a.json:
        import json

        with open(a.json, "w") as f:
            json.dump({"config": a.config, "width": scene.width, "spp": scene.spp, "f64": a.f64, "iters": a.iters,
                       "rays_per_launch": ctr["rays"] // max(a.iters, 1),
                       "paths_per_launch": ctr["paths"] // max(a.iters, 1), "counters": ctr}, f)


if __name__ == "__main__":
    main()
