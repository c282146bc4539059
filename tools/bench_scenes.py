"""Mrays/s of every scene the backend renders (BASELINE configs and the book-2 scenes), one GPU:
HIP-event kernel time over `--iters` launches of the full frame after one warm-up, rays counted
by the kernel. One JSON object per line; a summary table on stderr.

    python tools/bench_scenes.py [--spp-scale 0.25] [--iters 3] > gpurun_out/scenes.jsonl
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def scenes(spp_scale):
    import rustraytrace_amd as rrt

    def s(n):
        return max(1, int(n * spp_scale))

    yield "C1 three_spheres 400x225", rrt.config_scene("C1", samples_per_pixel=s(64))
    yield "C2 rtow 1920x1080", rrt.config_scene("C2", samples_per_pixel=s(512))
    yield "C4 earth_light 1920x1080", rrt.config_scene("C4", samples_per_pixel=s(1024))
    yield "C5 rtow 10k spheres 1920x1080", rrt.config_scene("C5", samples_per_pixel=s(256))
    hd = dict(image_width=1920, max_depth=50)
    yield "NW1 bouncing_spheres 1920x1080", rrt.next_week_scene(1, dict(hd, samples_per_pixel=s(256)))
    yield "NW2 checkered_spheres 1920x1080", rrt.next_week_scene(2, dict(hd, samples_per_pixel=s(256)))
    yield "NW3 earth 1920x1080", rrt.next_week_scene(3, dict(hd, samples_per_pixel=s(256)))
    yield "NW4 perlin_spheres 1920x1080", rrt.next_week_scene(4, dict(hd, samples_per_pixel=s(256)))
    sq = dict(image_width=1080, max_depth=50)
    yield "NW5 quads 1080x1080", rrt.next_week_scene(5, dict(sq, samples_per_pixel=s(256)))
    yield "NW6 simple_light 1920x1080", rrt.next_week_scene(6, dict(hd, samples_per_pixel=s(256)))
    yield "NW7 cornell_box 1080x1080", rrt.next_week_scene(7, dict(sq, samples_per_pixel=s(256)))
    yield "NW8 cornell_smoke 1080x1080", rrt.next_week_scene(8, dict(sq, samples_per_pixel=s(256)))
    yield "NW9 final_scene 1080x1080 d40", rrt.next_week_scene(9, dict(image_width=1080, samples_per_pixel=s(256)))
    yield "B3 rest_of_your_life 1080x1080", rrt.rest_of_your_life_scene(dict(sq, samples_per_pixel=s(256)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp-scale", type=float, default=0.25)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    import torch

    import rustraytrace_amd as rrt

    rows = []
    for name, sc in scenes(a.spp_scale):
        ds = rrt.DeviceScene(sc)
        tile = ds.tile(16, 0, 1, 0, sc.spp)
        buf = torch.empty((sc.height, sc.width, 4), dtype=torch.float32, device="cuda:0")
        stream = torch.cuda.current_stream()
        ds.render_tile_async(tile, buf.data_ptr(), stream.cuda_stream)  # warm-up
        torch.cuda.synchronize()
        ds.reset_counters()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record(stream)
        for _ in range(a.iters):
            ds.render_tile_async(tile, buf.data_ptr(), stream.cuda_stream)
        t1.record(stream)
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / a.iters
        ctr = ds.counters()
        info = ds.bvh_info()
        ds.close()
        rays = ctr["rays"] / a.iters
        row = dict(scene=name, width=sc.width, height=sc.height, spp=sc.spp, max_depth=sc.max_depth,
                   spheres=len(sc.spheres), quads=0 if sc.quads is None else len(sc.quads), kernel_ms=round(ms, 3), rays_per_frame=int(rays),
                   mrays_per_s=round(rays / ms / 1e3, 1), rays_per_path=round(rays / (sc.width * sc.height * sc.spp), 3),
                   bvh_nodes=info["n_nodes"])
        rows.append(row)
        print(json.dumps(row), flush=True)
    for r in rows:
        print(f"{r['scene']:34s} {r['spp']:5d} spp  {r['kernel_ms']:9.2f} ms  {r['mrays_per_s']:9.1f} Mrays/s  "
              f"{r['rays_per_path']:.2f} rays/path", file=sys.stderr)


if __name__ == "__main__":
    main()
