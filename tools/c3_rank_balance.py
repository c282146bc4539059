"""Per-rank render time of a config's row-band split, every rank's tile rendered on this one GPU
in turn (HIP events on the render stream): the load balance `bench.py --gpus N` will see on N
GPUs, before any gather. Prints one JSON line per N with each rank's kernel ms, max/mean - 1 and
rays per rank.

    python tools/c3_rank_balance.py [--config C3] [--ranks 2 4 8] [--spp S] [--reps 1]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--ranks", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--bands", type=int, nargs="*", default=None,
                    help="band heights to try (default: distributed.balanced_band per rank count)")
    a = ap.parse_args()
    import numpy as np
    import torch

    import rustraytrace_amd as rrt
    from rustraytrace_amd.distributed import balanced_band

    kw = {"samples_per_pixel": a.spp} if a.spp else {}
    scene = rrt.config_scene(a.config, **kw)
    ds = rrt.DeviceScene(scene)
    stream = torch.cuda.current_stream()
    for n, band in [(n, b) for n in a.ranks for b in (a.bands or [balanced_band(scene.height, n)])]:
        ms, rays = [], []
        for r in range(n):
            tile = ds.tile(band_rows=band, rank=r, n_ranks=n, sample_begin=0, sample_end=scene.spp)
            rows = ds.tile_rows(tile)
            buf = torch.empty((max(rows, 1), scene.width, 4), dtype=torch.float32, device="cuda")
            ds.render_tile_async(tile, buf.data_ptr(), stream.cuda_stream)  # warm
            torch.cuda.synchronize()
            ds.reset_counters()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps + 1)]
            for i in range(a.reps):
                ev[i].record(stream)
                ds.render_tile_async(tile, buf.data_ptr(), stream.cuda_stream)
            ev[a.reps].record(stream)
            torch.cuda.synchronize()
            ms.append(float(np.mean([ev[i].elapsed_time(ev[i + 1]) for i in range(a.reps)])))
            rays.append(int(ds.counters()["rays"] // a.reps))
            del buf
        mean = float(np.mean(ms))
        print(json.dumps({"config": a.config, "image": [scene.width, scene.height], "spp": scene.spp, "ranks": n,
                          "band_rows": band, "rank_ms": [round(x, 2) for x in ms], "sum_ms": round(sum(ms), 2),
                          "max_over_mean": round(max(ms) / mean - 1.0, 5),
                          "rays_max_over_mean": round(max(rays) / float(np.mean(rays)) - 1.0, 5), "rays": rays}),
              flush=True)
    ds.close()


if __name__ == "__main__":
    main()
