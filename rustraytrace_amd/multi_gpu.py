"""Multi-rank frame render with the row-band split (3840x2160x2048 spp
tile-split across 8 MI355X, one RCCL gather to rank 0).

One process per GPU, launched by torch.distributed.run:

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 -m rustraytrace_amd.multi_gpu --config C3 --out image.ppm

Every rank builds the same scene and BVH (KB-sized, replicated), renders the row bands it
owns (band b of period p = b // n goes to rank b % n for even p, n - 1 - b % n for odd p) over all samples, and the float tiles are gathered to rank 0
(`distributed.gather_rows`), which writes the render_io.rs PPM. The image is bit-identical to a
1-GPU render: each pixel's samples are keyed by (seed, global pixel, sample) only. Rank 0 prints
one JSON line: the slowest rank's kernel time, the gather time, Mrays/s over all ranks.

`--f64` renders with the f64 books kernel (RRT_FLAG_F64) and gathers f64 tiles; the PPM then comes
from the books path's own quantiser (color.rs), and the frame equals the 1-GPU f64 frame bit for bit.

`--backend gloo` gathers host copies instead of device tensors (ranks may then share a GPU:
device = local rank mod device count); it is the test path on a one-GPU box.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--config", default="C3", help="BASELINE config (C1..C5)")
    ap.add_argument("--width", type=int, default=None, help="image_width override")
    ap.add_argument("--spp", type=int, default=None, help="samples_per_pixel override")
    ap.add_argument("--depth", type=int, default=None, help="max_depth override")
    ap.add_argument("--band", type=int, default=0,
                    help="rows per band (0: the largest of 16..8 that gives every rank the same rows, else 16)")
    ap.add_argument("--backend", default=None, help="nccl (RCCL, default with >1 rank) or gloo")
    ap.add_argument("--out", default=None, help="PPM path on rank 0 ('-' = stdout, default: none)")
    ap.add_argument("--p6", action="store_true", help="binary P6 instead of the reference's P3")
    ap.add_argument("--save-accum", default=None, help="rank 0: save the float accum (.npy)")
    ap.add_argument("--f64", action="store_true",
                    help="the f64 books kernel (RRT_FLAG_F64): f64 tiles gathered, the PPM by the books path's own "
                         "quantiser (color.rs), bit-identical to the 1-GPU f64 frame")
    return ap.parse_args(argv)


def main(argv=None) -> int:
    args = parse(argv)
    import numpy as np
    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import rustraytrace_amd as rrt
    from rustraytrace_amd.distributed import balanced_band, gather_rows

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n_dev = rrt.device_count()
    if n_dev < 1:
        raise RuntimeError("multi_gpu: no HIP device visible")
    device = local % n_dev
    torch.cuda.set_device(device)
    backend = args.backend or "nccl"
    # An explicit --backend runs the process group and the gather even with one rank (the
    # RCCL init + gather path exercised on a one-GPU box; RCCL refuses two ranks on one GPU).
    use_dist = world > 1 or args.backend is not None
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {"device_id": torch.device(f"cuda:{device}")} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)

    over = {}
    if args.width:
        over["image_width"] = args.width
    if args.spp:
        over["samples_per_pixel"] = args.spp
    if args.depth:
        over["max_depth"] = args.depth
    scene = rrt.config_scene(args.config, **over)
    W, H, S = scene.width, scene.height, scene.spp

    ds = rrt.DeviceScene(scene, device=device, f64=args.f64)
    if args.band <= 0:
        args.band = balanced_band(H, world)
    tile = ds.tile(band_rows=args.band, rank=rank, n_ranks=world, sample_begin=0, sample_end=S)
    rows = ds.tile_rows(tile)
    accum = torch.empty((max(rows, 1), W, 4), dtype=torch.float64 if args.f64 else torch.float32,
                        device=f"cuda:{device}")
    render = ds.render_tile_f64_async if args.f64 else ds.render_tile_async
    stream = torch.cuda.current_stream()
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    start.record(stream)
    if rows:
        render(tile, accum.data_ptr(), stream.cuda_stream)
    end.record(stream)
    torch.cuda.synchronize()
    kernel_ms = start.elapsed_time(end)
    rays = ds.counters()["rays"]
    ds.close()

    local_rows = accum[:rows]
    t = time.perf_counter()
    if use_dist:
        src = local_rows if backend == "nccl" else local_rows.cpu()
        img = gather_rows(src, H, args.band, dist)
        if backend == "nccl":
            torch.cuda.synchronize()
    else:
        img = local_rows
    gather_ms = (time.perf_counter() - t) * 1e3
    if use_dist:
        dev = f"cuda:{device}" if backend == "nccl" else "cpu"
        stats = torch.tensor([kernel_ms, float(rays)], dtype=torch.float64, device=dev)
        kmax = stats[:1].clone()
        dist.all_reduce(kmax, op=dist.ReduceOp.MAX)
        tot = stats[1:].clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        kernel_ms, rays = float(kmax.item()), int(tot.item())

    if rank == 0:
        host = img.cpu().numpy()
        if args.save_accum:
            np.save(args.save_accum, host)
        if args.out and args.f64:  # the books path's PPM (camera.rs:87-94 through color.rs:6-32)
            rgb8 = rrt.quantize_accum_books_f64(W, H, host, S)
            rrt.write_pnm_from_rgb8(W, H, rgb8, args.p6, args.out)
        elif args.out:
            if args.p6:
                rgb8 = rrt.quantize_accum(W, H, host, S)
                rrt.write_pnm_from_rgb8(W, H, rgb8, True, args.out)
            else:
                rrt.write_ppm_from_accum(W, H, host, S, args.out)
        print(json.dumps({
            "config": args.config, "image": [W, H], "spp": S, "ranks": world, "backend": backend if use_dist else None,
            "dtype": "f64" if args.f64 else "f32",
            "split": f"{args.band}-row bands dealt in serpentine order", "kernel_ms_max_over_ranks": round(kernel_ms, 3),
            "gather_ms": round(gather_ms, 3), "rays": rays, "mrays_per_s": round(rays / kernel_ms / 1e3, 2),
        }), file=sys.stderr if args.out == "-" else sys.stdout, flush=True)
    if use_dist:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
