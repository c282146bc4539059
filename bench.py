"""Benchmark: Mrays/s and wall-clock for the RTOW final scene at 1920x1080x512 spp (BASELINE.json
configs[1] = C2) on MI355X through librrt_hip.so's device-resident C-ABI.

A step = one full C2 frame (every pixel x 512 samples, depth 100) rendered on each rank from
scene data already resident in HBM (BVH built before timing). Ray = one closest-hit query
(camera.rs:187), counted on the device by the kernel itself.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): weak
scaling. Rank r renders its own C2-sized unit of work — the full frame over samples
[512 r, 512 (r+1)) of a 512*N spp image — and the partial accums are gathered to rank 0
over RCCL and summed there in rank order (deterministic). value = rays of all ranks / the
max over ranks of the timed wall-clock.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mrays/sec + wall-clock for 1920×1080×512spp RTOW final scene"
# f32 VALU peak: CDNA4 SIMDs are 32 lanes wide, a wave64 v_fma_f32 issues in 2 cycles
# (MI355X_MICROARCH.md constants table; cdna_hip_programming.md "CU = 4 x SIMD-32"), so
# 256 CU x 4 SIMD x 32 lanes x 2 FLOP x 2.4 GHz = 157.3 TFLOP/s; v_pk_fma_f32 has the same peak.
PEAK_F32_VALU_TFLOPS = 157.3
FLOP_PER_SPHERE_TEST = 23  # sphere.rs:26-31
FLOP_PER_BOX_TEST = 12  # aabb.rs:56-82 with hoisted reciprocal
BYTES_PER_SPHERE_TEST = 16
BYTES_PER_NODE_VISIT = 56  # per BVH2 node visit: two child boxes (2 x 24 B) + two links (2 x 4 B)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C2", help="workload (BASELINE config name); C2 is the metric's config")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-breakdown", action="store_true", help="skip the wall-clock split (one extra frame)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_C2.json"),
                    help="per-launch HBM bytes from rocprofv3 PMC passes (written by tools/pmc_traffic.py)")
    return ap.parse_args()


def cpu_baseline(scene, budget_s):
    """Oracle BOOKS mode (f64, recursive, the reference's CPU semantics) on this host's cores,
    over a bounded sample of the same frame: every pixel of C2 at S spp, S sized to ~budget_s."""
    from oracle import oracle

    threads = min(16, os.cpu_count() or 1)
    t = time.perf_counter()
    _, rays1, _ = oracle.render(scene, oracle.BOOKS, samples=(0, 1), threads=threads)
    t1 = time.perf_counter() - t
    extra = int(max(0, min(scene.spp - 1, budget_s / max(t1, 1e-3) - 1)))
    rays, secs = rays1, t1
    if extra:
        t = time.perf_counter()
        _, r2, _ = oracle.render(scene, oracle.BOOKS, samples=(1, 1 + extra), threads=threads)
        secs += time.perf_counter() - t
        rays += r2
    spp_done = 1 + extra
    return {
        "value": round(rays / secs / 1e6, 3),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{scene.width}x{scene.height} C2 frame at {spp_done} of {scene.spp} spp "
                  f"(f64 books restatement, {threads} threads, {rays} rays in {secs:.2f} s; "
                  f"extrapolated full-frame wall-clock {secs * scene.spp / spp_done:.1f} s)",
    }


def wall_clock_breakdown(scene, accum, kernel_ms):
    """SURVEY 8(d) split of one C2 frame through the library, measured outside the timed
    region on rank 0: host BVH build, scene creation (BVH build + H2D upload), kernel (the
    timed loop's average), D2H of the float accum, P3 formatting (render_io.rs), and the
    end-to-end drop-in call rrt_hip_render (scene + kernel + D2H) plus the P3 write
    (render_io::write_ppm_from_accum to /dev/null)."""
    import torch

    import rustraytrace_amd as rrt

    def timed(fn):
        t = time.perf_counter()
        out = fn()
        return out, (time.perf_counter() - t) * 1e3

    from rustraytrace_amd.render import build_bvh

    _, bvh_ms = timed(lambda: build_bvh(scene))
    ds, create_ms = timed(lambda: rrt.DeviceScene(scene))
    ds.close()
    torch.cuda.synchronize()
    host, d2h_ms = timed(lambda: accum.cpu())
    _, fmt_ms = timed(lambda: rrt.write_ppm_from_accum(scene.width, scene.height, host.numpy(), scene.spp, os.devnull))
    e2e_accum, render_ms = timed(lambda: rrt.render(scene, n_gpus=1))
    _, fmt2_ms = timed(lambda: rrt.write_ppm_from_accum(scene.width, scene.height, e2e_accum, scene.spp, os.devnull))
    # output step on the device: render + device quantiser, 3 B/pixel D2H
    rgb8, rgb8_ms = timed(lambda: rrt.render_rgb8(scene, n_gpus=1))
    _, p3_ms = timed(lambda: rrt.write_pnm_from_rgb8(scene.width, scene.height, rgb8, False, os.devnull))
    _, p6_ms = timed(lambda: rrt.write_pnm_from_rgb8(scene.width, scene.height, rgb8, True, os.devnull))
    return {
        "bvh_build_ms": round(bvh_ms, 3),
        "scene_create_ms": round(create_ms, 3),
        "kernel_ms": round(kernel_ms, 3),
        "d2h_ms": round(d2h_ms, 3),
        "ppm_write_ms": round(fmt_ms, 3),
        "end_to_end_ms": round(render_ms + fmt2_ms, 3),
        "end_to_end_note": "rrt_hip_render (BVH build, H2D, kernel, D2H, 1 GPU) + P3 write of the frame",
        "end_to_end_rgb8_p3_ms": round(rgb8_ms + p3_ms, 3),
        "end_to_end_rgb8_p6_ms": round(rgb8_ms + p6_ms, 3),
        "rgb8_note": "rrt_hip_render_rgb8 (device quantiser, same bytes) + P3 / binary P6 write",
    }


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    import rustraytrace_amd as rrt
    from rustraytrace_amd.distributed import gather_sample_ranges

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RCCL ("nccl") between one process per GPU. RRT_BENCH_BACKEND=gloo is a rehearsal mode for
    # ranks sharing a GPU (device = local rank mod device count; host copies for the gather).
    backend = os.environ.get("RRT_BENCH_BACKEND", "nccl")
    device = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(device)
        kw = {"device_id": torch.device(f"cuda:{device}")} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    torch.cuda.set_device(device)

    kw = {}
    if args.width:
        kw["image_width"] = args.width
    if args.spp:
        kw["samples_per_pixel"] = args.spp
    scene = rrt.config_scene(args.config, **kw)
    W, H, S = scene.width, scene.height, scene.spp
    ds = rrt.DeviceScene(scene, device=device)
    tile = ds.tile(band_rows=16, rank=0, n_ranks=1, sample_begin=rank * S, sample_end=(rank + 1) * S)
    accum = torch.empty((H, W, 4), dtype=torch.float32, device=f"cuda:{device}")
    stream = torch.cuda.current_stream()

    total = torch.empty_like(accum) if rank == 0 else None

    def gather():  # the one exchange: partial accums -> rank 0, summed in rank order
        if backend == "gloo":
            res = gather_sample_ranges(accum.cpu(), dist)
            if res is not None:
                total.copy_(res)
        else:
            gather_sample_ranges(accum, dist, out=total)

    def step(i=None):
        if i is not None:
            k_start[i].record(stream)
        ds.render_tile_async(tile, accum.data_ptr(), stream.cuda_stream)
        if i is not None:
            k_end[i].record(stream)
        if world > 1:
            gather()

    k_start = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    k_end = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ds.reset_counters()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = [a.elapsed_time(b) for a, b in zip(k_start, k_end)]
    gather_ms = None
    if world > 1:  # the exchange step alone, untimed loop: partial accums -> rank 0
        dist.barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        gather()
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - t) * 1e3
    ctr = ds.counters()
    rays = ctr["rays"]
    if world > 1:
        red_dev = f"cuda:{device}" if backend == "nccl" else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        r = torch.tensor([rays], dtype=torch.int64, device=red_dev)
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
        rays = int(r.item())

    if rank == 0:
        work = ds.count_work(tile)  # instrumented twin kernel: same paths, per-frame work counts
        avg_kernel_s = float(np.mean(kernel_ms)) / 1e3
        flops = FLOP_PER_SPHERE_TEST * work["sphere_tests"] + FLOP_PER_BOX_TEST * work["box_tests"]
        achieved = flops / avg_kernel_s / 1e12
        alg_bytes = BYTES_PER_SPHERE_TEST * work["sphere_tests"] + BYTES_PER_NODE_VISIT * work["node_visits"]
        traffic, traffic_src = None, None
        if os.path.exists(args.traffic_json):
            try:
                with open(args.traffic_json) as f:
                    tj = json.load(f)
                if tj.get("config") == args.config and tj.get("width") == W and tj.get("spp") == S:
                    traffic = tj.get("hbm_bytes_per_launch")
                    import hashlib

                    with open(rrt._lib.LIB_PATH, "rb") as f:
                        cur = hashlib.sha256(f.read()).hexdigest()
                    same = cur == tj.get("lib_sha256")
                    traffic_src = (f"{os.path.relpath(args.traffic_json, ROOT)}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                                   f"passes, {'this' if same else 'an earlier'} librrt_hip.so build "
                                   f"({tj.get('lib_sha256', '')[:12]})")
            except (OSError, ValueError):
                traffic = None
        rays_per_frame = work["rays"]
        out = {
            "metric": METRIC,
            "value": round(rays / elapsed / 1e6, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {
                "workload": f"{args.config} RTOW final scene (gpu/mod.rs generator, seed 0x5EED1234), "
                            f"{W}x{H}x{S}spp, max_depth {scene.max_depth}, {len(scene.spheres)} spheres",
                "image": [W, H],
                "spp_per_rank": S,
                "max_depth": scene.max_depth,
                "parallelism": f"frame x sample-range per rank, {world} rank(s), RCCL gather of float accums",
            },
            "wall_clock_s_per_frame": round(elapsed / args.steps, 4),
            "rays_per_frame": rays_per_frame,
            "paths_per_frame": work["paths"],
            "gpaths_per_s": round(work["paths"] * args.steps * world / elapsed / 1e9, 3),
            "sphere_tests_per_s": round(work["sphere_tests"] / avg_kernel_s, 1),
            "kernel_ms_avg": round(avg_kernel_s * 1e3, 3),
            "bvh": ds.bvh_info(),
            "roofline": {
                "bound": "valu",
                "achieved": round(achieved, 3),
                "peak": PEAK_F32_VALU_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_F32_VALU_TFLOPS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_flop_per_launch": flops,
                "algorithmic_bytes_per_launch": alg_bytes,
                "effective_fetch_GBps": round(alg_bytes / avg_kernel_s / 1e9, 1),
                "note": "f32 VALU issue bound (SURVEY 8d): 23 FLOP/sphere test + 12 FLOP/box test over the "
                        "average HIP-event kernel time; peak = wave64 v_fma_f32 at 2 cycles on SIMD-32 "
                        "(SURVEY 8d's 78.6 assumed 16-lane SIMDs)",
            },
        }
        if world == 1 and not args.no_breakdown:
            out["wall_clock_breakdown"] = wall_clock_breakdown(scene, accum, avg_kernel_s * 1e3)
        if gather_ms is not None:
            out["gather_ms"] = round(gather_ms, 3)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(scene, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    ds.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
