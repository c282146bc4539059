"""Benchmark: Mrays/s and wall-clock for the RTOW final scene (BASELINE.json metric) on MI355X
through librrt_hip.so's device-resident C-ABI.

A step = one full frame of the configured workload rendered from scene data already resident in
HBM (BVH built and uploaded before timing). Ray = one closest-hit query (camera.rs:187), counted
on the device by the kernel itself.

* N = 1 (default): config C2, 1920x1080x512 spp (BASELINE.json configs[1], the metric's config),
  the whole frame on one GPU, no gather. The line also carries a 1-GPU C3 frame (`c3_one_gpu`,
  the strong-scaling base of the N > 1 runs), the C1 CPU-path config timed on the CPU and the
  GPU (`c1`), the wall-clock split, the CPU baseline, and (opt-in, `--ref-slot`) the reference's
  own GPU kernel (its CUDA_SOURCE built for gfx950, oracle/_ref) timed beside this backend on a
  bounded sample of the same workload (`reference_gpu_slot`).
* N > 1 (`python bench.py --gpus N` starts `python -m torch.distributed.run --nproc-per-node N
  bench.py --gpus N` as a child process before touching any device and forwards rank 0's line;
  under an external launcher WORLD_SIZE must equal N): config C3,
  3840x2160x2048 spp, tile-split the north star's way: row bands (10 rows at
  2/4/8 ranks, so every rank owns 2160/N rows; `distributed.balanced_band`) dealt in serpentine order (period p of
  N bands: ranks 0..N-1 for even p, N-1..0 for odd p; `distributed.band_owner`), every rank renders its bands over
  all samples, and the
  float tiles are gathered to rank 0 over RCCL inside the timed step (`distributed.gather_rows`).
  Strong scaling: the frame is fixed, value = all ranks' rays / the max over ranks of the timed
  wall-clock. The line carries each rank's kernel time, the gather time and the same frame on
  rank 0's GPU alone (`c3_one_gpu`), so `scaling_efficiency` is in the line. `--split samples` is the opt-in weak-scaling mode (every rank renders the whole
  frame over its own sample range; partial accums summed on rank 0 in rank order).
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
# f64 VALU peak: AMD's MI355X spec sheet, 78.6 TFLOP/s vector FP64 — half the FP32 rate (a wave64
# v_fma_f64 issues in 4 cycles on SIMD-32); MI355X_MICROARCH.md lists FP32 only
PEAK_F64_VALU_TFLOPS = 78.6
PEAK_HBM_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E ~8 TB/s
FLOP_PER_SPHERE_TEST = 23  # sphere.rs:26-31
FLOP_PER_BOX_TEST = 12  # aabb.rs:56-82 with hoisted reciprocal
BYTES_PER_SPHERE_TEST = 16
BYTES_PER_NODE_VISIT = 56  # per BVH2 node visit: two child boxes (2 x 24 B) + two links (2 x 4 B)
BAND_ROWS = 16
SCENES = {
    "C1": "three-sphere Lambertian scene (books CPU path)",
    "C2": "RTOW final scene (gpu/mod.rs generator, seed 0x5EED1234)",
    "C3": "RTOW final scene (gpu/mod.rs generator, seed 0x5EED1234)",
    "C4": "textured earth sphere (earthmap.jpg) + emissive light",
    "C5": "10k-sphere stress scene (RTOW generator, grid_half 50)",
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default=None,
                    help="workload (BASELINE config C1-C5, or a scene-table name NW1-NW10 / B3); default C2 (the metric's config) on 1 rank, C3 on N > 1")
    ap.add_argument("--split", choices=["bands", "samples"], default="bands",
                    help="bands: C3's row-band tiles, strong scaling (default); samples: whole frame per rank, "
                         "weak scaling")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-breakdown", action="store_true", help="skip the wall-clock split (one extra frame)")
    ap.add_argument("--no-extra", action="store_true", help="skip the 1-GPU C3 frame and the C1 timings")
    ap.add_argument("--no-f64", action="store_true", help="skip the f64 books-arithmetic leg (f64_books)")
    ap.add_argument("--f64", action="store_true",
                    help="time the f64 books kernel (RRT_FLAG_F64, bit-identical to the books path) as the headline "
                         "leg instead of the f32 kernel: value, dtype f64, the same band split and gather")
    ap.add_argument("--ref-slot", action="store_true",
                    help="also time the reference's own GPU kernel on a bounded sample (reference_gpu_slot; opt-in: "
                         "a third-party kernel, kept out of the default run)")
    ap.add_argument("--issue-json", default=None,
                    help="issue-side PMC record (tools/pmc_issue.py); default profiles/issue_<config>.json")
    ap.add_argument("--traffic-json", default=None,
                    help="per-launch HBM bytes from rocprofv3 PMC passes (tools/pmc_traffic.py); "
                         "default profiles/traffic_<config>.json")
    return ap.parse_args(argv)


def launcher_command(args, argv, env):
    """The child launch `python bench.py --gpus N` (N > 1) needs when no launcher started it, or
    None: one process per GPU, torch.distributed.run over 127.0.0.1 with this same argument list.
    Decided from the arguments and the environment alone — the parent never imports torch or
    touches a device, so it never holds a GPU context that a child (or an exec) could collide
    with."""
    if args.gpus <= 1 or "WORLD_SIZE" in env:
        return None
    port = env.get("MASTER_PORT")
    if not port:
        import socket

        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = str(s.getsockname()[1])
        s.close()
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def run_launcher(cmd):
    """Run the N-rank child and forward rank 0's JSON line to stdout (everything else the ranks
    print goes to stderr, so stdout carries exactly the one line); the child's exit status is
    returned, non-zero when any rank failed."""
    import subprocess

    print(f"bench.py: launching {' '.join(cmd[2:5])} (one process per GPU)", file=sys.stderr, flush=True)
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1)
    forwarded = False
    for line in proc.stdout:
        if not forwarded and line.startswith("{") and '"metric"' in line:
            sys.stdout.write(line)
            sys.stdout.flush()
            forwarded = True
        else:
            sys.stderr.write(line)
    rc = proc.wait()
    if rc == 0 and not forwarded:
        print("bench.py: the ranks exited without a result line", file=sys.stderr)
        return 1
    return rc


def host_cpus():
    """The cores this process may run on: its affinity set, capped by a cgroup CPU quota when one
    is set (a container's share of a large host), plus the machine's count and CPU model."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    usable = min(affinity, quota) if quota else affinity
    return {"threads": usable, "affinity_cpus": affinity, "cgroup_quota_cpus": quota,
            "machine_cpus": os.cpu_count(), "cpu_model": model}


def cpu_baseline(scene, budget_s, cpus):
    """Oracle BOOKS mode (f64, recursive, the reference's CPU semantics; rayon over rows in the
    reference, camera.rs:66-67) on every core this process is given, over a bounded sample of the
    same frame: every pixel of C2 at S spp, S sized to ~budget_s."""
    from oracle import oracle

    threads = cpus["threads"]
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
        "host": cpus,
        "sample": f"{scene.width}x{scene.height} {scene.name} frame at {spp_done} of {scene.spp} spp "
                  f"(f64 books restatement, {threads} threads = every core this process is given, {rays} rays "
                  f"in {secs:.2f} s; extrapolated full-frame wall-clock {secs * scene.spp / spp_done:.1f} s)",
    }


def c1_timings(cpus):
    """C1, the reference's CPU books path (configs[0]: 3-sphere Lambertian scene, 400x225, 64 spp,
    depth 8; camera.rs:59-100): the whole frame on the CPU (f64 books restatement, all cores) and
    on the GPU (HIP-event kernel time, scene resident)."""
    import numpy as np
    import torch

    import rustraytrace_amd as rrt
    from oracle import oracle

    scene = rrt.config_scene("C1")
    t = time.perf_counter()
    _, cpu_rays, _ = oracle.render(scene, oracle.BOOKS, threads=cpus["threads"])
    cpu_s = time.perf_counter() - t
    ds = rrt.DeviceScene(scene)
    tile = ds.tile(BAND_ROWS, 0, 1, 0, scene.spp)
    buf = torch.empty((scene.height, scene.width, 4), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream()
    ds.render_tile_async(tile, buf.data_ptr(), stream.cuda_stream)  # warm
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
    ds.reset_counters()
    for i in range(5):
        ev[i].record(stream)
        ds.render_tile_async(tile, buf.data_ptr(), stream.cuda_stream)
    ev[5].record(stream)
    torch.cuda.synchronize()
    gpu_ms = float(np.mean([ev[i].elapsed_time(ev[i + 1]) for i in range(5)]))
    gpu_rays = ds.counters()["rays"] // 5
    ds.close()
    return {
        "workload": f"C1 three-sphere Lambertian scene {scene.width}x{scene.height}x{scene.spp}spp depth {scene.max_depth}",
        "cpu_frame_s": round(cpu_s, 4), "cpu_threads": cpus["threads"], "cpu_rays": cpu_rays,
        "cpu_mrays_s": round(cpu_rays / cpu_s / 1e6, 2),
        "gpu_frame_ms": round(gpu_ms, 4), "gpu_rays": gpu_rays, "gpu_mrays_s": round(gpu_rays / gpu_ms / 1e3, 1),
    }


def one_gpu_frame(config="C3", kw=None, device=0):
    """One whole frame of `config` (default C3, 3840x2160x2048 spp) on one GPU: the 1-GPU base of
    the N > 1 strong-scaling runs (same workload, the band split with one rank, no gather)."""
    import torch

    import rustraytrace_amd as rrt

    scene = rrt.named_scene(config, **(kw or {}))
    ds = rrt.DeviceScene(scene, device=device)
    tile = ds.tile(BAND_ROWS, 0, 1, 0, scene.spp)
    buf = torch.empty((scene.height, scene.width, 4), dtype=torch.float32, device=f"cuda:{device}")
    stream = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    a.record(stream)
    ds.render_tile_async(tile, buf.data_ptr(), stream.cuda_stream)
    b.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t
    rays = ds.counters()["rays"]
    ds.close()
    del buf
    return {"workload": f"{config} {scene.width}x{scene.height}x{scene.spp}spp, 1 GPU, one frame (no warmup frame)",
            "frame_s": round(wall, 4), "kernel_ms": round(a.elapsed_time(b), 2), "rays": rays,
            "mrays_s": round(rays / wall / 1e6, 2)}


def f64_books_frame(config, frames=2, issue_json=None):
    """The same workload through the f64 books-arithmetic kernel (RRT_FLAG_F64, rrt_books64.hip):
    the reference CPU path's own arithmetic on the GPU, which tests/test_gpu_books64.py checks
    against the f64 books restatement (every channel within 1e-4, identical PPM bytes). One warmup
    frame, then `frames` frames timed with HIP events on the render stream; rays counted on the
    device. Not the headline (the headline is the f32 kernel, the reference GPU slot's precision)."""
    import numpy as np
    import torch

    import rustraytrace_amd as rrt

    scene = rrt.config_scene(config)
    ds = rrt.DeviceScene(scene, f64=True)
    tile = ds.tile(BAND_ROWS, 0, 1, 0, scene.spp)
    buf = torch.empty((scene.height, scene.width, 4), dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream()
    ds.render_tile_f64_async(tile, buf.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    ds.reset_counters()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(frames + 1)]
    t = time.perf_counter()
    for i in range(frames):
        ev[i].record(stream)
        ds.render_tile_f64_async(tile, buf.data_ptr(), stream.cuda_stream)
    ev[frames].record(stream)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) / frames
    ms = float(np.mean([ev[i].elapsed_time(ev[i + 1]) for i in range(frames)]))
    rays = ds.counters()["rays"] // frames
    work = ds.count_work(tile)  # the instrumented twin: the books path's sphere and box tests per frame
    ds.close()
    flops = FLOP_PER_SPHERE_TEST * work["sphere_tests"] + FLOP_PER_BOX_TEST * work["box_tests"]
    achieved = flops / (ms / 1e3) / 1e12
    roofline = {
        "bound": "valu",
        "achieved": round(achieved, 3),
        "peak": PEAK_F64_VALU_TFLOPS,
        "unit": "TFLOP/s",
        "frac": round(achieved / PEAK_F64_VALU_TFLOPS, 4),
        "traffic": None,
        "algorithmic_flop_per_launch": flops,
        "sphere_tests_per_launch": work["sphere_tests"],
        "box_tests_per_launch": work["box_tests"],
        "note": "f64 VALU issue bound: the books path's 23 FLOP per sphere test + 12 FLOP per box test (SURVEY 8d), "
                "all f64 in the reference, over the HIP-event time of the frame (render passes + in-order folds); "
                "peak = MI355X FP64 vector 78.6 TFLOP/s (AMD spec: half the FP32 rate). The kernel runs the box test "
                "in f32 with a proven bound (rrt_box32.h), so part of the work priced here at f64 issues at the f32 "
                "rate (the f32 sphere pre-test of rrt_sphere32.h is built but off: RRT_F64_SPHERE32=0)",
    }
    traffic, traffic_src = load_traffic(os.path.join(ROOT, "profiles", f"traffic_{config}_f64.json"), config,
                                        scene.width, scene.spp, rrt._lib.LIB_PATH)
    if traffic:  # HBM bytes of the render launch (PMC): the attenuation history and the tail radiances
        roofline.update({"traffic": traffic, "traffic_source": traffic_src,
                         "hbm_GBps": round(traffic / (ms / 1e3) / 1e9, 2),
                         "hbm_frac": round(traffic / (ms / 1e3) / 1e9 / PEAK_HBM_GBPS, 5)})
    rec = None
    path = issue_json or os.path.join(ROOT, "profiles", f"issue_{config}_f64.json")
    if os.path.exists(path):
        try:
            with open(path) as f:
                rec = json.load(f)
        except (OSError, ValueError):
            rec = None
    if rec and rec.get("f64") and rec.get("config") == config and rec.get("width") == scene.width \
            and rec.get("spp") == scene.spp:
        import hashlib

        with open(rrt._lib.LIB_PATH, "rb") as f:
            same = hashlib.sha256(f.read()).hexdigest() == rec.get("lib_sha256")
        roofline.update({k: rec[k] for k in ("valu_busy", "lanes_per_valu", "valu_insts_per_ray", "f64_share_of_valu")
                         if rec.get(k) is not None})
        weighted = rec.get("f64_share_of_valu") is not None
        roofline["issue_source"] = (f"{os.path.relpath(path, ROOT)}: rocprofv3 --pmc over one f64 {config} launch, "
                                    f"{'this' if same else 'an earlier'} librrt_hip.so build "
                                    f"({rec.get('lib_sha256', '')[:12]}); valu_busy = issue cycles / SIMD cycles, "
                                    + ("an f64 VALU instruction weighted 4 cycles and any other 2 (typed counters "
                                       "from a second pass)" if weighted else
                                       "2 cycles per VALU wave-instruction (an f64 one takes 4: an underestimate)"))
    return {"workload": f"{config} {scene.width}x{scene.height}x{scene.spp}spp, f64 books arithmetic (RRT_FLAG_F64)",
            "dtype": "f64", "value": round(rays / wall / 1e6, 2), "unit": "Mrays/s", "ms_per_frame": round(wall * 1e3, 3),
            "kernel_ms": round(ms, 3), "rays_per_frame": rays, "frames": frames,
            "parity": "tests/test_gpu_books64.py: every f64 pixel sum bit-identical to the books restatement "
                      "(closest hits, back-to-front throughput and camera.rs:72-76's sequential sums), so every "
                      "channel within 1e-4 and every PPM byte equal",
            "roofline": roofline}


def f64_band_leg(scene, config, band, rank, world, device, backend, dist, steps, warmup, base=True):
    """N > 1: the f64 books kernel (RRT_FLAG_F64, bit-identical to the books path: the north star's
    correctness bar) over the same row-band split as the f32 leg, timed the same way: `warmup` frames,
    then a barrier + synchronize, `steps` frames each followed by the RCCL gather of the f64 tiles to
    rank 0, synchronize + barrier, the max over ranks of the wall-clock. Every pixel is keyed by its
    global index and summed in sample order inside its rank, so the gathered f64 frame equals the
    1-GPU f64 frame bit for bit (tests/test_gpu_multirank.py). Rank 0 also renders the same frame
    alone after the timed steps (the f64 curve's 1-GPU base) unless `base` is False. Returns the
    record on rank 0, None elsewhere."""
    import numpy as np
    import torch

    import rustraytrace_amd as rrt
    from rustraytrace_amd.distributed import band_rows, gather_rows

    W, H, S = scene.width, scene.height, scene.spp
    ds = rrt.DeviceScene(scene, device=device, f64=True)
    tile = ds.tile(band_rows=band, rank=rank, n_ranks=world, sample_begin=0, sample_end=S)
    rows = ds.tile_rows(tile)
    accum = torch.empty((max(rows, 1), W, 4), dtype=torch.float64, device=f"cuda:{device}")
    stream = torch.cuda.current_stream()
    k0 = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
    k1 = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
    g1 = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]

    def step(i=None):
        if i is not None:
            k0[i].record(stream)
        if rows:
            ds.render_tile_f64_async(tile, accum.data_ptr(), stream.cuda_stream)
        if i is not None:
            k1[i].record(stream)
        src = accum[:rows] if backend == "nccl" else accum[:rows].cpu()
        gather_rows(src, H, band, dist)
        if i is not None:
            g1[i].record(stream)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    ds.reset_counters()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    kms = float(np.mean([a.elapsed_time(b) for a, b in zip(k0, k1)]))
    gms = float(np.mean([a.elapsed_time(b) for a, b in zip(k1, g1)]))
    rays = ds.counters()["rays"]
    ds.close()
    del accum
    red_dev = f"cuda:{device}" if backend == "nccl" else "cpu"
    every = [torch.zeros(3, dtype=torch.float64, device=red_dev) for _ in range(world)]
    dist.all_gather(every, torch.tensor([elapsed, kms, rays], dtype=torch.float64, device=red_dev))
    every = torch.stack(every).cpu().numpy()
    elapsed, rays = float(every[:, 0].max()), int(every[:, 2].sum())
    per_rank = [round(float(v), 3) for v in every[:, 1]]
    one = None
    if rank == 0 and base:
        one = one_gpu_frame_f64(scene, device)
    dist.barrier()
    if rank != 0:
        return None
    value = round(rays / elapsed / 1e6, 2)
    rec = {"workload": f"{config} {W}x{H}x{S}spp, f64 books arithmetic (RRT_FLAG_F64), {band}-row bands dealt in "
                       f"serpentine order over {world} ranks, RCCL gather of the f64 tiles to rank 0 inside the "
                       "timed step" + (" (gloo rehearsal: ranks share a GPU, host copies)" if backend == "gloo" else ""),
           "dtype": "f64", "value": value, "unit": "Mrays/s", "steps": steps, "warmup": warmup,
           "ms_per_step": round(elapsed / steps * 1e3, 3), "rays_per_step": rays // steps,
           "kernel_ms_per_rank": per_rank, "kernel_ms_max_over_ranks": max(per_rank),
           "rank_imbalance": round(max(per_rank) / float(np.mean(per_rank)) - 1.0, 5),
           "gather_ms": round(gms, 3), "rows_per_rank": [len(band_rows(H, band, r, world)) for r in range(world)],
           "parity": "tests/test_gpu_multirank.py: the gathered f64 frame equals the 1-GPU f64 frame bit for bit; "
                     "tests/test_gpu_books64.py: the 1-GPU f64 frame equals the books restatement bit for bit"}
    if one is not None:
        rec["one_gpu_base"] = one
        rec["scaling_efficiency"] = round(value / (world * one["mrays_s"]), 4)
    return rec


def one_gpu_frame_f64(scene, device=0):
    """The f64 band leg's 1-GPU base: the same frame through the f64 kernel on one GPU, one frame
    (no warmup frame), wall-clock around it."""
    import torch

    import rustraytrace_amd as rrt

    ds = rrt.DeviceScene(scene, device=device, f64=True)
    tile = ds.tile(BAND_ROWS, 0, 1, 0, scene.spp)
    buf = torch.empty((scene.height, scene.width, 4), dtype=torch.float64, device=f"cuda:{device}")
    stream = torch.cuda.current_stream()
    torch.cuda.synchronize()
    t = time.perf_counter()
    ds.render_tile_f64_async(tile, buf.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t
    rays = ds.counters()["rays"]
    ds.close()
    del buf
    return {"workload": f"{scene.name} {scene.width}x{scene.height}x{scene.spp}spp f64, 1 GPU, one frame (no warmup "
                        "frame)", "frame_s": round(wall, 4), "rays": rays, "mrays_s": round(rays / wall / 1e6, 2)}


def reference_gpu_slot(config, budget_s=1.5):
    """The reference's own GPU kernel on this GPU (oracle/_ref/ref_slot.hsaco: CUDA_SOURCE of
    src/cuda/mod.rs:15-335 compiled unmodified for gfx950, launched as imp::render launches it;
    oracle/ref_slot.cpp) against this backend on the identical bounded sample: the workload's
    image at the spp that fits ~budget_s of the reference kernel. The unit is paths/s (W*H*spp
    over HIP-event kernel time): the reference kernel counts no rays and its Russian roulette and
    f32 re-hits trace a slightly different number of them (tests/test_gpu_ref_slot.py)."""
    import numpy as np
    import torch

    import rustraytrace_amd as rrt
    from oracle import ref_slot

    if not ref_slot.available():
        return {"skipped": "oracle/_ref/ref_slot.hsaco not built (needs /root/reference at build time)"}
    probe = rrt.config_scene(config, samples_per_pixel=1)
    ref_slot.render(probe)  # module load + first launch
    _, ms1 = ref_slot.render(probe, return_ms=True)
    full = rrt.config_scene(config)
    spp = int(max(1, min(full.spp, 256, budget_s * 1e3 / max(ms1, 1e-3))))
    scene = rrt.config_scene(config, samples_per_pixel=spp)
    _, ref_ms = ref_slot.render(scene, return_ms=True)
    ds = rrt.DeviceScene(scene)
    tile = ds.tile(BAND_ROWS, 0, 1, 0, spp)
    buf = torch.empty((scene.height, scene.width, 4), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream()
    ds.render_tile_async(tile, buf.data_ptr(), stream.cuda_stream)  # warm
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    for i in range(3):
        ev[i].record(stream)
        ds.render_tile_async(tile, buf.data_ptr(), stream.cuda_stream)
    ev[3].record(stream)
    torch.cuda.synchronize()
    ours_ms = float(np.mean([ev[i].elapsed_time(ev[i + 1]) for i in range(3)]))
    ds.close()
    paths = scene.width * scene.height * spp
    return {
        "sample": f"{config} {scene.width}x{scene.height} at {spp} spp (max_depth {scene.max_depth}), both kernels on "
                  "this GPU, HIP-event kernel time",
        "kernel": "reference CUDA_SOURCE (src/cuda/mod.rs:15-335) built unmodified by hipcc for gfx950; brute-force "
                  "closest hit over every sphere, one thread per pixel, passes of <= 256 spp",
        "ref_ms": round(ref_ms, 3), "ref_mpaths_s": round(paths / ref_ms / 1e3, 2),
        "ours_ms": round(ours_ms, 3), "ours_mpaths_s": round(paths / ours_ms / 1e3, 2),
        "speedup": round(ref_ms / ours_ms, 2),
    }


def wall_clock_breakdown(scene, accum, kernel_ms):
    """SURVEY 8(d) split of one frame through the library, measured outside the timed region on
    rank 0: host BVH build, scene creation (BVH build + H2D upload), kernel (the timed loop's
    average), D2H of the float accum, P3 formatting (render_io.rs), and the end-to-end drop-in
    call rrt_hip_render (scene + kernel + D2H) plus the P3 write (render_io::write_ppm_from_accum
    to /dev/null)."""
    import numpy as np
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
    # the drop-in call three times: the first in the process pays the one-shot call's device
    # allocations and the first touch of the caller's fresh 33-MB host array; the line reports it
    # and the median of the two that follow
    e2e_accum, render_first_ms = timed(lambda: rrt.render(scene, n_gpus=1))
    render_ms = float(np.median([timed(lambda: rrt.render(scene, n_gpus=1))[1] for _ in range(2)]))
    # the same call as the Rust shim and the CLI make it (flags 0: progress lines on stderr, the
    # work-queue heads read every 100 ms, the end noticed within ~1 ms)
    _, progress_ms = timed(lambda: rrt.render(scene, n_gpus=1, quiet=False))
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
        "end_to_end_first_call_ms": round(render_first_ms + fmt2_ms, 3),
        "end_to_end_note": "rrt_hip_render (BVH build, H2D, kernel, D2H, 1 GPU) + P3 write of the frame; "
                           "end_to_end_ms: median of the 2nd and 3rd calls in the process, first_call: the 1st",
        "render_with_progress_ms": round(progress_ms, 3),
        "progress_note": "rrt_hip_render without RRT_FLAG_QUIET (as the Rust shim and the CLI call it), no P3 write",
        "end_to_end_rgb8_p3_ms": round(rgb8_ms + p3_ms, 3),
        "end_to_end_rgb8_p6_ms": round(rgb8_ms + p6_ms, 3),
        "rgb8_note": "rrt_hip_render_rgb8 (device quantiser, same bytes) + P3 / binary P6 write",
    }


def load_traffic(path, config, W, S, lib_path):
    """HBM bytes per launch of this config from a tools/pmc_traffic.py record, or (None, None)."""
    if not os.path.exists(path):
        return None, None
    try:
        with open(path) as f:
            tj = json.load(f)
    except (OSError, ValueError):
        return None, None
    if not (tj.get("config") == config and tj.get("width") == W and tj.get("spp") == S):
        return None, None
    import hashlib

    with open(lib_path, "rb") as f:
        same = hashlib.sha256(f.read()).hexdigest() == tj.get("lib_sha256")
    src = (f"{os.path.relpath(path, ROOT)}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes, "
           f"FETCH_SIZE x2 (gfx950 correction, MI355X_MICROARCH.md HBM section) + WRITE_SIZE, "
           f"{'this' if same else 'an earlier'} librrt_hip.so build ({tj.get('lib_sha256', '')[:12]})")
    return tj.get("hbm_bytes_per_launch_fetch_corrected", tj.get("hbm_bytes_per_launch")), src


def load_issue(path, config, W, S, lib_path):
    """valu_busy / lanes_per_valu / valu_insts_per_ray of this config from a tools/pmc_issue.py
    record (one PMC pass over a full-size launch), or None."""
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None
    if not (rec.get("config") == config and rec.get("width") == W and rec.get("spp") == S and not rec.get("f64")):
        return None
    import hashlib

    with open(lib_path, "rb") as f:
        same = hashlib.sha256(f.read()).hexdigest() == rec.get("lib_sha256")
    return {k: rec[k] for k in ("valu_busy", "lanes_per_valu", "valu_insts_per_ray")} | {
        "issue_source": f"{os.path.relpath(path, ROOT)}: rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU "
                        f"GRBM_GUI_ACTIVE ... over one {config} launch, {'this' if same else 'an earlier'} "
                        f"librrt_hip.so build ({rec.get('lib_sha256', '')[:12]}); valu_busy = 2 cycles x "
                        f"VALU wave-instructions / (1024 SIMDs x cycles)"}


def device_shortfall(backend: str, local_rank: int, n_devices: int):
    """Under RCCL each rank owns GPU `local_rank`: a box with fewer devices cannot run the job, so
    the rank stops with this message before init_process_group (where it would wait in the
    rendezvous for ranks that never come) and the launcher returns non-zero. None = runnable."""
    if backend == "nccl" and local_rank >= n_devices:
        return (f"bench.py: rank with LOCAL_RANK={local_rank} needs GPU {local_rank} but {n_devices} HIP "
                f"device(s) are visible (RCCL runs one process per GPU)")
    return None


def main():
    args = parse()
    cmd = launcher_command(args, sys.argv[1:], os.environ)
    if cmd is not None:  # --gpus N without a launcher: start the N ranks as a child, never exec
        sys.exit(run_launcher(cmd))
    import numpy as np
    import torch
    import torch.distributed as dist

    import rustraytrace_amd as rrt
    from rustraytrace_amd.distributed import balanced_band, band_rows, gather_rows, gather_sample_ranges

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if "WORLD_SIZE" in os.environ and world != args.gpus:
        sys.exit(f"bench.py: launched with WORLD_SIZE={world} but --gpus {args.gpus}")
    # RCCL ("nccl") between one process per GPU. RRT_BENCH_BACKEND=gloo is a rehearsal mode for
    # ranks sharing a GPU (device = local rank mod device count; host copies for the gather).
    backend = os.environ.get("RRT_BENCH_BACKEND", "nccl")
    short = device_shortfall(backend, local, torch.cuda.device_count())  # counts without a GPU context
    if short:
        print(short, file=sys.stderr, flush=True)
        sys.exit(2)
    device = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(device)
        kw = {"device_id": torch.device(f"cuda:{device}")} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    torch.cuda.set_device(device)

    config = args.config or ("C2" if world == 1 else "C3")
    bands = args.split == "bands"
    kw = {}
    if args.width:
        kw["image_width"] = args.width
    if args.spp:
        kw["samples_per_pixel"] = args.spp
    scene = rrt.named_scene(config, **kw)
    W, H, S = scene.width, scene.height, scene.spp
    f64 = args.f64
    ds = rrt.DeviceScene(scene, device=device, f64=f64)
    # bands of equal count per rank when the height allows it (C3: 10 rows at 2/4/8 ranks)
    band = balanced_band(H, world) if (bands and world > 1) else BAND_ROWS
    if bands:
        tile = ds.tile(band_rows=band, rank=rank, n_ranks=world, sample_begin=0, sample_end=S)
        rows = ds.tile_rows(tile)
    else:
        tile = ds.tile(band_rows=BAND_ROWS, rank=0, n_ranks=1, sample_begin=rank * S, sample_end=(rank + 1) * S)
        rows = H
    accum = torch.empty((max(rows, 1), W, 4), dtype=torch.float64 if f64 else torch.float32, device=f"cuda:{device}")
    render = ds.render_tile_f64_async if f64 else ds.render_tile_async
    stream = torch.cuda.current_stream()
    image = [None]  # rank 0: the gathered frame of the last step

    def gather():  # the one exchange: tiles (bands) or partial accums (samples) -> rank 0
        src = accum[:rows] if backend == "nccl" else accum[:rows].cpu()
        if bands:
            image[0] = gather_rows(src, H, band, dist)
        else:
            image[0] = gather_sample_ranges(src, dist)

    def step(i=None):
        if i is not None:
            k_start[i].record(stream)
        if rows:
            render(tile, accum.data_ptr(), stream.cuda_stream)
        if i is not None:
            k_end[i].record(stream)
        if world > 1:
            gather()
            if i is not None:
                g_end[i].record(stream)

    k_start = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    k_end = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    g_end = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
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
    gather_ms = [a.elapsed_time(b) for a, b in zip(k_end, g_end)] if world > 1 else None
    ctr = ds.counters()
    rays = ctr["rays"]
    kmax = float(np.mean(kernel_ms))
    rank_kernel_ms = [kmax]
    one_gpu = None
    if world > 1:
        red_dev = f"cuda:{device}" if backend == "nccl" else "cpu"
        every = [torch.zeros(3, dtype=torch.float64, device=red_dev) for _ in range(world)]
        dist.all_gather(every, torch.tensor([elapsed, kmax, rays], dtype=torch.float64, device=red_dev))
        every = torch.stack(every).cpu().numpy()
        elapsed, kmax = float(every[:, 0].max()), float(every[:, 1].max())
        rank_kernel_ms = [float(v) for v in every[:, 1]]
        rays = int(every[:, 2].sum())
        if rank == 0 and bands and not args.no_extra:
            # the strong-scaling base on this node: the same frame on rank 0's GPU alone, after the
            # timed region (the other ranks wait at the barrier below)
            one_gpu = one_gpu_frame_f64(scene, device) if f64 else one_gpu_frame(config, kw, device)
        dist.barrier()
    f64_leg = None
    if world > 1 and bands and not f64 and not args.no_f64 and config in ("C1", "C2", "C3", "C4", "C5"):
        # the path that meets the north star's bar, over the same split (after the f32 leg's timed
        # steps; its own barrier-bracketed timing and max over ranks)
        f64_leg = f64_band_leg(scene, config, band, rank, world, device, backend, dist,
                               steps=max(1, min(args.steps, 3)), warmup=1, base=not args.no_extra)

    if rank == 0:
        work = ds.count_work(tile)  # instrumented twin kernel: same paths, per-launch work counts
        avg_kernel_s = float(np.mean(kernel_ms)) / 1e3
        flops = FLOP_PER_SPHERE_TEST * work["sphere_tests"] + FLOP_PER_BOX_TEST * work["box_tests"]
        achieved = flops / avg_kernel_s / 1e12
        alg_bytes = BYTES_PER_SPHERE_TEST * work["sphere_tests"] + BYTES_PER_NODE_VISIT * work["node_visits"]
        traffic_json = args.traffic_json or os.path.join(ROOT, "profiles", f"traffic_{config}.json")
        traffic, traffic_src = (None, None)
        issue = None
        if rows == H and not f64:  # the PMC records are of a whole-frame f32 launch
            traffic, traffic_src = load_traffic(traffic_json, config, W, S, rrt._lib.LIB_PATH)
            issue = load_issue(args.issue_json or os.path.join(ROOT, "profiles", f"issue_{config}.json"), config, W, S,
                               rrt._lib.LIB_PATH)
        if bands:
            split = (f"{band}-row bands dealt in serpentine order over {world} rank(s), RCCL gather of the float tiles "
                     f"to rank 0 inside the timed step" if world > 1 else
                     "whole frame on 1 GPU (the band split with one rank), no gather")
        else:
            split = (f"whole frame per rank over its own {S}-sample range, {world} rank(s), RCCL gather + rank-order "
                     f"sum of the partial accums on rank 0" if world > 1 else "whole frame on 1 GPU, no gather")
        if world > 1 and backend == "gloo":
            split += " (gloo rehearsal: ranks share a GPU, host copies)"
        if f64:
            split += "; f64 books kernel (RRT_FLAG_F64), f64 tiles"
        peak = PEAK_F64_VALU_TFLOPS if f64 else PEAK_F32_VALU_TFLOPS
        roofline = {
            "bound": "valu",
            "achieved": round(achieved, 3),
            "peak": peak,
            "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "hbm_GBps": round(traffic / avg_kernel_s / 1e9, 2) if traffic else None,
            "hbm_frac": round(traffic / avg_kernel_s / 1e9 / PEAK_HBM_GBPS, 5) if traffic else None,
            "hbm_note": "measured HBM bytes per launch (PMC) / average kernel time, against 8 TB/s; the scene "
                        "is read from LDS (C2/C4) or L2 (C5), so HBM is not the bound",
            "algorithmic_flop_per_launch": flops,
            "algorithmic_scene_bytes_per_launch": alg_bytes,
            "lds_l2_scene_read_GBps_algorithmic": round(alg_bytes / avg_kernel_s / 1e9, 1),
            "note": "f32 VALU issue bound (SURVEY 8d): 23 FLOP/sphere test + 12 FLOP/box test over the "
                    "average HIP-event kernel time; peak = wave64 v_fma_f32 at 2 cycles on SIMD-32 "
                    "(SURVEY 8d's 78.6 assumed 16-lane SIMDs). lds_l2_scene_read_GBps_algorithmic = "
                    "(16 B/sphere test + 56 B/node visit) / kernel time: scene reads served by LDS/L2, not HBM",
        }
        if f64:
            roofline["note"] = ("f64 VALU issue bound: the books path's 23 FLOP per sphere test + 12 FLOP per box test "
                                "(SURVEY 8d), all f64 in the reference, over the average HIP-event time of the frame; "
                                "peak = MI355X FP64 vector 78.6 TFLOP/s (half the FP32 rate)")
        if scene.quads is not None or scene.media is not None:
            roofline["note"] += (" Book-2 scene: the kernel's primitive-test count (spheres, quads, medium boundaries) "
                                 "is priced at the sphere test's 23 FLOP / 16 B.")
        if issue:  # the binding limit: VALU issue slots and lanes per instruction (FLOP frac is low by construction)
            roofline.update(issue)
        out = {
            "metric": METRIC,
            "value": round(rays / elapsed / 1e6, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong" if bands else "weak",
            "vs_baseline": None,
            "dtype": "f64" if f64 else "f32",
            "data": "synthetic",
            "config": {
                "workload": f"{config + ' ' + SCENES[config] if config in SCENES else scene.name}, {W}x{H}x{S}spp, max_depth {scene.max_depth}, "
                            f"{len(scene.spheres)} spheres" + (f", {len(scene.quads)} quads" if scene.quads is not None else "")
                            + (f", {len(scene.media)} media" if scene.media is not None else ""),
                "image": [W, H],
                "spp": S,
                "max_depth": scene.max_depth,
                "parallelism": split,
            },
            "wall_clock_s_per_frame": round(elapsed / args.steps, 4),
            "rays_per_step": rays // args.steps,
            "rank0_rays_per_launch": work["rays"],
            "rank0_paths_per_launch": work["paths"],
            "sphere_tests_per_s": round(work["sphere_tests"] / avg_kernel_s, 1),
            "kernel_ms_avg": round(avg_kernel_s * 1e3, 3),
            "kernel_ms_max_over_ranks": round(kmax, 3),
            "bvh": ds.bvh_info(),
            "roofline": roofline,
        }
        if gather_ms is not None:
            out["gather_ms"] = round(float(np.mean(gather_ms)), 3)
            out["gather_note"] = "rank 0, HIP events between the end of its render and the end of the gather"
            if bands:
                out["rows_per_rank"] = [len(band_rows(H, band, r, world)) for r in range(world)]
        if world > 1:
            out["kernel_ms_per_rank"] = [round(v, 3) for v in rank_kernel_ms]
            out["kernel_ms_mean_over_ranks"] = round(float(np.mean(rank_kernel_ms)), 3)
            out["rank_imbalance"] = round(max(rank_kernel_ms) / float(np.mean(rank_kernel_ms)) - 1.0, 5)
            if one_gpu is not None:
                out["c3_one_gpu" if config == "C3" else "one_gpu_base"] = one_gpu
                out["scaling_efficiency"] = round(out["value"] / (world * one_gpu["mrays_s"]), 4)
                out["scaling_note"] = ("value / (n_gpus x the same frame on rank 0's GPU alone, measured in this run "
                                       "after the timed steps)")
        if f64_leg is not None:
            out["f64_books"] = f64_leg
        if world == 1 and not args.no_breakdown and not f64:
            out["wall_clock_breakdown"] = wall_clock_breakdown(scene, accum, avg_kernel_s * 1e3)
        cpus = host_cpus()
        if world == 1 and not args.no_extra and not f64:
            if config != "C3":
                out["c3_one_gpu"] = one_gpu_frame("C3")
            out["c1"] = c1_timings(cpus)
        if world == 1 and not args.no_f64 and not f64 and config in ("C1", "C2", "C4", "C5"):
            out["f64_books"] = f64_books_frame(config)
        if world == 1 and args.ref_slot and config in ("C1", "C2", "C5"):
            out["reference_gpu_slot"] = reference_gpu_slot(config)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(scene, args.cpu_seconds, cpus)
        print(json.dumps(out), flush=True)
    ds.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
