"""The row-band multi-rank renderer (rustraytrace_amd/multi_gpu.py, config C3's split) launched by
torch.distributed.run: 2 and 3 ranks sharing this box's GPU, tiles gathered over gloo. The
gathered image must equal the 1-GPU render bit for bit (every pixel keyed by global indices)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import rustraytrace_amd as rrt

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("ranks,backend,band", [(1, "gloo", 8), (2, "gloo", 8), (3, "gloo", 8), (1, "nccl", 8),
                                                (2, "gloo", 0)])
def test_row_bands_gathered_equal_one_gpu(tmp_path, ranks, backend, band):
    # band 0: balanced_band picks the height (54 rows, 2 ranks: 9-row bands, 27 rows each).
    # (1, "nccl"): the RCCL process group and gather on the device tensors (RCCL refuses two
    # ranks on one GPU, so more ranks share the box's GPU over gloo).
    out = str(tmp_path / "accum.npy")
    ppm = str(tmp_path / "img.ppm")
    args = ["--config", "C2", "--width", "96", "--spp", "8", "--depth", "20", "--band", str(band),
            "--backend", backend, "--save-accum", out, "--out", ppm]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", "-m", "rustraytrace_amd.multi_gpu"] + args
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""), OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT, env=env, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["ranks"] == ranks and line["rays"] > 0 and line["backend"] == backend
    scene = rrt.config_scene("C2", image_width=96, samples_per_pixel=8, max_depth=20)
    want = rrt.render(scene)
    got = np.load(out)
    assert got.shape == want.shape and np.array_equal(got, want)
    with open(ppm, "rb") as f:
        assert f.read() == rrt.format_ppm_from_accum(scene.width, scene.height, want, scene.spp)


@pytest.mark.parametrize("ranks", [2, 3])
def test_f64_row_bands_gathered_equal_one_gpu_f64(tmp_path, ranks):
    """The f64 books kernel's tiles (RRT_FLAG_F64) over the row-band split, gathered as f64 over gloo
    by ranks sharing the GPU: the frame equals the 1-GPU f64 frame bit for bit, and so its books-path
    PPM (color.rs) byte for byte."""
    out = str(tmp_path / "accum64.npy")
    ppm = str(tmp_path / "img64.ppm")
    args = ["--config", "C2", "--width", "96", "--spp", "16", "--depth", "20", "--backend", "gloo", "--f64",
            "--save-accum", out, "--out", ppm]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", "-m", "rustraytrace_amd.multi_gpu"] + args
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""), OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT, env=env, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["ranks"] == ranks and line["dtype"] == "f64"
    scene = rrt.config_scene("C2", image_width=96, samples_per_pixel=16, max_depth=20)
    want = rrt.render_f64(scene)
    got = np.load(out)
    assert got.dtype == np.float64 and got.shape == want.shape and np.array_equal(got, want)
    rgb8 = rrt.quantize_accum_books_f64(scene.width, scene.height, want, scene.spp)
    with open(ppm, "rb") as f:
        assert f.read() == rrt.format_pnm_from_rgb8(scene.width, scene.height, rgb8)


def test_bench_f64_band_leg():
    """bench.py's N > 1 line carries the f64 books kernel over the same band split (f64_books: value,
    per-rank kernel times, gather, 1-GPU base), 2 ranks sharing the GPU over gloo; and `--f64` makes
    the f64 kernel the timed headline leg (dtype f64)."""
    base = ["bench.py", "--gpus", "2", "--config", "C3", "--width", "256", "--spp", "8", "--steps", "2",
            "--warmup", "1", "--no-cpu-baseline", "--no-breakdown"]
    env = dict(os.environ, RRT_BENCH_BACKEND="gloo", OMP_NUM_THREADS="1")
    scene = rrt.config_scene("C3", image_width=256, samples_per_pixel=8)
    ds = rrt.DeviceScene(scene, f64=True)
    want = ds.count_work(ds.tile(16, 0, 1, 0, 8))["rays"]
    ds.close()
    for extra in ([], ["--f64"]):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
               "--master-addr", "127.0.0.1", f"--master-port={_free_port()}"] + base + extra
        r = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT, env=env, timeout=110)
        assert r.returncode == 0, r.stderr[-2000:]
        line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
        if extra:
            assert line["dtype"] == "f64" and line["rays_per_step"] == want and "f64_books" not in line
            assert line["c3_one_gpu"]["rays"] == want and line["scaling_efficiency"] > 0
        else:
            assert line["dtype"] == "f32"
            leg = line["f64_books"]
            assert leg["dtype"] == "f64" and leg["rays_per_step"] == want and leg["rows_per_rank"] == [72, 72]
            assert len(leg["kernel_ms_per_rank"]) == 2 and leg["gather_ms"] >= 0
            assert leg["one_gpu_base"]["rays"] == want and leg["scaling_efficiency"] > 0


@pytest.mark.parametrize("ranks", [1, 2])
def test_bench_band_split_line(ranks):
    # bench.py's N-rank path (C3's row-band split, gather inside the timed step) at a small size:
    # 2 ranks share the GPU over gloo (RRT_BENCH_BACKEND rehearsal mode); 1 rank runs the C3
    # default config only when launched with --config.
    args = ["bench.py", "--gpus", str(ranks), "--config", "C3", "--width", "256", "--spp", "8", "--steps", "2",
            "--warmup", "1", "--no-cpu-baseline", "--no-breakdown", "--no-extra"]
    if ranks > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
               "--master-addr", "127.0.0.1", f"--master-port={_free_port()}"] + args
    else:
        cmd = [sys.executable] + args
    env = dict(os.environ, RRT_BENCH_BACKEND="gloo", OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT, env=env, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == ranks and line["scaling"] == "strong" and line["config"]["image"] == [256, 144]
    scene = rrt.config_scene("C3", image_width=256, samples_per_pixel=8)
    ds = rrt.DeviceScene(scene)
    want = ds.count_work(ds.tile(16, 0, 1, 0, 8))["rays"]
    ds.close()
    assert line["rays_per_step"] == want  # every band rendered exactly once per step
    if ranks > 1:
        assert "gather_ms" in line and "bands" in line["config"]["parallelism"]
        assert sum(line["rows_per_rank"]) == 144
        assert line["rows_per_rank"] == [144 // ranks] * ranks  # balanced_band: 12-row bands at 2 ranks
    else:
        assert "no gather" in line["config"]["parallelism"]


def test_bench_spawns_its_own_ranks():
    # `python bench.py --gpus 2` with no external launcher: bench.py starts torch.distributed.run as
    # a child (2 ranks sharing this GPU over gloo), forwards rank 0's line, and the N > 1 line
    # carries the per-rank kernel times, the gather time and the same frame on one GPU.
    args = ["bench.py", "--gpus", "2", "--config", "C3", "--width", "256", "--spp", "8", "--steps", "2",
            "--warmup", "1", "--no-cpu-baseline", "--no-breakdown"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(RRT_BENCH_BACKEND="gloo", OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable] + args, capture_output=True, text=True, cwd=ROOT, env=env, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1  # stdout holds exactly rank 0's line
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["rows_per_rank"] == [72, 72] and "gather_ms" in line
    assert len(line["kernel_ms_per_rank"]) == 2 and line["kernel_ms_max_over_ranks"] == max(line["kernel_ms_per_rank"])
    base = line["c3_one_gpu"]
    assert base["workload"].startswith("C3 256x144x8spp")
    assert base["rays"] == line["rays_per_step"]  # the same frame, whole, on one GPU
    assert line["scaling_efficiency"] > 0
