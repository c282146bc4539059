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


@pytest.mark.parametrize("ranks", [1, 2, 3])
def test_row_bands_gathered_equal_one_gpu(tmp_path, ranks):
    out = str(tmp_path / "accum.npy")
    ppm = str(tmp_path / "img.ppm")
    args = ["--config", "C2", "--width", "96", "--spp", "8", "--depth", "20", "--band", "8",
            "--backend", "gloo", "--save-accum", out, "--out", ppm]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", "-m", "rustraytrace_amd.multi_gpu"] + args
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""), OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT, env=env, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["ranks"] == ranks and line["rays"] > 0
    scene = rrt.config_scene("C2", image_width=96, samples_per_pixel=8, max_depth=20)
    want = rrt.render(scene)
    got = np.load(out)
    assert got.shape == want.shape and np.array_equal(got, want)
    with open(ppm, "rb") as f:
        assert f.read() == rrt.format_ppm_from_accum(scene.width, scene.height, want, scene.spp)
