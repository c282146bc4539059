"""GPU side of the output step: the device render_io quantiser and the
rgb8 one-shot entry, byte-identical to the host quantiser of the float accum (which
tests/test_output.py pins against the oracle's render_io restatement)."""
import numpy as np
import pytest

import rustraytrace_amd as rrt
from oracle import oracle

pytestmark = pytest.mark.gpu
INF = float("inf")


def _torch():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


@pytest.mark.parametrize("n_px", [1, 3, 4, 5, 1000, 1920 * 1080 + 3])
def test_device_quantiser_matches_host(n_px):
    torch = _torch()
    rng = np.random.default_rng(n_px)
    spp = 13
    acc = (rng.uniform(-0.3, 1.4, size=(n_px, 4)) * spp).astype(np.float32)
    edge = np.array([0.0, INF, -INF, float("nan"), -0.0, 1e38, 0.999 ** 2 * spp, 1e-45], np.float32)
    acc[: min(n_px, len(edge)), 0] = edge[: min(n_px, len(edge))]
    d_acc = torch.from_numpy(acc).to("cuda:0")
    d_rgb = torch.full((n_px * 3,), 77, dtype=torch.uint8, device="cuda:0")
    rrt.quantize_accum_async(n_px, d_acc.data_ptr(), spp, d_rgb.data_ptr(),
                             torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = d_rgb.cpu().numpy().reshape(-1, 3)
    want = rrt.quantize_accum(n_px, 1, acc, spp).reshape(-1, 3)
    assert np.array_equal(got, want)
    assert np.array_equal(want, oracle.quantize_render_io(acc, spp))


@pytest.mark.parametrize("cfg", ["rtow", "earth", "bouncing", "perlin", "cornell_box", "cornell_smoke", "book3"])
def test_render_rgb8_equals_quantised_accum(cfg):
    # Every book through rrt_hip_render_rgb8_ex: moving spheres (bouncing), Perlin tables,
    # quads, media and the book-3 light list must reach the device quantiser path too.
    _torch()
    small = dict(image_width=64, samples_per_pixel=9, max_depth=10)
    if cfg == "rtow":
        scene = rrt.rtow(image_width=96, samples_per_pixel=6, max_depth=10)
    elif cfg == "earth":
        scene = rrt.earth_light(image_width=80, samples_per_pixel=5, max_depth=8)
    elif cfg == "book3":
        scene = rrt.rest_of_your_life_scene(small)
    else:
        k = {"bouncing": 1, "perlin": 4, "cornell_box": 7, "cornell_smoke": 8}[cfg]
        scene = rrt.next_week_scene(k, small)
    acc = rrt.render(scene)
    rgb = rrt.render_rgb8(scene)
    assert rgb.shape == (scene.height, scene.width, 3)
    assert np.array_equal(rgb, rrt.quantize_accum(scene.width, scene.height, acc, scene.spp))
    p3 = rrt.format_pnm_from_rgb8(scene.width, scene.height, rgb)
    assert p3 == rrt.format_ppm_from_accum(scene.width, scene.height, acc, scene.spp)


def test_cli_output_paths_agree(tmp_path):
    import os
    import subprocess

    _torch()
    cli = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rustraytrace_amd", "rrt")
    args = [cli, "--backend", "hip", "in_one_weekend", "--image_width", "64", "--samples_per_pixel", "3",
            "--max_depth", "6"]
    outs = {}
    for name, extra in [("dev", []), ("host", ["--host-quantise"]), ("p6", ["--p6"])]:
        path = tmp_path / f"{name}.ppm"
        r = subprocess.run(args + extra + ["-o", str(path)], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
        outs[name] = path.read_bytes()
    assert outs["dev"] == outs["host"]
    head, px = outs["p6"].split(b"\n255\n", 1)
    assert head == b"P6\n64 36"
    vals = [int(v) for v in outs["dev"].split(b"\n255\n", 1)[1].split()]
    assert list(px) == vals


def test_cli_reports_progress_within_the_render(tmp_path):
    # rrt_hip_render polls the work-queue heads while the kernel runs and prints the fraction
    # done (the reference prints one line per sample pass, cuda/mod.rs:426-431): a ~0.4 s render
    # shows intermediate percentages, increasing, then 100 % with the GPU count.
    import os
    import re
    import subprocess

    _torch()
    cli = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rustraytrace_amd", "rrt")
    r = subprocess.run([cli, "--backend", "hip", "in_one_weekend", "--image_width", "1920", "--samples_per_pixel",
                        "2048", "-o", str(tmp_path / "p.ppm"), "--p6"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    pcts = [int(p) for p in re.findall(r"HIP progress: (\d+)%", r.stderr)]
    assert pcts and pcts[-1] == 100 and "(1/1 GPUs done)" in r.stderr
    assert any(0 < p < 100 for p in pcts) and pcts == sorted(pcts)
