"""GPU against the f64 books path (the north star's correctness bar, camera.rs:182-209).

The kernel computes in f32 and is bit-exact against the oracle's f32 TWIN restatement
(test_gpu_parity.py). Against the f64 BOOKS restatement — the reference's own CPU arithmetic —
individual paths diverge where an f32/f64 rounding flips a discrete decision, so the gate is
statistical, on frames of >= 64x36x256: ray counts (GPU device counter) and mean radiance within
0.1 %, and stated minimum fractions of channels within the north star's 1e-4 and of equal u8
bytes. The round-1 kernel (no exit_skip: f32 bounces re-hit the r = 1000 ground sphere they
leave) traced +0.70 % rays at -0.21 % radiance on C2 and fails every C2/C5 bound here.

Measured at these sizes: C1 99.9 % / 100 %, C2 84.8 % / 97.3 %, C4 100 % / 100 %,
C5 77.7 % / 94.5 % (within 1e-4 / u8 equal).
"""
import numpy as np
import pytest

import rustraytrace_amd as rrt
from oracle import oracle

pytestmark = pytest.mark.gpu

# cfg: (min fraction of channels within 1e-4, min fraction of equal u8 bytes)
BOUNDS = {"C1": (0.99, 0.995), "C2": (0.80, 0.95), "C4": (0.995, 0.995), "C5": (0.72, 0.92)}


def _gpu_render_with_rays(scene):
    import torch

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    ds = rrt.DeviceScene(scene, device=0)
    tile = ds.tile(16, 0, 1, 0, scene.spp)
    rows = ds.tile_rows(tile)
    buf = torch.full((rows, scene.width, 4), float("nan"), dtype=torch.float32, device="cuda:0")
    ds.reset_counters()
    ds.render_tile_async(tile, buf.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    rays = int(ds.counters()["rays"])
    out = buf.cpu().numpy()
    ds.close()
    return out, rays


@pytest.mark.parametrize("cfg", sorted(BOUNDS))
def test_gpu_tracks_f64_books_path(cfg):
    scene = rrt.config_scene(cfg, image_width=64, samples_per_pixel=256)
    gpu, gpu_rays = _gpu_render_with_rays(scene)
    twin, twin_rays, _ = oracle.render(scene, oracle.TWIN, threads=16)
    assert np.array_equal(gpu.astype(np.float64), twin) and gpu_rays == twin_rays  # bit-exact vs TWIN
    books, books_rays, _ = oracle.render(scene, oracle.BOOKS, threads=16)
    S = scene.spp
    drays = gpu_rays / books_rays - 1.0
    drad = gpu[..., :3].astype(np.float64).mean() / books[..., :3].mean() - 1.0
    within = float((np.abs(gpu[..., :3] - books[..., :3]) / S <= 1e-4).mean())
    q_gpu = rrt.quantize_accum(scene.width, scene.height, gpu, S)
    q_books = rrt.quantize_accum(scene.width, scene.height, books.astype(np.float32), S)
    u8_equal = float((q_gpu == q_books).mean())
    print(f"{cfg}: rays {drays:+.4%} radiance {drad:+.4%} within 1e-4 {within:.4f} u8 equal {u8_equal:.4f}")
    assert abs(drays) < 1e-3, f"GPU traces {drays:+.4%} rays against the f64 books path"
    assert abs(drad) < 1e-3, f"GPU mean radiance {drad:+.4%} against the f64 books path"
    lo_within, lo_u8 = BOUNDS[cfg]
    assert within >= lo_within and u8_equal >= lo_u8
