"""GPU parity: librrt_hip.so (through its C-ABI) vs the oracle's f32 TWIN restatement of the
reference's books path (oracle/rrt_oracle.cpp). Tolerance: bit-exact accum (the north star's
per-channel 1e-4 bound is asserted too, and is strictly weaker) and byte-identical PPM.

Parity is "pinned" against the oracle; the oracle itself is pinned by tests/test_oracle.py
(known-answer vectors, committed golden fixtures, and its f64 BOOKS mode).
"""
import numpy as np
import pytest

import rustraytrace_amd as rrt
from oracle import oracle
from rustraytrace_amd.render import build_bvh

pytestmark = pytest.mark.gpu


def _torch():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


def gpu_tile(scene, band_rows=16, rank=0, n_ranks=1, s0=0, s1=None, count=False):
    """Render one tile through the device-resident API; returns (accum[rows,W,4], rows, counters)."""
    torch = _torch()
    ds = rrt.DeviceScene(scene, device=0)
    tile = ds.tile(band_rows, rank, n_ranks, s0, s1 if s1 is not None else scene.spp)
    rows = ds.tile_rows(tile)
    buf = torch.full((max(rows, 1), scene.width, 4), float("nan"), dtype=torch.float32, device="cuda:0")
    ds.reset_counters()
    stream = torch.cuda.current_stream()
    ds.render_tile_async(tile, buf.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    ctr = ds.counters()
    work = ds.count_work(tile) if count else None
    idx = ds.tile_row_indices(tile)
    out = buf[:rows].cpu().numpy()
    ds.close()
    return out, idx, ctr, work


def assert_bit_exact(gpu, ref, spp):
    ref32 = ref.astype(np.float32)
    assert np.array_equal(ref32.astype(np.float64), ref), "oracle TWIN sums must be exact f32"
    diff = np.abs(gpu.astype(np.float64) - ref)
    per_channel = diff[..., :3] / max(spp, 1)
    assert per_channel.max() <= 1e-4  # north-star tolerance (before u8 quantisation)
    assert diff.max() == 0.0, f"max |gpu - oracle| = {diff.max()} at {np.unravel_index(diff.argmax(), diff.shape)}"


SMALL = [
    ("C1", dict(image_width=64, samples_per_pixel=8)),
    ("C2", dict(image_width=64, samples_per_pixel=8)),
    ("C2", dict(image_width=96, samples_per_pixel=4, max_depth=6)),
    ("C4", dict(image_width=64, samples_per_pixel=8)),
    ("C5", dict(image_width=64, samples_per_pixel=4)),
]


@pytest.mark.parametrize("cfg,kw", SMALL, ids=[f"{c}-{k.get('image_width')}x{k.get('samples_per_pixel')}" for c, k in SMALL])
def test_one_shot_matches_oracle(cfg, kw):
    scene = rrt.config_scene(cfg, **kw)
    gpu = rrt.render(scene)
    ref, rays, _ = oracle.render(scene, oracle.TWIN)  # independent books-structured tree
    assert_bit_exact(gpu, ref, scene.spp)
    nodes, order, info = build_bvh(scene)
    kref, krays, _ = oracle.render_kbvh(scene, nodes, order, info)  # the kernel's own tree
    assert_bit_exact(gpu, kref, scene.spp)
    assert krays == rays
    assert np.all(gpu[..., 3] == scene.spp)
    a = rrt.format_ppm_from_accum(scene.width, scene.height, gpu, scene.spp)
    b = rrt.format_ppm_from_accum(scene.width, scene.height, ref.astype(np.float32), scene.spp)
    assert a == b


@pytest.mark.parametrize("depth", [0, 1, 2, 5, 6, 50])
def test_depth_and_roulette_boundaries(depth):
    scene = rrt.rtow(image_width=48, samples_per_pixel=6, max_depth=depth)
    gpu = rrt.render(scene)
    ref, _, _ = oracle.render(scene, oracle.TWIN)
    assert_bit_exact(gpu, ref, scene.spp)
    if depth == 0:
        assert np.all(gpu[..., :3] == 0)


def test_ray_counts_match_oracle():
    scene = rrt.rtow(image_width=64, samples_per_pixel=8, max_depth=20)
    gpu, idx, ctr, work = gpu_tile(scene, count=True)
    ref, rays, _ = oracle.render(scene, oracle.TWIN)
    assert_bit_exact(gpu, ref, scene.spp)
    assert ctr["rays"] == rays
    assert ctr["paths"] == scene.width * scene.height * scene.spp
    assert work["rays"] == rays and work["paths"] == ctr["paths"]
    assert work["node_visits"] > 0 and work["sphere_tests"] > 0


@pytest.mark.parametrize("n_ranks,band", [(2, 16), (3, 8), (8, 4)])
def test_row_band_tiles_reassemble(n_ranks, band):
    scene = rrt.rtow(image_width=40, samples_per_pixel=4, max_depth=10)
    full = rrt.render(scene)
    img = np.full_like(full, np.nan)
    for r in range(n_ranks):
        part, idx, _, _ = gpu_tile(scene, band_rows=band, rank=r, n_ranks=n_ranks)
        img[idx] = part
    assert np.array_equal(img, full)


def test_sample_range_tile_matches_oracle():
    scene = rrt.rtow(image_width=32, samples_per_pixel=16, max_depth=10)
    gpu, idx, _, _ = gpu_tile(scene, s0=5, s1=13)
    ref, _, _ = oracle.render(scene, oracle.TWIN, samples=(5, 13))
    assert_bit_exact(gpu, ref, 8)
    assert np.all(gpu[..., 3] == 8)


def test_background_mode_and_no_defocus():
    scene = rrt.build_in_one_weekend_scene(dict(image_width=48, samples_per_pixel=4, max_depth=8, defocus_angle=0.0,
                                                background=(0.2, 0.3, 0.9)))
    assert int(scene.camera["params_u"][0, 3]) == 1
    gpu = rrt.render(scene)
    ref, _, _ = oracle.render(scene, oracle.TWIN)
    assert_bit_exact(gpu, ref, scene.spp)


def test_multi_gpu_one_shot_equals_single():
    torch = _torch()
    n = torch.cuda.device_count()
    scene = rrt.rtow(image_width=48, samples_per_pixel=4, max_depth=8)
    a = rrt.render(scene, n_gpus=1)
    if n >= 2:
        b = rrt.render(scene, n_gpus=min(n, 8))
        assert np.array_equal(a, b)
    with pytest.raises(rrt.RrtError):
        rrt.render(scene, n_gpus=n + 1)


@pytest.mark.parametrize("spp,s0", [(200, 0), (130, 7), (128, 0), (100, 3), (9, 0), (129, 0), (300, 0), (600, 0),
                                    (256, 0), (257, 0), (64, 0), (65, 0)])
def test_chunked_accumulation_matches_oracle(spp, s0):
    # rrt_accum_chunk() = 256; frames of S <= 256 samples use K = 64 (tail chunks of K/4 = 16, or
    # K/8 = 8 when S <= 64: no big chunk), up to 512 K = 128 (tail chunks of 32), larger ones K = 256
    # (tail chunks of 64): (128, 0): 64 + 4 x 16; (100, 3): 64 + 2 x 16 + 4; (9, 0): 8 + 1; (129, 0):
    # 2 x 64 + 1; (200, 0): 3 x 64 + 8; (300, 0): 2 x 128 + 32 + 12; (600, 0): 2 x 256 + 64 + 24;
    # (256, 0): 3 x 64 + 4 x 16; (257, 0): 2 x 128 + 1; the ABI v11 boundary: (64, 0): 8 x 8,
    # (65, 0): 64 + 1.
    # > rrt_accum_chunk() samples: the persistent queue splits pixels into chunks whose sums are
    # combined in chunk order; the oracle reproduces that order (rows, partial last chunk, offset).
    assert rrt._lib.load().rrt_accum_chunk() == oracle.DEFAULT_CHUNK
    scene = rrt.rtow(image_width=24, samples_per_pixel=spp, max_depth=8)
    gpu, idx, ctr, _ = gpu_tile(scene, s0=s0, s1=s0 + spp)
    ref, rays, _ = oracle.render(scene, oracle.TWIN, samples=(s0, s0 + spp))
    assert_bit_exact(gpu, ref, spp)
    assert np.all(gpu[..., 3] == spp) and ctr["rays"] == rays


def test_sample_passes_are_bit_identical(monkeypatch):
    # A 1 MiB partial budget holds 4 chunks of this 160x90 frame (230 KB each): its 11 chunks
    # (K = 64 at 250 spp: 3 x 64 samples, then 7 x 8 + 2) run as 3 sample passes of 4, 4, 3
    # chunks — the first mixes big and tail chunks — whose combines continue one fold: same bits
    # as one pass.
    scene = rrt.rtow(image_width=160, samples_per_pixel=250, max_depth=8)
    one, _, ctr1, _ = gpu_tile(scene)
    monkeypatch.setenv("RRT_PARTIAL_MB", "1")
    passes, _, ctr4, _ = gpu_tile(scene)
    assert np.array_equal(one, passes) and ctr1["rays"] == ctr4["rays"]
    ref, rays, _ = oracle.render(scene, oracle.TWIN, threads=16)
    assert_bit_exact(passes, ref, scene.spp)
    assert ctr4["rays"] == rays


def test_zero_samples_tile():
    scene = rrt.rtow(image_width=16, samples_per_pixel=4, max_depth=4)
    gpu, idx, ctr, _ = gpu_tile(scene, s0=3, s1=3)
    assert np.all(gpu == 0) and ctr["rays"] == 0


def _book1_scene(kinds, textured):
    """A small book-1 scene with the given material kinds (0 Lambertian, 1 metal, 2 dielectric,
    4 light), optionally with the earth texture on the big sphere; sky background, defocus on."""
    from rustraytrace_amd import scenes as sc

    mats = [sc._material(3 if textured else 0, (0.5, 0.5, 0.5), tex=0)]
    sph = [sc._sphere((0.0, -1000.0, 0.0), 1000.0, 0), sc._sphere((0.0, 1.0, 0.0), 1.0, 0)]
    for i, k in enumerate(kinds):
        mats.append(sc._material(k, (0.7, 0.6, 0.5), fuzz=0.2, ref_idx=1.5))
        sph.append(sc._sphere((-3.0 + 2.0 * i, 0.6, 1.5), 0.6, len(mats) - 1))
    mats, sph = np.concatenate(mats), np.concatenate(sph)
    cam = sc.make_camera(aspect_ratio=16.0 / 9.0, image_width=48, samples_per_pixel=4, max_depth=12, vfov=30.0,
                         lookfrom=(6.0, 2.5, 8.0), lookat=(0.0, 0.5, 0.0), defocus_angle=0.6, focus_dist=9.0,
                         seed=7, n_spheres=len(sph))
    return sc.SceneData(cam, sph, mats, textures=[sc.earth_texture()] if textured else [], name="book1_classes")


@pytest.mark.parametrize("in_lds", ["1", "0"])
@pytest.mark.parametrize("kinds,textured", [((1, 2), True), ((0, 4), True), ((0, 4), False), ((1, 2), False)],
                         ids=["tex+specular", "tex+diffuse", "diffuse", "specular"])
def test_book1_kernel_classes_match_oracle(monkeypatch, kinds, textured, in_lds):
    # The host picks the book-1 kernel by the materials present and by where the scene lives:
    # textures and metal/dielectric compiled in or out (classes 0, -1, -2) on LDS scenes, the
    # 256 x 7 launch for scenes read from L2 (RRT_SCENE_IN_LDS=0). Every combination is
    # bit-exact against the oracle.
    monkeypatch.setenv("RRT_SCENE_IN_LDS", in_lds)
    scene = _book1_scene(kinds, textured)
    gpu = rrt.render(scene)
    ref, _, _ = oracle.render(scene, oracle.TWIN)
    assert_bit_exact(gpu, ref, scene.spp)


@pytest.mark.parametrize("width,spp", [(24, 3), (40, 300), (200, 9)])
def test_uneven_queues_drain(width, spp):
    """Every work unit is claimed whatever the queues' sizes (rrt_kernel.hip work-queue comment):
    frames whose 64-unit groups do not fill the 8 queues evenly (3 groups: queues 3-7 start empty;
    a partial last group), with tiles of very different cost (sky-only rows against ground rows),
    so the queues drain at different rates; every pixel's count w must equal the samples and the
    image must equal the oracle's."""
    scene = rrt.rtow(image_width=width, samples_per_pixel=spp, max_depth=8)
    gpu, idx, _, _ = gpu_tile(scene)
    assert np.all(gpu[..., 3] == spp)
    if width * spp <= 40 * 300:
        ref, _, _ = oracle.render(scene, oracle.TWIN, threads=16)
        assert_bit_exact(gpu, ref[idx], spp)


def test_counting_kernel_matches_oracle_test_counts():
    """The instrumented kernel's sphere-test count (bench.py's roofline numerator) equals the
    oracle's count over the kernel's own tree (KBVH): every primitive of a visited leaf range is
    a test, the exit_skip primitive included (left out of the loop, counted once)."""
    scene = rrt.rtow(image_width=48, samples_per_pixel=4, max_depth=8)
    _, _, ctr, work = gpu_tile(scene, count=True)
    nodes, order, info = build_bvh(scene)
    _, rays, tests = oracle.render_kbvh(scene, nodes, order, info, threads=16)
    assert work["rays"] == rays == ctr["rays"]
    assert work["sphere_tests"] == tests


@pytest.mark.parametrize("s", [1.0, 3000.0, 1e5])
def test_f16_global_nodes_at_every_scale(monkeypatch, s):
    """Scenes read from global memory walk 32-B f16 nodes (planes rounded outward, saturating to
    +-inf / 65504 beyond f16's range: tests/test_f16_nodes.py). The kernel reads them with
    v_fma_mix_f32 and must take the oracle KBVH walk's every decision on the same bits."""
    from test_f16_nodes import scaled_scene

    monkeypatch.setenv("RRT_SCENE_IN_LDS", "0")
    scene = scaled_scene(rrt.rtow(image_width=40, samples_per_pixel=4, max_depth=8), s)
    nodes, order, info = build_bvh(scene)
    assert info["node_stride"] == 32
    gpu, idx, ctr, _ = gpu_tile(scene)
    ref, rays, _ = oracle.render_kbvh(scene, nodes, order, info, threads=16)
    assert ctr["rays"] == rays
    assert_bit_exact(gpu, ref[idx], scene.spp)
