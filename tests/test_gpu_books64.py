"""The f64 books path (RRT_FLAG_F64, rrt_books64.hip) against the oracle's f64 BOOKS restatement:
the north star's correctness check "against the repo's own CPU books path on identical scene + RNG
seed (per-channel float tolerance <= 1e-4 before u8 quantisation; bit-exact PPM after)".

The kernel runs the books path's arithmetic (vec3.rs, sphere.rs:24-51, material.rs, camera.rs:
152-209 in f64, unfused, the reference's operation order) on the same per-path random stream, so
every path takes the same decisions as BOOKS and the closest-hit query counts are equal. It also
forms each path's radiance back to front like BOOKS' recursion (the attenuation history,
rrt_books64.hip fold_back64) and sums each pixel's samples in sample order like camera.rs:72-76
(`pixel_color += ray_color(..)`: a prefix chunk summed in the lane, the tail samples folded in after
the pass). So its f64 sums equal BOOKS' (the oracle's default for BOOKS: sequential sums) bit for
bit, and the bars written here are: every sum bit-identical (which implies the north star's
per-channel |gpu - books| / S <= 1e-4 and equal PPM bytes, both still checked and printed), the
query counts equal. The comparison against BOOKS summed in the f32 kernel's chunk schedule (the
round-4 order) is printed for reference, within 1e-4. Full-size rows also report how many channels
sit within 1e-12 (relative) of a quantisation step of color.rs: the bytes a last-ulp difference in
the sum could have moved, which the bit-identical sums rule out.
"""
import numpy as np
import pytest

import rustraytrace_amd as rrt
from oracle import oracle

pytestmark = pytest.mark.gpu

TOL = 1e-4  # north star: per-channel float tolerance before u8 quantisation


def _gpu_f64(scene, rows=None):
    import torch

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    ds = rrt.DeviceScene(scene, device=0, f64=True)
    tile = ds.tile(16, 0, 1, 0, scene.spp)
    n_rows = ds.tile_rows(tile)
    buf = torch.full((n_rows, scene.width, 4), float("nan"), dtype=torch.float64, device="cuda:0")
    ds.reset_counters()
    ds.render_tile_f64_async(tile, buf.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    rays = int(ds.counters()["rays"])
    # the float entry on the same scene: the f64 sums rounded to f32
    buf32 = torch.full((n_rows, scene.width, 4), float("nan"), dtype=torch.float32, device="cuda:0")
    ds.render_tile_async(tile, buf32.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    out, out32 = buf.cpu().numpy(), buf32.cpu().numpy()
    ds.close()
    return out, out32, rays


def _step_exposure(books, S):
    """Channels of the f64 sums whose color.rs value 256 clamp(sqrt(v / S), 0, .999) lies within
    1e-12 (relative) of an integer step: the ones a last-ulp change of the sum could move a byte."""
    v = np.sqrt(np.maximum(books[..., :3] / S, 0.0))
    x = 256.0 * np.minimum(v, 0.999)
    near = np.abs(x - np.round(x)) <= 1e-12 * np.maximum(x, 1e-300)
    return int((near & (x > 0)).sum())


def _check(scene, gpu, books, label, bar="bits"):
    """bar: "bits" (every sum identical; implies the rest), "bytes" (within 1e-4 and every PPM byte
    equal: the north star's bars), "tol" (within 1e-4 only)."""
    S = scene.spp
    assert np.array_equal(gpu[..., 3], books[..., 3])  # w = sample count
    err = np.abs(gpu[..., :3] - books[..., :3]) / S
    within = float((err <= TOL).mean())
    rel = float((np.abs(gpu[..., :3] - books[..., :3]) / np.maximum(np.abs(books[..., :3]), 1e-300)).max())
    q_gpu = rrt.quantize_accum_books_f64(scene.width, gpu.shape[0], np.ascontiguousarray(gpu), S)
    q_books = rrt.quantize_accum_books_f64(scene.width, books.shape[0], np.ascontiguousarray(books), S)
    u8_equal = float((q_gpu == q_books).mean())
    nbits = int((gpu[..., :3] != books[..., :3]).sum())
    print(f"{label}: max |diff|/S {err.max():.3e} max rel {rel:.3e} within 1e-4 {within:.6f} u8 equal {u8_equal:.6f}"
          f" bit-differing channels {nbits} of {books[..., :3].size}")
    assert within == 1.0, f"{label}: {1 - within:.2e} of channels outside {TOL}"
    if bar in ("bits", "bytes"):
        assert u8_equal == 1.0, f"{label}: {int((q_gpu != q_books).sum())} PPM bytes differ"
    if bar == "bits":
        assert nbits == 0, f"{label}: {nbits} channels differ in their bits"
    return rel


@pytest.mark.parametrize("cfg", ["C1", "C2", "C4", "C5"])
def test_f64_kernel_matches_books_path(cfg):
    scene = rrt.config_scene(cfg, image_width=64, samples_per_pixel=256)
    gpu, gpu32, gpu_rays = _gpu_f64(scene)
    books, books_rays, _ = oracle.render(scene, oracle.BOOKS, threads=16)  # camera.rs:72-76's order
    assert gpu_rays == books_rays, f"{cfg}: {gpu_rays} closest-hit queries vs BOOKS {books_rays}"
    _check(scene, gpu, books, cfg)
    chunked, _, _ = oracle.render(scene, oracle.BOOKS, threads=16, chunk=oracle.DEFAULT_CHUNK)
    _check(scene, gpu, chunked, f"{cfg} vs BOOKS in the f32 chunk schedule", bar="tol")
    assert np.array_equal(gpu32, gpu.astype(np.float32))
    # the PPM the books path prints (camera.rs:87-94) and the one from the GPU's f64 sums
    q = rrt.quantize_accum_books_f64(scene.width, scene.height, gpu, scene.spp)
    qb = rrt.quantize_accum_books_f64(scene.width, scene.height, books, scene.spp)
    assert rrt.format_pnm_from_rgb8(scene.width, scene.height, q) == rrt.format_pnm_from_rgb8(scene.width,
                                                                                              scene.height, qb)


def test_f64_earth_texels_whole_frame():
    """C4's whole frame at 640x360x64 (14.7 M paths, the earth from pole to pole): the texels the
    kernel decides from f32 enclosures of the fdlibm angles, and those it falls back to fdlibm for,
    are the books path's — every sum bit for bit (rrt_books64.hip texel_bytes64)."""
    scene = rrt.config_scene("C4", image_width=640, samples_per_pixel=64)
    gpu, _, gpu_rays = _gpu_f64(scene)
    books, books_rays, _ = oracle.render(scene, oracle.BOOKS, threads=16)
    assert gpu_rays == books_rays
    _check(scene, gpu, books, "C4 640x360x64")


def test_f64_one_shot_render_and_ppm():
    scene = rrt.config_scene("C2", image_width=48, samples_per_pixel=64)
    accum = rrt.render_f64(scene)
    books, _, _ = oracle.render(scene, oracle.BOOKS, threads=16)
    _check(scene, accum, books, "C2 one-shot")


@pytest.mark.parametrize("cfg,rows", [("C2", (536, 552)), ("C4", (536, 544)), ("C5", (600, 608))])
def test_f64_full_size_rows_match_books(cfg, rows):
    """Full BASELINE resolution and spp (C2 1920x1080x512, C4 x1024, C5 x256): the GPU renders the
    whole frame in f64; the oracle renders a band of rows of it in f64 (seconds on 16 threads)."""
    scene = rrt.config_scene(cfg)
    gpu, _, _ = _gpu_f64(scene)
    y0, y1 = rows
    books, _, _ = oracle.render(scene, oracle.BOOKS, rows=rows, threads=16)
    _check(scene, gpu[y0:y1], books, f"{cfg} rows {y0}-{y1}")
    print(f"{cfg} rows {y0}-{y1}: {_step_exposure(books, scene.spp)} of {books[..., :3].size} channels within "
          f"1e-12 (relative) of a color.rs quantisation step")
    assert np.all(gpu[..., 3] == scene.spp)
    assert np.isfinite(gpu).all()


def test_f64_deep_max_depth_keeps_the_full_grid(capfd):
    """max_depth 5000: 60 KB of attenuation history per lane slot, 15.7 GB for the full persistent grid
    (a fixed 4-GiB history cap cut the grid silently). The history is sized within the
    device's free memory, so the render keeps every lane and stays bit-identical to BOOKS."""
    scene = rrt.config_scene("C1", image_width=64, samples_per_pixel=16, max_depth=5000)
    gpu, _, gpu_rays = _gpu_f64(scene)
    books, books_rays, _ = oracle.render(scene, oracle.BOOKS, threads=16)
    assert gpu_rays == books_rays
    _check(scene, gpu, books, "C1 depth 5000")
    assert "grid is reduced" not in capfd.readouterr().err


def test_f64_rejects_book2_scenes():
    sc = rrt.next_week_scene(1, dict(image_width=32, samples_per_pixel=4, max_depth=4))
    with pytest.raises(rrt.RrtError, match="RRT_FLAG_F64"):
        rrt.DeviceScene(sc, device=0, f64=True)


def test_f64_sample_passes_are_bit_identical(monkeypatch):
    """The chunk partials in bounded sample passes continue one f64 fold: the bits do not depend
    on the partial budget (RRT_PARTIAL_MB)."""
    scene = rrt.config_scene("C2", image_width=64, samples_per_pixel=600)
    a, _, _ = _gpu_f64(scene)
    monkeypatch.setenv("RRT_PARTIAL_MB", "1")
    b, _, _ = _gpu_f64(scene)
    assert np.array_equal(a, b)


def _textured_specular_scene(image_width=64, samples_per_pixel=256):
    """A book-1 scene with an image texture AND metal and dielectric materials: the f64 kernel's
    full class (launch_render_pass_f64 picks it only when both are present; the BASELINE configs
    run the untextured (C2, C5) and diffuse (C1, C4) classes)."""
    from rustraytrace_amd import scenes as S

    mats = np.concatenate([S._material(3, (0.0, 0.0, 0.0), tex=0), S._material(1, (0.7, 0.6, 0.5), fuzz=0.1),
                           S._material(2, (1.0, 1.0, 1.0), ref_idx=1.5), S._material(0, (0.5, 0.5, 0.5)),
                           S._material(4, (4.0, 4.0, 4.0))])
    sph = np.concatenate([S._sphere((0.0, 0.0, 0.0), 2.0, 0), S._sphere((4.2, 0.0, 0.0), 1.5, 1),
                          S._sphere((-4.2, 0.0, 0.0), 1.5, 2), S._sphere((0.0, -1002.0, 0.0), 1000.0, 3),
                          S._sphere((0.0, 7.0, 0.0), 2.0, 4)])
    cam = S.make_camera(aspect_ratio=16.0 / 9.0, image_width=image_width, samples_per_pixel=samples_per_pixel,
                        max_depth=20, vfov=40.0, lookfrom=(0.0, 2.0, 14.0), lookat=(0.0, 0.0, 0.0),
                        seed=0x7E57, n_spheres=len(sph))
    return S.SceneData(cam, sph, mats, textures=[S.earth_texture()], name="textured_specular")


def test_f64_full_class_matches_books_path():
    scene = _textured_specular_scene()
    gpu, gpu32, gpu_rays = _gpu_f64(scene)
    books, books_rays, _ = oracle.render(scene, oracle.BOOKS, threads=16)
    assert gpu_rays == books_rays, f"{gpu_rays} closest-hit queries vs BOOKS {books_rays}"
    _check(scene, gpu, books, "textured + specular")
    assert np.array_equal(gpu32, gpu.astype(np.float32))


def _negative_albedo_scene(specular):
    """An image-textured class (the only classes whose history records can hold texel bytes) with
    Lambertian and metal albedos that are negative or -0 on some channels: BOOKS multiplies by them as
    given (the round-5 history read a negative albedo back as a texel byte)."""
    from rustraytrace_amd import scenes as S

    sc = _textured_specular_scene(image_width=48, samples_per_pixel=64)
    mats = sc.materials.copy()
    mats[3]["albedo_fuzz"][:3] = (-0.35, 0.5, -0.0)  # the ground
    if specular:
        mats[1]["albedo_fuzz"][:3] = (0.7, -0.6, 0.5)  # the metal
    else:  # no metal or dielectric: the diffuse class
        mats[1] = S._material(0, (-0.2, 0.6, 0.4))[0]
        mats[2] = S._material(0, (0.3, -0.0, -0.7))[0]
    return S.SceneData(sc.camera, sc.spheres, mats, textures=sc.textures, name=f"negative_albedo_{specular}")


@pytest.mark.parametrize("specular", [True, False])
def test_f64_negative_albedo_matches_books_path(specular):
    scene = _negative_albedo_scene(specular)
    gpu, _, gpu_rays = _gpu_f64(scene)
    books, books_rays, _ = oracle.render(scene, oracle.BOOKS, threads=16)
    assert gpu_rays == books_rays
    assert (books[..., :3] < 0).any(), "the scene must produce negative radiance sums"
    _check(scene, gpu, books, f"negative albedo (specular={specular})")


# rrt_testing_f64_layout: bit 0 widened Sphere64 records, bit 1 the 1/r table, bit 2 the f32
# pre-test records beside widened ones
LAYOUTS = [0, 1, 2, 3, 5, 7]


@pytest.mark.parametrize("which", ["C2", "textured_specular"])
def test_f64_every_lds_layout_renders_the_same_bits(which, monkeypatch):
    """Each LDS layout the f64 kernel may stage a scene in (launch64_placed's fallbacks for scenes near
    the block's 64 KB) renders the automatic layout's bits, and those match BOOKS; with the f32
    sphere pre-test switched off (RRT_F64_PRETEST=0) too."""
    from rustraytrace_amd import _lib

    lib = _lib.load()
    scene = (rrt.config_scene("C2", image_width=64, samples_per_pixel=64) if which == "C2"
             else _textured_specular_scene(image_width=48, samples_per_pixel=64))
    ref, _, ref_rays = _gpu_f64(scene)
    books, books_rays, _ = oracle.render(scene, oracle.BOOKS, threads=16)
    assert ref_rays == books_rays
    _check(scene, ref, books, f"{which} automatic layout")
    ran = []
    try:
        for lay in LAYOUTS:
            lib.rrt_testing_f64_layout(lay)
            try:
                out, _, rays = _gpu_f64(scene)
            except rrt.RrtError:
                continue  # the forced layout exceeds the block's 64 KB for this scene
            assert rays == ref_rays and np.array_equal(out, ref), f"layout {lay} differs"
            ran.append(lay)
    finally:
        lib.rrt_testing_f64_layout(-1)
    print(f"{which}: layouts run {ran}")
    assert set(ran) >= ({0, 1, 2, 3} if which == "C2" else set(LAYOUTS))
    monkeypatch.setenv("RRT_F64_PRETEST", "0")
    out, _, rays = _gpu_f64(scene)
    assert rays == ref_rays and np.array_equal(out, ref), "pre-test off differs"


@pytest.mark.parametrize("size,rows", [((64, 256), None), ((None, None), (536, 544))])
def test_f64_textured_matches_books_with_libm_trig(size, rows):
    """C4 against the books path with the sphere UV's acos / atan2 from the host's libm (the
    reference's f64::acos / atan2; oracle diagnostic bit 0x800), not the fdlibm restatement the
    kernel shares with the default BOOKS mode: the channel and PPM-byte mismatches are reported and
    must stay inside the north star's bars (<= 1 ulp in the angle moves a texel index only at a
    boundary; tests/test_oracle.py counts none on C4)."""
    w, spp = size
    scene = rrt.config_scene("C4", **({} if w is None else dict(image_width=w, samples_per_pixel=spp)))
    gpu, _, gpu_rays = _gpu_f64(scene)
    books, books_rays, _ = oracle.render(scene, oracle.BOOKS | 0x800, rows=rows, threads=16)
    if rows is None:
        assert gpu_rays == books_rays
    else:
        gpu = gpu[rows[0]:rows[1]]
    diff = np.abs(gpu[..., :3] - books[..., :3]) / scene.spp
    print(f"C4 vs libm-trig BOOKS: {int((diff > 1e-12).sum())} of {diff.size} channels differ beyond 1e-12")
    _check(scene, gpu, books, "C4 vs BOOKS (libm acos / atan2)", bar="bytes")
