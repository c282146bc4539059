"""CPU tests pinning the oracle (oracle/rrt_oracle.cpp) before it is trusted as the parity
checker. The reference has no tests or golden vectors, so the oracle is pinned by:
  * analytic known-answer vectors for every restated primitive (sphere.rs, aabb.rs, vec3.rs,
    material.rs, color.rs, render_io.rs),
  * closed-form images (white furnace, sky-only),
  * agreement of its two independent modes (f64 BOOKS recursion vs f32 TWIN),
  * its independent restatement of gpu::build_in_one_weekend_scene vs the product's builder,
  * the committed golden fixtures (regression pin; tests/golden/make_golden.py).
"""
import glob
import hashlib
import math
import os

import numpy as np
import pytest

import rustraytrace_amd as rrt
from oracle import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
INF = float("inf")


# ---- Sphere::hit (sphere.rs:24-51) ------------------------------------------------------------
@pytest.mark.parametrize("f32", [0, 1])
def test_sphere_hit_front(f32):
    t, n, front = oracle.sphere_hit((0, 0, -5), 1.0, (0, 0, 0), (0, 0, -1), f32=f32)
    assert t == 4.0 and front and list(n) == [0.0, 0.0, 1.0]
    # unnormalised direction: t scales by 1/|d|
    t, n, front = oracle.sphere_hit((0, 0, -5), 1.0, (0, 0, 0), (0, 0, -2), f32=f32)
    assert t == 2.0


@pytest.mark.parametrize("f32", [0, 1])
def test_sphere_hit_inside_uses_far_root(f32):
    t, n, front = oracle.sphere_hit((0, 0, -5), 1.0, (0, 0, -5), (0, 0, -1), f32=f32)
    assert t == 1.0 and not front and list(n) == [0.0, 0.0, 1.0]  # normal flipped against the ray


@pytest.mark.parametrize("f32", [0, 1])
def test_sphere_hit_tangent_miss_behind(f32):
    t, _, _ = oracle.sphere_hit((0, 1, -5), 1.0, (0, 0, 0), (0, 0, -1), f32=f32)  # disc == 0 accepted
    assert t == 5.0
    assert oracle.sphere_hit((0, 2, -5), 1.0, (0, 0, 0), (0, 0, -1), f32=f32) is None  # disc < 0
    assert oracle.sphere_hit((0, 0, 5), 1.0, (0, 0, 0), (0, 0, -1), f32=f32) is None  # both roots behind


@pytest.mark.parametrize("f32", [0, 1])
def test_sphere_hit_open_interval(f32):
    # interval.rs:30-32 surrounds is strict on both ends
    assert oracle.sphere_hit((0, 0, -5), 1.0, (0, 0, 0), (0, 0, -1), tmax=4.0, f32=f32) is None
    t, _, _ = oracle.sphere_hit((0, 0, -5), 1.0, (0, 0, 0), (0, 0, -1), tmin=4.0, f32=f32)
    assert t == 6.0
    # negative radius clamps to 0 (sphere.rs:17): only a ray through the centre point hits
    assert oracle.sphere_hit((0, 0, -5), -1.0, (0, 0, 0), (0, 1, -1), f32=f32) is None


# ---- Aabb::hit (aabb.rs:52-85) incl. 1/0 = inf and 0*inf = NaN branches ------------------------
@pytest.mark.parametrize("f32", [0, 1])
def test_aabb_axis_parallel(f32):
    lo, hi = (-1, -1, -1), (1, 1, 1)
    assert oracle.aabb_hit(lo, hi, (0, 0, -5), (0, 0, 1), f32=f32)
    assert not oracle.aabb_hit(lo, hi, (0, 0, -5), (0, 0, -1), f32=f32)
    assert oracle.aabb_hit(lo, hi, (0.5, 0, -5), (0, 0, 1), f32=f32)  # dx = 0, inside the x slab
    assert not oracle.aabb_hit(lo, hi, (2, 0, -5), (0, 0, 1), f32=f32)  # dx = 0, outside
    assert not oracle.aabb_hit(lo, hi, (0, 0, -5), (0, 0, 1), tmax=3.0, f32=f32)  # ends before the box
    assert not oracle.aabb_hit(lo, hi, (0, 0, -5), (0, 0, 1), tmax=4.0, f32=f32)  # max <= min rejects


@pytest.mark.parametrize("f32", [0, 1])
def test_aabb_on_plane_nan_branch(f32):
    lo, hi = (-1, -1, -1), (1, 1, 1)
    # origin exactly on the x = lo plane with dx = +0: t0 = 0*inf = NaN, t1 = +inf -> min = inf: reject
    assert not oracle.aabb_hit(lo, hi, (-1, 0, -5), (0.0, 0, 1), f32=f32)
    # dx = -0: t0 = NaN, t1 = -inf -> neither bound moves: accept (books branch order)
    assert oracle.aabb_hit(lo, hi, (-1, 0, -5), (-0.0, 0, 1), f32=f32)
    # on the x = hi plane with dx = +0: t0 = -inf, t1 = NaN -> max = -inf: reject
    assert not oracle.aabb_hit(lo, hi, (1, 0, -5), (0.0, 0, 1), f32=f32)


# ---- vec3.rs reflect/refract, material.rs Schlick ---------------------------------------------
@pytest.mark.parametrize("f32", [0, 1])
def test_reflect_refract_schlick(f32):
    refl, refr, sch = oracle.reflect_refract((1, -1, 0), (0, 1, 0), 1 / 1.5, 1.0, 1.5, f32=f32)
    assert list(refl) == [1.0, 1.0, 0.0]
    assert sch == pytest.approx(0.04, rel=1e-6)  # r0 = ((1-1.5)/(1+1.5))^2 at normal incidence
    _, refr, sch = oracle.reflect_refract((0, -1, 0), (0, 1, 0), 1 / 1.5, 0.0, 1.5, f32=f32)
    assert list(refr) == [0.0, -1.0, 0.0] and sch == 1.0  # straight through; grazing -> total
    s = math.sqrt(0.5)
    _, refr, _ = oracle.reflect_refract((s, -s, 0), (0, 1, 0), 1 / 1.5, 0.5, 1.0, f32=f32)
    tol = 1e-6 if f32 else 1e-14
    assert refr[0] == pytest.approx(s / 1.5, abs=tol)  # Snell: sin t = sin i / 1.5
    assert refr[1] == pytest.approx(-math.sqrt(1 - 0.5 / 2.25), abs=tol)
    _, _, sch = oracle.reflect_refract((0, -1, 0), (0, 1, 0), 1.0, 0.5, 1.0, f32=f32)
    assert sch == 0.5 ** 5  # r0 = 0 -> (1 - cos)^5 via x*((x*x)*(x*x))


# ---- quantisers: color.rs (f64) and render_io.rs (f32) ----------------------------------------
def test_write_color_edges():
    assert list(oracle.write_color([0.0, 0.25, 1.0])) == [0, 128, 255]
    assert list(oracle.write_color([-1.0, float("nan"), INF])) == [0, 0, 255]  # inf -> 255 in books


def test_render_io_quantiser_edges_match_product():
    spp = 4
    vals = np.array([0.0, 0.25, 1.0, 0.999 ** 2, INF, -INF, float("nan"), -0.5, 1e30, 4.0, 0.01, 3.99])
    acc = np.zeros((len(vals), 4), np.float32)
    acc[:, 0] = vals * spp
    acc[:, 1] = vals
    acc[:, 2] = 1.0
    ref = oracle.quantize_render_io(acc, spp)
    got = rrt.quantize_accum(len(vals), 1, acc, spp).reshape(-1, 3)
    assert np.array_equal(ref, got)
    assert list(ref[:7, 0]) == [0, 128, 255, 255, 0, 0, 0]  # non-finite -> 0 in render_io (unlike color.rs)
    ppm = rrt.format_ppm_from_accum(len(vals), 1, acc, spp)
    lines = ppm.decode().splitlines()
    assert lines[:3] == ["P3", f"{len(vals)} 1", "255"]
    assert [list(map(int, l.split())) for l in lines[3:]] == ref.tolist()


def test_books_quantiser_matches_write_color():
    # product rrt_quantize_accum_books == the oracle's color.rs:6-32 restatement, per channel:
    # (1/spp) * sum in f64, then write_color (inf -> 255, NaN -> 0)
    spp = 7
    rng = np.random.default_rng(5)
    sums = np.concatenate([
        np.array([0.0, 0.25, 1.0, 0.999 ** 2, INF, -INF, float("nan"), -0.5, 1e30, 4.0, 0.01, 3.99]) * spp,
        rng.uniform(0, 1.2 * spp, 500), rng.uniform(0, 1e-4, 100)]).astype(np.float32)
    n = len(sums) // 3
    acc = np.zeros((n, 4), np.float32)
    acc[:, :3] = sums[: 3 * n].reshape(n, 3)
    got = rrt.quantize_accum_books(n, 1, acc, spp).reshape(-1, 3)
    scale = 1.0 / spp
    want = np.array([oracle.write_color(scale * acc[i, :3].astype(np.float64)) for i in range(n)])
    assert np.array_equal(got, want)
    # rows: (0, .25, 1), (.998, inf, -inf), (nan, -.5, 1e30): inf -> 255 in color.rs (render_io: 0)
    assert got[:3].tolist() == [[0, 128, 255], [255, 255, 0], [0, 0, 255]]
    with pytest.raises(rrt.RrtError):
        rrt.quantize_accum_books(1, 1, acc[:1], 0)


# ---- camera / image height (camera.rs:102-150, gpu/mod.rs:174-198) ----------------------------
@pytest.mark.parametrize("w,h", [(400, 225), (1920, 1080), (3840, 2160), (64, 36), (1, 1)])
def test_image_height(w, h):
    cam = rrt.make_camera(aspect_ratio=16 / 9, image_width=w)
    assert int(cam["params_f"][0, 2]) == h


def test_camera_matches_gpu_mod_rs_math():
    W, H = 1920, 1080
    cam = rrt.build_in_one_weekend_scene(dict(image_width=W, samples_per_pixel=512, max_depth=100)).camera
    lookfrom, lookat, vup = np.array([13.0, 2, 3]), np.zeros(3), np.array([0.0, 1, 0])
    h = math.tan(math.radians(20.0) / 2)  # degrees * PI / 180
    vh = 2.0 * h * 10.0
    vw = vh * (W / H)
    w = (lookfrom - lookat) / np.linalg.norm(lookfrom - lookat)
    u = np.cross(vup, w)
    u = u / np.linalg.norm(u)
    v = np.cross(w, u)
    du, dv = u * vw / W, v * -vh / H
    p00 = lookfrom - w * 10.0 - u * vw / 2 - v * -vh / 2 + (du + dv) * 0.5
    np.testing.assert_allclose(cam["pixel00"][0, :3], p00, rtol=1e-6)
    np.testing.assert_allclose(cam["pixel_delta_u"][0, :3], du, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(cam["pixel_delta_v"][0, :3], dv, rtol=1e-6, atol=1e-9)
    assert cam["params_f"][0, 0] == np.float32(10.0 * math.tan(math.radians(0.3)))
    assert list(cam["params_u"][0]) == [100, cam["params_u"][0, 1], 486, 0]


# ---- RNG stream and f32 transcendentals -------------------------------------------------------
def _splitmix64(z):
    m = (1 << 64) - 1
    z = (z + 0x9E3779B97F4A7C15) & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def _xoshiro128p_stream(seed, pixel, sample, count):
    """Independent restatement of the per-path stream: xoshiro128+ (Blackman & Vigna's
    reference algorithm) seeded with (z, key | 2^32), key = splitmix64((seed << 32) ^ pixel),
    z = splitmix64(key + sample)."""
    m = 0xFFFFFFFF
    key = _splitmix64((seed << 32) ^ pixel)
    z = _splitmix64((key + sample) & ((1 << 64) - 1))
    a, b, c, d = z & m, z >> 32, key & m, (key >> 32) | 1
    out = []
    for _ in range(count):
        out.append((a + d) & m)
        t = (b << 9) & m
        c ^= a
        d ^= b
        b ^= c
        a ^= d
        c ^= t
        d = ((d << 11) | (d >> 21)) & m
    return np.array(out, dtype=np.uint32)


def test_path_stream_known_answer():
    for seed, pixel, sample in [(0x1234, 77, 5), (0, 0, 0), (0xFFFFFFFF, 2073599, 511)]:
        assert np.array_equal(oracle.path_stream(seed, pixel, sample, 64), _xoshiro128p_stream(seed, pixel, sample, 64))


def test_path_stream_deterministic_and_uniform():
    a = oracle.path_stream(0x1234, 77, 5, 4096)
    assert np.array_equal(a, oracle.path_stream(0x1234, 77, 5, 4096))
    assert not np.array_equal(a, oracle.path_stream(0x1234, 77, 6, 4096))
    assert not np.array_equal(a, oracle.path_stream(0x1234, 78, 5, 4096))
    u = (oracle.path_stream(7, 1, 2, 200000) >> 8) / 2.0 ** 24
    assert abs(u.mean() - 0.5) < 0.005 and u.min() >= 0.0 and u.max() < 1.0
    assert abs(np.histogram(u, bins=10)[0] / len(u) - 0.1).max() < 0.005


def test_cephes_acos_atan2_accuracy():
    for x in np.linspace(-1, 1, 2001, dtype=np.float32):
        a, _ = oracle.acos_atan2_f32(float(x), 0.5)
        assert abs(a - math.acos(float(x))) < 4e-7
    for ang in np.linspace(-math.pi + 1e-3, math.pi - 1e-3, 997):
        y, x = math.sin(ang), math.cos(ang)
        _, t = oracle.acos_atan2_f32(np.float32(x), np.float32(y))
        assert abs(t - math.atan2(np.float32(y), np.float32(x))) < 4e-7
    assert oracle.acos_atan2_f32(0.0, 1.0)[1] == pytest.approx(math.pi / 2)
    assert oracle.acos_atan2_f32(0.0, -1.0)[1] == pytest.approx(-math.pi / 2)


# ---- scene builder: product vs independent restatement ----------------------------------------
@pytest.mark.parametrize("grid_half,n", [(11, 486), (50, 10001)])
def test_rtow_scene_restatements_agree(grid_half, n):
    prod = rrt.build_in_one_weekend_scene(seed=0x5EED_1234, grid_half=grid_half)
    ref = oracle.rtow_scene(0x5EED_1234, grid_half)
    assert len(prod.spheres) == n
    assert np.array_equal(prod.spheres["center_radius"], ref["center_radius"])
    assert np.array_equal(prod.spheres["material_index"], ref["material_index"])
    assert np.array_equal(prod.materials["albedo_fuzz"], ref["albedo_fuzz"])
    assert np.array_equal(prod.materials["kind"], ref["kind"])
    assert np.array_equal(prod.materials["ref_idx"], ref["ref_idx"])
    assert int(prod.camera["params_u"][0, 1]) == ref["sample_seed"]


def test_rtow_scene_material_mix():
    s = rrt.build_in_one_weekend_scene()
    kind = s.materials["kind"]
    assert set(np.unique(kind)) == {0, 1, 2}
    small = s.spheres["center_radius"][1:-3]
    assert np.all(small[:, 3] == np.float32(0.2)) and np.all(small[:, 1] == np.float32(0.2))
    d = np.hypot(small[:, 0] - 4.0, small[:, 2])
    assert np.all(d > 0.9 - 1e-6)
    metal = s.materials[kind == 1][:-1]
    assert np.all(metal["albedo_fuzz"][:, :3] >= 0.5) and np.all(metal["albedo_fuzz"][:, 3] < 0.5)


# ---- closed-form images -----------------------------------------------------------------------
def _white_furnace(n_spheres=1, depth=10):
    from rustraytrace_amd.scenes import SceneData, _material, _sphere, make_camera

    mats = _material(0, (1.0, 1.0, 1.0))
    sph = _sphere((0.0, 0.0, -1.0), 0.5, 0)
    cam = make_camera(aspect_ratio=16 / 9, image_width=32, samples_per_pixel=8, max_depth=depth,
                      background=(1.0, 1.0, 1.0), seed=99, n_spheres=1)
    return SceneData(cam, sph, mats, name="white_furnace")


@pytest.mark.parametrize("mode", [oracle.TWIN, oracle.BOOKS])
def test_white_furnace_exact(mode):
    # albedo-1 convex sphere under background 1: every path returns exactly 1 (no RR before bounce 5,
    # a convex sphere is left after one bounce), so every pixel sums to exactly spp.
    sc = _white_furnace()
    acc, rays, _ = oracle.render(sc, mode)
    assert np.all(acc[..., :3] == sc.spp)
    assert rays >= sc.width * sc.height * sc.spp


def test_sky_only_twin_books_agree():
    from rustraytrace_amd.scenes import SceneData, make_camera

    cam = make_camera(aspect_ratio=16 / 9, image_width=40, samples_per_pixel=4, max_depth=5, seed=3,
                      defocus_angle=2.0, lookfrom=(0, 1, 0), lookat=(0, 1, -1))
    sc = SceneData(cam, np.zeros(0, rrt._lib.SPHERE_DTYPE), np.zeros(0, rrt._lib.MATERIAL_DTYPE))
    t, rt, _ = oracle.render(sc, oracle.TWIN)
    b, rb, _ = oracle.render(sc, oracle.BOOKS)
    assert rt == rb == 40 * 22 * 4
    np.testing.assert_allclose(t[..., :3], b[..., :3], rtol=2e-6)


# The f32 modes against the f64 books path (BOOKS) on the same scene and random stream.
# Individual paths still diverge where an f32/f64 rounding flips a discrete decision (a
# rejection-loop acceptance, a dielectric's reflect/refract draw), so the per-channel bar is a
# fraction; the means and the ray counts must agree to 0.1 %. Without exit_skip (diagnostic
# mode bit 0x200) f32 bounces re-hit the surface they leave: C2 +0.68 % rays / -0.20 %
# radiance, C5 +1.9 % / -0.55 % — both bounds below fail on that arithmetic.
BOOKS_BOUNDS = {  # per-channel |twin - books| / spp <= 1e-4: minimum fraction (64x36x64, measured 100/93/100/87 %)
    "C1": 0.995, "C2": 0.90, "C4": 0.995, "C5": 0.84,
}


def books_agreement(scene, twin, twin_rays, books, books_rays):
    """(ray-count ratio - 1, mean-radiance ratio - 1, fraction of channels within 1e-4, u8-equal fraction)."""
    S = scene.spp
    per_chan = np.abs(twin[..., :3] - books[..., :3]) / S
    q = lambda a: rrt.quantize_accum(scene.width, scene.height, np.ascontiguousarray(a, dtype=np.float32), S)
    return (twin_rays / books_rays - 1.0, twin[..., :3].mean() / books[..., :3].mean() - 1.0,
            float((per_chan <= 1e-4).mean()), float((q(twin) == q(books)).mean()))


@pytest.mark.parametrize("cfg", sorted(BOOKS_BOUNDS))
def test_books_vs_twin_statistical(cfg):
    sc = rrt.config_scene(cfg, image_width=64, samples_per_pixel=64)
    t, rt, _ = oracle.render(sc, oracle.TWIN, threads=8)
    b, rb, _ = oracle.render(sc, oracle.BOOKS, threads=8)
    drays, drad, within, _ = books_agreement(sc, t, rt, b, rb)
    assert abs(drays) < 1e-3, f"{cfg}: f32 traces {drays:+.4%} rays against the f64 books path"
    assert abs(drad) < 1e-3, f"{cfg}: mean radiance {drad:+.4%} against the f64 books path"
    assert within >= BOOKS_BOUNDS[cfg], f"{cfg}: {within:.3f} of channels within 1e-4"


def test_exit_skip_removes_the_f32_self_intersection_bias():
    """The mechanism, pinned: the same C2 frame without exit_skip (mode bit 0x200) re-hits the
    r = 1000 ground sphere it leaves (grazing Lambertian bounces), tracing > 0.5 % extra rays
    that end trapped inside it (darker); with exit_skip the f32 path tracks the f64 one."""
    sc = rrt.config_scene("C2", image_width=64, samples_per_pixel=32)
    b, rb, _ = oracle.render(sc, oracle.BOOKS, threads=8)
    n, rn, _ = oracle.render(sc, 0x200, threads=8)
    t, rt, _ = oracle.render(sc, oracle.TWIN, threads=8)
    assert rn / rb - 1.0 > 5e-3 and n[..., :3].mean() / b[..., :3].mean() - 1.0 < -1e-3
    assert abs(rt / rb - 1.0) < 1e-3


def test_books_vs_twin_book2_and_book3():
    """exit_skip also removes final_scene's f32 bias (|p| ~ 1e3: +4.4 % rays / -1.9 % radiance
    without it) and the quad scenes' re-hits of the face a ray leaves."""
    cases = [rrt.next_week_scene(n, overrides=dict(image_width=48, samples_per_pixel=16, max_depth=50))
             for n in (1, 4, 7, 9)]
    cases.append(rrt.rest_of_your_life_scene(overrides=dict(image_width=48, samples_per_pixel=16, max_depth=50)))
    for sc in cases:
        t, rt, _ = oracle.render(sc, oracle.TWIN, threads=8)
        b, rb, _ = oracle.render(sc, oracle.BOOKS, threads=8)
        drays, drad, _, _ = books_agreement(sc, t, rt, b, rb)
        assert abs(drays) < 2e-3 and abs(drad) < 5e-3, (sc.name, drays, drad)


# ---- golden fixtures (regression pin of the oracle) -------------------------------------------
GOLDENS = sorted(glob.glob(os.path.join(GOLDEN, "*.npz")))


def _golden_scene(name):
    import sys

    sys.path.insert(0, GOLDEN)
    from make_golden import CASES, scene_sha

    cfg, kw = CASES[name]
    sc = rrt.config_scene(cfg, **kw)
    return sc, scene_sha(sc)


@pytest.mark.parametrize("path", GOLDENS, ids=[os.path.basename(p) for p in GOLDENS])
def test_oracle_reproduces_golden(path):
    name = os.path.basename(path)[:-4]
    z = np.load(path, allow_pickle=False)
    sc, sha = _golden_scene(name)
    assert sha == str(z["scene_sha256"]), "scene builder output changed"
    acc, rays, _ = oracle.render(sc, oracle.TWIN, threads=4)
    assert np.array_equal(acc.astype(np.float32), z["accum"])
    assert rays == int(z["rays"])
    ppm = rrt.format_ppm_from_accum(sc.width, sc.height, z["accum"], sc.spp)
    assert ppm == z["ppm"].tobytes()
    bacc, brays, _ = oracle.render(sc, oracle.BOOKS, threads=4)
    assert np.array_equal(bacc, z["books_accum"]) and brays == int(z["books_rays"])


def test_goldens_present():
    assert len(GOLDENS) >= 5


# ---- KBVH mode (the kernel's tree, the kernel's order) vs the independent books tree ------------
@pytest.mark.parametrize("cfg,kw", [("C1", dict(image_width=48, samples_per_pixel=4)),
                                    ("C2", dict(image_width=48, samples_per_pixel=4)),
                                    ("C4", dict(image_width=48, samples_per_pixel=4)),
                                    ("C5", dict(image_width=32, samples_per_pixel=2))])
@pytest.mark.parametrize("width", [2, 4])
def test_kbvh_mode_agrees_with_books_tree(cfg, kw, width):
    from rustraytrace_amd.render import build_bvh

    sc = rrt.config_scene(cfg, **kw)
    a, ra, _ = oracle.render(sc, oracle.TWIN, threads=4)
    nodes, order, info = build_bvh(sc, width=width)
    assert info["width"] == width and sorted(order.tolist()) == list(range(len(sc.spheres)))
    b, rb, _ = oracle.render_kbvh(sc, nodes, order, info, threads=4)
    assert np.array_equal(a, b) and ra == rb


# ---- axis-parallel rays (a zero direction component) -------------------------------------------
def axis_parallel_scene(width=16, spp=4):
    """Every camera ray has d.x == 0 exactly (pixel00.x = origin.x, no x in the pixel deltas, no
    defocus) and runs through a black sphere whose box straddles x = 0 (lo.x < 0 < o.x): with
    1/d.x = inf, inf * lo.x - inf * o.x is -inf and inf * hi.x - inf * o.x NaN, which rejected
    the box before ray_consts clamped 1/d to +-2^64. Expected image: all 0 (every ray hits)."""
    from rustraytrace_amd.scenes import _material, _sphere, make_camera

    cam = make_camera(image_width=width, samples_per_pixel=spp, max_depth=4, background=(1.0, 1.0, 1.0), n_spheres=1)
    o = np.array([0.5, 0.3, 3.0, 0.0], dtype=np.float32)
    cam["origin"][0] = o
    cam["pixel00"][0] = o + np.array([0.0, -0.004, -1.0, 0.0], dtype=np.float32)
    cam["pixel_delta_u"][0] = (0.0, 0.0005, 0.0, 0.0)
    cam["pixel_delta_v"][0] = (0.0, -0.0005, 0.0, 0.0)
    cam["params_f"][0, 0] = 0.0
    sph = _sphere((0.2, 0.3, -1.0), 0.5, 0)
    return rrt.SceneData(cam, sph, _material(0, (0.0, 0.0, 0.0)), name="axis_parallel")


def test_axis_parallel_rays_hit_through_straddling_boxes():
    from rustraytrace_amd.render import build_bvh

    sc = axis_parallel_scene()
    twin, _, _ = oracle.render(sc, oracle.TWIN)
    nodes, order, info = build_bvh(sc)
    kb, _, _ = oracle.render_kbvh(sc, nodes, order, info)
    assert np.all(twin[..., :3] == 0) and np.array_equal(twin, kb)


def test_bvh2_node_layouts_hold_the_same_tree(monkeypatch):
    """RTOW fits the LDS budget: 80-B sign-ordered nodes; C5's 10k spheres do not: 32-B f16 nodes,
    in the global-memory shape (rrt_host.cpp scene_bvh: single-primitive leaves). Forcing global
    memory on RTOW with the LDS shape's leaves (RRT_MAX_LEAF_GLOBAL=3) gives the 32-B layout of the
    same tree: same links, and every f16 box holds its f32 box (rounded outward, no subnormal
    planes); a never-hit child stays never-hit."""
    from rustraytrace_amd.render import build_bvh, decode_bvh2

    sc = rrt.rtow(image_width=32, samples_per_pixel=2)
    nodes, order, info = build_bvh(sc)
    assert info["node_stride"] == 80 and nodes.size == 80 * info["n_nodes"]
    c5 = rrt.config_scene("C5", image_width=32, samples_per_pixel=2)
    assert build_bvh(c5)[2]["node_stride"] == 32
    monkeypatch.setenv("RRT_SCENE_IN_LDS", "0")
    assert build_bvh(sc)[2]["max_leaf_size"] == 1 and info["max_leaf_size"] == 3  # the global shape
    monkeypatch.setenv("RRT_MAX_LEAF_GLOBAL", "3")
    nodes_g, order_g, info_g = build_bvh(sc)
    assert info_g["node_stride"] == 32 and nodes_g.size == 32 * info_g["n_nodes"] and np.array_equal(order, order_g)
    lo, hi, first, count = decode_bvh2(nodes, 80)
    lo_h, hi_h, first_h, count_h = decode_bvh2(nodes_g, 32)
    assert np.array_equal(first, first_h) and np.array_equal(count, count_h)
    live = lo[..., 0] < 1e29
    assert np.all(lo_h[live] <= lo[live]) and np.all(hi_h[live] >= hi[live])
    assert np.all(hi_h[live] - lo_h[live] <= (hi[live] - lo[live]) * 1.01 + 2e-2)  # ~f16 ulps at RTOW scale
    planes = np.concatenate([lo_h.ravel(), hi_h.ravel()])
    assert not np.any((planes != 0) & (np.abs(planes) < 2.0 ** -14))  # no f16 subnormals
    assert np.all(lo_h[~live] == 65504.0) and np.all(hi_h[~live] == 65504.0)


@pytest.mark.parametrize("S,chunk", [(20, 8), (512, 64), (64, 64), (65, 64), (7, 0), (300, 128), (256, 128),
                                     (600, 256), (513, 256), (512, 256), (256, 256), (257, 256), (64, 256), (65, 256)])
def test_accum_chunk_schedule(S, chunk):
    """The TWIN accum groups samples as rrt_accum_chunk documents (include/rrt_hip.h): (S-1)/K
    chunks of K, then chunks of max(1, K/4), or max(1, K/8) when S <= chunk / 4 (ABI v11); in-order f32 sums per chunk, chunks added in order."""
    sc = rrt.config_scene("C1", image_width=8, samples_per_pixel=S, max_depth=4)
    got, _, _ = oracle.render(sc, oracle.TWIN, chunk=chunk)
    per = [oracle.render(sc, oracle.TWIN, samples=(s, s + 1))[0][..., :3].astype(np.float32)
           for s in range(S)]
    K = chunk if chunk else S  # the frame's chunk: halved while S <= 2K, down to chunk / 4
    while chunk and K > max(1, chunk // 4) and S <= 2 * K:
        K //= 2
    k = max(1, K // (8 if S <= chunk // 4 else 4)) if chunk else S
    nb = (S - 1) // K if chunk and S > K else 0
    bounds, c0 = [], 0
    while c0 < S:
        step = K if c0 < nb * K else k
        bounds.append((c0, min(S, c0 + step)))
        c0 += step
    total = None
    for a, b in bounds:
        cs = per[a].copy()
        for s in range(a + 1, b):
            cs = cs + per[s]
        total = cs if total is None else total + cs
    assert np.array_equal(got[..., :3].astype(np.float32), total) and np.all(got[..., 3] == S)


def test_fdlibm_acos_atan2_within_one_ulp_of_libm():
    """BOOKS' f64 acos / atan2 (the earth texture's get_sphere_uv, the_next_week/sphere.rs:46-52)
    restate fdlibm's algorithms, shared op for op with the f64 kernel (rrt_books64.hip). The
    reference calls the platform libm through Rust's f64::acos / atan2: the restatement stays
    within 1 ulp of glibc's over the unit sphere's normals and a wide atan2 range."""
    rng = np.random.default_rng(7)
    x = np.concatenate([rng.uniform(-1, 1, 200_000), rng.uniform(-1e-3, 1e-3, 2000),
                        [-1.0, 1.0, 0.0, -0.0, -0.5, 0.5, 0.4375, -0.4375, 1 - 2**-53]])
    y = rng.standard_normal(x.size) * np.exp(rng.uniform(-8, 8, x.size))
    a, b = oracle.acos_atan2_f64(x, y)

    def ulps(u, v):
        return np.abs(u.view(np.int64) - v.view(np.int64))

    assert ulps(a, np.arccos(x)).max() <= 1
    assert ulps(b, np.arctan2(y, x)).max() <= 1
    assert (a == np.arccos(x)).mean() > 0.9 and (b == np.arctan2(y, x)).mean() > 0.75
    # exact special values of fdlibm
    sa, sb = oracle.acos_atan2_f64(np.array([1.0, -1.0, 0.0]), np.array([0.0, 0.0, 1.0]))
    assert sa[0] == 0.0 and sa[1] == np.pi and sb[0] == 0.0 and sb[1] == np.pi and sb[2] == np.pi / 2


def test_books_libm_trig_changes_no_c4_pixel():
    """BOOKS computes the sphere UV's acos / atan2 with fdlibm's algorithms (shared op for op with
    the f64 kernel); the reference calls the platform libm. Diagnostic bit 0x800 switches BOOKS to
    this host's libm: on C4 (the textured BASELINE config) no channel, ray count or PPM byte
    changes, at a reduced frame and on full-size rows at the full 1024 spp (a <= 1-ulp angle moves
    the texel index only when u * width sits on an integer)."""
    for kw, rows in [(dict(image_width=320, samples_per_pixel=64), None), ({}, (536, 544))]:
        scene = rrt.config_scene("C4", **kw)
        a, ra, _ = oracle.render(scene, oracle.BOOKS, rows=rows, threads=8)
        b, rb, _ = oracle.render(scene, oracle.BOOKS | 0x800, rows=rows, threads=8)
        assert ra == rb
        assert np.array_equal(a, b)
        h = a.shape[0]
        assert np.array_equal(rrt.quantize_accum_books_f64(scene.width, h, a, scene.spp),
                              rrt.quantize_accum_books_f64(scene.width, h, b, scene.spp))
