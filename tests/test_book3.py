"""Book 3 on the CPU: the_rest_of_your_life's MIS integrator
(the_rest_of_your_life/camera.rs:184-254, pdf.rs, onb.rs, quad.rs / sphere.rs pdf_value and random)
restated by the oracle in f64 (BOOKS, recursive, the reference's order) and f32 (TWIN, the
kernel's throughput form), checked against each other, against the kernel's tree (KBVH), and for
unbiasedness against the book-2 integrator on the same geometry. The GPU side is
tests/test_gpu_book3.py.

Parity note: the book-3 scene has no random layout; the sample streams are the backend's
(per-path xoshiro128+), so these are restatement checks, not reference vectors (parity unpinned, as for
books 1 and 2)."""
import copy

import numpy as np

import rustraytrace_amd as rrt
from oracle import oracle
from rustraytrace_amd.render import build_bvh


def test_cos_f32_accuracy():
    x = np.linspace(0.0, 2.0 * np.pi, 200001).astype(np.float32)  # phi = 2 pi r1 range
    got = oracle.cos_f32(x).astype(np.float64)
    assert np.max(np.abs(got - np.cos(x.astype(np.float64)))) < 2e-7
    assert oracle.cos_f32([0.0])[0] == 1.0
    s = oracle.sin_f32(x).astype(np.float64)
    assert np.max(np.abs(got * got + s * s - 1.0)) < 1e-6


def test_rest_of_your_life_scene_structure():
    sc = rrt.rest_of_your_life_scene()
    assert (sc.width, sc.height, sc.spp, sc.max_depth) == (600, 600, 100, 50)
    assert sc.flags == rrt._lib.FLAG_RAY_TIME | rrt._lib.FLAG_BOOK3
    assert len(sc.spheres) == 1 and len(sc.quads) == 5 + 1 + 6 and sc.media is None
    kinds = sc.materials["kind"]
    assert kinds[sc.spheres["material_index"][0]] == 2  # the glass sphere
    assert (kinds[sc.quads["material_index"]] == 4).sum() == 1  # one DiffuseLight(15) quad
    assert sc.lights["kind"].tolist() == [0, 1]
    assert sc.lights["a"][0, :3].tolist() == [343.0, 554.0, 332.0] and sc.lights["a"][1].tolist() == [190, 90, 190, 90]
    assert np.allclose(sc.camera["background"][0, :3], 0.0)
    # Camera::initialize rounds samples_per_pixel down to sqrt_spp^2 (camera.rs:115-117)
    for spp, eff in ((1, 1), (10, 9), (99, 81), (100, 100), (1000, 961)):
        assert rrt.rest_of_your_life_scene(dict(image_width=8, samples_per_pixel=spp)).spp == eff


def test_book3_books_vs_twin_statistical():
    sc = rrt.rest_of_your_life_scene(dict(image_width=40, samples_per_pixel=64, max_depth=10))
    t, rt, _ = oracle.render(sc, oracle.TWIN, threads=8)
    b, rb, _ = oracle.render(sc, oracle.BOOKS, threads=8)
    assert np.isfinite(t).all() and np.isfinite(b).all()
    assert abs(t[..., :3].mean() - b[..., :3].mean()) / b[..., :3].mean() < 0.01
    assert abs(rt - rb) / rb < 0.01


def test_book3_kbvh_agrees_with_books_tree():
    sc = rrt.rest_of_your_life_scene(dict(image_width=40, samples_per_pixel=16, max_depth=10))
    a, ra, _ = oracle.render(sc, oracle.TWIN, threads=8)
    nodes, order, info = build_bvh(sc)
    assert info["width"] == 2
    b, rb, _ = oracle.render_kbvh(sc, nodes, order, info, threads=8)
    assert np.array_equal(a, b)  # ray counts may differ at exact quad-edge ties (test_book2.py)


def test_mis_is_unbiased_against_the_book2_integrator():
    """The mixture-pdf estimator and book 2's cosine-scatter estimator converge to the same
    image. Book 2's DiffuseLight is two-sided, so the light is moved to 0.001 below the ceiling
    (no room behind it) in both the world and the light list."""
    sc = rrt.rest_of_your_life_scene(dict(image_width=24, samples_per_pixel=2048, max_depth=10))
    q = sc.quads.copy()
    li = np.where(sc.materials["kind"][q["material_index"]] == 4)[0][0]
    q[li]["q"][1] = 554.999
    lt = sc.lights.copy()
    lt[0]["a"][1] = 554.999
    sc.quads, sc.lights = q, lt
    mis, _, _ = oracle.render(sc, oracle.TWIN, threads=8)
    plain = copy.copy(sc)
    plain.flags, plain.lights = rrt._lib.FLAG_RAY_TIME, None
    ref, _, _ = oracle.render(plain, oracle.TWIN, threads=8)
    m, r = mis[..., :3].mean(), ref[..., :3].mean()
    assert abs(m - r) / r < 0.04  # the plain estimator's fireflies dominate this tolerance
