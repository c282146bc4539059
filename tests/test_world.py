"""The books' scene API (rustraytrace_amd.world) and the object-graph flattener behind it
(rrt_flatten_scene): Translate / RotateY composition against numpy, shared objects,
media boundaries, error handling, and the books' own scenes rebuilt through the API equal to the
C++ scene builders — same primitives, same materials, same oracle image."""
import numpy as np
import pytest

import rustraytrace_amd as rrt
from oracle import oracle
from rustraytrace_amd import world as W


def cornell(smoke: bool):
    """the_next_week/mod.rs:359-410 (cornell_box) and 432-501 (cornell_smoke), as the book writes them."""
    red, white = W.Lambertian((0.65, 0.05, 0.05)), W.Lambertian((0.73, 0.73, 0.73))
    green, light = W.Lambertian((0.12, 0.45, 0.15)), W.DiffuseLight((7.0,) * 3 if smoke else (15.0,) * 3)
    w = W.HittableList()
    w.add(W.Quad((555, 0, 0), (0, 555, 0), (0, 0, 555), green))
    w.add(W.Quad((0, 0, 0), (0, 555, 0), (0, 0, 555), red))
    if smoke:
        w.add(W.Quad((113, 554, 127), (330, 0, 0), (0, 0, 305), light))
        w.add(W.Quad((0, 555, 0), (555, 0, 0), (0, 0, 555), white))
        w.add(W.Quad((0, 0, 0), (555, 0, 0), (0, 0, 555), white))
    else:
        w.add(W.Quad((343, 554, 332), (-130, 0, 0), (0, 0, -105), light))
        w.add(W.Quad((0, 0, 0), (555, 0, 0), (0, 0, 555), white))
        w.add(W.Quad((555, 555, 555), (-555, 0, 0), (0, 0, -555), white))
    w.add(W.Quad((0, 0, 555), (555, 0, 0), (0, 555, 0), white))
    box1 = W.Translate(W.RotateY(W.make_box((0, 0, 0), (165, 330, 165), white), 15.0), (265, 0, 295))
    box2 = W.Translate(W.RotateY(W.make_box((0, 0, 0), (165, 165, 165), white), -18.0), (130, 0, 65))
    if smoke:
        w.add(W.ConstantMedium(box1, 0.01, (0.0, 0.0, 0.0)))
        w.add(W.ConstantMedium(box2, 0.01, (1.0, 1.0, 1.0)))
    else:
        w.add(box1)
        w.add(box2)
    cam = W.Camera(aspect_ratio=1.0, image_width=600, samples_per_pixel=200, max_depth=50, background=(0, 0, 0),
                   vfov=40.0, lookfrom=(278, 278, -800), lookat=(278, 278, 0))
    return w, cam


def mats_of(sc, idx):
    return sc.materials[idx]


@pytest.mark.parametrize("smoke", [False, True])
def test_api_cornell_matches_the_scene_builder(smoke):
    ref = rrt.next_week_scene(8 if smoke else 7)
    w, cam = cornell(smoke)
    sc = W.build(w, cam, seed=int(ref.camera["params_u"][0, 1]))
    for f in ("q", "u", "v"):
        assert np.array_equal(sc.quads[f], ref.quads[f])
    assert np.array_equal(mats_of(sc, sc.quads["material_index"]), mats_of(ref, ref.quads["material_index"]))
    assert np.array_equal(sc.camera, ref.camera) and sc.flags == ref.flags
    if smoke:
        for f in ("boundary_kind", "first", "count", "density"):
            assert np.array_equal(sc.media[f], ref.media[f])
        assert np.array_equal(mats_of(sc, sc.media["material_index"]), mats_of(ref, ref.media["material_index"]))
        for f in ("q", "u", "v"):
            assert np.array_equal(sc.boundary_quads[f], ref.boundary_quads[f])
    else:
        assert sc.media is None
    # the same frame from both descriptions
    kw = dict(image_width=32)
    small = W.build(w, W.Camera(**{**cam.__dict__, "image_width": 32, "samples_per_pixel": 4, "max_depth": 8}),
                    seed=int(ref.camera["params_u"][0, 1]))
    small_ref = rrt.next_week_scene(8 if smoke else 7, dict(kw, samples_per_pixel=4, max_depth=8))
    a, ra, _ = oracle.render(small, oracle.TWIN, threads=8)
    b, rb, _ = oracle.render(small_ref, oracle.TWIN, threads=8)
    assert np.array_equal(a, b) and ra == rb


def test_nested_transforms_compose_like_the_reference():
    """RotateY(Translate(RotateY(x, 30), t), -75): each point goes through the reference's
    per-ray transforms' inverse, i.e. the forward maps in order; checked against numpy."""
    mat = W.Lambertian((0.5, 0.5, 0.5))
    s = W.Sphere.moving((1.0, 2.0, 3.0), (1.5, 2.0, 2.0), 0.5, mat)
    q = W.Quad((0.25, -1.0, 0.5), (2.0, 0.0, 0.0), (0.0, 1.0, 1.0), mat)
    inner = W.HittableList([s, q])
    obj = W.RotateY(W.Translate(W.RotateY(inner, 30.0), (10.0, -2.0, 5.0)), -75.0)
    spheres, motion, quads, _, _, _, _, _ = W.flatten(W.HittableList([obj]))

    def rot(deg):
        t = np.radians(deg)
        return np.array([[np.cos(t), 0, np.sin(t)], [0, 1, 0], [-np.sin(t), 0, np.cos(t)]])

    def point(p):
        return rot(-75.0) @ (rot(30.0) @ np.asarray(p, float) + np.array([10.0, -2.0, 5.0]))

    def vec(v):
        return rot(-75.0) @ rot(30.0) @ np.asarray(v, float)

    assert np.allclose(spheres["center_radius"][0, :3], point((1, 2, 3)), atol=1e-5)
    assert spheres["center_radius"][0, 3] == 0.5
    assert np.allclose(motion[0, :3], vec((0.5, 0.0, -1.0)), atol=1e-5)
    assert np.allclose(quads["q"][0, :3], point((0.25, -1.0, 0.5)), atol=1e-5)
    assert np.allclose(quads["u"][0, :3], vec((2, 0, 0)), atol=1e-5)
    assert np.allclose(quads["v"][0, :3], vec((0, 1, 1)), atol=1e-5)


def test_shared_objects_flatten_once_per_path():
    mat = W.Lambertian((0.2, 0.3, 0.4))
    box = W.make_box((0, 0, 0), (1, 1, 1), mat)
    w = W.HittableList([W.Translate(box, (5, 0, 0)), W.Translate(box, (-5, 0, 0)), box])
    _, _, quads, _, _, mats, _, _ = W.flatten(w)
    assert len(quads) == 18 and len(mats) == 1  # one material row for the shared Arc
    assert np.allclose(quads["q"][:6, 0] - quads["q"][12:, 0], 5.0)
    assert np.allclose(quads["q"][6:12, 0] - quads["q"][12:, 0], -5.0)


def test_sphere_medium_and_textured_materials():
    earth = W.ImageTexture(np.zeros((4, 8, 3), np.uint8))
    noise = W.NoiseTexture(0.2)
    w = W.HittableList([
        W.ConstantMedium(W.Translate(W.Sphere((0, 0, 0), 70.0, W.Dielectric(1.5)), (360, 150, 145)), 0.2, (0.2, 0.4, 0.9)),
        W.Sphere((400, 200, 400), 100.0, W.Lambertian(earth)),
        W.Sphere((220, 280, 300), 80.0, W.Lambertian(noise)),
        W.Sphere((0, 0, 0), 1.0, W.Lambertian(W.CheckerTexture.from_colors(0.32, (0.2, 0.3, 0.1), (0.9, 0.9, 0.9)))),
    ])
    sc = W.build(w, W.Camera(image_width=16, samples_per_pixel=2))
    assert sc.media["boundary_kind"].tolist() == [0] and sc.media["sphere"][0].tolist() == [360, 150, 145, 70]
    assert sc.materials["kind"][sc.media["material_index"][0]] == 7
    kinds = sc.materials["kind"][sc.spheres["material_index"]].tolist()
    assert kinds == [3, 6, 5] and len(sc.textures) == 1 and len(sc.perlin) == 1
    assert sorted(sc.perlin[0]["perm_x"].tolist()) == list(range(256))
    chk = sc.materials[sc.spheres["material_index"][2]]
    assert chk["albedo_fuzz"][3] == np.float32(1 / 0.32) and chk["ref_idx"] == np.float32(0.9)
    img, _, _ = oracle.render(sc, oracle.TWIN, threads=4)
    assert np.isfinite(img).all()


def test_book3_through_the_api_matches_the_builder():
    ref = rrt.rest_of_your_life_scene(dict(image_width=24, samples_per_pixel=16, max_depth=8))
    red, white = W.Lambertian((0.65, 0.05, 0.05)), W.Lambertian((0.73, 0.73, 0.73))
    green, light = W.Lambertian((0.12, 0.45, 0.15)), W.DiffuseLight((15.0, 15.0, 15.0))
    w = W.HittableList([
        W.Quad((555, 0, 0), (0, 0, 555), (0, 555, 0), green), W.Quad((0, 0, 555), (0, 0, -555), (0, 555, 0), red),
        W.Quad((0, 555, 0), (555, 0, 0), (0, 0, 555), white), W.Quad((0, 0, 555), (555, 0, 0), (0, 0, -555), white),
        W.Quad((555, 0, 555), (-555, 0, 0), (0, 555, 0), white),
        W.Quad((213, 554, 227), (130, 0, 0), (0, 0, 105), light),
        W.Translate(W.RotateY(W.make_box((0, 0, 0), (165, 330, 165), white), 15.0), (265, 0, 295)),
        W.Sphere((190, 90, 190), 90.0, W.Dielectric(1.5)),
    ])
    lights = W.HittableList([W.Quad((343, 554, 332), (-130, 0, 0), (0, 0, -105)), W.Sphere((190, 90, 190), 90.0)])
    cam = W.Camera(aspect_ratio=1.0, image_width=24, samples_per_pixel=16, max_depth=8, background=(0, 0, 0),
                   vfov=40.0, lookfrom=(278, 278, -800), lookat=(278, 278, 0))
    sc = W.build(w, cam, lights=lights, book=3, seed=int(ref.camera["params_u"][0, 1]))
    assert sc.flags == ref.flags and np.array_equal(sc.lights, ref.lights)
    a, _, _ = oracle.render(sc, oracle.TWIN, threads=8)
    b, _, _ = oracle.render(ref, oracle.TWIN, threads=8)
    assert np.array_equal(a, b)


def test_flattener_errors():
    mat = W.Lambertian((0.5, 0.5, 0.5))
    loop = W.HittableList()
    loop.add(loop)  # a cycle: refused by the serialiser ...
    with pytest.raises(ValueError, match="cycle"):
        W.flatten(loop)
    # ... and by the C flattener (a node listing itself as its child)
    import ctypes

    from rustraytrace_amd import _lib
    nodes = np.zeros(1, dtype=_lib.NODE_DTYPE)
    nodes[0]["kind"], nodes[0]["count"] = _lib.NODE_LIST, 1
    children = np.zeros(1, dtype=np.uint32)
    out = _lib.RrtBookScene()
    rc = _lib.load().rrt_flatten_scene(_lib.ptr(nodes), 1, _lib.ptr(children), 1, 0, ctypes.byref(out))
    assert rc != 0 and "deeper than 64" in _lib.load().rrt_hip_last_error().decode()
    children[0] = 7  # out of range
    rc = _lib.load().rrt_flatten_scene(_lib.ptr(nodes), 1, _lib.ptr(children), 1, 0, ctypes.byref(out))
    assert rc != 0 and "out of range" in _lib.load().rrt_hip_last_error().decode()
    mixed = W.ConstantMedium(W.HittableList([W.Sphere((0, 0, 0), 1.0, mat), W.Quad((0, 0, 0), (1, 0, 0), (0, 1, 0), mat)]),
                             0.5, (1, 1, 1))
    with pytest.raises(rrt.RrtError, match="one sphere or quads only"):
        W.flatten(W.HittableList([mixed]))
    nested = W.ConstantMedium(W.ConstantMedium(W.Sphere((0, 0, 0), 1.0, mat), 0.5, (1, 1, 1)), 0.5, (1, 1, 1))
    with pytest.raises(rrt.RrtError, match="inside a medium"):
        W.flatten(W.HittableList([nested]))
    with pytest.raises(ValueError):
        W.flatten(W.HittableList([W.Sphere((0, 0, 0), 1.0)]))
