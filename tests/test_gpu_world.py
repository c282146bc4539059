"""A scene written with the books' API (rustraytrace_amd.world) through the whole GPU path:
nested RotateY / Translate instances, a shared box, a moving sphere, a box-bounded and a
sphere-bounded medium, checker and noise textures — bit-exact against the oracle (KBVH)."""
import numpy as np
import pytest

import rustraytrace_amd as rrt
from oracle import oracle
from rustraytrace_amd import world as W
from rustraytrace_amd.render import build_bvh

from test_gpu_parity import assert_bit_exact

pytestmark = pytest.mark.gpu


def test_api_scene_renders_bit_exact():
    ground = W.Lambertian(W.CheckerTexture.from_colors(0.5, (0.2, 0.3, 0.1), (0.9, 0.9, 0.9)))
    white, red = W.Lambertian((0.73, 0.73, 0.73)), W.Lambertian((0.65, 0.05, 0.05))
    box = W.make_box((0, 0, 0), (1, 2, 1), white)
    w = W.HittableList([
        W.Sphere((0, -1000, 0), 1000, ground),
        W.Translate(W.RotateY(box, 20), (-2, 0, 0)),
        W.RotateY(W.Translate(W.RotateY(box, -35), (2, 0, -1)), 10),
        W.Sphere.moving((0, 1, 0), (0, 1.5, 0), 0.5, red),
        W.Sphere((0, 0.6, 2), 0.6, W.Lambertian(W.NoiseTexture(3.0))),
        W.ConstantMedium(W.Translate(W.make_box((0, 0, 0), (1, 1, 1), white), (-0.5, 0, 3)), 0.8, (0.9, 0.9, 0.9)),
        W.ConstantMedium(W.Sphere((3, 1, 2), 0.8, white), 1.5, (0.2, 0.4, 0.9)),
        W.Quad((-3, 4, -3), (6, 0, 0), (0, 0, 6), W.DiffuseLight((4, 4, 4))),
    ])
    cam = W.Camera(aspect_ratio=16 / 9, image_width=96, samples_per_pixel=8, max_depth=20, vfov=40,
                   lookfrom=(6, 3, 9), lookat=(0, 1, 0), background=(0.1, 0.1, 0.15))
    sc = W.build(w, cam, seed=99)
    gpu = rrt.render(sc)
    nodes, order, info = build_bvh(sc)
    ref, _, _ = oracle.render_kbvh(sc, nodes, order, info, threads=16)
    assert_bit_exact(gpu, ref, sc.spp)
    assert np.all(gpu[..., 3] == sc.spp) and gpu[..., :3].mean() > 0
