"""GPU edge cases through the C-ABI, bit-exact against the oracle: empty and one-sphere scenes,
zero / negative radii (Sphere::new clamps to 0, sphere.rs:16-21), exact t-ties between
coincident spheres (the winner is the first one tested in tree order: compared against KBVH,
which walks the kernel's tree in the kernel's order), partial 8x8 tiles, and sample counts that
are not multiples of the 64-sample accumulation chunk."""
import numpy as np
import pytest

import rustraytrace_amd as rrt
from oracle import oracle
from rustraytrace_amd.render import build_bvh
from rustraytrace_amd.scenes import _material, _sphere, make_camera

from test_gpu_parity import assert_bit_exact

pytestmark = pytest.mark.gpu


def scene_of(spheres, materials, width=61, spp=5, depth=8, **cam):
    cam = make_camera(aspect_ratio=16.0 / 9.0, image_width=width, samples_per_pixel=spp, max_depth=depth,
                      lookfrom=cam.get("lookfrom", (0.0, 0.5, 3.0)), lookat=(0.0, 0.0, -1.0), vfov=60.0, seed=1234,
                      n_spheres=len(spheres))
    sph = np.concatenate(spheres) if spheres else np.zeros(0, dtype=rrt._lib.SPHERE_DTYPE)
    mats = np.concatenate(materials) if materials else np.zeros(0, dtype=rrt._lib.MATERIAL_DTYPE)
    return rrt.SceneData(cam, sph, mats, name="edge")


def check(sc):
    gpu = rrt.render(sc)
    nodes, order, info = build_bvh(sc)
    ref, rays, _ = oracle.render_kbvh(sc, nodes, order, info)
    assert_bit_exact(gpu, ref, sc.spp)
    return gpu, ref


def test_empty_scene_is_sky():
    sc = scene_of([], [])
    gpu, ref = check(sc)
    twin, _, _ = oracle.render(sc, oracle.TWIN)
    assert_bit_exact(gpu, twin, sc.spp)
    assert np.all(gpu[..., :3] > 0)


def test_single_sphere_all_materials():
    for kind, rgb, fuzz, ri in [(0, (0.7, 0.3, 0.2), 0, 1), (1, (0.8, 0.8, 0.8), 0.3, 1), (2, (1, 1, 1), 0, 1.5)]:
        sc = scene_of([_sphere((0.0, 0.0, -1.0), 0.5, 0)], [_material(kind, rgb, fuzz, ri)], depth=20)
        gpu, _ = check(sc)
        twin, _, _ = oracle.render(sc, oracle.TWIN)
        assert_bit_exact(gpu, twin, sc.spp)


def test_zero_and_negative_radius_spheres():
    sph = [_sphere((0.0, -100.5, -1.0), 100.0, 0), _sphere((0.0, 0.0, -1.0), 0.0, 1), _sphere((0.5, 0.0, -1.0), -0.3, 1),
           _sphere((-0.6, 0.0, -1.0), 0.4, 1)]
    sc = scene_of(sph, [_material(0, (0.5, 0.5, 0.5)), _material(1, (0.9, 0.6, 0.3), 0.1)], depth=12)
    check(sc)


def test_coincident_spheres_exact_ties():
    # two identical spheres with different materials: every hit is an exact t-tie
    sph = [_sphere((0.0, -100.5, -1.0), 100.0, 0), _sphere((0.0, 0.0, -1.0), 0.5, 1), _sphere((0.0, 0.0, -1.0), 0.5, 2),
           _sphere((0.7, 0.0, -1.2), 0.3, 1), _sphere((0.7, 0.0, -1.2), 0.3, 2)]
    mats = [_material(0, (0.5, 0.5, 0.5)), _material(0, (0.9, 0.1, 0.1)), _material(0, (0.1, 0.1, 0.9))]
    check(scene_of(sph, mats, depth=10))


@pytest.mark.parametrize("width,spp", [(1, 3), (7, 1), (61, 65), (33, 129)])
def test_partial_tiles_and_chunk_remainders(width, spp):
    sc = rrt.rtow(image_width=width, samples_per_pixel=spp, max_depth=10)
    gpu, _ = check(sc)
    assert np.all(gpu[..., 3] == spp)


def test_axis_parallel_rays():
    # d.x == 0 for every camera ray, through a box that straddles x = 0 (test_oracle.py)
    from test_oracle import axis_parallel_scene

    gpu, _ = check(axis_parallel_scene())
    assert np.all(gpu[..., :3] == 0)
