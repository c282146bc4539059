"""The 32-B f16 BVH2 nodes of scenes read from global memory (rrt_internal.h GNodeH) at every
coordinate scale: the planes are rounded outward, so the kernel's tree never prunes a box whose
primitive a ray hits. CPU: the oracle's KBVH walk over those nodes renders the same image as its
TWIN mode over its own f32 tree, for the RTOW scene forced to global memory at scale 1, at 3000
(coordinates ~4e4, f16 steps of 32) and at 1e5 (beyond f16's 65504: planes saturate to +-inf or
65504, every box is entered, the walk degenerates to testing every leaf). GPU: the kernel against
KBVH on the same scaled scenes, bit for bit (tests/test_gpu_parity.py).
"""
import copy

import numpy as np
import pytest

import rustraytrace_amd as rrt
from oracle import oracle
from rustraytrace_amd.render import build_bvh, decode_bvh2


def scaled_scene(scene, s):
    """The scene with every length multiplied by s (centres, radii, camera origin, pixel grid,
    defocus radius): the same picture, at coordinates s times larger."""
    sc = copy.deepcopy(scene)
    sc.spheres["center_radius"] *= np.float32(s)
    cam = sc.camera
    for f in ("origin", "pixel00", "pixel_delta_u", "pixel_delta_v"):
        cam[f][..., :3] *= np.float32(s)
    cam["params_f"][..., 0] *= np.float32(s)  # defocus radius
    return sc


SCALES = [1.0, 3000.0, 1e5]


@pytest.mark.parametrize("s", SCALES)
def test_f16_nodes_lose_no_hit(monkeypatch, s):
    monkeypatch.setenv("RRT_SCENE_IN_LDS", "0")
    sc = scaled_scene(rrt.rtow(image_width=40, samples_per_pixel=4, max_depth=8), s)
    nodes, order, info = build_bvh(sc)
    assert info["node_stride"] == 32
    lo, hi, _, _ = decode_bvh2(nodes, 32)
    if s >= 1e5:
        assert np.isinf(lo).any() and np.isinf(hi).any()  # saturated planes occur
    kb, rays_k, _ = oracle.render_kbvh(sc, nodes, order, info, threads=8)
    tw, rays_t, _ = oracle.render(sc, oracle.TWIN, threads=8)
    assert rays_k == rays_t
    assert np.array_equal(kb, tw)
