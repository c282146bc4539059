"""A cluster of coincident spheres in a scene read from global memory (rrt_host.cpp scene_bvh): the
global-memory shape splits to single-primitive leaves, and the SAH sweep splits equal boxes 1 | n-1,
so a cluster of n spheres turns into a chain about n deep. When that chain needs more stack than the
kernels hold (kMaxStackDepth = 64 entries), the builder falls back to the caller's leaf size (3),
whose chain is two levels shorter, instead of failing scene creation for a scene that built with it
(ADVICE r4). Host only: rrt_build_bvh returns the tree rrt_scene_create would build."""
import numpy as np

from rustraytrace_amd.render import build_bvh
from rustraytrace_amd import scenes as S

MAX_STACK = 64


def _scene(n_cluster, n_field=3000, seed=11):
    rng = np.random.default_rng(seed)
    mats = S._material(0, (0.5, 0.5, 0.5))
    field = [S._sphere(rng.uniform(-200, 200, 3), 0.5, 0) for _ in range(n_field)]  # over the LDS budget
    cluster = [S._sphere((3.0, 1.0, -2.0), 0.25, 0) for _ in range(n_cluster)]
    sph = np.concatenate(field + cluster)
    cam = S.make_camera(image_width=16, samples_per_pixel=1, n_spheres=len(sph))
    return S.SceneData(cam, sph, mats, name=f"coincident{n_cluster}")


def test_coincident_cluster_falls_back_to_the_callers_leaf_size():
    rescued = 0
    for n in range(40, 72, 2):
        _, _, info = build_bvh(_scene(n))
        assert info["node_stride"] == 32  # read from global memory (f16 nodes)
        need = info["max_depth"] + 1
        if info["max_leaf_size"] == 1:
            assert need <= MAX_STACK  # the single-primitive shape is kept whenever it fits
        elif need <= MAX_STACK:
            rescued += 1  # single-primitive leaves needed more; leaves of 3 fit
    # the cluster sizes whose single-primitive chain is one or two levels too deep build now
    assert rescued >= 1, "no cluster size reached the fallback"
