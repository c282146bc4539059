"""Generate the committed golden fixtures under tests/golden/.

The reference ships no tests, fixtures or rendered images (`.MISSING_LARGE_BLOBS`
shows its image.ppm was stripped), so the fixtures are produced here by the oracle's f32 TWIN
restatement of the books path (oracle/rrt_oracle.cpp) on scenes from the product's scene
builders, and pinned by the analytic known-answer tests in tests/test_oracle.py.

Each case writes <name>.npz with:
    scene_sha256   SHA-256 of the flat #[repr(C)] scene bytes (camera + spheres + materials)
    accum          float32 (H, W, 4) TWIN accum (RGB sums, w = sample count)
    rays           closest-hit queries the oracle traced
    ppm            the render_io.rs P3 bytes (uint8 array)
    books_accum    float64 (H, W, 4) BOOKS accum (the f64 recursive restatement)
    books_rays     closest-hit queries of the BOOKS render

Round 2 regenerated every fixture: the f32 modes (and the kernel) gained exit_skip (the
primitive a scattered ray leaves is not tested for a hit again; oracle/rrt_oracle.cpp).
Regenerated again when the f32 modes and the kernel took fused multiply-adds for dot products,
the sphere discriminant and Ray::at (oracle/rrt_oracle.cpp dot3 / sphere_disc / ray_at).

    python tests/golden/make_golden.py
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

CASES = {
    "c1_64x36x8": ("C1", dict(image_width=64, samples_per_pixel=8)),
    "rtow_64x36x8": ("C2", dict(image_width=64, samples_per_pixel=8, max_depth=20)),
    "rtow_96x54x4_d100": ("C2", dict(image_width=96, samples_per_pixel=4)),
    "earth_64x36x8": ("C4", dict(image_width=64, samples_per_pixel=8)),
    "stress10k_48x27x4": ("C5", dict(image_width=48, samples_per_pixel=4)),
}


def scene_sha(scene) -> str:
    h = hashlib.sha256(scene.to_bytes())
    for t in scene.textures:
        h.update(np.ascontiguousarray(t).tobytes())
    return h.hexdigest()


def main():
    import rustraytrace_amd as rrt
    from oracle import oracle

    for name, (cfg, kw) in CASES.items():
        scene = rrt.config_scene(cfg, **kw)
        acc, rays, _ = oracle.render(scene, oracle.TWIN, threads=8)
        acc32 = acc.astype(np.float32)
        assert np.array_equal(acc32.astype(np.float64), acc)
        ppm = rrt.format_ppm_from_accum(scene.width, scene.height, acc32, scene.spp)
        bacc, brays, _ = oracle.render(scene, oracle.BOOKS, threads=8)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), scene_sha256=np.array(scene_sha(scene)),
                            accum=acc32, rays=np.array(rays, dtype=np.uint64),
                            ppm=np.frombuffer(ppm, dtype=np.uint8), books_accum=bacc,
                            books_rays=np.array(brays, dtype=np.uint64))
        print(name, scene.width, scene.height, scene.spp, rays)


if __name__ == "__main__":
    main()
