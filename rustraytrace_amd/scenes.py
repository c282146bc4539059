"""Scene construction — the callers on the near side of the boundary.

* `build_in_one_weekend_scene` == gpu::build_in_one_weekend_scene (src/gpu/mod.rs:124-301),
  implemented in C++ inside librrt_hip.so and exposed through the C-ABI.
* The BASELINE configs (BASELINE.json `configs`) as named scenes:
    C1 three_spheres   3-sphere Lambertian, 400x225, 64 spp, depth 8
    C2 rtow            RTOW final scene (seed 0x5EED_1234), 1920x1080, 512 spp, depth 100
    C3 rtow_4k         same scene, 3840x2160, 2048 spp (8-GPU tile split)
    C4 earth_light     textured earth + emissive sphere, 1920x1080, 1024 spp
    C5 stress10k       RTOW generator on a 100x100 grid (<=10,004 spheres), 1920x1080, 256 spp
* `next_week_scene` — book-2 scenes 1-10 (the_next_week/mod.rs:68-587), flattened by
  rrt_build_next_week_scene; `rest_of_your_life_scene` — book 3.
* Scenes of your own: the books' object API in `rustraytrace_amd.world` (Sphere, Quad,
  HittableList, BvhNode, Translate, RotateY, ConstantMedium, make_box, materials and textures),
  flattened by rrt_flatten_scene.
"""
from __future__ import annotations

import ctypes
import dataclasses
import os
from typing import Optional, Sequence

import numpy as np

from . import _lib

RTOW_SEED = 0x5EED_1234
C1_SEED = 0xC0FFEE
C4_SEED = 0xE4A7_0001
NEXT_WEEK_SEED = 0xB00C_0002
NEXT_WEEK_SCENES = {1: "bouncing_spheres", 2: "checkered_spheres", 3: "earth", 4: "perlin_spheres", 5: "quads",
                    6: "simple_light", 7: "cornell_box", 8: "cornell_smoke", 9: "final_scene_800",
                    10: "final_scene_400"}

# config.rs:50-62 committed OVERRIDES (width 2160, spp 5000, depth 100)
COMMITTED_OVERRIDES = dict(image_width=2160, samples_per_pixel=5000, max_depth=100)


@dataclasses.dataclass
class SceneData:
    """The flat #[repr(C)] scene the boundary takes (CameraUniform, Vec<SphereGpu>, Vec<MaterialGpu>)."""

    camera: np.ndarray  # shape (1,), CAMERA_DTYPE
    spheres: np.ndarray  # SPHERE_DTYPE
    materials: np.ndarray  # MATERIAL_DTYPE
    textures: list = dataclasses.field(default_factory=list)  # uint8 (H, W, 3) arrays
    flags: int = 0
    name: str = ""
    motion: Optional[np.ndarray] = None  # (n_spheres, 4) float32: center2 - center1 (book 2), or None
    perlin: Optional[np.ndarray] = None  # PERLIN_DTYPE tables for noise materials, or None
    quads: Optional[np.ndarray] = None  # QUAD_DTYPE quads (primitives n_spheres + j), or None
    media: Optional[np.ndarray] = None  # MEDIUM_DTYPE constant-density media, or None
    boundary_quads: Optional[np.ndarray] = None  # QUAD_DTYPE boundaries of quad-bounded media
    lights: Optional[np.ndarray] = None  # LIGHT_DTYPE book-3 MIS light list (FLAG_BOOK3)

    @property
    def width(self) -> int:
        return int(self.camera["params_f"][0, 1])

    @property
    def height(self) -> int:
        return int(self.camera["params_f"][0, 2])

    @property
    def spp(self) -> int:
        return max(int(self.camera["params_f"][0, 3]), 1)

    @property
    def max_depth(self) -> int:
        return int(self.camera["params_u"][0, 0])

    @property
    def seed(self) -> int:
        return int(self.camera["params_u"][0, 1])

    def to_bytes(self) -> bytes:
        return self.camera.tobytes() + self.spheres.tobytes() + self.materials.tobytes()


def _empty(dtype, n):
    return np.zeros(n, dtype=dtype)


def build_in_one_weekend_scene(overrides: Optional[dict] = None, seed: int = RTOW_SEED,
                               grid_half: int = 11) -> SceneData:
    """gpu::build_in_one_weekend_scene (gpu/mod.rs:124-301) with RenderOverrides `overrides`."""
    lib = _lib.load()
    ov = _lib.make_overrides(**(overrides or {}))
    n = ctypes.c_uint32(0)
    cam = _empty(_lib.CAMERA_DTYPE, 1)
    _lib.check(lib.rrt_build_in_one_weekend_scene(_lib.ptr(ov), seed, grid_half, _lib.ptr(cam), None, None, 0,
                                                  _lib.ptr(n)))
    spheres = _empty(_lib.SPHERE_DTYPE, n.value)
    mats = _empty(_lib.MATERIAL_DTYPE, n.value)
    _lib.check(lib.rrt_build_in_one_weekend_scene(_lib.ptr(ov), seed, grid_half, _lib.ptr(cam), _lib.ptr(spheres),
                                                  _lib.ptr(mats), n.value, _lib.ptr(n)))
    return SceneData(cam, spheres, mats, name=f"rtow(grid_half={grid_half})")


def make_camera(*, aspect_ratio=1.0, image_width=100, samples_per_pixel=10, max_depth=10, vfov=90.0,
                lookfrom=(0.0, 0.0, 0.0), lookat=(0.0, 0.0, -1.0), vup=(0.0, 1.0, 0.0), defocus_angle=0.0,
                focus_dist=10.0, background: Optional[Sequence[float]] = None, seed=0, n_spheres=0) -> np.ndarray:
    """Camera::initialize (camera.rs:102-150) cast to the f32 ABI (gpu/mod.rs:278-298).
    Defaults are Camera::default() (camera.rs:30-45)."""
    lib = _lib.load()
    cam = _empty(_lib.CAMERA_DTYPE, 1)
    f3 = lambda v: np.asarray(v, dtype=np.float64)
    lf, la, vu = f3(lookfrom), f3(lookat), f3(vup)
    bg = None if background is None else f3(background)
    _lib.check(lib.rrt_make_camera(float(aspect_ratio), int(image_width), int(samples_per_pixel), int(max_depth),
                                   float(vfov), _lib.ptr(lf), _lib.ptr(la), _lib.ptr(vu), float(defocus_angle),
                                   float(focus_dist), _lib.ptr(bg), int(seed) & 0xFFFFFFFF, int(n_spheres),
                                   _lib.ptr(cam)))
    return cam


def _material(kind, rgb, fuzz=0.0, ref_idx=1.0, tex=0):
    m = np.zeros(1, dtype=_lib.MATERIAL_DTYPE)
    m["albedo_fuzz"][0] = [rgb[0], rgb[1], rgb[2], fuzz]
    m["kind"][0] = kind
    m["ref_idx"][0] = ref_idx
    m["_pad"][0, 0] = tex
    return m


def _sphere(c, r, mat):
    s = np.zeros(1, dtype=_lib.SPHERE_DTYPE)
    s["center_radius"][0] = [c[0], c[1], c[2], r]
    s["material_index"][0] = mat
    return s


def three_spheres(image_width=400, samples_per_pixel=64, max_depth=8, seed=C1_SEED) -> SceneData:
    """C1: Camera::default() at 16:9, sky, three Lambertian spheres."""
    mats = np.concatenate([_material(0, (0.8, 0.8, 0.0)), _material(0, (0.1, 0.2, 0.5)), _material(0, (0.5, 0.5, 0.5))])
    sph = np.concatenate([_sphere((0.0, -100.5, -1.0), 100.0, 0), _sphere((0.0, 0.0, -1.2), 0.5, 1),
                          _sphere((-1.0, 0.0, -1.0), 0.5, 2)])
    cam = make_camera(aspect_ratio=16.0 / 9.0, image_width=image_width, samples_per_pixel=samples_per_pixel,
                      max_depth=max_depth, seed=seed, n_spheres=len(sph))
    return SceneData(cam, sph, mats, name="three_spheres")


def earth_texture() -> np.ndarray:
    """Decoded images/earthmap.jpg (1024x512 RGB8), see tools/make_earth_asset.py."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets", "earthmap_rgb8.npz")
    with np.load(path, allow_pickle=False) as z:
        return np.ascontiguousarray(z["rgb8"])


def earth_ppm_path() -> str:
    """The binary P6 copy of the earth texture the C++ CLI resolves like rtw_image.rs:11-36
    (rustraytrace_amd/assets/earthmap.ppm, next to the rrt executable's directory)."""
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets", "earthmap.ppm")


def ensure_earth_ppm() -> str:
    """Write earthmap.ppm (P6, the committed RGB8 decode of images/earthmap.jpg) if it is missing
    or differs; build() calls this. Returns its path."""
    rgb = earth_texture()
    data = b"P6\n%d %d\n255\n" % (rgb.shape[1], rgb.shape[0]) + rgb.tobytes()
    path = earth_ppm_path()
    try:
        with open(path, "rb") as f:
            if f.read() == data:
                return path
    except OSError:
        pass
    with open(path + ".tmp", "wb") as f:
        f.write(data)
    os.replace(path + ".tmp", path)
    return path


def earth_light(image_width=1920, samples_per_pixel=1024, max_depth=100, seed=C4_SEED) -> SceneData:
    """C4: the_next_week earth() (mod.rs:196-220) + DiffuseLight(4,4,4) sphere at (0,7,0) r=2
    (simple_light, mod.rs:330-331), background black (mod.rs:344). Book-2 camera (time draw)."""
    mats = np.concatenate([_material(3, (0.0, 0.0, 0.0), tex=0), _material(4, (4.0, 4.0, 4.0))])
    sph = np.concatenate([_sphere((0.0, 0.0, 0.0), 2.0, 0), _sphere((0.0, 7.0, 0.0), 2.0, 1)])
    cam = make_camera(aspect_ratio=16.0 / 9.0, image_width=image_width, samples_per_pixel=samples_per_pixel,
                      max_depth=max_depth, vfov=20.0, lookfrom=(0.0, 0.0, 12.0), lookat=(0.0, 0.0, 0.0),
                      background=(0.0, 0.0, 0.0), seed=seed, n_spheres=len(sph))
    return SceneData(cam, sph, mats, textures=[earth_texture()], flags=_lib.FLAG_RAY_TIME, name="earth_light")


def next_week_scene(scene: int, overrides: Optional[dict] = None, seed: int = NEXT_WEEK_SEED) -> SceneData:
    """The book-2 scene `scene` (1 bouncing_spheres, 2 checkered_spheres, 3 earth, 4 perlin_spheres,
    5 quads, 6 simple_light, 7 cornell_box, 8 cornell_smoke, 9 final_scene(800, 10000, 40),
    10 final_scene(400, 250, 4); the_next_week/mod.rs:68-587) under RenderOverrides `overrides`,
    with its motion rows, quads and media (instanced geometry baked to world space) and Perlin
    tables. Book-2 camera: background colour, a time draw per camera ray."""
    lib = _lib.load()
    return _book_scene(lambda ov, nw: lib.rrt_build_next_week_scene(int(scene), _lib.ptr(ov), seed, ctypes.byref(nw)),
                       overrides, NEXT_WEEK_SCENES[scene] if scene in NEXT_WEEK_SCENES else str(scene))


def rest_of_your_life_scene(overrides: Optional[dict] = None, seed: int = NEXT_WEEK_SEED) -> SceneData:
    """The book-3 scene (the_rest_of_your_life/mod.rs:69-161): Cornell box, a rotated box and a
    glass sphere, with the MIS light list {light quad, glass sphere}; stratified sampling rounds
    samples_per_pixel down to a square. Renders with FLAG_RAY_TIME | FLAG_BOOK3."""
    lib = _lib.load()
    return _book_scene(lambda ov, nw: lib.rrt_build_rest_of_your_life_scene(_lib.ptr(ov), seed, ctypes.byref(nw)),
                       overrides, "rest_of_your_life")


def _book_scene(build, overrides, name) -> SceneData:
    """Two-pass RrtBookScene build (sizes, then arrays) into a SceneData."""
    ov = _lib.make_overrides(**(overrides or {}))
    nw = _lib.RrtBookScene()
    _lib.check(build(ov, nw))  # sizes
    spheres = _empty(_lib.SPHERE_DTYPE, nw.n_spheres)
    motion = np.zeros((nw.n_spheres, 4), dtype=np.float32)
    mats = _empty(_lib.MATERIAL_DTYPE, nw.n_materials)
    quads = np.zeros(nw.n_quads, dtype=_lib.QUAD_DTYPE)
    perlin = np.zeros(nw.n_perlin, dtype=_lib.PERLIN_DTYPE)
    media = np.zeros(nw.n_media, dtype=_lib.MEDIUM_DTYPE)
    bquads = np.zeros(nw.n_boundary_quads, dtype=_lib.QUAD_DTYPE)
    lights = np.zeros(nw.n_lights, dtype=_lib.LIGHT_DTYPE)
    for field, arr in (("spheres", spheres), ("materials", mats), ("quads", quads), ("perlin", perlin),
                       ("media", media), ("boundary_quads", bquads), ("lights", lights)):
        setattr(nw, field, arr.ctypes.data)
    nw.sphere_motion = motion.ctypes.data
    nw.sphere_cap, nw.material_cap, nw.quad_cap = nw.n_spheres, nw.n_materials, nw.n_quads
    nw.perlin_cap, nw.media_cap, nw.boundary_quad_cap = nw.n_perlin, nw.n_media, nw.n_boundary_quads
    nw.light_cap = nw.n_lights
    _lib.check(build(ov, nw))
    cam = np.frombuffer(bytes(nw.camera), dtype=_lib.CAMERA_DTYPE).copy()
    textures = [earth_texture()] if nw.uses_texture0 else []
    return SceneData(cam, spheres, mats, textures=textures, flags=int(nw.flags), name=name,
                     motion=motion if np.any(motion[:, :3]) else None, perlin=perlin if len(perlin) else None,
                     quads=quads if len(quads) else None, media=media if len(media) else None,
                     boundary_quads=bquads if len(bquads) else None, lights=lights if len(lights) else None)


def rtow(image_width=1920, samples_per_pixel=512, max_depth=100, grid_half=11, seed=RTOW_SEED) -> SceneData:
    sc = build_in_one_weekend_scene(dict(image_width=image_width, samples_per_pixel=samples_per_pixel,
                                         max_depth=max_depth), seed=seed, grid_half=grid_half)
    sc.name = "rtow" if grid_half == 11 else f"rtow_grid{grid_half}"
    return sc


CONFIGS = {
    "C1": ("three_spheres", dict(image_width=400, samples_per_pixel=64, max_depth=8)),
    "C2": ("rtow", dict(image_width=1920, samples_per_pixel=512, max_depth=100)),
    "C3": ("rtow", dict(image_width=3840, samples_per_pixel=2048, max_depth=100)),
    "C4": ("earth_light", dict(image_width=1920, samples_per_pixel=1024, max_depth=100)),
    "C5": ("rtow", dict(image_width=1920, samples_per_pixel=256, max_depth=100, grid_half=50)),
}


def config_scene(name: str, **override) -> SceneData:
    """A BASELINE config scene; keyword overrides (image_width, samples_per_pixel, max_depth)
    shrink it for parity tests."""
    builder, kw = CONFIGS[name]
    kw = dict(kw, **override)
    fn = {"three_spheres": three_spheres, "rtow": rtow, "earth_light": earth_light}[builder]
    sc = fn(**kw)
    sc.name = name
    return sc


# The scene table's workloads (tools/bench_scenes.py at spp scale 1/4): book-2
# scenes at 1920x1080 (square scenes 1080x1080), 64 spp, max_depth 50 (final_scene keeps its 40).
_SQUARE = (5, 7, 8, 9, 10)
NAMED = {f"NW{k}": dict(image_width=1080 if k in _SQUARE else 1920, samples_per_pixel=64,
                        **({} if k in (9, 10) else dict(max_depth=50))) for k in range(1, 11)}
NAMED["B3"] = dict(image_width=1080, samples_per_pixel=64, max_depth=50)


def named_scene(name: str, **override) -> SceneData:
    """A BASELINE config (C1-C5) or a scene-table workload by name: NW1-NW10 (the_next_week
    scenes, `next_week_scene`) and B3 (`rest_of_your_life_scene`) at the NAMED sizes."""
    if name in CONFIGS:
        return config_scene(name, **override)
    if name not in NAMED:
        raise KeyError(f"unknown workload {name!r}: {sorted(CONFIGS) + sorted(NAMED)}")
    kw = dict(NAMED[name], **override)
    sc = rest_of_your_life_scene(kw) if name == "B3" else next_week_scene(int(name[2:]), kw)
    sc.name = f"{name} {sc.name}"
    return sc
