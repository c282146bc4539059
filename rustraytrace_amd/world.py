"""The books' scene-building API (the_next_week / the_rest_of_your_life: hittable.rs, sphere.rs,
quad.rs, hittable_list.rs, bvh.rs, constant_medium.rs, material.rs, texture.rs, camera.rs) on top
of the flat C-ABI: build a world the way the books do —

    world = HittableList()
    white = Lambertian((0.73, 0.73, 0.73))
    box1 = Translate(RotateY(make_box((0, 0, 0), (165, 330, 165), white), 15), (265, 0, 295))
    world.add(ConstantMedium(box1, 0.01, (0, 0, 0)))
    scene = build(world, Camera(aspect_ratio=1.0, image_width=600, ...), book=2)
    accum = rustraytrace_amd.render(scene)

`build` serialises the object graph into RrtSceneNode records (shared objects stay shared, as
`Arc`s are) and calls rrt_flatten_scene, which composes every Translate / RotateY and bakes it
into world-space spheres, quads and media. Materials and textures become
RrtMaterial rows (one per distinct object), Perlin tables and images the scene's side arrays.
A BvhNode is accepted and flattened like a list: the backend builds its own tree."""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from .scenes import SceneData, make_camera

Vec = Sequence[float]


# ---- textures (texture.rs) --------------------------------------------------------------------
@dataclass(eq=False)
class SolidColor:
    albedo: Vec


@dataclass(eq=False)
class CheckerTexture:
    """CheckerTexture::from_colors(scale, even, odd) (texture.rs:39-77)."""
    scale: float
    even: Vec
    odd: Vec

    @staticmethod
    def from_colors(scale: float, even: Vec, odd: Vec) -> "CheckerTexture":
        return CheckerTexture(scale, even, odd)


class Perlin:
    """Perlin::new (perlin.rs:12-22, 70-82) drawn from a numpy Generator (the reference draws from
    its entropy RNG): 256 unit vectors from [-1, 1)^3, three Fisher-Yates permutations."""

    def __init__(self, rng: Optional[np.random.Generator] = None):
        rng = rng if rng is not None else np.random.default_rng(0x9E3779B9)
        t = np.zeros(1, dtype=_lib.PERLIN_DTYPE)[0]
        v = rng.uniform(-1.0, 1.0, (256, 3))
        t["randvec"][:, :3] = v / np.sqrt((v * v).sum(axis=1, keepdims=True))
        for key in ("perm_x", "perm_y", "perm_z"):
            p = np.arange(256)
            for i in range(255, 0, -1):
                j = int(rng.integers(0, i + 1))
                p[i], p[j] = p[j], p[i]
            t[key] = p
        self.table = t


@dataclass(eq=False)
class NoiseTexture:
    """NoiseTexture::new(scale) (texture.rs:111-126)."""
    scale: float
    perlin: Perlin = field(default_factory=Perlin)


@dataclass(eq=False)
class ImageTexture:
    """ImageTexture over an RGB8 (H, W, 3) uint8 image (texture.rs:89-109)."""
    rgb8: np.ndarray


# ---- materials (material.rs) ------------------------------------------------------------------
@dataclass(eq=False)
class Lambertian:
    albedo: object  # an RGB triple or a texture


@dataclass(eq=False)
class Metal:
    albedo: Vec
    fuzz: float


@dataclass(eq=False)
class Dielectric:
    refraction_index: float


@dataclass(eq=False)
class DiffuseLight:
    emit: Vec


@dataclass(eq=False)
class Isotropic:
    albedo: Vec


# ---- hittables (hittable.rs:172-180) -----------------------------------------------------------
@dataclass(eq=False)
class Sphere:
    """Sphere::new / Sphere::new_moving (center2 given) (the_next_week/sphere.rs:14-40)."""
    center: Vec
    radius: float
    mat: object = None
    center2: Optional[Vec] = None

    @staticmethod
    def moving(center1: Vec, center2: Vec, radius: float, mat) -> "Sphere":
        return Sphere(center1, radius, mat, center2)


@dataclass(eq=False)
class Quad:
    q: Vec
    u: Vec
    v: Vec
    mat: object = None


class HittableList:
    def __init__(self, objects: Optional[List[object]] = None):
        self.objects = list(objects or [])

    def add(self, obj) -> None:
        self.objects.append(obj)

    def clear(self) -> None:
        self.objects.clear()


class BvhNode:
    """BvhNode::new(list) (bvh.rs): accepted and flattened like the list it wraps."""

    def __init__(self, objects):
        self.objects = list(objects.objects if isinstance(objects, HittableList) else objects)


@dataclass(eq=False)
class Translate:
    object: object
    offset: Vec


@dataclass(eq=False)
class RotateY:
    object: object
    angle: float  # degrees


@dataclass(eq=False)
class ConstantMedium:
    """ConstantMedium::from_color(boundary, density, albedo) / ::new with an Isotropic phase."""
    boundary: object
    density: float
    albedo: object  # an RGB triple or an Isotropic material


def make_box(a: Vec, b: Vec, mat) -> HittableList:
    """quad.rs:95-119: the six faces of the box spanned by a and b."""
    lo = [min(a[i], b[i]) for i in range(3)]
    hi = [max(a[i], b[i]) for i in range(3)]
    dx, dy, dz = (hi[0] - lo[0], 0.0, 0.0), (0.0, hi[1] - lo[1], 0.0), (0.0, 0.0, hi[2] - lo[2])
    ndx, ndz = (-dx[0], 0.0, 0.0), (0.0, 0.0, -dz[2])
    return HittableList([
        Quad((lo[0], lo[1], hi[2]), dx, dy, mat),
        Quad((hi[0], lo[1], hi[2]), ndz, dy, mat),
        Quad((hi[0], lo[1], lo[2]), ndx, dy, mat),
        Quad((lo[0], lo[1], lo[2]), dz, dy, mat),
        Quad((lo[0], hi[1], hi[2]), dx, ndz, mat),
        Quad((lo[0], lo[1], lo[2]), dx, dz, mat),
    ])


@dataclass
class Camera:
    """Camera's public fields with Camera::default() values (camera.rs:30-45). background None =
    book 1's sky gradient."""
    aspect_ratio: float = 1.0
    image_width: int = 100
    samples_per_pixel: int = 10
    max_depth: int = 10
    vfov: float = 90.0
    lookfrom: Vec = (0.0, 0.0, 0.0)
    lookat: Vec = (0.0, 0.0, -1.0)
    vup: Vec = (0.0, 1.0, 0.0)
    defocus_angle: float = 0.0
    focus_dist: float = 10.0
    background: Optional[Vec] = (0.70, 0.80, 1.00)


# ---- serialisation -----------------------------------------------------------------------------
class _Builder:
    def __init__(self):
        self.nodes: List[np.void] = []
        self.children: List[int] = []
        self.node_of = {}
        self.mats: List[np.ndarray] = []
        self.mat_of = {}
        self.perlin: List[np.void] = []
        self.perlin_of = {}
        self.textures: List[np.ndarray] = []
        self.texture_of = {}
        self.keep: List[object] = []  # every object keyed by id() stays alive: ids are never reused

    # materials -> RrtMaterial rows (one per distinct object, like an Arc)
    def material(self, m) -> int:
        if m is None:
            raise ValueError("a sphere or quad needs a material")
        if id(m) in self.mat_of:
            return self.mat_of[id(m)]
        row = np.zeros(1, dtype=_lib.MATERIAL_DTYPE)
        r = row[0]
        r["ref_idx"] = 1.0
        if isinstance(m, Lambertian):
            tex = m.albedo
            if isinstance(tex, SolidColor):
                tex = tex.albedo
            if isinstance(tex, CheckerTexture):
                odd = np.asarray(tex.odd, np.float32)
                r["kind"] = 5
                r["albedo_fuzz"] = [*tex.even, 1.0 / tex.scale]
                r["ref_idx"] = odd[0]
                r["_pad"] = odd[1:3].view(np.uint32)
            elif isinstance(tex, NoiseTexture):
                r["kind"] = 6
                r["albedo_fuzz"] = [0.5, 0.5, 0.5, tex.scale]
                r["_pad"][0] = self.perlin_table(tex.perlin)
            elif isinstance(tex, ImageTexture):
                r["kind"] = 3
                r["_pad"][0] = self.texture(tex)
            else:
                r["kind"] = 0
                r["albedo_fuzz"] = [*tex, 0.0]
        elif isinstance(m, Metal):
            r["kind"], r["albedo_fuzz"] = 1, [*m.albedo, m.fuzz]
        elif isinstance(m, Dielectric):
            r["kind"], r["albedo_fuzz"], r["ref_idx"] = 2, [1.0, 1.0, 1.0, 0.0], m.refraction_index
        elif isinstance(m, DiffuseLight):
            r["kind"], r["albedo_fuzz"] = 4, [*m.emit, 0.0]
        elif isinstance(m, Isotropic):
            r["kind"], r["albedo_fuzz"] = 7, [*m.albedo, 0.0]
        else:
            raise TypeError(f"unsupported material {type(m).__name__}")
        self.mat_of[id(m)] = len(self.mats)
        self.keep.append(m)
        self.mats.append(row)
        return self.mat_of[id(m)]

    def perlin_table(self, p: Perlin) -> int:
        if id(p) not in self.perlin_of:
            self.keep.append(p)
            self.perlin_of[id(p)] = len(self.perlin)
            self.perlin.append(p.table)
        return self.perlin_of[id(p)]

    def texture(self, t: ImageTexture) -> int:
        if id(t) not in self.texture_of:
            self.keep.append(t)
            self.texture_of[id(t)] = len(self.textures)
            self.textures.append(np.ascontiguousarray(t.rgb8, dtype=np.uint8))
        return self.texture_of[id(t)]

    # hittables -> RrtSceneNode records (a shared object is one node with several parents)
    def node(self, obj, _visiting=None) -> int:
        if id(obj) in self.node_of:
            return self.node_of[id(obj)]
        visiting = _visiting if _visiting is not None else set()
        if id(obj) in visiting:
            raise ValueError("the object graph has a cycle")
        visiting.add(id(obj))
        rec = np.zeros(1, dtype=_lib.NODE_DTYPE)[0]
        kids: List[int] = []
        if isinstance(obj, Sphere):
            rec["kind"], rec["material"] = _lib.NODE_SPHERE, self.material(obj.mat)
            rec["a"] = [*obj.center, obj.radius]
            if obj.center2 is not None:
                rec["b"][:3] = np.asarray(obj.center2, np.float64) - np.asarray(obj.center, np.float64)
        elif isinstance(obj, Quad):
            rec["kind"], rec["material"] = _lib.NODE_QUAD, self.material(obj.mat)
            rec["a"][:3], rec["b"][:3], rec["c"][:3] = obj.q, obj.u, obj.v
        elif isinstance(obj, (HittableList, BvhNode)):
            rec["kind"] = _lib.NODE_LIST if isinstance(obj, HittableList) else _lib.NODE_BVH
            kids = [self.node(o, visiting) for o in obj.objects]
        elif isinstance(obj, Translate):
            rec["kind"], rec["a"][:3] = _lib.NODE_TRANSLATE, obj.offset
            kids = [self.node(obj.object, visiting)]
        elif isinstance(obj, RotateY):
            rec["kind"], rec["a"][0] = _lib.NODE_ROTATE_Y, obj.angle
            kids = [self.node(obj.object, visiting)]
        elif isinstance(obj, ConstantMedium):
            phase = obj.albedo if isinstance(obj.albedo, Isotropic) else Isotropic(tuple(obj.albedo))
            rec["kind"], rec["material"], rec["a"][0] = _lib.NODE_CONSTANT_MEDIUM, self.material(phase), obj.density
            kids = [self.node(obj.boundary, visiting)]
        else:
            raise TypeError(f"unsupported hittable {type(obj).__name__}")
        rec["first"], rec["count"] = len(self.children), len(kids)
        self.children.extend(kids)
        visiting.discard(id(obj))
        self.node_of[id(obj)] = len(self.nodes)
        self.keep.append(obj)
        self.nodes.append(rec)
        return self.node_of[id(obj)]


def _light_records(lights) -> Optional[np.ndarray]:
    if lights is None:
        return None
    objs = lights.objects if isinstance(lights, (HittableList, BvhNode)) else list(lights)
    out = np.zeros(len(objs), dtype=_lib.LIGHT_DTYPE)
    for k, o in enumerate(objs):
        if isinstance(o, Quad):
            out[k]["kind"] = 0
            out[k]["a"][:3], out[k]["u"][:3], out[k]["v"][:3] = o.q, o.u, o.v
        elif isinstance(o, Sphere):
            out[k]["kind"] = 1
            out[k]["a"] = [*o.center, o.radius]
        else:
            raise TypeError("book-3 lights are quads and spheres")
    return out


def flatten(world):
    """rrt_flatten_scene over `world`: (spheres, motion or None, quads or None, media or None,
    boundary_quads or None, materials, perlin or None, textures)."""
    b = _Builder()
    root = b.node(world)
    nodes = np.array(b.nodes, dtype=_lib.NODE_DTYPE)
    children = np.array(b.children if b.children else [0], dtype=np.uint32)
    lib = _lib.load()
    out = _lib.RrtBookScene()
    args = (_lib.ptr(nodes), len(nodes), _lib.ptr(children), len(b.children), root)
    _lib.check(lib.rrt_flatten_scene(*args, ctypes.byref(out)))
    spheres = np.zeros(out.n_spheres, dtype=_lib.SPHERE_DTYPE)
    motion = np.zeros((out.n_spheres, 4), dtype=np.float32)
    quads = np.zeros(out.n_quads, dtype=_lib.QUAD_DTYPE)
    media = np.zeros(out.n_media, dtype=_lib.MEDIUM_DTYPE)
    bquads = np.zeros(out.n_boundary_quads, dtype=_lib.QUAD_DTYPE)
    out.spheres, out.sphere_motion, out.sphere_cap = spheres.ctypes.data, motion.ctypes.data, out.n_spheres
    out.quads, out.quad_cap = quads.ctypes.data, out.n_quads
    out.media, out.media_cap = media.ctypes.data, out.n_media
    out.boundary_quads, out.boundary_quad_cap = bquads.ctypes.data, out.n_boundary_quads
    _lib.check(lib.rrt_flatten_scene(*args, ctypes.byref(out)))
    mats = np.concatenate(b.mats) if b.mats else np.zeros(0, dtype=_lib.MATERIAL_DTYPE)
    perlin = np.array(b.perlin, dtype=_lib.PERLIN_DTYPE) if b.perlin else None
    none = lambda a: a if len(a) else None  # noqa: E731
    return (spheres, motion if np.any(motion[:, :3]) else None, none(quads), none(media), none(bquads), mats, perlin,
            b.textures)


def build(world, camera: Camera, lights=None, book: int = 2, seed: int = 0, name: str = "world") -> SceneData:
    """A SceneData for `world` seen by `camera` with the given book's integrator: 1 (sky
    background, no time draw), 2 (`camera.background`, a time draw per camera ray) or 3 (the MIS
    integrator over `lights`; samples_per_pixel rounded down to a square, camera.rs:115-117)."""
    spheres, motion, quads, media, bquads, mats, perlin, textures = flatten(world)
    spp = int(camera.samples_per_pixel)
    flags = 0
    if book >= 2:
        flags |= _lib.FLAG_RAY_TIME
    if book == 3:
        if lights is None:
            raise ValueError("book 3 needs a light list")
        sq = int(math.sqrt(max(spp, 1)))
        spp = sq * sq
        flags |= _lib.FLAG_BOOK3
    cam = make_camera(aspect_ratio=camera.aspect_ratio, image_width=camera.image_width, samples_per_pixel=spp,
                      max_depth=camera.max_depth, vfov=camera.vfov, lookfrom=camera.lookfrom, lookat=camera.lookat,
                      vup=camera.vup, defocus_angle=camera.defocus_angle, focus_dist=camera.focus_dist,
                      background=None if book == 1 else camera.background, seed=seed, n_spheres=len(spheres))
    return SceneData(cam, spheres, mats, textures=textures, flags=flags, name=name, motion=motion, perlin=perlin,
                     quads=quads, media=media, boundary_quads=bquads,
                     lights=_light_records(lights) if book == 3 else None)
