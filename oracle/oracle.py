"""ctypes binding of oracle/build/librrt_oracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker / CPU baseline. The product (rustraytrace_amd) never imports it.
See rrt_oracle.cpp for the reference file:line each restated function follows.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_float, c_int, c_uint8, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "librrt_oracle.so")
TWIN, BOOKS = 0, 1
# Accum summation chunk of the HIP backend (include/rrt_hip.h rrt_accum_chunk): a frame of S
# samples uses K = DEFAULT_CHUNK halved while S <= 2K, down to DEFAULT_CHUNK / 4 (256 for S > 512,
# 128 for 256 < S <= 512, 64 below); (S-1)/K chunks of K samples, then chunks of max(1, K/4) for the
# tail (max(1, K/8) when S <= DEFAULT_CHUNK / 4); samples summed in order within a chunk, chunk sums added in order. The f32 kernel sums in
# that schedule; the f64 books kernel (RRT_FLAG_F64) sums every pixel's samples in sample order, the
# reference's own order (camera.rs:72-76), which is BOOKS' default here (chunk 0 = one chunk).
DEFAULT_CHUNK = 256

_LIB = None


def build() -> None:
    import subprocess

    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load() -> ctypes.CDLL:
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        build()
    lib = ctypes.CDLL(LIB_PATH)
    P = c_void_p
    lib.oracle_render.restype = c_int
    lib.oracle_render.argtypes = [P, P, c_uint32, P, c_uint32, P, c_uint32, P, c_uint32, c_int, c_uint32, c_uint32,
                                  c_uint32, c_uint32, c_int, P, P, P, c_uint32]
    lib.oracle_render_kbvh.restype = c_int
    lib.oracle_render_kbvh.argtypes = [P, P, c_uint32, P, c_uint32, P, c_uint32, P, c_uint32, P, c_uint32, c_uint32, P,
                                       c_uint32, c_uint32, c_uint32, c_uint32, c_uint32, c_int, P, P, P, c_uint32]
    lib.oracle_sin_f32.restype = None
    lib.oracle_sin_f32.argtypes = [c_uint32, P, P]
    lib.oracle_cos_f32.restype = None
    lib.oracle_cos_f32.argtypes = [c_uint32, P, P]
    lib.oracle_log_f32.restype = None
    lib.oracle_log_f32.argtypes = [c_uint32, P, P]
    lib.oracle_medium_u.restype = None
    lib.oracle_medium_u.argtypes = [c_uint32, P, P, P]
    lib.oracle_book2_textures.restype = None
    lib.oracle_book2_textures.argtypes = [c_int, P, c_double, c_double, c_uint32, P, P, P, P]
    lib.oracle_rtow_scene.restype = c_int
    lib.oracle_rtow_scene.argtypes = [c_uint64, c_int, P, P, P, P, P, c_uint32, P, P]
    lib.oracle_write_color.restype = None
    lib.oracle_write_color.argtypes = [P, P]
    lib.oracle_quantize_render_io.restype = None
    lib.oracle_quantize_render_io.argtypes = [c_uint32, P, c_uint32, P]
    lib.oracle_sphere_hit.restype = c_int
    lib.oracle_sphere_hit.argtypes = [c_int, P, c_double, P, P, c_double, c_double, P, P, P]
    lib.oracle_quad_hit.restype = c_int
    lib.oracle_quad_hit.argtypes = [c_int, P, P, P, P, P, c_double, c_double, P, P, P]
    lib.oracle_aabb_hit.restype = c_int
    lib.oracle_aabb_hit.argtypes = [c_int, P, P, P, P, c_double, c_double]
    lib.oracle_reflect_refract.restype = None
    lib.oracle_reflect_refract.argtypes = [c_int, P, P, c_double, P, P, P]
    lib.oracle_path_stream.restype = None
    lib.oracle_path_stream.argtypes = [c_uint32, c_uint32, c_uint32, c_uint32, P]
    lib.oracle_acos_atan2_f64.restype = None
    lib.oracle_acos_atan2_f64.argtypes = [c_uint32, P, P, P, P]
    lib.oracle_acos_atan2_f32.restype = None
    lib.oracle_acos_atan2_f32.argtypes = [c_float, c_float, P, P]
    _LIB = lib
    return lib


def _p(a):
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        if a.size == 0:
            return None
        assert a.flags["C_CONTIGUOUS"]
        return c_void_p(a.ctypes.data)
    return ctypes.cast(ctypes.byref(a), c_void_p)


class _Tex(ctypes.Structure):
    _fields_ = [("rgb8", POINTER(c_uint8)), ("width", ctypes.c_int32), ("height", ctypes.c_int32)]


class _Ext(ctypes.Structure):  # RrtSceneExt (include/rrt_hip.h)
    _fields_ = [("sphere_motion", c_void_p), ("perlin", c_void_p), ("n_perlin", c_uint32), ("n_quads", c_uint32),
                ("quads", c_void_p), ("media", c_void_p), ("n_media", c_uint32), ("n_boundary_quads", c_uint32),
                ("boundary_quads", c_void_p), ("lights", c_void_p), ("n_lights", c_uint32), ("_pad", c_uint32)]


def _ext(scene):
    """(pointer to RrtSceneExt or None, keep-alive) from the scene's book-2 motion / Perlin / quad data."""
    motion, perlin = getattr(scene, "motion", None), getattr(scene, "perlin", None)
    quads, media = getattr(scene, "quads", None), getattr(scene, "media", None)
    bquads, lights = getattr(scene, "boundary_quads", None), getattr(scene, "lights", None)
    if motion is None and perlin is None and quads is None and media is None and lights is None:
        return None, []
    e, keep = _Ext(), []
    if motion is not None:
        m = np.ascontiguousarray(motion, dtype=np.float32)
        keep.append(m)
        e.sphere_motion = m.ctypes.data
    if perlin is not None:
        t = np.ascontiguousarray(perlin)
        assert t.dtype.itemsize == 6144, "RrtPerlin tables"
        keep.append(t)
        e.perlin = t.ctypes.data
        e.n_perlin = len(t)
    if quads is not None:
        q = np.ascontiguousarray(quads)
        assert q.dtype.itemsize == 64, "RrtQuad records"
        keep.append(q)
        e.quads = q.ctypes.data
        e.n_quads = len(q)
    if media is not None:
        md = np.ascontiguousarray(media)
        assert md.dtype.itemsize == 48, "RrtMedium records"
        keep.append(md)
        e.media = md.ctypes.data
        e.n_media = len(md)
    if bquads is not None:
        bq = np.ascontiguousarray(bquads)
        assert bq.dtype.itemsize == 64, "RrtQuad records"
        keep.append(bq)
        e.boundary_quads = bq.ctypes.data
        e.n_boundary_quads = len(bq)
    if lights is not None:
        lt = np.ascontiguousarray(lights)
        assert lt.dtype.itemsize == 64, "RrtLight records"
        keep.append(lt)
        e.lights = lt.ctypes.data
        e.n_lights = len(lt)
    keep.append(e)
    return ctypes.cast(ctypes.byref(e), c_void_p), keep


def render(scene, mode=TWIN, rows=None, samples=None, threads=1, chunk=None):
    """Render `scene` (rustraytrace_amd.SceneData-like: camera/spheres/materials/textures/flags).

    rows = (y0, y1) image rows, samples = (s0, s1) sample range. Returns (accum, rays, sphere_tests)
    with accum float64 (y1-y0, W, 4); in TWIN mode every value is an exact float32 sum. chunk: the
    summation schedule (None: sequential for BOOKS, camera.rs:72-76; DEFAULT_CHUNK for TWIN)."""
    if chunk is None:
        chunk = 0 if (int(mode) & 0xff) == BOOKS else DEFAULT_CHUNK
    lib = load()
    W, H = int(scene.camera["params_f"][0, 1]), int(scene.camera["params_f"][0, 2])
    spp = max(int(scene.camera["params_f"][0, 3]), 1)
    y0, y1 = rows if rows is not None else (0, H)
    s0, s1 = samples if samples is not None else (0, spp)
    accum = np.zeros((y1 - y0, W, 4), dtype=np.float64)
    keep = [np.ascontiguousarray(t, dtype=np.uint8) for t in scene.textures]
    tex = (_Tex * max(len(keep), 1))()
    for i, t in enumerate(keep):
        tex[i].rgb8 = t.ctypes.data_as(POINTER(c_uint8))
        tex[i].height, tex[i].width = t.shape[0], t.shape[1]
    rays, tests = c_uint64(0), c_uint64(0)
    ext, keep_ext = _ext(scene)
    rc = lib.oracle_render(_p(scene.camera), _p(scene.spheres), len(scene.spheres), _p(scene.materials),
                           len(scene.materials), ctypes.cast(tex, c_void_p) if keep else None, len(keep), ext,
                           int(scene.flags), int(mode), y0, y1, s0, s1, int(threads), _p(accum),
                           ctypes.byref(rays), ctypes.byref(tests), int(chunk))
    del keep_ext
    if rc != 0:
        raise RuntimeError(f"oracle_render failed ({rc})")
    return accum, rays.value, tests.value


def render_kbvh(scene, nodes, order, layout, rows=None, samples=None, threads=1, chunk=DEFAULT_CHUNK):
    """TWIN arithmetic, closest hits by walking the kernel's own BVH in the kernel's order
    (nodes/order/info from rustraytrace_amd.render.build_bvh; `layout` = that info dict — its
    node_stride and n_unbounded, the media tested after the walk — or the node stride in bytes:
    80 / 64 BVH2, 128 BVH4, for trees without unbounded media). Same return as render()."""
    stride = int(layout["node_stride"]) if isinstance(layout, dict) else int(layout)
    n_unbounded = int(layout.get("n_unbounded", 0)) if isinstance(layout, dict) else 0
    if stride not in (32, 80, 128):
        raise ValueError(f"render_kbvh: node stride {stride} (pass build_bvh's info dict)")
    lib = load()
    W, H = int(scene.camera["params_f"][0, 1]), int(scene.camera["params_f"][0, 2])
    spp = max(int(scene.camera["params_f"][0, 3]), 1)
    y0, y1 = rows if rows is not None else (0, H)
    s0, s1 = samples if samples is not None else (0, spp)
    accum = np.zeros((y1 - y0, W, 4), dtype=np.float64)
    keep = [np.ascontiguousarray(t, dtype=np.uint8) for t in scene.textures]
    tex = (_Tex * max(len(keep), 1))()
    for i, t in enumerate(keep):
        tex[i].rgb8 = t.ctypes.data_as(POINTER(c_uint8))
        tex[i].height, tex[i].width = t.shape[0], t.shape[1]
    nodes = np.ascontiguousarray(nodes, dtype=np.uint8)
    order = np.ascontiguousarray(order, dtype=np.uint32)
    n_nodes = nodes.size // stride
    rays, tests = c_uint64(0), c_uint64(0)
    ext, keep_ext = _ext(scene)
    rc = lib.oracle_render_kbvh(_p(scene.camera), _p(scene.spheres), len(scene.spheres), _p(scene.materials),
                                len(scene.materials), ctypes.cast(tex, c_void_p) if keep else None, len(keep), ext,
                                int(scene.flags), _p(nodes), n_nodes, stride, _p(order), n_unbounded, y0, y1, s0, s1,
                                int(threads), _p(accum), ctypes.byref(rays), ctypes.byref(tests), int(chunk))
    del keep_ext
    if rc != 0:
        raise RuntimeError(f"oracle_render_kbvh failed ({rc})")
    return accum, rays.value, tests.value


def rtow_scene(seed=0x5EED_1234, grid_half=11):
    """Restated gpu::build_in_one_weekend_scene sphere/material list (no camera)."""
    lib = load()
    n, sseed = c_uint32(0), c_uint32(0)
    lib.oracle_rtow_scene(seed, grid_half, None, None, None, None, None, 0, ctypes.byref(n), ctypes.byref(sseed))
    k = n.value
    cr = np.zeros((k, 4), np.float32)
    mi = np.zeros(k, np.uint32)
    af = np.zeros((k, 4), np.float32)
    kind = np.zeros(k, np.uint32)
    ri = np.zeros(k, np.float32)
    rc = lib.oracle_rtow_scene(seed, grid_half, _p(cr), _p(mi), _p(af), _p(kind), _p(ri), k, ctypes.byref(n),
                               ctypes.byref(sseed))
    assert rc == 0
    return dict(center_radius=cr, material_index=mi, albedo_fuzz=af, kind=kind, ref_idx=ri, sample_seed=sseed.value)


def write_color(pixel_color_scaled):
    lib = load()
    v = np.ascontiguousarray(pixel_color_scaled, dtype=np.float64)
    out = np.zeros(3, np.int32)
    lib.oracle_write_color(_p(v), _p(out))
    return out


def quantize_render_io(accum_f32, spp):
    lib = load()
    a = np.ascontiguousarray(accum_f32, dtype=np.float32).reshape(-1, 4)
    out = np.zeros((a.shape[0], 3), np.uint8)
    lib.oracle_quantize_render_io(a.shape[0], _p(a), spp, _p(out))
    return out


def sphere_hit(center, radius, o, d, tmin=0.001, tmax=float("inf"), f32=False):
    lib = load()
    t = c_double(0)
    n = np.zeros(3)
    front = c_int(0)
    c, oo, dd = (np.asarray(x, np.float64) for x in (center, o, d))
    hit = lib.oracle_sphere_hit(int(f32), _p(c), float(radius), _p(oo), _p(dd), tmin, tmax, ctypes.byref(t), _p(n),
                                ctypes.byref(front))
    return (t.value, n, bool(front.value)) if hit else None


def quad_hit(q, u, v, o, d, tmin=0.001, tmax=float("inf"), f32=False):
    """Quad::hit (the_next_week/quad.rs:61-87) -> (t, normal, front_face) or None."""
    lib = load()
    t = c_double(0)
    n = np.zeros(3)
    front = c_int(0)
    a = [np.asarray(x, np.float64) for x in (q, u, v, o, d)]
    hit = lib.oracle_quad_hit(int(f32), *(_p(x) for x in a), tmin, tmax, ctypes.byref(t), _p(n), ctypes.byref(front))
    return (t.value, n, bool(front.value)) if hit else None


def aabb_hit(lo, hi, o, d, tmin=0.001, tmax=float("inf"), f32=False):
    lib = load()
    a = [np.asarray(x, np.float64) for x in (lo, hi, o, d)]
    return bool(lib.oracle_aabb_hit(int(f32), *(_p(x) for x in a), tmin, tmax))


def reflect_refract(v, n, eta, cosine, ri, f32=False):
    lib = load()
    vv, nn = np.asarray(v, np.float64), np.asarray(n, np.float64)
    refl, refr = np.zeros(3), np.zeros(3)
    sc = np.array([cosine, ri, 0.0])
    lib.oracle_reflect_refract(int(f32), _p(vv), _p(nn), float(eta), _p(refl), _p(refr), _p(sc))
    return refl, refr, sc[2]


def path_stream(seed, pixel, sample, count):
    lib = load()
    out = np.zeros(count, np.uint32)
    lib.oracle_path_stream(seed, pixel, sample, count, _p(out))
    return out


def acos_atan2_f32(x, y):
    lib = load()
    a, b = c_float(0), c_float(0)
    lib.oracle_acos_atan2_f32(x, y, ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


def acos_atan2_f64(x, y):
    """BOOKS' f64 acos(x) and atan2(y, x) (fdlibm's algorithms restated) at each element."""
    lib = load()
    xs = np.ascontiguousarray(x, dtype=np.float64).ravel()
    ys = np.ascontiguousarray(np.broadcast_to(y, xs.shape), dtype=np.float64).ravel()
    a, b = np.zeros_like(xs), np.zeros_like(xs)
    lib.oracle_acos_atan2_f64(xs.size, _p(xs), _p(ys), _p(a), _p(b))
    return a, b


def cos_f32(x):
    """The f32 Cephes cos of the kernel (rrt_cosf) at each element of x."""
    lib = load()
    xs = np.ascontiguousarray(x, dtype=np.float32).ravel()
    out = np.zeros_like(xs)
    lib.oracle_cos_f32(xs.size, _p(xs), _p(out))
    return out


def log_f32(x):
    """The f32 Cephes log of the kernel (rrt_logf) at each element of x."""
    lib = load()
    xs = np.ascontiguousarray(x, dtype=np.float32).ravel()
    out = np.zeros_like(xs)
    lib.oracle_log_f32(xs.size, _p(xs), _p(out))
    return out


def medium_u(seg, medium):
    """The media free-flight uniforms u(seg, medium) (include/rrt_hip.h RrtMedium)."""
    lib = load()
    sg = np.ascontiguousarray(seg, dtype=np.uint64).ravel()
    md = np.ascontiguousarray(np.broadcast_to(medium, sg.shape), dtype=np.uint32)
    out = np.zeros(sg.size, dtype=np.float32)
    lib.oracle_medium_u(sg.size, _p(sg), _p(md), _p(out))
    return out


def sin_f32(x):
    """The f32 Cephes sin of the kernel (rrt_sinf) at each element of x."""
    lib = load()
    xs = np.ascontiguousarray(x, dtype=np.float32).ravel()
    out = np.zeros_like(xs)
    lib.oracle_sin_f32(xs.size, _p(xs), _p(out))
    return out


def book2_textures(perlin_table, points, scale=4.0, inv_scale=1.0 / 0.32, f32=True):
    """Perlin::noise, NoiseTexture::value and CheckerTexture parity at points (n, 3) for one
    RrtPerlin table (f32=True: the twin arithmetic, else f64). Returns (noise, value, even)."""
    lib = load()
    t = np.ascontiguousarray(perlin_table)
    pts = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 3)
    n = len(pts)
    noise, value, even = np.zeros(n), np.zeros(n), np.zeros(n, np.int32)
    lib.oracle_book2_textures(int(f32), _p(t), float(scale), float(inv_scale), n, _p(pts), _p(noise), _p(value),
                              _p(even))
    return noise, value, even.astype(bool)
