"""ctypes binding of librrt_hip.so (include/rrt_hip.h).

This is the Python twin of the cgo/Rust `extern "C"` shim a reference maintainer would add
(see INTEGRATION.md): plain pointers and sizes, numpy arrays for the #[repr(C)] structs of
src/gpu/mod.rs:13-42. There is no fallback: if the shared object is missing or fails to
load, every entry raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int32, c_size_t, c_uint8, c_uint32, c_uint64, c_void_p

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RRT_LIB_PATH") or os.path.join(PKG_DIR, "librrt_hip.so")  # override: experiments only

# ---- #[repr(C)] layouts (gpu/mod.rs:13-42) as numpy dtypes ------------------------------------
CAMERA_DTYPE = np.dtype(
    [
        ("origin", "<f4", 4),
        ("pixel00", "<f4", 4),
        ("pixel_delta_u", "<f4", 4),
        ("pixel_delta_v", "<f4", 4),
        ("u", "<f4", 4),
        ("v", "<f4", 4),
        ("background", "<f4", 4),
        ("params_f", "<f4", 4),
        ("params_u", "<u4", 4),
    ]
)
SPHERE_DTYPE = np.dtype([("center_radius", "<f4", 4), ("material_index", "<u4"), ("_pad", "<u4", 3)])
MATERIAL_DTYPE = np.dtype([("albedo_fuzz", "<f4", 4), ("kind", "<u4"), ("ref_idx", "<f4"), ("_pad", "<u4", 2)])
assert CAMERA_DTYPE.itemsize == 144 and SPHERE_DTYPE.itemsize == 32 and MATERIAL_DTYPE.itemsize == 32

MAT_LAMBERTIAN, MAT_METAL, MAT_DIELECTRIC, MAT_TEXTURED_LAMBERTIAN, MAT_DIFFUSE_LIGHT = range(5)
FLAG_RAY_TIME = 0x1
FLAG_QUIET = 0x2
FLAG_BOOK3 = 0x4
FLAG_F64 = 0x8  # the books path's f64 arithmetic (include/rrt_hip.h RRT_FLAG_F64)

# Every symbol include/rrt_hip.h declares (checked by tests/test_abi.py).
EXPORTED_SYMBOLS = (
    "rrt_hip_render",
    "rrt_hip_last_error",
    "rrt_hip_abi_version",
    "rrt_accum_chunk",
    "rrt_scene_create",
    "rrt_scene_destroy",
    "rrt_tile_rows",
    "rrt_tile_row_index",
    "rrt_render_tile_async",
    "rrt_scene_read_counters",
    "rrt_scene_reset_counters",
    "rrt_scene_count_work",
    "rrt_scene_bvh_info",
    "rrt_build_bvh",
    "rrt_build_in_one_weekend_scene",
    "rrt_make_camera",
    "rrt_apply_overrides",
    "rrt_write_ppm_from_accum",
    "rrt_format_ppm_from_accum",
    "rrt_quantize_accum",
    "rrt_hip_render_rgb8",
    "rrt_hip_render_rgb8_ex",
    "rrt_quantize_accum_books",
    "rrt_quantize_accum_async",
    "rrt_format_pnm_from_rgb8",
    "rrt_write_pnm_from_rgb8",
    "rrt_hip_render_ex",
    "rrt_scene_create_ex",
    "rrt_build_bvh_ex",
    "rrt_build_next_week_scene",
    "rrt_build_rest_of_your_life_scene",
    "rrt_flatten_scene",
    "rrt_device_count",
    "rrt_hip_render_f64",
    "rrt_render_tile_f64_async",
    "rrt_quantize_accum_books_f64",
    "rrt_testing_device_wrap",
    "rrt_testing_f64_layout",
    "rrt_testing_recip_check",
    "rrt_testing_trig32_check",
    "rrt_testing_sqrt64_check",
)


class RrtTexture(ctypes.Structure):
    _fields_ = [("rgb8", POINTER(c_uint8)), ("width", c_int32), ("height", c_int32)]


# == RrtPerlin (include/rrt_hip.h): 256 x float4 random vectors + 3 x 256 u16 permutations (+pad)
PERLIN_DTYPE = np.dtype([("randvec", "<f4", (256, 4)), ("perm_x", "<u2", 256), ("perm_y", "<u2", 256),
                         ("perm_z", "<u2", 256), ("_pad", "<u2", 256)])


# == RrtQuad (include/rrt_hip.h): corner q, edges u, v (xyz + pad), material index; 64 B
QUAD_DTYPE = np.dtype([("q", "<f4", 4), ("u", "<f4", 4), ("v", "<f4", 4), ("material_index", "<u4"),
                       ("_pad", "<u4", 3)])


# == RrtLight (include/rrt_hip.h): book-3 MIS light, kind 0 quad (a = q, u, v) / 1 sphere (a = c, r); 64 B
LIGHT_DTYPE = np.dtype([("kind", "<u4"), ("_pad", "<u4", 3), ("a", "<f4", 4), ("u", "<f4", 4), ("v", "<f4", 4)])

# == RrtMedium (include/rrt_hip.h): boundary sphere or quad range, phase material, density; 48 B
MEDIUM_DTYPE = np.dtype([("sphere", "<f4", 4), ("boundary_kind", "<u4"), ("first", "<u4"), ("count", "<u4"),
                         ("material_index", "<u4"), ("density", "<f4"), ("_pad", "<u4", 3)])


class RrtSceneExt(ctypes.Structure):
    _fields_ = [("sphere_motion", c_void_p), ("perlin", c_void_p), ("n_perlin", c_uint32), ("n_quads", c_uint32),
                ("quads", c_void_p), ("media", c_void_p), ("n_media", c_uint32), ("n_boundary_quads", c_uint32),
                ("boundary_quads", c_void_p), ("lights", c_void_p), ("n_lights", c_uint32), ("_pad", c_uint32)]


class RrtBookScene(ctypes.Structure):
    _fields_ = [("camera", ctypes.c_uint8 * 144), ("spheres", c_void_p), ("sphere_motion", c_void_p),
                ("materials", c_void_p), ("quads", c_void_p), ("perlin", c_void_p), ("media", c_void_p),
                ("boundary_quads", c_void_p), ("lights", c_void_p)] + [
        (f, c_uint32) for f in ("sphere_cap", "n_spheres", "material_cap", "n_materials", "quad_cap", "n_quads",
                                "perlin_cap", "n_perlin", "media_cap", "n_media", "boundary_quad_cap",
                                "n_boundary_quads", "light_cap", "n_lights", "uses_texture0", "flags")]


# == RrtSceneNode (include/rrt_hip.h): one node of the books' object graph, f64 payload; 112 B
NODE_DTYPE = np.dtype([("kind", "<u4"), ("material", "<u4"), ("first", "<u4"), ("count", "<u4"),
                       ("a", "<f8", 4), ("b", "<f8", 4), ("c", "<f8", 4)])
NODE_SPHERE, NODE_QUAD, NODE_LIST, NODE_BVH, NODE_TRANSLATE, NODE_ROTATE_Y, NODE_CONSTANT_MEDIUM = range(7)


class RrtOverrides(ctypes.Structure):
    _fields_ = [
        ("has_aspect_ratio", c_int32), ("aspect_ratio", c_double),
        ("has_image_width", c_int32), ("image_width", c_int32),
        ("has_samples_per_pixel", c_int32), ("samples_per_pixel", c_int32),
        ("has_max_depth", c_int32), ("max_depth", c_int32),
        ("has_vfov", c_int32), ("vfov", c_double),
        ("has_lookfrom", c_int32), ("lookfrom", c_double * 3),
        ("has_lookat", c_int32), ("lookat", c_double * 3),
        ("has_vup", c_int32), ("vup", c_double * 3),
        ("has_defocus_angle", c_int32), ("defocus_angle", c_double),
        ("has_focus_dist", c_int32), ("focus_dist", c_double),
        ("has_background", c_int32), ("background", c_double * 3),
    ]


class RrtTile(ctypes.Structure):
    _fields_ = [
        ("band_rows", c_uint32),
        ("rank", c_uint32),
        ("n_ranks", c_uint32),
        ("sample_begin", c_uint32),
        ("sample_end", c_uint32),
    ]


class RrtCounters(ctypes.Structure):
    _fields_ = [
        ("rays", c_uint64),
        ("paths", c_uint64),
        ("node_visits", c_uint64),
        ("box_tests", c_uint64),
        ("sphere_tests", c_uint64),
    ]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


class RrtBvhInfo(ctypes.Structure):
    _fields_ = [
        ("n_nodes", c_uint32),
        ("n_leaves", c_uint32),
        ("max_depth", c_uint32),
        ("max_leaf_size", c_uint32),
        ("node_bytes", c_uint64),
        ("prim_bytes", c_uint64),
        ("width", c_uint32),
        ("max_leaf_param", c_uint32),
        ("node_stride", c_uint32),
        ("n_unbounded", c_uint32),
    ]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_ if not k.startswith("_")}


class RrtError(RuntimeError):
    """A non-zero return of the C-ABI (the Rust shim's Err(rrt_hip_last_error()))."""

    def __init__(self, code: int, message: str):
        super().__init__(f"rrt error {code}: {message}")
        self.code = code


_LIB = None


def load() -> ctypes.CDLL:
    """Load librrt_hip.so from the package directory; raise if it is missing."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no CPU fallback for the HIP backend)"
        )
    # One HIP runtime per process: torch bundles its own libamdhip64 (soname libamdhip64.so.7)
    # which satisfies our DT_NEEDED when it is loaded first. Loaded the other way round,
    # torch would map a second runtime and lose the device ("One runtime").
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    P = c_void_p
    sig = {
        "rrt_hip_render": (c_int32, [P, P, c_uint32, P, c_uint32, P, c_uint32, c_uint32, c_uint32, c_uint32, P]),
        "rrt_hip_last_error": (c_char_p, []),
        "rrt_hip_abi_version": (c_uint32, []),
        "rrt_accum_chunk": (c_uint32, []),
        "rrt_scene_create": (c_int32, [P, P, c_uint32, P, c_uint32, P, c_uint32, c_uint32, c_int32, P]),
        "rrt_scene_destroy": (c_int32, [P]),
        "rrt_tile_rows": (c_int32, [c_uint32, P, P]),
        "rrt_tile_row_index": (c_int32, [c_uint32, P, c_uint32, P]),
        "rrt_render_tile_async": (c_int32, [P, P, P, P]),
        "rrt_scene_read_counters": (c_int32, [P, P]),
        "rrt_scene_reset_counters": (c_int32, [P]),
        "rrt_scene_count_work": (c_int32, [P, P, P]),
        "rrt_scene_bvh_info": (c_int32, [P, P]),
        "rrt_build_bvh": (c_int32, [P, c_uint32, c_uint32, c_uint32, P, c_size_t, P, P]),
        "rrt_build_in_one_weekend_scene": (c_int32, [P, c_uint64, c_int32, P, P, P, c_uint32, P]),
        "rrt_make_camera": (
            c_int32,
            [c_double, c_int32, c_int32, c_int32, c_double, P, P, P, c_double, c_double, P, c_uint32, c_uint32, P],
        ),
        "rrt_apply_overrides": (c_int32, [P, c_int32] + [P] * 12),
        "rrt_write_ppm_from_accum": (c_int32, [c_uint32, c_uint32, P, c_uint32, c_char_p]),
        "rrt_format_ppm_from_accum": (c_int32, [c_uint32, c_uint32, P, c_uint32, P, c_size_t, P]),
        "rrt_quantize_accum": (c_int32, [c_uint32, c_uint32, P, c_uint32, P]),
        "rrt_quantize_accum_books": (c_int32, [c_uint32, c_uint32, P, c_uint32, P]),
        "rrt_hip_render_rgb8": (c_int32, [P, P, c_uint32, P, c_uint32, P, c_uint32, c_uint32, c_uint32, c_uint32, P]),
        "rrt_hip_render_rgb8_ex": (c_int32, [P, P, c_uint32, P, c_uint32, P, c_uint32, P, c_uint32, c_uint32, c_uint32,
                                             P]),
        "rrt_quantize_accum_async": (c_int32, [c_uint32, P, c_uint32, P, P]),
        "rrt_format_pnm_from_rgb8": (c_int32, [c_uint32, c_uint32, P, c_int32, P, c_size_t, P]),
        "rrt_write_pnm_from_rgb8": (c_int32, [c_uint32, c_uint32, P, c_int32, c_char_p]),
        "rrt_hip_render_ex": (c_int32, [P, P, c_uint32, P, c_uint32, P, c_uint32, P, c_uint32, c_uint32, c_uint32, P]),
        "rrt_scene_create_ex": (c_int32, [P, P, c_uint32, P, c_uint32, P, c_uint32, P, c_uint32, c_int32, P]),
        "rrt_build_bvh_ex": (c_int32, [P, c_uint32, P, c_uint32, c_uint32, P, c_size_t, P, P]),
        "rrt_build_next_week_scene": (c_int32, [c_int32, P, c_uint64, P]),
        "rrt_build_rest_of_your_life_scene": (c_int32, [P, c_uint64, P]),
        "rrt_flatten_scene": (c_int32, [P, c_uint32, P, c_uint32, c_uint32, P]),
        "rrt_device_count": (c_int32, [P]),
        "rrt_hip_render_f64": (c_int32, [P, P, c_uint32, P, c_uint32, P, c_uint32, c_uint32, c_uint32, c_uint32, P]),
        "rrt_render_tile_f64_async": (c_int32, [P, P, P, P]),
        "rrt_quantize_accum_books_f64": (c_int32, [c_uint32, c_uint32, P, c_uint32, P]),
        "rrt_testing_device_wrap": (None, [c_int32]),
        "rrt_testing_f64_layout": (None, [c_int32]),
        "rrt_testing_recip_check": (c_int32, [P]),
        "rrt_testing_trig32_check": (c_int32, [P]),
        "rrt_testing_sqrt64_check": (c_int32, [P]),
    }
    experiment = "RRT_LIB_PATH" in os.environ  # A/B of older builds: tolerate symbols they lack
    for name, (res, args) in sig.items():
        if experiment and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def check(rc: int) -> None:
    if rc != 0:
        msg = load().rrt_hip_last_error()
        raise RrtError(rc, msg.decode() if msg else "")


def ptr(a) -> c_void_p:
    """Address of a numpy array / ctypes object (None for empty / None)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        if a.size == 0:
            return None
        assert a.flags["C_CONTIGUOUS"], "arrays passed through the C-ABI must be C-contiguous"
        return c_void_p(a.ctypes.data)
    return ctypes.cast(ctypes.byref(a), c_void_p)


def make_overrides(**kw) -> RrtOverrides:
    """RenderOverrides (config.rs:1-14) with the given fields set to Some(value)."""
    ov = RrtOverrides()
    for k, v in kw.items():
        if v is None:
            continue
        if not hasattr(ov, "has_" + k):
            raise KeyError(f"unknown override {k!r}")
        setattr(ov, "has_" + k, 1)
        if k in ("lookfrom", "lookat", "vup", "background"):
            getattr(ov, k)[:] = [float(x) for x in v]
        else:
            setattr(ov, k, v)
    return ov
