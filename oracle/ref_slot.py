"""The reference's own GPU slot run on the MI355X — TEST INFRASTRUCTURE ONLY.

`oracle/_ref/ref_slot.hsaco` is the reference's CUDA_SOURCE kernel (src/cuda/mod.rs:15-335)
compiled unmodified by hipcc for gfx950 (oracle/Makefile; built only where /root/reference
exists, then travels to the GPU box as a build artefact). `oracle/build/libref_slot.so`
(ref_slot.cpp) restates the host side of `imp::render` (cuda/mod.rs:342-439) around it.

Only tests/ and bench.py's reference leg use this, to pin the backend statistically against
the reference's own GPU output and to time the reference kernel on the same GPU. The product
(rustraytrace_amd) never imports oracle/.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_float, c_int, c_uint32, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
HSACO = os.path.join(HERE, "_ref", "ref_slot.hsaco")
LIB_PATH = os.path.join(HERE, "build", "libref_slot.so")

_LIB = None


def available() -> bool:
    return os.path.exists(HSACO) and os.path.exists(LIB_PATH)


def load() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        import rustraytrace_amd  # loads torch first: one HIP runtime in the process (see _lib.load)

        rustraytrace_amd.load()
        lib = ctypes.CDLL(LIB_PATH)
        lib.ref_slot_render.restype = c_int
        lib.ref_slot_render.argtypes = [c_char_p, c_void_p, c_void_p, c_uint32, c_void_p, c_uint32, c_void_p,
                                        POINTER(c_float)]
        lib.ref_slot_last_error.restype = c_char_p
        lib.ref_slot_last_error.argtypes = []
        _LIB = lib
    return _LIB


def render(scene, return_ms: bool = False):
    """imp::render(camera, spheres, materials) up to the accum it hands to write_ppm_from_accum:
    (H, W, 4) float32, RGB sums over the samples, w = samples. Book-1 ABI scenes only (the kernel
    knows material kinds 0, 1, 2)."""
    if scene.textures or scene.motion is not None or scene.quads is not None:
        raise ValueError("the reference GPU slot renders book-1 sphere scenes only (cuda/mod.rs:217-301)")
    lib = load()
    cam = np.ascontiguousarray(scene.camera)
    sph = np.ascontiguousarray(scene.spheres)
    mat = np.ascontiguousarray(scene.materials)
    out = np.zeros((scene.height, scene.width, 4), dtype=np.float32)
    ms = c_float(0.0)
    rc = lib.ref_slot_render(HSACO.encode(), cam.ctypes.data, sph.ctypes.data, len(sph), mat.ctypes.data, len(mat),
                             out.ctypes.data, ctypes.byref(ms))
    if rc != 0:
        raise RuntimeError(f"reference GPU slot: {lib.ref_slot_last_error().decode()}")
    return (out, float(ms.value)) if return_ms else out
