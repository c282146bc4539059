"""Render entry points over the C-ABI, mirroring the reference's Rust surface:

* `render_in_one_weekend()`  == cuda::render_in_one_weekend (cuda/mod.rs:337-340, 442-445)
* `render(scene)`            == cuda::imp::render(camera, &spheres, &materials) (cuda/mod.rs:342-439)
                                returning the RGBA accum instead of printing it
* `write_ppm_from_accum`     == render_io::write_ppm_from_accum (render_io.rs:3-31)
* `DeviceScene`              device-resident scene for benches / multi-rank hosts
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import _lib
from .scenes import SceneData, build_in_one_weekend_scene, COMMITTED_OVERRIDES


def _textures(scene: SceneData):
    if not scene.textures:
        return None, 0, []
    arr = (_lib.RrtTexture * len(scene.textures))()
    keep = []
    for i, t in enumerate(scene.textures):
        t = np.ascontiguousarray(t, dtype=np.uint8)
        assert t.ndim == 3 and t.shape[2] == 3, "textures are (H, W, 3) RGB8"
        keep.append(t)
        arr[i].rgb8 = t.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        arr[i].height, arr[i].width = int(t.shape[0]), int(t.shape[1])
    return arr, len(scene.textures), keep


def scene_ext(scene: SceneData):
    """(RrtSceneExt or None, keep-alive list) for the book-2 data of `scene` (motion, Perlin, quads)."""
    quads, media = getattr(scene, "quads", None), getattr(scene, "media", None)
    bquads, lights = getattr(scene, "boundary_quads", None), getattr(scene, "lights", None)
    if scene.motion is None and scene.perlin is None and quads is None and media is None and lights is None:
        return None, []
    ext = _lib.RrtSceneExt()
    keep = []
    if scene.motion is not None:
        m = np.ascontiguousarray(scene.motion, dtype=np.float32)
        assert m.shape == (len(scene.spheres), 4), "motion is (n_spheres, 4) float32"
        keep.append(m)
        ext.sphere_motion = m.ctypes.data
    if scene.perlin is not None:
        t = np.ascontiguousarray(scene.perlin, dtype=_lib.PERLIN_DTYPE)
        keep.append(t)
        ext.perlin = t.ctypes.data
        ext.n_perlin = len(t)
    if quads is not None:
        q = np.ascontiguousarray(quads, dtype=_lib.QUAD_DTYPE)
        keep.append(q)
        ext.quads = q.ctypes.data
        ext.n_quads = len(q)
    if media is not None:
        md = np.ascontiguousarray(media, dtype=_lib.MEDIUM_DTYPE)
        keep.append(md)
        ext.media = md.ctypes.data
        ext.n_media = len(md)
    if bquads is not None:
        bq = np.ascontiguousarray(bquads, dtype=_lib.QUAD_DTYPE)
        keep.append(bq)
        ext.boundary_quads = bq.ctypes.data
        ext.n_boundary_quads = len(bq)
    if lights is not None:
        lt = np.ascontiguousarray(lights, dtype=_lib.LIGHT_DTYPE)
        keep.append(lt)
        ext.lights = lt.ctypes.data
        ext.n_lights = len(lt)
    return ext, keep


def render(scene: SceneData, spp: Optional[int] = None, n_gpus: int = 1, quiet: bool = True) -> np.ndarray:
    """Render `scene` on `n_gpus` GPUs; returns the RGBA float32 accum (H, W, 4), w = sample count."""
    lib = _lib.load()
    accum = np.zeros((scene.height, scene.width, 4), dtype=np.float32)
    tex, ntex, keep = _textures(scene)
    ext, keep_ext = scene_ext(scene)
    flags = scene.flags | (_lib.FLAG_QUIET if quiet else 0)
    _lib.check(lib.rrt_hip_render_ex(_lib.ptr(scene.camera), _lib.ptr(scene.spheres), len(scene.spheres),
                                     _lib.ptr(scene.materials), len(scene.materials),
                                     ctypes.cast(tex, ctypes.c_void_p) if tex is not None else None, ntex,
                                     ctypes.byref(ext) if ext is not None else None,
                                     int(spp or 0), int(n_gpus), flags, _lib.ptr(accum)))
    del keep, keep_ext
    return accum


def render_f64(scene: SceneData, spp: Optional[int] = None, n_gpus: int = 1, quiet: bool = True) -> np.ndarray:
    """rrt_hip_render_f64: the books path's own f64 arithmetic (RRT_FLAG_F64, book-1 scenes);
    returns the RGBA float64 accum (H, W, 4) of f64 sums, w = sample count."""
    lib = _lib.load()
    if getattr(scene, "motion", None) is not None or getattr(scene, "quads", None) is not None:
        raise ValueError("render_f64: book-1 scenes only (RRT_FLAG_F64)")
    accum = np.zeros((scene.height, scene.width, 4), dtype=np.float64)
    tex, ntex, keep = _textures(scene)
    flags = scene.flags | _lib.FLAG_F64 | (_lib.FLAG_QUIET if quiet else 0)
    _lib.check(lib.rrt_hip_render_f64(_lib.ptr(scene.camera), _lib.ptr(scene.spheres), len(scene.spheres),
                                      _lib.ptr(scene.materials), len(scene.materials),
                                      ctypes.cast(tex, ctypes.c_void_p) if tex is not None else None, ntex,
                                      int(spp or 0), int(n_gpus), flags, _lib.ptr(accum)))
    del keep
    return accum


def render_rgb8(scene: SceneData, spp: Optional[int] = None, n_gpus: int = 1, quiet: bool = True) -> np.ndarray:
    """rrt_hip_render_rgb8_ex: render and quantise on the device (render_io.rs quantiser);
    returns (H, W, 3) uint8, identical to quantize_accum(render(scene)) at the same spp, for
    every book (the scene's RrtSceneExt — motion, Perlin tables, quads, media, lights — is passed)."""
    lib = _lib.load()
    out = np.zeros((scene.height, scene.width, 3), dtype=np.uint8)
    tex, ntex, keep = _textures(scene)
    ext, keep_ext = scene_ext(scene)
    flags = scene.flags | (_lib.FLAG_QUIET if quiet else 0)
    _lib.check(lib.rrt_hip_render_rgb8_ex(_lib.ptr(scene.camera), _lib.ptr(scene.spheres), len(scene.spheres),
                                          _lib.ptr(scene.materials), len(scene.materials),
                                          ctypes.cast(tex, ctypes.c_void_p) if tex is not None else None, ntex,
                                          ctypes.byref(ext) if ext is not None else None,
                                          int(spp or 0), int(n_gpus), flags, _lib.ptr(out)))
    del keep, keep_ext
    return out


def quantize_accum_async(n_pixels: int, d_accum_ptr: int, samples_per_pixel: int, d_rgb8_ptr: int,
                         stream_ptr: int = 0) -> None:
    """rrt_quantize_accum_async on device pointers (e.g. torch tensors' data_ptr())."""
    _lib.check(_lib.load().rrt_quantize_accum_async(int(n_pixels), ctypes.c_void_p(d_accum_ptr), int(samples_per_pixel),
                                                    ctypes.c_void_p(d_rgb8_ptr), ctypes.c_void_p(stream_ptr)))


def format_pnm_from_rgb8(width: int, height: int, rgb8: np.ndarray, binary: bool = False) -> bytes:
    """P3 (byte-identical to format_ppm_from_accum of the same image) or binary P6."""
    lib = _lib.load()
    rgb8 = np.ascontiguousarray(rgb8, dtype=np.uint8)
    assert rgb8.size == width * height * 3
    n = ctypes.c_size_t(0)
    _lib.check(lib.rrt_format_pnm_from_rgb8(width, height, _lib.ptr(rgb8), int(binary), None, 0, ctypes.byref(n)))
    buf = ctypes.create_string_buffer(n.value)
    _lib.check(lib.rrt_format_pnm_from_rgb8(width, height, _lib.ptr(rgb8), int(binary), buf, n.value,
                                            ctypes.byref(n)))
    return buf.raw[: n.value]


def write_pnm_from_rgb8(width: int, height: int, rgb8: np.ndarray, binary: bool = False, path: str = "-") -> None:
    rgb8 = np.ascontiguousarray(rgb8, dtype=np.uint8)
    assert rgb8.size == width * height * 3
    _lib.check(_lib.load().rrt_write_pnm_from_rgb8(width, height, _lib.ptr(rgb8), int(binary), path.encode()))


def render_in_one_weekend(path: str = "-", n_gpus: int = 1, overrides: Optional[dict] = None) -> None:
    """cuda::render_in_one_weekend: RTOW scene under config::OVERRIDES -> P3 PPM on stdout (or `path`)."""
    scene = build_in_one_weekend_scene(COMMITTED_OVERRIDES if overrides is None else overrides)
    accum = render(scene, n_gpus=n_gpus, quiet=False)
    write_ppm_from_accum(scene.width, scene.height, accum, scene.spp, path)


def write_ppm_from_accum(width: int, height: int, accum: np.ndarray, samples_per_pixel: int, path: str = "-") -> None:
    accum = np.ascontiguousarray(accum, dtype=np.float32)
    assert accum.size == width * height * 4
    _lib.check(_lib.load().rrt_write_ppm_from_accum(width, height, _lib.ptr(accum), samples_per_pixel,
                                                    path.encode()))


def format_ppm_from_accum(width: int, height: int, accum: np.ndarray, samples_per_pixel: int) -> bytes:
    lib = _lib.load()
    accum = np.ascontiguousarray(accum, dtype=np.float32)
    assert accum.size == width * height * 4
    n = ctypes.c_size_t(0)
    _lib.check(lib.rrt_format_ppm_from_accum(width, height, _lib.ptr(accum), samples_per_pixel, None, 0,
                                             ctypes.byref(n)))
    buf = ctypes.create_string_buffer(n.value)
    _lib.check(lib.rrt_format_ppm_from_accum(width, height, _lib.ptr(accum), samples_per_pixel, buf, n.value,
                                             ctypes.byref(n)))
    return buf.raw[: n.value]


def quantize_accum(width: int, height: int, accum: np.ndarray, samples_per_pixel: int) -> np.ndarray:
    accum = np.ascontiguousarray(accum, dtype=np.float32)
    out = np.zeros((height, width, 3), dtype=np.uint8)
    _lib.check(_lib.load().rrt_quantize_accum(width, height, _lib.ptr(accum), samples_per_pixel, _lib.ptr(out)))
    return out


def quantize_accum_books(width: int, height: int, accum: np.ndarray, samples_per_pixel: int) -> np.ndarray:
    """color.rs:6-32 write_color (the books CPU path's f64 quantiser) over a float accum:
    (H, W, 3) uint8. Differs from quantize_accum (render_io.rs) only on non-finite sums
    (+inf -> 255 here, 0 there) and where f64 vs f32 scaling crosses a byte boundary."""
    accum = np.ascontiguousarray(accum, dtype=np.float32)
    out = np.zeros((height, width, 3), dtype=np.uint8)
    _lib.check(_lib.load().rrt_quantize_accum_books(width, height, _lib.ptr(accum), samples_per_pixel, _lib.ptr(out)))
    return out


def quantize_accum_books_f64(width: int, height: int, accum: np.ndarray, samples_per_pixel: int) -> np.ndarray:
    """color.rs:6-32 write_color over f64 sums (render_f64): the books path's bytes, (H, W, 3) uint8."""
    accum = np.ascontiguousarray(accum, dtype=np.float64)
    out = np.zeros((height, width, 3), dtype=np.uint8)
    _lib.check(_lib.load().rrt_quantize_accum_books_f64(width, height, _lib.ptr(accum), samples_per_pixel,
                                                        _lib.ptr(out)))
    return out


def device_count() -> int:
    n = ctypes.c_int32(0)
    _lib.check(_lib.load().rrt_device_count(ctypes.byref(n)))
    return n.value


def tile_rows(height: int, tile) -> int:
    n = ctypes.c_uint32(0)
    _lib.check(_lib.load().rrt_tile_rows(height, ctypes.byref(tile), ctypes.byref(n)))
    return n.value


def tile_row_indices(height: int, tile) -> np.ndarray:
    lib = _lib.load()
    rows = tile_rows(height, tile)
    out = np.empty(rows, dtype=np.int64)
    r = ctypes.c_uint32(0)
    for i in range(rows):
        _lib.check(lib.rrt_tile_row_index(height, ctypes.byref(tile), i, ctypes.byref(r)))
        out[i] = r.value
    return out


def build_bvh(scene: SceneData, width: int = 0, max_leaf: int = 0):
    """The BVH rrt_scene_create builds for `scene` (host only): (node bytes uint8, leaf-order
    permutation uint32, info dict). width/max_leaf 0 = the library defaults."""
    lib = _lib.load()
    info = _lib.RrtBvhInfo()
    n = len(scene.spheres)
    ext, keep = scene_ext(scene)
    n_prims = n + (0 if ext is None else ext.n_quads + ext.n_media)
    if ext is not None or np.isin(scene.materials["kind"], (5, 6)).any():
        width = 2  # book-2 scenes render with the BVH2 kernel variant (rrt_scene_create_ex)
    def build(nodes_p, cap, order_p):
        if ext is None:
            return lib.rrt_build_bvh(_lib.ptr(scene.spheres), n, width, max_leaf, nodes_p, cap, order_p,
                                     ctypes.byref(info))
        return lib.rrt_build_bvh_ex(_lib.ptr(scene.spheres), n, ctypes.byref(ext), width, max_leaf, nodes_p, cap,
                                    order_p, ctypes.byref(info))

    _lib.check(build(None, 0, None))
    nodes = np.zeros(info.node_bytes, dtype=np.uint8)
    order = np.zeros(max(n_prims, 1), dtype=np.uint32)
    _lib.check(build(_lib.ptr(nodes), nodes.size, _lib.ptr(order)))
    return nodes, order[:n_prims], info.as_dict()


def decode_bvh2(nodes: np.ndarray, stride: int):
    """Decode build_bvh's width-2 node bytes (rrt_internal.h; stride = info["node_stride"]: 80 =
    GNode, sign-ordered lo/hi/lo planes, 32 = GNodeH, f16 planes): per node and child, box lo/hi (n, 2, 3),
    first primitive or child node (n, 2) and leaf count (n, 2; 0 = internal)."""
    words = stride // 4
    f = nodes.view(np.float32).reshape(-1, words)
    u = nodes.view(np.uint32).reshape(-1, words)
    if stride == 80:
        box = f[:, :18].reshape(-1, 2, 3, 3)  # [node][child][axis][lo, hi, lo]
        assert np.array_equal(box[..., 2], box[..., 0])
        lo, hi, links = box[..., 0].copy(), box[..., 1].copy(), u[:, 18:20]
    elif stride == 32:  # GNodeH: f16 planes, lo | hi << 16 per child and axis
        box = nodes.view(np.float16).reshape(-1, 16)[:, :12].astype(np.float32).reshape(-1, 2, 3, 2)  # [node][child][axis][lo, hi]
        lo, hi, links = box[..., 0].copy(), box[..., 1].copy(), u[:, 6:8]
    else:
        raise ValueError(f"decode_bvh2: stride {stride}")
    return lo, hi, (links & 0x0FFFFFFF).astype(np.int64), (links >> 28).astype(np.int64)


def make_tile(band_rows=16, rank=0, n_ranks=1, sample_begin=0, sample_end=0) -> _lib.RrtTile:
    t = _lib.RrtTile()
    t.band_rows, t.rank, t.n_ranks, t.sample_begin, t.sample_end = band_rows, rank, n_ranks, sample_begin, sample_end
    return t


class DeviceScene:
    """RrtScene*: scene + BVH resident on one device; renders tiles asynchronously on a stream."""

    def __init__(self, scene: SceneData, device: int = 0, f64: bool = False):
        """f64=True: the books path's f64 kernel (RRT_FLAG_F64, book-1 scenes)."""
        lib = _lib.load()
        self.scene = scene
        flags = scene.flags | (_lib.FLAG_F64 if f64 else 0)
        self._lib = lib
        self._h = ctypes.c_void_p()
        tex, ntex, keep = _textures(scene)
        ext, keep_ext = scene_ext(scene)
        texp = ctypes.cast(tex, ctypes.c_void_p) if tex is not None else None
        if ext is None:
            _lib.check(lib.rrt_scene_create(_lib.ptr(scene.camera), _lib.ptr(scene.spheres), len(scene.spheres),
                                            _lib.ptr(scene.materials), len(scene.materials), texp, ntex,
                                            flags, int(device), ctypes.byref(self._h)))
        else:
            _lib.check(lib.rrt_scene_create_ex(_lib.ptr(scene.camera), _lib.ptr(scene.spheres), len(scene.spheres),
                                               _lib.ptr(scene.materials), len(scene.materials), texp, ntex,
                                               ctypes.byref(ext), flags, int(device), ctypes.byref(self._h)))
        del keep, keep_ext

    def close(self):
        if self._h:
            self._lib.rrt_scene_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def tile(band_rows=16, rank=0, n_ranks=1, sample_begin=0, sample_end=None, spp=None) -> _lib.RrtTile:
        t = _lib.RrtTile()
        t.band_rows, t.rank, t.n_ranks = band_rows, rank, n_ranks
        t.sample_begin = sample_begin
        t.sample_end = sample_end if sample_end is not None else (sample_begin + (spp or 0))
        return t

    def tile_rows(self, tile) -> int:
        return tile_rows(self.scene.height, tile)

    def tile_row_indices(self, tile) -> np.ndarray:
        return tile_row_indices(self.scene.height, tile)

    def render_tile_async(self, tile, d_accum_ptr: int, stream_ptr: int = 0) -> None:
        _lib.check(self._lib.rrt_render_tile_async(self._h, ctypes.byref(tile), ctypes.c_void_p(d_accum_ptr),
                                                   ctypes.c_void_p(stream_ptr)))

    def render_tile_f64_async(self, tile, d_accum_ptr: int, stream_ptr: int = 0) -> None:
        """rrt_render_tile_f64_async: f64 sums (rows x W x 4 doubles) of a DeviceScene(f64=True)."""
        _lib.check(self._lib.rrt_render_tile_f64_async(self._h, ctypes.byref(tile), ctypes.c_void_p(d_accum_ptr),
                                                       ctypes.c_void_p(stream_ptr)))

    def counters(self) -> dict:
        c = _lib.RrtCounters()
        _lib.check(self._lib.rrt_scene_read_counters(self._h, ctypes.byref(c)))
        return c.as_dict()

    def reset_counters(self) -> None:
        _lib.check(self._lib.rrt_scene_reset_counters(self._h))

    def count_work(self, tile) -> dict:
        c = _lib.RrtCounters()
        _lib.check(self._lib.rrt_scene_count_work(self._h, ctypes.byref(tile), ctypes.byref(c)))
        return c.as_dict()

    def bvh_info(self) -> dict:
        b = _lib.RrtBvhInfo()
        _lib.check(self._lib.rrt_scene_bvh_info(self._h, ctypes.byref(b)))
        return b.as_dict()
