"""CPU tests of the C-ABI boundary (include/rrt_hip.h): the library loads, exports every declared
symbol, its struct layouts are the reference's #[repr(C)] layouts, host-side entry points work
without a GPU, and render entry points fail loudly (no CPU fallback) when no device exists."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import rustraytrace_amd as rrt
from rustraytrace_amd import _lib
from rustraytrace_amd.distributed import band_rows
from rustraytrace_amd.render import make_tile, tile_row_indices, tile_rows

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rrt_hip.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rrt_\w+)\s*\(", src)))


def test_every_declared_symbol_is_exported():
    lib = _lib.load()
    declared = header_functions()
    assert len(declared) >= 19
    assert sorted(_lib.EXPORTED_SYMBOLS) == declared
    for name in declared:
        assert hasattr(lib, name), name
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    exported = set(re.findall(r" T (rrt_\w+)", nm.stdout))
    assert set(declared) <= exported


def test_struct_layouts_match_reference_repr_c():
    # gpu/mod.rs:13-42: CameraUniform 9 x 16 B, SphereGpu 32 B, MaterialGpu 32 B
    assert _lib.CAMERA_DTYPE.itemsize == 144
    assert _lib.SPHERE_DTYPE.itemsize == 32 and _lib.SPHERE_DTYPE.fields["material_index"][1] == 16
    assert _lib.MATERIAL_DTYPE.itemsize == 32
    assert _lib.MATERIAL_DTYPE.fields["kind"][1] == 16 and _lib.MATERIAL_DTYPE.fields["ref_idx"][1] == 20
    assert _lib.CAMERA_DTYPE.fields["params_u"][1] == 128
    src = """
#include "rrt_hip.h"
#include <stddef.h>
_Static_assert(sizeof(RrtCamera) == 144, "camera");
_Static_assert(sizeof(RrtSphere) == 32, "sphere");
_Static_assert(sizeof(RrtMaterial) == 32, "material");
_Static_assert(offsetof(RrtMaterial, kind) == 16, "kind");
_Static_assert(sizeof(RrtTile) == 20, "tile");
_Static_assert(sizeof(RrtCounters) == 40, "counters");
int main(void) { return 0; }
"""
    r = subprocess.run(["gcc", "-std=c11", "-fsyntax-only", "-I", os.path.join(ROOT, "include"), "-x", "c", "-"],
                       input=src, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert ctypes.sizeof(_lib.RrtTile) == 20 and ctypes.sizeof(_lib.RrtCounters) == 40


def test_abi_version():
    assert _lib.load().rrt_hip_abi_version() == 11


def test_tile_rows_match_python_partition():
    for H in (1, 15, 16, 17, 225, 1080, 2160):
        for n in (1, 2, 3, 8):
            seen = []
            for r in range(n):
                t = make_tile(16, r, n, 0, 1)
                idx = tile_row_indices(H, t)
                assert tile_rows(H, t) == len(idx)
                assert np.array_equal(idx, band_rows(H, 16, r, n))
                seen.extend(idx.tolist())
            assert sorted(seen) == list(range(H))


def test_invalid_tile_rejected():
    with pytest.raises(rrt.RrtError):
        tile_rows(100, make_tile(0, 0, 1, 0, 1))
    with pytest.raises(rrt.RrtError):
        tile_rows(100, make_tile(16, 2, 2, 0, 1))
    with pytest.raises(rrt.RrtError):
        tile_rows(100, make_tile(16, 0, 1, 5, 1))


@pytest.mark.skipif(rrt.device_count() > 0, reason="checks the no-device error path")
def test_render_fails_loudly_without_device():
    scene = rrt.rtow(image_width=16, samples_per_pixel=1, max_depth=2)
    with pytest.raises(rrt.RrtError) as e:
        rrt.render(scene)
    assert e.value.code == -4 and "no HIP device" in str(e.value)
    with pytest.raises(rrt.RrtError):
        rrt.DeviceScene(scene)


def test_scene_validation_errors():
    scene = rrt.rtow(image_width=16, samples_per_pixel=1, max_depth=2)
    bad = scene.spheres.copy()
    bad["material_index"][0] = 10_000
    with pytest.raises(rrt.RrtError) as e:
        rrt.render(rrt.SceneData(scene.camera, bad, scene.materials))
    assert "material_index" in str(e.value) or "no HIP device" in str(e.value)


def test_write_ppm_file(tmp_path):
    acc = np.zeros((2, 3, 4), np.float32)
    acc[..., :3] = 0.25
    p = tmp_path / "x.ppm"
    rrt.write_ppm_from_accum(3, 2, acc, 1, str(p))
    assert p.read_bytes() == b"P3\n3 2\n255\n" + b"128 128 128\n" * 6


def test_overrides_semantics():
    base = rrt.build_in_one_weekend_scene()
    assert (base.width, base.height, base.spp, base.max_depth) == (1200, 675, 10, 20)  # gpu/mod.rs:125-128
    o = rrt.build_in_one_weekend_scene(dict(image_width=400, samples_per_pixel=7, max_depth=3, vfov=30.0,
                                            background=(0.1, 0.2, 0.3)))
    assert (o.width, o.height, o.spp, o.max_depth) == (400, 225, 7, 3)
    assert int(o.camera["params_u"][0, 3]) == 1 and np.allclose(o.camera["background"][0, :3], [0.1, 0.2, 0.3])
    assert np.array_equal(o.spheres, base.spheres)  # overrides never change the scene draw
    with pytest.raises(KeyError):
        _lib.make_overrides(bogus=1)


def test_cli_mirrors_main_rs():
    cli = os.path.join(ROOT, "rustraytrace_amd", "rrt")
    r = subprocess.run([cli, "--backend", "cpu"], capture_output=True, text=True)
    assert r.returncode == 2 and "CPU books renderer" in r.stderr
    if rrt.device_count() == 0:  # the default arm final_scene(400, 250, 4) renders (tests/test_gpu_cli.py)
        r = subprocess.run([cli, "--backend=hip", "the_next_week", "--image_width", "16", "--samples_per_pixel", "1"],
                           capture_output=True, text=True)
        assert r.returncode == 1 and "no HIP device" in r.stderr and "Could not load image" not in r.stderr
    r = subprocess.run([cli, "--backend=hip", "no_such_book"], capture_output=True, text=True)
    assert r.returncode == 2 and "the_rest_of_your_life" in r.stderr
    r = subprocess.run([cli, "--backend", "wgpu"], capture_output=True, text=True)
    assert r.returncode == 2
    if rrt.device_count() == 0:
        r = subprocess.run([cli, "--cuda", "in_one_weekend", "--image_width", "16", "--samples_per_pixel", "1"],
                           capture_output=True, text=True)
        assert r.returncode == 1 and "HIP render failed: no HIP device" in r.stderr


def test_accum_chunk_matches_oracle_default():
    from oracle import oracle

    assert _lib.load().rrt_accum_chunk() == oracle.DEFAULT_CHUNK
