"""CPU checks of the reference-GPU-slot harness (oracle/ref_slot.cpp, oracle/Makefile): the
code object is a gfx950 build of the reference kernel, no extracted reference source is kept,
and the launcher exports its entry points. No GPU calls (tests/test_gpu_ref_slot.py runs it)."""
import ctypes
import os

import pytest

from oracle import ref_slot

REF_DIR = os.path.join(os.path.dirname(ref_slot.HSACO))


@pytest.mark.skipif(not os.path.isdir(REF_DIR), reason="oracle/_ref not built")
def test_ref_dir_holds_only_the_code_object():
    # the Makefile deletes its scratch copy of CUDA_SOURCE after compiling it
    assert set(os.listdir(REF_DIR)) <= {"ref_slot.hsaco"}, os.listdir(REF_DIR)


@pytest.mark.skipif(not os.path.exists(ref_slot.HSACO), reason="oracle/_ref/ref_slot.hsaco not built")
def test_code_object_targets_gfx950_and_holds_the_render_kernel():
    data = open(ref_slot.HSACO, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    assert b"render" in data  # extern "C" __global__ void render(...) (cuda/mod.rs:303)


@pytest.mark.skipif(not os.path.exists(ref_slot.LIB_PATH), reason="oracle/build/libref_slot.so not built")
def test_launcher_exports_its_entry_points():
    import rustraytrace_amd

    rustraytrace_amd.load()  # torch's HIP runtime first (one runtime per process)
    lib = ctypes.CDLL(ref_slot.LIB_PATH)
    for sym in ("ref_slot_render", "ref_slot_last_error"):
        assert hasattr(lib, sym)


def test_refuses_scenes_beyond_book_1():
    import rustraytrace_amd as rrt

    scene = rrt.earth_light(image_width=32, samples_per_pixel=1)
    with pytest.raises(ValueError, match="book-1"):
        ref_slot.render(scene)
