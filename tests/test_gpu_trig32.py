"""The f64 books kernel decides the earth texture's texel from f32 acosf / atanf enclosures of the
fdlibm angles (rrt_books64.hip texel_bytes64) and falls back to fdlibm when an enclosure straddles
a texel edge. The enclosures hold when the device's acosf / atanf stay within the kernel's error
bounds: checked here over every f32 argument of their domains (through the test-only entry point
rrt_testing_trig32_check), with a factor of two to spare. The f64 parity suite
(tests/test_gpu_books64.py: C4 and the full-class scene, bit for bit against the books path) then
covers the decision itself, fallbacks included."""
import ctypes

import pytest

from rustraytrace_amd import _lib


@pytest.mark.gpu
def test_f32_trig_errors_within_the_enclosure_bounds():
    lib = _lib.load()
    out = (ctypes.c_double * 4)(-1.0, -1.0, -1.0, -1.0)
    _lib.check(lib.rrt_testing_trig32_check(out))
    e_acos, e_atan, b_acos, b_atan = list(out)
    print(f"acosf max error {e_acos:.3e} (bound {b_acos:.3e}), atanf max error {e_atan:.3e} (bound {b_atan:.3e})")
    assert 0.0 < e_acos <= 0.5 * b_acos
    assert 0.0 < e_atan <= 0.5 * b_atan


@pytest.mark.gpu
def test_f64_sqrt_without_scaling_equals_the_library_root():
    """rrt_books64.hip sqrt64_big: LLVM's f64 root expansion without its v_ldexp_f64 scalings, which are
    identities for arguments >= 2^-767; taken when no lane of the wave holds a smaller nonzero one.
    Bit for bit against the library root on 2^28 arguments (random and nearly-square mantissas over
    every exponent of the range, +-0, +inf)."""
    lib = _lib.load()
    out = (ctypes.c_uint64 * 2)(7, 7)
    _lib.check(lib.rrt_testing_sqrt64_check(out))
    bad, n = list(out)
    print(f"sqrt64_big: {bad} of {n} roots differ from the library's")
    assert n > (1 << 27) and bad == 0
