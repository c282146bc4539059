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
