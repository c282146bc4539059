"""The f32 kernel's short reciprocal (rrt_kernel.hip recip_rn: v_rcp_f32 and one Newton step by
fma; clamped_slope for the ray constants) is the IEEE quotient, and its short square root
(sqrt_rn_big) the IEEE root over its domain: exhaustive over every f32 bit pattern on the device, through the test-only entry point rrt_testing_recip_check. The parity suites
then hold the kernel bit-exact against the oracle's IEEE divisions."""
import ctypes

import pytest

from rustraytrace_amd import _lib


@pytest.mark.gpu
def test_short_reciprocal_is_the_ieee_quotient():
    lib = _lib.load()
    out = (ctypes.c_uint64 * 3)(7, 7, 7)
    _lib.check(lib.rrt_testing_recip_check(out))
    assert list(out) == [0, 0, 0], f"recip_rn {out[0]}, clamped_slope {out[1]}, sqrt_rn_big {out[2]} mismatches"
