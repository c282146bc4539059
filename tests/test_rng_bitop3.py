"""The kernels' xoshiro128+ step with three-input xors (rrt_device.h rng_next, RRT_RNG_BITOP3)
produces the same state sequence and outputs as the two-input form the oracle restates
(oracle/rrt_oracle.cpp PathRng): checked on random states, vectorised in numpy."""
import numpy as np


def _rotl(x, k):
    return ((x << np.uint32(k)) | (x >> np.uint32(32 - k))).astype(np.uint32)


def _step_two_input(a, b, c, d):
    r = (a + d).astype(np.uint32)
    t = (b << np.uint32(9)).astype(np.uint32)
    c = c ^ a
    d = d ^ b
    b = b ^ c
    a = a ^ d
    c = c ^ t
    d = _rotl(d, 11)
    return r, a, b, c, d


def _step_three_input(a, b, c, d):
    r = (a + d).astype(np.uint32)
    t = (b << np.uint32(9)).astype(np.uint32)
    db = d ^ b
    nb = b ^ c ^ a  # xor3_32(b, c, a)
    nc = c ^ a ^ t  # xor3_32(c, a, t)
    return r, a ^ db, nb, nc, _rotl(db, 11)


def test_three_input_xoshiro_step_equals_two_input():
    rng = np.random.default_rng(1234)
    s2 = [rng.integers(0, 2**32, size=1 << 16, dtype=np.uint64).astype(np.uint32) for _ in range(4)]
    s2[3] |= np.uint32(1)
    s3 = [x.copy() for x in s2]
    with np.errstate(over="ignore"):
        for _ in range(64):
            r2, *s2 = _step_two_input(*s2)
            r3, *s3 = _step_three_input(*s3)
            assert np.array_equal(r2, r3)
            for x, y in zip(s2, s3):
                assert np.array_equal(x, y)


def test_centred_draw_is_the_shifted_draw_minus_2_23():
    """rng_next_centred: (int32)(r + 2^31) >> 8 == (r >> 8) - 2^23 for every r (checked on a
    random sample and the edges)."""
    rng = np.random.default_rng(7)
    r = np.concatenate([rng.integers(0, 2**32, size=1 << 20, dtype=np.uint64),
                        np.array([0, 1, 255, 256, 2**31 - 1, 2**31, 2**31 + 255, 2**32 - 256, 2**32 - 1],
                                 dtype=np.uint64)])
    want = (r >> np.uint64(8)).astype(np.int64) - 2**23
    rc = ((r + 2**31) % 2**32).astype(np.uint32).view(np.int32).astype(np.int64)
    got = rc >> 8  # arithmetic shift of the signed value
    assert np.array_equal(got, want)


def _f32(x):
    return np.float32(x)


def _fma32(x, y, z):
    # exact for these operands: products of 24-bit integers (or their 2^-23 scalings) and sums of
    # such squares are exact in f64, so the single rounding to f32 is the fma's
    return (np.float64(x) * np.float64(y) + np.float64(z)).astype(np.float32)


def test_scaled_rejection_tests_decide_as_the_unscaled_ones():
    """The f32 kernel's rejection loops test |p|^2 * 2^46 on the 2^23-scaled candidates
    (rrt_kernel.hip random_unit_vector, camera_ray's disk loop): same decisions and the same
    accepted components as rnd_pm1's candidates tested against 1."""
    rng = np.random.default_rng(11)
    n = 1 << 18
    a, b, c = (rng.integers(-2**23, 2**23, size=n) for _ in range(3))
    # the edges of the ball / disk: |p|^2 at and around 1, and zero components
    a[:4], b[:4], c[:4] = [2**23 - 1, -2**23, 0, 0], [0, 0, 0, 1], [0, 0, 0, 0]
    fa, fb, fc = (x.astype(np.float32) for x in (a, b, c))
    pa, pb, pc = (_fma32(x.astype(np.float64) + 2**23, 2.0**-23, -1.0) for x in (a, b, c))  # rnd_pm1
    assert np.array_equal(pa, (fa * _f32(2.0**-23)).astype(np.float32))
    l_old = _fma32(pc, pc, _fma32(pb, pb, (pa * pa).astype(np.float32)))
    l_new = _fma32(fc, fc, _fma32(fb, fb, (fa * fa).astype(np.float32)))
    assert np.array_equal(l_old * np.float32(2.0**46), l_new)
    assert np.array_equal((l_old > 0) & (l_old <= 1), (l_new > 0) & (l_new <= _f32(2.0**46)))
    d_old = _fma32(pb, pb, (pa * pa).astype(np.float32))
    d_new = _fma32(fb, fb, (fa * fa).astype(np.float32))
    assert np.array_equal(d_old < 1, d_new < _f32(2.0**46))
