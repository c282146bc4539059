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
