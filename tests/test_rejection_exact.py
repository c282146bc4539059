"""The f64 books kernel's rejection loops (rrt_books64.hip random_unit_vector, random_in_unit_disk)
decide each candidate on the integer S = sum (a_i - 2^23)^2 (a_i the draws' 24-bit values): accept
when 0 < S <= 2^46 (sphere) or S < 2^46 (disk). This checks that decision against the reference's f64
comparison (vec3.rs:172-189: 1e-160 < x*x + y*y + z*z <= 1, x*x + y*y < 1, with x = a * 2^-24 * 2 - 1
as random_double_range(-1, 1) computes it) on 2e5 random draws and on draws placed on and around the
unit sphere / circle, where S is within a few units of 2^46."""
import numpy as np


def _pm1(a):  # random_double_range(-1, 1) of the 24-bit draw a, as the reference evaluates it in f64
    return np.float64(a) * 2.0 ** -24 * 2.0 + -1.0


def ref_unit(a, b, c):
    x, y, z = _pm1(a), _pm1(b), _pm1(c)
    lensq = x * x + y * y + z * z
    return bool(1e-160 < lensq <= 1.0)


def ref_disk(a, b):
    x, y = _pm1(a), _pm1(b)
    return bool(x * x + y * y < 1.0)


def int_unit(a, b, c):
    S = sum((int(v) - 2 ** 23) ** 2 for v in (a, b, c))
    return 0 < S <= 2 ** 46


def int_disk(a, b):
    return sum((int(v) - 2 ** 23) ** 2 for v in (a, b)) < 2 ** 46


def test_random_draws_decide_as_f64():
    rng = np.random.default_rng(11)
    for a, b, c in rng.integers(0, 2 ** 24, size=(200_000, 3)):
        assert int_unit(a, b, c) == ref_unit(a, b, c)
        assert int_disk(a, b) == ref_disk(a, b)
    assert not int_unit(2 ** 23, 2 ** 23, 2 ** 23) and not ref_unit(2 ** 23, 2 ** 23, 2 ** 23)  # 1e-160 < |p|^2
    # the centred value and its f64 image are exact: x = (a - 2^23) * 2^-23
    for a in (0, 1, 2 ** 23 - 1, 2 ** 23, 2 ** 24 - 1):
        assert _pm1(a) == np.float64(a - 2 ** 23) * 2.0 ** -23


def test_draws_on_the_sphere_decide_as_f64():
    rng = np.random.default_rng(12)
    n = 0
    for _ in range(20_000):
        fa, fb = (int(v) for v in rng.integers(-(2 ** 23), 2 ** 23, size=2))
        rest = 2 ** 46 - fa * fa - fb * fb
        if rest >= 0:
            c0 = int(np.sqrt(float(rest)))
            for fc in (c0 - 2, c0 - 1, c0, c0 + 1, c0 + 2, -c0, -c0 - 1):
                if -(2 ** 23) <= fc < 2 ** 23:
                    n += 1
                    a, b, c = fa + 2 ** 23, fb + 2 ** 23, fc + 2 ** 23
                    assert int_unit(a, b, c) == ref_unit(a, b, c), (fa, fb, fc)
        r2 = 2 ** 46 - fa * fa
        b0 = int(np.sqrt(float(r2)))
        for fb2 in (b0 - 1, b0, b0 + 1, -b0, -b0 - 1):
            if -(2 ** 23) <= fb2 < 2 ** 23:
                assert int_disk(fa + 2 ** 23, fb2 + 2 ** 23) == ref_disk(fa + 2 ** 23, fb2 + 2 ** 23), (fa, fb2)
    assert n > 50_000
    # exact boundary points: S = 2^46 is accepted by the sphere test (<= 1) and rejected by the disk (< 1)
    assert int_unit(0, 2 ** 23, 2 ** 23) and ref_unit(0, 2 ** 23, 2 ** 23)
    assert not int_disk(0, 2 ** 23) and not ref_disk(0, 2 ** 23)


# The kernel's f32 pre-decision (rrt_books64.hip in_ball, RRT_F64_REJ32): the f32 sum of squares
# fma(c, c, fma(b, b, a*a)) of the exact centred coordinates decides outside the band
# 2^46 (1 +- 2^-21); inside it the integers decide. Emulated exactly: a*a rounded to f32, each fma
# as the exact f64 sum (<= 49 significant bits) rounded once to f32.
LO, HI = np.float32(2.0 ** 46 * (1 - 2.0 ** -21)), np.float32(2.0 ** 46 * (1 + 2.0 ** -21))


def f32_decision(a, b, c, disk):
    a, b, c = (np.asarray(v, np.int64) - 2 ** 23 for v in (a, b, c))
    p = (a.astype(np.float64) ** 2).astype(np.float32)
    p = (b.astype(np.float64) ** 2 + p.astype(np.float64)).astype(np.float32)
    s32 = (c.astype(np.float64) ** 2 + p.astype(np.float64)).astype(np.float32)
    accept = (s32 <= LO) & ((s32 > 0) | disk)
    band = (s32 > LO) & (s32 <= HI)
    return accept, band


def test_f32_pre_decision_matches_the_integers():
    rng = np.random.default_rng(11)
    n = 400_000
    a, b, c = (rng.integers(0, 2 ** 24, n) for _ in range(3))
    # and candidates on and around the sphere / circle: S within +-2^30 of 2^46
    t = rng.normal(size=(n, 3))
    t /= np.linalg.norm(t, axis=1, keepdims=True)
    r = 2.0 ** 23 * (1 + rng.uniform(-2.0 ** -17, 2.0 ** -17, n))
    near = np.clip(np.round(t * r[:, None]) + 2 ** 23, 0, 2 ** 24 - 1).astype(np.int64)
    for disk in (False, True):
        for A, B, C in ((a, b, c), (near[:, 0], near[:, 1], near[:, 2] if not disk else np.full(n, 2 ** 23))):
            acc, band = f32_decision(A, B, C, disk)
            S = sum((np.asarray(v, np.int64) - 2 ** 23) ** 2 for v in (A, B, C))
            exact = (S < 2 ** 46) if disk else ((S > 0) & (S <= 2 ** 46))
            decided = ~band
            assert np.array_equal(acc[decided], exact[decided])
            assert band.mean() < 0.05  # the band is rare even among candidates placed at the boundary
    acc, band = f32_decision(a, b, c, False)
    assert band.mean() < 1e-5  # random candidates: ~7e-7 in the band
    assert f32_decision([2 ** 23], [2 ** 23], [2 ** 23], False)[0][0] == False  # S = 0 rejected (1e-160 < |p|^2)
    assert f32_decision([2 ** 23], [2 ** 23], [2 ** 23], True)[0][0] == True    # the disk takes S = 0
