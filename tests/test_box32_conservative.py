"""The f64 books kernel's box test (rustraytrace_amd/csrc/rrt_box32.h: f32 arithmetic on the f32 /
f16 BVH planes, widened per ray) must never reject a box that the f64 ray meets, or the kernel could
miss the books path's closest hit (aabb.rs:52-85 only prunes; sphere.rs:24-51 decides). The header is
compiled for the host here (tests/box32/box32_harness.cpp, the same source the device compiles) and
checked against
  * exact rational arithmetic (fractions) on corner, edge and face grazes, origins on and near the
    planes, far origins (|o| up to 1e5), direction components 0, -0 and tiny, closest hits just past
    the entry, and
  * a long-double sweep of 6e6 adversarial rays (the harness's box32_sweep),
with the hardware reciprocal's estimate emulated up to 2 ulps off 1/x either way.
Cases on an axis the test clamps (|1/d_a| > 2^64) with the origin within 4u|o_a| of that axis's plane
are outside the contract: the product's stored planes are grown past every primitive box by more
than that (rrt_host.cpp BoxSlack), so such a ray misses the primitive anyway."""
import ctypes
import os
import subprocess
from fractions import Fraction

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("box32") / "box32.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-shared", "-fPIC",
                    os.path.join(HERE, "box32", "box32_harness.cpp"), "-o", so], check=True)
    L = ctypes.CDLL(so)
    L.box32_sweep.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
    P = ctypes.c_void_p
    L.box32_eval.argtypes = [ctypes.c_uint32, P, P, P, P, P, P, P]
    L.box32_set_rcp_ulps.argtypes = [ctypes.c_int]
    return L


ULPS = [-2, -1, 0, 1, 2]  # the device's v_rcp_f32 estimate emulated this many ulps from 1/x


def _eval(L, o, d, lo, hi, closest):
    n = len(o)
    o, d = np.ascontiguousarray(o, np.float64), np.ascontiguousarray(d, np.float64)
    lo, hi = np.ascontiguousarray(lo, np.float32), np.ascontiguousarray(hi, np.float32)
    closest = np.ascontiguousarray(closest, np.float64)
    acc = np.zeros(n, np.uint8)
    tn = np.zeros(n, np.float32)
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    L.box32_eval(n, ptr(o), ptr(d), ptr(lo), ptr(hi), ptr(closest), ptr(acc), ptr(tn))
    return acc.astype(bool)


def _exact(o, d, lo, hi, closest):
    """1: the exact interval [max(entry, 0.001), min(exit, closest)] is nonempty, 0: empty, -1:
    outside the contract (clamped axis, origin within 4u|o_a| of its plane)."""
    te, tx = Fraction(1, 1000), (Fraction(closest) if np.isfinite(closest) else None)
    for a in range(3):
        L, H, oa, da = Fraction(float(lo[a])), Fraction(float(hi[a])), Fraction(float(o[a])), Fraction(float(d[a]))
        with np.errstate(divide="ignore"):
            q = np.float32(1.0) / np.float32(d[a])
        if abs(float(q)) > 2.0 ** 64:
            tol = 4 * Fraction(1, 2 ** 24) * abs(oa) + Fraction(1, 2 ** 120)
            if abs(oa - L) <= tol or abs(oa - H) <= tol:
                return -1
        if da == 0:
            if oa < L or oa > H:
                return 0
            continue
        t0, t1 = (L - oa) / da, (H - oa) / da
        t0, t1 = min(t0, t1), max(t0, t1)
        te = max(te, t0)
        tx = t1 if tx is None else min(tx, t1)
    return 1 if (tx is None or te <= tx) else 0


def _cases(n, seed):
    rng = np.random.default_rng(seed)
    o = np.zeros((n, 3))
    d = np.zeros((n, 3))
    lo = np.zeros((n, 3), np.float32)
    hi = np.zeros((n, 3), np.float32)
    closest = np.full(n, np.inf)
    for i in range(n):
        R = [1.0, 1e3, 2e4][i % 3]
        c = rng.uniform(-R, R, 3)
        e = np.exp(rng.uniform(np.log(1e-6), np.log(1e3), 3))
        lo[i] = np.minimum(np.float32(c - e), np.float32(c + e))
        hi[i] = np.maximum(np.float32(c - e), np.float32(c + e))
        kind = i % 4  # corner, edge, face, interior point
        p = lo[i] + (hi[i] - lo[i]) * rng.uniform(0, 1, 3)
        for a in range(3 - kind if kind < 3 else 0):
            p[a] = lo[i][a] if rng.uniform() < 0.5 else hi[i][a]
        if rng.uniform() < 0.15:  # origin on one of the box's planes, inside the box
            o[i] = lo[i] + (hi[i] - lo[i]) * rng.uniform(0, 1, 3)
            a = rng.integers(3)
            o[i][a] = lo[i][a] if rng.uniform() < 0.5 else hi[i][a]
        else:
            o[i] = p + rng.choice([-1, 1], 3) * rng.uniform(0, 1, 3) * np.exp(rng.uniform(np.log(1e-3), np.log(1e5)))
        d[i] = (p - o[i]) * np.exp(rng.uniform(np.log(1e-3), np.log(1e3)))
        m = rng.uniform()
        if m < 0.1:
            d[i][rng.integers(3)] = 0.0
        elif m < 0.15:
            d[i][rng.integers(3)] = -0.0
        elif m < 0.2:
            d[i][rng.integers(3)] = rng.choice([-1, 1]) * np.exp(rng.uniform(np.log(1e-30), np.log(1e-8)))
        if rng.uniform() < 0.4:  # nudge by f64 ulps
            a = rng.integers(3)
            for _ in range(rng.integers(1, 4)):
                d[i][a] = np.nextafter(d[i][a], -np.inf if rng.uniform() < 0.5 else np.inf)
        if rng.uniform() < 0.5:  # the closest hit just past the box entry
            te = Fraction(1, 1000)
            for a in range(3):
                if d[i][a] != 0:
                    t0 = (Fraction(float(lo[i][a])) - Fraction(o[i][a])) / Fraction(d[i][a])
                    t1 = (Fraction(float(hi[i][a])) - Fraction(o[i][a])) / Fraction(d[i][a])
                    te = max(te, min(t0, t1))
            if te > Fraction(10) ** 300:
                continue
            closest[i] = float(te)
            for _ in range(rng.integers(0, 3)):
                closest[i] = np.nextafter(closest[i], np.inf)
    return o, d, lo, hi, closest


def test_widened_f32_box_test_accepts_every_exactly_met_box(lib):
    o, d, lo, hi, closest = _cases(4000, 20261017)
    exact = np.array([_exact(o[i], d[i], lo[i], hi[i], closest[i]) for i in range(len(o))])
    inside = exact >= 0
    assert inside.mean() > 0.9 and (exact == 1).sum() > 1000  # the cases mostly meet the box
    for k in ULPS:
        lib.box32_set_rcp_ulps(k)
        acc = _eval(lib, o, d, lo, hi, closest)
        missed = np.flatnonzero((exact == 1) & ~acc)
        assert missed.size == 0, f"rcp {k:+d} ulp: {missed.size} met boxes rejected, first {missed[:5]}"
    lib.box32_set_rcp_ulps(0)


def test_widening_stays_tight(lib):
    # rays aimed just outside a box (a face point pushed out by 1e-3 of the distance scale): every
    # one the exact slab misses by more than 1e-4 (|t_entry| + max |o_a / d_a|) — about 800 times
    # the widening 8u(|t| + |o * inv|) — is rejected
    rng = np.random.default_rng(5)
    n = 2000
    lo = np.float32(rng.uniform(-100, 100, (n, 3)))
    hi = np.float32(lo + np.exp(rng.uniform(np.log(1e-3), np.log(10), (n, 3))))
    o = rng.uniform(-300, 300, (n, 3))
    p = lo + (hi - lo) * rng.uniform(0, 1, (n, 3))
    a = rng.integers(3, size=n)
    scale = np.abs(o).max(1) + 10.0
    for i in range(n):
        up = rng.uniform() < 0.5
        p[i][a[i]] = (hi[i][a[i]] + 1e-3 * scale[i]) if up else (lo[i][a[i]] - 1e-3 * scale[i])
    d = p - o
    lib.box32_set_rcp_ulps(2)
    acc = _eval(lib, o, d, lo, hi, np.full(n, np.inf))
    lib.box32_set_rcp_ulps(0)
    far = 0
    for i in range(n):
        te, tx = Fraction(1, 1000), None
        for k in range(3):
            t0 = (Fraction(float(lo[i][k])) - Fraction(o[i][k])) / Fraction(d[i][k])
            t1 = (Fraction(float(hi[i][k])) - Fraction(o[i][k])) / Fraction(d[i][k])
            te, tx = max(te, min(t0, t1)), (max(t0, t1) if tx is None else min(tx, max(t0, t1)))
        margin = 1e-4 * (abs(float(te)) + max(abs(o[i][k] / d[i][k]) for k in range(3)))
        if float(te - tx) > margin:
            far += 1
            assert not acc[i], f"case {i}: misses by {float(te - tx):.3g} yet accepted"
    assert far > n // 4


def test_sweep_six_million_adversarial_rays(lib):
    total = np.zeros(6, np.uint64)
    for seed, k in zip((1, 2, 3, 4, 5, 6), (0, 1, -1, 2, -2, 0)):
        lib.box32_set_rcp_ulps(k)
        out = (ctypes.c_uint64 * 6)()
        lib.box32_sweep(1_000_000, seed, out)
        total += np.array(list(out), np.uint64)
    lib.box32_set_rcp_ulps(0)
    cases, meets, accepted, violations, rejected, skipped = (int(v) for v in total)
    print(f"box32 sweep: {cases} cases in the contract ({skipped} outside), {meets} meet the box, "
          f"{accepted} accepted, {violations} met-but-rejected, {rejected} correctly rejected")
    assert violations == 0
    assert skipped < 0.05 * (cases + skipped) and meets > 0.5 * cases
