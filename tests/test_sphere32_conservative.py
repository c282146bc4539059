"""The f64 books kernel's sphere pre-test (rustraytrace_amd/csrc/rrt_sphere32.h: f32 arithmetic with a
proven error bound) may skip the f64 test of sphere.rs:24-51 only for a sphere whose f64 discriminant
is negative — one the f64 test would pass over — or the kernel could miss the books path's closest
hit. The header is compiled for the host (tests/sphere32/sphere32_harness.cpp, the same source the
device compiles) and checked against the kernel's own f64 discriminant (same operations, unfused):
  * grazing rays at r (1 + eps) from the center for eps = +-1e-12 .. 0.3 and exactly 0, from origins
    on the sphere (secondary rays), inside it and 1e-3 .. 1e5 away, centers up to 2^20, radii
    1e-4 .. 1e3, directions 1e-6 .. 1e6 long with zeroed components: 4e6 rays, 0 rejections of a
    sphere whose f64 discriminant is >= 0;
  * tightness: every clear miss in the domain (disc < -1e-3 a (|oc|^2 + r^2 + 1e-6 |o|^2)) is
    rejected (the f32 origin's own rounding, u |o|, is what the |o|^2 term prices);
  * the domain guard: rays outside it (|d|^2 beyond 2^+-40, |o| beyond 2^20) never reject."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("sphere32") / "sphere32.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-shared", "-fPIC",
                    os.path.join(HERE, "sphere32", "sphere32_harness.cpp"), "-o", so], check=True)
    L = ctypes.CDLL(so)
    L.sphere32_sweep.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
    P = ctypes.c_void_p
    L.sphere32_eval.argtypes = [ctypes.c_uint32, P, P, P, P, P, P]
    return L


def _eval(L, o, d, c, r):
    n = len(o)
    o, d = np.ascontiguousarray(o, np.float64), np.ascontiguousarray(d, np.float64)
    c, r = np.ascontiguousarray(c, np.float32), np.ascontiguousarray(r, np.float32)
    miss = np.zeros(n, np.uint8)
    disc = np.zeros(n, np.float64)
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    L.sphere32_eval(n, ptr(o), ptr(d), ptr(c), ptr(r), ptr(miss), ptr(disc))
    return miss.astype(bool), disc


def test_sweep_never_rejects_a_sphere_the_f64_test_keeps(lib):
    total = np.zeros(6, np.uint64)
    for seed in range(1, 5):
        out = (ctypes.c_uint64 * 6)()
        lib.sphere32_sweep(1_000_000, seed, out)
        total += np.array(list(out), np.uint64)
    cases, hits, rej, viol, clear, clear_rej = (int(v) for v in total)
    print(f"sphere32 sweep: {cases} rays, {hits} with f64 disc >= 0, {rej} rejected, {viol} violations, "
          f"{clear_rej} of {clear} clear misses rejected")
    assert viol == 0
    assert hits > 0.3 * cases and clear > 0.03 * cases  # the sweep straddles tangency
    assert clear_rej == clear


def test_exact_tangents_and_surface_origins(lib):
    # rays from points on the sphere along its tangent plane (disc ~ 0 up to rounding) and the
    # grazing rays one f64 ulp either side, at the C2 / C5 scales
    rng = np.random.default_rng(7)
    n = 20000
    c = np.float32(rng.uniform(-20, 20, (n, 3)))
    r = np.float32(np.exp(rng.uniform(np.log(0.05), np.log(1000), n)))
    nrm = rng.normal(size=(n, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    o = c.astype(np.float64) + r[:, None].astype(np.float64) * nrm
    t = rng.normal(size=(n, 3))
    t -= (t * nrm).sum(1, keepdims=True) * nrm
    d = t * np.exp(rng.uniform(-5, 5, n))[:, None]
    d = np.nextafter(d, np.where(rng.uniform(size=(n, 3)) < 0.5, -np.inf, np.inf))
    miss, disc = _eval(lib, o, d, c, r)
    assert not np.any(miss & (disc >= 0)), "rejected a sphere with f64 disc >= 0"


def test_domain_guard_never_rejects(lib):
    rng = np.random.default_rng(3)
    n = 2000
    c = np.float32(rng.uniform(-10, 10, (n, 3)))
    r = np.full(n, 0.1, np.float32)
    o = np.tile([[0.0, 0.0, 1e7]], (n, 1))  # |o|^2 > 2^40
    d = c - o
    miss, _ = _eval(lib, o, d + 50.0, c, r)  # clear misses, outside the domain
    assert not miss.any()
    o2 = np.zeros((n, 3))
    for scale in (1e-13, 1e13):  # |d|^2 outside [2^-40, 2^40]
        miss, _ = _eval(lib, o2, (c + 5.0) * scale, c, r)
        assert not miss.any()
    miss, _ = _eval(lib, o2, c + 5.0, c, r)  # in the domain the same misses are rejected
    assert miss.mean() > 0.5
