"""The kernels' texture-coordinate divisions by the constants 2 pi and pi (get_sphere_uv,
the_next_week/sphere.rs:50-51) run as one product and Markstein's fma correction
(rrt_kernel.hip div_by_const, rrt_books64.hip div_by_const64) instead of the IEEE division
expansion. This pins that the result is the IEEE quotient over the kernels' argument domain:
exhaustively for every f32 in [2^-100, 8] and +0 (phi is 0 or >= 2^-22, theta 0 or >= 3e-4), and
for 2e7 random f64 arguments in [2^-60, 8). CPU only (host FMA, -ffp-contract=off)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "divconst", "div_const_check.c")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_division_by_constant_is_the_ieee_quotient(tmp_path):
    exe = str(tmp_path / "div_const_check")
    subprocess.run(["gcc", "-O2", "-mfma", "-ffp-contract=off", SRC, "-o", exe, "-lm"], check=True)
    out = subprocess.run([exe, "20000000"], capture_output=True, text=True, timeout=300, check=True).stdout
    lines = [ln.split() for ln in out.strip().splitlines()]
    assert [ln[0] for ln in lines] == ["f32", "f32", "f64", "f64"]
    for kind, c, checked, bad in lines:
        assert int(checked) > (800_000_000 if kind == "f32" else 10_000_000)
        assert int(bad) == 0, f"{kind} c={c}: {bad} of {checked} quotients differ from x / c"
