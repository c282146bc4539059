"""FastDiv (rustraytrace_amd/csrc/rrt_internal.h): the kernel's work-queue index math divides by
uniform divisors as multiply-high + add + shift. Checked here against C++ `/` on the host, for
every divisor up to 4096 and random ones up to 2^31, over dividends in [0, 2^31)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = r'''
#include "rrt_internal.h"
#include <cstdio>
#include <random>
int main() {
    std::mt19937_64 g(7);
    long bad = 0;
    for (uint32_t d = 1; d <= 4096; ++d) {
        const rrt::FastDiv f = rrt::make_fastdiv(d);
        for (uint32_t n = 0; n < 2048; ++n) bad += rrt::fast_div(n, f) != n / d;
        for (int k = 0; k < 2000; ++k) {
            const uint32_t n = (uint32_t)(g() & 0x7fffffffu);
            bad += rrt::fast_div(n, f) != n / d;
        }
        bad += rrt::fast_div(0x7fffffffu, f) != 0x7fffffffu / d;
    }
    for (int k = 0; k < 1000000; ++k) {
        const uint32_t d = (uint32_t)(g() >> (33 + (k % 31))) + 1u;
        const uint32_t n = (uint32_t)(g() & 0x7fffffffu);
        const rrt::FastDiv f = rrt::make_fastdiv(d);
        bad += rrt::fast_div(n, f) != n / d;
    }
    std::printf("%ld\n", bad);
    return bad != 0;
}
'''


def test_fast_div_matches_integer_division(tmp_path):
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    src = tmp_path / "fd.cpp"
    src.write_text(SRC)
    exe = tmp_path / "fd"
    inc = os.path.join(ROOT, "rustraytrace_amd", "csrc")
    subprocess.run([hipcc, "-O2", "-std=c++17", "-I", inc, str(src), "-o", str(exe)], check=True, capture_output=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.strip() == "0", r.stdout + r.stderr
