"""i7m_sincos.h (the fp64 sincos of the dynamics kernels) against the host libm: compiled
for the host with hipcc (no GPU needed), 2M angles across the joint range, around multiples
of pi/2 and at tiny magnitudes; within 1 ulp of libm (glibc sin/cos are themselves < 1 ulp)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = r'''
#include "i7m_sincos.h"
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
static int64_t ord(double x) { int64_t i; std::memcpy(&i, &x, 8); return i < 0 ? INT64_MIN - i : i; }
int main() {
  std::mt19937_64 g(7);
  std::uniform_real_distribution<double> u(-20.0, 20.0);
  long ms = 0, mc = 0;
  for (int t = 0; t < 2000000; ++t) {
    double x = t < 20000 ? (t - 10000) * 0.7853981633974483 : u(g);
    if (t % 3 == 0) x *= 1e-3 * (t % 7 + 1);
    if (t % 11 == 0) x *= 1e-9;
    double s, c;
    i7m::sincos_q(x, &s, &c);
    const long es = labs(ord(s) - ord(std::sin(x))), ec = labs(ord(c) - ord(std::cos(x)));
    ms = es > ms ? es : ms;
    mc = ec > mc ? ec : mc;
  }
  double s, c;
  i7m::sincos_q(3.0e7, &s, &c);  // beyond the fast range: the library path
  const bool big = s == std::sin(3.0e7) && c == std::cos(3.0e7);
  std::printf("%ld %ld %d\n", ms, mc, big ? 1 : 0);
}
'''


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not available")
def test_sincos_within_one_ulp_of_libm(tmp_path):
    src = tmp_path / "t.hip"
    src.write_text(SRC)
    exe = tmp_path / "t"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-I" + os.path.join(ROOT, "indy7_mpc_amd", "csrc"), str(src),
                    "-o", str(exe)], check=True, capture_output=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    ms, mc, big = int(out[0]), int(out[1]), int(out[2])
    assert ms <= 1 and mc <= 1, (ms, mc)
    assert big == 1
