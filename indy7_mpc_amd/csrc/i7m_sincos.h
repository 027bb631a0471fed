// i7m_sincos.h — sin and cos of a joint angle together, for the dynamics kernels (fp64).
//
// The angles on the hot path are joint positions and line-search points (|q| of a few rad),
// so the general library sincos (a Payne-Hanek-capable reduction and two branchy kernels,
// ~80-100 instructions) is replaced by: Cody-Waite reduction by pi/2 with FMA (three-part
// pi/2, exact to far below an ulp for |x| < 2^20), then the classic minimax kernels on
// [-pi/4, pi/4] (the fdlibm __kernel_sin / __kernel_cos coefficients and formulas, the same
// polynomials glibc and musl use), ~35 instructions for both values.  Accuracy: within 1 ulp of
// the correctly rounded result on the tested range (tests/test_host.py checks against the host
// libm).  |x| >= 2^20 goes to the library sincos.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>

namespace i7m {

// the cold path, kept out of line so the library code is not inlined at every call site.  It
// returns its pair by value: passing the caller's output pointers to an out-of-line call takes the
// addresses of the callers' sin / cos arrays, which then live in scratch memory on the hot path too
// (k_linesearch stored and re-loaded all twelve values of a knot's evaluation through scratch).
struct SinCos {
  double s, c;
};
__host__ __device__ __noinline__ SinCos sincos_lib(double x) {
  SinCos r;
  sincos(x, &r.s, &r.c);
  return r;
}

__host__ __device__ __forceinline__ void sincos_q(double x, double* sp, double* cp) {
  if (!(fabs(x) < 1048576.0)) {  // also NaN / inf
    const SinCos r = sincos_lib(x);
    *sp = r.s;
    *cp = r.c;
    return;
  }
  const double n = rint(x * 0.6366197723675814);  // 2 / pi
  double r = fma(-n, 1.5707963267948966, x);       // pi/2 = P1 + P2 + P3
  r = fma(-n, 6.123233995736766e-17, r);
  r = fma(-n, -1.4973849048591698e-33, r);
  const double z = r * r;
  // sin(r) = r + r^3 (S1 + z S(z))
  const double ps = 8.33333333332248946124e-03 +
                    z * (-1.98412698298579493134e-04 +
                         z * (2.75573137070700676789e-06 + z * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10)));
  const double sr = r + (z * r) * (-1.66666666666666324348e-01 + z * ps);
  // cos(r) = 1 - z/2 + z^2 C(z), with the 1 - z/2 rounding error carried (fdlibm)
  const double pc = z * (4.16666666666666019037e-02 +
                         z * (-1.38888888888741095749e-03 +
                              z * (2.48015872894767294178e-05 +
                                   z * (-2.75573143513906633035e-07 +
                                        z * (2.08757232129817482790e-09 + z * -1.13596475577881948265e-11)))));
  const double hz = 0.5 * z;
  const double w = 1.0 - hz;
  const double cr = w + (((1.0 - w) - hz) + z * pc);
  const int q = (int)n & 3;
  const double s0 = (q & 1) ? cr : sr;
  const double c0 = (q & 1) ? sr : cr;
  *sp = (q & 2) ? -s0 : s0;
  *cp = ((q + 1) & 2) ? -c0 : c0;
}

}  // namespace i7m
