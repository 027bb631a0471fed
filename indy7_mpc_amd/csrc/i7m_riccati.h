// i7m_riccati.h — exact solve of the SQP subproblem QP, one wavefront per problem (gfx950, fp64).
//
// The reference hands OSQP (src/osqp_solver.py:137-143)
//     min 1/2 z'Pz + g'z   s.t.  -x_0 = -xs,   A_k x_k + B_k u_k - x_{k+1} = -c_k,
// whose KKT matrix is block-tridiagonal.  This kernel solves it exactly with the backward
// Riccati recursion over the 12x12 / 12x6 stage blocks (staged in LDS) and a forward rollout:
//     VA = V A, T = V_vv B_u, s = v + V c                      (round R1)
//     AtVA = A'VA + Q, G = B'VA, H = R + B'T, h = r + B's, vA = q + A's   (round R2)
//     [K | kff] = -H^-1 [G | h]                               (R3: 13 lanes, 6x6 Cholesky)
//     V <- AtVA + G'K, v <- vA + G'kff                         (round R4)
// A = [[I, dt I], [Aq, Av]], B = [0; Bu] — the identity / dt blocks are never multiplied.
//
// Each round is UNIFORM across the 64 lanes: lane l evaluates
//     out = sum_{m<6} sh[xo + m*xs] * sh[yo + m*ys] + alpha*sh[a1] + sh[a2] + sh[e1]*sh[e2]
// and stores it to sh[oo] and sh[oo2] (mirror for symmetric outputs).  The per-lane operand
// offsets come from a descriptor table built once on the host (build_riccati_desc), loaded
// into 24 VGPRs at kernel start: no per-stage index arithmetic and no divergent branches.
#pragma once

#include <stdint.h>

#include <vector>

#include "i7m_kernels.h"

namespace i7m {

// LDS layout (doubles) of one problem
enum : int {
  RO_V = 0,      // 144  V, overwritten in place by AtVA (R2) and V_new (R4)
  RO_v = 144,    // 12
  RO_AQ = 156,   // 36   | stage data stashed contiguously: lin (114) + cost (10) + XU_k (18)
  RO_AV = 192,   // 36   |
  RO_BU = 228,   // 36   |
  RO_A = 264,    // 6    |
  RO_W = 270,    // 10   | j(6) Qm dQm Rm |e|
  RO_X = 280,    // 18   |
  RO_CV = 298,   // 6    c_v
  RO_RU = 304,   // 6    Rm u
  RO_QV = 310,   // 12   Qm j | dQm v
  RO_VA = 322,   // 144
  RO_T = 466,    // 36
  RO_S = 502,    // 12
  RO_G = 514,    // 72
  RO_H = 586,    // 36
  RO_h = 622,    // 6
  RO_vA = 628,   // 12
  RO_K = 640,    // 78   K (6x12) + kff (6)
  RO_ZERO = 718,
  RO_ONE = 719,
  RO_DUMMY = 720,
  RO_TOTAL = 724,
};
constexpr int RIC_SUBROUNDS = 8;  // R1: 3, R2: 3, R4: 2
constexpr int RIC_DESC_WORDS = RIC_SUBROUNDS * 64 * 3;

// Host-side descriptor table: [subround][lane][3] uint32.
inline void build_riccati_desc(uint32_t* out) {
  struct D {
    int xo, xs, yo, ys, alpha, a1, a2, e1, e2, oo, oo2;
  };
  auto pack = [](const D& d, uint32_t* w) {
    auto sc = [](int s) { return s == 1 ? 0u : s == 6 ? 1u : s == 12 ? 2u : 3u; };
    w[0] = (uint32_t)d.xo | ((uint32_t)d.yo << 10) | ((uint32_t)d.a1 << 20) | ((uint32_t)d.alpha << 30);
    w[1] = (uint32_t)d.a2 | ((uint32_t)d.e1 << 10) | ((uint32_t)d.e2 << 20) | (sc(d.xs) << 30);
    w[2] = (uint32_t)d.oo | ((uint32_t)d.oo2 << 10) | (sc(d.ys) << 20);
  };
  const D dummy = {RO_ZERO, 1, RO_ZERO, 1, 0, RO_ZERO, RO_ZERO, RO_ZERO, RO_ZERO, RO_DUMMY, RO_DUMMY};
  std::vector<D> r1, r2, r4;
  // ---- R1
  for (int e = 0; e < 144; ++e) {
    const int r = e / 12, c = e % 12;
    D d = dummy;
    d.xo = RO_V + 12 * r + 6; d.xs = 1; d.ys = 6;
    if (c < 6) { d.yo = RO_AQ + c; d.alpha = 1; d.a1 = RO_V + 12 * r + c; }
    else { d.yo = RO_AV + (c - 6); d.alpha = 2; d.a1 = RO_V + 12 * r + (c - 6); }
    d.oo = d.oo2 = RO_VA + 12 * r + c;
    r1.push_back(d);
  }
  for (int t = 0; t < 36; ++t) {
    const int r = t / 6, c = t % 6;
    D d = dummy;
    d.xo = RO_V + 12 * (6 + r) + 6; d.xs = 1; d.yo = RO_BU + c; d.ys = 6;
    d.oo = d.oo2 = RO_T + 6 * r + c;
    r1.push_back(d);
  }
  for (int r = 0; r < 12; ++r) {
    D d = dummy;
    d.xo = RO_V + 12 * r + 6; d.xs = 1; d.yo = RO_CV; d.ys = 1; d.a2 = RO_v + r;
    d.oo = d.oo2 = RO_S + r;
    r1.push_back(d);
  }
  // ---- R2
  for (int r = 0; r < 12; ++r)
    for (int c = r; c < 12; ++c) {
      D d = dummy;
      d.yo = RO_VA + 72 + c; d.ys = 12; d.xs = 6;
      if (r < 6) {
        d.xo = RO_AQ + r; d.alpha = 1; d.a1 = RO_VA + 12 * r + c;
        if (c < 6) { d.e1 = RO_QV + r; d.e2 = RO_W + c; }          // + Qm j_r j_c
      } else {
        d.xo = RO_AV + (r - 6); d.alpha = 2; d.a1 = RO_VA + 12 * (r - 6) + c;
        if (r == c) { d.e1 = RO_W + 7; d.e2 = RO_ONE; }           // + dQm
      }
      d.oo = RO_V + 12 * r + c; d.oo2 = RO_V + 12 * c + r;
      r2.push_back(d);
    }
  for (int t = 0; t < 72; ++t) {
    const int r = t / 12, c = t % 12;
    D d = dummy;
    d.xo = RO_BU + r; d.xs = 6; d.yo = RO_VA + 72 + c; d.ys = 12;
    d.oo = d.oo2 = RO_G + 12 * r + c;
    r2.push_back(d);
  }
  for (int r = 0; r < 6; ++r)
    for (int c = r; c < 6; ++c) {
      D d = dummy;
      d.xo = RO_BU + r; d.xs = 6; d.yo = RO_T + c; d.ys = 6;
      if (r == c) d.a2 = RO_W + 8;  // + Rm
      d.oo = RO_H + 6 * r + c; d.oo2 = RO_H + 6 * c + r;
      r2.push_back(d);
    }
  for (int r = 0; r < 6; ++r) {
    D d = dummy;
    d.xo = RO_BU + r; d.xs = 6; d.yo = RO_S + 6; d.ys = 1; d.a2 = RO_RU + r;
    d.oo = d.oo2 = RO_h + r;
    r2.push_back(d);
  }
  for (int r = 0; r < 12; ++r) {
    D d = dummy;
    d.yo = RO_S + 6; d.ys = 1; d.xs = 6; d.a2 = RO_QV + r;
    if (r < 6) { d.xo = RO_AQ + r; d.alpha = 1; d.a1 = RO_S + r; }
    else { d.xo = RO_AV + (r - 6); d.alpha = 2; d.a1 = RO_S + (r - 6); }
    d.oo = d.oo2 = RO_vA + r;
    r2.push_back(d);
  }
  // ---- R4
  for (int r = 0; r < 12; ++r)
    for (int c = r; c < 12; ++c) {
      D d = dummy;
      d.xo = RO_G + r; d.xs = 12; d.yo = RO_K + c; d.ys = 12; d.alpha = 1; d.a1 = RO_V + 12 * r + c;
      d.oo = RO_V + 12 * r + c; d.oo2 = RO_V + 12 * c + r;
      r4.push_back(d);
    }
  for (int r = 0; r < 12; ++r) {
    D d = dummy;
    d.xo = RO_G + r; d.xs = 12; d.yo = RO_K + 72; d.ys = 1; d.alpha = 1; d.a1 = RO_vA + r;
    d.oo = d.oo2 = RO_v + r;
    r4.push_back(d);
  }
  auto emit = [&](const std::vector<D>& v, int nsub, int first) {
    for (int sr = 0; sr < nsub; ++sr)
      for (int l = 0; l < 64; ++l) {
        const size_t e = (size_t)sr * 64 + l;
        pack(e < v.size() ? v[e] : dummy, out + ((size_t)(first + sr) * 64 + l) * 3);
      }
  };
  emit(r1, 3, 0);
  emit(r2, 3, 3);
  emit(r4, 2, 6);
}

__device__ __forceinline__ void ric_round(double* sh, uint32_t w0, uint32_t w1, uint32_t w2, double dt) {
  // keep only the packed words live across the stage loop: decode every round (cheap SALU/VALU
  // bit-field extracts) instead of letting the compiler hoist ~100 decoded addresses
  asm volatile("" : "+v"(w0), "+v"(w1), "+v"(w2));
  const int xo = w0 & 1023, yo = (w0 >> 10) & 1023, a1 = (w0 >> 20) & 1023;
  const uint32_t al = w0 >> 30;
  const int a2 = w1 & 1023, e1 = (w1 >> 10) & 1023, e2 = (w1 >> 20) & 1023;
  const uint32_t xsc = w1 >> 30;
  const int oo = w2 & 1023, oo2 = (w2 >> 10) & 1023;
  const uint32_t ysc = (w2 >> 20) & 3;
  const int xs = xsc == 0 ? 1 : (xsc == 1 ? 6 : 12);
  const int ys = ysc == 0 ? 1 : (ysc == 1 ? 6 : 12);
  const double alpha = al == 0 ? 0.0 : (al == 1 ? 1.0 : dt);
  double acc = alpha * sh[a1] + sh[a2] + sh[e1] * sh[e2];
#pragma unroll
  for (int m = 0; m < 6; ++m) acc += sh[xo + m * xs] * sh[yo + m * ys];
  sh[oo] = acc;
  sh[oo2] = acc;
}

// Cholesky (lower) with reciprocal diagonal rd; solve L L' x = b.
__device__ __forceinline__ void chol6r(double A[6][6], double rd[6]) {
  chol6(A);
#pragma unroll
  for (int j = 0; j < 6; ++j) rd[j] = A[j][j];
}
__device__ __forceinline__ void chol6r_solve(const double L[6][6], const double rd[6], double b[6]) {
  (void)rd;
  chol6_solve(L, b);
}

__global__ void __launch_bounds__(64) k_riccati(SolveParams P, const uint32_t* __restrict__ desc,
                                                const double* __restrict__ xu, const double* __restrict__ xs,
                                                const double* __restrict__ lin, const double* __restrict__ cost,
                                                const int* __restrict__ active, double* __restrict__ kbuf,
                                                double* __restrict__ sol) {
  const int b = blockIdx.x;
  if (b >= P.B) return;
  if (active && !active[b]) return;
  const int l = threadIdx.x;
  const int N = P.N;
  const double dt = P.dt;
  __shared__ double sh[RO_TOTAL];
  const double* X = xu + (long)b * P.T;
  const double* LINb = lin + (long)b * (N - 1) * LIN_STRIDE;
  const double* CB = cost + (long)b * N * COST_STRIDE;
  double* KB = kbuf + (long)b * (N - 1) * KBUF_STRIDE;

  uint32_t dw[RIC_SUBROUNDS][3];
#pragma unroll
  for (int r = 0; r < RIC_SUBROUNDS; ++r)
#pragma unroll
    for (int i = 0; i < 3; ++i) dw[r][i] = desc[((size_t)r * 64 + l) * 3 + i];

  // ---- terminal cost-to-go: V = P_{N-1}, v = g_{N-1}
  if (l < COST_STRIDE) sh[RO_W + l] = CB[(N - 1) * COST_STRIDE + l];
  if (l == 0) { sh[RO_ZERO] = 0.0; sh[RO_ONE] = 1.0; }
  __syncthreads();
  for (int e = l; e < 144; e += 64) {
    const int r = e / 12, cc = e - 12 * r;
    double val = 0.0;
    if (r < 6 && cc < 6) val = sh[RO_W + 6] * (sh[RO_W + r] * sh[RO_W + cc]);
    else if (r == cc) val = sh[RO_W + 7];
    sh[RO_V + e] = val;
  }
  if (l < 12) sh[RO_v + l] = (l < 6) ? sh[RO_W + 6] * sh[RO_W + l] : sh[RO_W + 7] * X[18 * (N - 1) + l];

  // stage data prefetch: element e of [lin(114) | cost(10) | XU_k(18)] -> sh[RO_AQ + e]
  auto src = [&](int k, int e) -> const double* {
    if (e < LIN_STRIDE) return LINb + (long)k * LIN_STRIDE + e;
    if (e < LIN_STRIDE + COST_STRIDE) return CB + k * COST_STRIDE + (e - LIN_STRIDE);
    return X + 18 * k + (e - LIN_STRIDE - COST_STRIDE);
  };
  const int e2 = (l + 128 < 142) ? l + 128 : 141;
  double p0 = *src(N - 2, l), p1 = *src(N - 2, l + 64), p2 = *src(N - 2, e2);

  for (int k = N - 2; k >= 0; --k) {
    __syncthreads();
    sh[RO_AQ + l] = p0;
    sh[RO_AQ + l + 64] = p1;
    if (l + 128 < 142) sh[RO_AQ + l + 128] = p2;
    __syncthreads();
    if (k > 0) { p0 = *src(k - 1, l); p1 = *src(k - 1, l + 64); p2 = *src(k - 1, e2); }
    // pre-round: c_v (src/osqp_solver.py:76-81), Rm u, Qm j, dQm v
    if (l < 6) {
      double acc = 0.0;
#pragma unroll
      for (int jj = 0; jj < 6; ++jj)
        acc += sh[RO_AQ + 6 * l + jj] * sh[RO_X + jj] + sh[RO_AV + 6 * l + jj] * sh[RO_X + 6 + jj] +
               sh[RO_BU + 6 * l + jj] * sh[RO_X + 12 + jj];
      sh[RO_CV + l] = (sh[RO_X + 6 + l] + sh[RO_A + l] * dt) - acc;
    } else if (l < 12) {
      sh[RO_RU + l - 6] = sh[RO_W + 8] * sh[RO_X + 12 + (l - 6)];
    } else if (l < 18) {
      sh[RO_QV + l - 12] = sh[RO_W + 6] * sh[RO_W + (l - 12)];
    } else if (l < 24) {
      sh[RO_QV + 6 + (l - 18)] = sh[RO_W + 7] * sh[RO_X + 6 + (l - 18)];
    }
    __syncthreads();
    ric_round(sh, dw[0][0], dw[0][1], dw[0][2], dt);
    ric_round(sh, dw[1][0], dw[1][1], dw[1][2], dt);
    ric_round(sh, dw[2][0], dw[2][1], dw[2][2], dt);
    __syncthreads();
    ric_round(sh, dw[3][0], dw[3][1], dw[3][2], dt);
    ric_round(sh, dw[4][0], dw[4][1], dw[4][2], dt);
    ric_round(sh, dw[5][0], dw[5][1], dw[5][2], dt);
    __syncthreads();
    if (l < 13) {
      double L[6][6], rd[6], rhs[6];
#pragma unroll
      for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int jj = 0; jj < 6; ++jj) L[i][jj] = sh[RO_H + 6 * i + jj];
      chol6r(L, rd);
#pragma unroll
      for (int i = 0; i < 6; ++i) rhs[i] = (l < 12) ? sh[RO_G + 12 * i + l] : sh[RO_h + i];
      chol6r_solve(L, rd, rhs);
#pragma unroll
      for (int i = 0; i < 6; ++i) sh[(l < 12) ? (RO_K + 12 * i + l) : (RO_K + 72 + i)] = -rhs[i];
    }
    __syncthreads();
    ric_round(sh, dw[6][0], dw[6][1], dw[6][2], dt);
    ric_round(sh, dw[7][0], dw[7][1], dw[7][2], dt);
    // K, kff, c_v -> global for the forward rollout
    double* kk = KB + (long)k * KBUF_STRIDE;
    kk[l] = sh[RO_K + l];
    if (l < 20) kk[64 + l] = (l < 14) ? sh[RO_K + 64 + l] : sh[RO_CV + (l - 14)];
  }

  // ---- forward rollout: x_0 = xs; u_k = K x_k + kff; x_{k+1} = A x + B u + c  (one stage per step)
  double* S = sol + (long)b * P.T;
  double* sx = sh + RO_VA;        // x double buffer [2][12]
  double* su = sh + RO_VA + 24;   // u (6)
  double* sk = sh + RO_K;         // K(72) kff(6)
  double* sc = sh + RO_CV;        // c_v(6)
  double* sl = sh + RO_AQ;        // Aq Av Bu (108)
  // stage data: [kbuf(84) | lin(108)] = 192 values, 3 per lane
  auto fsrc = [&](int k, int e) -> const double* {
    return (e < KBUF_STRIDE) ? KB + (long)k * KBUF_STRIDE + e : LINb + (long)k * LIN_STRIDE + (e - KBUF_STRIDE);
  };
  auto fdst = [&](int e) -> double* { return (e < 78) ? sk + e : (e < 84 ? sc + (e - 78) : sl + (e - 84)); };
  __syncthreads();  // kbuf stores of this wave are visible to its own loads (same CU), finish LDS use
  double f0 = *fsrc(0, l), f1 = *fsrc(0, l + 64), f2 = *fsrc(0, l + 128);
  if (l < 12) {
    const double x0 = xs[(long)b * 12 + l];
    sx[l] = x0;
    S[l] = x0;
  }
  for (int k = 0; k < N - 1; ++k) {
    const int cur = k & 1;
    __syncthreads();
    *fdst(l) = f0;
    *fdst(l + 64) = f1;
    *fdst(l + 128) = f2;
    __syncthreads();
    if (k + 1 < N - 1) { f0 = *fsrc(k + 1, l); f1 = *fsrc(k + 1, l + 64); f2 = *fsrc(k + 1, l + 128); }
    const double* x = sx + 12 * cur;
    if (l < 6) {
      double acc = sk[72 + l];
#pragma unroll
      for (int jj = 0; jj < 12; ++jj) acc += sk[12 * l + jj] * x[jj];
      su[l] = acc;
      S[18 * k + 12 + l] = acc;
    }
    __syncthreads();
    if (l < 12) {
      double nx;
      if (l < 6) {
        nx = x[l] + dt * x[6 + l];
      } else {
        const int i = l - 6;
        double acc = sc[i];
#pragma unroll
        for (int jj = 0; jj < 6; ++jj)
          acc += sl[6 * i + jj] * x[jj] + sl[36 + 6 * i + jj] * x[6 + jj] + sl[72 + 6 * i + jj] * su[jj];
        nx = acc;
      }
      sx[12 * (cur ^ 1) + l] = nx;
      S[18 * (k + 1) + l] = nx;
    }
  }
}

}  // namespace i7m
