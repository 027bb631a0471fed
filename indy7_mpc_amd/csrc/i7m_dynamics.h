// i7m_dynamics.h — rigid-body kinematics/dynamics for a 6-DOF revolute-z serial chain,
// written for one GPU lane (gfx950, fp64): everything is fully unrolled into registers.
//
// Replaces the pinocchio calls on the reference hot path (reference paths):
//   forwardKinematics / oMi[6].translation       src/osqp_solver.py:146-148   -> fk_jac
//   computeJointJacobians / getJointJacobian     src/osqp_solver.py:150-155   -> fk_jac
//   aba                                          src/osqp_sqp.py:40           -> forward_dynamics
//   computeABADerivatives (+data.ddq)            src/osqp_solver.py:71,76     -> rnea<dual> + chol
// Conventions (pinocchio's): spatial vectors [linear; angular]; joint i frame placed in
// its parent by (Rp_i Rz(q_i), t_i); gravity enters as base acceleration -g.
// Derivatives: forward-mode dual numbers through RNEA at (q, v, a) — one tangent direction
// per lane — then da/dx = -M^-1 dtau/dx (a fixed). Exact to rounding, like pinocchio's
// analytical ABA derivatives.
#pragma once

#include <hip/hip_runtime.h>

#include "i7m_timeline.h"

namespace i7m {

// Workgroup barrier ordering LDS only (an LDS-scoped release / acquire around s_barrier, which
// the compiler drops for the single-wave workgroups used here): unlike __syncthreads() it does
// not wait for the wave's outstanding global stores (s_waitcnt vmcnt(0)), which no lane reads
// back in the same phase.  Where another lane does read global data this wave wrote, the
// kernels use __syncthreads().
__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// The same ordering among the lanes of ONE wavefront, for device bodies whose LDS region only
// their own wave touches (the linearisation's per-knot exchanges, the Riccati recursion): the
// fences of lds_sync() without the s_barrier.  In a single-wave workgroup this is exactly what
// lds_sync() compiles to; in a multi-wave workgroup (k_sqp_fused) the other waves need not
// take part.
//   A wavefront's LDS instructions execute in order, so within one wave only the compiler's order
// matters: I7M_WAVE_SYNC_FENCE 0 (default) keeps it with an empty asm with a memory clobber; 1 emits
// the fences, whose s_waitcnt lgkmcnt(0) also drains every outstanding LDS operation.  (No kernel
// here writes LDS by direct-from-memory loads, whose completion is not ordered with ds_* ops.)
#ifndef I7M_WAVE_SYNC_FENCE
#define I7M_WAVE_SYNC_FENCE 0
#endif
__device__ __forceinline__ void wave_sync_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
__device__ __forceinline__ void wave_sync() {
#if I7M_WAVE_SYNC_FENCE
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
#else
  __asm__ volatile("" ::: "memory");
#endif
}
// Wave priority (s_setprio 0..3; the SIMD's instruction arbiter otherwise favours the oldest
// wave).  The Riccati recursion sets it by progress (riccati_mfma_body, BC bit 2: equal-work
// waves, the one furthest behind first).  I7M_PRIO bits: 1 the line-search rounds, later rounds
// first (measured no change: 78.4 vs 78.8 us at B = 4096, not default), 2 the interior-point
// iterations of k_ipm_fused, the most work left first (6.00 -> 5.92 ms per QP, default).
#ifndef I7M_PRIO
#define I7M_PRIO 4
#endif
__device__ __forceinline__ void set_prio(int p) {  // p wave-uniform; s_setprio takes an immediate
  if (p <= 0) __builtin_amdgcn_s_setprio(0);
  else if (p == 1) __builtin_amdgcn_s_setprio(1);
  else if (p == 2) __builtin_amdgcn_s_setprio(2);
  else __builtin_amdgcn_s_setprio(3);
}

// ... and for global memory too (a lane reads what another lane of the wave stored): the
// __syncthreads() of a single-wave workgroup, without the barrier.
__device__ __forceinline__ void wave_sync_all() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
// Between the phases of k_sqp_fused: every wave's global stores complete and become visible to
// every wave of the workgroup, L1 lines read before the phase are dropped (agent-scope acquire:
// the next phase re-reads buffers an earlier phase cached and this one overwrote), then barrier.
__device__ __forceinline__ void block_sync_global() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// Device-side model: URDF numbers plus precomputed inertia about each joint origin.
struct DevModel {
  double Rp[6][9];   // row-major
  double tp[6][3];
  double m[6];
  double h[6][3];    // m * com
  double Io[6][6];   // inertia about the joint origin: xx xy xz yy yz zz
  double g[3];
  double qlo[6], qhi[6], vlim[6], ulim[6];
};

// ---------------------------------------------------------------- dual numbers
struct dual {
  double v, d;
};
__device__ __forceinline__ dual mk(double v, double d = 0.0) { return dual{v, d}; }
__device__ __forceinline__ dual operator+(dual a, dual b) { return {a.v + b.v, a.d + b.d}; }
__device__ __forceinline__ dual operator-(dual a, dual b) { return {a.v - b.v, a.d - b.d}; }
__device__ __forceinline__ dual operator-(dual a) { return {-a.v, -a.d}; }
__device__ __forceinline__ dual operator*(dual a, dual b) { return {a.v * b.v, fma(a.v, b.d, a.d * b.v)}; }
__device__ __forceinline__ dual operator*(double a, dual b) { return {a * b.v, a * b.d}; }
__device__ __forceinline__ dual operator*(dual b, double a) { return {a * b.v, a * b.d}; }
__device__ __forceinline__ dual operator+(dual a, double b) { return {a.v + b, a.d}; }

template <class T> __device__ __forceinline__ T zero();
template <> __device__ __forceinline__ double zero<double>() { return 0.0; }
template <> __device__ __forceinline__ dual zero<dual>() { return dual{0.0, 0.0}; }
template <class T> __device__ __forceinline__ T cst(double x);
template <> __device__ __forceinline__ double cst<double>(double x) { return x; }
template <> __device__ __forceinline__ dual cst<dual>(double x) { return dual{x, 0.0}; }

// ---------------------------------------------------------------- compile-time zeros
// With the Indy7 model baked in (kIndy7Model) many factors are exact zeros once the loops are
// unrolled: the identity joint rotations Rp_0 / Rp_2 and the zero entries of the other Rp_i,
// the zero components of t_i and of gravity, RNEA's qdd = 0, the base's zero velocity.  Strict
// IEEE forbids the compiler to drop 0 * x (NaN for x = inf) or x + 0 (the sign of -0), so it
// kept ~8 % of k_linesearch's fp64 instructions as products with a zero operand.  These
// helpers drop a term whose factor is a compile-time 0.0 (clang's __builtin_constant_p, resolved
// after inlining and unrolling; a dropped term's zero folds into the next helper) and are the
// plain expression, in the original evaluation order, for every runtime operand.  For finite
// operands the values are unchanged (up to the sign of a zero).  Measured: DESIGN.md §7.
__device__ __forceinline__ bool kz(double x) { return __builtin_constant_p(x) && x == 0.0; }
__device__ __forceinline__ bool kz(const dual&) { return false; }
template <class A, class B>
__device__ __forceinline__ auto kmul(const A& a, const B& b) {  // a b
  using R = decltype(a * b);
  if (kz(a) || kz(b)) return zero<R>();
  return R(a * b);
}
template <class T>
__device__ __forceinline__ T kadd(const T& a, const T& b) {  // a + b
  if (kz(b)) return a;
  if (kz(a)) return b;
  return a + b;
}
template <class T>
__device__ __forceinline__ T ksub(const T& a, const T& b) {  // a - b
  if (kz(b)) return a;
  if (kz(a)) return -b;
  return a - b;
}
template <class T, class A, class B>
__device__ __forceinline__ T kmadd(const T& s, const A& a, const B& b) {  // s + a b
  if (kz(a) || kz(b)) return s;
  if (kz(s)) return T(a * b);
  return s + a * b;
}
template <class T, class A, class B>
__device__ __forceinline__ T kmsub(const T& s, const A& a, const B& b) {  // s - a b
  if (kz(a) || kz(b)) return s;
  if (kz(s)) return -T(a * b);
  return s - a * b;
}
// a0 b0 + a1 b1 + a2 b2, left to right
template <class A, class B>
__device__ __forceinline__ auto kdot3(const A& a0, const B& b0, const A& a1, const B& b1, const A& a2, const B& b2) {
  return kmadd(kmadd(kmul(a0, b0), a1, b1), a2, b2);
}

// a x b
template <class T>
__device__ __forceinline__ void cross3(const T a[3], const T b[3], T o[3]) {
  o[0] = kmsub(kmul(a[1], b[2]), a[2], b[1]);
  o[1] = kmsub(kmul(a[2], b[0]), a[0], b[2]);
  o[2] = kmsub(kmul(a[0], b[1]), a[1], b[0]);
}

// y = Rp^T x   (Rp constant, row-major)
template <class T>
__device__ __forceinline__ void rpT(const double* R, const T x[3], T y[3]) {
  y[0] = kdot3(R[0], x[0], R[3], x[1], R[6], x[2]);
  y[1] = kdot3(R[1], x[0], R[4], x[1], R[7], x[2]);
  y[2] = kdot3(R[2], x[0], R[5], x[1], R[8], x[2]);
}
// y = Rp x
template <class T>
__device__ __forceinline__ void rp(const double* R, const T x[3], T y[3]) {
  y[0] = kdot3(R[0], x[0], R[1], x[1], R[2], x[2]);
  y[1] = kdot3(R[3], x[0], R[4], x[1], R[5], x[2]);
  y[2] = kdot3(R[6], x[0], R[7], x[1], R[8], x[2]);
}

// Spatial inertia (about joint origin) times motion (l, w): lin = m l - h x w, ang = Io w + h x l
template <class T>
__device__ __forceinline__ void inertia_mul(const DevModel& M, int i, const T l[3], const T w[3], T fl[3],
                                            T fn[3]) {
  const double m = M.m[i];
  const double* h = M.h[i];
  const double* I = M.Io[i];
  fl[0] = ksub(kmul(m, l[0]), kmsub(kmul(h[1], w[2]), h[2], w[1]));
  fl[1] = ksub(kmul(m, l[1]), kmsub(kmul(h[2], w[0]), h[0], w[2]));
  fl[2] = ksub(kmul(m, l[2]), kmsub(kmul(h[0], w[1]), h[1], w[0]));
  fn[0] = kadd(kdot3(I[0], w[0], I[1], w[1], I[2], w[2]), kmsub(kmul(h[1], l[2]), h[2], l[1]));
  fn[1] = kadd(kdot3(I[1], w[0], I[3], w[1], I[4], w[2]), kmsub(kmul(h[2], l[0]), h[0], l[2]));
  fn[2] = kadd(kdot3(I[2], w[0], I[4], w[1], I[5], w[2]), kmsub(kmul(h[0], l[1]), h[1], l[0]));
}

// LDS parking of RNEA link forces (NLDS > 0, T = double only): element (link i, component k)
// of this lane at fs[(6 i + k) * 64] — lane-interleaved, so a wave's accesses hit 64 banks.
template <class T> __device__ __forceinline__ void lds_put(double* p, const T& v);
template <> __device__ __forceinline__ void lds_put<double>(double* p, const double& v) { *p = v; }
template <> __device__ __forceinline__ void lds_put<dual>(double*, const dual&) {}

// Recursive Newton-Euler, local frames. c/s = cos/sin(q). Writes tau.
// fext6: optional local spatial force (lin, ang) on the last body (pinocchio f_ext[6]).
// NLDS: the forces of links 0..NLDS-1, which live from the forward to the end of the backward
// sweep, are kept in LDS (fs) instead of registers.
template <class T, int NLDS = 0>
__device__ __forceinline__ void rnea(const DevModel& M, const T c[6], const T s[6], const T qd[6], const T qdd[6],
                                     bool grav, const double* fext6, T tau[6], double* fs = nullptr) {
  T vl[3] = {zero<T>(), zero<T>(), zero<T>()};
  T vw[3] = {zero<T>(), zero<T>(), zero<T>()};
  T al[3], aw[3] = {zero<T>(), zero<T>(), zero<T>()};
  al[0] = cst<T>(grav ? -M.g[0] : 0.0);
  al[1] = cst<T>(grav ? -M.g[1] : 0.0);
  al[2] = cst<T>(grav ? -M.g[2] : 0.0);
  T f[6][6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    __builtin_amdgcn_sched_barrier(0);
    const double* R = M.Rp[i];
    const double* t = M.tp[i];
    // parent -> child: y = Rz^T Rp^T (x - t x w)
    T tw[3], x[3], y[3];
    T tt[3] = {cst<T>(t[0]), cst<T>(t[1]), cst<T>(t[2])};
    cross3(tt, vw, tw);
    x[0] = ksub(vl[0], tw[0]); x[1] = ksub(vl[1], tw[1]); x[2] = ksub(vl[2], tw[2]);
    rpT(R, x, y);
    vl[0] = kmadd(kmul(c[i], y[0]), s[i], y[1]);
    vl[1] = kmsub(kmul(c[i], y[1]), s[i], y[0]);
    vl[2] = y[2];
    rpT(R, vw, y);
    vw[0] = kmadd(kmul(c[i], y[0]), s[i], y[1]);
    vw[1] = kmsub(kmul(c[i], y[1]), s[i], y[0]);
    vw[2] = y[2];
    cross3(tt, aw, tw);
    x[0] = ksub(al[0], tw[0]); x[1] = ksub(al[1], tw[1]); x[2] = ksub(al[2], tw[2]);
    rpT(R, x, y);
    al[0] = kmadd(kmul(c[i], y[0]), s[i], y[1]);
    al[1] = kmsub(kmul(c[i], y[1]), s[i], y[0]);
    al[2] = y[2];
    rpT(R, aw, y);
    aw[0] = kmadd(kmul(c[i], y[0]), s[i], y[1]);
    aw[1] = kmsub(kmul(c[i], y[1]), s[i], y[0]);
    aw[2] = y[2];
    // joint motion: v += S qd ; a += S qdd + v x (S qd)
    vw[2] = kadd(vw[2], qd[i]);
    al[0] = kmadd(al[0], vl[1], qd[i]);
    al[1] = kmsub(al[1], vl[0], qd[i]);
    aw[0] = kmadd(aw[0], vw[1], qd[i]);
    aw[1] = kmsub(aw[1], vw[0], qd[i]);
    aw[2] = kadd(aw[2], qdd[i]);
    // f = I a + v x* (I v)
    T hl[3], hn[3], il[3], in_[3], t1[3], t2[3], t3[3];
    inertia_mul(M, i, vl, vw, hl, hn);
    inertia_mul(M, i, al, aw, il, in_);
    cross3(vw, hl, t1);
    cross3(vw, hn, t2);
    cross3(vl, hl, t3);
    T fi[6];
    fi[0] = kadd(il[0], t1[0]); fi[1] = kadd(il[1], t1[1]); fi[2] = kadd(il[2], t1[2]);
    fi[3] = kadd(kadd(in_[0], t2[0]), t3[0]);
    fi[4] = kadd(kadd(in_[1], t2[1]), t3[1]);
    fi[5] = kadd(kadd(in_[2], t2[2]), t3[2]);
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      if (i < NLDS) lds_put<T>(fs + (6 * i + k) * 64, fi[k]);
      else f[i][k] = fi[k];
    }
  }
  if (fext6 && NLDS < 6) {
#pragma unroll
    for (int k = 0; k < 6; ++k) f[5][k] = f[5][k] - cst<T>(fext6[k]);
  }
  // a parked link's force is read back one link ahead (during the previous link's transform),
  // so the LDS reads are in flight while that arithmetic runs
  double pk[6];
  if (NLDS == 6) {
#pragma unroll
    for (int k = 0; k < 6; ++k) pk[k] = fs[(30 + k) * 64];
  }
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    __builtin_amdgcn_sched_barrier(0);
    if (i < NLDS) {
      if (i == 5) {  // the tip: no child contribution; the external wrench acts here
#pragma unroll
        for (int k = 0; k < 6; ++k) f[5][k] = cst<T>(pk[k]) - cst<T>(fext6 ? fext6[k] : 0.0);
      } else {
#pragma unroll
        for (int k = 0; k < 6; ++k) f[i][k] = cst<T>(pk[k]) + f[i][k];
      }
    }
    if (i > 0 && i - 1 < NLDS) {
#pragma unroll
      for (int k = 0; k < 6; ++k) pk[k] = fs[(6 * (i - 1) + k) * 64];
    }
    tau[i] = f[i][5];
    if (i > 0) {
      const double* R = M.Rp[i];
      const double* t = M.tp[i];
      // child -> parent: F = Rp Rz f ; N = Rp Rz n + t x F
      T x[3], F[3], Nn[3], tF[3];
      x[0] = kmsub(kmul(c[i], f[i][0]), s[i], f[i][1]);
      x[1] = kmadd(kmul(s[i], f[i][0]), c[i], f[i][1]);
      x[2] = f[i][2];
      rp(R, x, F);
      x[0] = kmsub(kmul(c[i], f[i][3]), s[i], f[i][4]);
      x[1] = kmadd(kmul(s[i], f[i][3]), c[i], f[i][4]);
      x[2] = f[i][5];
      rp(R, x, Nn);
      T tt[3] = {cst<T>(t[0]), cst<T>(t[1]), cst<T>(t[2])};
      cross3(tt, F, tF);
      if (i - 1 < NLDS) {
        // parked link: its own force is added when the sweep reaches it
        f[i - 1][0] = F[0];
        f[i - 1][1] = F[1];
        f[i - 1][2] = F[2];
        f[i - 1][3] = kadd(Nn[0], tF[0]);
        f[i - 1][4] = kadd(Nn[1], tF[1]);
        f[i - 1][5] = kadd(Nn[2], tF[2]);
      } else {
        f[i - 1][0] = kadd(f[i - 1][0], F[0]);
        f[i - 1][1] = kadd(f[i - 1][1], F[1]);
        f[i - 1][2] = kadd(f[i - 1][2], F[2]);
        f[i - 1][3] = kadd(kadd(f[i - 1][3], Nn[0]), tF[0]);
        f[i - 1][4] = kadd(kadd(f[i - 1][4], Nn[1]), tF[1]);
        f[i - 1][5] = kadd(kadd(f[i - 1][5], Nn[2]), tF[2]);
      }
    }
  }
}

// Composite-rigid-body algorithm: joint-space inertia M (full, symmetric).  One running
// composite inertia (m, h, I about the current joint origin) is carried from the tip to the
// base, so only ~10 doubles of composite state are live at any time.
__device__ __forceinline__ void crba(const DevModel& Md, const double c[6], const double s[6], double Mq[6][6]) {
  double cm = Md.m[5], ch[3] = {Md.h[5][0], Md.h[5][1], Md.h[5][2]};
  double cI[6] = {Md.Io[5][0], Md.Io[5][1], Md.Io[5][2], Md.Io[5][3], Md.Io[5][4], Md.Io[5][5]};
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    __builtin_amdgcn_sched_barrier(0);
    // column i: F = IC_i S, S = (0; e_z): lin = e_z x h = (-h_y, h_x, 0), ang = I e_z
    double fl[3] = {-ch[1], ch[0], 0.0};
    double fn[3] = {cI[2], cI[4], cI[5]};
    Mq[i][i] = fn[2];
#pragma unroll
    for (int j = i; j >= 1; --j) {
      // express F (frame j) in frame j-1, then M[j-1][i] = n_z
      const double* R = Md.Rp[j];
      const double* t = Md.tp[j];
      double x[3], F[3], Nn[3];
      x[0] = kmsub(kmul(c[j], fl[0]), s[j], fl[1]);
      x[1] = kmadd(kmul(s[j], fl[0]), c[j], fl[1]);
      x[2] = fl[2];
      rp(R, x, F);
      x[0] = kmsub(kmul(c[j], fn[0]), s[j], fn[1]);
      x[1] = kmadd(kmul(s[j], fn[0]), c[j], fn[1]);
      x[2] = fn[2];
      rp(R, x, Nn);
      fn[0] = kadd(Nn[0], kmsub(kmul(t[1], F[2]), t[2], F[1]));
      fn[1] = kadd(Nn[1], kmsub(kmul(t[2], F[0]), t[0], F[2]));
      fn[2] = kadd(Nn[2], kmsub(kmul(t[0], F[1]), t[1], F[0]));
      fl[0] = F[0]; fl[1] = F[1]; fl[2] = F[2];
      Mq[i][j - 1] = fn[2];
      Mq[j - 1][i] = fn[2];
    }
    if (i > 0) {
      // IC_{i-1} = I_{i-1} + X_i^* IC_i X_i^{-1}: rotate (R = Rp Rz), then shift by t
      const double* R = Md.Rp[i];
      const double* t = Md.tp[i];
      const double m = cm;
      double hz[3] = {kmsub(kmul(c[i], ch[0]), s[i], ch[1]), kmadd(kmul(s[i], ch[0]), c[i], ch[1]), ch[2]};
      double hr[3];
      rp(R, hz, hr);
      const double* I = cI;
      const double cc = c[i] * c[i], ss = s[i] * s[i], cs = c[i] * s[i];
      double A[3][3];
      A[0][0] = cc * I[0] - 2.0 * cs * I[1] + ss * I[3];
      A[1][1] = ss * I[0] + 2.0 * cs * I[1] + cc * I[3];
      A[0][1] = cs * (I[0] - I[3]) + (cc - ss) * I[1];
      A[0][2] = c[i] * I[2] - s[i] * I[4];
      A[1][2] = s[i] * I[2] + c[i] * I[4];
      A[2][2] = I[5];
      A[1][0] = A[0][1]; A[2][0] = A[0][2]; A[2][1] = A[1][2];
      double RA[3][3];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int q = 0; q < 3; ++q) RA[r][q] = kdot3(R[3 * r], A[0][q], R[3 * r + 1], A[1][q], R[3 * r + 2], A[2][q]);
      double Bm[3][3];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int q = r; q < 3; ++q) Bm[r][q] = kdot3(RA[r][0], R[3 * q], RA[r][1], R[3 * q + 1], RA[r][2], R[3 * q + 2]);
      const double ht = kdot3(hr[0], t[0], hr[1], t[1], hr[2], t[2]);
      const double tt = t[0] * t[0] + t[1] * t[1] + t[2] * t[2];
      const double dg = 2.0 * ht + m * tt;
      const int iu[6][2] = {{0, 0}, {0, 1}, {0, 2}, {1, 1}, {1, 2}, {2, 2}};
      double nI[6];
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const int r = iu[k][0], q = iu[k][1];
        double v = ksub(ksub(Bm[r][q], kmadd(kmul(t[r], hr[q]), hr[r], t[q])), kmul(kmul(m, t[r]), t[q]));
        if (r == q) v += dg;
        nI[k] = Md.Io[i - 1][k] + v;
      }
#pragma unroll
      for (int k = 0; k < 6; ++k) cI[k] = nI[k];
      ch[0] = kadd(Md.h[i - 1][0], kmadd(hr[0], m, t[0]));
      ch[1] = kadd(Md.h[i - 1][1], kmadd(hr[1], m, t[1]));
      ch[2] = kadd(Md.h[i - 1][2], kmadd(hr[2], m, t[2]));
      cm = Md.m[i - 1] + m;
    }
  }
}

// 1/sqrt(d) to full fp64 precision: hardware v_rsq_f64 + one Newton step (instead of the
// IEEE sqrt and divide sequences, ~25 dependent instructions each).
__device__ __forceinline__ double rsqrt_nr(double d) {
  const double y = __builtin_amdgcn_rsq(d);
  return y * (1.5 - 0.5 * d * y * y);
}

// In-place Cholesky of a 6x6 SPD matrix: strict lower triangle = L, diagonal = 1 / L_jj.
__device__ __forceinline__ void chol6(double A[6][6]) {
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    double d = A[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) d -= A[j][k] * A[j][k];
    const double inv = rsqrt_nr(d);
    A[j][j] = inv;
#pragma unroll
    for (int i = j + 1; i < 6; ++i) {
      double v = A[i][j];
#pragma unroll
      for (int k = 0; k < j; ++k) v -= A[i][k] * A[j][k];
      A[i][j] = v * inv;
    }
  }
}
// Solve L L^T x = b in place (L from chol6: diagonal holds the reciprocals).
__device__ __forceinline__ void chol6_solve(const double L[6][6], double b[6]) {
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double v = b[i];
#pragma unroll
    for (int k = 0; k < i; ++k) v -= L[i][k] * b[k];
    b[i] = v * L[i][i];
  }
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    double v = b[i];
#pragma unroll
    for (int k = i + 1; k < 6; ++k) v -= L[k][i] * b[k];
    b[i] = v * L[i][i];
  }
}

// a = ABA(q, v, tau[, fext]) = M^-1 (tau - RNEA(q, v, 0)); L returns chol(M).
// NLDS / fs: see rnea (LDS parking of link forces).
template <int NLDS = 0>
__device__ __forceinline__ void forward_dynamics(const DevModel& Md, const double c[6], const double s[6],
                                                 const double v[6], const double tau[6], const double* fext6,
                                                 double L[6][6], double a[6], double* fs = nullptr) {
  double z[6] = {0, 0, 0, 0, 0, 0}, b[6];
  rnea<double, NLDS>(Md, c, s, v, z, true, fext6, b, fs);
#pragma unroll
  for (int i = 0; i < 6; ++i) a[i] = tau[i] - b[i];
  __builtin_amdgcn_sched_barrier(0);
  crba(Md, c, s, L);
  chol6(L);
  chol6_solve(L, a);
}

// Column `d` of the ABA derivatives at (q, v, a): d < 6 -> da/dq_d, 6 <= d < 12 -> da/dv_{d-6}.
// out = -M^-1 dRNEA/dx_d (a held fixed).
__device__ __forceinline__ void aba_deriv_column(const DevModel& Md, const double c[6], const double s[6],
                                                 const double v[6], const double a[6], const double L[6][6],
                                                 int d, const double* fext6, double out[6]) {
  dual dc[6], ds[6], dv[6], da[6], dt[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const bool isq = (d == i);
    dc[i] = dual{c[i], isq ? -s[i] : 0.0};
    ds[i] = dual{s[i], isq ? c[i] : 0.0};
    dv[i] = dual{v[i], (d - 6 == i) ? 1.0 : 0.0};
    da[i] = dual{a[i], 0.0};
  }
  rnea<dual>(Md, dc, ds, dv, da, true, fext6, dt);
#pragma unroll
  for (int i = 0; i < 6; ++i) out[i] = -dt[i].d;
  chol6_solve(L, out);
}

// Joint-6 origin in the world frame only (no Jacobian), by Horner's rule from the tip:
// p = t_0 + R_0 (t_1 + R_1 (... + R_4 t_5)), R_i = Rp_i Rz(q_i): ~16 ops per joint instead of the
// rotation-chain composition's ~48 (same point as fk_jac to rounding).
__device__ __forceinline__ void fk_pos(const DevModel& Md, const double c[6], const double s[6], double p[3]) {
  double w[3] = {Md.tp[5][0], Md.tp[5][1], Md.tp[5][2]};
#pragma unroll
  for (int i = 4; i >= 0; --i) {
    const double x[3] = {kmsub(kmul(c[i], w[0]), s[i], w[1]), kmadd(kmul(s[i], w[0]), c[i], w[1]), w[2]};
    double y[3];
    rp(Md.Rp[i], x, y);
    w[0] = kadd(Md.tp[i][0], y[0]);
    w[1] = kadd(Md.tp[i][1], y[1]);
    w[2] = kadd(Md.tp[i][2], y[2]);
  }
  p[0] = w[0];
  p[1] = w[1];
  p[2] = w[2];
}

// External wrench given in the WORLD frame (a spatial force [f; n] about the world origin, as
// the reference's callers build it: pin.Force(f_ext[:3], f_ext[3:]), src/gato_mpc_batch_sample.py:
// 155-158) -> the joint-6 LOCAL frame the dynamics take (pinocchio f_ext[6]):
// data.oMi[6].actInv(world_force) (:160), i.e. f_l = R' f, n_l = R' (n - p x f), with (R, p) the
// world placement of joint 6 at the configuration (c, s) = cos / sin(q).
__device__ __forceinline__ void wrench_world_to_local(const DevModel& Md, const double c[6], const double s[6],
                                                      const double* fw, double fl[6]) {
  double R[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
  double p[3] = {0, 0, 0};
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const double* Rp = Md.Rp[i];
    const double* t = Md.tp[i];
    double np_[3], RR[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r) np_[r] = kmadd(kmadd(kmadd(p[r], R[r][0], t[0]), R[r][1], t[1]), R[r][2], t[2]);
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int q = 0; q < 3; ++q) RR[r][q] = kdot3(R[r][0], Rp[q], R[r][1], Rp[3 + q], R[r][2], Rp[6 + q]);
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      R[r][0] = kmadd(kmul(RR[r][0], c[i]), RR[r][1], s[i]);
      R[r][1] = kmsub(kmul(RR[r][1], c[i]), RR[r][0], s[i]);
      R[r][2] = RR[r][2];
      p[r] = np_[r];
    }
  }
  const double f0 = fw[0], f1 = fw[1], f2 = fw[2];
  const double m0 = fw[3] - (p[1] * f2 - p[2] * f1);
  const double m1 = fw[4] - (p[2] * f0 - p[0] * f2);
  const double m2 = fw[5] - (p[0] * f1 - p[1] * f0);
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    fl[q] = kdot3(R[0][q], f0, R[1][q], f1, R[2][q], f2);
    fl[3 + q] = kdot3(R[0][q], m0, R[1][q], m1, R[2][q], m2);
  }
}

// World-frame forward kinematics of the joint-6 origin and its LOCAL_WORLD_ALIGNED linear
// Jacobian (rows 0..2).  J may be null.
__device__ __forceinline__ void fk_jac(const DevModel& Md, const double c[6], const double s[6], double p[3],
                                       double J[3][6]) {
  double R[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
  double pos[3] = {0, 0, 0};
  double zs[6][3], ps[6][3];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    __builtin_amdgcn_sched_barrier(0);
    const double* Rp = Md.Rp[i];
    const double* t = Md.tp[i];
    double np[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) np[r] = kmadd(kmadd(kmadd(pos[r], R[r][0], t[0]), R[r][1], t[1]), R[r][2], t[2]);
    // R <- R Rp Rz(q)
    double RR[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int q = 0; q < 3; ++q) RR[r][q] = kdot3(R[r][0], Rp[q], R[r][1], Rp[3 + q], R[r][2], Rp[6 + q]);
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const double x0 = RR[r][0], x1 = RR[r][1];
      R[r][0] = kmadd(kmul(x0, c[i]), x1, s[i]);
      R[r][1] = kmsub(kmul(x1, c[i]), x0, s[i]);
      R[r][2] = RR[r][2];
      zs[i][r] = RR[r][2];
      ps[i][r] = np[r];
      pos[r] = np[r];
    }
  }
  p[0] = pos[0]; p[1] = pos[1]; p[2] = pos[2];
  if (J) {
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const double d0 = ksub(pos[0], ps[j][0]), d1 = ksub(pos[1], ps[j][1]), d2 = ksub(pos[2], ps[j][2]);
      J[0][j] = kmsub(kmul(zs[j][1], d2), zs[j][2], d1);
      J[1][j] = kmsub(kmul(zs[j][2], d0), zs[j][0], d2);
      J[2][j] = kmsub(kmul(zs[j][0], d1), zs[j][1], d0);
    }
  }
}

}  // namespace i7m
