// i7m_linearize.h — knot-parallel linearisation of the SQP subproblem (gfx950, fp64).
//
// Replaces, per knot k of every problem (reference src/osqp_solver.py:70-135):
//   pin.computeABADerivatives + data.ddq + pin.integrate   (compute_dynamics_jacobians :70-81)
//   FK + LOCAL_WORLD_ALIGNED Jacobian + cost weights       (update_cost_matrix :103-135)
//
// Algorithm: analytic O(n^2) derivatives of inverse dynamics in the WORLD frame (the
// Carpentier-Mansard idea, restated from first principles): with S_j the world joint axes,
// V_j, A_j body velocities/accelerations, I_j world inertias, IC_j / dIC_j / HC_j the
// subtree sums of I_i, dI_i = V_i x* I_i - I_i V_i x (symmetric), I_i V_i, F^c the subtree
// forces, W_k = S_k x V_k, Z_k = S_k x A_k - W_k x V_k:
//   a_j = IC_j S_j, e_j = dIC_j S_j - S_j x* HC_j
//   j >= k: dtau_j/dq_k = -(a_j.Z_k + e_j.W_k),          dtau_j/dv_k = e_j.S_k - 2 a_j.W_k
//   j <  k: dtau_j/dq_k = S_j.y_k,  y_k = S_k x* F^c_k - IC_k Z_k - dIC_k W_k - W_k x* HC_k
//           dtau_j/dv_k = S_j.z_k,  z_k = dIC_k S_k - 2 IC_k W_k + S_k x* HC_k
//   M_jk = a_j.S_k (j >= k);  da/dx = -M^-1 dtau/dx at a = M^-1 (tau - b).
// (Verified against complex-step RNEA to 1e-16 relative; tests/test_gpu_parity.py checks the
// kernel against the oracle and against the independent dual-number path k_abad.)
//
// Lane mapping: one 64-lane wavefront = KPW knots x 6 link-lanes (lanes 60..63 idle); lane
// (g, j) owns link j of knot g.  The serial kinematic chain (~600 flops) is recomputed by every
// link-lane; the per-link work (world inertia, its rate, forces, subtree sums, one column of the
// derivative matrices and of M^-1) is split across the lanes; the lanes of a knot exchange
// per-link vectors through LDS in three rounds of <= 19 doubles per lane (inertias and rates;
// momenta and bias forces; a_j, e_j, S_j), each consumed as soon as it lands, and everything
// that does not need the joint accelerations is formed before M is factorised, so the register
// peak stays low.  The terminal knot of each problem only evaluates the cost.
#pragma once

#include "i7m_kernels.h"

namespace i7m {

constexpr int KPW = 10;   // knots per wavefront
constexpr int XS = 20;    // LDS doubles per link slot (round 1 uses 19)

// Where the 6x6 factor of M lives: 0 = every lane's registers (chol6; default), 1 = LDS,
// factorised by the knot's six lanes together (21 doubles fewer per lane).  Measured on
// MI355X at B = 4096: registers 96.1 us, LDS 99.7 us per launch.
#ifndef I7M_LIN_CHOL_LDS
#define I7M_LIN_CHOL_LDS 0
#endif

// Occupancy target of k_linearize (amdgpu_waves_per_eu): 0 = the compiler's choice (242 VGPRs,
// 2 waves per SIMD; default).  3 caps it at 168 VGPRs (its 12.7 KB of LDS allows 3 waves) and
// spills 21-42 VGPRs: 105-118 us against 96 us.
#ifndef I7M_LIN_WPE
#define I7M_LIN_WPE 0
#endif
#if I7M_LIN_WPE > 0
#define I7M_LIN_OCC __attribute__((amdgpu_waves_per_eu(I7M_LIN_WPE, I7M_LIN_WPE)))
#else
#define I7M_LIN_OCC
#endif

// spatial helpers on 6-vectors [lin; ang]
__device__ __forceinline__ void mcross(const double* a, const double* b, double* o) {  // a x b (motion)
  o[0] = kmsub(kmadd(kmsub(kmul(a[4], b[2]), a[5], b[1]), a[1], b[5]), a[2], b[4]);
  o[1] = kmsub(kmadd(kmsub(kmul(a[5], b[0]), a[3], b[2]), a[2], b[3]), a[0], b[5]);
  o[2] = kmsub(kmadd(kmsub(kmul(a[3], b[1]), a[4], b[0]), a[0], b[4]), a[1], b[3]);
  o[3] = kmsub(kmul(a[4], b[5]), a[5], b[4]);
  o[4] = kmsub(kmul(a[5], b[3]), a[3], b[5]);
  o[5] = kmsub(kmul(a[3], b[4]), a[4], b[3]);
}
__device__ __forceinline__ void fcross(const double* m, const double* f, double* o) {  // m x* f
  o[0] = m[4] * f[2] - m[5] * f[1];
  o[1] = m[5] * f[0] - m[3] * f[2];
  o[2] = m[3] * f[1] - m[4] * f[0];
  o[3] = m[4] * f[5] - m[5] * f[4] + m[1] * f[2] - m[2] * f[1];
  o[4] = m[5] * f[3] - m[3] * f[5] + m[2] * f[0] - m[0] * f[2];
  o[5] = m[3] * f[4] - m[4] * f[3] + m[0] * f[1] - m[1] * f[0];
}
__device__ __forceinline__ double dot6(const double* a, const double* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}
// inertia (m, h[3], I[6] sym xx xy xz yy yz zz, about the world origin) times motion x
__device__ __forceinline__ void imul(double m, const double* h, const double* I, const double* x, double* o) {
  o[0] = ksub(kmul(m, x[0]), kmsub(kmul(h[1], x[5]), h[2], x[4]));
  o[1] = ksub(kmul(m, x[1]), kmsub(kmul(h[2], x[3]), h[0], x[5]));
  o[2] = ksub(kmul(m, x[2]), kmsub(kmul(h[0], x[4]), h[1], x[3]));
  o[3] = kadd(kdot3(I[0], x[3], I[1], x[4], I[2], x[5]), kmsub(kmul(h[1], x[2]), h[2], x[1]));
  o[4] = kadd(kdot3(I[1], x[3], I[3], x[4], I[4], x[5]), kmsub(kmul(h[2], x[0]), h[0], x[2]));
  o[5] = kadd(kdot3(I[2], x[3], I[4], x[4], I[5], x[5]), kmsub(kmul(h[0], x[1]), h[1], x[0]));
}

// Solve L L^T x = b in place, L from chol6's layout (strict lower triangle = L, diagonal =
// 1 / L_jj), row-major 6x6 in LDS, read entry by entry (the operation order of chol6_solve).
__device__ __forceinline__ void chol6_solve_lds(const double* Lm, double b[6]) {
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double v = b[i];
#pragma unroll
    for (int k = 0; k < i; ++k) v -= Lm[6 * i + k] * b[k];
    b[i] = v * Lm[6 * i + i];
  }
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    double v = b[i];
#pragma unroll
    for (int k = i + 1; k < 6; ++k) v -= Lm[6 * k + i] * b[k];
    b[i] = v * Lm[6 * i + i];
  }
}

// Padding after each knot's six link slots (doubles).  The lanes of a knot read the same slot
// (a broadcast) while the knots of a ds_read_b128 lane group read different ones, so the knot
// stride decides the bank conflicts: unpadded (120 doubles = 240 dwords, 48 mod 64 banks) knots
// g and g + 4 share banks and every slot read was a 2-way conflict (SQ_LDS_BANK_CONFLICT: 3.3
// extra cycles per LDS instruction); 124 doubles (56 mod 64) give every knot of each lane group
// ({0,2,3,4}, {0..5}, {5,7,8,9}, {6,7,8} + the idle lanes, which read knot KPW - 1) its own
// four banks.
#ifndef I7M_LIN_XPAD
#define I7M_LIN_XPAD 4
#endif
struct alignas(16) KnotSlots {
  double s[6][XS];
#if I7M_LIN_XPAD > 0
  double pad[I7M_LIN_XPAD];
#endif
  __device__ __forceinline__ double* operator[](int i) { return s[i]; }
};
// LDS of one wave's linearisation pass (KPW knots): per-link exchange slots, M, RNEA bias.  16-byte
// aligned: the slot reads are ds_read_b128 (with 8-byte alignment the compiler falls back to
// ds_read2_b64, twice the LDS cycles: k_linearize 130 -> 203 us measured).
struct alignas(16) LinLds {
  KnotSlots xs[KPW];
  double sM[KPW][36];
  double st0[KPW][6];
};
constexpr int LINLDS_DOUBLES = (int)(sizeof(LinLds) / sizeof(double));

// The linearisation of knot k of problem b by the six lanes 6g..6g+5 of one wavefront (lane l,
// g = l / 6 < KPW); `valid` false: the lanes take part in the wave's exchanges but compute and
// store nothing of use.  The LDS region S belongs to this wave alone (wave_sync only), so the
// body runs in k_linearize (KPW knots of consecutive problems per wave) and in k_sqp_fused (the
// knots of one problem, several waves side by side).
// FW: the external wrench (fext, (B, 6) per problem) is a WORLD-frame spatial force about the
// world origin (I7M_WRENCH_WORLD); otherwise it is constant in the joint-6 frame (pinocchio
// f_ext, I7M_WRENCH_LOCAL).
template <bool SPEC, bool FW = false>
__device__ __forceinline__ void linearize_body(const DevModel* __restrict__ Mg, const SolveParams& P, const int b,
                                               const int k, const bool valid, const int l, LinLds& S,
                                               const double* __restrict__ xu, const double* __restrict__ goals,
                                               const double* __restrict__ fext, double* __restrict__ lin,
                                               double* __restrict__ cost, double* __restrict__ qpd) {
  const DevModel& Md = SPEC ? kIndy7Model : *Mg;
  const int g = l / 6;
  const int j = l - 6 * g;
  const bool dyn = valid && (k < P.N - 1);
  const int gg = g < KPW ? g : KPW - 1;  // the idle lanes 60..63 shadow the last knot (broadcast reads)
  auto& xs = S.xs;
  auto& sM = S.sM;
  auto& st0 = S.st0;

  const double* X = xu + (long)(valid ? b : 0) * P.T + 18 * (valid ? k : 0);
  double v[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) v[i] = (dyn ? X[6 + i] : 0.0);
  // each link-lane evaluates sincos of its own joint only; the knot's six lanes share them
  double c[6], s[6];
  {
    double sj, cj;
    sincos_q(X[j], &sj, &cj);
    const int base = 6 * gg;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      c[i] = __shfl(cj, base + i, 64);
      s[i] = __shfl(sj, base + i, 64);
    }
  }

  // ---- 1. serial chain: world placement of each joint, S, V, A0 (qdd = 0).  Lane j runs the
  // chain up to its own link (the updates of links i > j are masked off), so its registers end
  // holding link j's values with no per-link copies; the end-effector position comes from the
  // knot's link-5 lane.
  double Rj[9], pj[3], Sj[6], Vj[6], A0j[6], pE[3];
  {
    double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    double p[3] = {0, 0, 0};
    double V[6] = {0, 0, 0, 0, 0, 0};
    double A[6] = {-Md.g[0], -Md.g[1], -Md.g[2], 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      if (i <= j) {
        const double* Rp = Md.Rp[i];
        const double* t = Md.tp[i];
        double np_[3], RR[9];
#pragma unroll
        for (int r = 0; r < 3; ++r)
          np_[r] = kmadd(kmadd(kmadd(p[r], R[3 * r], t[0]), R[3 * r + 1], t[1]), R[3 * r + 2], t[2]);
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
          for (int qq = 0; qq < 3; ++qq) RR[3 * r + qq] = kdot3(R[3 * r], Rp[qq], R[3 * r + 1], Rp[3 + qq], R[3 * r + 2], Rp[6 + qq]);
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          R[3 * r] = kmadd(kmul(RR[3 * r], c[i]), RR[3 * r + 1], s[i]);
          R[3 * r + 1] = kmsub(kmul(RR[3 * r + 1], c[i]), RR[3 * r], s[i]);
          R[3 * r + 2] = RR[3 * r + 2];
          p[r] = np_[r];
        }
        // S = (p x z; z), z = R[:,2]
        double S[6];
        S[3] = R[2]; S[4] = R[5]; S[5] = R[8];
        S[0] = kmsub(kmul(p[1], S[5]), p[2], S[4]);
        S[1] = kmsub(kmul(p[2], S[3]), p[0], S[5]);
        S[2] = kmsub(kmul(p[0], S[4]), p[1], S[3]);
#pragma unroll
        for (int r = 0; r < 6; ++r) V[r] = kmadd(V[r], S[r], v[i]);
        double VS[6];
        mcross(V, S, VS);
#pragma unroll
        for (int r = 0; r < 6; ++r) A[r] = kmadd(A[r], VS[r], v[i]);
      }
    }
#pragma unroll
    for (int r = 0; r < 9; ++r) Rj[r] = R[r];
#pragma unroll
    for (int r = 0; r < 3; ++r) pj[r] = p[r];
#pragma unroll
    for (int r = 0; r < 6; ++r) { Vj[r] = V[r]; A0j[r] = A[r]; }
    Sj[3] = R[2]; Sj[4] = R[5]; Sj[5] = R[8];
    Sj[0] = p[1] * Sj[5] - p[2] * Sj[4];
    Sj[1] = p[2] * Sj[3] - p[0] * Sj[5];
    Sj[2] = p[0] * Sj[4] - p[1] * Sj[3];
    // joint-6 origin = the end effector: from the knot's link-5 lane
#pragma unroll
    for (int r = 0; r < 3; ++r) pE[r] = __shfl(p[r], 6 * gg + 5, 64);
  }

  double jte = 0.0, wreg = 1.0;  // (J^T e)_j and the cost regularisation weight of this knot
  // ---- cost linearisation (src/osqp_solver.py:103-135) from the chain: e = p_E - goal;
  // LOCAL_WORLD_ALIGNED column J_j = z_j x (p_E - p_j) = z_j x p_E + (p_j x z_j), so lane j
  // writes (J^T e)_j; lane 0 the weights.
  if (valid) {
    const double* goal = goals + (long)b * P.N * P.goal_stride + (long)k * P.goal_stride;
    const double e0 = pE[0] - goal[0], e1 = pE[1] - goal[1], e2 = pE[2] - goal[2];
    const double* z = Sj + 3;
    const double J0 = (z[1] * pE[2] - z[2] * pE[1]) + Sj[0];
    const double J1 = (z[2] * pE[0] - z[0] * pE[2]) + Sj[1];
    const double J2 = (z[0] * pE[1] - z[1] * pE[0]) + Sj[2];
    double* co = cost + ((long)b * P.N + k) * COST_STRIDE;
    jte = e0 * J0 + e1 * J1 + e2 * J2;
    co[j] = jte;
    const double nrm = sqrt(e0 * e0 + e1 * e1 + e2 * e2);
    wreg = P.regularize ? (1.0 / (fabs(nrm) + P.eps)) : 1.0;
    if (j == 0) {
      co[6] = (k == P.N - 1) ? P.QN : 1.0;
      co[7] = P.dQ * wreg;
      co[8] = P.R * wreg;
      co[9] = nrm;
    }
  }

  // ---- 2. own link: world inertia (m, h, Ib), its rate (hd, Ibd), momentum hV, bias force F0.
  // Everything that needs the link's placement (Rj, pj) is formed here, so it dies after this
  // block; the publish/sum rounds below keep the subtree sums' live ranges short (DESIGN.md §4.1:
  // the register peak decides the waves per SIMD).
  const double m = Md.m[j];
  double h[3], Ib[6], hV[6], F0[6];
  double* my = &xs[gg][j][0];
  double cm = 0, ch[3] = {0, 0, 0}, cI[6] = {0, 0, 0, 0, 0, 0}, chd[3] = {0, 0, 0}, cId[6] = {0, 0, 0, 0, 0, 0};
  {
    const double* hl = Md.h[j];
    const double* Io = Md.Io[j];
    // R Io R^T
    double Iof[9] = {Io[0], Io[1], Io[2], Io[1], Io[3], Io[4], Io[2], Io[4], Io[5]};
    double RI[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int qq = 0; qq < 3; ++qq) RI[3 * r + qq] = Rj[3 * r] * Iof[qq] + Rj[3 * r + 1] * Iof[3 + qq] + Rj[3 * r + 2] * Iof[6 + qq];
    double hr[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) hr[r] = Rj[3 * r] * hl[0] + Rj[3 * r + 1] * hl[1] + Rj[3 * r + 2] * hl[2];
    const double* t = pj;
    const double ht = hr[0] * t[0] + hr[1] * t[1] + hr[2] * t[2];
    const double tt = t[0] * t[0] + t[1] * t[1] + t[2] * t[2];
    const double dg = 2.0 * ht + m * tt;
    const int iu[6][2] = {{0, 0}, {0, 1}, {0, 2}, {1, 1}, {1, 2}, {2, 2}};
#pragma unroll
    for (int e = 0; e < 6; ++e) {
      const int r = iu[e][0], qq = iu[e][1];
      double val = RI[3 * r] * Rj[3 * qq] + RI[3 * r + 1] * Rj[3 * qq + 1] + RI[3 * r + 2] * Rj[3 * qq + 2];
      val -= (t[r] * hr[qq] + hr[r] * t[qq]) + m * t[r] * t[qq];
      if (r == qq) val += dg;
      Ib[e] = val;
    }
#pragma unroll
    for (int r = 0; r < 3; ++r) h[r] = hr[r] + m * t[r];
    imul(m, h, Ib, Vj, hV);
    double IA[6], VxH[6];
    imul(m, h, Ib, A0j, IA);
    fcross(Vj, hV, VxH);
#pragma unroll
    for (int r = 0; r < 6; ++r) F0[r] = IA[r] + VxH[r];
    if (FW && fext && j == 5 && valid) {
      // a world-frame wrench acts on link 6 as it is
      const double* fe = fext + 6L * b;
#pragma unroll
      for (int r = 0; r < 6; ++r) F0[r] -= fe[r];
    } else if (fext && j == 5 && valid) {
      // local joint-6 wrench -> world: f_w = R f, n_w = R n + p x f_w
      const double* fe = fext + 6L * b;
      double fw[3], nw[3];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        fw[r] = Rj[3 * r] * fe[0] + Rj[3 * r + 1] * fe[1] + Rj[3 * r + 2] * fe[2];
        nw[r] = Rj[3 * r] * fe[3] + Rj[3 * r + 1] * fe[4] + Rj[3 * r + 2] * fe[5];
      }
      F0[0] -= fw[0]; F0[1] -= fw[1]; F0[2] -= fw[2];
      F0[3] -= nw[0] + (pj[1] * fw[2] - pj[2] * fw[1]);
      F0[4] -= nw[1] + (pj[2] * fw[0] - pj[0] * fw[2]);
      F0[5] -= nw[2] + (pj[0] * fw[1] - pj[1] * fw[0]);
    }
    // rate: hd = m v + w x h ; Ibd = [w]x Ib - Ib [w]x - h v^T - v h^T + 2 (v.h) I
    const double* vl = Vj;
    const double* w = Vj + 3;
    double hd[3], Ibd[6];
    hd[0] = m * vl[0] + (w[1] * h[2] - w[2] * h[1]);
    hd[1] = m * vl[1] + (w[2] * h[0] - w[0] * h[2]);
    hd[2] = m * vl[2] + (w[0] * h[1] - w[1] * h[0]);
    double Ibf[9] = {Ib[0], Ib[1], Ib[2], Ib[1], Ib[3], Ib[4], Ib[2], Ib[4], Ib[5]};
    double WI[9];  // [w]x Ib
#pragma unroll
    for (int qq = 0; qq < 3; ++qq) {
      WI[qq] = w[1] * Ibf[6 + qq] - w[2] * Ibf[3 + qq];
      WI[3 + qq] = w[2] * Ibf[qq] - w[0] * Ibf[6 + qq];
      WI[6 + qq] = w[0] * Ibf[3 + qq] - w[1] * Ibf[qq];
    }
    const double vh = vl[0] * h[0] + vl[1] * h[1] + vl[2] * h[2];
#pragma unroll
    for (int e = 0; e < 6; ++e) {
      const int r = iu[e][0], qq = iu[e][1];
      // ([w]x Ib - Ib [w]x)_{r,qq} = WI[r][qq] + WI[qq][r]  (Ib symmetric)
      double val = WI[3 * r + qq] + WI[3 * qq + r] - (h[r] * vl[qq] + vl[r] * h[qq]);
      if (r == qq) val += 2.0 * vh;
      Ibd[e] = val;
    }
    // round 1: [0]m [1..3]h [4..9]Ib [10..12]hd [13..18]Ibd -> the inertia sums IC_j, dIC_j
    if (g < KPW) {
      my[0] = m;
#pragma unroll
      for (int r = 0; r < 3; ++r) { my[1 + r] = h[r]; my[10 + r] = hd[r]; }
#pragma unroll
      for (int r = 0; r < 6; ++r) { my[4 + r] = Ib[r]; my[13 + r] = Ibd[r]; }
    }
  }
  wave_sync();
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    if (i >= j) {
      const double* o = &xs[gg][i][0];
      cm = kadd(cm, o[0]);
#pragma unroll
      for (int r = 0; r < 3; ++r) { ch[r] = kadd(ch[r], o[1 + r]); chd[r] = kadd(chd[r], o[10 + r]); }
#pragma unroll
      for (int r = 0; r < 6; ++r) { cI[r] = kadd(cI[r], o[4 + r]); cId[r] = kadd(cId[r], o[13 + r]); }
    }
  }
  wave_sync();  // every lane has read round 1
  // round 2: [0..5]hV [6..11]F0 -> the momentum and force sums HC_j, F^c_j (without the
  // M^-1 (u - tau0) acceleration, which follows in step 4)
  if (g < KPW) {
#pragma unroll
    for (int r = 0; r < 6; ++r) { my[r] = hV[r]; my[6 + r] = F0[r]; }
  }
  wave_sync();
  double HC[6] = {0, 0, 0, 0, 0, 0}, Fc[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    if (i >= j) {
      const double* o = &xs[gg][i][0];
#pragma unroll
      for (int r = 0; r < 6; ++r) { HC[r] = kadd(HC[r], o[r]); Fc[r] = kadd(Fc[r], o[6 + r]); }
    }
  }

  // ---- 3. everything of link j that does not need the joint accelerations: a_j, e_j, z_j,
  // W_j, the acceleration-free parts of Z_j and y_j, and from them the acceleration-free part of
  // column j of dtau/dq and all of column j of dtau/dv.  dIC, HC, F^c, V, A0 die here.
  const double tau0 = dot6(Sj, Fc);
  double aj[6], ej[6], zj[6], Wj[6], Zp[6], yp[6];
  imul(cm, ch, cI, Sj, aj);
  {
    double bj[6], cj[6], t2[6];
    imul(0.0, chd, cId, Sj, bj);
    fcross(Sj, HC, cj);
#pragma unroll
    for (int r = 0; r < 6; ++r) ej[r] = bj[r] - cj[r];
    mcross(Sj, Vj, Wj);
    imul(cm, ch, cI, Wj, t2);
#pragma unroll
    for (int r = 0; r < 6; ++r) zj[r] = bj[r] - 2.0 * t2[r] + cj[r];
  }
  {
    double t1[6], t2[6];
    mcross(Sj, A0j, t1);
    mcross(Wj, Vj, t2);
#pragma unroll
    for (int r = 0; r < 6; ++r) Zp[r] = t1[r] - t2[r];
    double a1[6], a2[6], a3[6], a4[6];
    fcross(Sj, Fc, a1);
    imul(cm, ch, cI, Zp, a2);
    imul(0.0, chd, cId, Wj, a3);
    fcross(Wj, HC, a4);
#pragma unroll
    for (int r = 0; r < 6; ++r) yp[r] = a1[r] - a2[r] - a3[r] - a4[r];
  }
  wave_sync();  // every lane has read round 2
  // round 3: [0..5]a_j [6..11]e_j [12..17]S_j (kept to the end: M row, dA, derivative rows)
  if (g < KPW) {
#pragma unroll
    for (int r = 0; r < 6; ++r) { my[r] = aj[r]; my[6 + r] = ej[r]; my[12 + r] = Sj[r]; }
    st0[gg][j] = tau0;
  }
  wave_sync();
  // M row j: M_jk = a_j . S_k (k <= j)
  if (g < KPW) {
#pragma unroll
    for (int kk = 0; kk < 6; ++kk) {
      if (kk <= j) {
        const double mv = dot6(aj, &xs[gg][kk][12]);
        sM[gg][6 * j + kk] = mv;
        sM[gg][6 * kk + j] = mv;
      }
    }
  }
  // column j: dv (complete) and dq without the terms of dA = sum S_i a_i (added in step 4)
  double dq[6], dv[6];
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    const double* o = &xs[gg][r][0];
    if (r >= j) {
      dq[r] = -(dot6(o, Zp) + dot6(o + 6, Wj));
      dv[r] = dot6(o + 6, Sj) - 2.0 * dot6(o, Wj);
    } else {
      dq[r] = dot6(o + 12, yp);
      dv[r] = dot6(o + 12, zj);
    }
  }
  if (FW && fext && valid) {
    // The formulas above differentiate forces that move with the bodies.  A world-frame wrench
    // does not turn with the arm, so d tau_r / d q_j loses the term S_r . (S_j x* f_w) that a
    // body-fixed one carries (tau_r = S_r . F^c_r; d(X* f)/dq_j = S_j x* (X* f)): add it back
    // with the opposite sign of the subtracted wrench, i.e. +S_r . (S_j x* f_w).
    const double* fe = fext + 6L * b;
    double fw6[6], tS[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) fw6[r] = fe[r];
    fcross(Sj, fw6, tS);
#pragma unroll
    for (int r = 0; r < 6; ++r) dq[r] += dot6(&xs[gg][r][12], tS);
  }
  wave_sync();

#if I7M_LIN_CHOL_LDS
  // ---- 4. M = L L^T, factorised by the knot's six lanes together (lane r holds row r; column c
  // is closed by lane c, then by the lanes r > c, the finished rows passing through sM).  Same
  // operation order as chol6, so the same factor; it overwrites M in sM and stays there for
  // the solves (chol6_solve_lds): no lane holds the whole factor in registers.
  {
    double Lr[6];
#pragma unroll
    for (int cc = 0; cc < 6; ++cc) Lr[cc] = sM[gg][6 * j + cc];
    wave_sync();  // every lane has read its row of M
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      if (j == c) {
        double d = Lr[c];
#pragma unroll
        for (int kk = 0; kk < c; ++kk) d -= Lr[kk] * Lr[kk];
        Lr[c] = rsqrt_nr(d);
        if (g < KPW) {
#pragma unroll
          for (int kk = 0; kk <= c; ++kk) sM[gg][6 * c + kk] = Lr[kk];
        }
      }
      wave_sync();
      if (j > c) {
        const double* Lc = &sM[gg][6 * c];
        double v = Lr[c];
#pragma unroll
        for (int kk = 0; kk < c; ++kk) v -= Lr[kk] * Lc[kk];
        Lr[c] = v * Lc[c];
      }
    }
  }
  const double* Lm = &sM[gg][0];
  auto lsolve = [&](double* x) { chol6_solve_lds(Lm, x); };
#else
  // ---- 4. M = L L^T in every lane's registers (chol6)
  double L[6][6];
#pragma unroll
  for (int r = 0; r < 6; ++r)
#pragma unroll
    for (int cc = 0; cc < 6; ++cc) L[r][cc] = sM[gg][6 * r + cc];
  chol6(L);
  auto lsolve = [&](double* x) { chol6_solve(L, x); };
#endif
  // a = M^-1 (u - tau0) (every lane), dA_j = sum_{i<=j} S_i a_i, g_j = I_j dA_j,
  // Fs_j = sum_{i>=j} g_i; then with sd = S_j x dA_j (Z_j = Zp_j + sd, y_j = yp_j + S_j x* Fs_j
  // - IC_j sd):  dq_r += -a_r . sd (r >= j),  S_r . (S_j x* Fs_j - IC_j sd) (r < j)
  double accj = 0.0, dA[6] = {0, 0, 0, 0, 0, 0};
  {
    double acc[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) acc[r] = (dyn ? X[12 + r] : 0.0) - st0[gg][r];
    lsolve(acc);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      if (i == j) accj = acc[i];
      if (i <= j) {
        const double* Si = &xs[gg][i][12];
#pragma unroll
        for (int r = 0; r < 6; ++r) dA[r] = kmadd(dA[r], Si[r], acc[i]);
      }
    }
  }
  {
    // g_j goes where e_j was (e is not read after step 3)
    double gI[6];
    imul(m, h, Ib, dA, gI);
    if (g < KPW) {
#pragma unroll
      for (int r = 0; r < 6; ++r) my[6 + r] = gI[r];
    }
  }
  wave_sync();
  {
    double Fs[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      if (i >= j) {
#pragma unroll
        for (int r = 0; r < 6; ++r) Fs[r] = kadd(Fs[r], xs[gg][i][6 + r]);
      }
    }
    double sd[6], t1[6], t2[6];
    mcross(Sj, dA, sd);
    imul(cm, ch, cI, sd, t1);
    fcross(Sj, Fs, t2);
#pragma unroll
    for (int r = 0; r < 6; ++r) t2[r] -= t1[r];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const double* o = &xs[gg][r][0];
      dq[r] += (r >= j) ? -dot6(o, sd) : dot6(o + 12, t2);
    }
  }

  // ---- 5. -M^-1 of the columns and outputs, one matrix at a time (the fences make every
  // solve re-read the factor from LDS instead of holding it in registers)
  const double dt = P.dt;
  const double qj = dyn ? X[j] : 0.0, vj = dyn ? X[6 + j] : 0.0, uj = dyn ? X[12 + j] : 0.0;
  double* out = lin + ((long)(dyn ? b : 0) * (P.N - 1) + (dyn ? k : 0)) * LIN_STRIDE;
  double part[6];  // row r of (Aq q + Av v + Bu u), lane j's column term
  wave_sync();
  lsolve(dq);
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    const double aq = -dt * dq[r];
    if (dyn) out[6 * r + j] = aq;
    part[r] = aq * qj;
  }
  wave_sync();
  lsolve(dv);
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    const double av = (r == j ? 1.0 : 0.0) - dt * dv[r];
    if (dyn) out[36 + 6 * r + j] = av;
    part[r] += av * vj;
  }
  wave_sync();
  {
    double em[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) em[r] = (r == j) ? 1.0 : 0.0;
    lsolve(em);
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const double bu = dt * em[r];
      if (dyn && r <= j) {
        out[72 + 6 * r + j] = bu;
        out[72 + 6 * j + r] = bu;
      }
      part[r] += bu * uj;
    }
  }
  if (dyn) out[108 + j] = accj;
  if (qpd) {
    // the knot's QP record for k_riccati_mfma (QPD_* layout): c_v = v + dt a - (Aq q + Av v + Bu u)
    // (src/osqp_solver.py:76-81), the linear cost terms Qm j | dQm v | Rm u (src/osqp_solver.py:
    // 121-135), j, dQm, Rm.  Row r of Aq/Av/Bu is spread over the knot's lanes (lane j owns
    // column j): the partial products go through sM.
    wave_sync();  // every lane has read the factor
    if (g < KPW) {
#pragma unroll
      for (int r = 0; r < 6; ++r) sM[gg][6 * j + r] = part[r];
    }
    wave_sync();
    if (dyn) {
      double sacc = 0.0;
#pragma unroll
      for (int i = 0; i < 6; ++i) sacc += sM[gg][6 * i + j];
      const double qm = (k == P.N - 1) ? P.QN : 1.0;
      const double w = wreg;
      double* o = qpd + ((long)b * (P.N - 1) + k) * QPD_STRIDE;
      o[QPD_CV + j] = (vj + accj * dt) - sacc;
      o[QPD_LX + j] = qm * jte;
      o[QPD_LX + 6 + j] = (P.dQ * w) * vj;
      o[QPD_LU + j] = (P.R * w) * uj;
      o[QPD_J + j] = jte;
      if (j == 0) {
        o[QPD_DQM] = P.dQ * w;
        o[QPD_RM] = P.R * w;
      }
    }
  }
}

// KPW consecutive knots of the flattened (problem, knot) index per 64-lane wave.
template <bool SPEC, bool FW = false>
__global__ void __launch_bounds__(64) I7M_LIN_OCC k_linearize(const DevModel* __restrict__ Mg, SolveParams P,
                                                  const double* __restrict__ xu, const double* __restrict__ goals,
                                                  const double* __restrict__ fext, const int* __restrict__ active,
                                                  double* __restrict__ lin, double* __restrict__ cost,
                                                  double* __restrict__ qpd = nullptr, int* __restrict__ init_active = nullptr,
                                                  ProblemStats* __restrict__ init_stats = nullptr) {
  I7M_TL(1);
  const int l = threadIdx.x;
  const int g = l / 6;
  const int j = l - 6 * g;
  const long kg = (long)blockIdx.x * KPW + g;
  const int b = (int)(kg / P.N);
  const int k = (int)(kg - (long)b * P.N);
  const bool valid = (g < KPW) && (b < P.B) && (!active || active[b]);
  // first SQP iteration: every problem starts active with zeroed stats (knot 0's lanes)
  if (init_active && g < KPW && b < P.B && k == 0) {
    if (j == 0) init_active[b] = 1;
    double* z = reinterpret_cast<double*>(init_stats + b);
#pragma unroll
    for (int r = 0; r < 3; ++r) z[3 * j + r] = 0.0;
  }
  __shared__ LinLds S;
  linearize_body<SPEC, FW>(Mg, P, b, k, valid, l, S, xu, goals, fext, lin, cost, qpd);
}

}  // namespace i7m
