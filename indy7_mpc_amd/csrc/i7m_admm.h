// i7m_admm.h — ADMM mode (I7M_QP_ADMM): the reference's QP solver, OSQP, as a device kernel.
//
// The reference solves every SQP subproblem with one persistent osqp.OSQP() object
// (src/osqp_solver.py:38-40 setup, :137-143 update(Px), update(Ax), update(q, l, u), solve()).
// oracle/osqp_admm.py restates OSQP and is pinned by the notebook's printed closed loop (the
// first 12 goal distances of notebooks/pin_mpc_indy7.ipynb cell 2 to 1e-9); the C++ port
// (oracle/cpp/i7m_cpu.cpp, Solver::admm) runs it in the block form this kernel runs.
//
// One wavefront per problem, the QP in three launches (k_admm_scale, k_admm_factor, k_admm_iter):
//   1. OSQP's Ruiz equilibration (10 passes) of [P A'; A 0] with the previous QP's q (the
//      reference re-scales inside update(Ax), before update(q)), then the new q = c D g and
//      l = u = E l;
//   2. the x-update's matrix M = P + sigma I + A' diag(rho) A, block tridiagonal (18 x 18 blocks
//      per knot (x_k, u_k), 12 x 18 couplings x_{k+1} <- z_k), factored by a block Cholesky
//      whose diagonal factors are kept inverted (Linv_k) and whose couplings C_k = M_{k+1,k}
//      Linv_k' are kept, so every solve is two sweeps of mat-vecs;
//   3. OSQP's iteration from the problem's warm start (x, z, y, rho carried in HBM from call to
//      call like the reference's OSQP object): the solve, relaxation alpha, projection onto
//      [l, u], dual update; every `check` iterations the unscaled residuals and (OSQP 1.x) the
//      duality gap; optional adaptive rho with a refactorisation.
// Every row of A is an equality row (l = u), so rho_vec = 1e3 rho (RHO_EQ_OVER_RHO_INEQ).
// Per-stage blocks live in HBM as one record per stage (Linv packed 171, C 216, scaled J compact
// 120 doubles) and are staged through LDS per stage.
#pragma once

#include "i7m_kernels.h"

namespace i7m {

struct AdmmCfg {
  double rho0, sigma, alpha, eps_abs, eps_rel, adapt_tol;
  int max_iter, check, scaling, gap, adapt_interval, pad;
};

struct AdmmArgs {
  SolveParams P;
  AdmmCfg A;
  const double* lin;   // (B, N-1, 114) k_linearize
  const double* cost;  // (B, N, 10)
  const double* qpd;   // (B, N-1, 32): c_v
  const double* xu;    // (B, T) linearisation point
  const double* xs;    // (B, 12)
  const int* active;
  double* sol;         // (B, T) out: D x
  // OSQP state per problem (scaled x, z, y; the previous QP's q, unscaled; rho)
  double *sx, *sz, *sy, *sq, *srho;
  // scratch per problem
  double *Pq, *Pd, *I, *qs, *ls, *D, *E, *Dt, *Et, *R, *w;
  double* cs;  // (B) OSQP's cost scale c of the current QP (k_admm_prep -> k_admm_iter)
  int* iters;  // (B, I7M_MAX_SQP): OSQP iterations of SQP iteration `sqp_iter`
  int* status;  // (B, I7M_MAX_SQP): 1 OSQP's termination test passed, 0 max_iter reached
  int sqp_iter;
  int b0;      // first problem of this launch (chunked launches: problems [b0, b0 + grid))
  int ablate;  // I7M_DIAG builds only (I7M_ABLATE, timing variants, results invalid); 0 otherwise
};

// HBM layout of the per-stage blocks (what every OSQP iteration streams): the inverted diagonal
// factor packed lower-triangular (171 of 324), the scaled J_k as its q rows' two diagonals
// (E_i D_i for I, E_i dt D_{6+i} for dt I) and its v rows (6 x 18): 120 of 216.  Staged to LDS
// unpacked, so the arithmetic is the dense form's (the dropped entries are exact zeros).
#ifndef I7M_ADMM_WPE
#define I7M_ADMM_WPE 2  // waves per SIMD the adaptive-rho iteration kernel is compiled for
#endif
#ifndef I7M_ADMM_SYNC
#define I7M_ADMM_SYNC 0  // sweep steps' LDS ordering: 0 compiler-only (adm_sweep_sync), 1 wave_sync fences
#endif
#ifndef I7M_ADMM_DOT_CHAINS
#define I7M_ADMM_DOT_CHAINS 2  // fma chains per sweep dot product (adm_dot)
#endif
#ifndef I7M_ADMM_FSTRIDE
#define I7M_ADMM_FSTRIDE 19  // the register factor's LDS row stride for S and C (18: 3-way bank conflicts on row reads)
#endif
#ifndef I7M_ADMM_FACTOR
#define I7M_ADMM_FACTOR 2  // 2: register Cholesky (adm_factor), 1: LDS-staged (adm_factor_lds)
#endif
#ifndef I7M_ADMM_SCALE_WPE
#define I7M_ADMM_SCALE_WPE 3  // (127 VGPRs, 12 KB LDS: 3 waves per SIMD; 2.11 -> 2.08 ms prep)
#endif
#ifndef I7M_ADMM_FACTOR_WPE
#define I7M_ADMM_FACTOR_WPE 2
#endif
#ifndef I7M_ADMM_ITER_WPE
#define I7M_ADMM_ITER_WPE 2  // ... and k_admm_iter without adaptive rho (at 3: 78 spilled VGPRs, 30% slower)
#endif
constexpr int ADM_LP = 171, ADM_JC = 120;
// One record per stage, N per problem (problem b's at R + b N ADM_REC): [Linv_k packed lower
// (171) | compact J_k (120) | pad (1)] = 292 doubles, 16-byte aligned.  k_admm_iter streams it
// twice per OSQP iteration (forward and backward sweep); the coupling C_k = M_{k+1,k} Linv_k' of
// the factor is never stored: the sweeps apply it as re I_{k+1} J_k and the triangular pair.
constexpr int ADM_REC = 292, REC_J = ADM_LP;
__device__ __forceinline__ int adm_tri(int i, int j) { return i * (i + 1) / 2 + j; }
// dense 12 x 18 J_k into LDS from its compact form
__device__ __forceinline__ void adm_stage_J(double* sJ, const double* Jc, int l) {
  for (int e = l; e < 216; e += 64) {
    const int i = e / 18, j = e - 18 * i;
    double v;
    if (i < 6) v = j == i ? Jc[i] : (j == 6 + i ? Jc[6 + i] : 0.0);
    else v = Jc[12 + 18 * (i - 6) + j];
    sJ[e] = v;
  }
}

// init + sum_i a[sa i] b[i] over n LDS operands (the sweeps' dot products): every operand read is
// issued before the fma chains, so they pay one LDS latency instead of one per term; the terms are
// summed in i order (I7M_ADMM_DOT_CHAINS 1) or as two interleaved chains (2) (the dot
// products of the sweeps run over fixed lengths; Linv's upper triangle and the padding of the
// last knot's 12 x 12 blocks are exact zeros, which add nothing)
template <int n>
__device__ __forceinline__ double adm_dot(double init, const double* a, int sa, const double* b) {
  double av[n], bv[n];
#pragma unroll
  for (int i = 0; i < n; ++i) {
    av[i] = a[sa * i];
    bv[i] = b[i];
  }
  if constexpr (I7M_ADMM_DOT_CHAINS == 2) {
    // two interleaved fma chains (even / odd terms) summed at the end: half the dependent latency
    double a0 = init, a1 = 0.0;
#pragma unroll
    for (int i = 0; i < n; i += 2) {
      a0 += av[i] * bv[i];
      if (i + 1 < n) a1 += av[i + 1] * bv[i + 1];
    }
    return a0 + a1;
  } else {
    double acc = init;
#pragma unroll
    for (int i = 0; i < n; ++i) acc += av[i] * bv[i];
    return acc;
  }
}

// ... with both operands strided
template <int n>
__device__ __forceinline__ double adm_dot2(double init, const double* a, int sa, const double* b, int sb) {
  double av[n], bv[n];
#pragma unroll
  for (int i = 0; i < n; ++i) {
    av[i] = a[sa * i];
    bv[i] = b[sb * i];
  }
  double acc = init;
#pragma unroll
  for (int i = 0; i < n; ++i) acc += av[i] * bv[i];
  return acc;
}

// entry (i, j) of the compact J_k in HBM
__device__ __forceinline__ double adm_jc(const double* Jc, int i, int j) {
  if (i < 6) return j == i ? Jc[i] : (j == 6 + i ? Jc[6 + i] : 0.0);
  return Jc[12 + 18 * (i - 6) + j];
}

// max / sum over groups of W lanes (W = 64: the wave; 16: a DPP row)
template <int W>
__device__ __forceinline__ double adm_max(double v) {
#pragma unroll
  for (int off = W / 2; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off, W));
  return v;
}
template <int W>
__device__ __forceinline__ double adm_sum(double v) {
#pragma unroll
  for (int off = W / 2; off >= 1; off >>= 1) v += __shfl_xor(v, off, W);
  return v;
}
__device__ __forceinline__ double adm_wave_max(double v) { return adm_max<64>(v); }
__device__ __forceinline__ double adm_wave_sum(double v) { return adm_sum<64>(v); }
__device__ __forceinline__ double adm_limit(double v) { return v < 1e-4 ? 1.0 : (v > 1e4 ? 1e4 : v); }

// unscaled J_k = [[I, dt I, 0], [Aq, Av, Bu]] (rows of A's block k+1 on z_k; src/osqp_solver.py:
// 42-43, 70-81), from the linearisation record
__device__ __forceinline__ double adm_jk(const double* L, double dt, int i, int j) {
  if (i < 6) return j == i ? 1.0 : (j == 6 + i ? dt : 0.0);
  const int r = i - 6;
  return j < 6 ? L[6 * r + j] : (j < 12 ? L[36 + 6 * r + j - 6] : L[72 + 6 * r + j - 12]);
}

// coalesced copy of n doubles global -> LDS by the wave
__device__ __forceinline__ void adm_stage(double* dst, const double* src, int n, int l) {
  for (int e = l; e < n; e += 64) dst[e] = src[e];
}

// Ordering of one sweep step's LDS traffic between the lanes of its wave.  A wavefront's LDS
// instructions execute in order, so a lane reads what another lane of the same wave stored by an
// earlier instruction: only the compiler must keep the order (I7M_ADMM_SYNC 0, an empty asm with a
// memory clobber).  1: the wave_sync fence, which also waits for every outstanding LDS operation.
__device__ __forceinline__ void adm_sweep_sync() {
#if I7M_ADMM_SYNC
  wave_sync();
#else
  __asm__ volatile("" ::: "memory");
#endif
}

// OSQP's check_termination on the unscaled residuals (+ the duality gap) and, for adapt_rho,
// the scaled residual ratios; x, z, y scaled.  Returns solved; rho_est gets the estimate.  W lanes
// share one problem (lane l of W): 64 (one problem per wave) or 16 (k_admm_iter: a 16-lane row).
template <int W>
__device__ bool adm_check(const AdmmArgs& a, int N, int T, int m, double c, double rho, const double* x,
                          const double* z, const double* y, const double* qs, const double* ls, const double* D,
                          const double* E, const double* Jb, const double* Ib, const double* Pq, const double* Pd,
                          double* rho_est, int l) {
  double pr = 0.0, zn = 0.0, an = 0.0, pri = 0.0, pn = 0.0;
  double dr = 0.0, qn = 0.0, atn = 0.0, pxn = 0.0, dua = 0.0, dn = 0.0, xPx = 0.0, qx = 0.0, sc = 0.0;
  // rows: block 0 = I x_0, block k+1 = J_k z_k + I x_{k+1}
  for (int r = l; r < m; r += W) {
    const int k = r / 12, i = r - 12 * k;
    double ax;
    if (k == 0) {
      ax = Ib[r] * x[i];
    } else {
      const double* G = Jb + ADM_REC * (k - 1);
      const double* xk = x + 18 * (k - 1);
      double acc = 0.0;
      for (int j = 0; j < 18; ++j) acc += adm_jc(G, i, j) * xk[j];
      ax = acc + Ib[r] * x[18 * k + i];
    }
    const double ei = 1.0 / E[r];
    pr = fmax(pr, fabs(ei * (ax - z[r])));
    zn = fmax(zn, fabs(ei * z[r]));
    an = fmax(an, fabs(ei * ax));
    pri = fmax(pri, fabs(ax - z[r]));
    pn = fmax(pn, fmax(fabs(z[r]), fabs(ax)));
    sc += ls[r] * fmax(y[r], 0.0) + ls[r] * fmin(y[r], 0.0);
  }
  for (int e = l; e < T; e += W) {
    const int k = e / 18, j = e - 18 * k;
    double px;
    if (j < 6) {
      double acc = 0.0;
      for (int jj = 0; jj < 6; ++jj) acc += Pq[36 * k + 6 * j + jj] * x[18 * k + jj];
      px = acc;
    } else {
      px = Pd[e] * x[e];
    }
    double aty = j < 12 ? Ib[12 * k + j] * y[12 * k + j] : 0.0;
    if (k < N - 1) {
      const double* G = Jb + ADM_REC * k;
      for (int i = 0; i < 12; ++i) aty += adm_jc(G, i, j) * y[12 * (k + 1) + i];
    }
    const double di = 1.0 / D[e];
    dr = fmax(dr, fabs(di * ((qs[e] + px) + aty)));
    qn = fmax(qn, fabs(di * qs[e]));
    atn = fmax(atn, fabs(di * aty));
    pxn = fmax(pxn, fabs(di * px));
    dua = fmax(dua, fabs(qs[e] + px + aty));
    dn = fmax(dn, fmax(fabs(qs[e]), fmax(fabs(aty), fabs(px))));
    xPx += x[e] * px;
    qx += qs[e] * x[e];
  }
  pr = adm_max<W>(pr); zn = adm_max<W>(zn); an = adm_max<W>(an); pri = adm_max<W>(pri); pn = adm_max<W>(pn);
  dr = adm_max<W>(dr); qn = adm_max<W>(qn); atn = adm_max<W>(atn); pxn = adm_max<W>(pxn);
  dua = adm_max<W>(dua); dn = adm_max<W>(dn);
  xPx = adm_sum<W>(xPx); qx = adm_sum<W>(qx); sc = adm_sum<W>(sc);
  const double cinv = 1.0 / c;
  // OSQP compute_rho_estimate (scaled residuals)
  {
    const double p = pri / (pn + 1e-30), d = dua / (dn + 1e-30);
    double rn = rho * sqrt(p / (d + 1e-30));
    *rho_est = fmin(fmax(rn, 1e-6), 1e6);
  }
  dr *= cinv;
  if (!(pr < a.A.eps_abs + a.A.eps_rel * fmax(zn, an))) return false;
  if (!(dr < a.A.eps_abs + a.A.eps_rel * cinv * fmax(qn, fmax(atn, pxn)))) return false;
  if (a.A.gap) {
    xPx *= cinv; qx *= cinv; sc *= cinv;
    const double gp = xPx + qx + sc;
    if (!(fabs(gp) < a.A.eps_abs + a.A.eps_rel * fmax(fabs(xPx), fmax(fabs(qx), fabs(sc))))) return false;
  }
  return true;
}

// OSQP's scaling of the QP (src/osqp_solver.py:137-143: update(Px), update(Ax) rescale with the
// previous q; then update(q, l, u)), as oracle/cpp/i7m_cpu.cpp Solver::admm_setup: 10 Ruiz passes
// on [P A'; A 0] and the cost normalisation, then the scaled P blocks, J_k, the -I entries, q and l
// into HBM; returns the cost scale c.  D and E live in LDS during the passes; a lane owns columns
// e = l + 64 t (t < CT) and rows r = l + 64 t (t < 2 CT / 3), whose scale factors and q entries
// stay in its registers.  Every column's and row's inf-norm reads its entries unconditionally at
// clamped indices and selects (a P column: 6 entries of the quadratic block or the diagonal; an A
// column: the -I entry, J's identity / dt entry and 6 linearisation entries; an A row: its -I
// entry and 18 J entries), so the loads of all of a lane's columns issue together.  The products
// are the port's (|a_ij| D_j E_i in its order; max is exact), so D, E and c are the one-kernel
// version's to the bit, the cost sum's wave reduction aside.  Its LDS orderings are fences
// (wave_sync_fence): as compiler barriers (wave_sync) the kernel ran 0.59 -> 2.42 ms.
__device__ __forceinline__ double adm_pq(const double* w, int i, int j) { return w[6] * (w[i] * w[j]); }
template <int CT>
__device__ __forceinline__ double adm_scale(const AdmmArgs& a, int b, int N, int T, int m, const double* LIN,
                                            const double* CO, const double* QD, const double* X, double* qold,
                                            double* Pq, double* Pd, double* Jb, double* Ib, double* qs, double* ls,
                                            double* D, double* E, double* sD, double* sE, double* sDt, int l) {
  constexpr int RT = 2 * CT / 3;
  const double dt = a.P.dt;
  double qv[CT], etv[RT];
#pragma unroll
  for (int t = 0; t < CT; ++t) {
    const int e = l + 64 * t;
    qv[t] = 0.0;
    if (e < T) {
      sD[e] = 1.0;
      qv[t] = qold[e];
    }
  }
#pragma unroll
  for (int t = 0; t < RT; ++t)
    if (l + 64 * t < m) sE[l + 64 * t] = 1.0;
  wave_sync_fence();
  double c = 1.0;
  // the P part of column e's inf-norm (knot k, index j in the knot): max_i |P_ij| D_i D_j c
  auto pcol = [&](const double* Cp, int k, int j, double dj) {
    const double* w = Cp + COST_STRIDE * k;
    const int jq = j < 6 ? j : 0;
    double mq = 0.0;
#pragma unroll
    for (int i = 0; i < 6; ++i) mq = fmax(mq, fabs(adm_pq(w, i, jq)) * (sD[18 * k + i] * dj) * c);
    const double pd = j < 12 ? w[7] : w[8];
    return j < 6 ? mq : fabs(pd) * (dj * dj) * c;
  };
  for (int pass = 0; pass < a.A.scaling; ++pass) {
    // every pass recomputes its indices (hoisted out of the pass loop they would take ~300 VGPRs)
    const double* Lp = LIN;
    const double* Cp = CO;
    int lp = l;
    asm volatile("" : "+v"(lp));
#pragma unroll 3
    for (int t = 0; t < CT; ++t) {
      const int e = min(lp + 64 * t, T - 1), k = e / 18, j = e - 18 * k;
      const double dj = sD[e];
      double mx = pcol(Cp, k, j, dj);
      const double ei = sE[12 * k + (j < 12 ? j : 0)] * dj;
      if (j < 12) mx = fmax(mx, ei);
      // J_k's column j (rows of block k + 1; the last knot has none): the identity / dt entry, 6
      // linearisation entries
      const int kk = k < N - 1 ? k : N - 2;
      const double* L = Lp + LIN_STRIDE * kk;
      const double* Eb = sE + 12 * (kk + 1);
      const int jb = j < 6 ? j : (j < 12 ? 30 + j : 60 + j);
      const double eid = Eb[j < 6 ? j : (j < 12 ? j - 6 : 0)] * (j < 6 ? 1.0 : dt) * dj;
      double mj = j < 12 ? eid : 0.0;
#pragma unroll
      for (int r = 0; r < 6; ++r) mj = fmax(mj, Eb[6 + r] * fabs(L[jb + 6 * r]) * dj);
      if (k < N - 1) mx = fmax(mx, mj);
      sDt[lp + 64 * t] = 1.0 / sqrt(adm_limit(mx));
    }
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      const int r = min(lp + 64 * t, m - 1), blk = r / 12, i = r - 12 * blk;
      const double er = sE[r];
      double mx = er * sD[18 * blk + i];
      // row i of J_{blk-1} (block 0's rows are -I on x_0 alone)
      const int kk = blk > 0 ? blk - 1 : 0;
      const double* L = Lp + LIN_STRIDE * kk;
      const double* Db = sD + 18 * kk;
      // rows 0-5: the identity and dt entries; rows 6-11: 18 linearisation entries
      const int i6 = i < 6 ? i : i - 6;
      const double mi = fmax(er * 1.0 * Db[i6], er * dt * Db[6 + i6]);
      double ml = 0.0;
#pragma unroll
      for (int j = 0; j < 18; ++j) {
        const int jb = j < 6 ? j : (j < 12 ? 30 + j : 60 + j);
        ml = fmax(ml, er * fabs(L[jb + 6 * i6]) * Db[j]);
      }
      const double mj = i < 6 ? mi : ml;
      if (blk > 0) mx = fmax(mx, mj);
      etv[t] = 1.0 / sqrt(adm_limit(mx));
    }
    wave_sync_fence();
#pragma unroll
    for (int t = 0; t < CT; ++t) {
      const int e = lp + 64 * t;
      const double dtt = sDt[e];
      if (e < T) sD[e] = sD[e] * dtt;
      qv[t] = dtt * qv[t];
    }
#pragma unroll
    for (int t = 0; t < RT; ++t)
      if (lp + 64 * t < m) sE[lp + 64 * t] = sE[lp + 64 * t] * etv[t];
    wave_sync_fence();
    // cost normalisation: mean column norm of the scaled P, |q|
    double sm = 0.0, qm = 0.0;
#pragma unroll
    for (int t = 0; t < CT; ++t) {
      const int e = lp + 64 * t, ec = min(e, T - 1), k = ec / 18, j = ec - 18 * k;
      const double mx = pcol(Cp, k, j, sD[ec]);
      if (e < T) {
        sm += mx;
        qm = fmax(qm, fabs(qv[t]));
      }
    }
    sm = adm_wave_sum(sm);
    qm = adm_limit(adm_wave_max(qm));
    const double ct = 1.0 / adm_limit(fmax(sm / T, qm));
#pragma unroll
    for (int t = 0; t < CT; ++t) qv[t] = qv[t] * ct;
    c = c * ct;
  }
  // scaled data: P <- c D P D, J <- E J D, I <- -E D, q <- c D g (update(q)), l <- E l
  for (int e = l; e < T; e += 64) D[e] = sD[e];
  for (int r = l; r < m; r += 64) E[r] = sE[r];
#pragma unroll 4
  for (int x = l; x < 36 * N; x += 64) {
    const int k = x / 36, q = x - 36 * k, i = q / 6, j = q - 6 * i;
    Pq[x] = adm_pq(CO + COST_STRIDE * k, i, j) * (sD[18 * k + i] * sD[18 * k + j]) * c;
  }
#pragma unroll 4
  for (int x = l; x < 120 * (N - 1); x += 64) {
    const int k = x / 120, e = x - 120 * k;
    int i, j;
    if (e < 6) { i = e; j = e; }
    else if (e < 12) { i = e - 6; j = e; }
    else { i = 6 + (e - 12) / 18; j = (e - 12) % 18; }
    Jb[ADM_REC * k + e] = sE[12 * (k + 1) + i] * adm_jk(LIN + LIN_STRIDE * k, dt, i, j) * sD[18 * k + j];
  }
  for (int r = l; r < m; r += 64) {
    const int k = r / 12, i = r - 12 * k;
    Ib[r] = -sE[r] * sD[18 * k + i];
    double lv;
    if (k == 0) lv = -a.xs[12 * (long)b + i];
    else lv = i < 6 ? 0.0 : -QD[QPD_STRIDE * (k - 1) + QPD_CV + i - 6];
    ls[r] = sE[r] * lv;
  }
  for (int e = l; e < T; e += 64) {
    const int k = e / 18, j = e - 18 * k;
    const double* w = CO + COST_STRIDE * k;
    const double dd = sD[e];
    Pd[e] = j < 6 ? 0.0 : (j < 12 ? w[7] : w[8]) * (dd * dd) * c;
    const double g = j < 6 ? w[6] * w[j] : (j < 12 ? w[7] * X[e] : w[8] * X[e]);
    qold[e] = g;
    qs[e] = c * (dd * g);
  }
  wave_sync_all();
  return c;
}

// M = P + sigma I + A' rho A, block Cholesky with inverted diagonal factors (as Solver::
// admm_factor of the port): Linv_k (packed) into record k, C_k into record k+1.  Per stage: the
// block S_k in LDS (all lanes, every dot product's operands loaded before its fma chain), its
// right-looking Cholesky with row i in lane i's registers (the pivot by readlane, the column
// through LDS: one round trip per pivot), Linv_k by forward substitution with column j in lane j's
// registers, then C_k.  The last knot's 12 x 12 block is factored padded with an identity, whose
// entries are stored as the zeros the port has there.  Same operations in the port's order (the
// zeros the padding and the triangles add are exact).
__device__ __forceinline__ double adm_readlane(double v, int lane) {
  const long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)u, lane), hi = __builtin_amdgcn_readlane((int)(u >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ void adm_factor(const AdmmArgs& a, int N, double rho, const double* Pq, const double* Pd, const double* Ib,
                           double* Rb, double* sS, double* sJ, double* sL, double* sCp, int l0) {
  const double re = 1e3 * rho, sigma = a.A.sigma;
  const int T = 18 * N - 6;
  constexpr int FS = I7M_ADMM_FSTRIDE;  // row stride of S and C_{k-1} in LDS
  double* sCol = sL + 324;  // (the sweeps' C slot, free while factoring)
  for (int k = 0; k < N; ++k) {
    const int nk = k < N - 1 ? 18 : 12;
    // every stage recomputes the lane's indices (hoisted out of the stage loop they would take
    // more registers than the kernel has)
    int l = l0;
    asm volatile("" : "+v"(l));
    const int lr = l < 18 ? l : 17;  // lanes 18-63 shadow lane 17 (never read back)
    if (k < N - 1) adm_stage_J(sJ, Rb + ADM_REC * k + REC_J, l);
    wave_sync();
#pragma unroll
    for (int t = 0; t < 6; ++t) {
      const int e = l + 64 * t;
      if (e < 324) {
        const int i = e / 18, j = e - 18 * i, ic = i < 12 ? i : 11, jc = j < 12 ? j : 11;
        const double pq = Pq[36 * k + 6 * (i < 6 ? i : 0) + (j < 6 ? j : 0)];
        const double pd = Pd[min(18 * k + i, T - 1)];
        const double ib = Ib[12 * k + ic];
        const double dj = adm_dot2<12>(0.0, sJ + i, 18, sJ + j, 18);
        const double dc = adm_dot2<18>(0.0, sCp + FS * ic, 1, sCp + FS * jc, 1);
        double v = i < 6 && j < 6 ? pq : (i == j && i >= 6 ? pd : 0.0);
        if (i == j) v += sigma;
        if (i == j && i < 12) v += re * (ib * ib);
        if (k < N - 1) v += re * dj;
        if (k > 0 && i < 12 && j < 12) v -= dc;
        if (i >= nk || j >= nk) v = i == j ? 1.0 : 0.0;
        sS[FS * i + j] = v;
      }
    }
    wave_sync();
    double r[18];
#pragma unroll
    for (int j = 0; j < 18; ++j) r[j] = sS[FS * lr + j];
#pragma unroll
    for (int p = 0; p < 18; ++p) {
      const double d = sqrt(adm_readlane(r[p], p));
      const double id = 1.0 / d;
      r[p] = l == p ? d : (l > p ? r[p] * id : r[p]);
      if (p < 17) {
        // column p of L to the wave through LDS (double-buffered: no wait for the last reads)
        double* col = sCol + 32 * (p & 1);
        if (l < 18) col[l] = r[p];
        wave_sync();
#pragma unroll
        for (int j = p + 1; j < 18; ++j) r[j] = r[j] - r[p] * col[j];
      }
    }
    wave_sync();  // every lane has read S before L overwrites it
    if (l < 18) {
#pragma unroll
      for (int j = 0; j < 18; ++j) sS[FS * l + j] = r[j];
    }
    wave_sync();
    double x[18];
#pragma unroll
    for (int i = 0; i < 18; ++i) {
      // row i of L is read once x_{i-2} exists (two rows of loads in flight, not all 171)
      int o = FS * i;
      if (i >= 2) asm volatile("" : "+v"(o) : "v"(x[i - 2]));
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < i; ++q) acc += sS[o + q] * x[q];
      x[i] = ((i == lr ? 1.0 : 0.0) - acc) / sS[o + i];
    }
    if (l < 18) {
#pragma unroll
      for (int i = 0; i < 18; ++i) {
        const double v = i < nk && l < nk ? x[i] : 0.0;
        sL[18 * i + l] = v;
        if (i >= l) Rb[ADM_REC * k + adm_tri(i, l)] = v;
      }
    }
    wave_sync();
    if (k < N - 1) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int e = l + 64 * t;
        if (e < 216) {
          const int i = e / 18, j = e - 18 * i;
          const double acc = adm_dot2<18>(0.0, sJ + 18 * i, 1, sL + 18 * j, 1);
          const double cv = re * Ib[12 * (k + 1) + i] * acc;
          sCp[FS * i + j] = cv;
        }
      }
    }
    wave_sync_all();
  }
}

// The factor with every step's operands through LDS (the kernel before the register Cholesky;
// I7M_ADMM_FACTOR 1, A/B builds)
__device__ void adm_factor_lds(const AdmmArgs& a, int N, double rho, const double* Pq, const double* Pd, const double* Ib,
                           double* Rb, double* sS, double* sJ, double* sL, double* sCp,
                           int l) {
  const double re = 1e3 * rho, sigma = a.A.sigma;
  for (int k = 0; k < N; ++k) {
    const int nk = k < N - 1 ? 18 : 12;
    if (k < N - 1) adm_stage_J(sJ, Rb + ADM_REC * k + REC_J, l);
    wave_sync();
    for (int e = l; e < 324; e += 64) {
      const int i = e / 18, j = e - 18 * i;
      double v = 0.0;
      if (i < nk && j < nk) {
        if (i < 6 && j < 6) v = Pq[36 * k + 6 * i + j];
        else if (i == j && i >= 6) v = Pd[18 * k + i];
        if (i == j) v += sigma;
        if (i == j && i < 12) v += re * (Ib[12 * k + i] * Ib[12 * k + i]);
        if (k < N - 1) {
          double acc = 0.0;
          for (int r = 0; r < 12; ++r) acc += sJ[18 * r + i] * sJ[18 * r + j];
          v += re * acc;
        }
        if (k > 0 && i < 12 && j < 12) {
          double acc = 0.0;
          for (int q = 0; q < 18; ++q) acc += sCp[18 * i + q] * sCp[18 * j + q];
          v -= acc;
        }
      }
      sS[e] = v;
    }
    wave_sync();
    // right-looking Cholesky
    for (int p = 0; p < nk; ++p) {
      const double d = sqrt(sS[18 * p + p]);
      const double id = 1.0 / d;
      wave_sync();
      if (l == 0) sS[18 * p + p] = d;
      if (l > p && l < nk) sS[18 * l + p] = sS[18 * l + p] * id;
      wave_sync();
      for (int e = l; e < 324; e += 64) {
        const int i = e / 18, j = e - 18 * i;
        if (j > p && i >= j && i < nk) sS[e] = sS[e] - sS[18 * i + p] * sS[18 * j + p];
      }
      wave_sync();
    }
    // inverse of the lower factor, one column per lane
    for (int e = l; e < 324; e += 64) sL[e] = 0.0;
    wave_sync();
    if (l < nk) {
      const int j = l;
      sL[18 * j + j] = 1.0 / sS[18 * j + j];
      for (int i = j + 1; i < nk; ++i) {
        double acc = 0.0;
        for (int q = j; q < i; ++q) acc += sS[18 * i + q] * sL[18 * q + j];
        sL[18 * i + j] = -acc / sS[18 * i + i];
      }
    }
    wave_sync();
    for (int e = l; e < 324; e += 64) {
      const int i = e / 18, j = e - 18 * i;
      if (j <= i) Rb[ADM_REC * k + adm_tri(i, j)] = sL[e];
    }
    if (k < N - 1) {
      for (int e = l; e < 216; e += 64) {
        const int i = e / 18, j = e - 18 * i;
        double acc = 0.0;
        for (int q = 0; q <= j; ++q) acc += sJ[18 * i + q] * sL[18 * j + q];
        const double cv = re * Ib[12 * (k + 1) + i] * acc;
        sCp[e] = cv;
      }
    }
    wave_sync_all();
  }
}

// k_admm_scale (PH 1: scaling, the new q and l; c to a.cs) and k_admm_factor (PH 8: the block
// Cholesky), one problem per wave; each compiled for its own registers and LDS.
template <int PH, int CT>
__device__ __forceinline__ void admm_body(const AdmmArgs& a) {
  const int b = a.b0 + blockIdx.x;
  const SolveParams& P = a.P;
  if (b >= P.B || (a.active && !a.active[b])) return;
  const int l = threadIdx.x, N = P.N, T = P.T, m = 12 * N;
  constexpr bool FAC = (PH & 8) != 0;
  // (k_admm_scale: sB holds the column scale factors of a Ruiz pass)
  __shared__ double sB[(PH & 1) ? 64 * CT : 756], sS[FAC ? 18 * I7M_ADMM_FSTRIDE : 1], sCp[FAC ? 12 * I7M_ADMM_FSTRIDE : 1];
  __shared__ double sD[(PH & 1) ? 64 * CT : 1], sE[(PH & 1) ? 64 * (2 * CT / 3) : 1];
  double* sL = sB;
  double* sJ = sB + 540;
  const double* LIN = a.lin + (long)b * (N - 1) * LIN_STRIDE;
  const double* CO = a.cost + (long)b * N * COST_STRIDE;
  const double* QD = a.qpd + (long)b * (N - 1) * QPD_STRIDE;
  const double* X = a.xu + (long)b * T;
  double* qold = a.sq + (long)b * T;
  double* Pq = a.Pq + (long)b * N * 36;
  double* Pd = a.Pd + (long)b * T;
  double* Rb = a.R + (long)b * N * ADM_REC;
  double* Jb = Rb + REC_J;  // J_k at Jb + ADM_REC k
  double* Ib = a.I + (long)b * m;
  double* qs = a.qs + (long)b * T;
  double* ls = a.ls + (long)b * m;
  double* D = a.D + (long)b * T;
  double* E = a.E + (long)b * m;
  if constexpr (PH & 1) {
    const double c = adm_scale<CT>(a, b, N, T, m, LIN, CO, QD, X, qold, Pq, Pd, Jb, Ib, qs, ls, D, E, sD, sE, sB, l);
    if (l == 0) a.cs[b] = c;
  }
  if constexpr (PH & 8) {
#if I7M_ADMM_FACTOR == 1
    adm_factor_lds(a, N, a.srho[b], Pq, Pd, Ib, Rb, sS, sJ, sL, sCp, l);
#else
    adm_factor(a, N, a.srho[b], Pq, Pd, Ib, Rb, sS, sJ, sL, sCp, l);
#endif
  }
}

// ---- OSQP's iterations (k_admm_iter): four problems per wave, one per 16-lane DPP row --------
// Lane l works on problem b0 + 4 blockIdx.x + (l >> 4), row c = l & 15 of its 18-dim stage vectors:
// a stage vector v is (v_lo in lane c = v_c, c < 16; v16, v17 held by every lane of the row).  The
// sweeps are the block LDL' of M with S_k^-1 = Linv_k' Linv_k (oracle/cpp/i7m_cpu.cpp admm_solve):
//   forward   g_k = rhs_k - [re I_k (J_{k-1} h_{k-1}); 0],  h_k = Linv_k' (Linv_k g_k)
//   backward  xt_k = h_k - Linv_k' (Linv_k (J_k' (re I_{k+1} xt_{k+1}[:12])))
// then z~ = J_k xt_k + I_{k+1} xt_{k+1} for block k+1's rows, OSQP's relaxation, projection and dual
// update.  Every mat-vec is a chain of fma's whose broadcast operand comes from the row's own lanes
// by DPP (v_mov_b64_dpp row_newbcast: no LDS round trip on the sweep's chain); the matrix operand
// is read from the stage's LDS image.  Each step's stage record (Linv packed | compact J: 292
// doubles per problem, 10 dwordx4 per lane) is loaded two steps ahead into registers, then
// scattered into a dense LDS image (Linv 18 x 18, J 12 x 18, zeros fixed) at the step's start; the
// step's vectors ride in the same ring.  Problems stop at their own termination test; a finished
// row keeps shadowing the others' loads (its addresses are a running row's) and stores nothing.
constexpr int A4_PS = 541;  // doubles of one problem's LDS image (Linv 324 | J 216 | zero); odd:
                            // two problems of a lane half read disjoint banks
constexpr int A4_LJ = 324;
template <int n>
__device__ __forceinline__ double a4_bc(double v) {  // lane n of the 16-lane row, to every lane of it
  return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + n, 0xf, 0xf, false);
}
__device__ __forceinline__ double a4_dpp32(double v, int ctrl_is_shl) {
  const long long u = __double_as_longlong(v);
  int lo = (int)u, hi = (int)(u >> 32);
  if (ctrl_is_shl) {
    lo = __builtin_amdgcn_update_dpp(lo, lo, 0x106, 0xf, 0xf, false);
    hi = __builtin_amdgcn_update_dpp(hi, hi, 0x106, 0xf, 0xf, false);
  } else {
    lo = __builtin_amdgcn_update_dpp(lo, lo, 0x116, 0xf, 0xf, false);
    hi = __builtin_amdgcn_update_dpp(hi, hi, 0x116, 0xf, 0xf, false);
  }
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// lane c gets lane c - 6's value (c >= 6 of the row), keeps its own below / lane c + 6's (c < 10)
__device__ __forceinline__ double a4_shr6(double v) { return a4_dpp32(v, 0); }
__device__ __forceinline__ double a4_shl6(double v) { return a4_dpp32(v, 1); }
template <int I, int N, class F>
__device__ __forceinline__ void a4_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    a4_for<I + 1, N>(f);
  }
}
struct A4Vec {
  double lo, h16, h17;
};
// acc += (lane n of the row's v) * coef: v_fmac_f64_dpp with the broadcast fused (DP DPP takes only
// row_newbcast).  Four fma's per statement into four accumulators; the statement opens with the
// two wait states a DPP read of a VGPR a VALU just wrote needs (the compiler pads no asm).
template <int n>
__device__ __forceinline__ void a4_fmac4(double& a0, double& a1, double& a2, double& a3, double v, double c0, double c1,
                                         double c2, double c3) {
  asm volatile(
      "s_nop 1\n\t"
      "v_fmac_f64_dpp %0, %4, %5 row_newbcast:%9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, %4, %6 row_newbcast:%10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %2, %4, %7 row_newbcast:%11 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %3, %4, %8 row_newbcast:%12 row_mask:0xf bank_mask:0xf"
      : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)
      : "v"(v), "v"(c0), "v"(c1), "v"(c2), "v"(c3), "i"(n), "i"(n + 1), "i"(n + 2), "i"(n + 3));
}
template <int n>
__device__ __forceinline__ void a4_fmac2(double& a0, double& a1, double v, double c0, double c1) {
  asm volatile(
      "s_nop 1\n\t"
      "v_fmac_f64_dpp %0, %2, %3 row_newbcast:%5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, %2, %4 row_newbcast:%6 row_mask:0xf bank_mask:0xf"
      : "+v"(a0), "+v"(a1)
      : "v"(v), "v"(c0), "v"(c1), "i"(n), "i"(n + 1));
}
// sum_{l < 16} coef[l] * v_l as four interleaved chains (l mod 4), combined (a0 + a1) + (a2 + a3):
// the device's and the port's order (oracle/cpp/i7m_cpu.cpp dot16)
__device__ __forceinline__ double a4_dot16(double v, const double* cf) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  a4_fmac4<0>(a0, a1, a2, a3, v, cf[0], cf[1], cf[2], cf[3]);
  a4_fmac4<4>(a0, a1, a2, a3, v, cf[4], cf[5], cf[6], cf[7]);
  a4_fmac4<8>(a0, a1, a2, a3, v, cf[8], cf[9], cf[10], cf[11]);
  a4_fmac4<12>(a0, a1, a2, a3, v, cf[12], cf[13], cf[14], cf[15]);
  return __dadd_rn(__dadd_rn(a0, a1), __dadd_rn(a2, a3));
}
// sum_{r = 6..11} coef[r - 6] * u_r as two chains (r even / odd), combined
__device__ __forceinline__ double a4_dot6(double u, const double* cf) {
  double a0 = 0.0, a1 = 0.0;
  a4_fmac2<6>(a0, a1, u, cf[0], cf[1]);
  a4_fmac2<8>(a0, a1, u, cf[2], cf[3]);
  a4_fmac2<10>(a0, a1, u, cf[4], cf[5]);
  return __dadd_rn(a0, a1);
}
// One stage image's coefficients of a lane, read from LDS at the step's start (all reads issued
// before the first fma: one LDS latency per step, not one per chain)
struct A4Coef {
  double L[16], L16[17], L17[18];   // Linv row c, rows 16 and 17 (lmul)
  double Lt[16], Lt16c, Lt17c;      // Linv column c (l < 16), L[16][c], L[17][c] (ltmul)
  double l1616, l1716, l1717;       // the (16, 17) block (ltmul)
  double Jt[6], J16[6], J17[6], Jd; // J column c (rows 6..11), columns 16, 17 (rows 6..11), J[c % 6][c] (jtmul)
  double Jr[18], Jq0, Jq1;          // J row c (c in 6..11; row 11 above), J[q][q], J[q][6 + q] (jmul, q = c < 6 ? c : 0)
};
__device__ __forceinline__ void a4_coef(A4Coef& C, const double* Lb, int c) {
  const double* Jb = Lb + A4_LJ;
#pragma unroll
  for (int l = 0; l < 16; ++l) C.L[l] = Lb[18 * c + l];
#pragma unroll
  for (int l = 0; l < 17; ++l) C.L16[l] = Lb[18 * 16 + l];
#pragma unroll
  for (int l = 0; l < 18; ++l) C.L17[l] = Lb[18 * 17 + l];
#pragma unroll
  for (int l = 0; l < 16; ++l) C.Lt[l] = Lb[18 * l + c];
  C.Lt16c = Lb[18 * 16 + c];
  C.Lt17c = Lb[18 * 17 + c];
  C.l1616 = Lb[18 * 16 + 16];
  C.l1716 = Lb[18 * 17 + 16];
  C.l1717 = Lb[18 * 17 + 17];
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    C.Jt[r] = Jb[18 * (6 + r) + c];
    C.J16[r] = Jb[18 * (6 + r) + 16];
    C.J17[r] = Jb[18 * (6 + r) + 17];
  }
  C.Jd = Jb[18 * (c % 6) + c];
  const int rr = c < 12 ? c : 11;
#pragma unroll
  for (int l = 0; l < 18; ++l) C.Jr[l] = Jb[18 * rr + l];
  const int q = c < 6 ? c : 0;
  C.Jq0 = Jb[18 * q + q];
  C.Jq1 = Jb[18 * q + 6 + q];
}
// y = Linv v
__device__ __forceinline__ A4Vec a4_lmul(const A4Coef& C, const A4Vec& v) {
  const double lo = a4_dot16(v.lo, C.L);
  double b16 = a4_dot16(v.lo, C.L16), b17 = a4_dot16(v.lo, C.L17);
  b16 = __fma_rn(C.L16[16], v.h16, b16);
  b17 = __fma_rn(C.L17[16], v.h16, b17);
  b17 = __fma_rn(C.L17[17], v.h17, b17);
  return {lo, b16, b17};
}
// y = Linv' v
__device__ __forceinline__ A4Vec a4_ltmul(const A4Coef& C, const A4Vec& v) {
  double lo = a4_dot16(v.lo, C.Lt);
  lo = __fma_rn(C.Lt16c, v.h16, lo);
  lo = __fma_rn(C.Lt17c, v.h17, lo);
  return {lo, __fma_rn(C.l1716, v.h17, __dmul_rn(C.l1616, v.h16)), __dmul_rn(C.l1717, v.h17)};
}
// init + J' u: the q-row entry of column c (J[c % 6][c], zero for c >= 12) with u[c % 6], plus the
// v rows 6..11 (two chains); u in lanes 0..11, every lane's finite
__device__ __forceinline__ A4Vec a4_jtmul(const A4Coef& C, double u, A4Vec init) {
  const double us = a4_shr6(u);  // u[c - 6] for c >= 6, own below
  const double lo = __dadd_rn(__fma_rn(C.Jd, us, init.lo), a4_dot6(u, C.Jt));
  return {lo, __dadd_rn(init.h16, a4_dot6(u, C.J16)), __dadd_rn(init.h17, a4_dot6(u, C.J17))};
}
// (J v)_c, c < 12 (lanes 12-15: row 11's, unused)
__device__ __forceinline__ double a4_jmul(const A4Coef& C, int c, const A4Vec& v) {
  double a = a4_dot16(v.lo, C.Jr);
  a = __fma_rn(C.Jr[16], v.h16, a);
  a = __fma_rn(C.Jr[17], v.h17, a);
  const double sp = __fma_rn(C.Jq1, a4_shl6(v.lo), __dmul_rn(C.Jq0, v.lo));
  return c < 6 ? sp : a;
}

// The ring buffer of one step: the stage record (this lane's 10 chunks) and the step's vectors.
struct A4Buf {
  double2 rec[10];  // chunks c + 16 t of the lane's problem's stage record
  double v0, v1, z1, y1, l1, ib1;
  double2 hv0, hv1;
};

// Buffer-resource access (uniform base in SGPRs, 32-bit per-lane offset, hardware range check): a
// store or load at an offset past the range does nothing (loads return 0), which masks the stores
// of finished rows and of absent rows without branches.
typedef unsigned int a4u2 __attribute__((ext_vector_type(2)));
typedef unsigned int a4u4 __attribute__((ext_vector_type(4)));
constexpr int A4_OOB = 1 << 27;  // doubles: beyond every range
__device__ __forceinline__ __amdgpu_buffer_rsrc_t a4_rsrc(const void* base, long bytes) {
  const unsigned long long u = (unsigned long long)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u), hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
  const int nb = __builtin_amdgcn_readfirstlane((int)bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0, nb, 0x00020000);
}
__device__ __forceinline__ double a4_ld(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off * 8, 0, 0));
}
__device__ __forceinline__ double2 a4_ld2(__amdgpu_buffer_rsrc_t r, int off) {
  const a4u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off * 8, 0, 0);
  return make_double2(__builtin_bit_cast(double, a4u2{v.x, v.y}), __builtin_bit_cast(double, a4u2{v.z, v.w}));
}
__device__ __forceinline__ void a4_st(double v, __amdgpu_buffer_rsrc_t r, int off) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(a4u2, v), r, off * 8, 0, 0);
}

// OSQP's iteration loop of one wave (four problems).  Per-lane state lives in registers; the
// arrays are per-wave buffer resources (SGPRs) with small per-lane offsets.
template <bool ADAPT>
__device__ __forceinline__ void admm_iter4(const AdmmArgs& a) {
  const SolveParams& P = a.P;
  const int N = P.N, T = P.T, m = 12 * N;
  const int l = threadIdx.x, p = l >> 4, c = l & 15;
  __shared__ double sImg[4 * A4_PS];
  double* Lb = sImg + A4_PS * p;  // this problem's stage image: Linv dense (18 x 18), J dense at +324
  const int bb = a.b0 + 4 * (int)blockIdx.x;
  bool run = bb + p < P.B && !(a.active && !a.active[bb + p]);
  const bool act = run;
  if (!__ballot(run)) return;
  // the wave's four problems' rows of every array
  const long wT = (long)bb * T, wm = (long)bb * m, wR = (long)bb * N * ADM_REC;
  const auto rX = a4_rsrc(a.sx + wT, 32L * T), rZ = a4_rsrc(a.sz + wm, 32L * m), rY = a4_rsrc(a.sy + wm, 32L * m);
  const auto rQ = a4_rsrc(a.qs + wT, 32L * T), rL = a4_rsrc(a.ls + wm, 32L * m), rI = a4_rsrc(a.I + wm, 32L * m);
  const auto rH = a4_rsrc(a.w + wT, 32L * T), rR = a4_rsrc(a.R + wR, 32L * N * ADM_REC);
  int prow = p;  // the row whose problem this lane's loads read (a finished or idle row reads a running one's)
  auto pick_shadow = [&]() {
    const unsigned long long any = __ballot(run);
    if (any && !run) prow = (__ffsll((long long)any) - 1) >> 4;
  };
  pick_shadow();
  int oT = prow * T, om = prow * m, oR = prow * N * ADM_REC;
  const int bown = bb + p;
  const double c_cost = a.cs[bb + prow];
  double rho = a.srho[bb + prow];
  double rv = 1e3 * rho, ri = 1.0 / rv;
  const double al = a.A.alpha, sg = a.A.sigma, al1 = 1.0 - al;
  for (int e = l; e < 4 * A4_PS; e += 64) sImg[e] = 0.0;
  // this lane's chunk destinations in the image (packed Linv -> 18 i + j, compact J -> 324 + 18 i + j)
  int dst[10];
#pragma unroll
  for (int t = 0; t < 10; ++t) {
    int code = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      int e = 2 * (c + 16 * t) + h;
      if (e > ADM_REC - 1) e = ADM_REC - 1;
      int d;
      if (e < ADM_LP) {
        int i = 0;
        while ((i + 1) * (i + 2) / 2 <= e) ++i;
        d = 18 * i + (e - i * (i + 1) / 2);
      } else if (e < ADM_LP + ADM_JC) {
        const int q = e - ADM_LP;
        if (q < 6) d = A4_LJ + 19 * q;
        else if (q < 12) d = A4_LJ + 18 * (q - 6) + q;
        else d = A4_LJ + 18 * (6 + (q - 12) / 18) + (q - 12) % 18;
      } else {
        d = A4_PS - 1;
      }
      code |= d << (16 * h);
    }
    dst[t] = code;
  }
  const int cc = c < 12 ? c : 11;
  const int c16 = 16 + (c & 1);  // lanes 0, 1 store the u-part pair (16, 17)
  const bool lo12 = c < 12, lo2 = c < 2;
  int chk_off[10];
#pragma unroll
  for (int t = 0; t < 10; ++t) chk_off[t] = 2 * ((c + 16 * t) < 146 ? c + 16 * t : 145);
  // the loads of step s (< 2N) of an iteration: its stage record; forward: x_k, q_k; backward: h_k,
  // x_{k+1}; both: block k+1's z, y, l, I.  Every index in bounds (the last stage's missing rows
  // and u-parts read a neighbour, unused).
  auto issue = [&](A4Buf& B, int s) {
    const bool fwd = s < N;
    const int k = fwd ? s : 2 * N - 1 - s;
    const int k1 = k + 1 < N ? k + 1 : N - 1;
    const int kh = k < N - 1 ? k : N - 2;
#ifdef I7M_DIAG
    // I7M_ABLATE 21: every step reads stage 0's record (L2-resident: the sweep without its stream)
    const int ro = oR + (a.ablate == 21 ? 0 : k * ADM_REC);
#else
    const int ro = oR + k * ADM_REC;
#endif
#pragma unroll
    for (int t = 0; t < 10; ++t) B.rec[t] = a4_ld2(rR, ro + chk_off[t]);
    const int ci = k < N - 1 ? c : cc;
    const int kb = fwd ? k : k1;  // the stage of v1
    const int kbh = kb < N - 1 ? kb : N - 2;
    const int cb = kb < N - 1 ? c : cc;
    if (fwd) {
      B.v0 = a4_ld(rX, oT + 18 * k + ci);
      B.v1 = a4_ld(rQ, oT + 18 * kb + cb);
      B.hv0 = a4_ld2(rX, oT + 18 * kh + 16);
      B.hv1 = a4_ld2(rQ, oT + 18 * kbh + 16);
    } else {
      B.v0 = a4_ld(rH, oT + 18 * k + ci);
      B.v1 = a4_ld(rX, oT + 18 * kb + cb);
      B.hv0 = a4_ld2(rH, oT + 18 * kh + 16);
      B.hv1 = a4_ld2(rX, oT + 18 * kbh + 16);
    }
    const int ob = om + 12 * k1 + cc;
    B.z1 = a4_ld(rZ, ob);
    B.y1 = a4_ld(rY, ob);
    B.l1 = a4_ld(rL, ob);
    B.ib1 = a4_ld(rI, ob);
  };
  auto scatter = [&](const A4Buf& B) {
#pragma unroll
    for (int t = 0; t < 10; ++t) {
      Lb[dst[t] & 0xffff] = B.rec[t].x;
      Lb[dst[t] >> 16] = B.rec[t].y;
    }
  };
  A4Buf A0, A1;
  issue(A0, 0);
  issue(A1, 1);
  // carried between steps
  A4Vec hc{0.0, 0.0, 0.0};  // forward: J_{k-1} h_{k-1} (lanes 0..11) / backward: xt_{k+1}
  double tk = __dmul_rn(rv, __dsub_rn(a4_ld(rZ, om + cc), __dmul_rn(ri, a4_ld(rY, om + cc))));  // block k's t
  double ibk = a4_ld(rI, om + cc);
  // the state the backward sweep hands to the next forward sweep's first two steps (their memory
  // copies were loaded before the backward sweep wrote them)
  double nx0 = 0.0, nx1 = 0.0, nz1 = 0.0, ny1 = 0.0;
  double2 nx0h = make_double2(0.0, 0.0), nx1h = make_double2(0.0, 0.0);
  int done_it = 0;
  bool solved = false;
  // one step's start: the record into the image, the step's vectors out of the ring, the ring
  // advanced and the load of step s + 2 issued
  double v0, v1, z1, y1, l1, ib1;
  double2 hv0, hv1;
  A4Coef C;
  auto begin = [&](int s) {
    __asm__ volatile("" ::: "memory");
    scatter(A0);
    __asm__ volatile("" ::: "memory");
    a4_coef(C, Lb, c);
    v0 = A0.v0; v1 = A0.v1; z1 = A0.z1; y1 = A0.y1; l1 = A0.l1; ib1 = A0.ib1; hv0 = A0.hv0; hv1 = A0.hv1;
    A0 = A1;
    int sn = s + 2;
    if (sn >= 2 * N) sn -= 2 * N;
    issue(A1, sn);
  };
  // store offsets: masked (past the range) for rows that do not run
  auto so = [&](bool ok, int off) { return run && ok ? off : A4_OOB; };
  // forward step k < N - 1: rhs, g, h = Linv' Linv g (stored), the next coupling J_k h
  auto fwd = [&](int k) {
    const double t1 = __dmul_rn(rv, __dsub_rn(z1, __dmul_rn(ri, y1)));
    const double init = lo12 ? __dmul_rn(ibk, tk) : 0.0;
    A4Vec r = a4_jtmul(C, t1, A4Vec{init, 0.0, 0.0});
    r.lo = __dadd_rn(__dsub_rn(__dmul_rn(sg, v0), v1), r.lo);
    r.h16 = __dadd_rn(__dsub_rn(__dmul_rn(sg, hv0.x), hv1.x), r.h16);
    r.h17 = __dadd_rn(__dsub_rn(__dmul_rn(sg, hv0.y), hv1.y), r.h17);
    const double rc = __dsub_rn(r.lo, __dmul_rn(__dmul_rn(rv, ibk), hc.lo));  // k = 0: hc = 0
    r.lo = lo12 ? rc : r.lo;
    const A4Vec h = a4_ltmul(C, a4_lmul(C, r));
    a4_st(h.lo, rH, so(true, oT + 18 * k + c));
    a4_st(c == 0 ? h.h16 : h.h17, rH, so(lo2, oT + 18 * k + c16));
    hc.lo = a4_jmul(C, c, h);
    tk = t1;
    ibk = ib1;
  };
  // the last forward step (k = N - 1: 12 rows, no J, no u-part)
  auto fwd_last = [&]() {
    const int k = N - 1;
    A4Vec r{lo12 ? __dmul_rn(ibk, tk) : 0.0, 0.0, 0.0};
    r.lo = __dadd_rn(__dsub_rn(__dmul_rn(sg, v0), v1), r.lo);
    r.lo = __dsub_rn(r.lo, __dmul_rn(__dmul_rn(rv, ibk), hc.lo));
    r.lo = lo12 ? r.lo : 0.0;
    hc = a4_ltmul(C, a4_lmul(C, r));  // the backward sweep starts from xt_{N-1} = h_{N-1}
    a4_st(hc.lo, rH, so(lo12, oT + 18 * k + c));
  };
  // backward step k < N - 1: xt_k, then block k+1's rows and x_{k+1}
  auto bwd = [&](int k) {
    const double u = __dmul_rn(__dmul_rn(rv, ib1), hc.lo);
    const A4Vec s2 = a4_ltmul(C, a4_lmul(C, a4_jtmul(C, u, A4Vec{0.0, 0.0, 0.0})));
    const A4Vec xt{__dsub_rn(v0, s2.lo), __dsub_rn(hv0.x, s2.h16), __dsub_rn(hv0.y, s2.h17)};
    const double zt = __dadd_rn(a4_jmul(C, c, xt), __dmul_rn(ib1, hc.lo));
    const double zr = __dadd_rn(__dmul_rn(al, zt), __dmul_rn(al1, z1));
    double zn = __dadd_rn(zr, __dmul_rn(ri, y1));
    zn = fmin(fmax(zn, l1), l1);
    const double yn = __dadd_rn(y1, __dmul_rn(rv, __dsub_rn(zr, zn)));
    const double xn = __dadd_rn(__dmul_rn(al, hc.lo), __dmul_rn(al1, v1));
    const double xn16 = __dadd_rn(__dmul_rn(al, hc.h16), __dmul_rn(al1, hv1.x));
    const double xn17 = __dadd_rn(__dmul_rn(al, hc.h17), __dmul_rn(al1, hv1.y));
    const bool last1 = k + 1 == N - 1;  // x_{k+1} has no u-part
    const int ob = om + 12 * (k + 1) + c;
    a4_st(zn, rZ, so(lo12, ob));
    a4_st(yn, rY, so(lo12, ob));
    a4_st(xn, rX, so(!last1 || lo12, oT + 18 * (k + 1) + c));
    a4_st(c == 0 ? xn16 : xn17, rX, so(!last1 && lo2, oT + 18 * (k + 1) + c16));
    if (k == 0) {
      nx1 = xn;
      nx1h = make_double2(xn16, xn17);
      nz1 = zn;
      ny1 = yn;
    }
    hc = xt;
  };
  int it;
  for (it = 1; it <= a.A.max_iter; ++it) {
    int s = 0;
    for (int k = 0; k < N - 1; ++k, ++s) {
      begin(s);
      if (it > 1 && k == 0) {
        v0 = nx0; hv0 = nx0h; z1 = nz1; y1 = ny1;
      }
      if (it > 1 && k == 1) {
        v0 = nx1; hv0 = nx1h;
      }
      fwd(k);
    }
    begin(s++);
    if (it > 1 && N == 2) v0 = nx1;  // (N = 2: the last forward step is stage 1)
    fwd_last();
    begin(s++);  // backward k = N - 1: xt_{N-1} = h_{N-1} (in hc), nothing else
    for (int k = N - 2; k >= 0; --k, ++s) {
      begin(s);
      bwd(k);
    }
    // block 0's rows (z~ = I xt_0) and x_0
    {
      const double z0 = a4_ld(rZ, om + cc), y0 = a4_ld(rY, om + cc), l0 = a4_ld(rL, om + cc), i0 = a4_ld(rI, om + cc);
      const double x0 = a4_ld(rX, oT + c);
      const double2 x0h = a4_ld2(rX, oT + 16);
      const double zt = __dmul_rn(i0, hc.lo);
      const double zr = __dadd_rn(__dmul_rn(al, zt), __dmul_rn(al1, z0));
      double zn = __dadd_rn(zr, __dmul_rn(ri, y0));
      zn = fmin(fmax(zn, l0), l0);
      const double yn = __dadd_rn(y0, __dmul_rn(rv, __dsub_rn(zr, zn)));
      const double xn = __dadd_rn(__dmul_rn(al, hc.lo), __dmul_rn(al1, x0));
      const double xn16 = __dadd_rn(__dmul_rn(al, hc.h16), __dmul_rn(al1, x0h.x));
      const double xn17 = __dadd_rn(__dmul_rn(al, hc.h17), __dmul_rn(al1, x0h.y));
      a4_st(zn, rZ, so(lo12, om + c));
      a4_st(yn, rY, so(lo12, om + c));
      a4_st(xn, rX, so(true, oT + c));
      a4_st(c == 0 ? xn16 : xn17, rX, so(lo2, oT + c16));
      nx0 = xn;
      nx0h = make_double2(xn16, xn17);
      tk = __dmul_rn(rv, __dsub_rn(zn, __dmul_rn(ri, yn)));
      ibk = i0;
      hc = A4Vec{0.0, 0.0, 0.0};
    }
    const bool chk = a.A.check && it % a.A.check == 0;
    const bool adapt = ADAPT && a.A.adapt_interval && it % a.A.adapt_interval == 0;
    if (chk || adapt) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      double rest = rho;
      const long bq = bb + prow;
      const bool ok = adm_check<16>(a, N, T, m, c_cost, rho, a.sx + bq * T, a.sz + bq * m, a.sy + bq * m, a.qs + bq * T,
                                    a.ls + bq * m, a.D + bq * T, a.E + bq * m, a.R + bq * N * ADM_REC + REC_J,
                                    a.I + bq * m, a.Pq + bq * N * 36, a.Pd + bq * T, &rest, c);
      bool fin = false;
      if (chk && ok && run) {
        run = false;
        solved = true;
        done_it = it;
        fin = true;
      }
      bool reload = false;
      if constexpr (ADAPT) {
        const bool moved = run && adapt && (rest > rho * a.A.adapt_tol || rest < rho / a.A.adapt_tol);
        const unsigned long long mv = __ballot(moved);
        if (mv) {
          if (moved) {
            rho = rest;
            rv = 1e3 * rho;
            ri = 1.0 / rv;
          }
          // re-factor the rows whose rho moved, one problem at a time on the whole wave (the
          // image is the factor's scratch)
          for (int q = 0; q < 4; ++q) {
            if (!((mv >> (16 * q)) & 0xffff)) continue;
            const long bq2 = bb + q;
            const double rq = __shfl(rho, 16 * q, 64);
            double* scr = sImg;
            adm_factor(a, N, rq, a.Pq + bq2 * N * 36, a.Pd + bq2 * T, a.I + bq2 * m, a.R + bq2 * N * ADM_REC, scr,
                       scr + 30 * I7M_ADMM_FSTRIDE + 388, scr + 30 * I7M_ADMM_FSTRIDE, scr + 18 * I7M_ADMM_FSTRIDE, l);
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
          for (int e = l; e < 4 * A4_PS; e += 64) sImg[e] = 0.0;
          tk = __dmul_rn(rv, __dsub_rn(a4_ld(rZ, om + cc), __dmul_rn(ri, a4_ld(rY, om + cc))));
          reload = true;
        }
      }
      if (!__ballot(run)) break;
      if (__ballot(fin)) {
        // finished rows read a running row's lines from here on
        pick_shadow();
        oT = prow * T;
        om = prow * m;
        oR = prow * N * ADM_REC;
        reload = true;
      }
      if (reload) {
        issue(A0, 0);
        issue(A1, 1);
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  if (c == 0 && act) {
    a.srho[bown] = rho;
    if (a.iters) a.iters[(long)bown * 8 + a.sqp_iter] = solved ? done_it : a.A.max_iter;
    if (a.status) a.status[(long)bown * 8 + a.sqp_iter] = solved ? 1 : 0;
  }
  if (act) {
    const double* D = a.D + (long)bown * T;
    const double* xo = a.sx + (long)bown * T;
    double* so_ = a.sol + (long)bown * T;
    for (int e = c; e < T; e += 16) so_[e] = D[e] * xo[e];
  }
}

template <int CT>  // columns of [P; A] per lane: 9 for N <= 32, 18 for N <= 64
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(I7M_ADMM_SCALE_WPE, I7M_ADMM_SCALE_WPE)))
k_admm_scale(AdmmArgs a) {
  admm_body<1, CT>(a);
}
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(I7M_ADMM_FACTOR_WPE, I7M_ADMM_FACTOR_WPE)))
k_admm_factor(AdmmArgs a) {
  admm_body<8, 1>(a);
}
// four problems per wave (grid = ceil(problems / 4))
template <bool ADAPT>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1))) k_admm_iter(AdmmArgs a) {
  admm_iter4<ADAPT>(a);
}

}  // namespace i7m
