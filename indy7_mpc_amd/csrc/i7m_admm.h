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
// One record per stage, N + 1 per problem: record k = [Linv_k packed (171) | C_{k-1} (216; record
// 0's unused) | compact J_k (120; record N-1's and N's unused)].  The forward sweep's step k reads
// record k as it is; the backward sweep's step k needs C_k, which is record k+1's C — the same
// element offsets plus one record for the C part.  So a step's blocks are one base pointer and
// per-lane constant offsets (no per-element pointer selects).
constexpr int ADM_REC = ADM_LP + 216 + ADM_JC, REC_C = ADM_LP, REC_J = ADM_LP + 216;
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
// dense 18 x 18 lower-triangular Linv into LDS from its packed form
__device__ __forceinline__ void adm_stage_L(double* sL, const double* Lp, int l) {
  for (int e = l; e < 324; e += 64) {
    const int i = e / 18, j = e - 18 * i;
    sL[e] = j <= i ? Lp[adm_tri(i, j)] : 0.0;
  }
}
// A sweep step's blocks as one index space of ADM_ST doubles: packed Linv (171) | C (216) |
// compact J (120); element e of it goes to LDS position adm_pf_dst(e) of [Linv 18 x 18 | C 12 x 18 |
// J 12 x 18] (-1: beyond the space)
constexpr int ADM_ST = ADM_LP + 216 + ADM_JC;
__device__ __forceinline__ int adm_pf_dst(int e) {
  if (e < ADM_LP) {
    int i = 0;
    while ((i + 1) * (i + 2) / 2 <= e) ++i;
    return 18 * i + (e - i * (i + 1) / 2);
  }
  if (e < ADM_LP + 216) return 324 + (e - ADM_LP);
  if (e < ADM_ST) {
    const int c = e - ADM_LP - 216;
    if (c < 6) return 540 + 18 * c + c;
    if (c < 12) return 540 + 18 * (c - 6) + c;
    return 540 + 18 * (6 + (c - 12) / 18) + (c - 12) % 18;
  }
  return -1;
}
// A lane's element t of a step: its record offset for the forward sweep (bits 0-9), for the
// backward sweep (bits 10-19) and its LDS slot + 1 (bits 20-29; 0 = none), packed in one register.
__device__ __forceinline__ int adm_pf_code(int e) {
  if (e >= ADM_ST) return 0;
  const int ob = e + (e >= REC_C && e < REC_J ? ADM_REC : 0);
  return e | (ob << 10) | ((adm_pf_dst(e) + 1) << 20);
}
// one unconditional load per element from a record base and the lane's fixed offsets (lanes past
// the space re-read the base): no branches around the loads, so the wait for them is a counted
// vmcnt, not a vmcnt(0) at a control-flow join.  sh: 0 forward offsets, 10 backward.
__device__ __forceinline__ void adm_pf_load(double pf[8], const double* rec, const int code[8], int sh) {
#pragma unroll
  for (int t = 0; t < 8; ++t) pf[t] = rec[(code[t] >> sh) & 1023];
}
__device__ __forceinline__ void adm_pf_store(const double pf[8], double* sB, const int code[8]) {
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int d = code[t] >> 20;
    if (d) sB[d - 1] = pf[t];
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

__device__ __forceinline__ double adm_wave_max(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}
__device__ __forceinline__ double adm_wave_sum(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
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
// the scaled residual ratios; x, z, y scaled.  Returns solved; rho_est gets the estimate.
__device__ bool adm_check(const AdmmArgs& a, int N, int T, int m, double c, double rho, const double* x,
                          const double* z, const double* y, const double* qs, const double* ls, const double* D,
                          const double* E, const double* Jb, const double* Ib, const double* Pq, const double* Pd,
                          double* rho_est, int l) {
  double pr = 0.0, zn = 0.0, an = 0.0, pri = 0.0, pn = 0.0;
  double dr = 0.0, qn = 0.0, atn = 0.0, pxn = 0.0, dua = 0.0, dn = 0.0, xPx = 0.0, qx = 0.0, sc = 0.0;
  // rows: block 0 = I x_0, block k+1 = J_k z_k + I x_{k+1}
  for (int r = l; r < m; r += 64) {
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
  for (int e = l; e < T; e += 64) {
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
  pr = adm_wave_max(pr); zn = adm_wave_max(zn); an = adm_wave_max(an); pri = adm_wave_max(pri); pn = adm_wave_max(pn);
  dr = adm_wave_max(dr); qn = adm_wave_max(qn); atn = adm_wave_max(atn); pxn = adm_wave_max(pxn);
  dua = adm_wave_max(dua); dn = adm_wave_max(dn);
  xPx = adm_wave_sum(xPx); qx = adm_wave_sum(qx); sc = adm_wave_sum(sc);
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
__device__ void adm_factor(const AdmmArgs& a, int N, double rho, const double* Pq, const double* Pd, const double* Ib,
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
          Rb[ADM_REC * (k + 1) + REC_C + e] = cv;
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
        Rb[ADM_REC * (k + 1) + REC_C + e] = cv;
      }
    }
    wave_sync_all();
  }
}

// The QP in three launches: k_admm_scale (PH 1: scaling, the new q and l; c to a.cs), k_admm_factor
// (PH 8: the block Cholesky) and k_admm_iter (PH 2: OSQP's iterations and the output; PH 4: with
// adaptive rho, whose re-factor needs the factor's registers and LDS — without it the iteration
// kernel is compiled lean).  Each is compiled for its own registers and LDS.
template <int PH, int CT>
__device__ __forceinline__ void admm_body(const AdmmArgs& a) {
  const int b = a.b0 + blockIdx.x;
  const SolveParams& P = a.P;
  if (b >= P.B || (a.active && !a.active[b])) return;
  const int l = threadIdx.x, N = P.N, T = P.T, m = 12 * N;
  constexpr bool FAC = (PH & 8) || (PH & 4);
  // (k_admm_prep: sB holds the column scale factors of a Ruiz pass before the factor needs it)
  __shared__ double sB[(PH & 1) ? 64 * CT : 756], sS[FAC ? 18 * I7M_ADMM_FSTRIDE : 1], sCp[FAC ? 12 * I7M_ADMM_FSTRIDE : 1], sR[32], sW[32], sT0[16], sT1[16];
  __shared__ double sD[(PH & 1) ? 64 * CT : 1], sE[(PH & 1) ? 64 * (2 * CT / 3) : 1];
  double* sL = sB;
  double* sC = sB + 324;
  double* sJ = sB + 540;
  const double* LIN = a.lin + (long)b * (N - 1) * LIN_STRIDE;
  const double* CO = a.cost + (long)b * N * COST_STRIDE;
  const double* QD = a.qpd + (long)b * (N - 1) * QPD_STRIDE;
  const double* X = a.xu + (long)b * T;
  double* x = a.sx + (long)b * T;
  double* z = a.sz + (long)b * m;
  double* y = a.sy + (long)b * m;
  double* qold = a.sq + (long)b * T;
  double* Pq = a.Pq + (long)b * N * 36;
  double* Pd = a.Pd + (long)b * T;
#ifdef I7M_DIAG_ADMM_SHARED_REC  // (timing builds only: every problem's iterations read problem 0's stage records)
  double* Rb = a.R + (long)((PH & 2) ? 0 : b) * (N + 1) * ADM_REC;
#else
  double* Rb = a.R + (long)b * (N + 1) * ADM_REC;
#endif
  double* Jb = Rb + REC_J;  // J_k at Jb + ADM_REC k
  double* Ib = a.I + (long)b * m;
  double* qs = a.qs + (long)b * T;
  double* ls = a.ls + (long)b * m;
  double* D = a.D + (long)b * T;
  double* E = a.E + (long)b * m;

  double* wv = a.w + (long)b * T;
  const double dt = P.dt;

  double c = 1.0;
  if constexpr (PH & 1) {
    c = adm_scale<CT>(a, b, N, T, m, LIN, CO, QD, X, qold, Pq, Pd, Jb, Ib, qs, ls, D, E, sD, sE, sB, l);
    if (l == 0) a.cs[b] = c;
  }
  if constexpr (PH & 8) {
#if I7M_ADMM_FACTOR == 1
    adm_factor_lds(a, N, a.srho[b], Pq, Pd, Ib, Rb, sS, sJ, sL, sCp, l);
#else
    adm_factor(a, N, a.srho[b], Pq, Pd, Ib, Rb, sS, sJ, sL, sCp, l);
#endif
  }
  if constexpr (PH & 2) {
  if constexpr (!(PH & 1)) {
    // the LDS slots no sweep step writes (Linv's upper triangle, J's q-row zeros) are zeros
    for (int e = l; e < 324 + 216 + 216; e += 64) sB[e] = 0.0;
  }
  c = a.cs[b];
  double rho = a.srho[b];
  double rv = 1e3 * rho, ri = 1.0 / rv;
  const double al = a.A.alpha, sg = a.A.sigma;

  // ---- 3. OSQP iterations
  // Each sweep step stages the stage's blocks (packed Linv_k | C | compact J_k: ADM_ST doubles)
  // through LDS.  Everything the next step reads from HBM — its blocks (8 doubles per lane) and
  // its vector entries (x, q, the -I entries, z, y, l of the rows it finishes) — is loaded into
  // registers at the start of this step, before this step's stores, so the loads' latency hides
  // behind the step and waiting for them never waits for a store (vmcnt is in order).  The LDS
  // slots' fixed zeros (Linv's upper triangle, J's q-row zeros) are set above.
  int pcode[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) pcode[t] = adm_pf_code(l + 64 * t);
  int it;
  bool solved = false;
  const bool lx = l < 18, lr = l < 12;
  for (it = 1; it <= a.A.max_iter; ++it) {
    // forward sweep: w_k = Linv_k (rhs_k - C_{k-1} w_{k-1})
    // (the next step's loads are unconditional, at clamped stage / lane indices: in bounds always,
    // unused where a stage has no such block or entry)
    const int l17 = l < 17 ? l : 17, l11 = l < 11 ? l : 11;
    double pf[8], fx, fq, fi, fz, fy;
    adm_pf_load(pf, Rb, pcode, 0);
    fx = x[l17];
    fq = qs[l17];
    fi = Ib[l11];
    fz = z[12 + l11];
    fy = y[12 + l11];
    if (lr) sT0[l] = rv * (z[l] - ri * y[l]);
    for (int k = 0; k < N; ++k) {
      const int nk = k < N - 1 ? 18 : 12;
      adm_sweep_sync();
      adm_pf_store(pf, sB, pcode);
      const double xe = fx, qe = fq, ie = fi, t1 = rv * (fz - ri * fy);
      {
        const int kn = k + 1 < N ? k + 1 : N - 1, kz = k + 2 < N ? k + 2 : N - 1;
        adm_pf_load(pf, Rb + ADM_REC * kn, pcode, 0);
        const int ln = kn < N - 1 ? l17 : l11;
        fx = x[18 * kn + ln];
        fq = qs[18 * kn + ln];
        fi = Ib[12 * kn + l11];
        fz = z[12 * kz + l11];
        fy = y[12 * kz + l11];
      }
      if (k < N - 1 && lr) sT1[l] = t1;
      adm_sweep_sync();
      if (l < nk) {
        const int j = l;
        double acc = j < 12 ? ie * sT0[j] : 0.0;
        if (k < N - 1) acc = adm_dot<12>(acc, sJ + j, 18, sT1);
        double r = (sg * xe - qe) + acc;
        if (k > 0 && j < 12) r -= adm_dot<18>(0.0, sC + 18 * j, 1, sW);
        sR[j] = r;
      }
      adm_sweep_sync();
      double wk = 0.0;
      if (l < nk) {
        wk = adm_dot<18>(0.0, sL + 18 * l, 1, sR);
        wv[18 * k + l] = wk;
      }
      adm_sweep_sync();
      if (l < nk) sW[l] = wk;
      if (lr) sT0[l] = sT1[l];
    }
    // backward sweep: xt_k = Linv_k' (w_k - C_k' xt_{k+1}); then A xt for the rows of block k+1,
    // the relaxation of x_{k+1}, and the projection and dual update of block k+1 (block 0 after
    // the sweep).  xt never leaves registers: step k needs only xt_k and xt_{k+1}.  Every global
    // value a lane reads it wrote itself (lane = index within the knot / block).
    double bw, bz = 0.0, by = 0.0, bl = 0.0, bi = 0.0, bx = 0.0, xtp = 0.0;
    adm_pf_load(pf, Rb + ADM_REC * (N - 1), pcode, 10);
    bw = wv[18 * (N - 1) + l11];
    for (int k = N - 1; k >= 0; --k) {
      const int nk = k < N - 1 ? 18 : 12;
      adm_sweep_sync();
      adm_pf_store(pf, sB, pcode);
      const double we = bw, zr0 = bz, yr0 = by, lr0 = bl, ir0 = bi, xe1 = bx;
      // step k - 1's loads: its blocks, w_{k-1}, block k's rows, x_k (block 0's rows and x_0 at
      // k = 0: there the block loads re-read stage 0, unused)
      {
        const int kp = k > 0 ? k - 1 : 0;
        adm_pf_load(pf, Rb + ADM_REC * kp, pcode, 10);
        bw = wv[18 * kp + l17];
        bz = z[12 * k + l11];
        by = y[12 * k + l11];
        bl = ls[12 * k + l11];
        bi = Ib[12 * k + l11];
        bx = x[18 * k + (k < N - 1 ? l17 : l11)];
      }
      adm_sweep_sync();
      if (l < nk) {
        double r = we;
        if (k < N - 1) r -= adm_dot<12>(0.0, sC + l, 18, sW);
        sR[l] = r;
      }
      adm_sweep_sync();
      double xk = 0.0;
      if (l < nk) xk = adm_dot<18>(0.0, sL + l, 18, sR);
      // sW holds xt_{k+1}'s x part until block k+1's rows are done; sR takes xt_k once every lane
      // has read the right-hand side
      adm_sweep_sync();
      if (l < nk) sR[l] = xk;
      adm_sweep_sync();
      if (k < N - 1 && lr) {
        const int r = 12 * (k + 1) + l;
        const double zt = adm_dot<18>(0.0, sJ + 18 * l, 1, sR) + ir0 * sW[l];
        const double zr = al * zt + (1.0 - al) * zr0;
        double zn = zr + ri * yr0;
        zn = fmin(fmax(zn, lr0), lr0);
        y[r] = yr0 + rv * (zr - zn);
        z[r] = zn;
      }
      if (k < N - 1) {
        const int nn = k + 1 < N - 1 ? 18 : 12;
        if (l < nn) x[18 * (k + 1) + l] = al * xtp + (1.0 - al) * xe1;
      }
      xtp = xk;
      adm_sweep_sync();
      if (lr) sW[l] = sR[l];
    }
    // block 0 rows and x_0 (their old values were loaded at k = 0)
    if (lr) {
      const double zt = bi * sW[l];
      const double zr = al * zt + (1.0 - al) * bz;
      double zn = zr + ri * by;
      zn = fmin(fmax(zn, bl), bl);
      y[l] = by + rv * (zr - zn);
      z[l] = zn;
    }
    if (lx) x[l] = al * xtp + (1.0 - al) * bx;
    wave_sync_all();
    const bool chk = a.A.check && it % a.A.check == 0;
    const bool adapt = a.A.adapt_interval && it % a.A.adapt_interval == 0;
    if (chk || adapt) {
      double rest = rho;
      const bool ok = adm_check(a, N, T, m, c, rho, x, z, y, qs, ls, D, E, Jb, Ib, Pq, Pd, &rest, l);
      if (chk && ok) {
        solved = true;
        break;
      }
      if constexpr (PH & 4) {
        if (adapt && (rest > rho * a.A.adapt_tol || rest < rho / a.A.adapt_tol)) {
          rho = rest;
          rv = 1e3 * rho;
          ri = 1.0 / rv;
          adm_factor(a, N, rho, Pq, Pd, Ib, Rb, sS, sJ, sL, sCp, l);
        }
      }
    }
  }
  if (l == 0) {
    a.srho[b] = rho;
    if (a.iters) a.iters[(long)b * 8 + a.sqp_iter] = it > a.A.max_iter ? a.A.max_iter : it;
    if (a.status) a.status[(long)b * 8 + a.sqp_iter] = solved ? 1 : 0;
  }
  double* so = a.sol + (long)b * T;
  for (int e = l; e < T; e += 64) so[e] = D[e] * x[e];
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
template <bool ADAPT>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(ADAPT ? I7M_ADMM_WPE : I7M_ADMM_ITER_WPE,
                                                                       ADAPT ? I7M_ADMM_WPE : I7M_ADMM_ITER_WPE)))
k_admm_iter(AdmmArgs a) {
  admm_body<ADAPT ? 6 : 2, 1>(a);
}

}  // namespace i7m
