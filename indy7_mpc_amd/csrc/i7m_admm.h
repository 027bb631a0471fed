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
  int* status;  // (B, I7M_MAX_SQP): 1 solved, 2 solved inaccurate (OSQP's approximate test after max_iter), 0 max_iter reached
  int sqp_iter;
  int b0;      // first problem of this launch (chunked launches: problems [b0, b0 + grid))
  int ablate;  // I7M_DIAG builds only (I7M_ABLATE, timing variants, results invalid); 0 otherwise
  const double* abase;  // the handle's ADMM allocation (every array above lies in it) and its bytes (< 2 GiB)
  long abytes;
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
#define I7M_ADMM_SCALE_WPE 2  // (N <= 32: the linearisation magnitudes stay in registers for all ten passes)
#endif
#ifndef I7M_ADMM_FACTOR_WPE
#define I7M_ADMM_FACTOR_WPE 2
#endif
#ifndef I7M_ADMM_ITER_WPE
#define I7M_ADMM_ITER_WPE 2  // ... and k_admm_iter without adaptive rho (at 3: 78 spilled VGPRs, 30% slower)
#endif
constexpr int ADM_LP = 180, ADM_JC = 120;
// One record per stage, N per problem (problem b's at R + b N ADM_REC): [Linv_k | compact J_k]
// = 300 doubles (150 pieces of 16 B).  Linv_k's rows 0-15 are stored lower-triangular, each padded
// to an even width (a zero after the diagonal of the even rows: 144 doubles), rows 16 and 17 in full
// (36); J_k as its q rows' two diagonals (J[i][i], J[i][6 + i]) and its v rows (6 x 18).
// k_admm_iter streams the record twice per OSQP iteration (forward and backward sweep) into LDS,
// where its DMA lays Linv's rows 0-15 out at widths of four (A5_LREC: the extra pieces read as
// zeros), so every lane's row and column reads are a base plus a constant and the entries past a
// row's width are never read (the DPP fma's bank masks skip them).  The coupling
// C_k = M_{k+1,k} Linv_k' of the factor is never stored: the sweeps apply it as re I_{k+1} J_k and
// the triangular pair.
constexpr int ADM_REC = 300, REC_J = ADM_LP;
// entry (i, j) of Linv_k in the record, and the stored width of row i
__device__ __forceinline__ int adm_lw(int i) { return i < 16 ? 2 * ((i + 2) / 2) : 18; }
__device__ __forceinline__ int adm_lrow(int i) {
  const int h = i >> 1;  // rows 2h, 2h+1 have width 2h + 2
  return i < 16 ? 2 * h * (h + 1) + (i & 1) * (2 * h + 2) : 144 + 18 * (i - 16);
}
__device__ __forceinline__ int adm_lrec(int i, int j) { return adm_lrow(i) + j; }
// the LDS image of a record (k_admm_iter): rows 0-15 at widths 4, 8, 12, 16 (160 doubles), rows 16
// and 17 (36), J (120)
constexpr int A5_LREC = 316, A5_LJ = 196;
__device__ __forceinline__ int a5_lrow(int i) {
  const int g = i >> 2;
  return i < 16 ? 8 * g * (g + 1) + 4 * (g + 1) * (i - 4 * g) : 160 + 18 * (i - 16);
}
// Buffer-resource access (k_admm_factor's and k_admm_iter's DMA and stores): a uniform base in
// SGPRs, 32-bit per-lane byte offsets, the hardware's range check (an offset past the range reads
// zeros and drops stores: A5_OOB masks lanes without branches)
constexpr unsigned A5_OOB = 0x7ff00000u;  // a byte offset past every allocation (< 2 GiB enforced by the host)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t a4_rsrc(const void* base, long bytes) {
  const unsigned long long u = (unsigned long long)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u), hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
  const int nb = __builtin_amdgcn_readfirstlane((int)bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0, nb, 0x00020000);
}
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

// All of a row's (column's) loads issued before its first product: one memory round trip, not
// the default schedule's one per eight loads.
#define ADM_CHK_LOADS_FIRST()                          \
  do {                                                 \
    __builtin_amdgcn_sched_group_barrier(0x020, 24, 0); \
    __builtin_amdgcn_sched_group_barrier(0x002, 96, 0); \
  } while (0)

// OSQP's check_termination on the unscaled residuals (+ the duality gap) and, for adapt_rho,
// the scaled residual ratios; x, z, y scaled.  Returns solved; rho_est gets the estimate.  W lanes
// share one problem (lane l of W): 64 (one problem per wave) or 16 (k_admm_iter: a 16-lane row).
// es scales eps_abs and eps_rel: 1 OSQP's test, 10 its approximate one after max_iter ("solved
// inaccurate", oracle/osqp_admm.py OSQP._check(approximate=True)).
template <int W>
__device__ bool adm_check(const AdmmArgs& a, int N, int T, int m, double c, double rho, const double* x,
                          const double* z, const double* y, const double* qs, const double* ls, const double* D,
                          const double* E, const double* Jb, const double* Ib, const double* Pq, const double* Pd,
                          double* rho_est, int l, double es = 1.0) {
  double pr = 0.0, zn = 0.0, an = 0.0, pri = 0.0, pn = 0.0;
  double dr = 0.0, qn = 0.0, atn = 0.0, pxn = 0.0, dua = 0.0, dn = 0.0, xPx = 0.0, qx = 0.0, sc = 0.0;
  // rows: block 0 = I x_0, block k+1 = J_k z_k + I x_{k+1}.  J's structural zeros are skipped
  // (a q row has two entries: J[i][i], J[i][6 + i]; a column at most one q-row entry); the other
  // terms keep their order, so the sums are the full loops' (0 * x adds nothing).
  for (int r = l; r < m; r += W) {
    const int k = r / 12, i = r - 12 * k;
    // Every operand is loaded up front, from clamped (always valid) addresses, and the branches
    // are selects: one memory round trip per row (the lanes of a wave take both paths anyway).
    const int kk = k > 0 ? k - 1 : 0, iq = i < 6 ? i : 0, iv = i < 6 ? 0 : i - 6;
    const double* G = Jb + ADM_REC * kk;
    const double* xk = x + 18 * kk;
    const double* Gr = G + 12 + 18 * iv;
    const double ib = Ib[r], xr = x[18 * k + i], er = E[r], zr = z[r], yr = y[r], lr = ls[r];
    const double ga = G[iq], gb = G[6 + iq], xa = xk[iq], xb = xk[6 + iq];
    double gv[18], xv[18];
#pragma unroll
    for (int j = 0; j < 18; ++j) {
      gv[j] = Gr[j];
      xv[j] = xk[j];
    }
    ADM_CHK_LOADS_FIRST();
    double aq = 0.0, av = 0.0;  // a q row's two entries, a v row's 18
    aq += ga * xa;
    aq += gb * xb;
#pragma unroll
    for (int j = 0; j < 18; ++j) av += gv[j] * xv[j];
    const double acc = i < 6 ? aq : av;
    const double ax = k == 0 ? ib * xr : acc + ib * xr;
    const double ei = 1.0 / er;
    pr = fmax(pr, fabs(ei * (ax - zr)));
    zn = fmax(zn, fabs(ei * zr));
    an = fmax(an, fabs(ei * ax));
    pri = fmax(pri, fabs(ax - zr));
    pn = fmax(pn, fmax(fabs(zr), fabs(ax)));
    sc += lr * fmax(yr, 0.0) + lr * fmin(yr, 0.0);
  }
  for (int e = l; e < T; e += W) {
    const int k = e / 18, j = e - 18 * k;
    // as the rows: clamped addresses, selects for the branches
    const int jq = j < 12 ? j : 0, jc = j < 6 ? j : 0, kc = k < N - 1 ? k : 0;
    const int jy = j < 6 ? j : (j < 12 ? j - 6 : 0);  // column j's q-row entry: row j or j - 6
    const double* G = Jb + ADM_REC * kc;
    const double* yk = y + 12 * (k < N - 1 ? k + 1 : 0);
    const double xe = x[e], de = D[e], qe = qs[e], pde = Pd[e], ibj = Ib[12 * k + jq], yj = y[12 * k + jq];
    const double gq = G[jq], yq = yk[jy];
    double pq[6], xq[6], gv[6], yv[6];
#pragma unroll
    for (int t = 0; t < 6; ++t) {
      pq[t] = Pq[36 * k + 6 * jc + t];
      xq[t] = x[18 * k + t];
      gv[t] = G[12 + 18 * t + j];
      yv[t] = yk[6 + t];
    }
    ADM_CHK_LOADS_FIRST();
    double pa = 0.0;
#pragma unroll
    for (int t = 0; t < 6; ++t) pa += pq[t] * xq[t];
    const double px = j < 6 ? pa : pde * xe;
    const double at0 = j < 12 ? ibj * yj : 0.0;
    double at1 = j < 12 ? at0 + gq * yq : at0;
#pragma unroll
    for (int t = 0; t < 6; ++t) at1 += gv[t] * yv[t];
    const double aty = k < N - 1 ? at1 : at0;
    const double di = 1.0 / de;
    dr = fmax(dr, fabs(di * ((qe + px) + aty)));
    qn = fmax(qn, fabs(di * qe));
    atn = fmax(atn, fabs(di * aty));
    pxn = fmax(pxn, fabs(di * px));
    dua = fmax(dua, fabs(qe + px + aty));
    dn = fmax(dn, fmax(fabs(qe), fmax(fabs(aty), fabs(px))));
    xPx += xe * px;
    qx += qe * xe;
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
  const double ea = es * a.A.eps_abs, er = es * a.A.eps_rel;
  if (!(pr < ea + er * fmax(zn, an))) return false;
  if (!(dr < ea + er * cinv * fmax(qn, fmax(atn, pxn)))) return false;
  if (a.A.gap) {
    xPx *= cinv; qx *= cinv; sc *= cinv;
    const double gp = xPx + qx + sc;
    if (!(fabs(gp) < ea + er * fmax(fabs(xPx), fmax(fabs(qx), fabs(sc))))) return false;
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
                                            double* D, double* E, double* sD, double* sE, double* sDt, double* sRM, int l) {
  constexpr int RT = 2 * CT / 3;
  const double dt = a.P.dt;
  double qv[CT], etv[RT], dtv[CT <= 9 ? CT : 1];  // (a lane's q entries and its columns' / rows' pass factors)
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
  // N <= 32 (CT <= 9): the linearisation's 108 v-row entries of stage k live in the registers of
  // lanes 2k (rows 6-8 of block k + 1) and 2k + 1 (rows 9-11) for all passes, read once: each pass
  // forms their scaled magnitudes (E_i |a_ij|) D_j once, for both the row maxima (sRM) and, with the
  // partner lane's three rows, the column maxima (sDt); max is exact, so every norm is the port's.
  constexpr bool REG = CT <= 9;
  const int ks = l >> 1, hs = l & 1;
  const bool sv = REG && ks < N - 1;
  double av[REG ? 3 : 1][REG ? 18 : 1];
  if constexpr (REG) {
    const double* L = LIN + LIN_STRIDE * (sv ? ks : 0);
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int j = 0; j < 18; ++j) {
        const int jb = j < 6 ? j : (j < 12 ? 30 + j : 60 + j);
        av[r][j] = sv ? L[jb + 6 * (3 * hs + r)] : 0.0;  // (signed: the J output below uses it too)
      }
  }
#ifdef I7M_DIAG
  // I7M_ABLATE 300000 + P (tools/step_stamps.py --scale): s_memtime at the parts of Ruiz pass P of
  // workgroup 0 (record area 5 of the timeline buffer)
  const int ss_p = a.ablate >= 300000 ? a.ablate - 300000 : -1;
  const bool ss_on = ss_p >= 0 && blockIdx.x == 0;
  unsigned long long ss_t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define AS_STAMP(i)                                                                         \
  do {                                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    unsigned long long v_;                                                                  \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v_)::"memory");             \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    if (ss_on && pass == ss_p) ss_t[i] = v_;                                                \
  } while (0)
#else
#define AS_STAMP(i)
#endif
  for (int pass = 0; pass < a.A.scaling; ++pass) {
    AS_STAMP(0);
    // every pass recomputes its indices (hoisted out of the pass loop they would take ~300 VGPRs)
    const double* Lp = LIN;
    const double* Cp = CO;
    int lp = l;
    asm volatile("" : "+v"(lp));
    if constexpr (REG) {
      double cm[18];
#pragma unroll
      for (int j = 0; j < 18; ++j) cm[j] = 0.0;
      const int kq = sv ? ks : 0;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const double er = sE[12 * (kq + 1) + 6 + 3 * hs + r];
        double rm = 0.0;
#pragma unroll
        for (int j = 0; j < 18; ++j) {
          const double pv = er * fabs(av[r][j]) * sD[18 * kq + j];
          rm = fmax(rm, pv);
          cm[j] = fmax(cm[j], pv);
        }
        if (sv) sRM[12 * (kq + 1) + 6 + 3 * hs + r] = rm;
      }
      // the partner lane's rows (DPP quad_perm [1,0,3,2]), then lane h stores columns 9h..9h+8
#pragma unroll
      for (int j = 0; j < 18; ++j) {
        const long long u = __double_as_longlong(cm[j]);
        const int lo = __builtin_amdgcn_update_dpp(0, (int)u, 0xB1, 0xf, 0xf, true);
        const int hi = __builtin_amdgcn_update_dpp(0, (int)(u >> 32), 0xB1, 0xf, 0xf, true);
        cm[j] = fmax(cm[j], __longlong_as_double(((long long)hi << 32) | (unsigned int)lo));
      }
      if (sv) {
#pragma unroll
        for (int j = 0; j < 9; ++j) sDt[18 * kq + 9 * hs + j] = hs ? cm[9 + j] : cm[j];
      }
      wave_sync_fence();
    }
    AS_STAMP(1);
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
      if constexpr (REG) {
        mj = fmax(mj, sDt[e]);  // (the stage owners' max over the six v rows)
      } else {
#pragma unroll
        for (int r = 0; r < 6; ++r) mj = fmax(mj, Eb[6 + r] * fabs(L[jb + 6 * r]) * dj);
      }
      if (k < N - 1) mx = fmax(mx, mj);
      // (a lane's own pass factors: registers at N <= 32, LDS at the wide variant's register count)
      if constexpr (REG) dtv[t] = 1.0 / sqrt(adm_limit(mx));
      else sDt[lp + 64 * t] = 1.0 / sqrt(adm_limit(mx));
    }
    AS_STAMP(2);
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      const int r = min(lp + 64 * t, m - 1), blk = r / 12, i = r - 12 * blk;
      const double er = sE[r];
      double mx = er * sD[18 * blk + i];
      // row i of J_{blk-1} (block 0's rows are -I on x_0 alone)
      const int kk = blk > 0 ? blk - 1 : 0;
      const double* Db = sD + 18 * kk;
      // rows 0-5: the identity and dt entries; rows 6-11: 18 linearisation entries (at N <= 32
      // their max from the stage owners)
      const int i6 = i < 6 ? i : i - 6;
      const double mi = fmax(er * 1.0 * Db[i6], er * dt * Db[6 + i6]);
      double ml = 0.0;
      if constexpr (REG) {
        ml = sRM[r];
      } else {
        const double* L = Lp + LIN_STRIDE * kk;
#pragma unroll
        for (int j = 0; j < 18; ++j) {
          const int jb = j < 6 ? j : (j < 12 ? 30 + j : 60 + j);
          ml = fmax(ml, er * fabs(L[jb + 6 * i6]) * Db[j]);
        }
      }
      const double mj = i < 6 ? mi : ml;
      if (blk > 0) mx = fmax(mx, mj);
      etv[t] = 1.0 / sqrt(adm_limit(mx));
    }
    AS_STAMP(3);
    wave_sync_fence();
#pragma unroll
    for (int t = 0; t < CT; ++t) {
      const int e = lp + 64 * t;
      double dtt;
      if constexpr (CT <= 9) dtt = dtv[t];
      else dtt = sDt[e];
      if (e < T) sD[e] = sD[e] * dtt;
      qv[t] = dtt * qv[t];
    }
#pragma unroll
    for (int t = 0; t < RT; ++t)
      if (lp + 64 * t < m) sE[lp + 64 * t] = sE[lp + 64 * t] * etv[t];
    wave_sync_fence();
    AS_STAMP(4);
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
    AS_STAMP(5);
  }
#ifdef I7M_DIAG
  if (ss_on && l == 0 && g_tl) {
    unsigned long long* r = g_tl + 8 + 4 * (5ull << 16);
    for (int i = 0; i < 6; ++i) r[i] = ss_t[i];
    r[6] = 0;
    r[9] = (unsigned long long)a.ablate;
    r[10] = 3;  // the scaling's stamp layout
  }
#undef AS_STAMP
#endif
  // scaled data: P <- c D P D, J <- E J D, I <- -E D, q <- c D g (update(q)), l <- E l
  for (int e = l; e < T; e += 64) D[e] = sD[e];
  for (int r = l; r < m; r += 64) E[r] = sE[r];
#pragma unroll 4
  for (int x = l; x < 36 * N; x += 64) {
    const int k = x / 36, q = x - 36 * k, i = q / 6, j = q - 6 * i;
    Pq[x] = adm_pq(CO + COST_STRIDE * k, i, j) * (sD[18 * k + i] * sD[18 * k + j]) * c;
  }
  if constexpr (REG) {
    // J_k by its stage owners, from the registers (rows 6 + 3h .. 8 + 3h, and q rows 3h .. 3h + 2)
    if (sv) {
      double* Jk = Jb + ADM_REC * ks;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int i = 3 * hs + r;
        const double ev = sE[12 * (ks + 1) + 6 + i];
#pragma unroll
        for (int j = 0; j < 18; ++j) Jk[12 + 18 * i + j] = ev * av[r][j] * sD[18 * ks + j];
        const double eq = sE[12 * (ks + 1) + i];
        Jk[i] = eq * 1.0 * sD[18 * ks + i];
        Jk[6 + i] = eq * dt * sD[18 * ks + 6 + i];
      }
    }
  } else {
#pragma unroll 4
    for (int x = l; x < 120 * (N - 1); x += 64) {
      const int k = x / 120, e = x - 120 * k;
      int i, j;
      if (e < 6) { i = e; j = e; }
      else if (e < 12) { i = e - 6; j = e; }
      else { i = 6 + (e - 12) / 18; j = (e - 12) % 18; }
      Jb[ADM_REC * k + e] = sE[12 * (k + 1) + i] * adm_jk(LIN + LIN_STRIDE * k, dt, i, j) * sD[18 * k + j];
    }
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
// A stage's operands arrive one stage ahead by LDS DMA into `stg` (two buffers of 256 doubles:
// compact J_k 120 | P_k's quadratic block 36 | its diagonal 18 | I_k 12 | I_{k+1} 12), so no stage
// waits on a global load; the DMA (inline asm, the compiler does not see it) is waited for by a
// counted s_waitcnt at the next stage's start.
constexpr int AF_STG = 256;
__device__ __forceinline__ void adm_factor(const AdmmArgs& a, int N, double rho, const double* Pq, const double* Pd, const double* Ib,
                           double* Rb, double* sS, double* sJ, double* sL, double* sCp, double* stg, int l0) {
  const double re = 1e3 * rho, sigma = a.A.sigma;
  constexpr int FS = I7M_ADMM_FSTRIDE;  // row stride of S and C_{k-1} in LDS
  double* sCol = sL + 324;  // (the sweeps' C slot, free while factoring)
  const auto rA = a4_rsrc(a.abase, a.abytes);
  auto boff = [&](const double* q) { return (unsigned)__builtin_amdgcn_readfirstlane((int)((const char*)q - (const char*)a.abase)); };
  const unsigned oR = boff(Rb), oPq = boff(Pq), oPd = boff(Pd), oI = boff(Ib);
  const unsigned stg_lds = (unsigned)(unsigned long)(__attribute__((address_space(3))) void*)stg;
  // stage k's pieces: lane l's piece g = l (+ 64): [0, 60) J, [60, 78) Pq, [78, 87) Pd, [87, 93) I_k,
  // [93, 99) I_{k+1}, past 99 nothing
  auto fetch = [&](int k) {
    unsigned vo[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int g = 64 * u + l0;
      unsigned o;
      if (g < 60) o = oR + 8u * (unsigned)(ADM_REC * k + REC_J) + 16u * g;
      else if (g < 78) o = oPq + 8u * (unsigned)(36 * k) + 16u * (g - 60);
      else if (g < 87) o = oPd + 8u * (unsigned)(18 * k) + 16u * (g - 78);
      else if (g < 99) o = oI + 8u * (unsigned)(12 * k) + 16u * (g - 87);
      else o = A5_OOB;
      vo[u] = o - 1024u * u;
    }
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %1\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %2, %4, 0 offen lds\n\t"
        "buffer_load_dwordx4 %3, %4, 0 offen offset:1024 lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "s"(__builtin_amdgcn_readfirstlane(stg_lds + 8u * AF_STG * (k & 1))), "v"(vo[0]), "v"(vo[1]), "s"(rA)
        : "memory");
  };
  fetch(0);
#ifdef I7M_DIAG
  // I7M_ABLATE 200000 + K (tools/step_stamps.py --factor): s_memtime at the phases of stage K of
  // workgroup 0's factor (its own launch: the record area 5 of the timeline buffer)
  const int fs_k = a.ablate >= 200000 && a.ablate < 300000 ? a.ablate - 200000 : -1;
  const bool fs_on = fs_k >= 0 && blockIdx.x == 0;
  unsigned long long fs_t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define AF_STAMP(i)                                                                         \
  do {                                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    unsigned long long v_;                                                                  \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v_)::"memory");             \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    if (fs_on && k == fs_k) fs_t[i] = v_;                                                   \
  } while (0)
#else
#define AF_STAMP(i)
#endif
  for (int k = 0; k < N; ++k) {
    AF_STAMP(0);
    const int nk = k < N - 1 ? 18 : 12;
    // every stage recomputes the lane's indices (hoisted out of the stage loop they would take
    // more registers than the kernel has)
    int l = l0;
    asm volatile("" : "+v"(l));
    const int lr = l < 18 ? l : 17;  // lanes 18-63 shadow lane 17 (never read back)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stage k's operands have landed
    if (k + 1 < N) fetch(k + 1);
    const double* G = stg + AF_STG * (k & 1);
    if (k < N - 1) adm_stage_J(sJ, G, l);
    wave_sync();
    AF_STAMP(1);
    // S is symmetric to the bit (every term's products commute and sum in the same order), so the
    // lanes form its lower triangle (171 entries) and mirror it
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int e = l + 64 * t;
      if (e < 171) {
        int i = (int)((sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);
        i = (i + 1) * (i + 2) / 2 <= e ? i + 1 : (i * (i + 1) / 2 > e ? i - 1 : i);
        const int j = e - i * (i + 1) / 2, ic = i < 12 ? i : 11, jc = j < 12 ? j : 11;
        const double pq = G[120 + 6 * (i < 6 ? i : 0) + (j < 6 ? j : 0)];
        const double pd = G[156 + i];  // (the last stage's rows past 12: overwritten below)
        const double ib = G[174 + ic];
        const double dj = adm_dot2<12>(0.0, sJ + i, 18, sJ + j, 18);
        const double dc = adm_dot2<18>(0.0, sCp + FS * ic, 1, sCp + FS * jc, 1);
        double v = i < 6 && j < 6 ? pq : (i == j && i >= 6 ? pd : 0.0);
        if (i == j) v += sigma;
        if (i == j && i < 12) v += re * (ib * ib);
        if (k < N - 1) v += re * dj;
        if (k > 0 && i < 12 && j < 12) v -= dc;
        if (i >= nk || j >= nk) v = i == j ? 1.0 : 0.0;
        sS[FS * i + j] = v;
        sS[FS * j + i] = v;
      }
    }
    wave_sync();
    AF_STAMP(2);
    double r[18];
#pragma unroll
    for (int j = 0; j < 18; ++j) r[j] = sS[FS * lr + j];
    double myid = 1.0;  // 1 / L_ll of this lane's row (the inverse multiplies by it)
#pragma unroll
    for (int p = 0; p < 18; ++p) {
      const double d = sqrt(adm_readlane(r[p], p));
      const double id = 1.0 / d;
      myid = l == p ? id : myid;
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
    AF_STAMP(3);
    wave_sync();  // every lane has read S before L overwrites it
    static_assert(FS >= 19, "the row's spare column holds 1 / L_ii");
    if (l < 18) {
#pragma unroll
      for (int j = 0; j < 18; ++j) sS[FS * l + j] = r[j];
      sS[FS * l + 18] = myid;
    }
    wave_sync();
    AF_STAMP(4);
    double x[18];
#pragma unroll
    for (int i = 0; i < 18; ++i) {
      // row i of L is read once x_{i-2} exists (two rows of loads in flight, not all 171)
      int o = FS * i;
      if (i >= 2) asm volatile("" : "+v"(o) : "v"(x[i - 2]));
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < i; ++q) acc += sS[o + q] * x[q];
      x[i] = ((i == lr ? 1.0 : 0.0) - acc) * sS[o + 18];  // (the port's order: by 1 / L_ii)
    }
    if (l < 18) {
#pragma unroll
      for (int i = 0; i < 18; ++i) {
        const double v = i < nk && l < nk ? x[i] : 0.0;
        sL[18 * i + l] = v;
        if (l < adm_lw(i)) Rb[ADM_REC * k + adm_lrec(i, l)] = v;  // (+0 above the diagonal)
      }
    }
    wave_sync();
    AF_STAMP(5);
    if (k < N - 1) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int e = l + 64 * t;
        if (e < 216) {
          const int i = e / 18, j = e - 18 * i;
          const double acc = adm_dot2<18>(0.0, sJ + 18 * i, 1, sL + 18 * j, 1);
          const double cv = re * G[186 + i] * acc;
          sCp[FS * i + j] = cv;
        }
      }
    }
    // (LDS only: the stage's global stores are read by no later stage, and the kernel's end or the
    // re-factoring caller's fence orders them; a global release here waited for them every stage)
    wave_sync_fence();
    AF_STAMP(6);
  }
#ifdef I7M_DIAG
  if (fs_on && l0 == 0 && g_tl) {
    unsigned long long* r = g_tl + 8 + 4 * (5ull << 16);
    for (int i = 0; i < 7; ++i) r[i] = fs_t[i];
    r[9] = (unsigned long long)a.ablate;
    r[10] = 2;  // the factor's stamp layout
  }
#undef AF_STAMP
#endif
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
      if (j < adm_lw(i)) Rb[ADM_REC * k + adm_lrec(i, j)] = sL[e];
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
  __shared__ double sB[(PH & 1) ? 64 * CT : 756], sS[FAC ? 18 * I7M_ADMM_FSTRIDE : 1], sCp[FAC ? 12 * I7M_ADMM_FSTRIDE : 1];
  __shared__ double sD[(PH & 1) ? 64 * CT : 1], sE[(PH & 1) ? 64 * (2 * CT / 3) : 1], sRM[(PH & 1) ? 64 * (2 * CT / 3) : 1],
      sCO[(PH & 1) ? (64 * CT / 18 + 1) * COST_STRIDE : 1], sStg[FAC ? 2 * AF_STG : 1];
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
    // the cost blocks every pass reads, in LDS for the launch
    for (int e = l; e < N * COST_STRIDE; e += 64) sCO[e] = CO[e];
    const double c = adm_scale<CT>(a, b, N, T, m, LIN, sCO, QD, X, qold, Pq, Pd, Jb, Ib, qs, ls, D, E, sD, sE, sB, sRM, l);
    if (l == 0) a.cs[b] = c;
  }
  if constexpr (PH & 8) {
#if I7M_ADMM_FACTOR == 1
    adm_factor_lds(a, N, a.srho[b], Pq, Pd, Ib, Rb, sS, sJ, sL, sCp, l);
#else
    adm_factor(a, N, a.srho[b], Pq, Pd, Ib, Rb, sS, sJ, sL, sCp, sStg, l);
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
// by DPP (v_fmac_f64_dpp row_newbcast: no LDS round trip on the sweep's chain); the matrix operand
// is read from LDS, straight out of the stage record as HBM holds it (ADM_REC's padded rows make
// every read a base plus a constant).
//
// Every byte the sweeps read arrives by LDS DMA (buffer_load_dwordx4 ... lds): a step's four stage
// records (10 wave-instructions) and its vectors (3) land in one slot of a three-slot ring two steps
// before the step, so no register holds data in flight (a register ring costs 120 VGPRs, and a
// spilled or copied member waits for its load) and the wave's only waits on memory are one counted
// s_waitcnt vmcnt per step.  The DMA is issued from inline asm, so the compiler neither sees it nor
// drains it at its own waits; the ring's LDS reads are ordinary (compiler-scheduled) reads behind
// the asm's memory clobber.  All arrays are reached through one buffer resource over the handle's
// ADMM allocation (32-bit byte offsets; out-of-range offsets read zeros and drop stores, which
// masks finished and absent rows without branches).  Problems stop at their own termination test.
constexpr int A5_RI = 10;                      // record DMA wave-instructions per step (640 >= 4 x 158 pieces)
constexpr int A5_VI = 3;                       // vector DMA wave-instructions per step (192 >= 4 x 42 pieces)
constexpr int A5_SLOT = 64 * (A5_RI + A5_VI);  // 16-B pieces per ring slot (13 KB)
constexpr int A5_VP = 42;                      // vector pieces per problem and step
constexpr int A5_RP = A5_LREC / 2;             // LDS record pieces per problem and stage (158)
constexpr int A5_VD = 2 * 64 * A5_RI;          // the slot's vector part (doubles)
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
// row_newbcast); the asm opens with the two wait states a DPP read of a VGPR a VALU just wrote
// needs (the compiler pads no asm).  BM: the lanes written (bank b = lanes 4b..4b+3 of every row);
// masked lanes keep their sums.
// sum_{l < 16} coef[l] * v_l as four interleaved chains (l mod 4), combined (a0 + a1) + (a2 + a3):
// the device's and the port's order (oracle/cpp/i7m_cpu.cpp adm_dot16).  TRI 1: lane c takes
// terms l <= c only (a lower-triangular row: the terms of a group of four past lane c's bank are
// masked, those inside it read the row's zero padding); TRI 2: terms l >= c only (a column).  One
// asm statement: the compiler can put nothing between the fma's, so one pair of wait states (for
// a DPP read of v just written) serves all sixteen.
template <int TRI = 0>
__device__ __forceinline__ double a4_dot16(double v, const double* cf) {
  constexpr int M0 = TRI == 1 ? 0xf : TRI == 2 ? 0x1 : 0xf, M1 = TRI == 1 ? 0xe : TRI == 2 ? 0x3 : 0xf;
  constexpr int M2 = TRI == 1 ? 0xc : TRI == 2 ? 0x7 : 0xf, M3 = TRI == 1 ? 0x8 : 0xf;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
#define A4_F(acc, op, n, m) "v_fmac_f64_dpp " acc ", %4, " op " row_newbcast:" #n " row_mask:0xf bank_mask:" m "\n\t"
  asm volatile(
      "s_nop 1\n\t"
      A4_F("%0", "%5", 0, "%21") A4_F("%1", "%6", 1, "%21") A4_F("%2", "%7", 2, "%21") A4_F("%3", "%8", 3, "%21")
      A4_F("%0", "%9", 4, "%22") A4_F("%1", "%10", 5, "%22") A4_F("%2", "%11", 6, "%22") A4_F("%3", "%12", 7, "%22")
      A4_F("%0", "%13", 8, "%23") A4_F("%1", "%14", 9, "%23") A4_F("%2", "%15", 10, "%23") A4_F("%3", "%16", 11, "%23")
      A4_F("%0", "%17", 12, "%24") A4_F("%1", "%18", 13, "%24") A4_F("%2", "%19", 14, "%24") A4_F("%3", "%20", 15, "%24")
      : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)
      : "v"(v), "v"(cf[0]), "v"(cf[1]), "v"(cf[2]), "v"(cf[3]), "v"(cf[4]), "v"(cf[5]), "v"(cf[6]), "v"(cf[7]),
        "v"(cf[8]), "v"(cf[9]), "v"(cf[10]), "v"(cf[11]), "v"(cf[12]), "v"(cf[13]), "v"(cf[14]), "v"(cf[15]),
        "i"(M0), "i"(M1), "i"(M2), "i"(M3));
#undef A4_F
  return __dadd_rn(__dadd_rn(a0, a1), __dadd_rn(a2, a3));
}
// sum_{r = 6..11} coef[r - 6] * u_r as two chains (r even / odd), combined
__device__ __forceinline__ double a4_dot6(double u, const double* cf) {
  double a0 = 0.0, a1 = 0.0;
  asm volatile(
      "s_nop 1\n\t"
      "v_fmac_f64_dpp %0, %2, %3 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, %2, %4 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %2, %5 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, %2, %6 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %2, %7 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, %2, %8 row_newbcast:11 row_mask:0xf bank_mask:0xf"
      : "+v"(a0), "+v"(a1)
      : "v"(u), "v"(cf[0]), "v"(cf[1]), "v"(cf[2]), "v"(cf[3]), "v"(cf[4]), "v"(cf[5]));
  return __dadd_rn(a0, a1);
}
// sum over the row's 16 lanes of cf_c v_c (a pairwise tree: lane 15 gathers lanes 14, 12-13, 8-11,
// 0-7 by row_shr 1, 2, 4, 8; the first level fma(cf_c, v_c, p_{c-1})), broadcast to the row: the
// port's adm_rowsum order.  (bound_ctrl: lanes below the shift read 0; only lane 15 is kept)
template <int n>
__device__ __forceinline__ double a4_shr(double v) {
  const long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)u, 0x110 + n, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(u >> 32), 0x110 + n, 0xf, 0xf, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double a4_rowsum(double cf, double v) {
  double p = __fma_rn(cf, v, a4_shr<1>(__dmul_rn(cf, v)));
  p = __dadd_rn(p, a4_shr<2>(p));
  p = __dadd_rn(p, a4_shr<4>(p));
  p = __dadd_rn(p, a4_shr<8>(p));
  return a4_bc<15>(p);
}
// A stage's coefficients, read from the ring slot in four sets, each just before the phase ahead
// of the one that uses it (the reads stay where they are written: the fma asm is volatile).  R is
// the problem's record in the slot.
struct A4CJ {
  double Jt[6], J16[6], J17[6], Jd;  // J column c (rows 6..11), columns 16, 17 (rows 6..11), J[c % 6][c]
};
struct A4CL {
  double L[16];          // Linv row c (l < 16; the entries past the padded row are never used)
  double Lc16, Lc17;     // Linv[16][c], Linv[17][c]
  double d66, d76, d77;  // Linv[16][16], Linv[17][16], Linv[17][17]
};
struct A4CT {
  double Lt[16];  // Linv column c (rows l < 16; rows whose padded width ends before c are never used)
};
struct A4CR {
  double Jr[18], Jq0, Jq1;  // J row c (v rows 6..11; clamped outside them), J[q][q], J[q][6 + q] (q = c < 6 ? c : 0)
};
__device__ __forceinline__ void a4_ldj(A4CJ& C, const double* R, int c) {
  const double* J = R + A5_LJ;  // [J[i][i] (6) | J[i][6 + i] (6) | v rows 6 x 18]
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    C.Jt[r] = J[12 + 18 * r + c];
    C.J16[r] = J[12 + 18 * r + 16];
    C.J17[r] = J[12 + 18 * r + 17];
  }
  C.Jd = c < 12 ? J[c] : 0.0;
}
__device__ __forceinline__ void a4_ldl(A4CL& C, const double* R, const double* Rrow, int c) {
#pragma unroll
  for (int l = 0; l < 16; ++l) C.L[l] = Rrow[l];
  C.Lc16 = R[160 + c];
  C.Lc17 = R[178 + c];
  C.d66 = R[176];
  C.d76 = R[194];
  C.d77 = R[195];
}
// row l's entry c: R + adm_lrow(l) + c (adm_lrow a constant per l)
__device__ __forceinline__ void a4_ldt(A4CT& C, const double* R, int c) {
  constexpr int rs[16] = {0, 4, 8, 12, 16, 24, 32, 40, 48, 60, 72, 84, 96, 112, 128, 144};
#pragma unroll
  for (int l = 0; l < 16; ++l) C.Lt[l] = R[rs[l] + c];
}
__device__ __forceinline__ void a4_ldr(A4CR& C, const double* R, int c) {
  const double* J = R + A5_LJ;
  const int rr = c < 6 ? 0 : (c < 12 ? c - 6 : 5);
#pragma unroll
  for (int l = 0; l < 18; ++l) C.Jr[l] = J[12 + 18 * rr + l];
  const int q = c < 6 ? c : 0;
  C.Jq0 = J[q];
  C.Jq1 = J[6 + q];
}
// y = Linv v (rows 16, 17: the row sums of Linv[16 or 17][c] v_c, then the (16, 17) block)
__device__ __forceinline__ A4Vec a4_lmul(const A4CL& C, const A4Vec& v) {
  const double lo = a4_dot16<1>(v.lo, C.L);
  const double s16 = a4_rowsum(C.Lc16, v.lo), s17 = a4_rowsum(C.Lc17, v.lo);
  const double b16 = __fma_rn(C.d66, v.h16, s16);
  const double b17 = __fma_rn(C.d77, v.h17, __fma_rn(C.d76, v.h16, s17));
  return {lo, b16, b17};
}
// y = Linv' v
__device__ __forceinline__ A4Vec a4_ltmul(const A4CL& L, const A4CT& C, const A4Vec& v) {
  double lo = a4_dot16<2>(v.lo, C.Lt);
  lo = __fma_rn(L.Lc16, v.h16, lo);
  lo = __fma_rn(L.Lc17, v.h17, lo);
  return {lo, __fma_rn(L.d76, v.h17, __dmul_rn(L.d66, v.h16)), __dmul_rn(L.d77, v.h17)};
}
// init + J' u: the q-row entry of column c (J[c % 6][c], zero for c >= 12) with u[c % 6], plus the
// v rows 6..11 (two chains); u in lanes 0..11, every lane's finite
__device__ __forceinline__ A4Vec a4_jtmul(const A4CJ& C, double u, A4Vec init) {
  const double us = a4_shr6(u);  // u[c - 6] for c >= 6, own below
  const double lo = __dadd_rn(__fma_rn(C.Jd, us, init.lo), a4_dot6(u, C.Jt));
  return {lo, __dadd_rn(init.h16, a4_dot6(u, C.J16)), __dadd_rn(init.h17, a4_dot6(u, C.J17))};
}
// (J v)_c, c < 12 (lanes 12-15: row 11's, unused)
__device__ __forceinline__ double a4_jmul(const A4CR& C, int c, const A4Vec& v) {
  double a = a4_dot16(v.lo, C.Jr);
  a = __fma_rn(C.Jr[16], v.h16, a);
  a = __fma_rn(C.Jr[17], v.h17, a);
  const double sp = __fma_rn(C.Jq1, a4_shl6(v.lo), __dmul_rn(C.Jq0, v.lo));
  return c < 6 ? sp : a;
}

typedef unsigned int a4u2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double a5_ld(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
__device__ __forceinline__ void a5_st(double v, __amdgpu_buffer_rsrc_t r, unsigned off) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(a4u2, v), r, off, 0, 0);
}
// one step's DMA: 10 record wave-instructions (per-lane offsets ro[t], the stage in soffset) and 3
// vector ones (per-lane offsets vo[u]), to the slot at LDS byte address `lds`.  The instruction
// offset moves the LDS destination as well as the source (tools/probes/lds_dma_offset_probe), so
// M0 (saved and restored around) steps by 4 KB every four wave-instructions and the per-lane
// offsets carry -1 KB (t mod 4) (a5_dma_off).
__device__ __forceinline__ unsigned a5_dma_off(int t) { return 1024u * (unsigned)(t & 3); }
__device__ __forceinline__ void a5_dma(__amdgpu_buffer_rsrc_t r, unsigned lds, const unsigned (&ro)[A5_RI], unsigned so,
                                       const unsigned (&vo)[A5_VI]) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %2, %15, %16 offen lds\n\t"
      "buffer_load_dwordx4 %3, %15, %16 offen offset:1024 lds\n\t"
      "buffer_load_dwordx4 %4, %15, %16 offen offset:2048 lds\n\t"
      "buffer_load_dwordx4 %5, %15, %16 offen offset:3072 lds\n\t"
      "s_add_u32 m0, m0, 0x1000\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %6, %15, %16 offen lds\n\t"
      "buffer_load_dwordx4 %7, %15, %16 offen offset:1024 lds\n\t"
      "buffer_load_dwordx4 %8, %15, %16 offen offset:2048 lds\n\t"
      "buffer_load_dwordx4 %9, %15, %16 offen offset:3072 lds\n\t"
      "s_add_u32 m0, m0, 0x1000\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %10, %15, %16 offen lds\n\t"
      "buffer_load_dwordx4 %11, %15, %16 offen offset:1024 lds\n\t"
      "buffer_load_dwordx4 %12, %15, 0 offen offset:2048 lds\n\t"
      "buffer_load_dwordx4 %13, %15, 0 offen offset:3072 lds\n\t"
      "s_add_u32 m0, m0, 0x1000\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %14, %15, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(ro[0]), "v"(ro[1]), "v"(ro[2]), "v"(ro[3]), "v"(ro[4]), "v"(ro[5]), "v"(ro[6]), "v"(ro[7]),
        "v"(ro[8]), "v"(ro[9]), "v"(vo[0]), "v"(vo[1]), "v"(vo[2]), "s"(r), "s"(__builtin_amdgcn_readfirstlane(so))
      : "memory");
}
// the step's slot has landed: at most 13 vector-memory operations in flight (the next step's DMA,
// or the stores issued after its first ones: every operation completes in issue order)
__device__ __forceinline__ void a5_wait() { asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); }
// two problems per wave (k_admm_iter2): 5 record and 2 vector wave-instructions per step
__device__ __forceinline__ void a5_dma2(__amdgpu_buffer_rsrc_t r, unsigned lds, const unsigned (&ro)[5], unsigned so,
                                        const unsigned (&vo)[2]) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %2, %9, %10 offen lds\n\t"
      "buffer_load_dwordx4 %3, %9, %10 offen offset:1024 lds\n\t"
      "buffer_load_dwordx4 %4, %9, %10 offen offset:2048 lds\n\t"
      "buffer_load_dwordx4 %5, %9, %10 offen offset:3072 lds\n\t"
      "s_add_u32 m0, m0, 0x1000\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %6, %9, %10 offen lds\n\t"
      "buffer_load_dwordx4 %7, %9, 0 offen offset:1024 lds\n\t"
      "buffer_load_dwordx4 %8, %9, 0 offen offset:2048 lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(ro[0]), "v"(ro[1]), "v"(ro[2]), "v"(ro[3]), "v"(ro[4]),
        "v"(vo[0]), "v"(vo[1]), "s"(r), "s"(__builtin_amdgcn_readfirstlane(so))
      : "memory");
}
__device__ __forceinline__ void a5_wait2() { asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); }
__device__ __forceinline__ void a5_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// OSQP's iteration loop of one wave (PW problems: 4, or 2 in k_admm_iter2, whose rows 2 and 3 idle
// so that the ring takes 21 KB and two waves can share a SIMD).  Per-lane state lives in registers.
template <bool ADAPT, int PW = 4>
__device__ __forceinline__ void admm_iter4(const AdmmArgs& a) {
  static_assert(PW == 4 || PW == 2, "four or two problems per wave");
  constexpr int RI = PW == 4 ? A5_RI : 5, VI = PW == 4 ? A5_VI : 2;  // record / vector DMA wave-instructions
  constexpr int SLOT = 64 * (RI + VI), VD = 2 * 64 * RI;
  constexpr int PL = PW - 1;  // the last real row (idle rows read its slot data)
  const SolveParams& P = a.P;
  const int N = P.N, T = P.T, m = 12 * N;
  const int l = threadIdx.x, p = l >> 4, c = l & 15;
  __shared__ double2 sRing[3 * SLOT];
  double* const ring = (double*)sRing;
  const unsigned ring_lds = (unsigned)(unsigned long)(__attribute__((address_space(3))) void*)sRing;
  const int bb = a.b0 + PW * (int)blockIdx.x;
#ifdef I7M_DIAG
  // I7M_ABLATE 100000 + 100 IT + S (tools/step_stamps.py): s_memtime (shader cycles) at nine points
  // of sweep step S of OSQP iteration IT in workgroup 0, to the timeline buffer's record area 5
  // (stamps fenced by sched barriers: read the shares, not the length)
  const int tr_it = a.ablate >= 100000 && a.ablate < 200000 ? (a.ablate - 100000) / 100 : -1, tr_s = a.ablate % 100;
  const bool tr_on = tr_it >= 0 && blockIdx.x == 0;
  unsigned long long tr_t[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  int tr_cur = -1;
#define A5_STAMP(i)                                                                         \
  do {                                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    unsigned long long v_;                                                                  \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v_)::"memory");             \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    if (tr_on && it == tr_it && tr_cur == tr_s) tr_t[i] = v_;                               \
  } while (0)
#else
#define A5_STAMP(i)
#endif
  bool run = p < PW && bb + p < P.B && !(a.active && !a.active[bb + p]);
  const bool act = run;
  if (!__ballot(run)) return;
  const int bown = bb + p;
  // one resource over the whole allocation; every array as a byte offset in it
  const auto rA = a4_rsrc(a.abase, a.abytes);
  auto boff = [&](const double* q) { return (unsigned)__builtin_amdgcn_readfirstlane((int)((const char*)q - (const char*)a.abase)); };
  const unsigned oX = boff(a.sx), oZ = boff(a.sz), oY = boff(a.sy), oQ = boff(a.qs), oL = boff(a.ls), oI = boff(a.I);
  const unsigned oH = boff(a.w), oR = boff(a.R);
  // this lane's own rows (stores, the block-0 epilogue)
  const unsigned xT = oX + 8u * (unsigned)(bown * T), hT = oH + 8u * (unsigned)(bown * T);
  const unsigned zM = oZ + 8u * (unsigned)(bown * m), yM = oY + 8u * (unsigned)(bown * m);
  const unsigned lM = oL + 8u * (unsigned)(bown * m), iM = oI + 8u * (unsigned)(bown * m);
  const double c_cost = a.cs[bown < P.B ? bown : bb];
  double rho = a.srho[bown < P.B ? bown : bb];
  double rv = 1e3 * rho, ri = 1.0 / rv;
  const double al = a.A.alpha, sg = a.A.sigma, al1 = 1.0 - al;
  const int cc = c < 12 ? c : 11;
  const int c16 = 16 + (c & 1);  // lanes 0, 1 store the u-part pair (16, 17)
  const bool lo12 = c < 12, lo2 = c < 2;
  // DMA source offsets of this lane's pieces (rows that do not run read nothing: out of range).
  // Records: piece g = 64 t + l of the four problems' 632; vectors: piece g = 64 u + l of their
  // 168, problem g / 42 piece j = g % 42: [0, 9) v0, [9, 18) v1, [18, 42) z, y, l, I (6 each).
  unsigned ro[RI], vF[VI], vB[VI], vD[VI], vZ[VI], vo[VI];
  int vcls[VI];
  auto offsets = [&]() {
    const unsigned long long rm = __ballot(run);
#pragma unroll
    for (int t = 0; t < RI; ++t) {
      const int g = 64 * t + l, q = g / A5_RP, j = g - A5_RP * q;
      const bool ok = q < PW && ((rm >> (16 * q)) & 1);
      // LDS piece j of the record -> its piece in HBM (rows 0-15 from width 4 to the stored even
      // width: the pieces past it read as zeros)
      int hp;
      if (j < 80) {
        int r = 0;
#pragma unroll
        for (int i = 1; i < 16; ++i) r = 2 * j >= a5_lrow(i) ? i : r;
        const int cp = 2 * j - a5_lrow(r);
        hp = cp < adm_lw(r) ? (adm_lrow(r) + cp) / 2 : -1;
      } else {
        hp = j - 8;  // rows 16, 17 and J: HBM piece 72 + (j - 80) / 90 + (j - 98)
      }
      ro[t] = (ok && hp >= 0 ? oR + 8u * (unsigned)((bb + q) * N * ADM_REC) + 16u * hp : A5_OOB) - a5_dma_off(t);
    }
#pragma unroll
    for (int u = 0; u < VI; ++u) {
      const int g = 64 * u + l, q = g / A5_VP, j = g - A5_VP * q;
      const bool ok = q < PW && ((rm >> (16 * q)) & 1);
      const unsigned rT = 8u * (unsigned)((bb + q) * T), rM = 8u * (unsigned)((bb + q) * m);
      unsigned f, bk;
      int cl;
      if (j < 9) {
        f = oX + rT + 16u * j; bk = oH + rT + 16u * j; cl = 0;
      } else if (j < 18) {
        f = oQ + rT + 16u * (j - 9); bk = oX + rT + 16u * (j - 9); cl = 1;
      } else {
        const int jj = j - 18, w = jj / 6;
        f = (w == 0 ? oZ + 0u : w == 1 ? oY + 0u : w == 2 ? oL + 0u : oI + 0u) + rM + 16u * (jj - 6 * w);
        bk = f; cl = w == 0 ? 3 : 2;
      }
      const unsigned o = a5_dma_off(RI + u);
      vF[u] = (ok ? f : A5_OOB) - o;
      vB[u] = (ok ? bk : A5_OOB) - o;
      vD[u] = ok ? (cl < 2 ? 144u : 96u) : 0u;  // bytes per stage
      vZ[u] = ok && cl == 3 ? oL - oZ : 0u;     // z's pieces from l's lines
      vcls[u] = cl;
    }
  };
  offsets();
  // step s's vector offsets from scratch (s < 2N): forward: x_k, q_k; backward: h_k, x_{k+1};
  // both: block k+1's z, y, l, I (the last stage's missing block reads block N-1's, unused).
  // (zl: the step is past the first iteration, where z = l: every block's projection onto its
  // equality rows, fmin(fmax(., l), l), is l itself, so z's pieces come from l's lines)
  auto vfull = [&](int s, bool zl) {
    const bool fwd = s < N;
    const int k = fwd ? s : 2 * N - 1 - s;
    const int k1 = k + 1 < N ? k + 1 : N - 1;
    const int kb = fwd ? k : k1;
#pragma unroll
    for (int u = 0; u < VI; ++u) {
      const unsigned st = vcls[u] == 0 ? 144u * k : (vcls[u] == 1 ? 144u * kb : 96u * k1);
      vo[u] = (fwd ? vF[u] + 0u : vB[u] + 0u) + (zl ? vZ[u] + st : st);
    }
  };
  // issue step s's DMA into ring slot `slot`: the vector offsets advance by one stage (forward
  // steps 1..N-2 and backward steps N+2.. are the previous step's one stage on) or are recomputed
  auto issue = [&](int s, int slot, bool zl) {
    const bool fwd = s < N;
    const int k = fwd ? s : 2 * N - 1 - s;
    if (s == 0 || s == N - 1 || s == N || s == N + 1) {
      vfull(s, zl);
    } else {
#pragma unroll
      for (int u = 0; u < VI; ++u) vo[u] = fwd ? vo[u] + vD[u] : vo[u] - vD[u];
    }
#ifdef I7M_DIAG
    // I7M_ABLATE 21: every step reads stage 0's record (L2-resident: the sweep without its stream)
    const unsigned so = 8u * (unsigned)(a.ablate == 21 ? 0 : k * ADM_REC);
#else
    const unsigned so = 8u * (unsigned)(k * ADM_REC);
#endif
    if constexpr (PW == 4)
      a5_dma(rA, ring_lds + 16u * SLOT * slot, ro, so, vo);
    else
      a5_dma2(rA, ring_lds + 16u * SLOT * slot, ro, so, vo);
  };
  issue(0, 0, false);
  issue(1, 1, false);
  int it = 1;
  // carried between steps
  A4Vec hc{0.0, 0.0, 0.0};  // forward: J_{k-1} h_{k-1} (lanes 0..11) / backward: xt_{k+1}
  // block 0's rows and x_0 (only the epilogue updates them) and the state the backward sweep hands
  // to the next forward sweep's first two steps (their DMA was issued before the sweep wrote them)
  double b0z = a5_ld(rA, zM + 8 * cc), b0y = a5_ld(rA, yM + 8 * cc), b0l = a5_ld(rA, lM + 8 * cc), b0i = a5_ld(rA, iM + 8 * cc);
  double nx0 = a5_ld(rA, xT + 8 * c), nx1 = 0.0, nz1 = 0.0, ny1 = 0.0;
  double2 nx0h = make_double2(a5_ld(rA, xT + 8 * 16), a5_ld(rA, xT + 8 * 17)), nx1h = make_double2(0.0, 0.0);
  double tk = __dmul_rn(rv, __dsub_rn(b0z, __dmul_rn(ri, b0y)));  // block k's t
  double ibk = b0i;
  int done_it = 0;
  bool solved = false;
  double v0, v1, z1, y1, l1, ib1;
  double2 hv0, hv1;
  A4CJ CJ;
  A4CL CL;
  A4CT CT;
  A4CR CR;
  const double* R = nullptr;
  // one step's start: wait for its slot, issue step s + 2's DMA into the slot step s - 1 used, read
  // the step's vectors (rows ci of v0, cb of v1: the last stage's 12 rows clamped) and the first
  // two coefficient sets
  auto begin = [&](int s, int slot, int ci, int cb) {
#ifdef I7M_DIAG
    tr_cur = s;
#endif
    A5_STAMP(0);
    if constexpr (PW == 4)
      a5_wait();
    else
      a5_wait2();
    A5_STAMP(1);
    int sn = s + 2, sl = slot + 2;
    if (sn >= 2 * N) sn -= 2 * N;
    if (sl >= 3) sl -= 3;
    issue(sn, sl, it > 1 || sn < s);
    A5_STAMP(2);
    const double* S = ring + 2 * SLOT * slot;
    R = S + A5_LREC * (p < PW ? p : PL);
    const double* V = S + VD + 2 * A5_VP * (p < PW ? p : PL);  // [v0 18 | v1 18 | z 12 | y 12 | l 12 | I 12]
    v0 = V[ci];
    v1 = V[18 + cb];
    hv0 = make_double2(V[16], V[17]);
    hv1 = make_double2(V[34], V[35]);
    z1 = V[36 + cc];
    y1 = V[48 + cc];
    l1 = V[60 + cc];
    ib1 = V[72 + cc];
    a4_ldj(CJ, R, c);
    a4_ldl(CL, R, R + a5_lrow(c), c);
    A5_STAMP(3);
  };
  // store offsets: masked (past the range) for rows that do not run
  auto so = [&](bool ok, unsigned off) { return run && ok ? off + 0u : A5_OOB + 0u; };
  // Linv' Linv r, with J's row set read behind the first product when `jr`
  auto llt = [&](const A4Vec& r, bool jr) {
    A5_STAMP(4);
    a4_ldt(CT, R, c);
    const A4Vec y = a4_lmul(CL, r);
    A5_STAMP(5);
    if (jr) a4_ldr(CR, R, c);
    const A4Vec o = a4_ltmul(CL, CT, y);
    A5_STAMP(6);
    return o;
  };
  // forward step k < N - 1: rhs, g, h = Linv' Linv g (stored), the next coupling J_k h
  auto fwd = [&](int k) {
    const double t1 = __dmul_rn(rv, __dsub_rn(z1, __dmul_rn(ri, y1)));
    const double init = lo12 ? __dmul_rn(ibk, tk) : 0.0;
    A4Vec r = a4_jtmul(CJ, t1, A4Vec{init, 0.0, 0.0});
    r.lo = __dadd_rn(__dsub_rn(__dmul_rn(sg, v0), v1), r.lo);
    r.h16 = __dadd_rn(__dsub_rn(__dmul_rn(sg, hv0.x), hv1.x), r.h16);
    r.h17 = __dadd_rn(__dsub_rn(__dmul_rn(sg, hv0.y), hv1.y), r.h17);
    const double rc = __dsub_rn(r.lo, __dmul_rn(__dmul_rn(rv, ibk), hc.lo));  // k = 0: hc = 0
    r.lo = lo12 ? rc : r.lo;
    const A4Vec h = llt(r, true);
    a5_st(h.lo, rA, so(true, hT + 8u * (18 * k + c)));
    a5_st(c == 0 ? h.h16 + 0.0 : h.h17 + 0.0, rA, so(lo2, hT + 8u * (18 * k + c16)));
    A5_STAMP(7);
    hc.lo = a4_jmul(CR, c, h);
    tk = t1;
    ibk = ib1;
    A5_STAMP(8);
  };
  // the last forward step (k = N - 1: 12 rows, no J, no u-part)
  auto fwd_last = [&]() {
    const int k = N - 1;
    A4Vec r{lo12 ? __dmul_rn(ibk, tk) : 0.0, 0.0, 0.0};
    r.lo = __dadd_rn(__dsub_rn(__dmul_rn(sg, v0), v1), r.lo);
    r.lo = __dsub_rn(r.lo, __dmul_rn(__dmul_rn(rv, ibk), hc.lo));
    r.lo = lo12 ? r.lo : 0.0;
    hc = llt(r, false);  // the backward sweep starts from xt_{N-1} = h_{N-1}
    a5_st(hc.lo, rA, so(lo12, hT + 8u * (18 * k + c)));
  };
  // backward step k < N - 1: xt_k, then block k+1's rows and x_{k+1}
  auto bwd = [&](int k) {
    const double u = __dmul_rn(__dmul_rn(rv, ib1), hc.lo);
    const A4Vec s2 = llt(a4_jtmul(CJ, u, A4Vec{0.0, 0.0, 0.0}), true);
    const A4Vec xt{__dsub_rn(v0, s2.lo), __dsub_rn(hv0.x, s2.h16), __dsub_rn(hv0.y, s2.h17)};
    const double zt = __dadd_rn(a4_jmul(CR, c, xt), __dmul_rn(ib1, hc.lo));
    A5_STAMP(7);
    const double zr = __dadd_rn(__dmul_rn(al, zt), __dmul_rn(al1, z1));
    double zn = __dadd_rn(zr, __dmul_rn(ri, y1));
    zn = fmin(fmax(zn, l1), l1);
    const double yn = __dadd_rn(y1, __dmul_rn(rv, __dsub_rn(zr, zn)));
    const double xn = __dadd_rn(__dmul_rn(al, hc.lo), __dmul_rn(al1, v1));
    const double xn16 = __dadd_rn(__dmul_rn(al, hc.h16), __dmul_rn(al1, hv1.x));
    const double xn17 = __dadd_rn(__dmul_rn(al, hc.h17), __dmul_rn(al1, hv1.y));
    const bool last1 = k + 1 == N - 1;  // x_{k+1} has no u-part
    const unsigned ob = 8u * (12 * (k + 1) + c);
    a5_st(zn, rA, so(lo12 && it == 1, zM + ob));  // (l from the second iteration on: already stored)
    a5_st(yn, rA, so(lo12, yM + ob));
    a5_st(xn, rA, so(!last1 || lo12, xT + 8u * (18 * (k + 1) + c)));
    a5_st(c == 0 ? xn16 + 0.0 : xn17 + 0.0, rA, so(!last1 && lo2, xT + 8u * (18 * (k + 1) + c16)));
    if (k == 0) {
      nx1 = xn;
      nx1h = make_double2(xn16, xn17);
      nz1 = zn;
      ny1 = yn;
    }
    hc = xt;
    A5_STAMP(8);
  };
  // an iteration's 2N steps (ring slot `slot` = the step count mod 3): forward k = s < N - 1, the
  // last forward step (s = N - 1), the backward sweep's start (s = N: xt_{N-1} = h_{N-1}, already in
  // hc), backward k = 2N - 1 - s; each segment a loop of its own (no per-step dispatch)
  int slot = 0;
  auto next = [&]() { slot = slot == 2 ? 0 : slot + 1; };
  for (; it <= a.A.max_iter; ++it) {
    for (int s = 0; s < N - 1; ++s) {
      begin(s, slot, c, c);
      if (it > 1 && s == 0) {
        v0 = nx0; hv0 = nx0h; z1 = nz1; y1 = ny1;
      }
      if (it > 1 && s == 1) {
        v0 = nx1; hv0 = nx1h;
      }
      fwd(s);
      next();
    }
    begin(N - 1, slot, cc, cc);
    if (it > 1 && N == 2) v0 = nx1;  // (N = 2: the last forward step is stage 1)
    fwd_last();
    next();
    begin(N, slot, cc, cc);
    next();
    for (int s = N + 1; s < 2 * N; ++s) {
      begin(s, slot, c, s == N + 1 ? cc : c + 0);
      bwd(2 * N - 1 - s);
      next();
    }
    // block 0's rows (z~ = I xt_0) and x_0
    {
      // (block 0 is the epilogue's alone: its state rides in registers across iterations)
      const double z0 = b0z, y0 = b0y, l0 = b0l, i0 = b0i, x0 = nx0, x016 = nx0h.x, x017 = nx0h.y;
      const double zt = __dmul_rn(i0, hc.lo);
      const double zr = __dadd_rn(__dmul_rn(al, zt), __dmul_rn(al1, z0));
      double zn = __dadd_rn(zr, __dmul_rn(ri, y0));
      zn = fmin(fmax(zn, l0), l0);
      const double yn = __dadd_rn(y0, __dmul_rn(rv, __dsub_rn(zr, zn)));
      const double xn = __dadd_rn(__dmul_rn(al, hc.lo), __dmul_rn(al1, x0));
      const double xn16 = __dadd_rn(__dmul_rn(al, hc.h16), __dmul_rn(al1, x016));
      const double xn17 = __dadd_rn(__dmul_rn(al, hc.h17), __dmul_rn(al1, x017));
      a5_st(zn, rA, so(lo12 && it == 1, zM + 8u * c));
      a5_st(yn, rA, so(lo12, yM + 8u * c));
      a5_st(xn, rA, so(true, xT + 8u * c));
      a5_st(c == 0 ? xn16 + 0.0 : xn17 + 0.0, rA, so(lo2, xT + 8u * c16));
      nx0 = xn;
      nx0h = make_double2(xn16, xn17);
      b0z = zn;
      b0y = yn;
      tk = __dmul_rn(rv, __dsub_rn(zn, __dmul_rn(ri, yn)));
      ibk = i0;
      hc = A4Vec{0.0, 0.0, 0.0};
    }
    const bool chk = a.A.check && it % a.A.check == 0;
    const bool adapt = ADAPT && a.A.adapt_interval && it % a.A.adapt_interval == 0;
    if (chk || adapt) {
      a5_drain();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      double rest = rho;
      const long bq = bown < P.B ? bown : bb;
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
          // ring is the factor's scratch)
          for (int q = 0; q < PW; ++q) {
            if (!((mv >> (16 * q)) & 0xffff)) continue;
            const long bq2 = bb + q;
            const double rq = __shfl(rho, 16 * q, 64);
            double* scr = ring;
            adm_factor(a, N, rq, a.Pq + bq2 * N * 36, a.Pd + bq2 * T, a.I + bq2 * m, a.R + bq2 * N * ADM_REC, scr,
                       scr + 30 * I7M_ADMM_FSTRIDE + 388, scr + 30 * I7M_ADMM_FSTRIDE, scr + 18 * I7M_ADMM_FSTRIDE,
                       scr + 2048, l);
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
          tk = __dmul_rn(rv, __dsub_rn(b0z, __dmul_rn(ri, b0y)));
          reload = true;
        }
      }
      if (!__ballot(run)) break;
      if (__ballot(fin)) {  // finished rows read nothing from here on
        offsets();
        vfull(1, true);  // (the running vector offsets: the last issued step's)
      }
      if (reload) {
        slot = 0;
        issue(0, 0, true);
        issue(1, 1, true);
      }
    }
  }
  a5_drain();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  // OSQP after max_iter without a passed test (oracle/osqp_admm.py OSQP.solve, :344-349): the test
  // once more at the final iterate unless the last iteration ran it, then the approximate test
  // (eps x 10): status 1 solved, 2 solved inaccurate, 0 max_iter reached.  The iterate is unchanged.
  int st_v = solved ? 1 : 0;
  if (__ballot(act && !solved)) {
    const long bq = bown < P.B ? bown : bb;
    auto test = [&](double es) {
      double rest = rho;
      return adm_check<16>(a, N, T, m, c_cost, rho, a.sx + bq * T, a.sz + bq * m, a.sy + bq * m, a.qs + bq * T,
                           a.ls + bq * m, a.D + bq * T, a.E + bq * m, a.R + bq * N * ADM_REC + REC_J, a.I + bq * m,
                           a.Pq + bq * N * 36, a.Pd + bq * T, &rest, c, es);
    };
    const bool last_checked = a.A.check && a.A.max_iter % a.A.check == 0;
    const bool exact = last_checked ? false : test(1.0);
    const bool approx = exact ? false : test(10.0);
    st_v = solved ? 1 : (exact ? 1 : (approx ? 2 : 0));
  }
#ifdef I7M_DIAG
  if (tr_on && l == 0 && g_tl) {
    unsigned long long* r = g_tl + 8 + 4 * (5ull << 16);
    for (int i = 0; i < 9; ++i) r[i] = tr_t[i];
    r[9] = (unsigned long long)a.ablate;
  }
#undef A5_STAMP
#endif
  if (c == 0 && act) {
    a.srho[bown] = rho;
    if (a.iters) a.iters[(long)bown * 8 + a.sqp_iter] = solved ? done_it : a.A.max_iter;
    if (a.status) a.status[(long)bown * 8 + a.sqp_iter] = st_v;
  }
  if (act) {
    const double* D = a.D + (long)bown * T;
    const double* xo = a.sx + (long)bown * T;
    double* so_ = a.sol + (long)bown * T;
    for (int e = c; e < T; e += 16) so_[e] = D[e] * xo[e];
  }
}

// ---- k_admm_iter_res: one problem per wave, everything it reads resident in LDS -------------
// The streaming kernel's step issues 13 (or 7) LDS-DMA wave-instructions and 2-4 buffer stores,
// and a lone wave's step is bound by their issue (tools/step_stamps.py: ~400 of ~1700 cycles for
// the DMA, ~70 per store).  A launch of at most a CU's worth of problems has the LDS for a better
// layout: one problem per workgroup, its N stage records (the streaming ring's image, 2.5 KB per
// stage) and its vectors x, q, h, z, y, l, I (0.8 KB per stage) copied into LDS once, the sweeps
// reading and writing LDS only (no DMA, no vector-memory wait in the loop), the vectors written
// back before each termination test (which reads global memory) and at the end.  All four 16-lane
// rows compute the problem (identical values to identical LDS addresses), so no lane is masked.
// The same operations in the same order as admm_iter4 (bit-identical: its register patches for
// data the ring loaded before the sweep wrote it read the same values from LDS here, except block
// 1's z, which the ring takes from l's lines after the first iteration, as here).  Horizons up to
// ARES_N (N = 32: 107 KB).
constexpr int ARES_N = 32;
__device__ __forceinline__ void a5_dma1(__amdgpu_buffer_rsrc_t r, unsigned lds, unsigned off) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %2, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(off), "s"(r)
      : "memory");
}
template <int NR>
__device__ __forceinline__ void admm_iter_res(const AdmmArgs& a) {
  const SolveParams& P = a.P;
  const int N = P.N, T = P.T, m = 12 * N;
  const int l = threadIdx.x, c = l & 15;
  const int b = a.b0 + (int)blockIdx.x;
  if (b >= P.B || (a.active && !a.active[b])) return;
  __shared__ double2 sRec2[NR * A5_LREC / 2];
  __shared__ double2 sV2[(3 * 18 + 4 * 12) * NR / 2 + 8];
  double* const sRec = (double*)sRec2;
  double* const sX = (double*)sV2;  // x | q | h (18 per stage) | z | y | l | I (12 per stage) | 16 spare
  double* const sQ = sX + 18 * NR;
  double* const sH = sQ + 18 * NR;
  double* const sZ = sH + 18 * NR;
  double* const sY = sZ + 12 * NR;
  double* const sL = sY + 12 * NR;
  double* const sI = sL + 12 * NR;
  double* const sJunk = sI + 12 * NR;  // stores of lanes that have none
  auto lds = [](const void* q) { return (unsigned)(unsigned long)(__attribute__((address_space(3))) const void*)q; };
  const auto rA = a4_rsrc(a.abase, a.abytes);
  auto boff = [&](const double* q) { return (unsigned)__builtin_amdgcn_readfirstlane((int)((const char*)q - (const char*)a.abase)); };
  const unsigned oX = boff(a.sx + (long)b * T), oQ = boff(a.qs + (long)b * T), oZ = boff(a.sz + (long)b * m);
  const unsigned oY = boff(a.sy + (long)b * m), oL = boff(a.ls + (long)b * m), oI = boff(a.I + (long)b * m);
  const unsigned oR = boff(a.R + (long)b * N * ADM_REC);
  // the stage records, in the ring's image (piece j of a stage from its HBM piece, zeros past a
  // row's stored width), and the vectors; the stage-N-1 tails of x and q (never used) zeroed
  {
    const int np = N * A5_RP;
    for (int g0 = 0; g0 < np; g0 += 64) {
      const int g = g0 + l, k = g / A5_RP, j = g - A5_RP * k;
      int hp;
      if (j < 80) {
        int r = 0;
#pragma unroll
        for (int i = 1; i < 16; ++i) r = 2 * j >= a5_lrow(i) ? i : r;
        const int cp = 2 * j - a5_lrow(r);
        hp = cp < adm_lw(r) ? (adm_lrow(r) + cp) / 2 : -1;
      } else {
        hp = j - 8;
      }
      a5_dma1(rA, lds(sRec) + 16u * g0, g < np && hp >= 0 ? oR + 8u * (unsigned)(k * ADM_REC) + 16u * hp : A5_OOB);
    }
    auto copy = [&](double* dst, unsigned src, int n) {  // n doubles (even)
      for (int g0 = 0; g0 < n / 2; g0 += 64) a5_dma1(rA, lds(dst) + 16u * g0, g0 + l < n / 2 ? src + 16u * (g0 + l) : A5_OOB);
    };
    copy(sX, oX, T);
    copy(sQ, oQ, T);
    copy(sZ, oZ, m);
    copy(sY, oY, m);
    copy(sL, oL, m);
    copy(sI, oI, m);
    if (l < 6) {
      sX[T + l] = 0.0;
      sQ[T + l] = 0.0;
    }
    a5_drain();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  // the vectors the termination test reads, back to global memory (every lane a different entry)
  auto flush = [&]() {
    for (int e = l; e < T; e += 64) a5_st(sX[e], rA, oX + 8u * e);
    for (int e = l; e < m; e += 64) {
      a5_st(sZ[e], rA, oZ + 8u * e);
      a5_st(sY[e], rA, oY + 8u * e);
    }
    a5_drain();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  };
  const double c_cost = a.cs[b];
  const double rho = a.srho[b], rv = 1e3 * rho, ri = 1.0 / rv;
  const double al = a.A.alpha, sg = a.A.sigma, al1 = 1.0 - al;
  const int cc = c < 12 ? c : 11;
  const bool lo12 = c < 12, lo2 = c < 2;
  double* const junk = sJunk + c;
  int it = 1;
  A4Vec hc{0.0, 0.0, 0.0};
  double b0z = sZ[cc], b0y = sY[cc], b0l = sL[cc], b0i = sI[cc];
  double nz1 = 0.0;
  // x_0 rides in registers from epilogue to epilogue, as in admm_iter4 (the same value as sX, but
  // the compiler's fusing of the epilogue's products into its sum follows where the operand comes
  // from: read from LDS there, x_0's update rounded differently in the last place)
  double nx0 = sX[c];
  double2 nx0h = make_double2(sX[16], sX[17]);
  double tk = __dmul_rn(rv, __dsub_rn(b0z, __dmul_rn(ri, b0y)));
  double ibk = b0i;
  int done_it = 0;
  bool solved = false;
  double v0, v1, z1, y1, l1, ib1;
  double2 hv0, hv1;
  A4CJ CJ;
  A4CL CL;
  A4CT CT;
  A4CR CR;
  const double* R = nullptr;
  // a step's operands: stage k's record, v0 / v1 (rows ci / cb) from the given vectors, block
  // k1's rows (z from l's lines after the first iteration), the first two coefficient sets
#ifdef I7M_DIAG
  // the step stamps of admm_iter4 (I7M_ABLATE 100000 + 100 IT + S; tools/step_stamps.py --res):
  // step start, its reads issued, right-hand side, Linv r, Linv' y, stores, end
  const int tr_it = a.ablate >= 100000 && a.ablate < 200000 ? (a.ablate - 100000) / 100 : -1, tr_s = a.ablate % 100;
  const bool tr_on = tr_it >= 0 && blockIdx.x == 0;
  unsigned long long tr_t[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  int tr_cur = -1;
#define AR_STAMP(i)                                                                         \
  do {                                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    unsigned long long v_;                                                                  \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v_)::"memory");             \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    if (tr_on && it == tr_it && tr_cur == tr_s) tr_t[i] = v_;                               \
  } while (0)
#else
#define AR_STAMP(i)
#endif
  auto begin = [&](int k, const double* V0, const double* V1, int k1, int ci, int cb) {
#ifdef I7M_DIAG
    tr_cur = k1 == k + 1 && V0 == sH + 18 * k ? 2 * N - 1 - k : k;
#endif
    AR_STAMP(0);
    R = sRec + A5_LREC * k;
    v0 = V0[ci];
    v1 = V1[cb];
    hv0 = make_double2(V0[16], V0[17]);
    hv1 = make_double2(V1[16], V1[17]);
    z1 = (it > 1 ? sL : sZ)[12 * k1 + cc];
    y1 = sY[12 * k1 + cc];
    l1 = sL[12 * k1 + cc];
    ib1 = sI[12 * k1 + cc];
    a4_ldj(CJ, R, c);
    a4_ldl(CL, R, R + a5_lrow(c), c);
    AR_STAMP(1);
  };
  auto llt = [&](const A4Vec& r, bool jr) {
    AR_STAMP(2);
    a4_ldt(CT, R, c);
    const A4Vec y = a4_lmul(CL, r);
    AR_STAMP(3);
    if (jr) a4_ldr(CR, R, c);
    const A4Vec o = a4_ltmul(CL, CT, y);
    AR_STAMP(4);
    return o;
  };
  for (; it <= a.A.max_iter; ++it) {
    // forward steps k < N - 1
    for (int k = 0; k < N - 1; ++k) {
      begin(k, sX + 18 * k, sQ + 18 * k, k + 1, c, c);
      if (it > 1 && k == 0) z1 = nz1;
      const double t1 = __dmul_rn(rv, __dsub_rn(z1, __dmul_rn(ri, y1)));
      const double init = lo12 ? __dmul_rn(ibk, tk) : 0.0;
      A4Vec r = a4_jtmul(CJ, t1, A4Vec{init, 0.0, 0.0});
      r.lo = __dadd_rn(__dsub_rn(__dmul_rn(sg, v0), v1), r.lo);
      r.h16 = __dadd_rn(__dsub_rn(__dmul_rn(sg, hv0.x), hv1.x), r.h16);
      r.h17 = __dadd_rn(__dsub_rn(__dmul_rn(sg, hv0.y), hv1.y), r.h17);
      const double rc = __dsub_rn(r.lo, __dmul_rn(__dmul_rn(rv, ibk), hc.lo));
      r.lo = lo12 ? rc : r.lo;
      const A4Vec h = llt(r, true);
      double* const H = sH + 18 * k;
      H[c] = h.lo;
      *(lo2 ? H + 16 + c : junk) = c == 0 ? h.h16 : h.h17;
      AR_STAMP(5);
      hc.lo = a4_jmul(CR, c, h);
      tk = t1;
      ibk = ib1;
      AR_STAMP(6);
    }
    // the last forward step (12 rows, no J, no u-part): xt_{N-1} = h_{N-1}, kept in registers
    {
      const int k = N - 1;
      begin(k, sX + 18 * k, sQ + 18 * k, k, cc, cc);
      A4Vec r{lo12 ? __dmul_rn(ibk, tk) : 0.0, 0.0, 0.0};
      r.lo = __dadd_rn(__dsub_rn(__dmul_rn(sg, v0), v1), r.lo);
      r.lo = __dsub_rn(r.lo, __dmul_rn(__dmul_rn(rv, ibk), hc.lo));
      r.lo = lo12 ? r.lo : 0.0;
      hc = llt(r, false);
    }
    // backward steps k = N - 2 .. 0: xt_k, then block k+1's rows and x_{k+1}
    for (int k = N - 2; k >= 0; --k) {
      const bool last1 = k + 1 == N - 1;  // x_{k+1} has no u-part
      begin(k, sH + 18 * k, sX + 18 * (k + 1), k + 1, c, last1 ? cc : c);
      const double u = __dmul_rn(__dmul_rn(rv, ib1), hc.lo);
      const A4Vec s2 = llt(a4_jtmul(CJ, u, A4Vec{0.0, 0.0, 0.0}), true);
      const A4Vec xt{__dsub_rn(v0, s2.lo), __dsub_rn(hv0.x, s2.h16), __dsub_rn(hv0.y, s2.h17)};
      const double zt = __dadd_rn(a4_jmul(CR, c, xt), __dmul_rn(ib1, hc.lo));
      AR_STAMP(5);
      const double zr = __dadd_rn(__dmul_rn(al, zt), __dmul_rn(al1, z1));
      double zn = __dadd_rn(zr, __dmul_rn(ri, y1));
      zn = fmin(fmax(zn, l1), l1);
      const double yn = __dadd_rn(y1, __dmul_rn(rv, __dsub_rn(zr, zn)));
      const double xn = __dadd_rn(__dmul_rn(al, hc.lo), __dmul_rn(al1, v1));
      const double xn16 = __dadd_rn(__dmul_rn(al, hc.h16), __dmul_rn(al1, hv1.x));
      const double xn17 = __dadd_rn(__dmul_rn(al, hc.h17), __dmul_rn(al1, hv1.y));
      const int ob = 12 * (k + 1);
      *(lo12 && it == 1 ? sZ + ob + c : junk) = zn;
      *(lo12 ? sY + ob + c : junk) = yn;
      double* const X1 = sX + 18 * (k + 1);
      *(!last1 || lo12 ? X1 + c : junk) = xn;
      *(!last1 && lo2 ? X1 + 16 + c : junk) = c == 0 ? xn16 : xn17;
      if (k == 0) nz1 = zn;
      hc = xt;
      AR_STAMP(6);
    }
    // block 0's rows (z~ = I xt_0) and x_0
    {
      const double x0 = nx0, x016 = nx0h.x, x017 = nx0h.y;
      const double zt = __dmul_rn(b0i, hc.lo);
      const double zr = __dadd_rn(__dmul_rn(al, zt), __dmul_rn(al1, b0z));
      double zn = __dadd_rn(zr, __dmul_rn(ri, b0y));
      zn = fmin(fmax(zn, b0l), b0l);
      const double yn = __dadd_rn(b0y, __dmul_rn(rv, __dsub_rn(zr, zn)));
      const double xn = __dadd_rn(__dmul_rn(al, hc.lo), __dmul_rn(al1, x0));
      const double xn16 = __dadd_rn(__dmul_rn(al, hc.h16), __dmul_rn(al1, x016));
      const double xn17 = __dadd_rn(__dmul_rn(al, hc.h17), __dmul_rn(al1, x017));
      *(lo12 && it == 1 ? sZ + c : junk) = zn;
      *(lo12 ? sY + c : junk) = yn;
      sX[c] = xn;
      *(lo2 ? sX + 16 + c : junk) = c == 0 ? xn16 : xn17;
      nx0 = xn;
      nx0h = make_double2(xn16, xn17);
      b0z = zn;
      b0y = yn;
      tk = __dmul_rn(rv, __dsub_rn(zn, __dmul_rn(ri, yn)));
      ibk = b0i;
      hc = A4Vec{0.0, 0.0, 0.0};
    }
    if (a.A.check && it % a.A.check == 0) {
      flush();
      double rest = rho;
      const bool ok = adm_check<16>(a, N, T, m, c_cost, rho, a.sx + (long)b * T, a.sz + (long)b * m, a.sy + (long)b * m,
                                    a.qs + (long)b * T, a.ls + (long)b * m, a.D + (long)b * T, a.E + (long)b * m,
                                    a.R + (long)b * N * ADM_REC + REC_J, a.I + (long)b * m, a.Pq + (long)b * N * 36,
                                    a.Pd + (long)b * T, &rest, c);
      if (ok) {
        solved = true;
        done_it = it;
        break;
      }
    }
  }
  if (!solved) flush();
  // OSQP's closing tests after max_iter (as admm_iter4)
  int st_v = solved ? 1 : 0;
  if (!solved) {
    auto test = [&](double es) {
      double rest = rho;
      return adm_check<16>(a, N, T, m, c_cost, rho, a.sx + (long)b * T, a.sz + (long)b * m, a.sy + (long)b * m,
                           a.qs + (long)b * T, a.ls + (long)b * m, a.D + (long)b * T, a.E + (long)b * m,
                           a.R + (long)b * N * ADM_REC + REC_J, a.I + (long)b * m, a.Pq + (long)b * N * 36,
                           a.Pd + (long)b * T, &rest, c, es);
    };
    const bool last_checked = a.A.check && a.A.max_iter % a.A.check == 0;
    const bool exact = last_checked ? false : test(1.0);
    const bool approx = exact ? false : test(10.0);
    st_v = exact ? 1 : (approx ? 2 : 0);
  }
#ifdef I7M_DIAG
  if (tr_on && l == 0 && g_tl) {
    unsigned long long* r = g_tl + 8 + 4 * (5ull << 16);
    for (int i = 0; i < 9; ++i) r[i] = tr_t[i];
    r[9] = (unsigned long long)a.ablate;
    r[10] = 1;  // the resident kernel's stamp layout
  }
#undef AR_STAMP
#endif
  if (l == 0) {
    a.srho[b] = rho;
    if (a.iters) a.iters[(long)b * 8 + a.sqp_iter] = solved ? done_it : a.A.max_iter;
    if (a.status) a.status[(long)b * 8 + a.sqp_iter] = st_v;
  }
  const double* D = a.D + (long)b * T;
  double* so_ = a.sol + (long)b * T;
  for (int e = l; e < T; e += 64) so_[e] = D[e] * sX[e];
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
#ifndef I7M_ADMM_PREP_ONLY  // (i7m_admm_prep_tu.hip: no copies of the iteration kernels)
// two problems per wave (grid = ceil(problems / 2)): a 21 KB ring, two waves per SIMD possible.  Per
// problem the same arithmetic (bit-identical); a step issues 7 DMA wave-instructions instead of 13,
// so a wave's step is shorter when the batch is small (launches of <= 512 problems use it), while
// at B = 4096 the doubled instruction count per problem costs more than the second wave hides
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2))) k_admm_iter2(AdmmArgs a) {
  admm_iter4<false, 2>(a);
}
// one problem per workgroup, records and vectors resident in LDS (grid = problems; N <= ARES_N)
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1))) k_admm_iter_res(AdmmArgs a) {
  admm_iter_res<ARES_N>(a);
}
#endif

}  // namespace i7m
