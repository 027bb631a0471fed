// i7m_kernels.h — the batched SQP-MPC kernels (gfx950, fp64).
//
// One SQP iteration of src/osqp_sqp.py:76-93 for B independent problems is three launches:
//
//   k_linearize   (i7m_linearize.h) six lanes per knot: analytic world-frame derivatives of
//                 the dynamics + cost linearisation.  Replaces src/osqp_solver.py:70-135.
//   k_riccati_mfma (i7m_riccati_mfma.h) one wavefront per problem: exact solve of the
//                 equality-constrained QP (src/osqp_solver.py:137-143), Riccati recursion.
//   k_linesearch  one wavefront per problem, lanes = (candidate alpha, knot): merit of the
//                 base point and of the backtracking alphas, several candidates per round,
//                 first-accept rule of src/osqp_sqp.py:58-72, then the SQP step, step-size
//                 norm and break test (src/osqp_sqp.py:79-91).
#pragma once

#include <cstddef>

#include "i7m_dynamics.h"
#include "i7m_indy7_model.h"
#include "i7m_sincos.h"

namespace i7m {

constexpr int LIN_STRIDE = 114;   // Aq(36) Av(36) Bu(36) a(6)
constexpr int COST_STRIDE = 10;   // j(6) Qm dQm Rm |e|
constexpr int KBUF_STRIDE = 84;   // K(6x12) kff(6) c_v(6)
// per-knot QP record written by k_linearize for k_riccati_mfma (knots 0..N-2)
constexpr int QPD_STRIDE = 32;
constexpr int QPD_CV = 0;    // c_v (6): dynamics offset of the v rows
constexpr int QPD_LX = 6;    // linear state terms (12): Qm j | dQm v
constexpr int QPD_LU = 18;   // linear control terms (6): Rm u
constexpr int QPD_J = 24;    // j = J^T e (6): the rank-1 factor of the q block
constexpr int QPD_DQM = 30;  // dQm
constexpr int QPD_RM = 31;   // Rm
constexpr int NALPHA = 8;
constexpr int MAXN = 64;

struct SolveParams {
  int N, T, B, goal_stride, regularize, max_iters;
  double dt, dQ, R, QN, eps, mu, step_tol;
};

struct ProblemStats {
  int qp_iters, n_alphas, n_steps, pad;
  double alphas[8];
  double stepsizes[8];
};

__device__ __forceinline__ void sincos6(const double* q, double c[6], double s[6]) {
#pragma unroll
  for (int i = 0; i < 6; ++i) sincos_q(q[i], &s[i], &c[i]);
}

// ---------------------------------------------------------------------------------------
// Cost linearisation of knot k (src/osqp_solver.py:103-135): writes j = J^T e, Qm, dQm, Rm.
__device__ __forceinline__ void cost_knot(const DevModel& Md, const SolveParams& P, const double* q,
                                          const double* goal, int k, double* out) {
  double c[6], s[6], p[3], J[3][6];
  sincos6(q, c, s);
  fk_jac(Md, c, s, p, J);
  const double e0 = p[0] - goal[0], e1 = p[1] - goal[1], e2 = p[2] - goal[2];
  const double nrm = sqrt(e0 * e0 + e1 * e1 + e2 * e2);
  const double w = P.regularize ? (1.0 / (fabs(nrm) + P.eps)) : 1.0;
#pragma unroll
  for (int j = 0; j < 6; ++j) out[j] = e0 * J[0][j] + e1 * J[1][j] + e2 * J[2][j];
  out[6] = (k == P.N - 1) ? P.QN : 1.0;
  out[7] = P.dQ * w;
  out[8] = P.R * w;
  out[9] = nrm;
}

// ---------------------------------------------------------------------------------------
// Merit pieces of one knot (src/osqp_sqp.py:13-47): qcost, vcost, ucost, integrator error.
// x: 18 values of knot k (12 at the last knot), xn: the 12 state values of knot k+1.
__device__ __forceinline__ void merit_knot(const DevModel& Md, const SolveParams& P, int k, const double* x,
                                           const double* xn, const double* goal, const double* f6, bool fw,
                                           double out[4]) {
  double c[6], s[6], p[3];
  sincos6(x, c, s);
  fk_jac(Md, c, s, p, nullptr);
  const double e0 = p[0] - goal[0], e1 = p[1] - goal[1], e2 = p[2] - goal[2];
  const double Qm = (k == P.N - 1) ? P.QN : 1.0;
  out[0] = Qm * (e0 * e0 + e1 * e1 + e2 * e2);
  double vv = 0.0;
#pragma unroll
  for (int i = 0; i < 6; ++i) vv += x[6 + i] * x[6 + i];
  out[1] = P.dQ * vv;
  out[2] = 0.0;
  out[3] = 0.0;
  if (k < P.N - 1) {
    double uu = 0.0;
#pragma unroll
    for (int i = 0; i < 6; ++i) uu += x[12 + i] * x[12 + i];
    out[2] = P.R * uu;
    double L[6][6], a[6], fl[6];
    if (fw && f6) {
      wrench_world_to_local(Md, c, s, f6, fl);
      f6 = fl;
    }
    forward_dynamics(Md, c, s, x + 6, x + 12, f6, L, a);
    double eq = 0.0, ev = 0.0;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const double dq = (x[i] + x[6 + i] * P.dt) - xn[i];
      const double dv = (x[6 + i] + a[i] * P.dt) - xn[6 + i];
      eq += dq * dq;
      ev += dv * dv;
    }
    out[3] = sqrt(eq) + sqrt(ev);
  }
}

// Line search (+ step) — one wavefront per problem.  Candidates: 0 = base point (merit of XU
// itself, src/osqp_sqp.py:52-55), 1..8 = alphas 1, 1/2, ..., 1/128.  R = max(1, 64/N)
// candidates per round; the first accepted candidate in alpha order wins (identical to the
// sequential loop).  mode 0: apply step + stats + break flag; mode 1: only output alpha; mode 2: as
// 0 for a QP solver that carries state between calls (I7M_QP_ADMM): alpha = 0 records this
// iteration only, and the next iteration re-solves (src/osqp_sqp.py:81-82 `continue`; OSQP's
// warm start makes the re-solve differ).
// With lin / cost (the k_linearize outputs at this XU) the base merit is assembled from them —
// a = ABA(q, v, u) and |e| of every knot are already there — so no round evaluates candidate 0.
// SPEC: Indy7 constants baked in (kIndy7Model, generated from the URDF) instead of read from Mg.
// k_linesearch register budget: 2 waves/SIMD (<= 256 VGPRs) with the forces of
// links 0..2 parked in LDS and XU / sol staged in LDS: 18.3 KB LDS per wave at N = 32, i.e. 8
// waves per CU.  Measured 151 -> 132 us (1 wave/SIMD before); now ~236 VGPRs, no VGPR spill
// (the ~120 SGPRs the baked constants need spill to VGPR lanes: ~6 % of the round's VALU).
constexpr int LS_NLDS = 3;  // links whose RNEA forces k_linesearch parks in LDS
// per-wave LDS parking of k_linesearch (RNEA forces; the non-power-of-2 reduction reuses it)
constexpr int LS_PARK = 6 * LS_NLDS * 64 > 256 ? 6 * LS_NLDS * 64 : 256;
// dynamic LDS of k_linesearch for trajectory length T and W waves per problem
inline size_t ls_lds_bytes(int T, int W = 1) { return sizeof(double) * (size_t)(2 * T + W * LS_PARK); }
// A trajectory entry staged for the line search: XU and the QP step sol - XU side by side, so
// a line-search point x + al d is one 16-byte LDS read.
struct alignas(16) XD {
  double x, d;
};

// Merit terms of one (candidate, knot) lane of k_linesearch: qcost, vcost, ucost and the
// integrator error (src/osqp_sqp.py:13-47) at the line-search point XU + al (sol - XU)
// (src/osqp_sqp.py:60), from the LDS copies of XU / sol; the knot values are re-read from LDS
// where used instead of being held in registers across the dynamics, each group of reads issued
// ahead of its arithmetic.  (As a separate inlined function the kernel allocates spill-free;
// written in the round loop it spilled, 115 -> 110 us.)
// FW: f6 is a world-frame wrench, converted to joint 6's frame at this knot's configuration.
// I7M_LS_NOSEL (default 1): the base point (candidate 0, al = 0) is XU + 0 (sol - XU), equal to XU
// for every finite step entry but for the sign of an exact zero, so the point values need no
// per-value select between x and x + al d (two v_cndmask per value, ~100 per evaluation); the
// base merit of the SQP loop comes from the linearisation anyway, candidate 0 is evaluated only
// without it.
#ifndef I7M_LS_NOSEL
#define I7M_LS_NOSEL 1
#endif
__device__ __forceinline__ double ls_pick(bool base_pt, double x, double v) { return (I7M_LS_NOSEL || !base_pt) ? v : x; }
template <bool SPEC, bool FW = false>
__device__ __forceinline__ void ls_merit_terms(const DevModel* __restrict__ Mg, const SolveParams& P, const int k,
                                                      const bool last, const bool base_pt, const double al,
                                                      const XD* sXD, const double* goal,
                                                      const double* f6, double* fpark, double* o) {
  const DevModel& Md = SPEC ? kIndy7Model : *Mg;
  const int ok = 18 * k, on = 18 * (last ? k : k + 1);
  // both halves of the pair in one 16-byte read and a select (written as `base_pt ? x : x + al d`
  // the compiler made the d read a branch of its own, serialising every knot value's LDS reads)
  auto val = [&](int e) -> double {
    const XD p = sXD[e];
    const double v = p.x + al * p.d;
    return ls_pick(base_pt, p.x, v);
  };
  double c[6], sn[6], pe[3];
  {
    double q[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) q[i] = val(ok + i);
    sincos6(q, c, sn);
  }
  fk_pos(Md, c, sn, pe);
  const double e0 = pe[0] - goal[0], e1 = pe[1] - goal[1], e2 = pe[2] - goal[2];
  o[0] = (last ? P.QN : 1.0) * (e0 * e0 + e1 * e1 + e2 * e2);
  double vv = 0.0, uu = 0.0;
  double v[6], u[6];
  {
    // the knot's v and u pairs: all 12 reads issued before their arithmetic
    XD pv[6], pu[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      pv[i] = sXD[ok + 6 + i];
      pu[i] = sXD[last ? ok + 6 + i : ok + 12 + i];  // (the last knot has no u: unused)
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const double vi = pv[i].x + al * pv[i].d, ui = pu[i].x + al * pu[i].d;
      v[i] = ls_pick(base_pt, pv[i].x, vi);
      u[i] = ls_pick(base_pt, pu[i].x, ui);
      vv += v[i] * v[i];
    }
  }
  o[1] = P.dQ * vv;
  if (!last) {
    double L[6][6], a[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) uu += u[i] * u[i];
    o[2] = P.R * uu;
    if (FW && f6) {
      double fl[6];
      wrench_world_to_local(Md, c, sn, f6, fl);
      forward_dynamics<LS_NLDS>(Md, c, sn, v, u, fl, L, a, fpark);
    } else {
      forward_dynamics<LS_NLDS>(Md, c, sn, v, u, f6, L, a, fpark);
    }
    asm volatile("" ::: "memory");  // re-read the knot values from LDS below
    // the knot values in two halves of 12 LDS pair reads, each half issued before its
    // arithmetic (interleaved with it, the scheduler reused one register set and waited on each
    // read in turn)
    double eq = 0.0, ev = 0.0;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      XD pq[3], pv[3], pn[3], pw[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        pq[i] = sXD[ok + 3 * hf + i];
        pv[i] = sXD[ok + 6 + 3 * hf + i];
        pn[i] = sXD[on + 3 * hf + i];
        pw[i] = sXD[on + 6 + 3 * hf + i];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        auto pt = [&](const XD& p) {
          const double v = p.x + al * p.d;
          return ls_pick(base_pt, p.x, v);
        };
        const double xq = pt(pq[i]), xv = pt(pv[i]), nq = pt(pn[i]), nv = pt(pw[i]);
        const double dq = (xq + xv * P.dt) - nq;
        const double dv = (xv + a[3 * hf + i] * P.dt) - nv;
        eq += dq * dq;
        ev += dv * dv;
      }
    }
    o[3] = sqrt(eq) + sqrt(ev);
  }
}

// Line search in two launches (I7M_LS_TAIL): the first launch evaluates the
// candidates below c_end only; a problem none of them accepts stores its base merit, raises
// pending[b] and leaves XU, the stats and the break flag to the second launch, which evaluates
// the rest (c_begin on, base merit from `base`) with several waves per problem.  The candidates'
// merits and the first-accept rule are those of the one-launch search, so alphas are identical.
struct LsSplit {
  int c_begin = 0;            // first candidate of this launch (0: the whole search, base first)
  int c_end = 1 + NALPHA;     // candidates [.., c_end) in this launch
  double* base = nullptr;     // (B) base merits handed from the first launch to the second
  int* pending = nullptr;     // (B) 1: the second launch finishes this problem
};

// k_linesearch's kernel arguments as laid out in its kernarg segment (the parameters in order,
// each at its natural alignment: the C layout of this struct).  With KA, linesearch_body reads the
// parameters it needs in a round, and everything it needs after the rounds, from there through a
// laundered scalar pointer (re-loaded by s_load where used) instead of holding them in SGPRs across
// the candidate rounds, where the baked model's constants already fill the SGPR file and the rest
// spilled into VGPR lanes (v_writelane / v_readlane, VALU instructions, in every round).
struct LsKernArgs {
  const DevModel* Mg;
  SolveParams P;
  const double* xu;
  double* xu_out;
  const double* sol;
  const double* goals;
  const double* fext;
  int* active;
  ProblemStats* stats;
  double* alpha_out;
  int iter, mode;
  const double* lin;
  const double* cost;
  LsSplit sp;
};
static_assert(offsetof(LsKernArgs, P) == 8 && offsetof(LsKernArgs, xu) == 88 && offsetof(LsKernArgs, iter) == 152 &&
                  offsetof(LsKernArgs, lin) == 160 && offsetof(LsKernArgs, sp) == 176 && sizeof(LsKernArgs) == 200,
              "LsKernArgs must mirror k_linesearch's kernarg layout (code object metadata: P 8, xu 88, iter 152, "
              "lin 160, sp 176)");
__device__ __forceinline__ const LsKernArgs* kernarg_ls() {
  auto p = __builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return (const LsKernArgs*)p;
}

// W waves per problem (small batches, where the GPU is otherwise idle): wave w evaluates the
// candidate slots c0 + w R .. c0 + w R + R - 1 of each round, so W R candidates per round (all
// eight alphas in one round at N = 32, W = 4).  Same first-accept rule, same merits.
// FW: fext is a world-frame wrench (I7M_WRENCH_WORLD), see ls_merit_terms.
// The line search of problem b by the W waves of a workgroup (wave w, lane l): the body of
// k_linesearch, and the third phase of each SQP iteration of k_sqp_fused.  ls_dyn: the dynamic
// LDS of ls_lds_bytes(T, W); merit: 9 doubles of LDS.
// LDS ordering inside the line search: with one wave per problem (W = 1) its LDS instructions
// execute in order, so a compiler barrier is enough (I7M_LS_WSYNC 1); with W waves, lds_sync.
#ifndef I7M_LS_WSYNC
#define I7M_LS_WSYNC 1
#endif
template <int W>
__device__ __forceinline__ void ls_sync() {
  if constexpr (W == 1 && I7M_LS_WSYNC) __asm__ volatile("" ::: "memory");
  else lds_sync();
}
template <bool SPEC, int ABL = 0, int W = 1, bool FW = false, bool KA = false>
__device__ __forceinline__ void linesearch_body(const DevModel* __restrict__ Mg, const SolveParams& P, const int b,
                                                const int w, const int l, double* __restrict__ ls_dyn,
                                                double* __restrict__ merit, const double* xu, double* xu_out,
                                                const double* __restrict__ sol, const double* __restrict__ goals,
                                                const double* __restrict__ fext, int* __restrict__ active,
                                                ProblemStats* __restrict__ stats, double* __restrict__ alpha_out,
                                                int iter, int mode, const double* __restrict__ lin,
                                                const double* __restrict__ cost, const LsSplit sp = LsSplit{}) {
  const int N = P.N;
  const int R = (N >= 64) ? 1 : 64 / N;
  const int slot = l / N;
  const int k = l - slot * N;
  const DevModel& Md = SPEC ? kIndy7Model : *Mg;
  const double* X = xu + (long)b * P.T;
  double* XO = xu_out + (long)b * P.T;  // the updated XU (may be X itself)
  const double* S = sol + (long)b * P.T;
  // the problem's XU and QP minimiser, staged once in LDS for every round
  // dynamic LDS (ls_lds_bytes): (XU, sol - XU) pairs (T) | RNEA link-force parking (rnea NLDS), which
  // also holds the non-power-of-2 reduction (a different phase of each round)
  XD* sXD = reinterpret_cast<XD*>(ls_dyn);
  double* fpark = ls_dyn + 2 * P.T + w * LS_PARK;
  double (*part)[4] = reinterpret_cast<double (*)[4]>(fpark);
  int step_nz = 0;  // does this lane stage a nonzero step entry sol - XU?
  {
    // chunks of 6 entries per lane with every load issued before the first use (the plain loop
    // waited out a global-memory round trip per entry: ~9 per wave at N = 32)
    constexpr int SU = 6;
    for (int e0 = 64 * w + l; e0 < P.T; e0 += 64 * W * SU) {
      double xv[SU], sv[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int e = min(e0 + 64 * W * u, P.T - 1);
        xv[u] = X[e];
        sv[u] = S[e];
      }
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int e = e0 + 64 * W * u;
        if (e < P.T) {
          const double d = sv[u] - xv[u];
          sXD[e] = XD{xv[u], d};
          step_nz |= (d != 0.0);
        }
      }
    }
  }
  const double alphas[NALPHA] = {1.0, 0.5, 0.25, 0.125, 0.0625, 0.03125, 0.015625, 0.0078125};
  const bool pow2 = (N & (N - 1)) == 0;
  const double* goal = goals + (long)b * N * P.goal_stride + (long)(k < N ? k : 0) * P.goal_stride;
  const double* f6 = fext ? fext + 6L * b : nullptr;
  // A step of exactly zero (sol == XU): every candidate point IS XU, so the reference's
  // merit_new equals basemerit bit for bit and alpha = 1 is accepted (src/osqp_sqp.py:58-72).
  // Decided here, not by comparing merits, because the base merit below comes from the
  // linearisation and rounds differently from the candidate evaluation.
  bool zero_step;
  if constexpr (W == 1 && I7M_LS_WSYNC) {
    zero_step = __ballot(step_nz) == 0;
    ls_sync<W>();
  } else {
    zero_step = __syncthreads_or(step_nz) == 0;
  }
  // sum the N knot terms of each candidate slot and store the merit of candidate c0 + slot
  // (c0 already offset by this wave's share of the round; `store` false: compute only)
  double mu_r = P.mu;  // (KA: re-read per round)
  auto reduce_store = [&](double o[4], int c0, bool store) {
    if (pow2) {
      // tree-sum the N knots of each candidate slot with shuffles (segments of width N); the
      // four terms' shuffles of one level are issued together (one LDS round trip per level)
      for (int off = N >> 1; off >= 1; off >>= 1) {
        double t[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) t[j] = __shfl_xor(o[j], off, 64);
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] += t[j];
      }
      if (store && k == 0 && slot < R && c0 + slot < 1 + NALPHA) merit[c0 + slot] = o[0] + o[1] + o[2] + mu_r * o[3];
    } else {
      part[l][0] = o[0]; part[l][1] = o[1]; part[l][2] = o[2]; part[l][3] = o[3];
      ls_sync<W>();
      if (store && l < R && c0 + l < 1 + NALPHA) {
        double qc = 0.0, vc = 0.0, uc = 0.0, cv = 0.0;
        for (int kk = 0; kk < N; ++kk) {
          qc += part[l * N + kk][0];
          vc += part[l * N + kk][1];
          uc += part[l * N + kk][2];
          cv += part[l * N + kk][3];
        }
        merit[c0 + l] = qc + vc + uc + mu_r * cv;
      }
    }
    ls_sync<W>();
  };
  int cstart = 0;
  if (sp.c_begin > 0) {
    // the second launch of a split search: base merit from the first
    if (l == 0 && w == 0) merit[0] = sp.base[b];
    ls_sync<W>();
    cstart = sp.c_begin;
  } else if (lin && !zero_step) {
    // base merit (src/osqp_sqp.py:52-55) from the linearisation of this XU: |e| (cost[9]) and
    // a = ABA(q, v, u) (lin[108..113]) per knot; slot 0 of the candidate layout
    const double* LB = lin + (long)b * (N - 1) * LIN_STRIDE;
    const double* CB = cost + (long)b * N * COST_STRIDE;
    double o[4] = {0.0, 0.0, 0.0, 0.0};
    if (slot == 0 && k < N) {
      const bool last = (k == N - 1);
      const int ok = 18 * k, on = 18 * (last ? k : k + 1);
      const double nrm = CB[k * COST_STRIDE + 9];
      o[0] = CB[k * COST_STRIDE + 6] * (nrm * nrm);
      double vv = 0.0, uu = 0.0, eq = 0.0, ev = 0.0;
#pragma unroll
      for (int i = 0; i < 6; ++i) vv += sXD[ok + 6 + i].x * sXD[ok + 6 + i].x;
      o[1] = P.dQ * vv;
      if (!last) {
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          uu += sXD[ok + 12 + i].x * sXD[ok + 12 + i].x;
          const double dq = (sXD[ok + i].x + sXD[ok + 6 + i].x * P.dt) - sXD[on + i].x;
          const double dv = (sXD[ok + 6 + i].x + LB[k * LIN_STRIDE + 108 + i] * P.dt) - sXD[on + 6 + i].x;
          eq += dq * dq;
          ev += dv * dv;
        }
        o[2] = P.R * uu;
        o[3] = sqrt(eq) + sqrt(ev);
      }
    }
    reduce_store(o, 0, w == 0);
    cstart = 1;
  }
  double base = 0.0;
  int found = zero_step ? 1 : -1;
  const int c_end = sp.c_end < 1 + NALPHA ? sp.c_end : 1 + NALPHA;
  for (int c0 = cstart; c0 < c_end && found < 0; c0 += R * W) {
    if (I7M_PRIO & 2) set_prio((c0 - cstart) / (R * W));  // later rounds first: the longest searches
    const int cw = c0 + w * R;  // this wave's first candidate of the round
    const int cand = cw + slot;
    const LsKernArgs* KR = KA ? kernarg_ls() : nullptr;
    const SolveParams& PR = KA ? KR->P : P;
    if (KA) mu_r = PR.mu;
    const double* f6r = KA ? (KR->fext ? KR->fext + 6L * b : nullptr) : f6;
    double o[4] = {0.0, 0.0, 0.0, 0.0};
    if (slot < R && k < N && cand < 1 + NALPHA) {
      // merit terms of (candidate, knot k): the knot values are recomputed from the LDS copy of
      // XU / sol where they are used instead of being held in registers across the dynamics
      // (the line-search point XU + al (sol - XU), src/osqp_sqp.py:60)
      const bool last = (k == N - 1);
      const bool base_pt = (cand == 0);
      const double al = base_pt ? 0.0 : alphas[cand - 1];
      const int ok = 18 * k, on = 18 * (last ? k : k + 1);
      auto val = [&](int e) -> double {
        const XD p = sXD[e];
        const double v = p.x + al * p.d;
        return ls_pick(base_pt, p.x, v);
      };
      if (ABL == 1) {  // diagnostic timing build: dynamics replaced by trivial math
        o[0] = val(ok) * val(ok + 1); o[1] = val(ok + 6) * val(ok + 6); o[2] = val(ok + 12) * val(on);
        o[3] = val(on + 6) + val(ok + 11);
      } else {
        ls_merit_terms<SPEC, FW>(Mg, PR, k, last, base_pt, al, sXD, goal, f6r, fpark + l, o);
      }
      if (k == 0 && cand > 0) {
        // + |XU_new[:12] - XU[:12]|   (src/osqp_sqp.py:63)
        double dd = 0.0;
        XD p0[12];
#pragma unroll
        for (int i = 0; i < 12; ++i) p0[i] = sXD[i];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 12; ++i) {
          const double vi = p0[i].x + al * p0[i].d;
          const double t = ls_pick(base_pt, p0[i].x, vi) - p0[i].x;
          dd += t * t;
        }
        o[3] += sqrt(dd);
      }
    }
    reduce_store(o, cw, true);
    base = merit[0];
    for (int cc = (c0 == 0 ? 1 : c0); cc < c0 + R * W && cc < c_end; ++cc) {
      if (merit[cc] <= base) { found = cc; break; }
    }
    ls_sync<W>();
  }
  // (KA: everything below from the kernarg segment, not held across the rounds)
  const LsKernArgs* KE = KA ? kernarg_ls() : nullptr;
  const SolveParams& PE = KA ? KE->P : P;
  const LsSplit spE = KA ? KE->sp : sp;
  if (spE.pending) {
    // first launch of a split search: hand an unresolved problem to the second launch
    const int pend = (found < 0 && c_end < 1 + NALPHA) ? 1 : 0;
    if (l == 0 && w == 0) {
      spE.pending[b] = pend;
      if (pend) spE.base[b] = merit[0];
    }
    if (pend) return;
  }
  if (W > 1 && w != 0) return;  // one wave applies the step
  const double alpha = (found > 0) ? alphas[found - 1] : 0.0;
  const int modeE = KA ? KE->mode : mode, iterE = KA ? KE->iter : iter;
  if (modeE == 1) {
    if (l == 0) (KA ? KE->alpha_out : alpha_out)[b] = alpha;
    return;
  }
  ProblemStats* st = (KA ? KE->stats : stats) + b;
  int* const actE = KA ? KE->active : active;
  const double* XE = KA ? KE->xu + (long)b * PE.T : X;
  double* XOE = KA ? KE->xu_out + (long)b * PE.T : XO;
  if (alpha == 0.0) {
    // src/osqp_sqp.py:81-82: `continue` re-solves the SAME QP from the same XU; the exact
    // solve is deterministic, so every remaining iteration repeats alpha = 0.  A stateful QP
    // solver (mode 2) re-solves from its new state: this iteration only.
    if (l == 0) {
      if (modeE == 2) {
        st->alphas[st->n_alphas++] = 0.0;
        st->qp_iters = iterE + 1;
        if (iterE + 1 >= PE.max_iters) actE[b] = 0;
      } else {
        for (int it = iterE; it < PE.max_iters; ++it) st->alphas[st->n_alphas++] = 0.0;
        st->qp_iters = PE.max_iters;
        actE[b] = 0;
      }
    }
    if (XOE != XE)
      for (int e = l; e < PE.T; e += 64) XOE[e] = sXD[e].x;
    return;
  }
  double ss = 0.0;
  for (int e = l; e < PE.T; e += 64) {
    const XD p = sXD[e];
    const double xv = p.x;
    const double stp = alpha * p.d;
    XOE[e] = xv + stp;
    ss += stp * stp;
  }
  // wave reduction
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) ss += __shfl_xor(ss, off, 64);
  if (l == 0) {
    const double stepsize = sqrt(ss);
    st->alphas[st->n_alphas++] = alpha;
    st->stepsizes[st->n_steps++] = stepsize;
    st->qp_iters = iterE + 1;
    if (stepsize < PE.step_tol || iterE + 1 >= PE.max_iters) actE[b] = 0;
  }
}

#ifndef I7M_LS_WPE
#define I7M_LS_WPE 2  // waves per SIMD the line search is compiled for (A/B builds: 3)
#endif
#ifndef I7M_LS_KARG
#define I7M_LS_KARG 1  // k_linesearch re-reads its parameters from the kernarg segment (LsKernArgs)
#endif
template <bool SPEC, int ABL = 0, int W = 1, bool FW = false>
__global__ void __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(I7M_LS_WPE, I7M_LS_WPE))) k_linesearch(const DevModel* __restrict__ Mg, SolveParams P,
                                                   const double* xu, double* xu_out, const double* __restrict__ sol,
                                                   const double* __restrict__ goals, const double* __restrict__ fext,
                                                   int* __restrict__ active,
                                                   ProblemStats* __restrict__ stats, double* __restrict__ alpha_out,
                                                   int iter, int mode, const double* __restrict__ lin = nullptr,
                                                   const double* __restrict__ cost = nullptr, const LsSplit sp = LsSplit{}) {
  I7M_TL(3);
  const int b = blockIdx.x;
  if (b >= P.B) return;
  if (active && !active[b]) return;
  // the second launch of a split search runs only the problems the first one handed over
  if (sp.c_begin > 0 && !sp.pending[b]) return;
  extern __shared__ __attribute__((aligned(16))) double ls_dyn[];
  __shared__ double merit[9];
  linesearch_body<SPEC, ABL, W, FW, I7M_LS_KARG != 0>(Mg, P, b, W > 1 ? (int)(threadIdx.x >> 6) : 0, threadIdx.x & 63,
                                                      ls_dyn, merit, xu, xu_out, sol, goals, fext, active, stats,
                                                      alpha_out, iter, mode, lin, cost, sp);
}

// Merit pieces of a given XU (hooks for SQP_OSQP.eepos_cost / integrator_err).
__global__ void __launch_bounds__(64) k_merit(const DevModel* __restrict__ Mg, SolveParams P,
                                              const double* __restrict__ xu, const double* __restrict__ xu_ref,
                                              const double* __restrict__ goals, const double* __restrict__ fext,
                                              int fext_world, double* __restrict__ out) {
  const int b = blockIdx.x;
  if (b >= P.B) return;
  const int l = threadIdx.x;
  const double* X = xu + (long)b * P.T;
  __shared__ double part[MAXN][4];
  for (int k = l; k < P.N; k += 64) {
    double o[4];
    merit_knot(*Mg, P, k, X + 18 * k, (k < P.N - 1) ? X + 18 * (k + 1) : X, goals + (long)b * P.N * P.goal_stride + (long)k * P.goal_stride,
               fext ? fext + 6L * b : nullptr, fext_world != 0, o);
    part[k][0] = o[0]; part[k][1] = o[1]; part[k][2] = o[2]; part[k][3] = o[3];
  }
  lds_sync();
  if (l == 0) {
    double acc[4] = {0, 0, 0, 0};
    for (int k = 0; k < P.N; ++k)
      for (int j = 0; j < 4; ++j) acc[j] += part[k][j];
    double dd = 0.0;
    for (int i = 0; i < 12; ++i) {
      const double t = X[i] - xu_ref[(long)b * P.T + i];
      dd += t * t;
    }
    for (int j = 0; j < 4; ++j) out[b * 5 + j] = acc[j];
    out[b * 5 + 4] = sqrt(dd);
  }
}

// ---------------------------------------------------------------------------------------
// Query kernels (one thread per query).
__global__ void __launch_bounds__(256) k_eepos(const DevModel* __restrict__ Mg, int n, const double* __restrict__ q,
                                               double* __restrict__ p, double* __restrict__ J) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double c[6], s[6], pp[3], JJ[3][6];
  sincos6(q + 6L * i, c, s);
  fk_jac(*Mg, c, s, pp, JJ);
  for (int r = 0; r < 3; ++r) p[3L * i + r] = pp[r];
  if (J)
    for (int r = 0; r < 3; ++r)
      for (int j = 0; j < 6; ++j) J[18L * i + 6 * r + j] = JJ[r][j];
}

// fext (n, 6) or null; fext_world: it is a world-frame wrench (converted at q), else local.
__global__ void __launch_bounds__(256) k_aba(const DevModel* __restrict__ Mg, int n, const double* __restrict__ q,
                                             const double* __restrict__ v, const double* __restrict__ tau,
                                             const double* __restrict__ fext, int fext_world, double* __restrict__ a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double c[6], s[6], L[6][6], aa[6], fl[6];
  sincos6(q + 6L * i, c, s);
  const double* f6 = fext ? fext + 6L * i : nullptr;
  if (f6 && fext_world) {
    wrench_world_to_local(*Mg, c, s, f6, fl);
    f6 = fl;
  }
  forward_dynamics(*Mg, c, s, v + 6L * i, tau + 6L * i, f6, L, aa);
  for (int r = 0; r < 6; ++r) a[6L * i + r] = aa[r];
}

// thread per (query, direction d<12)
__global__ void __launch_bounds__(256) k_abad(const DevModel* __restrict__ Mg, int n, const double* __restrict__ q,
                                              const double* __restrict__ v, const double* __restrict__ tau,
                                              double* __restrict__ dq, double* __restrict__ dv,
                                              double* __restrict__ Minv, double* __restrict__ a) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int i = (int)(gid / 12), d = (int)(gid - 12L * (gid / 12));
  if (i >= n) return;
  double c[6], s[6], L[6][6], aa[6], col[6];
  sincos6(q + 6L * i, c, s);
  forward_dynamics(*Mg, c, s, v + 6L * i, tau + 6L * i, nullptr, L, aa);
  aba_deriv_column(*Mg, c, s, v + 6L * i, aa, L, d, nullptr, col);
  if (d < 6) {
    for (int r = 0; r < 6; ++r) dq[36L * i + 6 * r + d] = col[r];
    double e[6] = {0, 0, 0, 0, 0, 0};
    e[d] = 1.0;
    chol6_solve(L, e);
    for (int r = 0; r <= d; ++r) {
      Minv[36L * i + 6 * r + d] = e[r];
      Minv[36L * i + 6 * d + r] = e[r];
    }
    if (d == 0)
      for (int r = 0; r < 6; ++r) a[6L * i + r] = aa[r];
  } else {
    for (int r = 0; r < 6; ++r) dv[36L * i + 6 * r + (d - 6)] = col[r];
  }
}

// utils.rk4 (src/utils.py:3-18): 4 ABA evaluations, pin.integrate = q + v*dt.
// fext_world: fext is a world-frame wrench, converted to joint 6's frame ONCE at the start
// configuration q and held for the four stages, as the reference's host plant does
// (src/gato_mpc_batch_sample.py:270-279: actInv at x_last, then rk4 with that local force).
// One plant step of one lane: q, v, u (6 each) -> qo, vo; f6 a local joint-6 wrench or null.
__device__ __forceinline__ void rk4_step(const DevModel& Md, const double* q, const double* v, const double* u, double dt,
                                         const double* f6, bool fext_world, double* qo, double* vo) {
  double q0[6], v0[6], uu[6], c[6], s[6], L[6][6], fl[6];
  for (int r = 0; r < 6; ++r) { q0[r] = q[r]; v0[r] = v[r]; uu[r] = u[r]; }
  double k1v[6], k2v[6], k3v[6], k4v[6], k2q[6], k3q[6], k4q[6], qq[6];
  sincos6(q0, c, s);
  if (f6 && fext_world) {
    wrench_world_to_local(Md, c, s, f6, fl);
    f6 = fl;
  }
  forward_dynamics(Md, c, s, v0, uu, f6, L, k1v);
  for (int r = 0; r < 6; ++r) { qq[r] = q0[r] + v0[r] * dt / 2; k2q[r] = v0[r] + k1v[r] * dt / 2; }
  sincos6(qq, c, s);
  forward_dynamics(Md, c, s, k2q, uu, f6, L, k2v);
  for (int r = 0; r < 6; ++r) { qq[r] = q0[r] + k2q[r] * dt / 2; k3q[r] = v0[r] + k2v[r] * dt / 2; }
  sincos6(qq, c, s);
  forward_dynamics(Md, c, s, k3q, uu, f6, L, k3v);
  for (int r = 0; r < 6; ++r) { qq[r] = q0[r] + k3q[r] * dt; k4q[r] = v0[r] + k3v[r] * dt; }
  sincos6(qq, c, s);
  forward_dynamics(Md, c, s, k4q, uu, f6, L, k4v);
  for (int r = 0; r < 6; ++r) {
    vo[r] = v0[r] + (dt / 6) * (k1v[r] + 2 * k2v[r] + 2 * k3v[r] + k4v[r]);
    const double avg = (v0[r] + 2 * k2q[r] + 2 * k3q[r] + k4q[r]) / 6;
    qo[r] = q0[r] + avg * dt;
  }
}

__global__ void __launch_bounds__(256) k_rk4(const DevModel* __restrict__ Mg, int n, const double* __restrict__ q,
                                             const double* __restrict__ v, const double* __restrict__ u, double dt,
                                             const double* __restrict__ fext, int fext_world, double* __restrict__ qo,
                                             double* __restrict__ vo) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  rk4_step(*Mg, q + 6L * i, v + 6L * i, u + 6L * i, dt, fext ? fext + 6L * i : nullptr, fext_world != 0, qo + 6L * i,
           vo + 6L * i);
}

}  // namespace i7m
