// i7m_box.h — interior-point iteration of the box-constrained QP mode (I7M_QP_BOX, SURVEY.md
// §8d config 4).  Restates oracle/box_ipm.py::ipm_box step by step; the Newton steps
// themselves are k_riccati_mfma<0, true> (i7m_riccati_mfma.h) on the same linearisation.
//
// One wavefront per problem, lanes strided over the T = 18N-6 trajectory entries.  Per
// problem, in (B, T) device arrays: the iterate x, the bound duals z_l / z_u, the Riccati
// inputs Sigma / h, and the predictor step dx_aff; and in IpmState the scalars.
// Slacks s_l = x - lo, s_u = hi - x are recomputed from x (never stored).
#pragma once

#include "i7m_kernels.h"
#include "i7m_riccati_mfma.h"

#ifndef I7M_IPM_WPE
#define I7M_IPM_WPE 4
#endif
// cross-lane broadcasts of the box body's Newton steps (riccati_mfma_body BC): 3 = the rollout's and
// the pivots' by DPP (5.45 -> 5.42 ms per k_ipm_fused launch against 2, the rollout's only; bit-identical;
// DESIGN.md §4.2)
#ifndef I7M_IPM_BC
#define I7M_IPM_BC 3
#endif

namespace i7m {

struct BoxParams {
  int mask;       // I7M_BOX_Q | I7M_BOX_V | I7M_BOX_U
  int max_iters;
  double tol;
  double theta;   // initial interior margin, fraction of the box width
  double eta;     // step-to-boundary fraction
  double z0;      // centred start: z_l = z0 / s_l, z_u = z0 / s_u, so mu_0 = z0
};

struct IpmState {
  double mu, rfrac, smu;  // complementarity, prod(1 - alpha), sigma * mu of the corrector
  int iters, nb;          // corrector steps taken, bounded entries
  int converged, pad;
};

// Bounds of trajectory entry e (knot e / 18, slot e % 18); false if unbounded.  The initial
// state is fixed by the equality rows and never bounded (oracle/box_ipm.py::box_bounds).
// The per-slot bounds of the mask are staged once per kernel in LDS (BoxTab), so the element
// passes below read them there instead of from the model in global memory.
struct BoxTab {
  double lo[18], hi[18];
  int on[18];
};
__device__ __forceinline__ void box_tab_fill(const DevModel& M, int mask, BoxTab* t) {
  const int j = threadIdx.x;
  if (j < 18) {
    double lo = 0.0, hi = 0.0;
    int on = 0;
    if (j < 6) {
      on = mask & 1;
      lo = M.qlo[j];
      hi = M.qhi[j];
    } else if (j < 12) {
      on = mask & 2;
      hi = M.vlim[j - 6];
      lo = -hi;
    } else {
      on = mask & 4;
      hi = M.ulim[j - 12];
      lo = -hi;
    }
    t->lo[j] = lo;
    t->hi[j] = hi;
    t->on[j] = on != 0;
  }
  __syncthreads();
}
__device__ __forceinline__ bool box_of(const BoxTab& t, int e, double& lo, double& hi) {
  const int k = e / 18, j = e - 18 * k;
  if ((k == 0 && j < 12) || !t.on[j]) return false;
  lo = t.lo[j];
  hi = t.hi[j];
  return true;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
// two minima at once: both shuffles of a level in flight together
__device__ __forceinline__ void wave_min2(double& a, double& b) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double ta = __shfl_xor(a, off, 64), tb = __shfl_xor(b, off, 64);
    a = fmin(a, ta);
    b = fmin(b, tb);
  }
}
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmin(v, __shfl_xor(v, off, 64));
  return v;
}
__device__ __forceinline__ int wave_isum(int v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
// the largest t <= 1 with v + t dv >= 0 (v > 0), folded into a running minimum
__device__ __forceinline__ double ratio_min(double t, double v, double dv) {
  return (dv < 0.0) ? fmin(t, -v / dv) : t;
}
// both primal tests of a bounded entry (s_l + t d >= 0, s_u - t d >= 0): at most one binds, so one
// division — (-s_l) / d for d < 0, s_u / d for d > 0, the same values ratio_min gives bit for bit
__device__ __forceinline__ double ratio_min_box(double t, double sl, double su, double d) {
  const double q = ((d < 0.0) ? -sl : su) / d;
  return (d != 0.0) ? fmin(t, q) : t;
}

// The three phases of one interior-point iteration, as wave-level device functions of problem
// b (one wavefront; every lane ends with the same IpmState, reductions are xor-shuffle trees).
// k_ipm_init / k_ipm_pred / k_ipm_corr launch them one at a time (I7M_IPM=split), and
// k_ipm_fused runs the whole iteration of one problem in one wave.

// x = clip(x_eq) into the interior, the centred duals z = z0 / s, mu, and the first predictor's
// Sigma and h.
__device__ __forceinline__ IpmState ipm_init_body(const BoxTab& Bt, const SolveParams& P, const BoxParams& BP, const int b,
                                                  const double* __restrict__ xeq, double* __restrict__ x,
                                                  double* __restrict__ zl, double* __restrict__ zu,
                                                  double* __restrict__ sig, double* __restrict__ h) {
  const int l = threadIdx.x;
  const long o = (long)b * P.T;
  double acc = 0.0;
  int nb = 0;
  for (int e = l; e < P.T; e += 64) {
    double lo, hi, xv = xeq[o + e], a = 0.0, c = 0.0, s = 0.0;
    if (box_of(Bt, e, lo, hi)) {
      const double w = hi - lo;
      xv = fmin(fmax(xv, lo + BP.theta * w), hi - BP.theta * w);
      const double sl = xv - lo, su = hi - xv, isl = 1.0 / sl, isu = 1.0 / su;
      a = BP.z0 * isl;
      c = BP.z0 * isu;
      acc += sl * a + su * c;
      s = a * isl + c * isu;
      ++nb;
    }
    x[o + e] = xv;
    zl[o + e] = a;
    zu[o + e] = c;
    sig[o + e] = s;
    h[o + e] = -s * xv;
  }
  acc = wave_sum(acc);
  nb = wave_isum(nb);
  IpmState S;
  S.mu = nb ? acc / (2.0 * nb) : 0.0;
  S.rfrac = 1.0;
  S.smu = 0.0;
  S.iters = 0;
  S.nb = nb;
  S.converged = (nb == 0);
  S.pad = 0;
  return S;
}

// Predictor: dx_aff = y - x; affine step lengths and mu_aff (one pass); sigma*mu (-> S.smu);
// the corrector's h (a second pass).
// Every element term divides by the slacks through their reciprocals 1 / s_l, 1 / s_u, formed once
// per element and pass (oracle/box_ipm.py and the C++ port form them the same way): 26 IEEE
// divisions per bounded entry and iteration became 16 (the ratio tests keep theirs, and the two
// primal tests share one).
// Element passes run in chunks of IPM_U elements per lane: the chunk's operands are all loaded
// (clamped addresses, no branches) before any is used, so one wave has IPM_U x (2..5) loads in
// flight instead of waiting out the memory latency element by element.  The per-lane order of
// every accumulation is unchanged (chunks and their elements in increasing e), so the results
// are bit-identical to the element-by-element loops.
#ifndef I7M_IPM_U
#define I7M_IPM_U 6
#endif
constexpr int IPM_U = I7M_IPM_U;

__device__ __forceinline__ void ipm_pred_body(const BoxTab& Bt, const SolveParams& P, const BoxParams& BP, const int b,
                                              const double* __restrict__ y, const double* __restrict__ x,
                                              const double* __restrict__ zl, const double* __restrict__ zu,
                                              double* __restrict__ dxa, double* __restrict__ h, IpmState& S,
                                              double* __restrict__ dh = nullptr) {
  const int l = threadIdx.x;
  const int T = P.T;
  const long o = (long)b * T;
  // pass 1: dx_aff = y - x, the affine step lengths, and mu_aff from four sums of the same pass —
  // the complementarity after the affine step is bilinear in (ap, ad):
  //   (s_l + ap d)(z_l + ad dz_l) + (s_u - ap d)(z_u + ad dz_u)
  //     = [s_l z_l + s_u z_u] + ad [s_l dz_l + s_u dz_u] + ap [d z_l - d z_u] + ap ad [d dz_l - d dz_u]
  // (oracle/box_ipm.py forms it the same way; one pass over x, z_l, z_u instead of two)
  double ap = 1.0, ad = 1.0, s00 = 0.0, s01 = 0.0, s10 = 0.0, s11 = 0.0;
  for (int e0 = l; e0 < T; e0 += 64 * IPM_U) {
    double yv[IPM_U], xv[IPM_U], av[IPM_U], cv[IPM_U];
#pragma unroll
    for (int u = 0; u < IPM_U; ++u) {
      const int e = min(e0 + 64 * u, T - 1);
      yv[u] = y[o + e];
      xv[u] = x[o + e];
      av[u] = zl[o + e];
      cv[u] = zu[o + e];
    }
#pragma unroll
    for (int u = 0; u < IPM_U; ++u) {
      const int e = e0 + 64 * u;
      if (e < T) {
        const double d = yv[u] - xv[u];
        dxa[o + e] = d;
        double lo, hi;
        if (box_of(Bt, e, lo, hi)) {
          const double xx = xv[u], sl = xx - lo, su = hi - xx, a = av[u], c = cv[u];
          const double isl = 1.0 / sl, isu = 1.0 / su;
          const double dzl = -a - a * d * isl, dzu = -c + c * d * isu;
          ap = ratio_min_box(ap, sl, su, d);
          ad = ratio_min(ratio_min(ad, a, dzl), c, dzu);
          s00 += sl * a + su * c;
          s01 += sl * dzl + su * dzu;
          s10 += d * a - d * c;
          s11 += d * dzl - d * dzu;
        }
      }
    }
  }
  wave_min2(ap, ad);
  s00 = wave_sum(s00);
  s01 = wave_sum(s01);
  s10 = wave_sum(s10);
  s11 = wave_sum(s11);
  // clamped at 0: near convergence s00 ~ 2 nb mu cancels against the other sums
  const double mua = fmax(((s00 + ad * s01) + ap * (s10 + ad * s11)) / (2.0 * S.nb), 0.0);
  const double r = mua / S.mu;
  const double smu = r * r * r * S.mu;
  // pass 2: the corrector's linear-term shift h
  for (int e0 = l; e0 < T; e0 += 64 * IPM_U) {
    double dv[IPM_U], xv[IPM_U], av[IPM_U], cv[IPM_U], hold[IPM_U];
#pragma unroll
    for (int u = 0; u < IPM_U; ++u) {
      const int e = min(e0 + 64 * u, T - 1);
      dv[u] = dxa[o + e];
      xv[u] = x[o + e];
      av[u] = zl[o + e];
      cv[u] = zu[o + e];
      hold[u] = dh ? h[o + e] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < IPM_U; ++u) {
      const int e = e0 + 64 * u;
      if (e < T) {
        double lo, hi, hv = 0.0;
        if (box_of(Bt, e, lo, hi)) {
          const double d = dv[u], xx = xv[u], sl = xx - lo, su = hi - xx, a = av[u], c = cv[u];
          const double isl = 1.0 / sl, isu = 1.0 / su;
          const double dzl = -a - a * d * isl, dzu = -c + c * d * isu;
          const double rl = sl * a + d * dzl - smu, ru = su * c - d * dzu - smu;
          const double s = a * isl + c * isu;
          hv = -a + c + (rl * isl - ru * isu) - s * xx;
        }
        if (dh) dh[o + e] = hv - hold[u];  // the corrector's change of the linear terms
        h[o + e] = hv;
      }
    }
  }
  S.smu = smu;
}

// Corrector: dx = y - x, common step, update (x, z_l, z_u), new mu, convergence, and the next
// predictor's Sigma and h.
__device__ __forceinline__ void ipm_corr_body(const BoxTab& Bt, const SolveParams& P, const BoxParams& BP, const int b,
                                              const double* __restrict__ y, double* __restrict__ x,
                                              double* __restrict__ zl, double* __restrict__ zu,
                                              const double* __restrict__ dxa, double* __restrict__ sig,
                                              double* __restrict__ h, IpmState& S) {
  const int l = threadIdx.x;
  const int T = P.T;
  const long o = (long)b * T;
  const double smu = S.smu;
  double t = 1.0;
  for (int e0 = l; e0 < T; e0 += 64 * IPM_U) {
    double yv[IPM_U], xv[IPM_U], dav[IPM_U], av[IPM_U], cv[IPM_U];
#pragma unroll
    for (int u = 0; u < IPM_U; ++u) {
      const int e = min(e0 + 64 * u, T - 1);
      yv[u] = y[o + e];
      xv[u] = x[o + e];
      dav[u] = dxa[o + e];
      av[u] = zl[o + e];
      cv[u] = zu[o + e];
    }
#pragma unroll
    for (int u = 0; u < IPM_U; ++u) {
      const int e = e0 + 64 * u;
      double lo, hi;
      if (e < T && box_of(Bt, e, lo, hi)) {
        const double d = yv[u] - xv[u], da = dav[u];
        const double xx = xv[u], sl = xx - lo, su = hi - xx, a = av[u], c = cv[u];
        const double isl = 1.0 / sl, isu = 1.0 / su;
        const double dzla = -a - a * da * isl, dzua = -c + c * da * isu;
        const double rl = sl * a + da * dzla - smu, ru = su * c - da * dzua - smu;
        const double dzl = (-rl - a * d) * isl, dzu = (-ru + c * d) * isu;
        t = ratio_min_box(t, sl, su, d);
        t = ratio_min(ratio_min(t, a, dzl), c, dzu);
      }
    }
  }
  t = wave_min(t);
  const double al = fmin(1.0, BP.eta * t);
  double acc = 0.0;
  for (int e0 = l; e0 < T; e0 += 64 * IPM_U) {
    double yv[IPM_U], xv[IPM_U], dav[IPM_U], av[IPM_U], cv[IPM_U];
#pragma unroll
    for (int u = 0; u < IPM_U; ++u) {
      const int e = min(e0 + 64 * u, T - 1);
      yv[u] = y[o + e];
      xv[u] = x[o + e];
      dav[u] = dxa[o + e];
      av[u] = zl[o + e];
      cv[u] = zu[o + e];
    }
#pragma unroll
    for (int u = 0; u < IPM_U; ++u) {
      const int e = e0 + 64 * u;
      if (e < T) {
        const double d = yv[u] - xv[u];
        const double xx = xv[u];
        double lo, hi;
        if (box_of(Bt, e, lo, hi)) {
          const double da = dav[u], sl = xx - lo, su = hi - xx, a = av[u], c = cv[u];
          const double isl = 1.0 / sl, isu = 1.0 / su;
          const double dzla = -a - a * da * isl, dzua = -c + c * da * isu;
          const double rl = sl * a + da * dzla - smu, ru = su * c - da * dzua - smu;
          const double dzl = (-rl - a * d) * isl, dzu = (-ru + c * d) * isu;
          const double xn = xx + al * d, an = a + al * dzl, cn = c + al * dzu;
          x[o + e] = xn;
          zl[o + e] = an;
          zu[o + e] = cn;
          const double sln = xn - lo, sun = hi - xn;
          acc += sln * an + sun * cn;
          const double s = an * (1.0 / sln) + cn * (1.0 / sun);
          sig[o + e] = s;
          h[o + e] = -s * xn;
        } else {
          x[o + e] = xx + al * d;
          sig[o + e] = 0.0;
          h[o + e] = 0.0;
        }
      }
    }
  }
  acc = wave_sum(acc);
  S.mu = acc / (2.0 * S.nb);
  S.rfrac *= 1.0 - al;
  S.iters += 1;
  S.converged = (S.mu < BP.tol && S.rfrac < BP.tol);
}

// The state is wave-uniform (every lane computed it from the same xor-shuffle reductions);
// readfirstlane tells the compiler so, and the state lives in SGPRs across the Newton steps.
__device__ __forceinline__ void ipm_uniform(IpmState& S) {
  S.mu = readlane_f64(S.mu, 0);
  S.rfrac = readlane_f64(S.rfrac, 0);
  S.smu = readlane_f64(S.smu, 0);
  S.iters = __builtin_amdgcn_readfirstlane(S.iters);
  S.nb = __builtin_amdgcn_readfirstlane(S.nb);
  S.converged = __builtin_amdgcn_readfirstlane(S.converged);
}

__device__ __forceinline__ bool ipm_done(const IpmState& S, const BoxParams& BP) {
  return S.converged || S.iters >= BP.max_iters;
}

__global__ void __launch_bounds__(64) k_ipm_init(const DevModel* __restrict__ Mg, SolveParams P, BoxParams BP,
                                                 const double* __restrict__ xeq, const int* __restrict__ active,
                                                 double* __restrict__ x, double* __restrict__ zl, double* __restrict__ zu,
                                                 double* __restrict__ sig, double* __restrict__ h,
                                                 IpmState* __restrict__ st, int* __restrict__ ipm_active) {
  const int b = blockIdx.x;
  if (b >= P.B) return;
  if (active && !active[b]) {  // a finished problem keeps its last QP's state and record
    if (threadIdx.x == 0) ipm_active[b] = 0;
    return;
  }
  __shared__ BoxTab Bt;
  box_tab_fill(*Mg, BP.mask, &Bt);
  const IpmState S = ipm_init_body(Bt, P, BP, b, xeq, x, zl, zu, sig, h);
  if (threadIdx.x == 0) {
    st[b] = S;
    ipm_active[b] = (active ? active[b] : 1) && S.nb > 0;
  }
}

__global__ void __launch_bounds__(64) k_ipm_pred(const DevModel* __restrict__ Mg, SolveParams P, BoxParams BP,
                                                 const double* __restrict__ y, const double* __restrict__ x,
                                                 const double* __restrict__ zl, const double* __restrict__ zu,
                                                 double* __restrict__ dxa, double* __restrict__ h,
                                                 IpmState* __restrict__ st, const int* __restrict__ ipm_active) {
  const int b = blockIdx.x;
  if (b >= P.B || !ipm_active[b]) return;
  __shared__ BoxTab Bt;
  box_tab_fill(*Mg, BP.mask, &Bt);
  IpmState S = st[b];
  ipm_pred_body(Bt, P, BP, b, y, x, zl, zu, dxa, h, S);
  if (threadIdx.x == 0) st[b].smu = S.smu;
}

__global__ void __launch_bounds__(64) k_ipm_corr(const DevModel* __restrict__ Mg, SolveParams P, BoxParams BP,
                                                 const double* __restrict__ y, double* __restrict__ x,
                                                 double* __restrict__ zl, double* __restrict__ zu,
                                                 const double* __restrict__ dxa, double* __restrict__ sig,
                                                 double* __restrict__ h, IpmState* __restrict__ st,
                                                 int* __restrict__ ipm_active) {
  const int b = blockIdx.x;
  if (b >= P.B || !ipm_active[b]) return;
  __shared__ BoxTab Bt;
  box_tab_fill(*Mg, BP.mask, &Bt);
  IpmState S = st[b];
  ipm_corr_body(Bt, P, BP, b, y, x, zl, zu, dxa, sig, h, S);
  if (threadIdx.x == 0) {
    st[b] = S;
    if (ipm_done(S, BP)) ipm_active[b] = 0;
  }
}

// The whole interior-point solve of one problem in one wavefront: init from the equality-QP
// minimiser xeq, then predictor / corrector Newton steps until the problem converges or reaches
// max_iters.  One launch per QP instead of 2 + 4 max_iters; each wave runs exactly its own
// iteration count and the iteration state stays in registers.
// !DELTA (default): both Newton steps are full Riccati solves, the same arithmetic as the split
// kernels phase for phase.  DELTA (I7M_IPM=delta): the predictor step is a full
// riccati_mfma_body<0, true, true> (which also stores every stage's H^-1) and the corrector
// reuses that factorisation (riccati_delta_body: same Hessian, only the linear terms change by
// dh).  Measured slower (14.7 vs 13.7 ms per QP at B = 4096, N = 64): the vector pass streams
// as many bytes per stage as the full step and is as latency-bound.
// Newton iterates go to y (B, T), the iterate to x.
// Everything k_ipm_fused reads, passed as one kernel argument.  The kernel re-reads it from the
// kernarg segment through a laundered scalar pointer in every Newton step, so the ~20 buffer
// pointers are reloaded (s_load, scalar cache) where used instead of pinned in SGPRs across the
// whole loop (which spilled them into VGPR lanes, and VGPRs to scratch).
struct IpmFusedArgs {
  const DevModel* Mg;
  SolveParams P;
  BoxParams BP;
  const double *xu, *xs, *lin, *cost, *qpd;
  const int* active;
  double* kbuf;
  const double* xeq;
  double *y, *x, *zl, *zu, *sig, *h, *dxa;
  IpmState* st;
  int* ipm_active;
  double *hinv, *dh;
#ifdef I7M_DIAG
  // I7M_ABLATE (diagnostic timing builds only, results invalid): 40 every problem runs exactly
  // IPM_ABL_IT interior-point iterations (convergence ignored), 41 + the predictor's element passes
  // skipped, 42 + the corrector's, 43 + both (Newton steps only), 44 + the Newton steps skipped
  // (element passes only) — the per-iteration cost of each part at a fixed iteration count
  int ablate;
#endif
};
constexpr int IPM_ABL_IT = 7;
// the kernarg segment, laundered (the cast back to a generic pointer is inferred to the
// constant address space again, so the fields are scalar loads)
__device__ __forceinline__ const IpmFusedArgs* kernarg_ipm() {
  auto p = __builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return (const IpmFusedArgs*)p;
}

template <bool DELTA>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(I7M_IPM_WPE, I7M_IPM_WPE)))
k_ipm_fused(IpmFusedArgs args) {
  I7M_TL(4);
  const int b = blockIdx.x;
  if (b >= args.P.B) return;
  if (args.active && !args.active[b]) return;  // a finished problem keeps its last QP's state and record
  __shared__ double sh[MO_TOTAL];
  __shared__ BoxTab Bt;
  IpmState S;
  bool run;
  {
    const IpmFusedArgs& a = args;
    box_tab_fill(*a.Mg, a.BP.mask, &Bt);
    S = ipm_init_body(Bt, a.P, a.BP, b, a.xeq, a.x, a.zl, a.zu, a.sig, a.h);
    ipm_uniform(S);
    run = (a.active ? a.active[b] != 0 : true) && S.nb > 0;
  }
  // The lane id and the argument pointer are laundered per step (an empty asm the compiler must
  // treat as redefining them): the Riccati operand maps, the box bounds and the buffer pointers
  // are rebuilt / reloaded per step instead of hoisted out of the loop and held live across it.
  // !DELTA: one Riccati call site (half 0: predictor, half 1: corrector) keeps one inlined copy.
#ifdef I7M_DIAG
  const int abl = args.ablate;
  const bool skip_newton = abl == 44, skip_pred = abl == 41 || abl == 43, skip_corr = abl == 42 || abl == 43;
#else
  constexpr int abl = 0;
  constexpr bool skip_newton = false, skip_pred = false, skip_corr = false;
#endif
  for (int half = 0; run; half ^= 1) {
    int l = threadIdx.x;
    const IpmFusedArgs* A = kernarg_ipm();
    asm volatile("" : "+v"(l));
    const SolveParams P = A->P;
    __syncthreads();
    if (skip_newton) {
    } else if (!DELTA) {
      // the corrector (half 1) stores only K~'s feedforward column: its gain is the predictor's
      riccati_mfma_body<0, true, false, I7M_IPM_BC>(b, P, A->xu, A->xs, A->lin, A->cost, A->qpd, A->kbuf, A->y, A->sig,
                                                    A->h, sh, l, nullptr, half == 1);
    } else if (half == 0) {
      riccati_mfma_body<0, true, true>(b, P, A->xu, A->xs, A->lin, A->cost, A->qpd, A->kbuf, A->y, A->sig, A->h, sh, l,
                                       A->hinv);
    } else {
      riccati_delta_body(b, P, A->lin, A->kbuf, A->hinv, A->dh, A->y, sh, l);
    }
    __syncthreads();
    const IpmFusedArgs* B = kernarg_ipm();
    const BoxParams BP = B->BP;
    // the most work left first: remaining iterations ~ log(mu / tol) (mu_0 = z0 = 0.1, tol 1e-8)
    if (I7M_PRIO & 4) set_prio((int)(log10(fmax(S.mu / BP.tol, 1.0)) * (1.0 / 2.5)));
    if (half == 0) {
      if (!skip_pred) {
        ipm_pred_body(Bt, B->P, BP, b, B->y, B->x, B->zl, B->zu, B->dxa, B->h, S, DELTA ? B->dh : nullptr);
        ipm_uniform(S);
      }
    } else {
      if (!skip_corr) {
        ipm_corr_body(Bt, B->P, BP, b, B->y, B->x, B->zl, B->zu, B->dxa, B->sig, B->h, S);
        ipm_uniform(S);
      } else {
        S.iters += 1;
      }
      run = abl >= 40 ? S.iters < IPM_ABL_IT : !ipm_done(S, BP);
    }
  }
  if (threadIdx.x == 0) {
    args.st[b] = S;
    args.ipm_active[b] = 0;
  }
}

}  // namespace i7m
