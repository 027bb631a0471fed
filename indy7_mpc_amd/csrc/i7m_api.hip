// i7m_api.hip — C-ABI of libindy7mpc.so (declared in include/indy7_mpc.h).
//
// Host orchestration of the SQP of src/osqp_sqp.py:76-93 on MI355X: per SQP iteration
// k_linearize -> k_riccati -> k_linesearch on one HIP stream, all buffers device-resident,
// sized once at i7m_create for max_batch problems (the reference's OSQP setup-once analogue,
// src/osqp_solver.py:39-41).  No allocation or host sync inside i7m_solve_device.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/indy7_mpc.h"
#include "i7m_kernels.h"
#include "i7m_linearize.h"
#include "i7m_riccati_mfma.h"
#include "i7m_box.h"
#include "i7m_admm.h"
#include "i7m_mpc.h"

// Source hash of the tree this library was built from (__graft_entry__.build passes it), so
// tests and smoke() can check that the loaded binary matches the sources they run against.
#ifndef I7M_SRC_HASH
#define I7M_SRC_HASH "unknown"
#endif
#ifdef I7M_DIAG
#define I7M_BUILD_KIND "diag"
#else
#define I7M_BUILD_KIND "release"
#endif

using namespace i7m;

// i7m_lin_tu.hip (its own translation unit: a different machine-scheduler setting)
void i7m_launch_linearize_kernel(bool spec, int grid, hipStream_t s, hipEvent_t ea, hipEvent_t eb, const void* model,
                                 const void* params, const double* xu, const double* goals, const double* fext,
                                 bool fext_world, const int* active, double* lin, double* cost, double* qpd,
                                 int* init_active, void* init_stats);

// i7m_admm_prep_tu.hip (the ADMM scaling and factor kernels under the max-ILP scheduler): kernel 0
// k_admm_scale<9>, 1 k_admm_scale<18>, 2 k_admm_factor; args: const AdmmArgs*
hipError_t i7m_launch_admm_prep(int kernel, int grid, hipStream_t s, hipEvent_t ea, hipEvent_t eb, const void* args);

// i7m_fused_tu.hip (k_sqp_fused in a unit of its own)
hipError_t i7m_launch_sqp_fused(bool spec, int W, bool fext_world, int it, hipStream_t s, hipEvent_t ea, hipEvent_t eb,
                                const void* model, const void* params, const double* xu_in, double* xu_out,
                                const double* xs, const double* goals, const double* fext, double* lin, double* cost,
                                double* qpd, double* kbuf, double* sol, int* active, void* stats);
hipError_t i7m_prepare_sqp_fused(int dev, int N);

static_assert(sizeof(i7m_problem_stats) == sizeof(ProblemStats), "stats layout");

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                             \
  do {                                                                                           \
    hipError_t e_ = (expr);                                                                      \
    if (e_ != hipSuccess)                                                                        \
      return fail(I7M_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_));                  \
  } while (0)

struct Timing {
  int kid;
  hipEvent_t a, b;
};

}  // namespace

// k_riccati_mfma's Gauss-Jordan pivot broadcasts switch from v_readlane to DPP from this batch
// size on (riccati_mfma_body BC)
// DPP pivot broadcasts at every batch size since the round-3 stage changes (re-measured: 57.9 -> 54.7 us
// at B = 1024, 44.3 -> 42.6 at 512, 41.4 -> 40.0 at 64, 40.7 -> 39.5 at B = 1; before them they
// cost ~4.5 us below 2048; profiles/r03_ric_bc_retune_ab.txt)
constexpr int RIC_DPP_MIN_B = 0;
constexpr int RIC_W2_MAX_B = 128;     // two-wave Riccati up to this batch size (I7M_RIC_W2 forces): 43.9 -> 42.0 us at B = 1, 44.6 -> 42.7 at 64; slower from 512
// wave priority by progress once Riccati waves share SIMDs: from 768 problems (re-measured in round 3:
// 55.2 -> 52.4 us at B = 768, 42.5 -> 43.3 at 512; profiles/r03_ric_bc_retune_ab.txt)
constexpr int RIC_PRIO_MIN_B = 768;

struct i7m_handle {
  i7m_config cfg;
  int dev = 0;
  hipStream_t own = nullptr, stream = nullptr;
  DevModel* d_model = nullptr;
  // batch buffers (max_batch problems)
  double *d_xu = nullptr, *d_xs = nullptr, *d_goal = nullptr, *d_sol = nullptr, *d_lin = nullptr,
         *d_cost = nullptr, *d_kbuf = nullptr, *d_aux = nullptr, *d_out = nullptr;
  double* d_qpd = nullptr;  // (max_batch, N-1, QPD_STRIDE) per-knot QP records (k_linearize -> k_riccati_mfma)
  int* d_active = nullptr;
  ProblemStats* d_stats = nullptr;
  double* d_fext = nullptr;   // (max_batch, 6) joint-6 wrench per problem, frame fext_frame
  int fext_frame = I7M_WRENCH_LOCAL;
  // I7M_QP_BOX (i7m_box.h): iterate, bound duals, Riccati inputs, predictor step; (max_batch, T)
  double *d_bx = nullptr, *d_bzl = nullptr, *d_bzu = nullptr, *d_bsig = nullptr, *d_bh = nullptr, *d_bdxa = nullptr;
  double *d_bhinv = nullptr, *d_bdh = nullptr;  // per-stage H^-1 (max_batch, N-1, 36); corrector dh (max_batch, T)
  IpmState* d_bst = nullptr;
  int* d_bact = nullptr;
  // I7M_QP_ADMM (i7m_admm.h): one allocation, per-problem OSQP state and k_admm scratch
  double* d_admm = nullptr;
  int* d_admm_it = nullptr;  // 2 x (max_batch, I7M_MAX_SQP): OSQP iterations, then OSQP status, per SQP iteration
  // box QP: 1 k_ipm_fused<false> (default), 0 I7M_IPM=delta (k_ipm_fused<true>: the corrector
  // reuses the predictor's factorisation; measured slower), 2 I7M_IPM=split
  int ipm_mode = 1;
  int ablate = 0;                  // I7M_DIAG builds only (I7M_ABLATE): timing variants, results invalid
  bool spec = false;               // model == kIndy7Model: use the kernels with the constants baked in
  bool has_fext = false;
  size_t goal_cap = 0;
  // hipGraph replay of run_sqp (run_sqp_graphed): a few instantiated graphs keyed by the call
  struct GraphEntry {
    int B, goal_stride, has_fext;
    const void *xu_in, *xu, *xs, *goals, *st, *stream;
    hipGraphExec_t exec;
    unsigned long long last_use;
  };
  std::vector<GraphEntry> graphs;
  unsigned long long graph_clock = 0;
  bool use_graph = false;  // I7M_GRAPH=1: capture the solve once per buffer set, replay it
                           // (measured 4-5 us slower per solve at B = 1 and 64, level at 4096)
  int ls_waves = 0;  // waves per problem in k_linesearch: 0 automatic (4 for B <= 768), else I7M_LS_WAVES (1, 2 or 4)
  // I7M_LS_TAIL = r > 0: split line search — the first launch (one wave per problem) stops after r
  // rounds, a second launch with two waves per problem finishes the unresolved problems
  int ls_tail = 0;
  double* d_lsbase = nullptr;  // (max_batch) base merits handed to the second launch
  int* d_lspend = nullptr;     // (max_batch) pending flags
  int pipeline = I7M_PIPE_AUTO;  // cfg.pipeline, or I7M_PIPE=split|fused
  int ric_w2 = -1;               // k_riccati_mfma_w2 (two waves per problem): 1 / 0, -1 = by batch size
  int ric_bc = -1;               // k_riccati_mfma broadcast variant (BC bits), -1 = by batch size
  // host-to-host i7m_solve split into chunks on two streams, so the copies of one chunk overlap
  // the solve of another (0 = one piece on h->stream; I7M_H2H_CHUNKS or cfg.h2h_chunks)
  int h2h_chunks = 0;
  int admm_chunk = 0;  // I7M_ADMM_CHUNK: k_admm launched over this many problems at a time (0: all)
  int dev_ranges = 0;  // I7M_DEV_RANGES: i7m_solve_device in this many ranges on the two chunk streams (A/B)
  // ADMM mode, i7m_solve_device with B >= admm_stagger_min_b: the batch as admm_ranges ranges on
  // streams of their own, each started once the one before has passed a mark (1: its first QP's
  // scaling and factor; 2: its first QP; A/B: 3 its first linearisation, 4 its first scaling), so one range's latency-bound phases (the factor, the
  // OSQP iterations after the first termination check) overlap another's stream-bound ones
  // (DESIGN.md §4.7).  0: one range.  I7M_ADMM_STAGGER, I7M_ADMM_RANGES, I7M_ADMM_STAGGER_MIN_B.
  int admm_stagger = 1;
  int stagger_modes = 1 << I7M_QP_ADMM;  // the QP modes that stagger (bit per mode; I7M_STAGGER_MODES)
  int admm_ranges = 2;
  // k_admm_iter2 (two problems per wave) for launches of at most 512 problems: 3.5 % shorter at
  // B <= 256, level at 1 024, 19-32 % longer at 4 096 (profiles/r06p, r06q); I7M_ADMM_ITER2 = 0
  // never, 1 always, -1 (default) by that size
  int admm_iter2 = -1;
  // k_admm_iter_res (one problem per workgroup, its records and vectors resident in LDS) for
  // launches of at most admm_res_max problems at N <= ARES_N without rho adaptation; I7M_ADMM_RES
  // = 0 never, 1 whenever it fits, -1 (default) by that size
  int admm_res = -1;
  int admm_res_max = 256;
  // k_admm_scale / k_admm_factor as built under the max-ILP scheduler (i7m_admm_prep_tu.hip) for
  // launches of at most admm_prep_ilp_max problems, else this unit's: 6 % shorter at B <= 256, but
  // at config 3 (staggered ranges of 2048) the step 0.6 % longer beside the other range's
  // iteration (profiles/r06zn, r06zo); I7M_ADMM_PREP_ILP = 0 never, 1 always, -1 (default) by size
  int admm_prep_ilp = -1;
  int admm_prep_ilp_max = 1024;
  // extra dynamic LDS per k_admm_iter workgroup (I7M_ADMM_ITER_DYN_LDS, bytes; A/B): past 160 KB / 4
  // it leaves one SIMD of every CU, and its LDS, to the other range's kernels
  int admm_iter_dyn_lds = 0;
  int admm_chains = 1;  // ranges r wait for range r - chains's mark (I7M_ADMM_CHAINS, A/B: 2 = two independent stagger chains)
  int admm_split = 500;  // two ranges: the first's share of the batch, per mille (I7M_ADMM_SPLIT, A/B)
  int admm_stagger_min_b = 3072;  // measured, two ranges: B = 8192 / 4096 / 3072 +9 / +17 / +5 %; 2048 / 1024 -8 / -11 %
  static constexpr int kMaxRanges = 4;
  hipStream_t rs[kMaxRanges] = {};  // ranges 2.. (0 and 1 run on cs[0], cs[1]); created on first use
  hipEvent_t ev_rmark[kMaxRanges] = {}, ev_rdone[kMaxRanges] = {};
  hipEvent_t mark_ev = nullptr;  // set: solve_qp records it at the mark, once, and clears it
  hipStream_t cs[2] = {nullptr, nullptr};
  hipStream_t cs2 = nullptr;  // h2h_pipe >= 2: the second solve stream (created on first use)
  hipEvent_t ev_order = nullptr, ev_done[2] = {nullptr, nullptr};
  // pipelined host-to-host chunks (h2h_pipe 1 / 2; I7M_H2H_PIPE=0: the first cut's two alternating
  // streams): per chunk, copy-in on cs[0] -> solve -> copy-out on cs[1]
  // 2 (default): the chunks' solves alternate over two streams, so one chunk's solve may overlap the
  // next one's start; 1: all solves on the handle's stream (A/B); 3: as 2, with the
  // copies out issued by a second host thread (pageable copies block the issuing thread)
  int h2h_pipe = 2;
  int h2h_taper = 1;  // I7M_H2H_TAPER=0: equal chunks (A/B)
  std::vector<hipEvent_t> ev_in, ev_cmp;
  // timing
  bool timing = false;
  std::vector<Timing> ev;
  std::vector<hipEvent_t> pool;
  double ms_sum[I7M_K_COUNT] = {};
  int counts[I7M_K_COUNT] = {};
};

namespace {

DevModel make_dev_model(const i7m_model& m) {
  DevModel d;
  std::memset(&d, 0, sizeof(d));
  for (int i = 0; i < 6; ++i) {
    for (int k = 0; k < 9; ++k) d.Rp[i][k] = m.placement_R[i][k];
    for (int k = 0; k < 3; ++k) d.tp[i][k] = m.placement_t[i][k];
    const double mass = m.mass[i];
    const double* c = m.com[i];
    d.m[i] = mass;
    for (int k = 0; k < 3; ++k) d.h[i][k] = mass * c[k];
    // inertia about the joint origin: Ic + m (|c|^2 I - c c^T)
    const double cc = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
    const double* I = m.inertia[i];
    d.Io[i][0] = I[0] + mass * (cc - c[0] * c[0]);
    d.Io[i][1] = I[1] - mass * c[0] * c[1];
    d.Io[i][2] = I[2] - mass * c[0] * c[2];
    d.Io[i][3] = I[3] + mass * (cc - c[1] * c[1]);
    d.Io[i][4] = I[4] - mass * c[1] * c[2];
    d.Io[i][5] = I[5] + mass * (cc - c[2] * c[2]);
    d.qlo[i] = m.q_lower[i];
    d.qhi[i] = m.q_upper[i];
    d.vlim[i] = m.v_limit[i];
    d.ulim[i] = m.effort_limit[i];
  }
  for (int k = 0; k < 3; ++k) d.g[k] = m.gravity[k];
  return d;
}

SolveParams params_of(const i7m_handle* h, int B, int goal_stride) {
  SolveParams P;
  P.N = h->cfg.N;
  P.T = 18 * h->cfg.N - 6;
  P.B = B;
  P.goal_stride = goal_stride;
  P.regularize = h->cfg.regularize;
  P.max_iters = h->cfg.max_sqp_iters;
  P.dt = h->cfg.dt;
  P.dQ = h->cfg.dQ_cost;
  P.R = h->cfg.R_cost;
  P.QN = h->cfg.QN_cost;
  P.eps = h->cfg.eps;
  P.mu = h->cfg.mu;
  P.step_tol = h->cfg.step_tol;
  return P;
}

int check_batch(const i7m_handle* h, int B, int goal_stride) {
  if (!h) return fail(I7M_EINVAL, "null handle");
  if (B < 0 || B > h->cfg.max_batch)
    return fail(I7M_EINVAL, "batch " + std::to_string(B) + " outside [0, max_batch=" +
                                std::to_string(h->cfg.max_batch) + "]");
  if (goal_stride != 3 && goal_stride != 6) return fail(I7M_EINVAL, "goal_stride must be 3 or 6");
  return I7M_OK;
}

hipEvent_t get_event(i7m_handle* h) {
  if (!h->pool.empty()) {
    hipEvent_t e = h->pool.back();
    h->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// Per-kernel timing: the start / stop events ride on the kernel's own dispatch packet
// (hipExtLaunchKernelGGL), so timing adds no marker packets between launches; with timing off
// the events are null and the launch is a plain dispatch.  `launch(ea, eb)` does the launch.
template <class F>
int timed(i7m_handle* h, hipStream_t s, int kid, F&& launch) {
  hipEvent_t a = nullptr, b = nullptr;
  if (h->timing) {
    a = get_event(h);
    b = get_event(h);
    if (!a || !b) a = b = nullptr;
  }
  launch(a, b);
  HIPCHK(hipGetLastError());
  if (a && b) h->ev.push_back({kid, a, b});
  return I7M_OK;
}

// Per-problem work buffers of a contiguous range of problems [b0, b0 + B): every kernel indexes
// them by its local problem index, so a range is just offset base pointers.
struct Bufs {
  double* lin;
  double* cost;
  double* qpd;
  double* kbuf;
  const double* fext;  // nullptr: no external wrench
  // box mode only (nullptr otherwise)
  double *bx, *bzl, *bzu, *bsig, *bh, *bdxa, *bhinv, *bdh;
  IpmState* bst;
  int* bact;
  // ADMM mode only: AdmmArgs' per-problem pointers for this range (P, A, sqp_iter filled at launch)
  AdmmArgs adm;
};

// per-problem sizes of the ADMM buffers (doubles), in the order admm_layout lays them out
constexpr int ADM_NBUF = 15;
void admm_sizes(long N, long sz[ADM_NBUF]) {
  const long T = 18 * N - 6, m = 12 * N;
  const long v[ADM_NBUF] = {T, m, m, T, 1,                        // x z y q rho (state)
                            36 * N, T, m, T, m, T, m,               // Pq Pd I qs ls D E
                            ADM_REC * N, T, 1};                     // stage records, w (h), c
  for (int i = 0; i < ADM_NBUF; ++i) sz[i] = v[i];
}
// AdmmArgs pointers of problems [b0, ...) in the handle's ADMM allocation (array-of-buffers, each
// (max_batch, size) row-major)
AdmmArgs admm_layout(double* base, int* its, long Bm, long N, long b0) {
  long sz[ADM_NBUF];
  admm_sizes(N, sz);
  double* p[ADM_NBUF];
  double* cur = base;
  for (int i = 0; i < ADM_NBUF; ++i) {
    p[i] = cur + b0 * sz[i];
    cur += (Bm * sz[i] + 1) & ~1L;  // every buffer 16-byte aligned (k_admm_iter's 16-byte loads)
  }
  AdmmArgs a{};
  a.sx = p[0]; a.sz = p[1]; a.sy = p[2]; a.sq = p[3]; a.srho = p[4];
  a.Pq = p[5]; a.Pd = p[6]; a.I = p[7]; a.qs = p[8]; a.ls = p[9]; a.D = p[10]; a.E = p[11];
  a.R = p[12]; a.w = p[13]; a.cs = p[14];
  a.iters = its + b0 * I7M_MAX_SQP;
  a.status = its + (Bm + b0) * I7M_MAX_SQP;
  a.abase = base;  // k_admm_iter reaches every array through one buffer resource over the allocation
  a.abytes = (long)(cur - base) * 8;
  return a;
}
size_t admm_doubles(long Bm, long N) {
  long sz[ADM_NBUF];
  admm_sizes(N, sz);
  size_t t = 0;
  for (int i = 0; i < ADM_NBUF; ++i) t += (size_t)((Bm * sz[i] + 1) & ~1L);
  return t;
}

Bufs bufs_at(const i7m_handle* h, long b0) {
  const long N = h->cfg.N, T = 18 * N - 6;
  Bufs W{h->d_lin + b0 * (N - 1) * LIN_STRIDE, h->d_cost + b0 * N * COST_STRIDE,
         h->d_qpd + b0 * (N - 1) * QPD_STRIDE, h->d_kbuf + b0 * (N - 1) * KBUF_STRIDE, h->has_fext ? h->d_fext + 6 * b0 : nullptr,
         nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  if (h->cfg.qp_mode == I7M_QP_BOX) {
    W.bx = h->d_bx + b0 * T;
    W.bzl = h->d_bzl + b0 * T;
    W.bzu = h->d_bzu + b0 * T;
    W.bsig = h->d_bsig + b0 * T;
    W.bh = h->d_bh + b0 * T;
    W.bdxa = h->d_bdxa + b0 * T;
    W.bhinv = h->d_bhinv + b0 * (N - 1) * 36;
    W.bdh = h->d_bdh + b0 * T;
    W.bst = h->d_bst + b0;
    W.bact = h->d_bact + b0;
  }
  if (h->cfg.qp_mode == I7M_QP_ADMM) W.adm = admm_layout(h->d_admm, h->d_admm_it, h->cfg.max_batch, N, b0);
  return W;
}

AdmmCfg admm_cfg_of(const i7m_config& c) {
  AdmmCfg A{};
  A.rho0 = c.admm_rho;
  A.sigma = c.admm_sigma;
  A.alpha = c.admm_alpha;
  A.eps_abs = c.admm_eps_abs;
  A.eps_rel = c.admm_eps_rel;
  A.adapt_tol = c.admm_adaptive_rho_tolerance;
  A.max_iter = c.admm_max_iter;
  A.check = c.admm_check_termination;
  A.scaling = c.admm_scaling;
  A.gap = c.admm_check_dualgap;
  A.adapt_interval = c.admm_adaptive_rho_interval;
  return A;
}

// init_active / init_stats (first SQP iteration only): the kernel marks every problem active
// and zeroes its stats, so a solve needs no separate memset launches.
int launch_linearize(i7m_handle* h, hipStream_t s, const Bufs& W, const SolveParams& P, const double* xu,
                     const double* goals, const int* active, int* init_active = nullptr,
                     ProblemStats* init_stats = nullptr) {
  const long knots = (long)P.B * P.N;
  if (knots == 0) return I7M_OK;
  const int grid = (int)((knots + KPW - 1) / KPW);
  return timed(h, s, I7M_K_LIN, [&](hipEvent_t ea, hipEvent_t eb) {
    i7m_launch_linearize_kernel(h->spec, grid, s, ea, eb, h->d_model, &P, xu, goals, W.fext,
                                h->fext_frame == I7M_WRENCH_WORLD, active, W.lin, W.cost, W.qpd, init_active, init_stats);
  });
}

template <int ABL>
void launch_riccati_mfma(hipStream_t s, hipEvent_t ea, hipEvent_t eb, const Bufs& W, const SolveParams& P,
                         const double* xu, const double* xs, const int* active, double* sol) {
  hipExtLaunchKernelGGL(k_riccati_mfma<ABL>, dim3(P.B), dim3(64), 0, s, ea, eb, 0, P, xu, xs, W.lin, W.cost, W.qpd, active,
                        W.kbuf, sol, (const double*)nullptr, (const double*)nullptr, (double*)nullptr);
}

// vout (i7m_qp_value): the first knot's cost-to-go V~_0 (B, 13, 13) instead of the rollout (one-wave
// kernel only)
int launch_riccati(i7m_handle* h, hipStream_t s, const Bufs& W, const SolveParams& P, const double* xu,
                   const double* xs, const int* active, double* sol, double* vout = nullptr) {
  if (P.B == 0) return I7M_OK;
  return timed(h, s, I7M_K_RICCATI, [&](hipEvent_t ea, hipEvent_t eb) {
#ifdef I7M_DIAG
    if (!vout) {
    // I7M_ABLATE -> ABL bits of riccati_mfma_body (diagnostic timing builds, results invalid;
    // compiled only into the -DI7M_DIAG library that tools/ load, never the shipping one)
    bool ablated = true;
    switch (h->ablate) {
      case 1: launch_riccati_mfma<1>(s, ea, eb, W, P, xu, xs, active, sol); break;      // no rollout
      case 2: launch_riccati_mfma<6>(s, ea, eb, W, P, xu, xs, active, sol); break;      // scaling for GJ
      case 8: launch_riccati_mfma<4>(s, ea, eb, W, P, xu, xs, active, sol); break;      // LDS-exchange GJ
      case 10: launch_riccati_mfma<8>(s, ea, eb, W, P, xu, xs, active, sol); break;     // kbuf slot 0
      case 11: launch_riccati_mfma<24>(s, ea, eb, W, P, xu, xs, active, sol); break;    // + lin slot 0
      case 13: launch_riccati_mfma<32>(s, ea, eb, W, P, xu, xs, active, sol); break;    // rollout dead
      case 18: launch_riccati_mfma<448>(s, ea, eb, W, P, xu, xs, active, sol); break;   // rollout chain only
      case 19: launch_riccati_mfma<513>(s, ea, eb, W, P, xu, xs, active, sol); break;   // phase timestamps, no rollout
      default: ablated = false;
    }
    if (ablated) return;
    }
#endif
    // (the diag library's default path is the release selection below, so its per-wave timelines
    // show the shipping kernels)
    // cross-lane broadcasts (riccati_mfma_body BC): the rollout's and the pivots' by DPP (from
    // RIC_DPP_MIN_B problems on, now every size); I7M_RIC_BC=0..3 forces one (A/B)
    // wave priority by progress (BC bit 2) once SIMDs hold more than one wave: -6 % at B = 4096,
    // -4 % at B = 1024 (uneven dispatch puts two waves on some SIMDs), +1 us at B = 64
    const int bc = h->ric_bc >= 0 ? h->ric_bc
                                  : (P.B >= RIC_DPP_MIN_B ? 3 : 2) | (P.B >= RIC_PRIO_MIN_B ? 4 : 0);
    // small batches: two waves per problem (k_riccati_mfma_w2), the stage's MFMA chains split
    const bool w2 = !vout && (h->ric_w2 >= 0 ? h->ric_w2 != 0 : P.B <= RIC_W2_MAX_B);
    if (w2) {
      auto go2 = [&](auto kern) {
        hipExtLaunchKernelGGL(kern, dim3(P.B), dim3(128), 0, s, ea, eb, 0, P, xu, xs, W.lin, W.cost, W.qpd, active,
                              W.kbuf, sol);
      };
      if (bc & 1) go2(k_riccati_mfma_w2<3>);
      else go2(k_riccati_mfma_w2<2>);
      return;
    }
    auto go = [&](auto kern) {
      hipExtLaunchKernelGGL(kern, dim3(P.B), dim3(64), 0, s, ea, eb, 0, P, xu, xs, W.lin, W.cost, W.qpd, active, W.kbuf,
                            sol, (const double*)nullptr, (const double*)nullptr, vout);
    };
    switch (bc) {
      case 1: go(k_riccati_mfma<0, false, 1>); break;
      case 2: go(k_riccati_mfma<0, false, 2>); break;
      case 3: go(k_riccati_mfma<0, false, 3>); break;
      case 6: go(k_riccati_mfma<0, false, 6>); break;
      case 7: go(k_riccati_mfma<0, false, 7>); break;
      default: go(k_riccati_mfma<0, false, 0>);
    }
  });
}

// waves per problem of the line search (k_linesearch) and of k_sqp_fused
// (k_linesearch: 4 waves per problem up to 768 problems — re-measured in round 3: 28.2 -> 19.0 us at
// B = 384, 28.6 -> 19.8 at 512, 29.9 -> 28.8 at 768, 30.6 -> 35.2 at 1024, profiles/r03_ls_waves_ab.txt;
// k_sqp_fused keeps the 256 it was measured with)
constexpr int LS_W4_MAX_B = 768, FUSED_W4_MAX_B = 256;
int waves_for(const i7m_handle* h, int B, int max_b4 = LS_W4_MAX_B) {
  return h->ls_waves > 0 ? h->ls_waves : (B <= max_b4 ? 4 : 1);
}

// base_from_lin: lin/cost of W hold the linearisation of this xu (the SQP loop), so the base
// merit comes from them (k_linesearch); otherwise candidate 0 is evaluated.
// xu: the linearisation point; xu_out: where the updated XU goes (may be xu itself).
int launch_linesearch(i7m_handle* h, hipStream_t s, const Bufs& W, const SolveParams& P, const double* xu,
                      double* xu_out, const double* sol, const double* goals, int* active, ProblemStats* st,
                      double* alpha_out, int iter, int mode, bool base_from_lin) {
  if (P.B == 0) return I7M_OK;
  // small batches leave most SIMDs idle: spend them on evaluating every candidate in one round
  const int nw = waves_for(h, P.B);
  const size_t lds = ls_lds_bytes(P.T, nw);
  const double* ln = base_from_lin ? W.lin : nullptr;
  const double* cs = base_from_lin ? W.cost : nullptr;
  const bool fw = W.fext && h->fext_frame == I7M_WRENCH_WORLD;
  if (h->ls_tail > 0 && nw == 1 && mode == 0 && base_from_lin) {
    // split search: r rounds of one wave per problem, then two waves per problem
    // for the problems that have not accepted a candidate
    const int R = P.N >= 64 ? 1 : 64 / P.N;
    const int c_split = 1 + R * h->ls_tail;
    const long b0 = W.lin - h->d_lin;  // this range's first problem (bufs_at offsets lin by b0 (N-1) stride)
    const long pb = b0 / ((long)(P.N - 1) * LIN_STRIDE);
    const LsSplit first{0, c_split, h->d_lsbase + pb, h->d_lspend + pb};
    const LsSplit second{c_split, 1 + NALPHA, h->d_lsbase + pb, h->d_lspend + pb};
    int rc = timed(h, s, I7M_K_LINESEARCH, [&](hipEvent_t ea, hipEvent_t eb) {
      auto go = [&](auto kern) {
        hipExtLaunchKernelGGL(kern, dim3(P.B), dim3(64), lds, s, ea, eb, 0, h->d_model, P, xu, xu_out, sol, goals, W.fext,
                              active, st, alpha_out, iter, mode, W.lin, W.cost, first);
      };
      if (h->spec) fw ? go(k_linesearch<true, 0, 1, true>) : go(k_linesearch<true, 0, 1>);
      else fw ? go(k_linesearch<false, 0, 1, true>) : go(k_linesearch<false, 0, 1>);
    });
    if (rc) return rc;
    const size_t lds2 = ls_lds_bytes(P.T, 2);
    return timed(h, s, I7M_K_LINESEARCH_TAIL, [&](hipEvent_t ea, hipEvent_t eb) {
      auto go = [&](auto kern) {
        hipExtLaunchKernelGGL(kern, dim3(P.B), dim3(128), lds2, s, ea, eb, 0, h->d_model, P, xu, xu_out, sol, goals, W.fext,
                              active, st, alpha_out, iter, mode, W.lin, W.cost, second);
      };
      if (h->spec) fw ? go(k_linesearch<true, 0, 2, true>) : go(k_linesearch<true, 0, 2>);
      else fw ? go(k_linesearch<false, 0, 2, true>) : go(k_linesearch<false, 0, 2>);
    });
  }
  return timed(h, s, I7M_K_LINESEARCH, [&](hipEvent_t ea, hipEvent_t eb) {
    auto go = [&](auto kern, int threads) {
      hipExtLaunchKernelGGL(kern, dim3(P.B), dim3(threads), lds, s, ea, eb, 0, h->d_model, P, xu, xu_out, sol, goals, W.fext,
                            active, st, alpha_out, iter, mode, ln, cs, LsSplit{});
    };
#ifdef I7M_DIAG
    if (h->ablate == 4 && nw == 1) {
      go(k_linesearch<true, 1>, 64);
      return;
    }
#endif
    if (nw == 4) {
      if (h->spec) fw ? go(k_linesearch<true, 0, 4, true>, 256) : go(k_linesearch<true, 0, 4>, 256);
      else fw ? go(k_linesearch<false, 0, 4, true>, 256) : go(k_linesearch<false, 0, 4>, 256);
    } else if (nw == 2) {  // A/B only (I7M_LS_WAVES=2)
      if (h->spec) fw ? go(k_linesearch<true, 0, 2, true>, 128) : go(k_linesearch<true, 0, 2>, 128);
      else fw ? go(k_linesearch<false, 0, 2, true>, 128) : go(k_linesearch<false, 0, 2>, 128);
    } else {
      if (h->spec) fw ? go(k_linesearch<true, 0, 1, true>, 64) : go(k_linesearch<true, 0, 1>, 64);
      else fw ? go(k_linesearch<false, 0, 1, true>, 64) : go(k_linesearch<false, 0, 1>, 64);
    }
  });
}

BoxParams box_params(const i7m_handle* h) {
  BoxParams BP;
  BP.mask = h->cfg.box_mask;
  BP.max_iters = h->cfg.box_max_iters;
  BP.tol = h->cfg.box_tol;
  BP.theta = 0.2;  // oracle/box_ipm.py::ipm_box defaults (6.9 vs 12.2 iterations
  BP.eta = 0.99;   // per config-4 QP against theta = 0.01, z = 1)
  BP.z0 = 0.1;
  return BP;
}

// The QP of one SQP iteration: the exact equality-constrained solve (k_riccati_mfma), and in
// box mode the interior-point iteration started from it (i7m_box.h; oracle/box_ipm.py).
// Returns where the minimiser is: `sol`, or W.bx in box mode.
int solve_qp(i7m_handle* h, hipStream_t s, const Bufs& W, const SolveParams& P, const double* xu, const double* xs,
             const int* active, double* sol, const double** out, int sqp_iter = 0) {
  int rc;
  if (h->cfg.qp_mode == I7M_QP_ADMM) {
    // OSQP's iteration from the problems' carried state (i7m_admm.h; oracle/osqp_admm.py)
    *out = sol;
    if (P.B == 0) return I7M_OK;
    AdmmArgs a = W.adm;
    a.P = P;
    a.A = admm_cfg_of(h->cfg);
    a.lin = W.lin;
    a.cost = W.cost;
    a.qpd = W.qpd;
    a.xu = xu;
    a.xs = xs;
    a.active = active;
    a.sol = sol;
    a.sqp_iter = sqp_iter;
#ifdef I7M_DIAG
    a.ablate = h->ablate;
#endif
    // I7M_ADMM_CHUNK = c > 0: the batch as consecutive launches of c problems, so one launch's
    // factors (the blocks every OSQP iteration re-reads) can stay in the 256 MB MALL
    const int chunk = h->admm_chunk > 0 ? std::min(h->admm_chunk, P.B) : P.B;
    for (int lo = 0; lo < P.B; lo += chunk) {
      a.b0 = lo;
      const int n = std::min(chunk, P.B - lo);
      int rc2 = timed(h, s, I7M_K_ADMM_PREP, [&](hipEvent_t ea, hipEvent_t eb) {
        // scaling, then the factor (one event pair around both)
        // the max-ILP-scheduled copies (i7m_admm_prep_tu.hip) or this unit's (default scheduler)
        const bool ilp = h->admm_prep_ilp > 0 || (h->admm_prep_ilp < 0 && n <= h->admm_prep_ilp_max);
        if (ilp)
          (void)i7m_launch_admm_prep(P.N <= 32 ? 0 : 1, n, s, ea, nullptr, &a);
        else if (P.N <= 32)
          hipExtLaunchKernelGGL(k_admm_scale<9>, dim3(n), dim3(64), 0, s, ea, nullptr, 0, a);
        else
          hipExtLaunchKernelGGL(k_admm_scale<18>, dim3(n), dim3(64), 0, s, ea, nullptr, 0, a);
        if (h->mark_ev && h->admm_stagger == 4) {  // (A/B: the mark between scaling and factor)
          (void)hipEventRecord(h->mark_ev, s);
          h->mark_ev = nullptr;
        }
        if (ilp)
          (void)i7m_launch_admm_prep(2, n, s, nullptr, eb, &a);
        else
          hipExtLaunchKernelGGL(k_admm_factor, dim3(n), dim3(64), 0, s, nullptr, eb, 0, a);
      });
      if (rc2) return rc2;
      if (h->mark_ev && h->admm_stagger == 1) {
        HIPCHK(hipEventRecord(h->mark_ev, s));
        h->mark_ev = nullptr;
      }
      rc2 = timed(h, s, I7M_K_ADMM, [&](hipEvent_t ea, hipEvent_t eb) {
        // four problems per wave: the launch covers [lo, lo + n) (a.b0 = lo), rows past it idle
        SolveParams P4 = a.P;
        P4.B = lo + n;
        AdmmArgs a4 = a;
        a4.P = P4;
        const dim3 g((n + 3) / 4);
        const bool res_fits = !a.A.adapt_interval && a.P.N <= ARES_N;
        if (a.A.adapt_interval)
          hipExtLaunchKernelGGL(k_admm_iter<true>, g, dim3(64), 0, s, ea, eb, 0, a4);
        else if (res_fits && (h->admm_res > 0 || (h->admm_res < 0 && n <= h->admm_res_max)))
          hipExtLaunchKernelGGL(k_admm_iter_res, dim3(n), dim3(64), 0, s, ea, eb, 0, a4);
        else if (h->admm_iter2 > 0 || (h->admm_iter2 < 0 && n <= 512))  // two problems per wave
          hipExtLaunchKernelGGL(k_admm_iter2, dim3((n + 1) / 2), dim3(64), 0, s, ea, eb, 0, a4);
        else
          hipExtLaunchKernelGGL(k_admm_iter<false>, g, dim3(64), h->admm_iter_dyn_lds, s, ea, eb, 0, a4);
      });
      if (rc2) return rc2;
    }
    if (h->mark_ev && h->admm_stagger == 2) {
      HIPCHK(hipEventRecord(h->mark_ev, s));
      h->mark_ev = nullptr;
    }
    return I7M_OK;
  }
  if ((rc = launch_riccati(h, s, W, P, xu, xs, active, sol))) return rc;
  *out = sol;
  if (h->cfg.qp_mode != I7M_QP_BOX || P.B == 0) return I7M_OK;
  const BoxParams BP = box_params(h);
  const dim3 g(P.B), blk(64);
  if (h->ipm_mode != 2) {
#ifdef I7M_DIAG
    const IpmFusedArgs fa{h->d_model, P, BP, xu, xs, W.lin, W.cost, W.qpd, active, W.kbuf, sol, sol,
                          W.bx, W.bzl, W.bzu, W.bsig, W.bh, W.bdxa, W.bst, W.bact, W.bhinv, W.bdh, h->ablate};
#else
    const IpmFusedArgs fa{h->d_model, P, BP, xu, xs, W.lin, W.cost, W.qpd, active, W.kbuf, sol, sol,
                          W.bx, W.bzl, W.bzu, W.bsig, W.bh, W.bdxa, W.bst, W.bact, W.bhinv, W.bdh};
#endif
    rc = timed(h, s, I7M_K_IPM_FUSED, [&](hipEvent_t ea, hipEvent_t eb) {
      if (h->ipm_mode == 0)
        hipExtLaunchKernelGGL(k_ipm_fused<true>, g, blk, 0, s, ea, eb, 0, fa);
      else
        hipExtLaunchKernelGGL(k_ipm_fused<false>, g, blk, 0, s, ea, eb, 0, fa);
    });
    if (rc) return rc;
    *out = W.bx;
    return I7M_OK;
  }
  rc = timed(h, s, I7M_K_IPM, [&](hipEvent_t ea, hipEvent_t eb) {
    hipExtLaunchKernelGGL(k_ipm_init, g, blk, 0, s, ea, eb, 0, h->d_model, P, BP, sol, active, W.bx, W.bzl, W.bzu, W.bsig, W.bh,
                       W.bst, W.bact);
  });
  if (rc) return rc;
  for (int it = 0; it < BP.max_iters; ++it) {
    for (int half = 0; half < 2; ++half) {
      rc = timed(h, s, I7M_K_RICCATI_BOX, [&](hipEvent_t ea, hipEvent_t eb) {
        hipExtLaunchKernelGGL((k_riccati_mfma<0, true>), g, blk, 0, s, ea, eb, 0, P, xu, xs, W.lin, W.cost, W.qpd, W.bact, W.kbuf,
                           sol, W.bsig, W.bh, (double*)nullptr);
      });
      if (rc) return rc;
      rc = timed(h, s, I7M_K_IPM, [&](hipEvent_t ea, hipEvent_t eb) {
        if (half == 0)
          hipExtLaunchKernelGGL(k_ipm_pred, g, blk, 0, s, ea, eb, 0, h->d_model, P, BP, sol, W.bx, W.bzl, W.bzu, W.bdxa, W.bh,
                             W.bst, W.bact);
        else
          hipExtLaunchKernelGGL(k_ipm_corr, g, blk, 0, s, ea, eb, 0, h->d_model, P, BP, sol, W.bx, W.bzl, W.bzu, W.bdxa, W.bsig,
                             W.bh, W.bst, W.bact);
      });
      if (rc) return rc;
    }
  }
  *out = W.bx;
  return I7M_OK;
}

// Does this solve run as one k_sqp_fused launch?  (Direct QP only; the box mode's interior point
// has its own fused kernel between the Riccati and the line search.)  AUTO is the split pipeline
// at every batch size: the fused one measured 1.1-2.4x slower from B = 1 to 4096.
bool use_fused(const i7m_handle* h, int B) {
  (void)B;
  if (h->cfg.qp_mode != I7M_QP_DIRECT) return false;
  return h->pipeline == I7M_PIPE_FUSED || h->pipeline == I7M_PIPE_FUSED_ITER;
}


int launch_fused(i7m_handle* h, hipStream_t s, const Bufs& W, const SolveParams& P, const double* xu_in, double* xu_out,
                 const double* xs, const double* goals, ProblemStats* st, long b0) {
  const int nw = waves_for(h, P.B, FUSED_W4_MAX_B);
  // I7M_PIPE_FUSED_ITER: one launch per SQP iteration, else one per solve
  const int launches = h->pipeline == I7M_PIPE_FUSED_ITER ? h->cfg.max_sqp_iters : 1;
  for (int i = 0; i < launches; ++i) {
    hipError_t e = hipSuccess;
    const int rc = timed(h, s, I7M_K_SQP_FUSED, [&](hipEvent_t ea, hipEvent_t eb) {
      e = i7m_launch_sqp_fused(h->spec, nw, h->fext_frame == I7M_WRENCH_WORLD, launches > 1 ? i : -1, s, ea, eb, h->d_model,
                               &P, i == 0 ? xu_in : xu_out, xu_out, xs, goals, W.fext, W.lin, W.cost, W.qpd, W.kbuf,
                               h->d_sol + b0 * P.T, h->d_active + b0, st);
    });
    if (rc) return rc;
    if (e != hipSuccess) return fail(I7M_EHIP, std::string("k_sqp_fused launch: ") + hipGetErrorString(e));
  }
  return I7M_OK;
}

// The SQP loop on device buffers: iteration 1 reads xu_in and its line search writes every
// row of xu_out; later iterations update xu_out in place (xu_in == xu_out is allowed).  The
// first linearisation also initialises the active flags and the stats (no memset launches).
// The B problems use the handle's per-problem work buffers from problem b0 on, and run on
// stream s (h->stream unless the host-to-host path splits the batch into chunks).
// (Splitting a device-resident batch into ranges on several streams, so that waves of different
// kernels share a SIMD, was measured at 2-4 ranges and gave nothing: DESIGN.md §7.)
int run_sqp(i7m_handle* h, int B, const double* d_xu_in, double* d_xu, const double* d_xs, const double* d_goals,
            int goal_stride, ProblemStats* d_st, long b0 = 0, hipStream_t s = nullptr) {
  const Bufs W = bufs_at(h, b0);
  const SolveParams P = params_of(h, B, goal_stride);
  if (!s) s = h->stream;
  int* act = h->d_active + b0;
  double* qbuf = h->d_sol + b0 * P.T;
  if (use_fused(h, B)) return launch_fused(h, s, W, P, d_xu_in, d_xu, d_xs, d_goals, d_st, b0);
  if (h->cfg.qp_mode == I7M_QP_ADMM && B > 0) {
    // this solve's OSQP records start at -1 ("no QP"): a problem that stops after SQP iteration
    // 0 must not report an earlier call's counts for the iterations it did not run
    HIPCHK(hipMemsetAsync(W.adm.iters, 0xff, (size_t)B * I7M_MAX_SQP * sizeof(int), s));
    HIPCHK(hipMemsetAsync(W.adm.status, 0xff, (size_t)B * I7M_MAX_SQP * sizeof(int), s));
  }
  for (int it = 0; it < h->cfg.max_sqp_iters; ++it) {
    const double* xin = it == 0 ? d_xu_in : d_xu;
    int rc;
    if (it == 0)
      rc = launch_linearize(h, s, W, P, xin, d_goals, nullptr, act, d_st);
    else
      rc = launch_linearize(h, s, W, P, xin, d_goals, act);
    if (rc) return rc;
    // the staggered ranges' mark outside ADMM mode (which marks inside its QP): after the first
    // linearisation (admm_stagger 1) or the first QP (2)
    const bool mark_here = h->mark_ev && h->cfg.qp_mode != I7M_QP_ADMM;
    if (h->mark_ev && (h->admm_stagger == 3 || (mark_here && h->admm_stagger == 1))) {
      HIPCHK(hipEventRecord(h->mark_ev, s));
      h->mark_ev = nullptr;
    }
    const double* qsol = nullptr;
    if ((rc = solve_qp(h, s, W, P, xin, d_xs, act, qbuf, &qsol, it))) return rc;
    if (mark_here && h->mark_ev && h->admm_stagger == 2) {
      HIPCHK(hipEventRecord(h->mark_ev, s));
      h->mark_ev = nullptr;
    }
    // mode 2: the ADMM mode's QP solver carries state, so an alpha = 0 iteration is re-solved
    if ((rc = launch_linesearch(h, s, W, P, xin, d_xu, qsol, d_goals, act, d_st, nullptr, it,
                                h->cfg.qp_mode == I7M_QP_ADMM ? 2 : 0, h->ablate != 6)))
      return rc;
  }
  return I7M_OK;
}

void drop_graphs(i7m_handle* h) {
  for (auto& g : h->graphs) (void)hipGraphExecDestroy(g.exec);
  h->graphs.clear();
}

// run_sqp through a cached hipGraph: the 6-8 launches of a solve become one graph launch, which
// removes the per-launch host cost and the dispatch gaps (what dominates small-batch latency).
// A graph is keyed by every argument that reaches a kernel; a miss captures the same launch
// sequence once.  Timing runs (events) and multi-range runs go direct.
int run_sqp_graphed(i7m_handle* h, int B, const double* d_xu_in, double* d_xu, const double* d_xs, const double* d_goals,
                    int goal_stride, ProblemStats* d_st) {
  if (!h->use_graph || h->timing)
    return run_sqp(h, B, d_xu_in, d_xu, d_xs, d_goals, goal_stride, d_st);
  const int hf = h->has_fext ? 1 : 0;
  i7m_handle::GraphEntry* hit = nullptr;
  for (auto& g : h->graphs)
    if (g.B == B && g.goal_stride == goal_stride && g.has_fext == hf && g.xu_in == d_xu_in && g.xu == d_xu && g.xs == d_xs &&
        g.goals == d_goals && g.st == d_st && g.stream == (const void*)h->stream)
      hit = &g;
  if (!hit) {
    HIPCHK(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
    const int rc = run_sqp(h, B, d_xu_in, d_xu, d_xs, d_goals, goal_stride, d_st);
    hipGraph_t graph = nullptr;
    const hipError_t e = hipStreamEndCapture(h->stream, &graph);
    if (rc) {
      if (graph) (void)hipGraphDestroy(graph);
      return rc;
    }
    if (e != hipSuccess) return fail(I7M_EHIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
    hipGraphExec_t exec = nullptr;
    const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (ei != hipSuccess) return fail(I7M_EHIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(ei));
    if (h->graphs.size() >= 4) {  // evict the least recently used
      size_t lru = 0;
      for (size_t i = 1; i < h->graphs.size(); ++i)
        if (h->graphs[i].last_use < h->graphs[lru].last_use) lru = i;
      (void)hipGraphExecDestroy(h->graphs[lru].exec);
      h->graphs.erase(h->graphs.begin() + lru);
    }
    h->graphs.push_back({B, goal_stride, hf, d_xu_in, d_xu, d_xs, d_goals, d_st, (const void*)h->stream, exec, 0});
    hit = &h->graphs.back();
  }
  hit->last_use = ++h->graph_clock;
  HIPCHK(hipGraphLaunch(hit->exec, h->stream));
  return I7M_OK;
}

// chunks of a host-to-host solve of B problems: the handle's setting, else automatic — three
// (tapered) from 3 072 problems, two from 2 048, one piece below (config 3: 1.42 -> 1.21 ms;
// at B = 1 024 one piece is fastest; DESIGN.md §5 has the A/B)
// Does a batch of B run as staggered ranges (i7m_handle::admm_stagger)?
bool stagger_applies(const i7m_handle* h, int B) {
  return ((h->stagger_modes >> h->cfg.qp_mode) & 1) && h->admm_stagger > 0 && h->admm_ranges > 1 &&
         B >= h->admm_stagger_min_b && h->dev_ranges <= 1;
}


int h2h_chunks_for(const i7m_handle* h, int B) {
  if (h->h2h_chunks > 0) return h->h2h_chunks;
  // ADMM mode where the device solve staggers: two chunks, the second's solve behind the first's
  // mark (solve_h2h_pipelined_body), i.e. the staggered halves with the copies overlapped
  if (h->cfg.qp_mode == I7M_QP_ADMM && stagger_applies(h, B)) return 2;
  return B >= 3072 ? 3 : (B >= 2048 ? 2 : 1);
}

int copy_in(i7m_handle* h, double* dst, const double* src, size_t n, hipStream_t s = nullptr) {
  if (n) HIPCHK(hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyHostToDevice, s ? s : h->stream));
  return I7M_OK;
}
int copy_out(i7m_handle* h, double* dst, const double* src, size_t n, hipStream_t s = nullptr) {
  if (n) HIPCHK(hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyDeviceToHost, s ? s : h->stream));
  return I7M_OK;
}

// Host-to-host solve in `nch` contiguous chunks of the batch, alternating over two streams: each
// chunk is H2D of its rows -> its SQP -> D2H of its rows and stats, so chunk i's solve runs while
// chunk i+1 is copied in and chunk i-1 copied out (PCIe is full duplex), instead of copy-in,
// solve, copy-out back to back.  Ordered after earlier work on h->stream; synchronous.
int solve_h2h_pipelined(i7m_handle* h, int B, const double* xu_in, const double* xcur, const double* goals,
                        int goal_stride, double* xu_out, i7m_problem_stats* stats, int nch);

int solve_h2h_chunked_body(i7m_handle* h, int B, const double* xu_in, const double* xcur, const double* goals,
                           int goal_stride, double* xu_out, i7m_problem_stats* stats, int nch) {
  const size_t T = 18 * (size_t)h->cfg.N - 6, N = h->cfg.N;
  int rc;
  HIPCHK(hipEventRecord(h->ev_order, h->stream));
  for (int c = 0; c < 2; ++c) HIPCHK(hipStreamWaitEvent(h->cs[c], h->ev_order, 0));
  for (int i = 0; i < nch; ++i) {
    const long lo = (long)B * i / nch, hi = (long)B * (i + 1) / nch;
    const int n = (int)(hi - lo);
    if (n == 0) continue;
    hipStream_t s = h->cs[i & 1];
    double* dxu = h->d_xu + lo * T;
    double* dxs = h->d_xs + lo * 12;
    double* dg = h->d_goal + lo * N * goal_stride;
    if ((rc = copy_in(h, dxu, xu_in + lo * T, n * T, s))) return rc;
    if ((rc = copy_in(h, dxs, xcur + lo * 12, (size_t)n * 12, s))) return rc;
    if ((rc = copy_in(h, dg, goals + lo * N * goal_stride, n * N * goal_stride, s))) return rc;
    if ((rc = run_sqp(h, n, dxu, dxu, dxs, dg, goal_stride, h->d_stats + lo, lo, s))) return rc;
    if ((rc = copy_out(h, xu_out + lo * T, dxu, n * T, s))) return rc;
    if (stats)
      HIPCHK(hipMemcpyAsync(stats + lo, h->d_stats + lo, sizeof(ProblemStats) * (size_t)n, hipMemcpyDeviceToHost, s));
  }
  for (int c = 0; c < 2; ++c) {
    HIPCHK(hipEventRecord(h->ev_done[c], h->cs[c]));
    HIPCHK(hipStreamWaitEvent(h->stream, h->ev_done[c], 0));
  }
  HIPCHK(hipStreamSynchronize(h->stream));
  return I7M_OK;
}

// The chunks as a three-stage pipeline: copies in on cs[0], the solves on the handle's stream
// (h2h_pipe 1) or alternating between it and cs2 (2, default: a chunk's solve can start while the
// previous one drains), copies out on cs[1]; chunk i's solve waits only for its own copy-in, its
// copy-out only for its solve.  Issued in the order in(0) solve(0) [in(i) solve(i) out(i-1)]...
// out(n-1): with pinned host memory every call returns at once and the three queues overlap; with
// pageable memory (whose copies block the calling thread until done) the host still copies chunk
// i in, and chunk i-1 out, while the device solves the chunk before.  The alternating two-stream
// layout above issued all copy-ins at once: they shared the link and finished together, then the
// solves ran, then the copy-outs — no overlap.
int solve_h2h_pipelined_body(i7m_handle* h, int B, const double* xu_in, const double* xcur, const double* goals,
                             int goal_stride, double* xu_out, i7m_problem_stats* stats, int nch) {
  const size_t T = 18 * (size_t)h->cfg.N - 6, N = h->cfg.N;
  while ((int)h->ev_in.size() < nch) {
    hipEvent_t a = nullptr, b = nullptr;
    HIPCHK(hipEventCreateWithFlags(&a, hipEventDisableTiming));
    if (hipEventCreateWithFlags(&b, hipEventDisableTiming) != hipSuccess) {
      (void)hipEventDestroy(a);
      return fail(I7M_EHIP, "chunk event creation failed");
    }
    h->ev_in.push_back(a);
    h->ev_cmp.push_back(b);
  }
  int rc;
  if (h->h2h_pipe >= 2 && !h->cs2) HIPCHK(hipStreamCreateWithFlags(&h->cs2, hipStreamNonBlocking));
  HIPCHK(hipEventRecord(h->ev_order, h->stream));
  for (int c = 0; c < 2; ++c) HIPCHK(hipStreamWaitEvent(h->cs[c], h->ev_order, 0));
  if (h->h2h_pipe >= 2) HIPCHK(hipStreamWaitEvent(h->cs2, h->ev_order, 0));
  auto sstream = [&](int i) { return (h->h2h_pipe >= 2 && (i & 1)) ? h->cs2 : h->stream; };
  // taper (default; I7M_H2H_TAPER=0 for equal chunks): the first and the last chunk half the size
  // of the others, so the copy-in before the first solve and the copy-out after the last are short
  auto lo_of = [&](int i) -> long {
    if (!h->h2h_taper || nch < 3) return (long)B * i / nch;
    if (i == 0) return 0;
    if (i == nch) return B;
    return (long)((double)B * (2 * i - 1) / (2.0 * (nch - 1)));
  };
  // (each stage keeps its status in a local: with h2h_pipe 3 out() runs on another thread)
  auto in = [&](int i) -> int {
    const long lo = lo_of(i), n = lo_of(i + 1) - lo;
    int r;
    if ((r = copy_in(h, h->d_xu + lo * T, xu_in + lo * T, n * T, h->cs[0]))) return r;
    if ((r = copy_in(h, h->d_xs + lo * 12, xcur + lo * 12, (size_t)n * 12, h->cs[0]))) return r;
    if ((r = copy_in(h, h->d_goal + lo * N * goal_stride, goals + lo * N * goal_stride, n * N * goal_stride, h->cs[0])))
      return r;
    HIPCHK(hipEventRecord(h->ev_in[i], h->cs[0]));
    return I7M_OK;
  };
  // ADMM mode where the device solve staggers, in two chunks: the second chunk's solve also waits
  // for the first's mark (its first scaling + factor), as the staggered halves of i7m_solve_device
  const bool stag = nch == 2 && h->cfg.qp_mode == I7M_QP_ADMM && stagger_applies(h, B);
  if (stag && !h->ev_rmark[0]) HIPCHK(hipEventCreateWithFlags(&h->ev_rmark[0], hipEventDisableTiming));
  bool marked0 = false;
  auto solve = [&](int i) -> int {
    const long lo = lo_of(i), n = lo_of(i + 1) - lo;
    const hipStream_t ss = sstream(i);
    HIPCHK(hipStreamWaitEvent(ss, h->ev_in[i], 0));
    if (stag && i == 1 && marked0) HIPCHK(hipStreamWaitEvent(ss, h->ev_rmark[0], 0));
    double* dxu = h->d_xu + lo * T;
    int r;
    h->mark_ev = stag && i == 0 ? h->ev_rmark[0] : nullptr;
    r = n > 0 ? run_sqp(h, (int)n, dxu, dxu, h->d_xs + lo * 12, h->d_goal + lo * N * goal_stride, goal_stride,
                        h->d_stats + lo, lo, ss)
              : I7M_OK;
    if (stag && i == 0) marked0 = !h->mark_ev;
    h->mark_ev = nullptr;
    if (r) return r;
    HIPCHK(hipEventRecord(h->ev_cmp[i], ss));
    return I7M_OK;
  };
  auto out = [&](int i) -> int {
    const long lo = lo_of(i), n = lo_of(i + 1) - lo;
    HIPCHK(hipStreamWaitEvent(h->cs[1], h->ev_cmp[i], 0));
    int r;
    if ((r = copy_out(h, xu_out + lo * T, h->d_xu + lo * T, n * T, h->cs[1]))) return r;
    if (stats && n > 0)
      HIPCHK(hipMemcpyAsync(stats + lo, h->d_stats + lo, sizeof(ProblemStats) * (size_t)n, hipMemcpyDeviceToHost,
                            h->cs[1]));
    return I7M_OK;
  };
  if (h->h2h_pipe == 3) {
    // copies out on a second host thread: a pageable copy blocks the thread that issues it, so
    // with one thread every copy-out sat between two copy-ins and the link ran one direction at a
    // time; here the calling thread issues in(0) solve(0) in(1) solve(1) ... back to back while the
    // helper issues out(i) as soon as solve(i) has been issued (it then blocks in the copy until
    // the solve and the copy are done) — both directions of the link in flight together
    std::atomic<int> issued{0};
    int rc_out = I7M_OK;
    std::string err_out;
    std::thread helper([&] {
      if (hipSetDevice(h->dev) != hipSuccess) {
        rc_out = I7M_EHIP;
        err_out = "hipSetDevice failed (copy-out thread)";
        return;
      }
      int r = I7M_OK;
      for (int i = 0; i < nch && r == I7M_OK; ++i) {
        int k;
        while ((k = issued.load(std::memory_order_acquire)) <= i) {
          if (k < 0) return;  // the calling thread failed: nothing more to copy
          std::this_thread::yield();
        }
        r = out(i);
      }
      if (r != I7M_OK) {
        rc_out = r;
        err_out = g_err;  // thread_local: hand the message to the calling thread
      }
    });
    int r = I7M_OK;
    for (int i = 0; i < nch && r == I7M_OK; ++i) {
      if ((r = in(i)) == I7M_OK && (r = solve(i)) == I7M_OK) issued.store(i + 1, std::memory_order_release);
    }
    if (r != I7M_OK) issued.store(-1, std::memory_order_release);
    helper.join();
    if (r != I7M_OK) return r;
    if (rc_out != I7M_OK) return fail(rc_out, err_out);
  } else {
    if ((rc = in(0)) || (rc = solve(0))) return rc;
    for (int i = 1; i < nch; ++i)
      if ((rc = in(i)) || (rc = solve(i)) || (rc = out(i - 1))) return rc;
    if ((rc = out(nch - 1))) return rc;
  }
  HIPCHK(hipEventRecord(h->ev_done[1], h->cs[1]));
  HIPCHK(hipStreamWaitEvent(h->stream, h->ev_done[1], 0));
  HIPCHK(hipStreamSynchronize(h->stream));
  return I7M_OK;
}

// Error exit of a chunked call: chunks already queued on cs[0], cs[1] and cs2 keep
// running after a failed call returns, and their copies out could land in caller memory after the
// error (or race the next call's copies in, which order only after h->stream).  So every error
// return waits for all the streams the chunks use (their own errors ignored; the first message kept).
int drain_after_error(i7m_handle* h, int rc) {
  if (rc == I7M_OK) return rc;
  const std::string msg = g_err;
  for (int c = 0; c < 2; ++c)
    if (h->cs[c]) (void)hipStreamSynchronize(h->cs[c]);
  if (h->cs2) (void)hipStreamSynchronize(h->cs2);
  for (int r = 2; r < i7m_handle::kMaxRanges; ++r)  // the staggered ranges' own streams
    if (h->rs[r]) (void)hipStreamSynchronize(h->rs[r]);
  (void)hipStreamSynchronize(h->stream);
  g_err = msg;
  return rc;
}
int solve_h2h_pipelined(i7m_handle* h, int B, const double* xu_in, const double* xcur, const double* goals,
                        int goal_stride, double* xu_out, i7m_problem_stats* stats, int nch) {
  return drain_after_error(h, solve_h2h_pipelined_body(h, B, xu_in, xcur, goals, goal_stride, xu_out, stats, nch));
}
int solve_h2h_chunked(i7m_handle* h, int B, const double* xu_in, const double* xcur, const double* goals, int goal_stride,
                      double* xu_out, i7m_problem_stats* stats, int nch) {
  if (h->h2h_pipe) return solve_h2h_pipelined(h, B, xu_in, xcur, goals, goal_stride, xu_out, stats, nch);
  return drain_after_error(h, solve_h2h_chunked_body(h, B, xu_in, xcur, goals, goal_stride, xu_out, stats, nch));
}

}  // namespace

extern "C" {

const char* i7m_last_error(void) { return g_err.c_str(); }

#ifdef I7M_DIAG
// Diagnostic library only (not declared in include/indy7_mpc.h): point every instrumented
// kernel of both translation units at a per-wave timeline buffer (i7m_timeline.h; nullptr: off).
int i7m_lin_tu_set_timeline(void* p);
int i7m_admm_prep_tu_set_timeline(void* p);
int i7m_diag_timeline(void* p) {
  return (i7m::tl_set(p) == 0 && i7m_lin_tu_set_timeline(p) == 0 && i7m_admm_prep_tu_set_timeline(p) == 0) ? 0 : -1;
}
#endif

int i7m_abi_version(void) { return I7M_ABI_VERSION; }

const char* i7m_version(void) { return "indy7_mpc_amd 0.3 (gfx950, fp64, " I7M_BUILD_KIND ") src " I7M_SRC_HASH; }

int i7m_device_count(int* n) {
  if (!n) return fail(I7M_EINVAL, "null");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    *n = 0;
    return fail(I7M_ENODEV, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
  }
  *n = c;
  return I7M_OK;
}

int i7m_config_default(i7m_config* c) {
  if (!c) return fail(I7M_EINVAL, "null config");
  i7m_model keep = c->model;
  std::memset(c, 0, sizeof(*c));
  c->model = keep;
  c->N = 32;
  c->regularize = 1;
  c->dt = 0.01;
  c->dQ_cost = 0.01;
  c->R_cost = 1e-5;
  c->QN_cost = 100.0;
  c->eps = 1.0;
  c->mu = 10.0;
  c->step_tol = 1e-3;
  c->max_sqp_iters = 2;
  c->max_batch = 1;
  c->device_id = 0;
  c->qp_mode = I7M_QP_DIRECT;
  c->box_mask = I7M_BOX_Q | I7M_BOX_V | I7M_BOX_U;
  c->box_max_iters = 30;
  c->box_tol = 1e-8;
  // OSQP's defaults, with the duality-gap test and no rho adaptation: the settings that reproduce
  // the reference's printed closed loop (oracle/osqp_admm.py)
  c->admm_rho = 0.1;
  c->admm_sigma = 1e-6;
  c->admm_alpha = 1.6;
  c->admm_eps_abs = 1e-3;
  c->admm_eps_rel = 1e-3;
  c->admm_max_iter = 4000;
  c->admm_check_termination = 25;
  c->admm_scaling = 10;
  c->admm_check_dualgap = 1;
  c->admm_adaptive_rho_interval = 0;
  c->admm_adaptive_rho_tolerance = 5.0;
  c->precision = I7M_PREC_F64;
  return I7M_OK;
}

int i7m_create(const i7m_config* cfg, i7m_handle** out) {
  if (!cfg || !out) return fail(I7M_EINVAL, "null argument");
  *out = nullptr;
  if (cfg->N < 2 || cfg->N > I7M_MAX_N) return fail(I7M_EINVAL, "N must be in [2, 64]");
  if (cfg->max_batch < 1) return fail(I7M_EINVAL, "max_batch must be >= 1");
  if (cfg->precision != I7M_PREC_F64)
    return fail(I7M_EINVAL, cfg->precision == I7M_PREC_F32
                                ? "precision I7M_PREC_F32 is not built: every kernel computes in double (I7M_PREC_F64)"
                                : "unknown precision");
  if (cfg->max_sqp_iters < 1 || cfg->max_sqp_iters > I7M_MAX_SQP) return fail(I7M_EINVAL, "max_sqp_iters in [1, 8]");
  if (cfg->qp_mode != I7M_QP_DIRECT && cfg->qp_mode != I7M_QP_BOX && cfg->qp_mode != I7M_QP_ADMM)
    return fail(I7M_EINVAL, "unsupported qp_mode");
  if (cfg->qp_mode == I7M_QP_ADMM) {
    if (!(cfg->admm_rho > 0.0) || !(cfg->admm_sigma > 0.0)) return fail(I7M_EINVAL, "admm_rho and admm_sigma must be > 0");
    if (!(cfg->admm_alpha > 0.0 && cfg->admm_alpha < 2.0)) return fail(I7M_EINVAL, "admm_alpha must be in (0, 2)");
    if (!(cfg->admm_eps_abs >= 0.0) || !(cfg->admm_eps_rel >= 0.0)) return fail(I7M_EINVAL, "admm eps must be >= 0");
    if (cfg->admm_max_iter < 1 || cfg->admm_max_iter > 1000000) return fail(I7M_EINVAL, "admm_max_iter in [1, 1e6]");
    if (cfg->admm_check_termination < 0 || cfg->admm_scaling < 0 || cfg->admm_scaling > 100 ||
        cfg->admm_adaptive_rho_interval < 0)
      return fail(I7M_EINVAL, "admm_check_termination / admm_adaptive_rho_interval >= 0, admm_scaling in [0, 100]");
    if (!(cfg->admm_adaptive_rho_tolerance >= 1.0)) return fail(I7M_EINVAL, "admm_adaptive_rho_tolerance must be >= 1");
  }
  if (cfg->pipeline < I7M_PIPE_AUTO || cfg->pipeline > I7M_PIPE_FUSED_ITER) return fail(I7M_EINVAL, "unsupported pipeline");
  if (cfg->qp_mode == I7M_QP_BOX) {
    if (cfg->box_mask < 0 || cfg->box_mask > 7) return fail(I7M_EINVAL, "box_mask must be a subset of Q|V|U (0..7)");
    if (cfg->box_max_iters < 1 || cfg->box_max_iters > 200) return fail(I7M_EINVAL, "box_max_iters in [1, 200]");
    if (!(cfg->box_tol > 0.0)) return fail(I7M_EINVAL, "box_tol must be > 0");
  }
  if (!(cfg->dt > 0.0)) return fail(I7M_EINVAL, "dt must be > 0");
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) return fail(I7M_ENODEV, "no HIP device available");
  if (cfg->device_id < 0 || cfg->device_id >= ndev) return fail(I7M_EINVAL, "device_id out of range");
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, cfg->device_id));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(I7M_ENODEV, std::string("built for gfx950, device is ") + prop.gcnArchName);

  i7m_handle* h = new i7m_handle();
  h->cfg = *cfg;
  h->dev = cfg->device_id;
  auto bail = [&](int rc) {
    i7m_destroy(h);
    return rc;
  };
  if (hipSetDevice(h->dev) != hipSuccess) return bail(fail(I7M_EHIP, "hipSetDevice failed"));
  // the handle's own stream is a blocking one: it orders with the legacy null stream, so a caller
  // that fills the inputs on the default (null) stream and never calls i7m_set_stream still has
  // its copies ordered before the solve and the solve before its reads
  if (hipStreamCreateWithFlags(&h->own, hipStreamDefault) != hipSuccess)
    return bail(fail(I7M_EHIP, "hipStreamCreate failed"));
  h->stream = h->own;
#ifdef I7M_DIAG
  if (const char* e = std::getenv("I7M_ABLATE")) h->ablate = std::atoi(e);
#else
  if (std::getenv("I7M_ABLATE"))
    return bail(fail(I7M_EINVAL, "I7M_ABLATE is set, but this is the release library: the ablation "
                                 "timing kernels exist only in the -DI7M_DIAG build (tools/)"));
#endif
  if (const char* e = std::getenv("I7M_IPM"))
    h->ipm_mode = std::strcmp(e, "split") == 0 ? 2 : (std::strcmp(e, "delta") == 0 ? 0 : 1);
  if (const char* e = std::getenv("I7M_LS_TAIL")) h->ls_tail = std::min(std::max(std::atoi(e), 0), 3);
  if (const char* e = std::getenv("I7M_LS_WAVES")) h->ls_waves = std::atoi(e) == 4 ? 4 : (std::atoi(e) == 2 ? 2 : 1);
  if (const char* e = std::getenv("I7M_GRAPH")) h->use_graph = std::atoi(e) != 0;
  if (const char* e = std::getenv("I7M_RIC_W2")) h->ric_w2 = std::atoi(e) != 0;
  if (const char* e = std::getenv("I7M_RIC_BC")) {
    const int v = std::atoi(e) & 7;
    h->ric_bc = (v == 4 || v == 5) ? (v & 3) : v;  // instantiated: 0 1 2 3 6 7
  }
  h->h2h_chunks = cfg->h2h_chunks;
  if (const char* e = std::getenv("I7M_H2H_CHUNKS")) h->h2h_chunks = std::atoi(e);
  if (const char* e = std::getenv("I7M_H2H_PIPE")) h->h2h_pipe = std::min(std::max(std::atoi(e), 0), 3);
  if (const char* e = std::getenv("I7M_H2H_TAPER")) h->h2h_taper = std::atoi(e) != 0;
  if (const char* e = std::getenv("I7M_ADMM_CHUNK")) h->admm_chunk = std::max(std::atoi(e), 0);
  if (const char* e = std::getenv("I7M_DEV_RANGES")) h->dev_ranges = std::min(std::max(std::atoi(e), 0), 64);
  if (const char* e = std::getenv("I7M_ADMM_STAGGER")) h->admm_stagger = std::min(std::max(std::atoi(e), 0), 4);
  if (const char* e = std::getenv("I7M_ADMM_STAGGER_MIN_B")) h->admm_stagger_min_b = std::max(std::atoi(e), 2);
  if (const char* e = std::getenv("I7M_ADMM_SPLIT")) h->admm_split = std::min(std::max(std::atoi(e), 100), 900);
  if (const char* e = std::getenv("I7M_STAGGER_MODES")) h->stagger_modes = std::atoi(e);
  if (const char* e = std::getenv("I7M_ADMM_RANGES"))
    h->admm_ranges = std::min(std::max(std::atoi(e), 1), (int)i7m_handle::kMaxRanges);
  if (const char* e = std::getenv("I7M_ADMM_CHAINS")) h->admm_chains = std::min(std::max(std::atoi(e), 1), 2);
  if (const char* e = std::getenv("I7M_ADMM_ITER2")) h->admm_iter2 = std::min(std::max(std::atoi(e), -1), 1);
  if (const char* e = std::getenv("I7M_ADMM_RES")) h->admm_res = std::min(std::max(std::atoi(e), -1), 1);
  if (const char* e = std::getenv("I7M_ADMM_RES_MAX")) h->admm_res_max = std::max(std::atoi(e), 0);
  if (const char* e = std::getenv("I7M_ADMM_PREP_ILP")) h->admm_prep_ilp = std::min(std::max(std::atoi(e), -1), 1);
  if (const char* e = std::getenv("I7M_ADMM_PREP_ILP_MAX")) h->admm_prep_ilp_max = std::max(std::atoi(e), 0);
  if (const char* e = std::getenv("I7M_ADMM_ITER_DYN_LDS")) h->admm_iter_dyn_lds = std::min(std::max(std::atoi(e), 0), 65536);
  if (h->h2h_chunks < 0 || h->h2h_chunks > 64) return bail(fail(I7M_EINVAL, "h2h_chunks must be in [0, 64]"));
  if (hipStreamCreateWithFlags(&h->cs[0], hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&h->cs[1], hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_order, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_done[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_done[1], hipEventDisableTiming) != hipSuccess)
    return bail(fail(I7M_EHIP, "chunk stream / event creation failed"));
  h->pipeline = cfg->pipeline;
  if (const char* e = std::getenv("I7M_PIPE"))
    h->pipeline = std::strcmp(e, "fused") == 0 ? I7M_PIPE_FUSED
                   : std::strcmp(e, "fused_iter") == 0 ? I7M_PIPE_FUSED_ITER
                   : std::strcmp(e, "split") == 0 ? I7M_PIPE_SPLIT
                   : h->pipeline;
  if (h->pipeline == I7M_PIPE_FUSED || h->pipeline == I7M_PIPE_FUSED_ITER) {
    const hipError_t ef = i7m_prepare_sqp_fused(h->dev, cfg->N);
    if (ef != hipSuccess) return bail(fail(I7M_EHIP, std::string("k_sqp_fused LDS limit: ") + hipGetErrorString(ef)));
  }
  const size_t Bm = (size_t)cfg->max_batch, N = (size_t)cfg->N, T = 18 * N - 6;
  // scratch for the query hooks: >= 114 doubles for each of >= 256 queries
  const size_t scratch = std::max(Bm * T, (size_t)256 * 114);
  auto alloc = [&](void** p, size_t bytes) -> bool { return hipMalloc(p, bytes ? bytes : 8) == hipSuccess; };
  bool ok = alloc((void**)&h->d_model, sizeof(DevModel)) && alloc((void**)&h->d_xu, Bm * T * 8) &&
            alloc((void**)&h->d_xs, Bm * 12 * 8) && alloc((void**)&h->d_goal, Bm * N * 6 * 8) &&
            alloc((void**)&h->d_sol, scratch * 8) && alloc((void**)&h->d_lin, Bm * (N - 1) * LIN_STRIDE * 8) &&
            alloc((void**)&h->d_cost, Bm * N * COST_STRIDE * 8) &&
            alloc((void**)&h->d_kbuf, Bm * (N - 1) * KBUF_STRIDE * 8) && alloc((void**)&h->d_aux, scratch * 8) &&
            alloc((void**)&h->d_qpd, Bm * (N - 1) * QPD_STRIDE * 8) &&
            alloc((void**)&h->d_out, scratch * 8) &&
            alloc((void**)&h->d_active, Bm * sizeof(int)) && alloc((void**)&h->d_stats, Bm * sizeof(ProblemStats)) &&
            alloc((void**)&h->d_fext, Bm * 6 * 8) && alloc((void**)&h->d_lsbase, Bm * 8) &&
            alloc((void**)&h->d_lspend, Bm * sizeof(int));
  if (ok && cfg->qp_mode == I7M_QP_BOX)
    ok = alloc((void**)&h->d_bx, Bm * T * 8) && alloc((void**)&h->d_bzl, Bm * T * 8) &&
         alloc((void**)&h->d_bzu, Bm * T * 8) && alloc((void**)&h->d_bsig, Bm * T * 8) &&
         alloc((void**)&h->d_bh, Bm * T * 8) && alloc((void**)&h->d_bdxa, Bm * T * 8) &&
         alloc((void**)&h->d_bhinv, Bm * (N - 1) * 36 * 8) && alloc((void**)&h->d_bdh, Bm * T * 8) &&
         alloc((void**)&h->d_bst, Bm * sizeof(IpmState)) && alloc((void**)&h->d_bact, Bm * sizeof(int));
  if (ok && cfg->qp_mode == I7M_QP_ADMM) {
    // k_admm_iter addresses the allocation with 32-bit byte offsets below its 0x7ff00000 marker
    if (admm_doubles((long)Bm, (long)N) * 8 >= 0x7ff00000ull)
      return bail(fail(I7M_EINVAL, "ADMM mode: max_batch=" + std::to_string(cfg->max_batch) + " at N=" + std::to_string(N) +
                                       " needs over 2 GiB of ADMM state; use a smaller max_batch per handle"));
    ok = alloc((void**)&h->d_admm, admm_doubles((long)Bm, (long)N) * 8) &&
         alloc((void**)&h->d_admm_it, 2 * Bm * I7M_MAX_SQP * sizeof(int));
    h->cfg.qp_mode = I7M_QP_ADMM;
    if (ok && i7m_admm_reset(h, cfg->max_batch, I7M_ADMM_RESET_ALL) != I7M_OK) ok = false;
  }
  if (!ok) return bail(fail(I7M_ENOMEM, "hipMalloc failed for max_batch=" + std::to_string(cfg->max_batch)));
  DevModel dm = make_dev_model(cfg->model);
  // the Indy7-specialised kernels are used only for a model bit-identical to the baked one
  h->spec = std::memcmp(&dm, &kIndy7Model, sizeof(DevModel)) == 0;
  if (const char* e = std::getenv("I7M_GENERIC")) h->spec = h->spec && std::atoi(e) == 0;
  if (hipMemcpy(h->d_model, &dm, sizeof(dm), hipMemcpyHostToDevice) != hipSuccess)
    return bail(fail(I7M_EHIP, "model upload failed"));
  *out = h;
  return I7M_OK;
}

void i7m_destroy(i7m_handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->dev);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  void* bufs[] = {h->d_model, h->d_xu, h->d_xs, h->d_goal, h->d_sol, h->d_lin, h->d_cost,
                  h->d_kbuf, h->d_aux, h->d_out, h->d_active, h->d_stats, h->d_fext, h->d_qpd, h->d_lsbase, h->d_lspend,
                  h->d_bx, h->d_bzl, h->d_bzu, h->d_bsig, h->d_bh, h->d_bdxa, h->d_bst, h->d_bact,
                  h->d_bhinv, h->d_bdh, h->d_admm, h->d_admm_it};
  for (void* p : bufs)
    if (p) (void)hipFree(p);
  for (auto& t : h->ev) {
    (void)hipEventDestroy(t.a);
    (void)hipEventDestroy(t.b);
  }
  for (auto e : h->pool) (void)hipEventDestroy(e);
  for (auto e : h->ev_in) (void)hipEventDestroy(e);
  for (auto e : h->ev_cmp) (void)hipEventDestroy(e);
  drop_graphs(h);
  if (h->cs2) {
    (void)hipStreamSynchronize(h->cs2);
    (void)hipStreamDestroy(h->cs2);
  }
  for (int c = 0; c < 2; ++c) {
    if (h->cs[c]) {
      (void)hipStreamSynchronize(h->cs[c]);
      (void)hipStreamDestroy(h->cs[c]);
    }
    if (h->ev_done[c]) (void)hipEventDestroy(h->ev_done[c]);
  }
  if (h->ev_order) (void)hipEventDestroy(h->ev_order);
  for (int r = 0; r < i7m_handle::kMaxRanges; ++r) {
    if (h->rs[r]) {
      (void)hipStreamSynchronize(h->rs[r]);
      (void)hipStreamDestroy(h->rs[r]);
    }
    if (h->ev_rmark[r]) (void)hipEventDestroy(h->ev_rmark[r]);
    if (h->ev_rdone[r]) (void)hipEventDestroy(h->ev_rdone[r]);
  }
  if (h->own) (void)hipStreamDestroy(h->own);
  delete h;
}

int i7m_set_stream(i7m_handle* h, void* stream) {
  if (!h) return fail(I7M_EINVAL, "null handle");
  h->stream = stream ? (hipStream_t)stream : h->own;
  return I7M_OK;
}

int i7m_set_external_wrench(i7m_handle* h, int32_t B, const double* fext, int32_t frame) {
  if (!h) return fail(I7M_EINVAL, "null handle");
  if (!fext) {
    h->has_fext = false;
    drop_graphs(h);  // captured graphs hold the wrench kernel choice
    return I7M_OK;
  }
  if (frame != I7M_WRENCH_LOCAL && frame != I7M_WRENCH_WORLD)
    return fail(I7M_EINVAL, "frame must be I7M_WRENCH_LOCAL or I7M_WRENCH_WORLD");
  if (B < 1 || B > h->cfg.max_batch) return fail(I7M_EINVAL, "external wrench batch outside [1, max_batch]");
  HIPCHK(hipSetDevice(h->dev));
  HIPCHK(hipMemsetAsync(h->d_fext, 0, (size_t)h->cfg.max_batch * 6 * 8, h->stream));
  HIPCHK(hipMemcpyAsync(h->d_fext, fext, (size_t)B * 6 * 8, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->has_fext = true;
  h->fext_frame = frame;
  // captured graphs hold the old wrench pointer / kernel choice
  drop_graphs(h);
  return I7M_OK;
}

int i7m_reset(i7m_handle* h) {
  if (!h) return fail(I7M_EINVAL, "null handle");
  HIPCHK(hipSetDevice(h->dev));
  HIPCHK(hipStreamSynchronize(h->stream));
  drop_graphs(h);
  if (h->cfg.qp_mode == I7M_QP_ADMM) {
    const int rc = i7m_admm_reset(h, h->cfg.max_batch, I7M_ADMM_RESET_ALL);
    if (rc) return rc;
  }
  return i7m_reset_kernel_times(h);
}

int i7m_admm_reset(i7m_handle* h, int32_t B, int32_t what) {
  if (!h) return fail(I7M_EINVAL, "null handle");
  if (h->cfg.qp_mode != I7M_QP_ADMM) return fail(I7M_EINVAL, "handle is not in I7M_QP_ADMM mode");
  if (B < 0 || B > h->cfg.max_batch) return fail(I7M_EINVAL, "batch outside [0, max_batch]");
  if (what & ~I7M_ADMM_RESET_ALL) return fail(I7M_EINVAL, "unknown I7M_ADMM_RESET_* bits");
  if (B == 0) return I7M_OK;
  HIPCHK(hipSetDevice(h->dev));
  const long N = h->cfg.N, T = 18 * N - 6, m = 12 * N;
  const AdmmArgs a = admm_layout(h->d_admm, h->d_admm_it, h->cfg.max_batch, N, 0);
  if (what & I7M_ADMM_RESET_PRIMAL) {
    HIPCHK(hipMemsetAsync(a.sx, 0, (size_t)B * T * 8, h->stream));
    HIPCHK(hipMemsetAsync(a.sz, 0, (size_t)B * m * 8, h->stream));
    HIPCHK(hipMemsetAsync(a.sq, 0, (size_t)B * T * 8, h->stream));
  }
  if (what & I7M_ADMM_RESET_DUAL) HIPCHK(hipMemsetAsync(a.sy, 0, (size_t)B * m * 8, h->stream));
  if (what & I7M_ADMM_RESET_RHO) {
    std::vector<double> r((size_t)B, h->cfg.admm_rho);
    HIPCHK(hipMemcpyAsync(a.srho, r.data(), (size_t)B * 8, hipMemcpyHostToDevice, h->stream));
  }
  HIPCHK(hipMemsetAsync(a.iters, 0xff, (size_t)B * I7M_MAX_SQP * sizeof(int), h->stream));
  HIPCHK(hipMemsetAsync(a.status, 0xff, (size_t)B * I7M_MAX_SQP * sizeof(int), h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return I7M_OK;
}

int i7m_get_admm_stats(i7m_handle* h, int32_t B, int32_t* iters, double* rho) {
  if (!h) return fail(I7M_EINVAL, "null handle");
  if (h->cfg.qp_mode != I7M_QP_ADMM) return fail(I7M_EINVAL, "handle is not in I7M_QP_ADMM mode");
  if (B < 0 || B > h->cfg.max_batch) return fail(I7M_EINVAL, "batch outside [0, max_batch]");
  if (B == 0) return I7M_OK;
  HIPCHK(hipSetDevice(h->dev));
  const AdmmArgs a = admm_layout(h->d_admm, h->d_admm_it, h->cfg.max_batch, h->cfg.N, 0);
  if (iters) HIPCHK(hipMemcpyAsync(iters, a.iters, (size_t)B * I7M_MAX_SQP * sizeof(int), hipMemcpyDeviceToHost, h->stream));
  if (rho) HIPCHK(hipMemcpyAsync(rho, a.srho, (size_t)B * 8, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return I7M_OK;
}

int i7m_get_admm_status(i7m_handle* h, int32_t B, int32_t* status) {
  if (!h || !status) return fail(I7M_EINVAL, "null handle or output");
  if (h->cfg.qp_mode != I7M_QP_ADMM) return fail(I7M_EINVAL, "handle is not in I7M_QP_ADMM mode");
  if (B < 0 || B > h->cfg.max_batch) return fail(I7M_EINVAL, "batch outside [0, max_batch]");
  if (B == 0) return I7M_OK;
  HIPCHK(hipSetDevice(h->dev));
  const AdmmArgs a = admm_layout(h->d_admm, h->d_admm_it, h->cfg.max_batch, h->cfg.N, 0);
  HIPCHK(hipMemcpyAsync(status, a.status, (size_t)B * I7M_MAX_SQP * sizeof(int), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return I7M_OK;
}

int i7m_get_admm_dual(i7m_handle* h, int32_t B, double* y) {
  if (!h || !y) return fail(I7M_EINVAL, "null handle or output");
  if (h->cfg.qp_mode != I7M_QP_ADMM) return fail(I7M_EINVAL, "handle is not in I7M_QP_ADMM mode");
  if (B < 0 || B > h->cfg.max_batch) return fail(I7M_EINVAL, "batch outside [0, max_batch]");
  if (B == 0) return I7M_OK;
  HIPCHK(hipSetDevice(h->dev));
  const long m = 12 * (long)h->cfg.N;
  const AdmmArgs a = admm_layout(h->d_admm, h->d_admm_it, h->cfg.max_batch, h->cfg.N, 0);
  std::vector<double> e((size_t)B * m), c((size_t)B);
  int rc;
  if ((rc = copy_out(h, y, a.sy, (size_t)B * m)) || (rc = copy_out(h, e.data(), a.E, (size_t)B * m)) ||
      (rc = copy_out(h, c.data(), a.cs, (size_t)B)))
    return rc;
  HIPCHK(hipStreamSynchronize(h->stream));
  // OSQP's unscale_solution: y = E y_s / c, with the scaling of each problem's last QP
  for (long b = 0; b < B; ++b)
    for (long r = 0; r < m; ++r) y[b * m + r] = e[b * m + r] * y[b * m + r] / c[b];
  return I7M_OK;
}

int i7m_get_admm_state(i7m_handle* h, int32_t B, double* x, double* z, double* y, double* q, double* rho) {
  if (!h) return fail(I7M_EINVAL, "null handle");
  if (h->cfg.qp_mode != I7M_QP_ADMM) return fail(I7M_EINVAL, "handle is not in I7M_QP_ADMM mode");
  if (B < 0 || B > h->cfg.max_batch) return fail(I7M_EINVAL, "batch outside [0, max_batch]");
  if (B == 0) return I7M_OK;
  HIPCHK(hipSetDevice(h->dev));
  const long N = h->cfg.N, T = 18 * N - 6, m = 12 * N;
  const AdmmArgs a = admm_layout(h->d_admm, h->d_admm_it, h->cfg.max_batch, N, 0);
  int rc;
  if (x && (rc = copy_out(h, x, a.sx, (size_t)B * T))) return rc;
  if (z && (rc = copy_out(h, z, a.sz, (size_t)B * m))) return rc;
  if (y && (rc = copy_out(h, y, a.sy, (size_t)B * m))) return rc;
  if (q && (rc = copy_out(h, q, a.sq, (size_t)B * T))) return rc;
  if (rho && (rc = copy_out(h, rho, a.srho, (size_t)B))) return rc;
  HIPCHK(hipStreamSynchronize(h->stream));
  return I7M_OK;
}

int i7m_synchronize(i7m_handle* h) {
  if (!h) return fail(I7M_EINVAL, "null handle");
  HIPCHK(hipStreamSynchronize(h->stream));
  return I7M_OK;
}

extern "C++" {  // (C++ helpers inside the C-ABI block)
// The batch as h->admm_ranges contiguous ranges, each on a stream of its own and started when
// the range before it has passed its mark (the first run_sqp of its `body` records it; see
// i7m_handle::admm_stagger), every range forked from and joined back into h->stream.
// body(lo, n, stream) enqueues the work of problems [lo, lo + n).  Results are the one-range
// run's: the problems are independent.
template <class Body>
static int run_staggered(i7m_handle* h, int B, Body&& body) {
  const int R = h->admm_ranges;
  hipStream_t ss[i7m_handle::kMaxRanges];
  for (int r = 0; r < R; ++r) {
    if (r < 2) {
      ss[r] = h->cs[r];
    } else {
      if (!h->rs[r]) HIPCHK(hipStreamCreateWithFlags(&h->rs[r], hipStreamNonBlocking));
      ss[r] = h->rs[r];
    }
    if (!h->ev_rmark[r]) HIPCHK(hipEventCreateWithFlags(&h->ev_rmark[r], hipEventDisableTiming));
    if (!h->ev_rdone[r]) HIPCHK(hipEventCreateWithFlags(&h->ev_rdone[r], hipEventDisableTiming));
  }
  // range boundaries, clamped to [0, B] (the rounded split of a small B or an extreme
  // I7M_ADMM_SPLIT must not run past the batch); an empty range is skipped
  auto cut = [&](int q) {
    const long c = R == 2 && q == 1 ? ((long)B * h->admm_split / 1000 + 3) / 4 * 4 : (long)B * q / R;
    return std::min<long>(std::max<long>(c, 0), B);
  };
  HIPCHK(hipEventRecord(h->ev_order, h->stream));
  // range r starts behind range r - C's mark (C = admm_chains: 1 one chain of ranges, 2 two
  // interleaved chains started together)
  const int C = std::min(h->admm_chains, R);
  bool marked[i7m_handle::kMaxRanges] = {};
  for (int r = 0; r < R; ++r) {
    const long lo = cut(r), hi = cut(r + 1);
    HIPCHK(hipStreamWaitEvent(ss[r], h->ev_order, 0));
    if (hi <= lo) continue;
    if (r >= C && marked[r - C]) HIPCHK(hipStreamWaitEvent(ss[r], h->ev_rmark[r - C], 0));
    h->mark_ev = r + C < R ? h->ev_rmark[r] : nullptr;
    const int rc = body(lo, (int)(hi - lo), ss[r]);
    marked[r] = r + C < R && !h->mark_ev;
    h->mark_ev = nullptr;
    if (rc) {
      // join the ranges already started back into h->stream before the error returns:
      // the caller's cleanup after a synchronize of h->stream must not race them
      const std::string msg = g_err;
      for (int q = 0; q <= r; ++q) {
        (void)hipEventRecord(h->ev_rdone[q], ss[q]);
        (void)hipStreamWaitEvent(h->stream, h->ev_rdone[q], 0);
      }
      g_err = msg;
      return rc;
    }
  }
  for (int r = 0; r < R; ++r) {
    HIPCHK(hipEventRecord(h->ev_rdone[r], ss[r]));
    HIPCHK(hipStreamWaitEvent(h->stream, h->ev_rdone[r], 0));
  }
  return I7M_OK;
}
}  // extern "C++"

int i7m_solve_device(i7m_handle* h, int32_t B, const double* d_xu_in, const double* d_xcur, const double* d_goals,
                     int32_t goal_stride, double* d_xu_out, i7m_problem_stats* d_stats) {
  int rc = check_batch(h, B, goal_stride);
  if (rc) return rc;
  if (B == 0) return I7M_OK;
  if (!d_xu_in || !d_xcur || !d_goals || !d_xu_out) return fail(I7M_EINVAL, "null device pointer");
  HIPCHK(hipSetDevice(h->dev));
  ProblemStats* st = d_stats ? reinterpret_cast<ProblemStats*>(d_stats) : h->d_stats;
  if (stagger_applies(h, B)) {
    const size_t T = 18 * (size_t)h->cfg.N - 6, N = h->cfg.N;
    return run_staggered(h, B, [&](long lo, int n, hipStream_t s) {
      return run_sqp(h, n, d_xu_in + lo * T, d_xu_out + lo * T, d_xcur + lo * 12, d_goals + lo * N * goal_stride,
                     goal_stride, st + lo, lo, s);
    });
  }
  if (h->dev_ranges > 1 && B >= h->dev_ranges) {
    // A/B knob (I7M_DEV_RANGES): the batch as contiguous ranges on the two chunk streams, so one
    // range's kernels can fill the SIMDs another range's kernel tail leaves idle
    const size_t T = 18 * (size_t)h->cfg.N - 6, N = h->cfg.N;
    HIPCHK(hipEventRecord(h->ev_order, h->stream));
    for (int c = 0; c < 2; ++c) HIPCHK(hipStreamWaitEvent(h->cs[c], h->ev_order, 0));
    for (int i = 0; i < h->dev_ranges; ++i) {
      const long lo = (long)B * i / h->dev_ranges, hi = (long)B * (i + 1) / h->dev_ranges;
      if ((rc = run_sqp(h, (int)(hi - lo), d_xu_in + lo * T, d_xu_out + lo * T, d_xcur + lo * 12,
                        d_goals + lo * N * goal_stride, goal_stride, st + lo, lo, h->cs[i & 1])))
        return rc;
    }
    for (int c = 0; c < 2; ++c) {
      HIPCHK(hipEventRecord(h->ev_done[c], h->cs[c]));
      HIPCHK(hipStreamWaitEvent(h->stream, h->ev_done[c], 0));
    }
    return I7M_OK;
  }
  return run_sqp_graphed(h, B, d_xu_in, d_xu_out, d_xcur, d_goals, goal_stride, st);
}

int i7m_solve(i7m_handle* h, int32_t B, const double* xu_in, const double* xcur, const double* goals,
              int32_t goal_stride, double* xu_out, i7m_problem_stats* stats) {
  int rc = check_batch(h, B, goal_stride);
  if (rc) return rc;
  if (B == 0) return I7M_OK;
  if (!xu_in || !xcur || !goals || !xu_out) return fail(I7M_EINVAL, "null pointer");
  HIPCHK(hipSetDevice(h->dev));
  const size_t T = 18 * (size_t)h->cfg.N - 6, N = h->cfg.N;
  const int nch = std::min(h2h_chunks_for(h, B), B);
  if (nch > 1) return solve_h2h_chunked(h, B, xu_in, xcur, goals, goal_stride, xu_out, stats, nch);
  if ((rc = copy_in(h, h->d_xu, xu_in, (size_t)B * T))) return rc;
  if ((rc = copy_in(h, h->d_xs, xcur, (size_t)B * 12))) return rc;
  if ((rc = copy_in(h, h->d_goal, goals, (size_t)B * N * goal_stride))) return rc;
  if ((rc = run_sqp_graphed(h, B, h->d_xu, h->d_xu, h->d_xs, h->d_goal, goal_stride, h->d_stats))) return rc;
  if ((rc = copy_out(h, xu_out, h->d_xu, (size_t)B * T))) return rc;
  if (stats)
    HIPCHK(hipMemcpyAsync(stats, h->d_stats, sizeof(ProblemStats) * (size_t)B, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return I7M_OK;
}

int i7m_qp(i7m_handle* h, int32_t B, const double* xu, const double* xcur, const double* goals, int32_t goal_stride,
           double* sol) {
  int rc = check_batch(h, B, goal_stride);
  if (rc) return rc;
  if (B == 0) return I7M_OK;
  if (!xu || !xcur || !goals || !sol) return fail(I7M_EINVAL, "null pointer");
  HIPCHK(hipSetDevice(h->dev));
  const size_t T = 18 * (size_t)h->cfg.N - 6, N = h->cfg.N;
  SolveParams P = params_of(h, B, goal_stride);
  if ((rc = copy_in(h, h->d_xu, xu, (size_t)B * T))) return rc;
  if ((rc = copy_in(h, h->d_xs, xcur, (size_t)B * 12))) return rc;
  if ((rc = copy_in(h, h->d_goal, goals, (size_t)B * N * goal_stride))) return rc;
  if ((rc = launch_linearize(h, h->stream, bufs_at(h, 0), P, h->d_xu, h->d_goal, nullptr))) return rc;
  const double* qsol = nullptr;
  if ((rc = solve_qp(h, h->stream, bufs_at(h, 0), P, h->d_xu, h->d_xs, nullptr, h->d_sol, &qsol))) return rc;
  if ((rc = copy_out(h, sol, qsol, (size_t)B * T))) return rc;
  HIPCHK(hipStreamSynchronize(h->stream));
  return I7M_OK;
}

int i7m_qp_value(i7m_handle* h, int32_t B, const double* xu, const double* xcur, const double* goals, int32_t goal_stride,
                 double* V0) {
  int rc = check_batch(h, B, goal_stride);
  if (rc) return rc;
  if (B == 0) return I7M_OK;
  if (!xu || !xcur || !goals || !V0) return fail(I7M_EINVAL, "null pointer");
  if (h->cfg.qp_mode != I7M_QP_DIRECT) return fail(I7M_EINVAL, "i7m_qp_value: the equality-constrained QP only");
  const size_t T = 18 * (size_t)h->cfg.N - 6, N = h->cfg.N;
  // (B x 169 doubles in the solution buffer: T = 18 N - 6 >= 169 from N = 10) — a precondition,
  // checked before any copy or launch
  if (T < 169) return fail(I7M_EINVAL, "i7m_qp_value needs N >= 10");
  HIPCHK(hipSetDevice(h->dev));
  SolveParams P = params_of(h, B, goal_stride);
  if ((rc = copy_in(h, h->d_xu, xu, (size_t)B * T))) return rc;
  if ((rc = copy_in(h, h->d_xs, xcur, (size_t)B * 12))) return rc;
  if ((rc = copy_in(h, h->d_goal, goals, (size_t)B * N * goal_stride))) return rc;
  if ((rc = launch_linearize(h, h->stream, bufs_at(h, 0), P, h->d_xu, h->d_goal, nullptr))) return rc;
  double* vbuf = h->d_sol;
  if ((rc = launch_riccati(h, h->stream, bufs_at(h, 0), P, h->d_xu, h->d_xs, nullptr, h->d_sol, vbuf))) return rc;
  if ((rc = copy_out(h, V0, vbuf, (size_t)B * 169))) return rc;
  HIPCHK(hipStreamSynchronize(h->stream));
  return I7M_OK;
}

int i7m_get_box_stats(i7m_handle* h, int32_t B, int32_t* iters, int32_t* converged, double* mu) {
  if (!h) return fail(I7M_EINVAL, "null handle");
  if (h->cfg.qp_mode != I7M_QP_BOX) return fail(I7M_EINVAL, "handle is not in I7M_QP_BOX mode");
  if (B < 0 || B > h->cfg.max_batch) return fail(I7M_EINVAL, "batch outside [0, max_batch]");
  HIPCHK(hipSetDevice(h->dev));
  std::vector<IpmState> st((size_t)B);
  if (B) HIPCHK(hipMemcpyAsync(st.data(), h->d_bst, sizeof(IpmState) * (size_t)B, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  for (int b = 0; b < B; ++b) {
    if (iters) iters[b] = st[b].iters;
    if (converged) converged[b] = st[b].converged;
    if (mu) mu[b] = st[b].mu;
  }
  return I7M_OK;
}

int i7m_linearize(i7m_handle* h, int32_t B, const double* xu, const double* goals, int32_t goal_stride, double* lin,
                  double* cost) {
  int rc = check_batch(h, B, goal_stride);
  if (rc) return rc;
  if (B == 0) return I7M_OK;
  if (!xu || !goals) return fail(I7M_EINVAL, "null pointer");
  HIPCHK(hipSetDevice(h->dev));
  const size_t T = 18 * (size_t)h->cfg.N - 6, N = h->cfg.N;
  SolveParams P = params_of(h, B, goal_stride);
  if ((rc = copy_in(h, h->d_xu, xu, (size_t)B * T))) return rc;
  if ((rc = copy_in(h, h->d_goal, goals, (size_t)B * N * goal_stride))) return rc;
  if ((rc = launch_linearize(h, h->stream, bufs_at(h, 0), P, h->d_xu, h->d_goal, nullptr))) return rc;
  if (lin && (rc = copy_out(h, lin, h->d_lin, (size_t)B * (N - 1) * LIN_STRIDE))) return rc;
  if (cost && (rc = copy_out(h, cost, h->d_cost, (size_t)B * N * COST_STRIDE))) return rc;
  HIPCHK(hipStreamSynchronize(h->stream));
  return I7M_OK;
}

int i7m_merit(i7m_handle* h, int32_t B, const double* xu, const double* xu_ref, const double* goals,
              int32_t goal_stride, double* out) {
  int rc = check_batch(h, B, goal_stride);
  if (rc) return rc;
  if (B == 0) return I7M_OK;
  if (!xu || !xu_ref || !goals || !out) return fail(I7M_EINVAL, "null pointer");
  HIPCHK(hipSetDevice(h->dev));
  const size_t T = 18 * (size_t)h->cfg.N - 6, N = h->cfg.N;
  SolveParams P = params_of(h, B, goal_stride);
  if ((rc = copy_in(h, h->d_xu, xu, (size_t)B * T))) return rc;
  if ((rc = copy_in(h, h->d_aux, xu_ref, (size_t)B * T))) return rc;
  if ((rc = copy_in(h, h->d_goal, goals, (size_t)B * N * goal_stride))) return rc;
  hipLaunchKernelGGL(k_merit, dim3(B), dim3(64), 0, h->stream, h->d_model, P, h->d_xu, h->d_aux, h->d_goal,
                     h->has_fext ? h->d_fext : nullptr, (int)(h->fext_frame == I7M_WRENCH_WORLD), h->d_out);
  HIPCHK(hipGetLastError());
  if ((rc = copy_out(h, out, h->d_out, (size_t)B * 5))) return rc;
  HIPCHK(hipStreamSynchronize(h->stream));
  return I7M_OK;
}

int i7m_linesearch(i7m_handle* h, int32_t B, const double* xu, const double* xu_full, const double* goals,
                   int32_t goal_stride, double* alpha) {
  int rc = check_batch(h, B, goal_stride);
  if (rc) return rc;
  if (B == 0) return I7M_OK;
  if (!xu || !xu_full || !goals || !alpha) return fail(I7M_EINVAL, "null pointer");
  HIPCHK(hipSetDevice(h->dev));
  const size_t T = 18 * (size_t)h->cfg.N - 6, N = h->cfg.N;
  SolveParams P = params_of(h, B, goal_stride);
  if ((rc = copy_in(h, h->d_xu, xu, (size_t)B * T))) return rc;
  if ((rc = copy_in(h, h->d_sol, xu_full, (size_t)B * T))) return rc;
  if ((rc = copy_in(h, h->d_goal, goals, (size_t)B * N * goal_stride))) return rc;
  if ((rc = launch_linesearch(h, h->stream, bufs_at(h, 0), P, h->d_xu, h->d_xu, h->d_sol, h->d_goal, nullptr, h->d_stats, h->d_out, 0, 1,
                             false))) return rc;
  if ((rc = copy_out(h, alpha, h->d_out, (size_t)B))) return rc;
  HIPCHK(hipStreamSynchronize(h->stream));
  return I7M_OK;
}

// ---- query hooks: chunk through the max_batch*T-sized scratch buffers ----------------------
static size_t scratch_doubles(const i7m_handle* h) {
  return std::max((size_t)h->cfg.max_batch * (18 * (size_t)h->cfg.N - 6), (size_t)256 * 114);
}
static size_t query_cap(const i7m_handle* h) { return scratch_doubles(h) / 36; }  // <= 36 doubles/query

int i7m_eepos(i7m_handle* h, int32_t Bq, const double* q, double* p_out, double* J_out) {
  if (!h) return fail(I7M_EINVAL, "null handle");
  if (Bq < 0 || !q || !p_out) return fail(I7M_EINVAL, "bad arguments");
  HIPCHK(hipSetDevice(h->dev));
  const size_t cap = query_cap(h);
  int rc;
  for (size_t o = 0; o < (size_t)Bq; o += cap) {
    const int n = (int)std::min(cap, (size_t)Bq - o);
    if ((rc = copy_in(h, h->d_aux, q + 6 * o, 6 * (size_t)n))) return rc;
    hipLaunchKernelGGL(k_eepos, dim3((n + 255) / 256), dim3(256), 0, h->stream, h->d_model, n, h->d_aux, h->d_sol,
                       J_out ? h->d_out : nullptr);
    HIPCHK(hipGetLastError());
    if ((rc = copy_out(h, p_out + 3 * o, h->d_sol, 3 * (size_t)n))) return rc;
    if (J_out && (rc = copy_out(h, J_out + 18 * o, h->d_out, 18 * (size_t)n))) return rc;
    HIPCHK(hipStreamSynchronize(h->stream));
  }
  return I7M_OK;
}

int i7m_aba(i7m_handle* h, int32_t Bq, const double* q, const double* v, const double* tau, const double* fext,
            int32_t frame, double* a_out) {
  if (!h) return fail(I7M_EINVAL, "null handle");
  if (Bq < 0 || !q || !v || !tau || !a_out) return fail(I7M_EINVAL, "bad arguments");
  HIPCHK(hipSetDevice(h->dev));
  const size_t cap = query_cap(h);
  int rc;
  for (size_t o = 0; o < (size_t)Bq; o += cap) {
    const int n = (int)std::min(cap, (size_t)Bq - o);
    double* dq = h->d_aux;
    double* dv = h->d_aux + 6 * (size_t)n;
    double* dtau = h->d_aux + 12 * (size_t)n;
    double* df = h->d_aux + 18 * (size_t)n;
    if ((rc = copy_in(h, dq, q + 6 * o, 6 * (size_t)n))) return rc;
    if ((rc = copy_in(h, dv, v + 6 * o, 6 * (size_t)n))) return rc;
    if ((rc = copy_in(h, dtau, tau + 6 * o, 6 * (size_t)n))) return rc;
    if (fext && (rc = copy_in(h, df, fext + 6 * o, 6 * (size_t)n))) return rc;
    hipLaunchKernelGGL(k_aba, dim3((n + 255) / 256), dim3(256), 0, h->stream, h->d_model, n, dq, dv, dtau,
                       fext ? df : nullptr, (int)(frame == I7M_WRENCH_WORLD), h->d_sol);
    HIPCHK(hipGetLastError());
    if ((rc = copy_out(h, a_out + 6 * o, h->d_sol, 6 * (size_t)n))) return rc;
    HIPCHK(hipStreamSynchronize(h->stream));
  }
  return I7M_OK;
}

int i7m_aba_derivatives(i7m_handle* h, int32_t Bq, const double* q, const double* v, const double* tau, double* dq_out,
                        double* dv_out, double* Minv_out, double* a_out) {
  if (!h) return fail(I7M_EINVAL, "null handle");
  if (Bq < 0 || !q || !v || !tau || !dq_out || !dv_out || !Minv_out || !a_out)
    return fail(I7M_EINVAL, "bad arguments");
  HIPCHK(hipSetDevice(h->dev));
  // outputs need 3*36+6 doubles per query: put them in d_out/d_sol/d_lin regions
  const size_t cap = scratch_doubles(h) / 114;
  int rc;
  for (size_t o = 0; o < (size_t)Bq; o += cap) {
    const int n = (int)std::min(cap, (size_t)Bq - o);
    double* iq = h->d_aux;
    double* iv = h->d_aux + 6 * (size_t)n;
    double* it = h->d_aux + 12 * (size_t)n;
    double* oq = h->d_sol;
    double* ov = h->d_sol + 36 * (size_t)n;
    double* om = h->d_sol + 72 * (size_t)n;
    double* oa = h->d_sol + 108 * (size_t)n;
    if ((rc = copy_in(h, iq, q + 6 * o, 6 * (size_t)n))) return rc;
    if ((rc = copy_in(h, iv, v + 6 * o, 6 * (size_t)n))) return rc;
    if ((rc = copy_in(h, it, tau + 6 * o, 6 * (size_t)n))) return rc;
    const long nthr = 12L * n;
    hipLaunchKernelGGL(k_abad, dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, h->stream, h->d_model, n, iq, iv,
                       it, oq, ov, om, oa);
    HIPCHK(hipGetLastError());
    if ((rc = copy_out(h, dq_out + 36 * o, oq, 36 * (size_t)n))) return rc;
    if ((rc = copy_out(h, dv_out + 36 * o, ov, 36 * (size_t)n))) return rc;
    if ((rc = copy_out(h, Minv_out + 36 * o, om, 36 * (size_t)n))) return rc;
    if ((rc = copy_out(h, a_out + 6 * o, oa, 6 * (size_t)n))) return rc;
    HIPCHK(hipStreamSynchronize(h->stream));
  }
  return I7M_OK;
}

int i7m_rk4(i7m_handle* h, int32_t Bq, const double* q, const double* v, const double* u, double dt,
            const double* fext, int32_t frame, double* q_out, double* v_out) {
  if (!h) return fail(I7M_EINVAL, "null handle");
  if (Bq < 0 || !q || !v || !u || !q_out || !v_out) return fail(I7M_EINVAL, "bad arguments");
  HIPCHK(hipSetDevice(h->dev));
  const size_t cap = query_cap(h);
  int rc;
  for (size_t o = 0; o < (size_t)Bq; o += cap) {
    const int n = (int)std::min(cap, (size_t)Bq - o);
    double* iq = h->d_aux;
    double* iv = h->d_aux + 6 * (size_t)n;
    double* iu = h->d_aux + 12 * (size_t)n;
    double* iff = h->d_aux + 18 * (size_t)n;
    double* oq = h->d_sol;
    double* ov = h->d_sol + 6 * (size_t)n;
    if ((rc = copy_in(h, iq, q + 6 * o, 6 * (size_t)n))) return rc;
    if ((rc = copy_in(h, iv, v + 6 * o, 6 * (size_t)n))) return rc;
    if ((rc = copy_in(h, iu, u + 6 * o, 6 * (size_t)n))) return rc;
    if (fext && (rc = copy_in(h, iff, fext + 6 * o, 6 * (size_t)n))) return rc;
    hipLaunchKernelGGL(k_rk4, dim3((n + 255) / 256), dim3(256), 0, h->stream, h->d_model, n, iq, iv, iu, dt,
                       fext ? iff : nullptr, (int)(frame == I7M_WRENCH_WORLD), oq, ov);
    HIPCHK(hipGetLastError());
    if ((rc = copy_out(h, q_out + 6 * o, oq, 6 * (size_t)n))) return rc;
    if ((rc = copy_out(h, v_out + 6 * o, ov, 6 * (size_t)n))) return rc;
    HIPCHK(hipStreamSynchronize(h->stream));
  }
  return I7M_OK;
}

int i7m_mpc_run(i7m_handle* h, int32_t B, const double* xstart, const double* endpoints, int32_t n_endpoints,
                int32_t num_steps, double* dist_out, double* q_out, double* xcur_out, double* xu_out) {
  int rc = check_batch(h, B, 3);
  if (rc) return rc;
  if (n_endpoints < 1 || num_steps < 0 || !endpoints || !xstart || !dist_out)
    return fail(I7M_EINVAL, "mpc_run: need xstart, >= 1 endpoint, num_steps >= 0, dist_out");
  // MPC_OSQP has no external wrench (src/osqp_mpc.py:56 calls rk4 without f_ext): with one set
  // on the handle the planner (run_sqp) would use it and the plant (k_mpc_advance) would not
  if (h->has_fext)
    return fail(I7M_EINVAL, "mpc_run: the handle has an external wrench set; MPC_OSQP's closed loop has none "
                            "(clear it with i7m_set_external_wrench(h, 0, NULL, 0))");
  if (B == 0) return I7M_OK;
  HIPCHK(hipSetDevice(h->dev));
  const int N = h->cfg.N;
  const size_t T = 18 * (size_t)N - 6;
  // per-run state beyond the handle's buffers (this is a whole closed-loop run, not the solve
  // hot path): endpoints, goal index, alive flag, the distance and q histories
  double *d_ep = nullptr, *d_dist = nullptr, *d_q = nullptr;
  int *d_gi = nullptr, *d_alive = nullptr;
  auto cleanup = [&]() {
    for (void* p : {(void*)d_ep, (void*)d_dist, (void*)d_q, (void*)d_gi, (void*)d_alive})
      if (p) (void)hipFree(p);
  };
  const size_t hist = (size_t)std::max(num_steps, 1) * B;
  if (hipMalloc(&d_ep, 3 * 8 * (size_t)n_endpoints) != hipSuccess || hipMalloc(&d_dist, 8 * hist) != hipSuccess ||
      hipMalloc(&d_q, 6 * 8 * hist) != hipSuccess || hipMalloc(&d_gi, 4 * (size_t)B) != hipSuccess ||
      hipMalloc(&d_alive, 4 * (size_t)B) != hipSuccess) {
    cleanup();
    return fail(I7M_ENOMEM, "mpc_run: device allocation failed");
  }
  auto run = [&]() -> int {
    // src/osqp_mpc.py:14-27: goal = endpoint 0 tiled, XU = 0, XU = sqp(xcur, goal, XU)
    std::vector<double> goals((size_t)B * 3 * N);
    for (size_t b = 0; b < (size_t)B; ++b)
      for (int k = 0; k < N; ++k)
        for (int r = 0; r < 3; ++r) goals[(b * N + k) * 3 + r] = endpoints[r];
    std::vector<int> ones((size_t)B, 1);
    int rc2;
    if ((rc2 = copy_in(h, h->d_xs, xstart, (size_t)B * 12))) return rc2;
    if ((rc2 = copy_in(h, h->d_goal, goals.data(), goals.size()))) return rc2;
    if ((rc2 = copy_in(h, d_ep, endpoints, 3 * (size_t)n_endpoints))) return rc2;
    HIPCHK(hipMemsetAsync(d_gi, 0, 4 * (size_t)B, h->stream));
    HIPCHK(hipMemcpyAsync(d_alive, ones.data(), 4 * (size_t)B, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemsetAsync(h->d_xu, 0, 8 * (size_t)B * T, h->stream));
    // the instances [lo, lo + n) through every MPC step on stream s (the whole batch on the
    // handle's stream, or, where the solve staggers, each range on its own: the instances are
    // independent, so a range runs its steps without waiting for the other)
    auto loop = [&](long lo, int n, hipStream_t s) -> int {
      const double* xu0 = h->d_xu + lo * T;
      double *xu = h->d_xu + lo * T, *out = h->d_out + lo * T, *xs = h->d_xs + lo * 12, *g = h->d_goal + lo * 3 * N;
      int rc3;
      if ((rc3 = run_sqp(h, n, xu0, xu, xs, g, 3, h->d_stats + lo, lo, s))) return rc3;
      for (int i = 0; i < num_steps; ++i) {
        hipLaunchKernelGGL(k_mpc_goal, dim3((n + 255) / 256), dim3(256), 0, s, h->d_model, n, N, xs, g, d_ep, n_endpoints,
                           d_gi + lo, d_alive + lo, d_dist + (size_t)i * B + lo);
        HIPCHK(hipGetLastError());
        // xu_new = sqp(xcur, goal, XU) into the scratch buffer d_out (XU itself is read only)
        if ((rc3 = run_sqp(h, n, xu, out, xs, g, 3, h->d_stats + lo, lo, s))) return rc3;
        hipLaunchKernelGGL(k_mpc_advance, dim3(n), dim3(64), 0, s, h->d_model, n, N, h->cfg.dt, xs, xu, out, d_alive + lo,
                           d_q + ((size_t)i * B + lo) * 6);
        HIPCHK(hipGetLastError());
      }
      return I7M_OK;
    };
    if (stagger_applies(h, B)) {
      if ((rc2 = run_staggered(h, B, loop))) return rc2;
    } else if ((rc2 = loop(0, B, h->stream))) {
      return rc2;
    }
    if (num_steps > 0) {
      if ((rc2 = copy_out(h, dist_out, d_dist, (size_t)num_steps * B))) return rc2;
      if (q_out && (rc2 = copy_out(h, q_out, d_q, (size_t)num_steps * B * 6))) return rc2;
    }
    if (xcur_out && (rc2 = copy_out(h, xcur_out, h->d_xs, (size_t)B * 12))) return rc2;
    if (xu_out && (rc2 = copy_out(h, xu_out, h->d_xu, (size_t)B * T))) return rc2;
    HIPCHK(hipStreamSynchronize(h->stream));
    return I7M_OK;
  };
  rc = run();
  (void)hipStreamSynchronize(h->stream);
  cleanup();
  return rc;
}

int i7m_set_timing(i7m_handle* h, int enable) {
  if (!h) return fail(I7M_EINVAL, "null handle");
  h->timing = enable != 0;
  return I7M_OK;
}

int i7m_get_kernel_times(i7m_handle* h, double* ms_sum, int32_t* counts, int32_t n) {
  if (!h) return fail(I7M_EINVAL, "null handle");
  HIPCHK(hipStreamSynchronize(h->stream));
  for (auto& t : h->ev) {
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, t.a, t.b));
    h->ms_sum[t.kid] += ms;
    h->counts[t.kid] += 1;
    h->pool.push_back(t.a);
    h->pool.push_back(t.b);
  }
  h->ev.clear();
  for (int i = 0; i < n && i < I7M_K_COUNT; ++i) {
    if (ms_sum) ms_sum[i] = h->ms_sum[i];
    if (counts) counts[i] = h->counts[i];
  }
  return I7M_OK;
}

int i7m_reset_kernel_times(i7m_handle* h) {
  if (!h) return fail(I7M_EINVAL, "null handle");
  int rc = i7m_get_kernel_times(h, nullptr, nullptr, 0);
  if (rc) return rc;
  for (int i = 0; i < I7M_K_COUNT; ++i) {
    h->ms_sum[i] = 0;
    h->counts[i] = 0;
  }
  return I7M_OK;
}

}  // extern "C"
