// i7m_fused.h — the whole SQP solve of one problem in ONE launch (k_sqp_fused): the reference's
// SQP_OSQP.sqp (src/osqp_sqp.py:76-93) with its linearisation / QP / line search
// (src/osqp_solver.py:70-143, src/osqp_sqp.py:49-74) as the phases of one workgroup per problem,
// the <= max_sqp_iters loop on the device, stats and active flags initialised in-kernel.
//
// Per SQP iteration, with W waves per problem (1 for large batches, 4 for small ones):
//   1. linearisation: the problem's N knots, KPW per wave and pass, all W waves side by side
//      (linearize_body; per-wave LDS, wave-local syncs only);
//   2. QP: the Riccati recursion and rollout on wave 0 (riccati_mfma_body); the others wait;
//   3. line search + step by all W waves (linesearch_body).
// Phases hand over through the same per-problem buffers as the three-kernel path (lin, cost, qpd,
// kbuf, sol), so every phase does exactly the arithmetic of its kernel there and the results are
// bit-identical to it; between phases: block_sync_global().  What the fusion removes is the
// launches (3 per SQP iteration -> 1 per solve), the host-side dispatch gaps between them, and
// the per-launch re-staging of each problem's data; what it costs is the register file: the
// workgroup holds the largest phase's VGPRs (the linearisation's, 2 waves per SIMD) for the
// whole solve, where the split path runs the Riccati phase at 4 waves per SIMD.
#pragma once

#include "i7m_kernels.h"
#include "i7m_linearize.h"
#include "i7m_riccati_mfma.h"

namespace i7m {

// dynamic LDS (doubles) of k_sqp_fused: the phases' regions overlap (one phase at a time), the
// line search's merit slots after all of them
__host__ __device__ inline int fused_merit_offset(int T, int W) {
  int m = W * LINLDS_DOUBLES;
  if (MO_TOTAL > m) m = MO_TOTAL;
  const int ls = 2 * T + W * LS_PARK;
  if (ls > m) m = ls;
  return (m + 1) & ~1;  // keep 16-byte alignment of what follows
}
// + the merit slots (10 doubles) + the lane-id slots (64 W ints)
inline size_t fused_lds_bytes(int T, int W) {
  return sizeof(double) * (size_t)(fused_merit_offset(T, W) + 10) + sizeof(int) * 64 * W;
}

// The lane id re-read per phase from an LDS slot through a volatile load, which the compiler can
// neither hoist out of the phase nor merge with another phase's: each body rebuilds its per-lane
// operand maps and addresses inside its phase instead of holding them live across the others
// (which spilled).  (An empty-asm launder, as in k_ipm_fused, crashes this compiler here.)
__device__ __forceinline__ int phase_lane(const int* ids) { return ((const volatile int*)ids)[threadIdx.x]; }

// LOOP: the whole solve (every SQP iteration) in one launch; otherwise one launch per SQP
// iteration `it0` (fewer live values across phases: 29 VGPRs spilled instead of ~120 with the
// loop; DESIGN.md §4.5 measures both).
template <bool SPEC, int W, bool FW = false, bool LOOP = true>
__global__ void __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_sqp_fused(const DevModel* __restrict__ Mg, SolveParams P, const double* xu_in, double* xu_out,
            const double* __restrict__ xs, const double* __restrict__ goals, const double* __restrict__ fext,
            double* __restrict__ lin, double* __restrict__ cost, double* __restrict__ qpd, double* __restrict__ kbuf,
            double* __restrict__ sol, int* __restrict__ active, ProblemStats* __restrict__ stats, const int it0) {
  const int b = blockIdx.x;
  if (b >= P.B) return;  // uniform over the workgroup
  const int w = W > 1 ? (int)(threadIdx.x >> 6) : 0;
  const int l = threadIdx.x & 63;
  extern __shared__ __attribute__((aligned(16))) double fsm[];
  double* merit = fsm + fused_merit_offset(P.T, W);
  int* lane_ids = reinterpret_cast<int*>(merit + 10);
  lane_ids[threadIdx.x] = l;
  if (it0 == 0) {
    // the first-iteration duties of k_linearize: zeroed stats, problem active
    if (threadIdx.x < (int)(sizeof(ProblemStats) / sizeof(double)))
      reinterpret_cast<double*>(stats + b)[threadIdx.x] = 0.0;
    if (threadIdx.x == 0) active[b] = 1;
    block_sync_global();
  } else if (!active[b]) {
    return;  // converged or alpha = 0 in an earlier iteration (uniform over the workgroup)
  }
  const int it_end = LOOP ? P.max_iters : it0 + 1;
  for (int it = it0; it < it_end; ++it) {
    const double* xin = it == 0 ? xu_in : xu_out;
    // 1. linearisation: wave w takes knots w KPW + g, + W KPW per pass
    for (int k0 = w * KPW; k0 < P.N; k0 += W * KPW) {
      const int lp = phase_lane(lane_ids);
      const int k = k0 + lp / 6;
      linearize_body<SPEC, FW>(Mg, P, b, k, lp / 6 < KPW && k < P.N, lp, reinterpret_cast<LinLds*>(fsm)[w], xin, goals,
                               fext, lin, cost, qpd);
    }
    block_sync_global();
    // 2. the QP (wave 0; its lane id is not re-read: that crashes this compiler)
    if (w == 0) riccati_mfma_body<0, false>(b, P, xin, xs, lin, cost, qpd, kbuf, sol, nullptr, nullptr, fsm, l);
    block_sync_global();
    // 3. line search and step; clears active[b] when the SQP loop ends (src/osqp_sqp.py:81-91)
    linesearch_body<SPEC, 0, W, FW>(Mg, P, b, w, phase_lane(lane_ids), fsm, merit, xin, xu_out, sol, goals, fext,
                                    active, stats, nullptr, it, 0, lin, cost);
    if (LOOP) {
      block_sync_global();
      if (!*(volatile int*)(active + b)) break;
    }
  }
}

}  // namespace i7m
