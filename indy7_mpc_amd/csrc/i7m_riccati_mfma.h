// i7m_riccati_mfma.h — the SQP subproblem QP solved with fp64 MFMA (v_mfma_f64_16x16x4), one
// wavefront per problem: the exact solve of the equality-constrained QP the reference hands
// OSQP (src/osqp_solver.py:137-143), a Riccati recursion laid out for the matrix cores.
//
// Homogeneous coordinates x~ = [x; 1] (13 states, padded to a 16x16 tile) fold the affine
// dynamics offset c and every linear cost term into the matrix products:
//     A~ = [[A, c], [0, 1]],  B~ = [B; 0],  Q~ = [[Q, q], [q', 0]],  N~ = [0 | r]
//     W0 = V~ A~,  Qxx = A~' W0 + Q~,  W1 = V~ B~,  H = B~' W1 + R,  G~ = B~' W0 + N~
//     K~ = -H^-1 G~  (6x13: [K | kff]),   V~ <- Qxx + K~' G~
// (First form: sixteen 16x16x4 MFMAs per stage; now 7 of them and 8 4x4x4_4b, I7M_RIC_44 and
// I7M_QXX_K0_VALU below.)  V~ never leaves the accumulator registers: it is
// symmetric, so the C/D layout of V~ (lane holds V[(l>>4)+4i][l&15]) is exactly the A-operand
// layout (V[l&15][4s+(l>>4)]) the next stage needs.  Likewise W0 / W1 / G~ are consumed as
// B operands straight from their accumulators.  LDS only carries the stage data, H and G~
// for the 6x6 Cholesky (13 lanes), and K~.
// MFMA f64 layouts (gfx950; checked by tools/probes/mfma_f64_layout.hip):
//     A[row=l&15][k=l>>4], B[k=l>>4][col=l&15], D[row=(l>>4)+4i][col=l&15], i=0..3.
#pragma once

#ifndef I7M_RIC_FD
#define I7M_RIC_FD 2  // forward-rollout prefetch depth (stages)
#endif

#include "i7m_kernels.h"

namespace i7m {

typedef double d4 __attribute__((ext_vector_type(4)));

enum : int {
  // stage stash: Aq(36) Av(36) Bu(36) | QP record of k_linearize (QPD_*, 32) | [BOX: Sigma(18) h(18)]
  MO_AQ = 0,
  MO_AV = 36,
  MO_BU = 72,
  MO_QP = 108,
  MO_CV = MO_QP + QPD_CV,   // c_v (6)
  MO_LX = MO_QP + QPD_LX,   // Qm j | dQm v (12)
  MO_LU = MO_QP + QPD_LU,   // Rm u (6)
  MO_J = MO_QP + QPD_J,     // j (6)
  MO_DQM = MO_QP + QPD_DQM,
  MO_RM = MO_QP + QPD_RM,
  MO_SIG = 140,  // BOX: interior-point diagonal Sigma of the knot (q v u)
  MO_HB = 158,   // BOX: linear-term shift h of the knot (q v u)
  MO_H = 176,    // 36
  MO_G = 212,    // 78  G~ (6 x 13)
  MO_KT = 290,   // 78  K~ (6 x 13)
  MO_ZERO = 368,
  MO_ONE = 369,
  MO_GJ = 370,   // 6 x 40  per-pivot Gauss-Jordan exchange slots (diagnostic variant)
  MO_DUMMY = MO_GJ,  // 64: lane l's sink for the stores it has nothing to write (branch-free)
  // 4x4-block products (S44): V~'s v-v block, W = V_vv Bu, W0's v rows (all 6 x 6 / 6 x 13 row-major)
  MO_VV = 610,
  MO_WV = 646,
  MO_W0V = 682,
  MO_DT = 760,   // dt (A~'s q rows read as LDS operands like its v rows)
  MO_TOTAL = 762,
  MO_QX = 762,   // 256  two-wave body: Qxx~ of wave 1 in the accumulator layout (64 i + lane)
  MO_TOTAL_W2 = 1018,
};

// I7M_RIC_44 (default 1): the stage's small products — H = Bu V_vv Bu + R and G~ = Bu W0_v + N~
// — on v_mfma_f64_4x4x4_4b blocks instead of padded 16x16x4 MFMAs.  On gfx950
// fp64 MFMA and fp64 VALU share one rate, and the 4x4x4_4b form retires FMAs at the 16x16x4 rate
// (tools/probes/fp64_pipes.hip), so an MFMA costs its padded size: H's two 16x16x4 steps (128
// cycles) did 216 useful FMAs of 2048, W1 = V B~ and G~ 23 % each.  As blocks: W (2 instructions),
// H (2), G~ (4) = 128 cycles for what took 384.  Bit-identical to the 16x16 form: both MFMAs
// accumulate their k-steps as an fma chain in k order and the padding adds exact zeros
// (tools/lib_diff.py, -DI7M_RIC_44=0 against the default: 0 of 4096 config-3 problems, 0 of 256
// config-4 problems and none of the 500 closed-loop steps differ in any bit).  The two-wave
// kernel (B <= 128) keeps the 16x16 forms: there G~ feeds wave 0's elimination straight from
// the accumulators, and the 4x4 blocks would put an LDS round trip on that chain (+2 us per launch
// at B <= 64).
#ifndef I7M_RIC_44
#define I7M_RIC_44 1
#endif
// I7M_QXX_K0_VALU (default 1): Qxx's k-step over A~'s q rows 0..3 as VALU adds / fmas and a lane-half
// swap instead of a 16x16x4 MFMA (one-wave body); bit-identical (one nonzero term per entry).
#ifndef I7M_QXX_K0_VALU
#define I7M_QXX_K0_VALU 1
#endif
#ifndef I7M_RIC_VV_PLAIN
#define I7M_RIC_VV_PLAIN 0
#endif
// I7M_RIC_44X (default 0, an A/B build): Qxx's v-row k-steps and V~'s update on
// 4x4x4_4b blocks without the homogeneous row block.  A 4x4x4_4b instruction whose B operand is a 16x16x4 B operand
// (the layouts coincide) and whose A operand replicates one row block rb of the left factor over
// its four block slots yields exactly register rb of the 16x16 D layout.  Rows 12..15 of Qxx and V~
// (register 3) held only V~[12][12], the cost-to-go's constant, which no gain, x or u depends on:
// three row blocks per k-step instead of the 16x16 MFMA's four (2 x 64 -> 6 x 16 cycles for Qxx,
// the same for V~), A operands from LDS.  Both forms accumulate each entry's k-steps as an fma chain
// in k order, so the results are bit-identical (tools/lib_diff.py: 0 of 4096 config-3, 0 of 256
// config-4 problems, none of the 500 closed-loop steps).  Measured slower (profiles/r04_ric44x_ab.txt):
// 97.9 -> 108.2 us per launch at B = 4096, 54.7 -> 67.0 at 1024, k_ipm_fused 5.43 -> 5.53 ms — the
// twelve A-operand LDS reads per stage (the 16x16 form reads two and reuses A~'s B-operand registers
// as Qxx's A operand), their map registers (4 VGPRs spilled at the 128 cap) and unpacking cost more
// than the 64 fp64-pipe cycles the row blocks save.
#ifndef I7M_RIC_44X
#define I7M_RIC_44X 0
#endif


// v_mfma_f64_4x4x4_4b: four independent 4 x 4 x 4 blocks.  Lane layouts (gfx950, probed by
// tools/probes/mfma_f64_4x4_layout.hip): A lane 16k + 4s + i = A_s[i][k], B lane 16k + 4s + j =
// B_s[k][j], D lane 16i + 4s + j = D_s[i][j] — the 16x16x4 operand layouts with the 4 x 4
// diagonal blocks of the product as results.  Block s of a 2 x 2 block product takes (row block,
// column block) = (s & 1, (s ^ (s >> 1)) & 1): 0 (0,0), 1 (1,1), 2 (0,1), 3 (1,0).
__device__ __forceinline__ double mfma44(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}
// f64 MFMA neg modifiers (the blgp field: bit 0 negates A, bit 1 B, bit 2 C): -(a b) - c, -(a b) + c
__device__ __forceinline__ double mfma44_nac(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 5);
}
__device__ __forceinline__ double mfma44_na(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 1);
}
__device__ __forceinline__ int blk_r(int s) { return s & 1; }
__device__ __forceinline__ int blk_c(int s) { return (s ^ (s >> 1)) & 1; }

// Per-lane LDS offsets of the 4x4-block products (fixed for the kernel), two 16-bit offsets per
// 32-bit word (lo | hi << 16), laundered once per stage (ric44_launder) so that the unpacked
// offsets are formed where used rather than hoisted out of the stage loop — unpacked, the maps
// held ~36 VGPRs across the loop.  Invalid (padding) entries read MO_ZERO; results with nothing
// to store go to the lane's sink slot.  BOX: the interior point's Sigma_u joins H's diagonal and
// its h_u G~'s last column (second C-input words hR2 / gN2).
struct Ric44Maps {
  unsigned wAB[2];   // W = V_vv' Bu: A | B of k-step ks
  unsigned hAB[2];   // H = Bu' W + R: A | B of k-step ks
  unsigned hDR;      // H's store | its C input (Rm on the diagonal, else MO_ZERO)
  unsigned wDhR2;    // W's store | BOX: Sigma_u on H's diagonal (else MO_ZERO)
  unsigned gA[2];    // G~ = Bu' W0_v + N~: A of row block 0 | row block 1, k-step ks
  unsigned gB;       // B of k-step 0 | 1
  unsigned gD;       // stores of row block 0 | 1
  unsigned gN;       // C inputs (r in column 12) of row block 0 | 1
  unsigned gN2;      // BOX: h_u in column 12 of row block 0 | 1
  unsigned oGB;      // G~ in the 16x16x4 B layout (k-step s: G~[4s + lq][lr]) for V~'s update: s = 0 | 1
  unsigned vvS;      // stores of V~'s v-v block: register 1 | register 2
  unsigned w0S;      // stores of W0's v rows: register 1 | register 2
};
__device__ __forceinline__ unsigned pk16(int lo, int hi) { return (unsigned)lo | ((unsigned)hi << 16); }
__device__ __forceinline__ int lo16(unsigned v) { return (int)(v & 0xffffu); }
__device__ __forceinline__ int hi16(unsigned v) { return (int)(v >> 16); }
template <bool BOX>
__device__ __forceinline__ Ric44Maps ric44_maps(const int l) {
  Ric44Maps M;
  const int hi = l >> 4, s = (l >> 2) & 3, lo = l & 3, lq = l >> 4, lr = l & 15;
  const int rA = 4 * blk_r(s) + lo, cB = 4 * blk_c(s) + lo;   // A row / B column of this lane
  const int rD = 4 * blk_r(s) + hi, cD = 4 * blk_c(s) + lo;   // D element of this lane
  const int sink = MO_DUMMY + l;
  int gB[2], oGB[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const int k = 4 * ks + hi;  // this lane's k in the A and B layouts
    M.wAB[ks] = pk16((rA < 6 && k < 6) ? MO_VV + 6 * rA + k : MO_ZERO, (k < 6 && cB < 6) ? MO_BU + 6 * k + cB : MO_ZERO);
    M.hAB[ks] = pk16((rA < 6 && k < 6) ? MO_BU + 6 * k + rA : MO_ZERO,   // Bu' [rA][k]
                     (k < 6 && cB < 6) ? MO_WV + 6 * k + cB : MO_ZERO);
    gB[ks] = (k < 6 && 4 * s + lo < 13) ? MO_W0V + 13 * k + 4 * s + lo : MO_ZERO;
    // Bu' [r][k] = Bu[k][r], row blocks 0 | 1
    M.gA[ks] = pk16((lo < 6 && k < 6) ? MO_BU + 6 * k + lo : MO_ZERO, (4 + lo < 6 && k < 6) ? MO_BU + 6 * k + 4 + lo : MO_ZERO);
    oGB[ks] = (4 * ks + lq < 6 && lr < 13) ? MO_G + 13 * (4 * ks + lq) + lr : MO_ZERO;
  }
  M.gB = pk16(gB[0], gB[1]);
  M.oGB = pk16(oGB[0], oGB[1]);
  const bool dg = rD == cD && rD < 6;
  M.wDhR2 = pk16((rD < 6 && cD < 6) ? MO_WV + 6 * rD + cD : sink, (BOX && dg) ? MO_SIG + 12 + rD : MO_ZERO);
  M.hDR = pk16((rD < 6 && cD < 6) ? MO_H + 6 * rD + cD : sink, dg ? MO_RM : MO_ZERO);
  int gD[2], gN[2], gN2[2];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    const int r = 4 * rb + hi, c = 4 * s + lo;
    gD[rb] = (r < 6 && c < 13) ? MO_G + 13 * r + c : sink;
    gN[rb] = (r < 6 && c == 12) ? MO_LU + r : MO_ZERO;
    gN2[rb] = (BOX && r < 6 && c == 12) ? MO_HB + 12 + r : MO_ZERO;
  }
  M.gD = pk16(gD[0], gD[1]);
  M.gN = pk16(gN[0], gN[1]);
  M.gN2 = pk16(gN2[0], gN2[1]);
  // V~ (accumulator layout: register i holds row lq + 4i of column lr): rows 6..11 are register 1
  // (lq = 2, 3) and register 2 (all lq); V_vv takes columns 6..11, W0_v columns 0..12.
  // V_vv is stored TRANSPOSED: the 16x16 products take V~'s accumulator registers as their A
  // operand, i.e. they use V~' (W0 = V~' A~, the old W1 = V~' B~).  V~ = Qxx + K~'G~ is symmetric
  // only to the accuracy of K~ = -H^-1 G~, and H can be very ill-conditioned (R = 1e-5 w against
  // Bu' V Bu), so H = Bu' (V~')_vv Bu keeps the recursion on the one matrix V~' throughout — with
  // V~_vv instead, 1e-8 relative errors at N = 32 and 1e-4 at N = 64 (measured).
  // (-DI7M_RIC_VV_PLAIN=1, a test build only: V~_vv un-transposed, the recursion that loses accuracy
  // — tests/test_gpu_riccati_value.py fails on it)
#if I7M_RIC_VV_PLAIN
  M.vvS = pk16((lq >= 2 && lr >= 6 && lr < 12) ? MO_VV + 6 * (lq - 2) + (lr - 6) : sink,
               (lr >= 6 && lr < 12) ? MO_VV + 6 * (lq + 2) + (lr - 6) : sink);
#else
  M.vvS = pk16((lq >= 2 && lr >= 6 && lr < 12) ? MO_VV + 6 * (lr - 6) + (lq - 2) : sink,
               (lr >= 6 && lr < 12) ? MO_VV + 6 * (lr - 6) + (lq + 2) : sink);
#endif
  M.w0S = pk16((lq >= 2 && lr < 13) ? MO_W0V + 13 * (lq - 2) + lr : sink, (lr < 13) ? MO_W0V + 13 * (lq + 2) + lr : sink);
  return M;
}
// Laundered in the box body only (k_ipm_fused: 69 -> 24 VGPRs spilled).  The plain QP has the
// registers for the hoisted unpacked maps (122 VGPRs), and unpacking at every use cost it ~6 %
// (k_riccati_mfma 254 -> 270 us at B = 4096, N = 64); I7M_RIC44_LAUNDER_ALL=1 launders there too (A/B).
#ifndef I7M_RIC44_LAUNDER_ALL
#define I7M_RIC44_LAUNDER_ALL 0
#endif
__device__ __forceinline__ void ric44_launder(Ric44Maps& M) {
  asm volatile("" : "+v"(M.wAB[0]), "+v"(M.wAB[1]), "+v"(M.hAB[0]), "+v"(M.hAB[1]), "+v"(M.hDR), "+v"(M.wDhR2),
               "+v"(M.gA[0]), "+v"(M.gA[1]), "+v"(M.gB), "+v"(M.gD), "+v"(M.gN), "+v"(M.gN2), "+v"(M.oGB), "+v"(M.vvS),
               "+v"(M.w0S));
}
// W = V_vv' Bu, then H = Bu' W + R (+ Sigma_u) into MO_H (needs V_vv', Bu, Rm in LDS; one wave)
template <bool BOX>
__device__ __forceinline__ void ric44_h(const Ric44Maps& M, double* __restrict__ sh) {
  double w = 0.0;
  w = mfma44(sh[lo16(M.wAB[0])], sh[hi16(M.wAB[0])], w);
  w = mfma44(sh[lo16(M.wAB[1])], sh[hi16(M.wAB[1])], w);
  sh[lo16(M.wDhR2)] = w;
  wave_sync();
  double h = BOX ? sh[hi16(M.hDR)] + sh[hi16(M.wDhR2)] : sh[hi16(M.hDR)];
  h = mfma44(sh[lo16(M.hAB[0])], sh[hi16(M.hAB[0])], h);
  h = mfma44(sh[lo16(M.hAB[1])], sh[hi16(M.hAB[1])], h);
  sh[lo16(M.hDR)] = h;
}
// -G~ = -(Bu' W0_v + N~ (+ h_u)) into MO_G (needs W0_v, Bu, r in LDS; one wave).  Negated by the
// MFMA's neg modifiers (first k-step: A and C, second: A), which negate every rounded partial sum
// exactly: the elimination of [H | -G~] then ends at K~ = -H^-1 G~ itself (no negation pass), and
// V~'s update takes -G~ with its B operand negated.
template <bool BOX>
__device__ __forceinline__ void ric44_g(const Ric44Maps& M, double* __restrict__ sh) {
  const double b0 = sh[lo16(M.gB)], b1 = sh[hi16(M.gB)];
  double g0 = sh[lo16(M.gN)], g1 = sh[hi16(M.gN)];
  if (BOX) {
    g0 += sh[lo16(M.gN2)];
    g1 += sh[hi16(M.gN2)];
  }
  g0 = mfma44_nac(sh[lo16(M.gA[0])], b0, g0);
  g1 = mfma44_nac(sh[hi16(M.gA[0])], b0, g1);
  g0 = mfma44_na(sh[lo16(M.gA[1])], b1, g0);
  g1 = mfma44_na(sh[hi16(M.gA[1])], b1, g1);
  sh[lo16(M.gD)] = g0;
  sh[hi16(M.gD)] = g1;
}

__device__ __forceinline__ d4 mfma(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ double mfma44_nb(double a, double b, double c) {  // a (-b) + c, 4x4x4_4b
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 2);
}
__device__ __forceinline__ d4 mfma_nb(double a, double b, d4 c) {  // a (-b) + c
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 2);
}

// v from lane `src` (wave-uniform src) into every lane, via two v_readlane_b32 (SGPR broadcast).
__device__ __forceinline__ double readlane_f64(double v, int src) {
  const long long bits = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(bits & 0xffffffffLL), src);
  const int hi = __builtin_amdgcn_readlane((int)(bits >> 32), src);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// v from lane J of each 16-lane row into every lane of that row: one v_mov_b64_dpp
// row_newbcast:J (gfx950 has 64-bit DPP for row_newbcast), the result in a VGPR.  Against
// readlane_f64: one instruction instead of two, and no VALU-writes-SGPR hazard.
template <int J>
__device__ __forceinline__ double row_bcast_f64(double v) {
  return __builtin_amdgcn_mov_dpp(v, 0x150 + J, 0xf, 0xf, false);
}
template <int J, int NJ>
struct RowBcast {  // out[j] = row_bcast_f64<j>(v), j = J .. NJ-1
  static __device__ __forceinline__ void run(double v, double* out) {
    out[J] = row_bcast_f64<J>(v);
    RowBcast<J + 1, NJ>::run(v, out);
  }
};
template <int NJ>
struct RowBcast<NJ, NJ> {
  static __device__ __forceinline__ void run(double, double*) {}
};
// row_bcast_f64 with the source lane as an argument that is a constant after unrolling (the DPP
// control must be an immediate: the switch folds away)
__device__ __forceinline__ double row_bcast_f64_at(double v, const int j) {
  switch (j) {
    case 0: return row_bcast_f64<0>(v);
    case 1: return row_bcast_f64<1>(v);
    case 2: return row_bcast_f64<2>(v);
    case 3: return row_bcast_f64<3>(v);
    case 4: return row_bcast_f64<4>(v);
    default: return row_bcast_f64<5>(v);
  }
}

// lane l <- lane l + 6 within each 16-lane row (DPP row_shl:6), fp64 as two 32-bit moves
__device__ __forceinline__ double row_shl6_f64(double v) {
  const long long bits = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(bits & 0xffffffffLL), 0x106, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(bits >> 32), 0x106, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// 1/d: v_rcp_f64 (about half the fp64 mantissa) + Newton steps, each doubling the correct
// bits (I7M_RCP_NR, default 1: within ~2 ulp; 2 were used before, 1 is off the pivot chain of
// every Gauss-Jordan step).
#ifndef I7M_RCP_NR
#define I7M_RCP_NR 1
#endif
__device__ __forceinline__ double rcp_nr(double d) {
  double y = __builtin_amdgcn_rcp(d);
#pragma unroll
  for (int i = 0; i < I7M_RCP_NR; ++i) y = fma(y, fma(-d, y, 1.0), y);
  return y;
}

// ABL (diagnostic builds only, results invalid; I7M_ABLATE in i7m_api.hip maps onto them):
// bit 0 skips the forward rollout, bit 2 selects the LDS-exchange Gauss-Jordan (bit 1 then
// replaces it by a scaling), bit 3 sends every stage's kbuf traffic to stage 0's slot
// (cache-resident), bit 4 the rollout's lin re-reads likewise, bit 5 drops the rollout's
// stores (the compiler then drops the rollout's arithmetic), bit 6 feeds x instead of u to the
// rollout's B u term (shorter chain), bit 7 skips the rollout's LDS staging, bit 8 keeps only
// the last stage's stores, bit 9 writes per-stage phase timestamps (s_memtime) of problem 0
// into sol (tools/ric_phases.py); used to split the kernel's time.
// BOX: the interior-point Newton step of the box-constrained QP (oracle/box_ipm.py): the same
// QP with Hessian P + diag(Sigma) and linear term g + h, Sigma and h given per variable in
// bsig / bh (B, T).  The equality rows are unchanged, so the result is the Newton iterate
// x + dx itself.
// 4 waves/SIMD (<= 128 VGPRs, MFMA accumulators in VGPRs): B = 4096 single-wave problems fit the
// 1024 SIMDs in one round.
// The body of one problem's solve (problem b, one wavefront, lane l, `sh` = MO_TOTAL doubles of
// LDS); k_riccati_mfma runs it once, k_ipm_fused (i7m_box.h) once per Newton step.
// HINV (box predictor steps): also carry the identity through the elimination and store H^-1
// of every stage in hinv (B, N-1, 36) for riccati_delta_body (column-per-lane elimination).
// BC: cross-lane broadcasts by DPP row_newbcast instead of v_readlane — bit 0 the Gauss-Jordan
// pivot columns, bit 1 the rollout's x and u; bit-identical either way.  Bit 2: wave priority by
// progress (ric_prio_back / _fwd), for launches with several waves per SIMD.  Measured (DESIGN.md
// §4.2): bit 1 helps at every batch size; bit 0 cost ~4.5 us per launch at B <= 256 (a longer
// pivot chain) until the round-3 stage changes, and helps at every batch size since, in the
// config-4 body (BOX, k_ipm_fused, I7M_IPM_BC) too.
#ifndef I7M_RIC_PRIO_S
#define I7M_RIC_PRIO_S 1  // 0: quarters of the backward sweep (A/B: 113.8 vs 112.8 us at B = 4096)
#endif
// Wave priority by progress (BC bit 2, several waves per SIMD): every problem is the same amount
// of work, and the SIMD's oldest-first arbitration otherwise lets the first wave run ahead while
// the youngest finishes alone at the end.  Priority falls as a wave advances, so the waves
// behind are issued first and the four waves of a SIMD finish together.  Backward stage k of
// N - 1 (k counts down) and forward stage k of the rollout; the default scheme keeps the lowest
// level short (the second half of the rollout), since the lead a wave takes there is never
// corrected:
__device__ __forceinline__ int ric_prio_back(int k, int N) {
  if (I7M_RIC_PRIO_S == 1) return 2 * k >= N - 1 ? 3 : (4 * k >= N - 1 ? 2 : 1);
  return (4 * k) / (N - 1);  // 3 .. 0 in quarters of the backward sweep; the rollout at 0
}
__device__ __forceinline__ int ric_prio_fwd(int k, int N) {
  if (I7M_RIC_PRIO_S == 1) return 2 * k < N - 1 ? 1 : 0;
  return 0;
}

// The forward rollout of one problem's QP solution (lane l of its wave, `sh` the body's LDS):
// x_0 = xs; u_k = K~ [x_k; 1]; x_{k+1} = A x + B u + c, from the gains the backward sweep stored
// in kbuf (K~, c_v) and the dynamics in lin; writes the minimiser to sol.
template <int ABL, int BC>
__device__ __forceinline__ void riccati_rollout(const int b, const SolveParams& P, const double* __restrict__ xs,
                                                const double* __restrict__ LINb, const double* __restrict__ KB,
                                                double* __restrict__ sol, double* __restrict__ sh, const int l) {
  const int N = P.N;
  const double dt = P.dt;
  constexpr bool PRIO = (BC & 4) != 0;
  // ---- forward rollout: x_0 = xs; u_k = K~ [x_k; 1]; x_{k+1} = A x + B u + c.
  // Lane l < 12 holds x_l and lane m < 6 holds u_m; the lanes of DPP row 0 see the full vectors
  // through row_newbcast (one 64-bit DPP move per value).  A stage's data (K~ 78 | c_v 6 | Aq Av Bu 108 = 192 doubles) is loaded coalesced
  // (3 per lane) two stages ahead into registers and dropped into one LDS slot permuted so that
  // the 19 values each lane needs are contiguous: lane m < 6 the row m of K~ (13, then zeros),
  // lane 6 + i c_v[i] and row i of Aq, Av, Bu; lanes >= 12 an all-zero block.  Every lane then
  // reads its block with the same ds_read_b128 sequence (no divergent gathers).
  constexpr int FB = 20;  // doubles per lane block
  wave_sync_all();  // kbuf stores of the backward sweep -> loads below (other lanes of this wave)
  double* S = sol + (long)b * P.T;
  // stage element e of stage k lives at base + k * stride (resolved once per lane)
  auto fbase = [&](int e, int& stride) -> const double* {
    if (e < KBUF_STRIDE) {
      stride = (ABL & 8) ? 0 : KBUF_STRIDE;
      return KB + e;
    }
    stride = (ABL & 16) ? 0 : LIN_STRIDE;
    return LINb + (e - KBUF_STRIDE);
  };
  int fs0, fs1, fs2;
  // running pointers to the next stage to prefetch (nf), stepped one stage per load and held at
  // the last stage (the loads past it are dummies): no per-load stride multiply
  const double* fb0 = fbase(l, fs0);
  const double* fb1 = fbase(l + 64, fs1);
  const double* fb2 = fbase(l + 128, fs2);
  int nf = 0;
  // slot position of stage element e
  // lane m < 6: K~ row m (K 0..11, kff 12); lane 6 + i: Aq row i (0..5), Av row i (6..11), c_v[i]
  // (12), Bu row i (13..18) — the same places for x and the constant, so one 12-term chain gives
  // u on lanes 0..5 and A x + c on lanes 6..11
  auto fpos = [](int e) -> int {
    if (e < 78) return FB * (e / 13) + e % 13;
    if (e < 84) return FB * (6 + e - 78) + 12;
    const int t = e - 84, blk = t / 36, w = t % 36;
    return FB * (6 + w / 6) + (blk < 2 ? 6 * blk : 13) + w % 6;
  };
  const int w0 = fpos(l), w1 = fpos(l + 64), w2 = fpos(l + 128);
  double* myb = sh + FB * (l < 12 ? l : 12);
  // zero the slot once (K~ rows' tails and the spare block stay zero)
  for (int e = l; e < FB * 13; e += 64) sh[e] = 0.0;
  // FD prefetch buffers used in turn (the loop is unrolled by FD), each refilled FD stages
  // ahead right after it is dropped into LDS: no register rotation, whose copies made every
  // stage wait for the loads it had just issued.
  constexpr int FD = I7M_RIC_FD;
  double f[FD][3];
  auto fload = [&](double* f) {
    f[0] = *fb0;
    f[1] = *fb1;
    f[2] = *fb2;
    if (nf < N - 2) {  // wave-uniform
      ++nf;
      fb0 += fs0;
      fb1 += fs1;
      fb2 += fs2;
    }
  };
  double xreg = (l < 12) ? xs[(long)b * 12 + l] : 0.0;
  if (l < 12) S[l] = xreg;
  // drain x_0 before the prefetch: otherwise the waitcnt pass carries the (lane-conditional)
  // x_0 load into the loop and every stage waits for the loads it has just issued
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
#pragma unroll
  for (int d = 0; d < FD; ++d) fload(f[d]);
  auto stage = [&](const int k, double* fk) {
    if (PRIO && I7M_RIC_PRIO_S != 0) set_prio(ric_prio_fwd(k, N));
    double r[19];
    if (ABL & 128) {
#pragma unroll
      for (int j = 0; j < 19; ++j) r[j] = fk[j % 3] * (j + 1);
      fload(fk);
    } else {
    wave_sync();
    sh[w0] = fk[0];
    sh[w1] = fk[1];
    sh[w2] = fk[2];
    fload(fk);
    wave_sync();
#pragma unroll
    for (int j = 0; j < 19; ++j) r[j] = myb[j];
    }
    // x (lanes 0..11, all in DPP row 0) to every lane of the row
    double X[12];
    if (BC & 2) {
      RowBcast<0, 12>::run(xreg, X);
    } else {
#pragma unroll
      for (int j = 0; j < 12; ++j) X[j] = readlane_f64(xreg, j);
    }
    // u = K~ [x; 1] on lanes 0..5 and c_v + Aq x_q + Av x_v on lanes 6..11 by the same chain
    // (two partial sums to halve its length)
    double ua = r[12], ub = 0.0;
#pragma unroll
    for (int j = 0; j < 6; ++j) { ua += r[j] * X[j]; ub += r[6 + j] * X[6 + j]; }
    const double ureg = ua + ub;
    if (!(ABL & 32) && (!(ABL & 256) || k == N - 2) && l < 6) S[18 * k + 12 + l] = ureg;
    double U[6];
    if (BC & 2) {
      RowBcast<0, 6>::run(ureg, U);
    } else {
#pragma unroll
      for (int j = 0; j < 6; ++j) U[j] = readlane_f64(ureg, j);
    }
    double vc = 0.0;
#pragma unroll
    for (int j = 0; j < 6; ++j) vc += r[13 + j] * ((ABL & 64) ? X[j] : U[j]);
    // q lanes: q + dt v, v_l = x_{6+l} from lane l + 6 (DPP row shift, same 16-lane row)
    const double vq = row_shl6_f64(xreg);
    const double nx = (l < 6) ? xreg + dt * vq : ureg + vc;
    xreg = nx;
    if (!(ABL & 32) && (!(ABL & 256) || k == N - 2) && l < 12) S[18 * (k + 1) + l] = nx;
  };
  // all FD stages unconditional inside the loop (the tail after it): a path that skips a stage
  // and loops back would make the next stage wait for its own refill
  int k = 0;
  for (; k + FD - 1 < N - 1; k += FD) {
#pragma unroll
    for (int d = 0; d < FD; ++d) stage(k + d, f[d]);
  }
#pragma unroll
  for (int d = 0; d < FD - 1; ++d)
    if (k + d < N - 1) stage(k + d, f[d]);
}

// W2: two waves per problem (a 128-lane workgroup, small batches where most SIMDs are idle): the
// MFMA chains of a stage are split so that the elimination starts after five MFMAs instead of
// nine and the Qxx chain runs under it — wave 0: W0 = V A~, G~, the Gauss-Jordan elimination,
// kbuf, the rollout; wave 1: W1 = V B~, H, then W0 and Qxx = A~' W0 + Q~ (handed over through
// LDS, MO_QX).  Both waves form V~ <- Qxx + K~' G~ from the same operands (wave 1 reads G~ from
// the elimination's LDS copy), so they hold bit-identical V~ and the result is bit-identical to
// the one-wave body.  Three workgroup barriers per stage (stash, H / G~, K~ / Qxx).
template <int ABL, bool BOX, bool HINV = false, int BC = 0, bool W2 = false>
__device__ __forceinline__ void riccati_mfma_body(const int b, const SolveParams& P, const double* __restrict__ xu,
                                                  const double* __restrict__ xs, const double* __restrict__ lin,
                                                  const double* __restrict__ cost, const double* __restrict__ qpd,
                                                  double* __restrict__ kbuf, double* __restrict__ sol,
                                                  const double* __restrict__ bsig, const double* __restrict__ bh,
                                                  double* __restrict__ sh, const int l,
                                                  double* __restrict__ hinv = nullptr, const bool kff_only = false,
                                                  double* __restrict__ vout = nullptr) {
  static_assert(!W2 || (!BOX && !HINV && ABL == 0), "two-wave body: plain QP only");
  const int lr = l & 15, lq = l >> 4;
  const int N = P.N;
  constexpr bool PRIO = (BC & 4) && !BOX && !W2;
  const int w = W2 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
  const double dt = P.dt;
  const double* X = xu + (long)b * P.T;
  const double* LINb = lin + (long)b * (N - 1) * LIN_STRIDE;
  const double* CB = cost + (long)b * N * COST_STRIDE;
  const double* QB = qpd + (long)b * (N - 1) * QPD_STRIDE;
  double* KB = kbuf + (long)b * (N - 1) * KBUF_STRIDE;

  // ---- per-lane operand maps (fixed for the whole kernel)
  // A~[4s+lq][lr] = sh[offA[s]] for k-steps s = 1, 2 (the q rows' 1 and dt from the MO_ONE / MO_DT
  // slots, so no per-stage add of a constant); k-step 0 is all q rows, the stage-invariant cA0.
  // (k-step 3 — row 12 — is the select on W0 / Qxx below, not an MFMA.)
  int offA[4];
  const double cA0 = (lr == lq) ? 1.0 : (lr == lq + 6 ? dt : 0.0);
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int k = 4 * s + lq, c = lr;
    offA[s] = MO_ZERO;
    if (k < 6) {
      offA[s] = (c == k) ? MO_ONE : (c == k + 6 ? MO_DT : MO_ZERO);
    } else if (k < 12) {
      const int i = k - 6;
      offA[s] = c < 6 ? MO_AQ + 6 * i + c : (c < 12 ? MO_AV + 6 * i + (c - 6) : (c == 12 ? MO_CV + i : MO_ZERO));
    }
  }
  auto opA = [&](int s) -> double { return s == 0 ? cA0 : sh[offA[s]]; };
  // B~[4s+lq][lr] for s = 1, 2
  int offB[2];
#pragma unroll
  for (int s = 1; s < 3; ++s) {
    const int k = 4 * s + lq;
    offB[s - 1] = (k >= 6 && lr < 6) ? MO_BU + 6 * (k - 6) + lr : MO_ZERO;
  }
  // Q~[lq+4i][lr] = sh[q1[i]] * sh[q2[i]]: rank-1 (Qm j) j' q block, dQm on the v diagonal, the
  // linear terms in row / column 12;  R on the u diagonal;  N~ = r in column 12.
  // BOX adds Sigma on the diagonals and h on the linear terms (oS for Q~, oR2 / oN2 for R, N~).
  int q1[4], q2[4], oR[4], oN[4], oS[4], oR2[4], oN2[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = lq + 4 * i, c = lr;
    q1[i] = MO_ZERO;
    q2[i] = MO_ZERO;
    if (r < 6 && c < 6) { q1[i] = MO_LX + r; q2[i] = MO_J + c; }
    else if (r >= 6 && r < 12 && r == c) { q1[i] = MO_DQM; q2[i] = MO_ONE; }
    else if (r < 12 && c == 12) { q1[i] = MO_LX + r; q2[i] = MO_ONE; }
    else if (r == 12 && c < 12) { q1[i] = MO_LX + c; q2[i] = MO_ONE; }
    oR[i] = (r == c && r < 6) ? MO_RM : MO_ZERO;
    oN[i] = (c == 12 && r < 6) ? MO_LU + r : MO_ZERO;
    oS[i] = MO_ZERO;
    if (BOX) {
      if (r == c && r < 12) oS[i] = MO_SIG + r;
      else if (r < 12 && c == 12) oS[i] = MO_HB + r;
      else if (r == 12 && c < 12) oS[i] = MO_HB + c;
    }
    oR2[i] = (BOX && r == c && r < 6) ? MO_SIG + 12 + r : MO_ZERO;
    oN2[i] = (BOX && c == 12 && r < 6) ? MO_HB + 12 + r : MO_ZERO;
  }
  const double m12 = (lr == 12) ? 1.0 : 0.0, mlq0 = (lq == 0) ? 1.0 : 0.0;
  const double mdt_hi = (lq >= 2) ? dt : 0.0, mdt_lo = (lq < 2) ? dt : 0.0;
  // K~[4s+lq][lr] for s = 0, 1
  int oK[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int u = 4 * s + lq;
    oK[s] = (u < 6 && lr < 13) ? MO_KT + 13 * u + lr : MO_ZERO;
  }

  // the small products on 4x4x4 blocks (I7M_RIC_44), the box body too (its Sigma_u / h_u join
  // the C inputs); not the two-wave kernel (see I7M_RIC_44) nor the diagnostic LDS-exchange elimination
  constexpr bool S44 = I7M_RIC_44 && !(ABL & 4) && !W2;
  Ric44Maps M44 = ric44_maps<BOX>(l);
  // I7M_RIC_44X: A operands of the row-block products (lane l: k = l >> 4, row i = l & 3 of the block)
  //   Qxx: A~'[4rb + i][4ks + k] = A~[4ks + k][4rb + i], k-steps ks = 1, 2 (packed lo | hi)
  //   V~ : K~'[4rb + i][4ks + k] = K~[4ks + k][4rb + i], k-steps ks = 0, 1
  constexpr bool X44 = I7M_RIC_44X && S44;
  unsigned qxA[3], vxA[3];
#pragma unroll
  for (int rb = 0; rb < 3; ++rb) {
    const int k = l >> 4, c = 4 * rb + (l & 3);
    int a[2];
#pragma unroll
    for (int ks = 1; ks < 3; ++ks) {
      const int r = 4 * ks + k;
      int o = MO_ZERO;
      if (r < 6) o = (c == r) ? MO_ONE : (c == r + 6 ? MO_DT : MO_ZERO);
      else o = c < 6 ? MO_AQ + 6 * (r - 6) + c : MO_AV + 6 * (r - 6) + (c - 6);
      a[ks - 1] = o;
    }
    qxA[rb] = pk16(a[0], a[1]);
    vxA[rb] = pk16(MO_KT + 13 * k + c, k < 2 ? MO_KT + 13 * (4 + k) + c : MO_ZERO);
  }
  constexpr int SE = BOX ? 176 : 140;  // stash length
  // Branch-free lane-conditional stores (lanes with nothing to store write a per-lane sink slot,
  // DESIGN.md §7) in the plain QP only: in the box body (k_ipm_fused) the sink addresses and
  // the duplicated tail stores raised its VGPR spill 35 -> 78 and the launch 6.3 -> 8.4 ms, so
  // it keeps the exec-masked stores.
  constexpr bool BF = !BOX;
  // kbuf tail (K~ 64..77, c_v): 20 doubles; every lane stores one (lane l the entry l % 20)
  const int l20 = l % 20;
  const int ko20 = (l20 < 14) ? MO_KT + 64 + l20 : MO_CV + (l20 - 14);
  // stash element e of stage k lives at base(e) + k * stride(e): resolved once per lane for its
  // three elements, so the per-stage loads are one multiply-add each (no divergent selects)
  auto base_of = [&](int e, int& stride) -> const double* {
    if (e < MO_QP) { stride = LIN_STRIDE; return LINb + e; }
    if (e < MO_SIG) { stride = QPD_STRIDE; return QB + (e - MO_QP); }
    stride = 18;
    if (e < MO_HB) return bsig + (long)b * P.T + (e - MO_SIG);
    return bh + (long)b * P.T + (e - MO_HB);
  };
  const int e2 = (l + 128 < SE) ? l + 128 : SE - 1;
  int st0, st1, st2;
  // running pointers, stepped back one stage per stage: a per-lane stride times the stage index
  // cost two v_mad_u64_u32 (quarter rate) and their moves per element and stage
  const double* sb0 = base_of(l, st0) + (long)(N - 2) * st0;
  const double* sb1 = base_of(l + 64, st1) + (long)(N - 2) * st1;
  const double* sb2 = base_of(e2, st2) + (long)(N - 2) * st2;
  // (the first stage's stash is requested before the terminal record, so its latency overlaps
  // the record's own loads)
  double p0 = *sb0, p1 = *sb1, p2 = *sb2;
  auto stash_next = [&]() {
    sb0 -= st0;
    sb1 -= st1;
    sb2 -= st2;
    p0 = *sb0;
    p1 = *sb1;
    p2 = *sb2;
  };

  // ---- terminal cost-to-go V~ = Q~_{N-1}: the terminal knot's record from cost and XU
  {
    const double* ct = CB + (N - 1) * COST_STRIDE;
    if (l < 6) {
      sh[MO_J + l] = ct[l];
      sh[MO_LX + l] = ct[6] * ct[l];
    } else if (l < 12) {
      sh[MO_LX + l] = ct[7] * X[18 * (N - 1) + l];
    } else if (l == 12) {
      sh[MO_DQM] = ct[7];
    } else if (l == 13) {
      sh[MO_ZERO] = 0.0;
      sh[MO_ONE] = 1.0;
      sh[MO_DT] = dt;
    }
    if (BOX && l < 12) {
      sh[MO_SIG + l] = bsig[(long)b * P.T + 18 * (N - 1) + l];
      sh[MO_HB + l] = bh[(long)b * P.T + 18 * (N - 1) + l];
    }
  }
  if (W2) lds_sync(); else wave_sync();
  d4 V;
#pragma unroll
  for (int i = 0; i < 4; ++i) V[i] = BOX ? sh[q1[i]] * sh[q2[i]] + sh[oS[i]] : sh[q1[i]] * sh[q2[i]];

  // ABL bit 9 (diagnostic): per-stage phase timestamps (s_memtime) of problem 0 into sol
  long long tm0 = 0, tm1 = 0, tm2 = 0, tm3 = 0, ta = 0, tb = 0, td = 0, te = 0, tp = 0;
  auto tstamp = [](double dep) -> long long {
    asm volatile("" ::"v"(dep));
    return (long long)__builtin_amdgcn_s_memtime();
  };
  for (int k = N - 2; k >= 0; --k) {
    if constexpr (S44 && (BOX || I7M_RIC44_LAUNDER_ALL)) ric44_launder(M44);
    if constexpr (W2) {
      lds_sync();  // every wave is done with the previous stage's LDS
      if (w == 0) {
        sh[MO_AQ + l] = p0;
        sh[MO_AQ + l + 64] = p1;
        sh[l + 128 < SE ? MO_AQ + l + 128 : MO_DUMMY + l] = p2;
        if constexpr (S44) {
          sh[lo16(M44.vvS)] = V[1];
          sh[hi16(M44.vvS)] = V[2];
        }
      }
      lds_sync();
      if (w == 0 && k > 0) stash_next();
      double bA[3], bB[2];
#pragma unroll
      for (int s = 0; s < 3; ++s) bA[s] = opA(s);
      bB[0] = sh[offB[0]];
      bB[1] = sh[offB[1]];
      d4 W0, Z00, Z10;
      if (w == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) W0[i] = (lr == 12) ? V[i] : 0.0;
#pragma unroll
        for (int s = 0; s < 3; ++s) W0 = mfma(V[s], bA[s], W0);
        if constexpr (S44) {
          sh[lo16(M44.w0S)] = W0[1];
          sh[hi16(M44.w0S)] = W0[2];
          wave_sync();
          ric44_g<BOX>(M44, sh);
        } else {
        d4 Ni;
#pragma unroll
        for (int i = 0; i < 4; ++i) Ni[i] = sh[oN[i]];
        Z10 = mfma(bB[0], W0[1], Ni);
        Z10 = mfma(bB[1], W0[2], Z10);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int r = lq + 4 * i;
          sh[(r < 6 && lr < 13) ? MO_G + 13 * r + lr : MO_DUMMY + l] = Z10[i];
        }
        }
      } else if (S44) {
        ric44_h<BOX>(M44, sh);
      } else {
        d4 Ri;
#pragma unroll
        for (int i = 0; i < 4; ++i) Ri[i] = sh[oR[i]];
        d4 W1 = {0.0, 0.0, 0.0, 0.0};
        W1 = mfma(V[1], bB[0], W1);
        W1 = mfma(V[2], bB[1], W1);
        d4 Z11 = mfma(bB[0], W1[1], Ri);
        Z11 = mfma(bB[1], W1[2], Z11);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int r = lq + 4 * i;
          sh[(r < 6 && lr < 6) ? MO_H + 6 * r + lr : MO_DUMMY + l] = Z11[i];
        }
      }
      lds_sync();  // H and G~ in LDS
      if (w == 0) {
        // column-per-lane Gauss-Jordan on [H | G~], as in the one-wave body below
        double E[6];
        const int m16 = l & 15;
        const int cc_own = !(BC & 1) ? l : (l < 16) ? m16 : (l < 32 ? (m16 < 6 ? m16 : (m16 < 9 ? m16 + 10 : -1)) : -1);
        const int cc = !(BC & 1) ? (l < 19 ? l : 18) : (cc_own < 0 ? 0 : cc_own);
        const int eo = (cc < 6) ? MO_H + cc : MO_G + (cc - 6), es = (cc < 6) ? 6 : 13;
#pragma unroll
        for (int i = 0; i < 6; ++i) E[i] = sh[eo + es * i];
#pragma unroll
        for (int p = 0; p < 6; ++p) {
          double Pc[6];
#pragma unroll
          for (int i = 0; i < 6; ++i) Pc[i] = (BC & 1) ? row_bcast_f64_at(E[i], p) : readlane_f64(E[i], p);
          const double inv = rcp_nr(Pc[p]);
          const double ep = E[p] * inv;
#pragma unroll
          for (int i = 0; i < 6; ++i) E[i] = (i == p) ? ep : E[i] - Pc[i] * ep;
        }
        const bool kw = cc_own >= 6 && cc_own < 19;
#pragma unroll
        for (int i = 0; i < 6; ++i) sh[kw ? MO_KT + 13 * i + (cc_own - 6) : MO_DUMMY + l] = -E[i];
      } else {
        d4 Qi;
#pragma unroll
        for (int i = 0; i < 4; ++i) Qi[i] = sh[q1[i]] * sh[q2[i]];
#pragma unroll
        for (int i = 0; i < 4; ++i) W0[i] = (lr == 12) ? V[i] : 0.0;
#pragma unroll
        for (int s = 0; s < 3; ++s) W0 = mfma(V[s], bA[s], W0);
        Z00 = Qi;
        if (lq == 0) Z00[3] += W0[3];
#pragma unroll
        for (int s = 0; s < 3; ++s) Z00 = mfma(bA[s], W0[s], Z00);
#pragma unroll
        for (int i = 0; i < 4; ++i) sh[MO_QX + 64 * i + l] = Z00[i];
      }
      lds_sync();  // K~ and Qxx in LDS
      if (w == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) Z00[i] = sh[MO_QX + 64 * i + l];
      }
      if (w != 0 || S44) {
        // G~ as wave 0's accumulators held it (rows >= 6 and columns >= 13 are exact zeros there);
        // S44: both waves (G~ came from 4x4 blocks, not from a 16x16 accumulator)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int r = lq + 4 * i;
          Z10[i] = (r < 6 && lr < 13) ? sh[MO_G + 13 * r + lr] : 0.0;
        }
      }
      V = mfma(sh[oK[0]], Z10[0], Z00);
      V = mfma(sh[oK[1]], Z10[1], V);
      if (w == 0) {
        double* kk = KB + (long)k * KBUF_STRIDE;
        kk[l] = sh[MO_KT + l];
        kk[64 + l20] = sh[ko20];
      }
      continue;
    }
    if (PRIO) set_prio(ric_prio_back(k, N));
    wave_sync();
    if (ABL & 512) tm0 = tstamp(V[0]);
    if (ABL & 512) tp = tstamp(p0 + p1 + p2);
    sh[MO_AQ + l] = p0;
    sh[MO_AQ + l + 64] = p1;
    if (BF) sh[l + 128 < SE ? MO_AQ + l + 128 : MO_DUMMY + l] = p2;
    else if (l + 128 < SE) sh[MO_AQ + l + 128] = p2;
    if constexpr (S44) {  // V~'s v-v block for H = Bu' V_vv Bu (4x4 blocks)
      sh[lo16(M44.vvS)] = V[1];
      sh[hi16(M44.vvS)] = V[2];
    }
    wave_sync();
    if (k > 0) stash_next();
    double bA[3], bB[2];
#pragma unroll
    for (int s = 0; s < 3; ++s) bA[s] = opA(s);
    d4 Qi, Ri, Ni;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      // (x + 0.0 is not folded for doubles: the box shifts are added only in BOX builds)
      // (rows >= 8 — registers 2, 3 — hold no rank-1 entries: their second factor is 1 or the
      // first is 0, so the product is the first factor itself)
      Qi[i] = BOX ? (i < 2 ? sh[q1[i]] * sh[q2[i]] : sh[q1[i]]) + sh[oS[i]] : (i < 2 ? sh[q1[i]] * sh[q2[i]] : sh[q1[i]]);
    if constexpr (!S44) {
      bB[0] = sh[offB[0]];
      bB[1] = sh[offB[1]];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        Ri[i] = BOX ? sh[oR[i]] + sh[oR2[i]] : sh[oR[i]];
        Ni[i] = BOX ? sh[oN[i]] + sh[oN2[i]] : sh[oN[i]];
      }
    }
    // W0 = V A~ ; Qxx = A~' W0 + Q~.  Rows 12..15 of A~ are e_12' and 0: their k-step is a
    // select (W0[:,12] += V[:,12], Qxx[12,:] += W0[12,:]) instead of an MFMA.
    if (ABL & 512) ta = tstamp(bA[0] + bA[1] + bA[2] + bB[0] + bB[1] + Qi[0] + Ri[0] + Ni[0]);
    d4 W0;
    // (lr == 12 ? V : +0) as one fma per register instead of two 32-bit selects
#pragma unroll
    for (int i = 0; i < 4; ++i) W0[i] = (X44 && i == 3) ? 0.0 : fma(V[i], m12, 0.0);
#pragma unroll
    for (int s = 0; s < 3; ++s) W0 = mfma(V[s], bA[s], W0);
    if (ABL & 512) tb = tstamp(W0[0] + W0[1] + W0[2] + W0[3]);
    d4 Z00 = Qi;
    d4 Z10, Z11;
    if constexpr (S44) {
      // W0's v rows for G~; then H = Bu' V_vv Bu + R (under the Qxx chain), G~ = Bu' W0_v + N~,
      // both stored into MO_H / MO_G for the elimination
      sh[lo16(M44.w0S)] = W0[1];
      sh[hi16(M44.w0S)] = W0[2];
      ric44_h<BOX>(M44, sh);
      if (!X44) Z00[3] = fma(W0[3], mlq0, Z00[3]);  // row 12's k-step: + W0[12][:] on the lanes lq == 0
      if constexpr (I7M_QXX_K0_VALU) {
        // k-step 0 (A~'s q rows 0..3: 1 at (k, k), dt at (k, k + 6)) on the VALU: rows 0..3 of Qxx
        // gain W0's rows 0..3 (same lanes), rows 6..9 dt times them (the other half of the wave:
        // one v_permlane32_swap per dword).  One nonzero term per entry, rounded as the MFMA's
        // k-step rounds it (bit-identical).
        // Q~'s rank-1 products stay rounded on their own, as the MFMA's C input (otherwise the
        // compiler contracts them into the adds below)
        asm volatile("" : "+v"(Z00[0]), "+v"(Z00[1]));
        Z00[0] = Z00[0] + W0[0];
        const long long wb = __double_as_longlong(W0[0]);
        const auto slo = __builtin_amdgcn_permlane32_swap((unsigned)wb, (unsigned)wb, false, false);
        const auto shi = __builtin_amdgcn_permlane32_swap((unsigned)(wb >> 32), (unsigned)(wb >> 32), false, false);
        // lanes 32..63 of the first result: W0 from lanes 0..31 (rows 0, 1); lanes 0..31 of the
        // second: from lanes 32..63 (rows 2, 3)
        const double up = __longlong_as_double(((long long)shi[0] << 32) | (unsigned)slo[0]);
        const double dn = __longlong_as_double(((long long)shi[1] << 32) | (unsigned)slo[1]);
        // (an fma: the MFMA's k-step adds its exact product to C — measured: a separately rounded
        // product changes 4 091 of 4 096 config-3 solves, the fma none)
        Z00[1] = fma(up, mdt_hi, Z00[1]);  // rows 6, 7 (lq 2, 3)
        Z00[2] = fma(dn, mdt_lo, Z00[2]);  // rows 8, 9 (lq 0, 1)
        if constexpr (X44) {
          // k-steps 1, 2 as three row blocks each (the 16x16 D registers 0..2)
#pragma unroll
          for (int rb = 0; rb < 3; ++rb) {
            Z00[rb] = mfma44(sh[lo16(qxA[rb])], W0[1], Z00[rb]);
            Z00[rb] = mfma44(sh[hi16(qxA[rb])], W0[2], Z00[rb]);
          }
        } else {
#pragma unroll
          for (int s = 1; s < 3; ++s) Z00 = mfma(bA[s], W0[s], Z00);
        }
      } else {
#pragma unroll
        for (int s = 0; s < 3; ++s) Z00 = mfma(bA[s], W0[s], Z00);
      }
      ric44_g<BOX>(M44, sh);
    } else {
    if (lq == 0) Z00[3] += W0[3];
#pragma unroll
    for (int s = 0; s < 3; ++s) Z00 = mfma(bA[s], W0[s], Z00);
    // W1 = V B~ ; H = B~' W1 + R ; G~ = B~' W0 + N~   (B~ rows 6..11 only: k-steps 1, 2)
    d4 W1 = {0.0, 0.0, 0.0, 0.0};
    W1 = mfma(V[1], bB[0], W1);
    W1 = mfma(V[2], bB[1], W1);
    Z11 = mfma(bB[0], W1[1], Ri);
    Z11 = mfma(bB[1], W1[2], Z11);
    if (ABL & 512) tm1 = tstamp(bA[0] + bA[1] + bA[2] + Qi[0] + Ri[0] + Ni[0]);
    Z10 = mfma(bB[0], W0[1], Ni);
    Z10 = mfma(bB[1], W0[2], Z10);
    if (ABL & 512) tm2 = tstamp(Z10[0] + Z10[1] + Z11[0] + Z11[1]);
    }
    double* kk = KB + (long)((ABL & 8) ? 0 : k) * KBUF_STRIDE;
    if ((ABL & 4) && !BOX) {
      // (Diagnostic alternative, I7M_ABLATE=8: measured 5 us slower per launch at B = 1 and
      // level at B = 4096 than the column-per-lane elimination below)
      // K~ = -H^-1 G~ by Gauss-Jordan on [H | G~] (6 x 19) in place in the MFMA accumulator
      // layout: lane l holds column lr of rows lq and lq + 4 (lq < 2) of H (lr < 6) and of G~
      // (lr < 13).  Pivot p needs, per lane, M[r][p] of its two rows (published by the lanes
      // lr == p) and M[p][lr] of its column (published by the lanes lq == p & 3): a per-pivot
      // LDS slot, two writes and three broadcast-friendly reads, instead of 12 v_readlane per
      // pivot.  The arithmetic is the column-per-lane elimination's, operation for operation.
      // SPD H: no pivoting.  K~ ends where the V~ update wants it: the A operand of k-step s is
      // K~[4s + lq][lr], i.e. this lane's G~ entry of row lq + 4s.  (The box variants keep the
      // column-per-lane form below: fewer live registers next to their Sigma / h operand maps.)
      double eh0 = Z11[0], eh1 = Z11[1], eg0 = Z10[0], eg1 = Z10[1];
      if (ABL & 2) {
        eh0 *= 1e-3; eh1 *= 1e-3; eg0 *= 1e-3; eg1 *= 1e-3;
      } else {
#pragma unroll
        for (int p = 0; p < 6; ++p) {
          double* col = sh + MO_GJ + 40 * p;  // col[2 lq + i] = M[lq + 4i][p]
          double* row = col + 8;              // row[2 lr + j] = M[p][lr] of H (j = 0), G~ (j = 1)
          if (lr == p) {
            col[2 * lq] = eh0;
            col[2 * lq + 1] = eh1;
          }
          if (lq == (p & 3)) {
            row[2 * lr] = (p >> 2) ? eh1 : eh0;
            row[2 * lr + 1] = (p >> 2) ? eg1 : eg0;
          }
          wave_sync();
          const double mr0 = col[2 * lq], mr1 = col[2 * lq + 1];
          const double mph = row[2 * lr], mpg = row[2 * lr + 1];
          const double inv = rcp_nr(row[2 * p]);
          const double eph = mph * inv, epg = mpg * inv;
          eh0 = (lq == p) ? eph : eh0 - mr0 * eph;
          eg0 = (lq == p) ? epg : eg0 - mr0 * epg;
          eh1 = (lq + 4 == p) ? eph : eh1 - mr1 * eph;
          eg1 = (lq + 4 == p) ? epg : eg1 - mr1 * epg;
        }
      }
      const double ka0 = (lr < 13) ? -eg0 : 0.0;
      const double ka1 = (lq < 2 && lr < 13) ? -eg1 : 0.0;
      // V~ <- Qxx + K~' G~
      V = mfma(ka0, Z10[0], Z00);
      V = mfma(ka1, Z10[1], V);
      // K~ (78, row-major 6 x 13) and c_v (6) -> global for the forward rollout
      if (lr < 13) {
        kk[13 * lq + lr] = ka0;
        if (lq < 2) kk[13 * (lq + 4) + lr] = ka1;
      }
      if (l < 6) kk[78 + l] = sh[MO_CV + l];
    } else {
      // Column-per-lane Gauss-Jordan (every variant by default): H, G~ through LDS, one column
      // of [H | G~ (| I)] per lane, the pivot column broadcast by DPP row_newbcast, which stays
      // inside a 16-lane row — so each of the two rows used carries its own copy of H's six
      // columns: row 0 = H 0..5, G~ 0..9; row 1 = H 0..5 again, G~ 10..12 and (HINV) the
      // identity columns, which end as H^-1.  The two copies of H evolve identically.
      // (stores of lanes with nothing to store go to their own dummy slot: no exec-mask branches)
      if constexpr (!S44) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r = lq + 4 * i;
        if (BF) {
          sh[(r < 6 && lr < 6) ? MO_H + 6 * r + lr : MO_DUMMY + l] = Z11[i];
          sh[(r < 6 && lr < 13) ? MO_G + 13 * r + lr : MO_DUMMY + l] = Z10[i];
        } else if (r < 6) {
          if (lr < 6) sh[MO_H + 6 * r + lr] = Z11[i];
          if (lr < 13) sh[MO_G + 13 * r + lr] = Z10[i];
        }
      }
      }
      wave_sync();
      if constexpr (S44) {  // G~ in the 16x16x4 B layout for V~'s update below
        Z10[0] = sh[lo16(M44.oGB)];
        Z10[1] = sh[hi16(M44.oGB)];
      }
      double E[6];
      // column of lane l: 0..5 H, 6..18 G~, 19..24 identity (HINV); -1 unused (rows 2, 3 and
      // row 1's tail compute a copy of H column 0 and store nothing)
      const int m16 = l & 15;
      const int ncol = HINV ? 25 : 19;
      const int cc_own = !(BC & 1) ? l
                         : (l < 16) ? m16 : (l < 32 ? (m16 < 6 ? m16 : (m16 < (HINV ? 15 : 9) ? m16 + 10 : -1)) : -1);
      const int cc = !(BC & 1) ? (l < ncol ? l : ncol - 1) : (cc_own < 0 ? 0 : cc_own);
      const int eo = (cc < 6) ? MO_H + cc : MO_G + (cc - 6), es = (cc < 6) ? 6 : 13;
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        E[i] = sh[eo + es * (HINV && cc >= 19 ? 0 : i)];
        if (HINV && cc >= 19) E[i] = (i == cc - 19) ? 1.0 : 0.0;
      }
      if (ABL & 512) td = tstamp(E[0] + E[1] + E[2] + E[3] + E[4] + E[5]);
#pragma unroll
      for (int p = 0; p < 6; ++p) {
        double Pc[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) Pc[i] = (BC & 1) ? row_bcast_f64_at(E[i], p) : readlane_f64(E[i], p);
        const double inv = rcp_nr(Pc[p]);
        const double ep = E[p] * inv;
#pragma unroll
        for (int i = 0; i < 6; ++i) E[i] = (i == p) ? ep : E[i] - Pc[i] * ep;
      }
      if (ABL & 512) te = tstamp(E[0] + E[1] + E[2] + E[3] + E[4] + E[5]);
      {  // K~ columns (lanes of G~ columns; (BC & 1) == 0: lane l = column l), others to the sink
        const bool kw = cc_own >= 6 && cc_own < 19;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          const double ki = S44 ? E[i] : -E[i];  // S44: the G~ columns were eliminated from -G~
          if (BF) sh[kw ? MO_KT + 13 * i + (cc_own - 6) : MO_DUMMY + l] = ki;
          else if (kw) sh[MO_KT + 13 * i + (cc_own - 6)] = ki;
        }
      }
      if (HINV && cc_own >= 19 && cc_own < 25) {
        double* hk = hinv + ((long)b * (N - 1) + k) * 36;
#pragma unroll
        for (int i = 0; i < 6; ++i) hk[6 * i + (cc_own - 19)] = E[i];
      }
      wave_sync();
      if (ABL & 512) tm3 = tstamp(E[0]);
      if constexpr (X44) {  // Z10 holds -G~ (ric44_g); row blocks 0..2 of V~
#pragma unroll
        for (int rb = 0; rb < 3; ++rb) {
          V[rb] = mfma44_nb(sh[lo16(vxA[rb])], Z10[0], Z00[rb]);
          V[rb] = mfma44_nb(sh[hi16(vxA[rb])], Z10[1], V[rb]);
        }
      } else if constexpr (S44) {  // Z10 holds -G~ (ric44_g)
        V = mfma_nb(sh[oK[0]], Z10[0], Z00);
        V = mfma_nb(sh[oK[1]], Z10[1], V);
      } else {
        V = mfma(sh[oK[0]], Z10[0], Z00);
        V = mfma(sh[oK[1]], Z10[1], V);
      }
      if (ABL & 512) {
        const long long tm4 = tstamp(V[0] + V[1] + V[2] + V[3]);
        if (b == 0 && l == 0) {
          double* o = sol + 8 * k;
          o[0] = (double)(ta - tp);    // stash LDS round trip + operand reads (+ MFMA chains)
          o[2] = (double)(tp - tm0);   // the stash loads of the stage (issued a stage ahead)
          o[1] = (double)(tb - ta);    // W0 chain
          o[3] = (double)(tm2 - tm1);  // G~ issue
          o[4] = (double)(td - tm2);   // H, G~ results -> LDS -> per-lane columns
          o[5] = (double)(te - td);    // six pivots
          o[6] = (double)(tm3 - te);   // K~ -> LDS
          o[7] = (double)(tm4 - tm3);  // V~ update
        }
      }
      if (BOX && kff_only) {
        // a corrector step of the interior point: same Hessian as the predictor's, so its gain K is
        // bit for bit the one the predictor stored (each K~ column is eliminated on its own with
        // H's pivots, and the hom row / column of V~ never enters the first twelve columns); only
        // the feedforward column changes, and c_v does not
        if (l < 6) kk[13 * l + 12] = sh[MO_KT + 13 * l + 12];
      } else {
      kk[l] = sh[MO_KT + l];
      if (BF) kk[64 + l20] = sh[ko20];  // lanes >= 20 repeat the stores of lanes l % 20 (same values)
      else if (l < 20) kk[64 + l] = (l < 14) ? sh[MO_KT + 64 + l] : sh[MO_CV + (l - 14)];
      }
    }
  }

  if constexpr (!W2 && !BOX) {
    // i7m_qp_value: the cost-to-go of the first knot, V~_0 (13 x 13, as the accumulators hold it:
    // lane l register i = row lq + 4i, column lr), instead of the rollout (vout wave-uniform)
    if (vout) {
      // rows 0..11 as held (I7M_RIC_44X: row 12 is not formed; it is filled from column 12, and the
      // constant V~[12][12], which nothing depends on, is NaN)
      double* o = vout + (long)b * 169;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int r = lq + 4 * i;
        if (lr < 13) o[13 * r + lr] = V[i];
        if (lr == 12) o[13 * 12 + r] = V[i];
      }
      if (l == 12) o[168] = X44 ? __builtin_nan("") : V[3];
      return;
    }
  }
  if (W2) {
    lds_sync();  // wave 1's last reads of the stage LDS before the rollout reuses it
    if (w != 0) return;
  }
  if (ABL & 1) return;
  riccati_rollout<ABL, BC>(b, P, xs, LINb, KB, sol, sh, l);
}

// The corrector Newton step of I7M_QP_BOX (k_ipm_fused): the QP of the last
// riccati_mfma_body<0, true, true> run (same Hessian, dynamics and x_0) with its linear terms
// changed by dh (B, T).  The KKT system is linear, so the new minimiser is the old one, y, plus
// the minimiser of the change: a vector-only Riccati pass with that run's gains K (kbuf) and
// H^-1 (hinv), zero dynamics offsets and zero initial state:
//   p_{N-1} = dq_{N-1};  g_u = dr_k + B' p,  g_x = dq_k + A' p,  kff_k = -H^-1 g_u,  p <- g_x + K' g_u;
//   du_k = K dx_k + kff_k,  dx_{k+1} = A dx_k + B du_k,  dx_0 = 0;   y += (dx, du).
// No factorisation and no MFMA: ~1/4 of a full step.  kff overwrites kbuf's feedforward column.
__device__ __forceinline__ void riccati_delta_body(const int b, const SolveParams& P, const double* __restrict__ lin,
                                                   double* __restrict__ kbuf, const double* __restrict__ hinv,
                                                   const double* __restrict__ dh, double* __restrict__ y,
                                                   double* __restrict__ sh, const int l) {
  const int N = P.N;
  const double dt = P.dt;
  const double* LINb = lin + (long)b * (N - 1) * LIN_STRIDE;
  double* KB = kbuf + (long)b * (N - 1) * KBUF_STRIDE;
  const double* HB = hinv + (long)b * (N - 1) * 36;
  const double* DH = dh + (long)b * P.T;
  // backward stage slot: Aq | Av | Bu | K~ (78) | H^-1 (36) | dh_k (18);  then p (12), g_u (6)
  enum { DA = 0, DV = 36, DB = 72, DK = 108, DI = 186, DD = 222, DP = 240, DG = 252 };
  auto src = [&](int k, int e) -> const double* {
    if (e < DK) return LINb + (long)k * LIN_STRIDE + e;
    if (e < DI) return KB + (long)k * KBUF_STRIDE + (e - DK);
    if (e < DD) return HB + (long)k * 36 + (e - DI);
    return DH + 18 * k + (e - DD);
  };
  const int e3 = (l + 192 < DP) ? l + 192 : DP - 1;
  double q0 = *src(N - 2, l), q1 = *src(N - 2, l + 64), q2 = *src(N - 2, l + 128), q3 = *src(N - 2, e3);
  double preg = (l < 12) ? DH[18 * (N - 1) + l] : 0.0;  // p_{N-1} = dq of the terminal knot
  const int c6 = (l < 6) ? l : (l < 12 ? l - 6 : 0);
  const int cc = (l < 12) ? l : 0;
  const int oa = (l < 6) ? DA : DV;  // g_x of lane c < 6 uses Aq' , of lane 6 + j Av'
  for (int k = N - 2; k >= 0; --k) {
    wave_sync();
    sh[l] = q0;
    sh[l + 64] = q1;
    sh[l + 128] = q2;
    if (l + 192 < DP) sh[l + 192] = q3;
    if (l < 12) sh[DP + l] = preg;
    wave_sync();
    if (k > 0) { q0 = *src(k - 1, l); q1 = *src(k - 1, l + 64); q2 = *src(k - 1, l + 128); q3 = *src(k - 1, e3); }
    // g_x (lanes 0..11): dq + [p_q + Aq' p_v ; dt p_q + Av' p_v];  g_u (lanes 0..5): dr + Bu' p_v
    double gx = sh[DD + cc] + ((l < 6) ? preg : dt * sh[DP + c6]);
    double gu = sh[DD + 12 + c6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const double pv = sh[DP + 6 + i];
      gx += sh[oa + 6 * i + c6] * pv;
      gu += sh[DB + 6 * i + c6] * pv;
    }
    if (l < 6) sh[DG + l] = gu;
    wave_sync();
    double g[6];
#pragma unroll
    for (int m = 0; m < 6; ++m) g[m] = sh[DG + m];
    double kf = 0.0;
#pragma unroll
    for (int n = 0; n < 6; ++n) kf -= sh[DI + 6 * c6 + n] * g[n];
    if (l < 6) KB[(long)k * KBUF_STRIDE + 13 * l + 12] = kf;
#pragma unroll
    for (int m = 0; m < 6; ++m) gx += sh[DK + 13 * m + cc] * g[m];
    preg = gx;
  }
  // forward: as the main rollout (stage slot K~ 78 | c_v 6 | Aq Av Bu 108), c = 0, x_0 = 0, and
  // the result added to y by the lanes that wrote y's entries
  wave_sync_all();  // kff stores -> loads below
  double* Y = y + (long)b * P.T;
  const int iv = (l >= 6 && l < 12) ? l - 6 : 0;
  const int ik = l < 6 ? l : 0;
  auto fsrc = [&](int k, int e) -> const double* {
    return (e < KBUF_STRIDE) ? KB + (long)k * KBUF_STRIDE + e : LINb + (long)k * LIN_STRIDE + (e - KBUF_STRIDE);
  };
  // two alternating prefetch buffers, as the main rollout
  double fa[3], fb[3];
  auto fload = [&](double* f, int kk) {
    f[0] = *fsrc(kk, l);
    f[1] = *fsrc(kk, l + 64);
    f[2] = *fsrc(kk, l + 128);
  };
  fload(fa, 0);
  fload(fb, N - 1 > 1 ? 1 : 0);
  double xreg = 0.0;
  auto stage = [&](const int k, double* f) {
    wave_sync();
    sh[l] = f[0];
    sh[l + 64] = f[1];
    sh[l + 128] = f[2];
    fload(f, (k + 2 < N - 1) ? k + 2 : k);
    wave_sync();
    double r[19];
    if (l < 6) {
#pragma unroll
      for (int j = 0; j < 13; ++j) r[j] = sh[13 * ik + j];
#pragma unroll
      for (int j = 13; j < 19; ++j) r[j] = 0.0;
    } else {
      r[0] = 0.0;
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        r[1 + j] = sh[84 + 6 * iv + j];
        r[7 + j] = sh[84 + 36 + 6 * iv + j];
        r[13 + j] = sh[84 + 72 + 6 * iv + j];
      }
    }
    double X[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) X[j] = readlane_f64(xreg, j);
    double ua = r[12], ub = 0.0;
#pragma unroll
    for (int j = 0; j < 6; ++j) { ua += r[j] * X[j]; ub += r[6 + j] * X[6 + j]; }
    const double ureg = ua + ub;
    if (l < 6) Y[18 * k + 12 + l] += ureg;
    double U[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) U[j] = readlane_f64(ureg, j);
    double va = r[0], vb = 0.0, vc = 0.0, vq = 0.0;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      va += r[1 + j] * X[j];
      vb += r[7 + j] * X[6 + j];
      vc += r[13 + j] * U[j];
      vq = (l == j) ? X[6 + j] : vq;
    }
    const double nx = (l < 6) ? xreg + dt * vq : (va + vb) + vc;
    xreg = nx;
    if (l < 12) Y[18 * (k + 1) + l] += nx;
  };
  int k = 0;
  for (; k + 1 < N - 1; k += 2) {
    stage(k, fa);
    stage(k + 1, fb);
  }
  if (k < N - 1) stage(k, fa);
}

// Two waves per problem (riccati_mfma_body W2), for small batches.
template <int BC>
__global__ void __launch_bounds__(128) k_riccati_mfma_w2(SolveParams P, const double* __restrict__ xu,
                                                       const double* __restrict__ xs, const double* __restrict__ lin,
                                                       const double* __restrict__ cost, const double* __restrict__ qpd,
                                                       const int* __restrict__ active, double* __restrict__ kbuf,
                                                       double* __restrict__ sol) {
  I7M_TL(2);
  const int b = blockIdx.x;
  if (b >= P.B) return;
  if (active && !active[b]) return;
  __shared__ double sh[MO_TOTAL_W2];
  riccati_mfma_body<0, false, false, BC, true>(b, P, xu, xs, lin, cost, qpd, kbuf, sol, nullptr, nullptr, sh,
                                               threadIdx.x & 63);
}

template <int ABL, bool BOX = false, int BC = 0>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4, 4))) k_riccati_mfma(SolveParams P, const double* __restrict__ xu,
                                                     const double* __restrict__ xs, const double* __restrict__ lin,
                                                     const double* __restrict__ cost, const double* __restrict__ qpd,
                                                     const int* __restrict__ active,
                                                     double* __restrict__ kbuf, double* __restrict__ sol,
                                                     const double* __restrict__ bsig = nullptr,
                                                     const double* __restrict__ bh = nullptr,
                                                     double* __restrict__ vout = nullptr) {
  I7M_TL(2);
  const int b = blockIdx.x;
  if (b >= P.B) return;
  if (active && !active[b]) return;
  __shared__ double sh[MO_TOTAL];
  riccati_mfma_body<ABL, BOX, false, BC>(b, P, xu, xs, lin, cost, qpd, kbuf, sol, bsig, bh, sh, threadIdx.x, nullptr,
                                         false, vout);
}

}  // namespace i7m
