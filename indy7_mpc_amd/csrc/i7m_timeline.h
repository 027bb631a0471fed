// i7m_timeline.h — per-wave timeline records for the -DI7M_DIAG library only (tools/timeline.py):
// each instrumented kernel's waves record [start, end] (s_memrealtime, the 100 MHz device-wide
// clock), the hardware slot they ran on (HW_ID, XCC_ID) and the kernel / workgroup, so a tool can
// see how a launch's waves were spread over the 1024 SIMDs and how much of the launch each SIMD
// sat idle (load imbalance, tails).  The release library compiles I7M_TL to nothing.
//
// Buffer layout (device, u64): [0] unused, [1] capacity (records), [2..7] unused, then 4 u64 per
// record: t_start, t_end, HW_ID | XCC_ID << 32, kernel id | workgroup << 8.  Record slot =
// kernel id << 16 | wave index in the grid: no atomics (a counter shared by every wave serialised
// the waves' exits and stretched a B = 4096 launch 3x), so a buffer holds one launch per kernel —
// the tool runs a single SQP iteration.
#pragma once

#include <hip/hip_runtime.h>

#ifdef I7M_DIAG
namespace i7m {

// one copy per translation unit (no -fgpu-rdc): each unit exports its own setter
static __device__ unsigned long long* g_tl = nullptr;

struct TlScope {
  unsigned long long t0;
  int kid;
  __device__ __forceinline__ explicit TlScope(int k) : kid(k) { t0 = __builtin_amdgcn_s_memrealtime(); }
  __device__ __forceinline__ ~TlScope() {
    unsigned long long* tl = g_tl;
    if (tl && (threadIdx.x & 63) == 0) {
      const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
      // s_getreg: HW_ID (id 4) and XCC_ID (id 20), all 32 bits
      const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
      const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
      const unsigned long long wv = (unsigned long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
      const unsigned long long i = ((unsigned long long)kid << 16) + wv;
      if (wv < (1ULL << 16) && i < tl[1]) {  // (a launch of more than 65536 waves records its first 65536)
        unsigned long long* r = tl + 8 + 4 * i;
        r[0] = t0;
        r[1] = t1;
        r[2] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
        r[3] = (unsigned long long)kid | ((unsigned long long)blockIdx.x << 8);
      }
    }
  }
};

// host side: point this unit's kernels at a record buffer (nullptr: off)
static inline int tl_set(void* p) {
  unsigned long long* v = static_cast<unsigned long long*>(p);
  return hipMemcpyToSymbol(HIP_SYMBOL(g_tl), &v, sizeof(v)) == hipSuccess ? 0 : -1;
}

}  // namespace i7m
#define I7M_TL(kid) i7m::TlScope i7m_tl_scope_(kid)
#else
#define I7M_TL(kid)
#endif
