// i7m_admm_prep_tu.hip — the ADMM QP's preparation kernels (k_admm_scale, k_admm_factor of
// i7m_admm.h) in a translation unit of their own, compiled with the max-ILP machine scheduler
// (-mllvm -amdgpu-sched-strategy=max-ilp, as i7m_lin_tu.hip).  Measured with the flag on every
// unit (profiles/r06zm_sched_maxilp_ab.txt): the scaling + factor 352 -> 330 us per QP at B = 1,
// 356 -> 334 at B = 64, 1102-1122 -> 1067-1086 at B = 4096, bit-identical, while the same flag
// makes k_admm_iter 3-4 % longer at config 3 and leaves k_admm_iter_res level — hence the split.
// i7m_api.hip keeps its own default-scheduled copies for the staggered ranges of config 3, where
// these make the step 0.6 % longer (profiles/r06zo; i7m_handle::admm_prep_ilp picks by size).
//
// i7m_admm.h included inside an anonymous namespace: this unit's kernels and device functions stay
// internal (I7M_ADMM_PREP_ONLY: no copies of the iteration kernels).  The launcher is the only
// external symbol, with builtin parameter types only.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cmath>

#include "../../include/indy7_mpc.h"

#define I7M_ADMM_PREP_ONLY 1
namespace {
#include "i7m_admm.h"
}  // namespace

#ifdef I7M_DIAG
// this unit's copy of the timeline buffer pointer (i7m_timeline.h; set by i7m_diag_timeline)
extern "C" int i7m_admm_prep_tu_set_timeline(void* p) { return i7m::tl_set(p); }
#endif

// kernel 0: k_admm_scale<9> (N <= 32), 1: k_admm_scale<18>, 2: k_admm_factor; grid = problems,
// one wave each.  args: the AdmmArgs (i7m_admm.h) i7m_api.hip built.
hipError_t i7m_launch_admm_prep(int kernel, int grid, hipStream_t s, hipEvent_t ea, hipEvent_t eb, const void* args) {
  const i7m::AdmmArgs& a = *static_cast<const i7m::AdmmArgs*>(args);
  if (kernel == 0)
    hipExtLaunchKernelGGL(i7m::k_admm_scale<9>, dim3(grid), dim3(64), 0, s, ea, eb, 0, a);
  else if (kernel == 1)
    hipExtLaunchKernelGGL(i7m::k_admm_scale<18>, dim3(grid), dim3(64), 0, s, ea, eb, 0, a);
  else if (kernel == 2)
    hipExtLaunchKernelGGL(i7m::k_admm_factor, dim3(grid), dim3(64), 0, s, ea, eb, 0, a);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}
