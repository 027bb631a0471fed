// i7m_lin_tu.hip — k_linearize in a translation unit of its own, so that it can be compiled
// with the max-ILP machine scheduler (-mllvm -amdgpu-sched-strategy=max-ilp; __graft_entry__
// builds this file with it and the rest of the library with the default).  Measured at B = 4096,
// N = 32: k_linearize 133.8 -> 130.1 us with max-ILP, while the same flag costs k_riccati_mfma
// 1.6 us — hence the split.
//
// The kernel headers define non-template kernels and device functions too; included inside an
// anonymous namespace here, this unit's copies stay internal and do not collide with
// i7m_api.hip's at link time.  The launcher below is the only external symbol, with builtin
// parameter types only.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cmath>

namespace {
#include "i7m_linearize.h"
}  // namespace

// Launch of k_linearize (the model-specialised or the generic instantiation) with the dispatch
// events of i7m_api.hip's kernel timing (ea / eb may be null).  model: DevModel*, params:
// SolveParams*, init_stats: ProblemStats* (i7m_kernels.h).
// fext_world: fext (non-null) is a world-frame wrench (k_linearize<., true>).
#ifdef I7M_DIAG
// this unit's copy of the timeline buffer pointer (i7m_timeline.h; set by i7m_diag_timeline)
extern "C" int i7m_lin_tu_set_timeline(void* p) { return i7m::tl_set(p); }
#endif

void i7m_launch_linearize_kernel(bool spec, int grid, hipStream_t s, hipEvent_t ea, hipEvent_t eb, const void* model,
                                 const void* params, const double* xu, const double* goals, const double* fext,
                                 bool fext_world, const int* active, double* lin, double* cost, double* qpd,
                                 int* init_active, void* init_stats) {
  const i7m::DevModel* M = static_cast<const i7m::DevModel*>(model);
  const i7m::SolveParams& P = *static_cast<const i7m::SolveParams*>(params);
  i7m::ProblemStats* st = static_cast<i7m::ProblemStats*>(init_stats);
  auto go = [&](auto kern) {
    hipExtLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, s, ea, eb, 0, M, P, xu, goals, fext, active, lin, cost, qpd,
                          init_active, st);
  };
  const bool fw = fext && fext_world;
  if (spec && fw) go(i7m::k_linearize<true, true>);
  else if (spec) go(i7m::k_linearize<true, false>);
  else if (fw) go(i7m::k_linearize<false, true>);
  else go(i7m::k_linearize<false, false>);
}
