// i7m_fused_tu.hip — k_sqp_fused (i7m_fused.h) in a translation unit of its own, behind one
// launcher with builtin parameter types (as i7m_lin_tu.hip): its instantiations stay internal.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cmath>
#include <map>
#include <mutex>
#include <type_traits>

#include "../../include/indy7_mpc.h"

namespace {
#include "i7m_fused.h"
}  // namespace

// B problems (params: SolveParams*, model: DevModel*, stats: ProblemStats*), W = 1 or 4 waves per
// problem, fext_world: fext (non-null) is a world-frame wrench.  it < 0: the whole solve in this
// launch (k_sqp_fused<.., LOOP = true>); it >= 0: SQP iteration `it` only.
hipError_t i7m_launch_sqp_fused(bool spec, int W, bool fext_world, int it, hipStream_t s, hipEvent_t ea, hipEvent_t eb,
                                const void* model, const void* params, const double* xu_in, double* xu_out,
                                const double* xs, const double* goals, const double* fext, double* lin, double* cost,
                                double* qpd, double* kbuf, double* sol, int* active, void* stats) {
  using namespace i7m;
  const DevModel* M = static_cast<const DevModel*>(model);
  const SolveParams& P = *static_cast<const SolveParams*>(params);
  ProblemStats* st = static_cast<ProblemStats*>(stats);
  const size_t lds = fused_lds_bytes(P.T, W);
  const bool fw = fext && fext_world;
  const int it0 = it < 0 ? 0 : it;
  // the dynamic-LDS limits were raised once, by i7m_prepare_sqp_fused (never inside a capture)
  auto go = [&](auto kern, int threads) -> hipError_t {
    hipExtLaunchKernelGGL(kern, dim3(P.B), dim3(threads), lds, s, ea, eb, 0, M, P, xu_in, xu_out, xs, goals, fext, lin, cost,
                          qpd, kbuf, sol, active, st, it0);
    return hipGetLastError();
  };
  // (spec, W, fw, loop) -> instantiation
  auto pick = [&](auto spec_c, auto w_c) -> hipError_t {
    constexpr bool SP = decltype(spec_c)::value;
    constexpr int WW = decltype(w_c)::value;
    if (it < 0) return fw ? go(k_sqp_fused<SP, WW, true, true>, 64 * WW) : go(k_sqp_fused<SP, WW, false, true>, 64 * WW);
    return fw ? go(k_sqp_fused<SP, WW, true, false>, 64 * WW) : go(k_sqp_fused<SP, WW, false, false>, 64 * WW);
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  using W1 = std::integral_constant<int, 1>;
  using W4 = std::integral_constant<int, 4>;
  if (W == 4) return spec ? pick(T_{}, W4{}) : pick(F_{}, W4{});
  return spec ? pick(T_{}, W1{}) : pick(F_{}, W1{});
}

// Raise every k_sqp_fused instantiation's dynamic-LDS limit beyond the 64 KB default (four waves
// hold four linearisation regions) to what a horizon of N knots needs, on device `dev`; called by
// i7m_create for a handle that may run the fused pipeline, so launches (and graph captures) never
// call hipFuncSetAttribute.  The limit is per device: one record per device id of the largest
// horizon raised so far, so a second handle on another device (or with a longer horizon) raises
// its own, and a failure is not cached for later handles.
hipError_t i7m_prepare_sqp_fused(int dev, int N) {
  using namespace i7m;
  static std::mutex mu;
  static std::map<int, int> raised;  // device id -> horizon the limits cover
  std::lock_guard<std::mutex> lock(mu);
  const auto it = raised.find(dev);
  if (it != raised.end() && it->second >= N) return hipSuccess;
  hipError_t err = hipSetDevice(dev);
  if (err != hipSuccess) return err;
  auto set = [&](auto kern, int W) {
    const int lds = (int)fused_lds_bytes(18 * N - 6, W);
    const hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess && err == hipSuccess) err = e;
  };
  set(k_sqp_fused<true, 1, false, false>, 1);
  set(k_sqp_fused<true, 1, false, true>, 1);
  set(k_sqp_fused<true, 1, true, false>, 1);
  set(k_sqp_fused<true, 1, true, true>, 1);
  set(k_sqp_fused<false, 1, false, false>, 1);
  set(k_sqp_fused<false, 1, false, true>, 1);
  set(k_sqp_fused<false, 1, true, false>, 1);
  set(k_sqp_fused<false, 1, true, true>, 1);
  set(k_sqp_fused<true, 4, false, false>, 4);
  set(k_sqp_fused<true, 4, false, true>, 4);
  set(k_sqp_fused<true, 4, true, false>, 4);
  set(k_sqp_fused<true, 4, true, true>, 4);
  set(k_sqp_fused<false, 4, false, false>, 4);
  set(k_sqp_fused<false, 4, false, true>, 4);
  set(k_sqp_fused<false, 4, true, false>, 4);
  set(k_sqp_fused<false, 4, true, true>, 4);
  if (err == hipSuccess) raised[dev] = N;
  return err;
}
