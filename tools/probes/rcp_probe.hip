// Accuracy of v_rcp_f64 and of one / two Newton steps after it, against the correctly rounded
// host 1/d, over pivots spanning [1e-8, 1e8] (the Riccati H pivots are R + B'VB: ~1e-5..1e3).
//   hipcc --offload-arch=gfx950 -O3 tools/probes/rcp_probe.hip -o /tmp/rcp_probe && /tmp/rcp_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

__global__ void k_rcp(const double* d, double* r0, double* r1, double* r2, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double x = d[i];
  double y = __builtin_amdgcn_rcp(x);
  r0[i] = y;
  y = fma(y, fma(-x, y, 1.0), y);
  r1[i] = y;
  y = fma(y, fma(-x, y, 1.0), y);
  r2[i] = y;
}

static double ulps(double a, double b) {  // |a - b| in ulps of b
  int64_t ia, ib;
  std::memcpy(&ia, &a, 8);
  std::memcpy(&ib, &b, 8);
  return std::fabs((double)(ia - ib));
}

int main() {
  const int n = 1 << 22;
  std::vector<double> d(n), r0(n), r1(n), r2(n);
  std::mt19937_64 g(7);
  std::uniform_real_distribution<double> u(-8.0, 8.0);
  for (auto& x : d) x = std::pow(10.0, u(g));
  double *dd, *a, *b, *c;
  if (hipMalloc(&dd, n * 8) || hipMalloc(&a, n * 8) || hipMalloc(&b, n * 8) || hipMalloc(&c, n * 8)) return 1;
  if (hipMemcpy(dd, d.data(), n * 8, hipMemcpyHostToDevice)) return 1;
  k_rcp<<<n / 256, 256>>>(dd, a, b, c, n);
  if (hipMemcpy(r0.data(), a, n * 8, hipMemcpyDeviceToHost) || hipMemcpy(r1.data(), b, n * 8, hipMemcpyDeviceToHost) ||
      hipMemcpy(r2.data(), c, n * 8, hipMemcpyDeviceToHost))
    return 1;
  double m0 = 0, m1 = 0, m2 = 0;
  for (int i = 0; i < n; ++i) {
    const double ex = 1.0 / d[i];
    m0 = std::fmax(m0, ulps(r0[i], ex));
    m1 = std::fmax(m1, ulps(r1[i], ex));
    m2 = std::fmax(m2, ulps(r2[i], ex));
  }
  std::printf("max ulp error over %d pivots: v_rcp_f64 %.0f, +1 Newton %.0f, +2 Newton %.0f\n", n, m0, m1, m2);
  return 0;
}
