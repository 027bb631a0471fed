// Probe: fp64 DPP broadcast (v_fmac_f64_dpp / v_mov_b64_dpp row_newbcast:n) on gfx950.
// Each 16-lane row r holds a vector x (lane c: x_c) and computes y_c = sum_j A[c][j] x_j with
// v_fmac_f64_dpp acc, x(bcast lane j of the row), A[c][j].  Checked against a host matvec.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probes/dpp64_probe.hip -o tools/probes/dpp64_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

template <int n>
__device__ __forceinline__ void fmac_bc(double& acc, double x, double a) {
  asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
               : "+v"(acc) : "v"(x), "v"(a), "i"(n));
}
template <int n>
__device__ __forceinline__ double mov_bc(double x) {
  double r;
  asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(x), "i"(n));
  return r;
}

template <int j>
__device__ __forceinline__ void step(double& acc, double x, const double* arow) {
  if constexpr (j < 16) {
    fmac_bc<j>(acc, x, arow[j]);
    step<j + 1>(acc, x, arow);
  }
}

__global__ void k(const double* A, const double* X, double* Y, double* B) {
  const int l = threadIdx.x, r = l / 16, c = l % 16;
  const double x = X[l];
  double acc = 0.0;
  step<0>(acc, x, A + (r * 16 + c) * 16);
  Y[l] = acc;
  B[l] = mov_bc<7>(x);
}

int main() {
  std::vector<double> A(64 * 16), X(64), Y(64), Bc(64);
  for (int i = 0; i < 64 * 16; ++i) A[i] = std::sin(0.37 * i + 1.0);
  for (int i = 0; i < 64; ++i) X[i] = std::cos(0.11 * i) + 0.01 * i;
  double *dA, *dX, *dY, *dB;
  hipMalloc(&dA, A.size() * 8);
  hipMalloc(&dX, 64 * 8);
  hipMalloc(&dY, 64 * 8);
  hipMalloc(&dB, 64 * 8);
  hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dX, X.data(), 64 * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dX, dY, dB);
  hipMemcpy(Y.data(), dY, 64 * 8, hipMemcpyDeviceToHost);
  hipMemcpy(Bc.data(), dB, 64 * 8, hipMemcpyDeviceToHost);
  double err = 0.0, berr = 0.0;
  for (int l = 0; l < 64; ++l) {
    const int r = l / 16, c = l % 16;
    double acc = 0.0;
    for (int j = 0; j < 16; ++j) acc = std::fma(X[r * 16 + j], A[(r * 16 + c) * 16 + j], acc);
    err = std::fmax(err, std::fabs(acc - Y[l]));
    berr = std::fmax(berr, std::fabs(Bc[l] - X[r * 16 + 7]));
  }
  std::printf("{\"probe\": \"dpp64_row_newbcast\", \"fmac_max_abs_err\": %.3e, \"mov_max_abs_err\": %.3e, \"ok\": %s}\n", err,
              berr, (err == 0.0 && berr == 0.0) ? "true" : "false");
  return (err == 0.0 && berr == 0.0) ? 0 : 1;
}
