// Probe: issue rate and dependent latency of v_mfma_f64_16x16x4_f64 on gfx950 (one wave per
// block, one block per CU so the SIMD is otherwise idle).  Prints cycles per MFMA.
//   hipcc --offload-arch=gfx950 -O3 tools/probes/mfma_f64_rate.hip -o /tmp/mfma_rate && /tmp/mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int CHAINS>
__global__ void k(double* out, long long* cyc, int iters) {
  d4 acc[CHAINS];
  for (int c = 0; c < CHAINS; ++c) acc[c] = d4{0.0, 0.0, 0.0, 0.0};
  const double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
  __syncthreads();
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
  }
  double s = 0.0;
  for (int c = 0; c < CHAINS; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  const long long t1 = clock64();
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int CHAINS>
void run(double* d, long long* c, int waves_per_simd) {
  const int iters = 256 / CHAINS;
  // blocks of 64 threads; 256 CUs x 4 SIMDs x waves_per_simd
  const int blocks = 1024 * waves_per_simd;
  hipLaunchKernelGGL(k<CHAINS>, dim3(blocks), dim3(64), 0, 0, d, c, iters);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(k<CHAINS>, dim3(blocks), dim3(64), 0, 0, d, c, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  long long h[4];
  hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
  const double mf = 10.0 * blocks * 256.0;  // MFMAs issued
  printf("chains=%d waves/SIMD=%d: %lld clock64 ticks per MFMA in-wave (%d MFMAs), chip %.1f TFLOP/s f64\n", CHAINS,
         waves_per_simd, h[0] / 256, 256, mf * 2048.0 / (ms * 1e-3) / 1e12);
}

int main() {
  double* d;
  long long* c;
  hipMalloc(&d, 8 * 1024 * 64 * 8);
  hipMalloc(&c, 8 * 1024 * 8);
  run<1>(d, c, 1);
  run<4>(d, c, 1);
  run<1>(d, c, 4);
  run<4>(d, c, 4);
  return 0;
}
