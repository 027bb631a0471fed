// Probe: do fp64 MFMA (v_mfma_f64_16x16x4 / 4x4x4_4b) and fp64 VALU FMA of DIFFERENT waves on one
// SIMD execute side by side, or share one fp64 pipe?  8-wave workgroups (two waves per SIMD), one
// per CU; role of each wave by its index (waves 0-3 one role, 4-7 another), each wave a fixed
// amount of independent work.  Compare the mixed launch with the pure ones:
//   side by side  -> mixed ~ max(pure_mfma, pure_valu) / 2 ... both halves finish as if alone
//   shared pipe   -> mixed ~ (pure_mfma + pure_valu) / 2
// Also the rate of v_mfma_f64_4x4x4_4b (256 FMAs per instruction).
//   hipcc --offload-arch=gfx950 -O3 tools/probes/fp64_pipes.hip -o /tmp/fp64_pipes && /tmp/fp64_pipes
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

// role: 0 = 16x16x4 MFMA, 1 = VALU fma, 2 = 4x4x4 MFMA, 3 = idle
__device__ double work(int role, int iters) {
  const double a = 1.0 + threadIdx.x * 1e-12, b = 1.0 - threadIdx.x * 1e-12;
  double s = 0.0;
  if (role == 0) {
    d4 acc[4];
    for (int c = 0; c < 4; ++c) acc[c] = d4{0.0, 0.0, 0.0, 0.0};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
    }
    for (int c = 0; c < 4; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  } else if (role == 1) {
    // 16 FMA per lane per MFMA-equivalent: one 16x16x4 MFMA = 1024 FMAs = 16 per lane
    double x[8];
    for (int c = 0; c < 8; ++c) x[c] = a + c * 1e-3;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int r = 0; r < 8; ++r) {
#pragma unroll
        for (int c = 0; c < 8; ++c) x[c] = fma(x[c], b, a);
      }
    }
    for (int c = 0; c < 8; ++c) s += x[c];
  } else if (role == 2) {
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[c], 0, 0, 0);
      }
    }
    for (int c = 0; c < 4; ++c) s += acc[c];
  }
  return s;
}

__global__ void __launch_bounds__(512) k(double* out, int lo_role, int hi_role, int iters) {
  const int w = threadIdx.x >> 6;
  const double s = work(w < 4 ? lo_role : hi_role, iters);
  out[blockIdx.x * 512 + threadIdx.x] = s;
}

float run(double* d, int lo, int hi, int iters) {
  const int blocks = 256 * 2;  // two 8-wave workgroups per CU: 4 waves per SIMD
  hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, d, lo, hi, iters);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, d, lo, hi, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  double* d;
  hipMalloc(&d, 8L * 512 * 512);
  const int it = 512;  // per wave: 2048 16x16x4 MFMAs, or 64 x 512 = 32768 FMA instructions (same FMAs)
  const char* nm[4] = {"mfma16", "valu", "mfma4", "idle"};
  const int cases[][2] = {{0, 0}, {1, 1}, {0, 3}, {1, 3}, {0, 1}, {2, 2}, {2, 3}, {2, 1}};
  for (auto& c : cases) {
    const float ms = run(d, c[0], c[1], it);
    printf("waves 0-3 %-6s + waves 4-7 %-6s : %.3f ms\n", nm[c[0]], nm[c[1]], ms);
  }
  return 0;
}
