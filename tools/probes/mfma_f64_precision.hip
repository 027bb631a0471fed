// Probe: arithmetic precision of v_mfma_f64_4x4x4_4b against v_mfma_f64_16x16x4 and an fma chain,
// on random operands: each lane prints its result so the host can compare with exact sums.
// Output: "<kind> <lane> <value %.17g>" lines.
//   hipcc --offload-arch=gfx950 -O3 tools/probes/mfma_f64_precision.hip -o /tmp/mp && /tmp/mp
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void k(const double* A, const double* B, const double* C, double* o44, double* o16) {
  const int l = threadIdx.x;
  o44[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(A[l], B[l], C[l], 0, 0, 0);
  d4 c = {C[l], C[64 + l], C[128 + l], C[192 + l]};
  d4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(A[l], B[l], c, 0, 0, 0);
  for (int i = 0; i < 4; ++i) o16[64 * i + l] = d[i];
}
int main() {
  double hA[64], hB[64], hC[256];
  unsigned long long x = 88172645463325252ull;
  auto rnd = [&]() {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    return ((double)(x >> 11) / 9007199254740992.0) * 2.0 - 1.0;
  };
  for (int i = 0; i < 64; ++i) { hA[i] = rnd() * (1.0 + 1000.0 * (i % 3 == 0)); hB[i] = rnd() / 3.0; }
  for (int i = 0; i < 256; ++i) hC[i] = rnd() * 1e-3;
  double *dA, *dB, *dC, *d44, *d16;
  if (hipMalloc(&dA, 512) || hipMalloc(&dB, 512) || hipMalloc(&dC, 2048) || hipMalloc(&d44, 512) || hipMalloc(&d16, 2048))
    return 1;
  if (hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice) || hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice) ||
      hipMemcpy(dC, hC, 2048, hipMemcpyHostToDevice))
    return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC, d44, d16);
  double h44[64], h16[256];
  if (hipMemcpy(h44, d44, 512, hipMemcpyDeviceToHost) || hipMemcpy(h16, d16, 2048, hipMemcpyDeviceToHost)) return 1;
  for (int i = 0; i < 64; ++i) printf("A %d %.17g\nB %d %.17g\n", i, hA[i], i, hB[i]);
  for (int i = 0; i < 256; ++i) printf("C %d %.17g\n", i, hC[i]);
  for (int i = 0; i < 64; ++i) printf("D44 %d %.17g\n", i, h44[i]);
  for (int i = 0; i < 256; ++i) printf("D16 %d %.17g\n", i, h16[i]);
  return 0;
}
