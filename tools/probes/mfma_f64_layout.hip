// Probe: verify the v_mfma_f64_16x16x4 operand / accumulator lane layouts on gfx950.
// A[row=lane&15][k=lane>>4], B[k=lane>>4][col=lane&15], D[row=(lane>>4)+4i][col=lane&15].
// Computes C = A*B for a 16x16x16 product (4 k-steps) with asymmetric integer data and
// compares with the host product.  Exit code 0 = layout confirmed.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void k(const double* A, const double* B, double* C) {
  const int l = threadIdx.x;
  d4 acc = {0, 0, 0, 0};
  for (int s = 0; s < 4; ++s) {
    double a = A[(l & 15) * 16 + 4 * s + (l >> 4)];
    double b = B[(4 * s + (l >> 4)) * 16 + (l & 15)];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
  for (int i = 0; i < 4; ++i) C[((l >> 4) + 4 * i) * 16 + (l & 15)] = acc[i];
}
int main() {
  double hA[256], hB[256], hC[256], ref[256];
  for (int i = 0; i < 256; ++i) { hA[i] = (i * 7 % 13) - 6; hB[i] = (i * 5 % 11) - 5 + (i / 16); }
  for (int r = 0; r < 16; ++r) for (int c = 0; c < 16; ++c) { double s = 0; for (int m = 0; m < 16; ++m) s += hA[r*16+m]*hB[m*16+c]; ref[r*16+c] = s; }
  double *dA, *dB, *dC;
  hipMalloc(&dA, 2048); hipMalloc(&dB, 2048); hipMalloc(&dC, 2048);
  hipMemcpy(dA, hA, 2048, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 2048, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  hipMemcpy(hC, dC, 2048, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 256; ++i) if (hC[i] != ref[i]) ++bad;
  printf("mfma_f64_16x16x4 layout: %d / 256 mismatches\n", bad);
  return bad != 0;
}
