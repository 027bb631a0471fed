// Probe: operand / result lane layout of v_mfma_f64_4x4x4_4b (four independent 4x4x4 blocks).
// For every A lane L: A = e_L (one-hot), B[lane] = lane + 1; then D[o] is the index + 1 of the B
// lane multiplied with A lane L into output lane o (0 if none).  Prints 64 lines "L: D[0..63]".
//   hipcc --offload-arch=gfx950 -O3 tools/probes/mfma_f64_4x4_layout.hip -o /tmp/l44 && /tmp/l44
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(double* out) {
  const int l = threadIdx.x;
  for (int L = 0; L < 64; ++L) {
    const double a = (l == L) ? 1.0 : 0.0;
    const double b = (double)(l + 1);
    const double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
    out[L * 64 + l] = d;
  }
}
int main() {
  double* d;
  if (hipMalloc(&d, 64 * 64 * 8) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  double h[64 * 64];
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int L = 0; L < 64; ++L) {
    printf("%d:", L);
    for (int o = 0; o < 64; ++o) printf(" %d", (int)h[L * 64 + o]);
    printf("\n");
  }
  return 0;
}
