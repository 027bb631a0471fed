// Probe: lane mapping of v_permlane32_swap / v_permlane16_swap / DPP row_newbcast on gfx950.
// Prints, for each lane, the source lane each result came from (inputs = lane ids).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* o) {
  const unsigned x = threadIdx.x;
  auto r32 = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  auto r16 = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  const int b3 = __builtin_amdgcn_update_dpp(-1, (int)x, 0x153, 0xf, 0xf, false);
  const int s6 = __builtin_amdgcn_update_dpp(-1, (int)x, 0x106, 0xf, 0xf, false);
  const int r6 = __builtin_amdgcn_update_dpp(-1, (int)x, 0x116, 0xf, 0xf, false);
  int* p = o + 7 * threadIdx.x;
  p[0] = r32[0]; p[1] = r32[1]; p[2] = r16[0]; p[3] = r16[1]; p[4] = b3; p[5] = s6; p[6] = r6;
}
int main() {
  int* d; hipMalloc(&d, 64 * 7 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  int h[64 * 7]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("lane: p32.vdst p32.vsrc p16.vdst p16.vsrc newbcast3 row_shl6 row_shr6\n");
  for (int l = 0; l < 64; ++l) printf("%2d: %2d %2d %2d %2d %2d %2d %2d\n", l, h[7*l], h[7*l+1], h[7*l+2], h[7*l+3], h[7*l+4], h[7*l+5], h[7*l+6]);
  return 0;
}
