// Probe: can buffer_load_dwordx4 ... lds (M0 = the LDS destination) write above 64 KB of LDS on
// gfx950 (160 KB per workgroup)?  A 150 KB static LDS array is filled with -1, one DMA wave-
// instruction lands 1 KB at each of the byte offsets 0, 60 KB, 70 KB, 100 KB and 149 KB, and the
// image is read back: each target must hold the source, nothing else may change.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probes/lds_dma_high_probe.hip -o tools/probes/lds_dma_high_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int NB = 150 * 1024 / 16;  // double2 entries
__global__ void __launch_bounds__(64) k(const double* src, double* out, const int* targets, int nt) {
  __shared__ double2 img[NB];
  const int l = threadIdx.x;
  for (int i = l; i < NB; i += 64) img[i] = make_double2(-1.0, -1.0);
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 1 << 20, 0x00020000);
  const unsigned base = (unsigned)(unsigned long)(__attribute__((address_space(3))) void*)img;
  for (int t = 0; t < nt; ++t) {
    const unsigned lds = base + (unsigned)targets[t];
    const unsigned v = 16u * (64u * t + l);
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %2, %3, 0 offen lds\n\t"
        "s_mov_b32 m0, %0\n\ts_waitcnt vmcnt(0)"
        : "=&s"(keep)
        : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(v), "s"(r)
        : "memory");
  }
  __syncthreads();
  for (int i = l; i < NB; i += 64) {
    out[2 * i] = img[i].x;
    out[2 * i + 1] = img[i].y;
  }
}

int main() {
  const int targets[] = {0, 60 * 1024, 70 * 1024, 100 * 1024, 149 * 1024};
  const int nt = 5;
  std::vector<double> h(nt * 128), o(2 * NB);
  for (int i = 0; i < nt * 128; ++i) h[i] = 1000.0 + i;
  double *ds, *dout;
  int* dt;
  hipMalloc(&ds, 1 << 20);
  hipMalloc(&dout, 16 * NB);
  hipMalloc(&dt, sizeof(targets));
  hipMemcpy(ds, h.data(), 8 * h.size(), hipMemcpyHostToDevice);
  hipMemcpy(dt, targets, sizeof(targets), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, ds, dout, dt, nt);
  if (hipDeviceSynchronize() != hipSuccess) {
    std::printf("{\"probe\": \"lds_dma_high\", \"error\": \"launch\"}\n");
    return 1;
  }
  hipMemcpy(o.data(), dout, 16 * NB, hipMemcpyDeviceToHost);
  std::vector<int> expect(2 * NB, -1);
  for (int t = 0; t < nt; ++t)
    for (int i = 0; i < 128; ++i) expect[targets[t] / 8 + i] = t * 128 + i;
  int bad = 0, first_bad = -1;
  for (int i = 0; i < 2 * NB; ++i) {
    const double e = expect[i] < 0 ? -1.0 : 1000.0 + expect[i];
    if (o[i] != e) {
      if (first_bad < 0) first_bad = i;
      ++bad;
    }
  }
  std::printf("{\"probe\": \"lds_dma_high\", \"targets_kb\": [0, 60, 70, 100, 149], \"wrong_doubles\": %d, \"first_wrong_byte\": %d, \"ok\": %s}\n",
              bad, first_bad < 0 ? -1 : 8 * first_bad, bad == 0 ? "true" : "false");
  return bad == 0 ? 0 : 2;
}
