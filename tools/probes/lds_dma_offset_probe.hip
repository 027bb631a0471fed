// Probe: does a buffer_load_dwordx4 ... lds instruction offset move the LDS destination as well as
// the memory address?  Each lane loads 16 B from src + 16 lane + OFF (voffset 16 lane - OFF when
// compensated) into LDS at M0 + OFF? + 16 lane; the LDS image is read back and compared.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probes/lds_dma_offset_probe.hip -o tools/probes/lds_dma_offset_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k(const double* src, double* out) {
  __shared__ double2 ring[256];  // 4 KB
  const int l = threadIdx.x;
  for (int i = l; i < 256; i += 64) ring[i] = make_double2(-1.0, -1.0);
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 8192, 0x00020000);
  const unsigned lds = (unsigned)(unsigned long)(__attribute__((address_space(3))) void*)ring;
  // instruction 0: offset 0, voffset 16 l -> src pieces 0..63 ; instruction 1: offset:1024 with
  // voffset 16 l (memory pieces 64..127); where do they land?
  const unsigned v0 = 16u * l;
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %2, %3, 0 offen lds\n\t"
      "buffer_load_dwordx4 %2, %3, 0 offen offset:1024 lds\n\t"
      "buffer_load_dwordx4 %2, %3, 0 offen offset:2048 lds\n\t"
      "s_mov_b32 m0, %0\n\ts_waitcnt vmcnt(0)"
      : "=&s"(keep) : "s"(lds), "v"(v0), "s"(r) : "memory");
  __syncthreads();
  for (int i = l; i < 256; i += 64) {
    out[2 * i] = ring[i].x;
    out[2 * i + 1] = ring[i].y;
  }
}

int main() {
  std::vector<double> h(1024), o(512);
  for (int i = 0; i < 1024; ++i) h[i] = i;
  double *ds, *dout;
  hipMalloc(&ds, 8192);
  hipMalloc(&dout, 4096);
  hipMemcpy(ds, h.data(), 8192, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, ds, dout);
  hipMemcpy(o.data(), dout, 4096, hipMemcpyDeviceToHost);
  // expectation A (offset moves LDS too): LDS double i = src double i for i < 384
  // expectation B (offset moves memory only): LDS doubles 0..127 = src 256..383 (last write wins)
  bool a = true, b = true;
  for (int i = 0; i < 384; ++i) a = a && o[i] == (double)i;
  for (int i = 0; i < 128; ++i) b = b && o[i] == (double)(256 + i);
  std::printf("{\"probe\": \"lds_dma_inst_offset\", \"offset_moves_lds\": %s, \"offset_memory_only\": %s, \"lds0\": %g, \"lds128\": %g, \"lds256\": %g}\n",
              a ? "true" : "false", b ? "true" : "false", o[0], o[128], o[256]);
  return 0;
}
