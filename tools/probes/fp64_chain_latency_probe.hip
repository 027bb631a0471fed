// Probe: the latencies a lone wave's ADMM sweep step is built from (the resident
// kernel's wave is ready but for its own operands half its cycles).  One wave, s_memtime around
// each chain (cycles per link, the loop's own cost included; `realtime` at 100 MHz calibrates the
// clock):
//   fma      dependent v_fma_f64 (a = a * b + c)
//   dpp_fma  dependent v_fmac_f64_dpp row_newbcast, all lanes (the dot products' form), with the two
//            wait states a DPP read of a just-written VGPR needs
//   dot16    the kernel's 16-term dot product (four interleaved chains, closed by three adds), the
//            next dot's broadcast operand its result: per dot
//   rowsum   a row sum of the kernel's form (fma, then row_shr 2 / 4 / 8 adds, a row broadcast): per sum
//   lds      dependent ds_read_b64 (the next address from the value read)
//   lds_dpp  ds_read_b64 then a DPP fma on its value, dependent (a coefficient read feeding a dot)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/fp64_chain_latency_probe.hip -o tools/probes/fp64_chain_latency_probe
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int L = 64;

__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long v;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");
  return v;
}
__device__ __forceinline__ unsigned long long rstamp() {
  unsigned long long v;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");
  return v;
}

__global__ void __launch_bounds__(64) k(const double* in, double* out, unsigned long long* t) {
  __shared__ double lds[1024];
  const int l = threadIdx.x;
  for (int i = l; i < 1024; i += 64) lds[i] = (double)((i * 37 + 11) & 1023);  // a permutation chain
  __syncthreads();
  double a = in[l], b = in[64 + l], c = in[128 + l];
  double cf[16];
  for (int i = 0; i < 16; ++i) cf[i] = in[192 + 16 * (l & 15) + i];
  int n = 0;
  unsigned long long t0, t1, r0, r1;

  r0 = rstamp();
  t0 = stamp();
  for (int i = 0; i < L; ++i) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
  t1 = stamp();
  r1 = rstamp();
  t[n++] = t1 - t0;
  t[n++] = r1 - r0;

  t0 = stamp();
  for (int i = 0; i < L; ++i)
    asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(a) : "v"(b), "v"(c));
  t1 = stamp();
  t[n++] = t1 - t0;

  t0 = stamp();
  for (int i = 0; i < L / 4; ++i) {
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
#define F(acc, op, m) "v_fmac_f64_dpp " acc ", %4, " op " row_newbcast:" #m " row_mask:0xf bank_mask:0xf\n\t"
    asm volatile("s_nop 1\n\t" F("%0", "%5", 0) F("%1", "%6", 1) F("%2", "%7", 2) F("%3", "%8", 3)
                     F("%0", "%9", 4) F("%1", "%10", 5) F("%2", "%11", 6) F("%3", "%12", 7)
                         F("%0", "%13", 8) F("%1", "%14", 9) F("%2", "%15", 10) F("%3", "%16", 11)
                             F("%0", "%17", 12) F("%1", "%18", 13) F("%2", "%19", 14) F("%3", "%20", 15)
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)
                 : "v"(a), "v"(cf[0]), "v"(cf[1]), "v"(cf[2]), "v"(cf[3]), "v"(cf[4]), "v"(cf[5]), "v"(cf[6]),
                   "v"(cf[7]), "v"(cf[8]), "v"(cf[9]), "v"(cf[10]), "v"(cf[11]), "v"(cf[12]), "v"(cf[13]),
                   "v"(cf[14]), "v"(cf[15]));
#undef F
    a = (a0 + a1) + (a2 + a3);
  }
  t1 = stamp();
  t[n++] = t1 - t0;

  t0 = stamp();
  for (int i = 0; i < L / 4; ++i) {
    double p = __fma_rn(b, a, c);
    const long long u = __double_as_longlong(p);
    for (int s = 2; s <= 8; s *= 2) {
      const long long w = __double_as_longlong(p);
      const int ctrl = 0x110 + s;
      int lo, hi;
      if (s == 2) {
        lo = __builtin_amdgcn_update_dpp(0, (int)w, 0x112, 0xf, 0xf, true);
        hi = __builtin_amdgcn_update_dpp(0, (int)(w >> 32), 0x112, 0xf, 0xf, true);
      } else if (s == 4) {
        lo = __builtin_amdgcn_update_dpp(0, (int)w, 0x114, 0xf, 0xf, true);
        hi = __builtin_amdgcn_update_dpp(0, (int)(w >> 32), 0x114, 0xf, 0xf, true);
      } else {
        lo = __builtin_amdgcn_update_dpp(0, (int)w, 0x118, 0xf, 0xf, true);
        hi = __builtin_amdgcn_update_dpp(0, (int)(w >> 32), 0x118, 0xf, 0xf, true);
      }
      (void)ctrl;
      p = p + __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
    }
    (void)u;
    // broadcast lane 15 of the row to the row (row_newbcast through a DPP fma by 1.0)
    double r = 0.0;
    asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:15 row_mask:0xf bank_mask:0xf" : "+v"(r) : "v"(p), "v"(1.0));
    a = r;
  }
  t1 = stamp();
  t[n++] = t1 - t0;

  int idx = l;
  t0 = stamp();
  for (int i = 0; i < L / 2; ++i) idx = (int)lds[idx & 1023];
  t1 = stamp();
  t[n++] = t1 - t0;

  t0 = stamp();
  for (int i = 0; i < L / 2; ++i) {
    double v = lds[idx & 1023];
    asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf" : "+v"(v) : "v"(a), "v"(b));
    idx = (int)v & 1023;
  }
  t1 = stamp();
  t[n++] = t1 - t0;

  out[l] = a + (double)idx;
}

int main() {
  double h[448];
  for (int i = 0; i < 448; ++i) h[i] = 1.0 + 1e-3 * (i % 17);
  double *din, *dout;
  unsigned long long* dt;
  if (hipMalloc(&din, sizeof(h)) != hipSuccess || hipMalloc(&dout, 512) != hipSuccess ||
      hipMalloc(&dt, 16 * 8) != hipSuccess)
    return 1;
  (void)hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
  unsigned long long t[16] = {};
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, din, dout, dt);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    (void)hipMemcpy(t, dt, 16 * 8, hipMemcpyDeviceToHost);
  }
  const double mhz = t[1] ? 100.0 * (double)t[0] / (double)t[1] : 0.0;  // s_memtime ticks per us
  std::printf("{\"probe\": \"fp64_chain_latency\", \"memtime_MHz\": %.0f, \"per_link\": {\"fma\": %.1f, \"dpp_fma\": %.1f, "
              "\"dot16\": %.1f, \"rowsum\": %.1f, \"lds\": %.1f, \"lds_dpp\": %.1f}}\n",
              mhz, (double)t[0] / L, (double)t[2] / L, (double)t[3] / (L / 4), (double)t[4] / (L / 4), (double)t[5] / (L / 2),
              (double)t[6] / (L / 2));
  return 0;
}
