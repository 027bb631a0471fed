// Probe: back-to-back DPP fma's on one accumulator whose bank masks SHRINK (a lower-triangular
// row: term group t written only to lanes of bank >= t).  Found while building row-split dot
// products for k_admm_iter_res (each 16-lane row one fma chain): without wait states between the
// fma's, the lanes a later fma masks out get back the accumulator as that fma read it, before the
// previous fma's write landed — they lose their earlier terms (lane 13, in bank 3, keeps all
// four and is right).  With `s_nop 1` (the DPP read's two wait states) between them every lane
// is right.  The four-chain forms of i7m_admm.h never meet this: a chain's next fma is four
// instructions behind its last.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/rowsplit_probe.hip -o tools/probes/rowsplit_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <bool NOPS>
__device__ double chain(double v, const double* cf) {
  double a = 0.0;
  if constexpr (NOPS)
    asm volatile(
        "s_nop 1\n\t"
        "v_fmac_f64_dpp %0, %1, %2 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\ts_nop 1\n\t"
        "v_fmac_f64_dpp %0, %1, %3 row_newbcast:4 row_mask:0xf bank_mask:0xe\n\ts_nop 1\n\t"
        "v_fmac_f64_dpp %0, %1, %4 row_newbcast:8 row_mask:0xf bank_mask:0xc\n\ts_nop 1\n\t"
        "v_fmac_f64_dpp %0, %1, %5 row_newbcast:12 row_mask:0xf bank_mask:0x8"
        : "+v"(a)
        : "v"(v), "v"(cf[0]), "v"(cf[1]), "v"(cf[2]), "v"(cf[3]));
  else
    asm volatile(
        "s_nop 1\n\t"
        "v_fmac_f64_dpp %0, %1, %2 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %1, %3 row_newbcast:4 row_mask:0xf bank_mask:0xe\n\t"
        "v_fmac_f64_dpp %0, %1, %4 row_newbcast:8 row_mask:0xf bank_mask:0xc\n\t"
        "v_fmac_f64_dpp %0, %1, %5 row_newbcast:12 row_mask:0xf bank_mask:0x8"
        : "+v"(a)
        : "v"(v), "v"(cf[0]), "v"(cf[1]), "v"(cf[2]), "v"(cf[3]));
  return a;
}

__global__ void __launch_bounds__(64) k(const double* v, const double* cf, double* out) {
  const int l = threadIdx.x, c = l & 15;
  double four[4];
  for (int t = 0; t < 4; ++t) four[t] = cf[16 * c + 4 * t];
  out[l] = chain<false>(v[c], four);
  out[64 + l] = chain<true>(v[c], four);
}

int main() {
  std::vector<double> v(16), cf(256), o(128);
  unsigned s = 12345u;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (double)(s >> 8) / (1 << 24) - 0.5; };
  for (auto& e : v) e = rnd();
  for (auto& e : cf) e = rnd();
  double *dv, *dc, *dout;
  if (hipMalloc(&dv, 8 * 16) != hipSuccess || hipMalloc(&dc, 8 * 256) != hipSuccess || hipMalloc(&dout, 8 * 128) != hipSuccess) return 1;
  (void)hipMemcpy(dv, v.data(), 8 * 16, hipMemcpyHostToDevice);
  (void)hipMemcpy(dc, cf.data(), 8 * 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dv, dc, dout);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  (void)hipMemcpy(o.data(), dout, 8 * 128, hipMemcpyDeviceToHost);
  int bad[2] = {0, 0};
  for (int l = 0; l < 64; ++l) {
    const int c = l & 15, b = c / 4;
    double e = 0.0;  // the chain's terms t <= the lane's bank, in order, each fused
    for (int t = 0; t <= b; ++t) e = __builtin_fma(cf[16 * c + 4 * t], v[4 * t], e);
    for (int n = 0; n < 2; ++n) bad[n] += o[64 * n + l] != e;
  }
  std::printf("{\"probe\": \"dpp_shrinking_bank_mask\", \"wrong_lanes_back_to_back\": %d, \"wrong_lanes_with_s_nop_1\": %d}\n", bad[0], bad[1]);
  return bad[1] ? 2 : 0;
}
