// VALU issue rate on gfx950 for the integer ops the walk and the merge set pass are made of
// (v_add_u32 / v_xor_b32 chains) against f32 FMA, with W waves per SIMD resident: per-wave shader
// cycles per instruction (s_memtime deltas) and the derived SIMD cycles per wave64 instruction.
// Build: hipcc -O3 --offload-arch=gfx950 tools/valubench.hip -o tools/valubench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

template <int KIND>
__global__ __launch_bounds__(256) void k_valu(uint32_t* out, int iters, unsigned long long* cyc) {
  uint32_t a = KIND == 2 ? blockIdx.x : threadIdx.x, b = a * 3u, c = a * 5u, d = a * 7u, e = a ^ 9u, f = a + 11u, g = a * 13u, h = a * 17u;
  float x0 = a, x1 = b, x2 = c, x3 = d, x4 = e, x5 = f, x6 = g, x7 = h;
  const unsigned long long t0 = clock64();
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++) {
      if (KIND == 0 || KIND == 2) {  // integer add / xor, 8 independent chains (2: wave-uniform: SALU)
        a = a + b; b = b ^ c; c = c + d; d = d ^ e; e = e + f; f = f ^ g; g = g + h; h = h ^ a;
      } else {  // f32 fma
        x0 = fmaf(x0, 1.0001f, x1); x1 = fmaf(x1, 0.9999f, x2); x2 = fmaf(x2, 1.0001f, x3); x3 = fmaf(x3, 0.9999f, x4);
        x4 = fmaf(x4, 1.0001f, x5); x5 = fmaf(x5, 0.9999f, x6); x6 = fmaf(x6, 1.0001f, x7); x7 = fmaf(x7, 0.9999f, x0);
      }
    }
  }
  const unsigned long long t1 = clock64();
  const uint32_t r = KIND != 1 ? (a ^ b ^ c ^ d ^ e ^ f ^ g ^ h)
                               : __float_as_uint(x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7);
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int iters = 2000;
  for (int kind = 0; kind < 3; kind++) {
    for (int wps : {1, 2, 4, 8}) {  // waves per SIMD: blocks of 4 waves, wps blocks per CU
      const int blocks = cus * wps;
      uint32_t* out;
      unsigned long long* cyc;
      hipMalloc(&out, (size_t)blocks * 256 * 4);
      hipMalloc(&cyc, (size_t)blocks * 4 * 8);
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      for (int rep = 0; rep < 2; rep++) {
        hipEventRecord(e0, 0);
        if (kind == 0) hipLaunchKernelGGL(k_valu<0>, dim3(blocks), dim3(256), 0, 0, out, iters, cyc);
        else if (kind == 1) hipLaunchKernelGGL(k_valu<1>, dim3(blocks), dim3(256), 0, 0, out, iters, cyc);
        else hipLaunchKernelGGL(k_valu<2>, dim3(blocks), dim3(256), 0, 0, out, iters, cyc);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
      }
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      std::vector<unsigned long long> c((size_t)blocks * 4);
      hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost);
      double avg = 0;
      for (auto v : c) avg += (double)v;
      avg /= c.size();
      const double instr = (double)iters * 16 * 8;
      // per-wave cycles per instruction; with wps waves sharing a SIMD: SIMD cycles per instruction
      const double per_simd = (double)instr * wps;  // instructions one SIMD (or its share of the CU) issued
      std::printf("{\"kind\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"G_instr_per_s_per_simd\": %.3f}\n",
                  kind == 0 ? "int add/xor (VALU)" : kind == 1 ? "f32 fma (VALU)" : "int add/xor uniform (SALU)", wps, ms,
                  per_simd / (ms * 1e-3) / 1e9);
      hipFree(out);
      hipFree(cyc);
    }
  }
  return 0;
}
