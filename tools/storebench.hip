// Store-pattern probe for k_hot (not part of the engine): 4 GiB written as
//  (a) 64 KiB contiguous per wave, (b) 8 KiB pieces at scattered places,
//  (c) 16 interleaved streams per wave, 8 KiB per stream per round (64 KiB per stream).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

// mode 0: wave w writes rows [w*4096, +4096)
// mode 1: wave w writes 8 pieces of 512 rows at piece ids perm(w*8 + k)
// mode 2: wave w owns 16 streams of 4096 rows (a 64K-row region), writes 512 rows to each in turn
__global__ __launch_bounds__(256) void k_pat(u32x4* dst, uint64_t n, int mode) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t w = blockIdx.x * 4ull + (threadIdx.x >> 6);
  const u32x4 v = {(uint32_t)w, lane, 7u, 9u};
  if (mode == 0) {
    const uint64_t x0 = w * 4096;
    for (uint32_t r = lane; r < 4096; r += 64) if (x0 + r < n) __builtin_nontemporal_store(v, dst + x0 + r);
  } else if (mode == 1) {
    const uint64_t pieces = n / 512;
    for (uint32_t k = 0; k < 8; k++) {
      const uint64_t pid = ((w * 8 + k) * 0x9E3779B97F4A7C15ull >> 20) % pieces;
      for (uint32_t r = lane; r < 512; r += 64) __builtin_nontemporal_store(v, dst + pid * 512 + r);
    }
  } else {
    const uint64_t base = (w / 16) * 65536;  // 16 waves share... each wave: 16 streams
    const uint64_t region = w * 65536;
    if (region + 65536 > n) return;
    for (uint32_t round = 0; round < 8; round++)
      for (uint32_t st = 0; st < 16; st++)
        for (uint32_t r = lane; r < 512; r += 64)
          __builtin_nontemporal_store(v, dst + region + st * 4096 + round * 512 + r);
    (void)base;
  }
}

int main() {
  const uint64_t n = (4ull << 30) / 16;
  u32x4* dst;
  CK(hipMalloc(&dst, n * 16));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const char* names[3] = {"64 KiB contiguous per wave", "8 KiB scattered pieces", "16 interleaved streams per wave"};
  for (int mode = 0; mode < 3; mode++) {
    const uint64_t rows_per_wave = mode == 2 ? 65536 : 4096;
    const uint32_t waves = (uint32_t)(n / rows_per_wave);
    for (int i = 0; i < 2; i++) hipLaunchKernelGGL(k_pat, dim3(waves / 4), dim3(256), 0, 0, dst, n, mode);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < 5; i++) hipLaunchKernelGGL(k_pat, dim3(waves / 4), dim3(256), 0, 0, dst, n, mode);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("%-36s %7.3f ms %7.0f GB/s\n", names[mode], ms / 5, n * 16.0 / (ms / 5 * 1e-3) / 1e9);
  }
  return 0;
}
