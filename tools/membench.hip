// Write-bandwidth probe for the k_copy design (not part of the engine): pure stores and
// list-copies into a 4 GiB destination, nontemporal vs default policy. Prints GB/s per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <bool NT>
__global__ __launch_bounds__(256) void k_store(u32x4* dst, uint64_t n, uint32_t tile) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t w = blockIdx.x * 4ull + (threadIdx.x >> 6);
  const uint64_t x0 = w * tile, x1 = x0 + tile < n ? x0 + tile : n;
  u32x4 v = {(uint32_t)w, lane, 1u, 2u};
  for (uint64_t x = x0 + lane; x < x1; x += 64) {
    if (NT) __builtin_nontemporal_store(v, dst + x); else dst[x] = v;
  }
}

// copy runs of `run` rows from pseudo-random starts in a pool of `pool` rows
template <bool NT, int U>
__global__ __launch_bounds__(256) void k_copyruns(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t n,
                                                 uint32_t tile, uint32_t run, uint32_t pool) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t w = blockIdx.x * 4ull + (threadIdx.x >> 6);
  const uint64_t x0 = w * tile, x1 = x0 + tile < n ? x0 + tile : n;
  for (uint64_t r0 = x0; r0 < x1; r0 += 64 * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      uint64_t x = r0 + u * 64 + lane;
      if (x >= x1) x = x1 - 1;
      const uint64_t rid = x / run;
      const uint32_t start = (uint32_t)((rid * 0x9E3779B97F4A7C15ull) >> 40) % (pool - run);
      v[u] = src[start + (x % run)];
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t x = r0 + u * 64 + lane;
      if (x < x1) { if (NT) __builtin_nontemporal_store(v[u], dst + x); else dst[x] = v[u]; }
    }
  }
}

int main() {
  const uint64_t n = (4ull << 30) / 16;  // 4 GiB of 16-B rows
  const uint32_t pool = 10u << 20;      // 160 MiB source pool
  u32x4 *dst, *src;
  CK(hipMalloc(&dst, n * 16));
  CK(hipMalloc(&src, (uint64_t)pool * 16));
  CK(hipMemset(src, 1, (uint64_t)pool * 16));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 2; i++) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    const int R = 5;
    for (int i = 0; i < R; i++) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("%-40s %8.3f ms  %7.0f GB/s written\n", name, ms / R, n * 16.0 / (ms / R * 1e-3) / 1e9);
    return 0;
  };
  for (uint32_t tile : {1024u, 4096u, 16384u}) {
    const uint32_t waves = (uint32_t)((n + tile - 1) / tile);
    char nm[64];
    snprintf(nm, sizeof nm, "store nt tile %u", tile);
    run(nm, [&] { hipLaunchKernelGGL(k_store<true>, dim3((waves + 3) / 4), dim3(256), 0, 0, dst, n, tile); });
    snprintf(nm, sizeof nm, "store default tile %u", tile);
    run(nm, [&] { hipLaunchKernelGGL(k_store<false>, dim3((waves + 3) / 4), dim3(256), 0, 0, dst, n, tile); });
  }
  for (uint32_t runlen : {64u, 1300u, 5000u}) {
    const uint32_t tile = 4096, waves = (uint32_t)((n + tile - 1) / tile);
    char nm[64];
    snprintf(nm, sizeof nm, "copyruns nt U8 run %u", runlen);
    run(nm, [&] { hipLaunchKernelGGL((k_copyruns<true, 8>), dim3((waves + 3) / 4), dim3(256), 0, 0, src, dst, n, tile, runlen, pool); });
    snprintf(nm, sizeof nm, "copyruns default U8 run %u", runlen);
    run(nm, [&] { hipLaunchKernelGGL((k_copyruns<false, 8>), dim3((waves + 3) / 4), dim3(256), 0, 0, src, dst, n, tile, runlen, pool); });
    snprintf(nm, sizeof nm, "copyruns nt U4 run %u", runlen);
    run(nm, [&] { hipLaunchKernelGGL((k_copyruns<true, 4>), dim3((waves + 3) / 4), dim3(256), 0, 0, src, dst, n, tile, runlen, pool); });
  }
  // small hot source (fits L2): the root-'#' list re-read by every topic
  {
    const uint32_t tile = 4096, waves = (uint32_t)((n + tile - 1) / tile);
    run("copyruns nt U8 run 1300 pool 64K", [&] { hipLaunchKernelGGL((k_copyruns<true, 8>), dim3((waves + 3) / 4), dim3(256), 0, 0, src, dst, n, tile, 1300u, 65536u); });
  }
  printf("done\n");
  return 0;
}
