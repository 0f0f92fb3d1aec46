// Random-access ceiling for k_walk (not part of the engine): 32-byte records read at random from
// a table the size of the 10M-subscription edge table (134M slots x 32 B = 4.3 GB), one thread
// per "topic" as the walk runs.
//   dep   each thread follows a chain of K dependent loads (the next slot is a hash of the loaded
//         record), as a walk's probes depend on the previous level: latency- and request-bound
//   indep each thread issues K loads whose addresses do not depend on each other
// Prints loads/s and the bytes those loads imply at 32 B (record) and 64 B (HBM access) each.
//   hipcc --offload-arch=gfx950 -O3 tools/randbench.hip -o tools/randbench && tools/randbench
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("%s: %s\n", #x, hipGetErrorString(e));                        \
      return 1;                                                            \
    }                                                                      \
  } while (0)

struct Rec {  // the EdgeSlot's size and alignment
  uint64_t k0, k1;
  uint32_t a, b, c, d;
};

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

__global__ void k_fill(Rec* t, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    t[i] = Rec{mix(i), mix(i + 1), (uint32_t)i, 1u, 2u, 3u};
}

template <bool DEP>
__global__ __launch_bounds__(256) void k_probe(const Rec* __restrict__ t, uint64_t mask, uint32_t n, uint32_t k,
                                               uint64_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t h = mix(i * 0x9E3779B97F4A7C15ull + 7), acc = 0;
  for (uint32_t j = 0; j < k; j++) {
    const Rec r = t[h & mask];
    acc += r.k0 ^ r.a;
    h = DEP ? mix(r.k1 + j) : mix(h + j + 1);
  }
  out[i] = acc;
}

// Coalesced streaming read of the whole table, 16 B per lane (the access width the guide's FETCH_SIZE
// correction is stated for): a known byte count to calibrate the counters against.
__global__ __launch_bounds__(256) void k_stream(const uint4* __restrict__ t, uint64_t n16, uint64_t* __restrict__ out) {
  uint64_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = t[i];
    acc += v.x ^ v.w;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  const uint64_t slots = 1ull << 27;  // 134M x 32 B = 4.3 GB
  const uint32_t topics = 1u << 20, k = 20;
  Rec* t;
  uint64_t* out;
  CK(hipMalloc(&t, slots * sizeof(Rec)));
  CK(hipMalloc(&out, (topics > 65536 * 256 ? topics : 65536 * 256) * sizeof(uint64_t)));
  hipLaunchKernelGGL(k_fill, dim3(65536), dim3(256), 0, 0, t, slots);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int rep = 0; rep < 2; rep++) {  // known bytes: slots x 32 B read, coalesced
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL(k_stream, dim3(65536), dim3(256), 0, 0, reinterpret_cast<const uint4*>(t), slots * 2, out);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("stream read of %.2f GB, 16 B per lane: %.3f ms  %.0f GB/s\n", slots * 32 / 1e9, ms, slots * 32 / ms / 1e6);
  }
  for (int dep = 1; dep >= 0; dep--) {
    for (int rep = 0; rep < 4; rep++) {
      CK(hipEventRecord(a, 0));
      if (dep) hipLaunchKernelGGL(k_probe<true>, dim3(topics / 256), dim3(256), 0, 0, t, slots - 1, topics, k, out);
      else hipLaunchKernelGGL(k_probe<false>, dim3(topics / 256), dim3(256), 0, 0, t, slots - 1, topics, k, out);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      if (rep == 0) continue;  // warm-up
      const double loads = (double)topics * k;
      printf("%-5s %u threads x %u loads of 32 B over 4.3 GB: %.3f ms  %.1f G loads/s  %.0f GB/s at 32 B  %.0f GB/s at 64 B\n",
             dep ? "dep" : "indep", topics, k, ms, loads / ms / 1e6, loads * 32 / ms / 1e6, loads * 64 / ms / 1e6);
    }
  }
  CK(hipFree(t));
  CK(hipFree(out));
  printf("done\n");
  return 0;
}
