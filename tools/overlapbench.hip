// Copy/compute overlap probe (not part of the engine): does a D2H copy into pinned host memory
// on one stream run beside a kernel on another? Times a memory-bound kernel alone, a 400 MB D2H
// alone, and both issued together on two non-blocking streams (and the D2H split over two
// streams), each with events. Build: hipcc --offload-arch=gfx950 -O2 tools/overlapbench.hip -o build/overlapbench
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

// dependent random reads over a large table (a walk-like kernel): `iters` rounds per thread
__global__ __launch_bounds__(256) void k_chase(const uint32_t* __restrict__ t, uint64_t mask, uint32_t iters,
                                              uint32_t* __restrict__ out) {
  uint32_t x = blockIdx.x * 256 + threadIdx.x;
  for (uint32_t i = 0; i < iters; i++) x = t[(x * 2654435761u + i) & mask] + x;
  if (x == 0x12345678u) out[0] = x;
}

int main() {
  const uint64_t tn = 1ull << 28;  // 1 GiB table
  const size_t copy_bytes = 400ull << 20;
  uint32_t *t = nullptr, *out = nullptr;
  char *dsrc = nullptr, *hdst = nullptr;
  CK(hipMalloc(&t, tn * 4));
  CK(hipMemset(t, 1, tn * 4));
  CK(hipMalloc(&out, 4));
  CK(hipMalloc(&dsrc, copy_bytes));
  CK(hipMemset(dsrc, 2, copy_bytes));
  CK(hipHostMalloc(&hdst, copy_bytes, hipHostMallocDefault));
  hipStream_t a, b, c;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
  hipEvent_t e0, e1, e2, e3;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  CK(hipEventCreate(&e3));
  const uint32_t blocks = 4096, iters = 400;
  auto wall = [] { return std::chrono::steady_clock::now(); };
  auto ms = [](auto x, auto y) { return std::chrono::duration<double, std::milli>(y - x).count(); };
  for (int rep = 0; rep < 3; rep++) {
    // kernel alone
    CK(hipDeviceSynchronize());
    auto w0 = wall();
    hipLaunchKernelGGL(k_chase, dim3(blocks), dim3(256), 0, a, t, tn - 1, iters, out);
    CK(hipStreamSynchronize(a));
    auto w1 = wall();
    // copy alone
    CK(hipMemcpyAsync(hdst, dsrc, copy_bytes, hipMemcpyDeviceToHost, b));
    CK(hipStreamSynchronize(b));
    auto w2 = wall();
    // both
    CK(hipEventRecord(e0, a));
    hipLaunchKernelGGL(k_chase, dim3(blocks), dim3(256), 0, a, t, tn - 1, iters, out);
    CK(hipEventRecord(e1, a));
    CK(hipEventRecord(e2, b));
    CK(hipMemcpyAsync(hdst, dsrc, copy_bytes, hipMemcpyDeviceToHost, b));
    CK(hipEventRecord(e3, b));
    CK(hipStreamSynchronize(a));
    CK(hipStreamSynchronize(b));
    auto w3 = wall();
    float k_ms = 0, c_ms = 0;
    CK(hipEventElapsedTime(&k_ms, e0, e1));
    CK(hipEventElapsedTime(&c_ms, e2, e3));
    // the copy in two halves on two streams, beside the kernel
    CK(hipDeviceSynchronize());
    auto w4 = wall();
    hipLaunchKernelGGL(k_chase, dim3(blocks), dim3(256), 0, a, t, tn - 1, iters, out);
    CK(hipMemcpyAsync(hdst, dsrc, copy_bytes / 2, hipMemcpyDeviceToHost, b));
    CK(hipMemcpyAsync(hdst + copy_bytes / 2, dsrc + copy_bytes / 2, copy_bytes / 2, hipMemcpyDeviceToHost, c));
    CK(hipDeviceSynchronize());
    auto w5 = wall();
    printf("rep %d: kernel alone %.2f ms, D2H alone %.2f ms (%.1f GB/s); together %.2f ms wall (kernel %.2f, copy %.2f "
           "by events); split copy + kernel %.2f ms\n",
           rep, ms(w0, w1), ms(w1, w2), copy_bytes / ms(w1, w2) / 1e6, ms(w2, w3), k_ms, c_ms, ms(w4, w5));
  }
  return 0;
}
