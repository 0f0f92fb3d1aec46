// Which HIP call pays a thread's one-time runtime set-up (a reader's first
// match on a new OS thread held the handle lock ~10 ms longer). On fresh threads, times each call
// of the sequence a span batch makes, in order; the main thread has set the device up already.
// Build: hipcc -O2 tools/thread_init.cpp -o tools/thread_init
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

int main() {
  using clk = std::chrono::steady_clock;
  CK(hipSetDevice(0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  void* d = nullptr;
  void* h = nullptr;
  CK(hipMalloc(&d, 1 << 20));
  CK(hipHostMalloc(&h, 1 << 20, hipHostMallocDefault));
  CK(hipMemcpyAsync(h, d, 4096, hipMemcpyDeviceToHost, s));
  CK(hipStreamSynchronize(s));
  for (int round = 0; round < 3; round++) {
    std::thread t([&] {
      std::vector<std::pair<const char*, double>> ts;
      auto step = [&](const char* name, auto&& f) {
        const auto t0 = clk::now();
        f();
        ts.emplace_back(name, std::chrono::duration<double, std::milli>(clk::now() - t0).count());
      };
      hipEvent_t ev;
      step("hipGetLastError", [&] { (void)hipGetLastError(); });
      step("hipSetDevice", [&] { CK(hipSetDevice(0)); });
      step("hipStreamQuery", [&] { (void)hipStreamQuery(s); });
      step("hipEventCreate", [&] { CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming)); });
      step("hipMemcpyAsync H2D", [&] { CK(hipMemcpyAsync(d, h, 4096, hipMemcpyHostToDevice, s)); });
      step("hipMemsetAsync", [&] { CK(hipMemsetAsync(d, 0, 64, s)); });
      step("hipEventRecord", [&] { CK(hipEventRecord(ev, s)); });
      step("hipStreamSynchronize", [&] { CK(hipStreamSynchronize(s)); });
      step("hipMemcpyAsync D2H + sync", [&] {
        CK(hipMemcpyAsync(h, d, 4096, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
      });
      step("hipEventDestroy", [&] { CK(hipEventDestroy(ev)); });
      std::printf("{\"round\": %d", round);
      for (auto& p : ts) std::printf(", \"%s\": %.3f", p.first, p.second);
      std::printf("}\n");
    });
    t.join();
  }
  CK(hipFree(d));
  CK(hipHostFree(h));
  CK(hipStreamDestroy(s));
  return 0;
}
