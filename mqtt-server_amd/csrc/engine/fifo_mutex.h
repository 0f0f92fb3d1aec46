// A mutex that hands itself over in arrival order (a ticket lock over a condition variable).
// std::mutex lets the thread that just unlocked take the lock straight back before a woken
// waiter runs, so two threads updating back to back can keep a third waiting for hundreds of
// milliseconds (measured: one mirror update waited 542 ms for a lock no update held longer than
// 14 ms, profiles/r04/n). Updates take this one instead: each waits at most for the ones that
// arrived before it.
// A waiter spins a little (kSpinNs) before it sleeps: the host image's critical sections are tens of
// microseconds, and a waiter woken from the condition variable on a busy host was measured taking
// 3 ms to run (an update waited 3.1 ms for a lock no update held longer than 0.1 ms,
// profiles/r06/k) — with a ticket lock every later waiter waits for that one too.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <thread>

namespace mq {

class FifoMutex {
 public:
  void lock() {
    const uint64_t ticket = next_.fetch_add(1, std::memory_order_relaxed);
    if (serving_.load(std::memory_order_acquire) == ticket) return;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t k = 1;; k++) {
      if (serving_.load(std::memory_order_acquire) == ticket) return;
      if ((k & 63) == 0) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::nanoseconds(kSpinNs)) break;
        std::this_thread::yield();
      }
    }
    std::unique_lock<std::mutex> g(mu_);
    cv_.wait(g, [&] { return serving_.load(std::memory_order_acquire) == ticket; });
  }
  void unlock() {
    {
      std::lock_guard<std::mutex> g(mu_);  // (a waiter between its check and its sleep sees the change)
      serving_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
  }

 private:
  static constexpr int64_t kSpinNs = 200000;
  std::atomic<uint64_t> next_{0}, serving_{0};
  std::mutex mu_;
  std::condition_variable cv_;
};

}  // namespace mq
