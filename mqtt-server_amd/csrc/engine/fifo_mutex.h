// A mutex that hands itself over in arrival order (a ticket lock over a condition variable).
// std::mutex lets the thread that just unlocked take the lock straight back before a woken
// waiter runs, so two threads updating back to back can keep a third waiting for hundreds of
// milliseconds (measured: one mirror update waited 542 ms for a lock no update held longer than
// 14 ms, profiles/r04/n). Updates take this one instead: each waits at most for the ones that
// arrived before it.
#pragma once

#include <condition_variable>
#include <cstdint>
#include <mutex>

namespace mq {

class FifoMutex {
 public:
  void lock() {
    std::unique_lock<std::mutex> g(mu_);
    const uint64_t ticket = next_++;
    cv_.wait(g, [&] { return serving_ == ticket; });
  }
  void unlock() {
    {
      std::lock_guard<std::mutex> g(mu_);
      serving_++;
    }
    cv_.notify_all();
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  uint64_t next_ = 0, serving_ = 0;
};

}  // namespace mq
