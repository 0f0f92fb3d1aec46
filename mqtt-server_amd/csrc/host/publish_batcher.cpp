// Publish batching stage over the host TopicsIndex (publish_batcher.h).
#include "publish_batcher.h"

#include <exception>
#include <utility>

namespace mq {
namespace host {

PublishBatcher::PublishBatcher(TopicsIndex& ix, size_t max_batch, std::chrono::microseconds max_delay)
    : ix_(ix), max_batch_(max_batch ? max_batch : 1), max_delay_(max_delay), th_([this] { run(); }) {}

PublishBatcher::~PublishBatcher() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  th_.join();
}

std::future<Subscribers> PublishBatcher::Submit(std::string topic) {
  std::promise<Subscribers> p;
  std::future<Subscribers> f = p.get_future();
  bool wake = false;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (topics_.empty()) {
      oldest_ = std::chrono::steady_clock::now();
      wake = true;  // starts the delay timer
    }
    topics_.push_back(std::move(topic));
    waiters_.push_back(std::move(p));
    wake |= topics_.size() >= max_batch_;
  }
  if (wake) cv_.notify_one();
  return f;
}

PublishBatcher::Stats PublishBatcher::stats() const {
  std::lock_guard<std::mutex> lk(mu_);
  return st_;
}

void PublishBatcher::run() {
  for (;;) {
    std::vector<std::string> topics;
    std::vector<std::promise<Subscribers>> waiters;
    {
      std::unique_lock<std::mutex> lk(mu_);
      for (;;) {
        if (!topics_.empty() &&
            (stop_ || topics_.size() >= max_batch_ || std::chrono::steady_clock::now() - oldest_ >= max_delay_))
          break;
        if (stop_) return;  // nothing queued
        if (topics_.empty()) cv_.wait(lk);
        else cv_.wait_until(lk, oldest_ + max_delay_);
      }
      const size_t n = std::min(topics_.size(), max_batch_);
      topics.assign(std::make_move_iterator(topics_.begin()), std::make_move_iterator(topics_.begin() + n));
      waiters.assign(std::make_move_iterator(waiters_.begin()), std::make_move_iterator(waiters_.begin() + n));
      topics_.erase(topics_.begin(), topics_.begin() + n);
      waiters_.erase(waiters_.begin(), waiters_.begin() + n);
      if (!topics_.empty()) oldest_ = std::chrono::steady_clock::now();
      st_.batches++;
      st_.topics += n;
      if (n > st_.largest) st_.largest = n;
    }
    try {
      std::vector<Subscribers> res = ix_.SubscribersBatch(topics);
      for (size_t i = 0; i < waiters.size(); i++) waiters[i].set_value(std::move(res[i]));
    } catch (...) {
      for (auto& w : waiters) w.set_exception(std::current_exception());
    }
  }
}

}  // namespace host
}  // namespace mq
