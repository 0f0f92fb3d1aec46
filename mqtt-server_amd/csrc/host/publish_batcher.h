// The batching stage of the publish pipeline (north star): publishToSubscribers
// (/root/reference/server.go:984-1021) asks Topics.Subscribers(pk.TopicName) once per publish,
// from many connection goroutines at once. Here those calls are accumulated and matched as one
// GPU batch: producers Submit() a topic and wait on the future; a dispatcher thread seals a
// batch when it holds max_batch topics or its oldest topic has waited max_delay, matches it and
// fulfils the futures in submission order. The results are exactly those of Subscribers(topic)
// on the index state the batch was matched against (readers take no root lock in the reference
// either, topics.go:583, Q11); SelectShared / MergeSharedSelected and the fan-out stay with the
// caller, as in the reference.
//   PublishBatcher      futures of Subscribers (the Go-shaped maps, TopicsIndex::SubscribersBatch)
//   PublishViewBatcher  futures of TopicView (the recipients as a view over the batch's span
//                       result, TopicsIndex::SubscribersViews: no maps are built)
#pragma once

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <exception>
#include <functional>
#include <future>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "topics_index.h"

namespace mq {
namespace host {

template <class R>
class BasicBatcher {
 public:
  struct Stats {
    uint64_t batches = 0;     // match calls
    uint64_t topics = 0;      // topics matched
    uint64_t largest = 0;     // largest batch
  };
  using MatchFn = std::function<std::vector<R>(const std::vector<std::string>&)>;

  BasicBatcher(MatchFn match, size_t max_batch, std::chrono::microseconds max_delay)
      : match_(std::move(match)), max_batch_(max_batch ? max_batch : 1), max_delay_(max_delay),
        th_([this] { run(); }) {}
  ~BasicBatcher() {  // matches what is still queued, then stops the dispatcher
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  BasicBatcher(const BasicBatcher&) = delete;
  BasicBatcher& operator=(const BasicBatcher&) = delete;

  // Thread-safe. The future throws EngineError if the batch's match failed.
  std::future<R> Submit(std::string topic) {
    std::promise<R> p;
    std::future<R> f = p.get_future();
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
  Stats stats() const {
    std::lock_guard<std::mutex> lk(mu_);
    return st_;
  }

 private:
  void run() {
    for (;;) {
      std::vector<std::string> topics;
      std::vector<std::promise<R>> waiters;
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
        std::vector<R> res = match_(topics);
        for (size_t i = 0; i < waiters.size(); i++) waiters[i].set_value(std::move(res[i]));
      } catch (...) {
        for (auto& w : waiters) w.set_exception(std::current_exception());
      }
    }
  }

  MatchFn match_;
  const size_t max_batch_;
  const std::chrono::microseconds max_delay_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::vector<std::string> topics_;
  std::vector<std::promise<R>> waiters_;
  std::chrono::steady_clock::time_point oldest_;
  bool stop_ = false;
  Stats st_;
  std::thread th_;
};

class PublishBatcher : public BasicBatcher<Subscribers> {
 public:
  explicit PublishBatcher(TopicsIndex& ix, size_t max_batch = 65536,
                          std::chrono::microseconds max_delay = std::chrono::microseconds(200))
      : BasicBatcher([&ix](const std::vector<std::string>& t) { return ix.SubscribersBatch(t); }, max_batch,
                     max_delay) {}
};

class PublishViewBatcher : public BasicBatcher<TopicView> {
 public:
  explicit PublishViewBatcher(TopicsIndex& ix, size_t max_batch = 65536,
                              std::chrono::microseconds max_delay = std::chrono::microseconds(200))
      : BasicBatcher([&ix](const std::vector<std::string>& t) { return ix.SubscribersViews(t); }, max_batch,
                     max_delay) {}
};

}  // namespace host
}  // namespace mq
