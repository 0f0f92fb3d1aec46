// The batching stage of the publish pipeline (north star): publishToSubscribers
// (/root/reference/server.go:984-1021) asks Topics.Subscribers(pk.TopicName) once per publish,
// from many connection goroutines at once. Here those calls are accumulated and matched as one
// GPU batch: producers Submit() a topic and wait on the future; a dispatcher thread seals a
// batch when it holds max_batch topics or its oldest topic has waited max_delay, runs
// TopicsIndex::SubscribersBatch and fulfils the futures in submission order. The results are
// exactly those of Subscribers(topic) on the index state the batch was matched against
// (readers take no root lock in the reference either, topics.go:583, Q11); SelectShared /
// MergeSharedSelected and the fan-out stay with the caller, as in the reference.
#pragma once

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <future>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "topics_index.h"

namespace mq {
namespace host {

class PublishBatcher {
 public:
  struct Stats {
    uint64_t batches = 0;     // SubscribersBatch calls
    uint64_t topics = 0;      // topics matched
    uint64_t largest = 0;     // largest batch
  };

  explicit PublishBatcher(TopicsIndex& ix, size_t max_batch = 65536,
                          std::chrono::microseconds max_delay = std::chrono::microseconds(200));
  ~PublishBatcher();  // matches what is still queued, then stops the dispatcher
  PublishBatcher(const PublishBatcher&) = delete;
  PublishBatcher& operator=(const PublishBatcher&) = delete;

  // Thread-safe. The future throws EngineError if the batch's match failed.
  std::future<Subscribers> Submit(std::string topic);
  Stats stats() const;

 private:
  void run();

  TopicsIndex& ix_;
  const size_t max_batch_;
  const std::chrono::microseconds max_delay_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::vector<std::string> topics_;
  std::vector<std::promise<Subscribers>> waiters_;
  std::chrono::steady_clock::time_point oldest_;
  bool stop_ = false;
  Stats st_;
  std::thread th_;
};

}  // namespace host
}  // namespace mq
