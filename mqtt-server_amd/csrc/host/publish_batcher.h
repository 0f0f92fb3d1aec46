// The batching stage of the publish pipeline (north star): publishToSubscribers
// (/root/reference/server.go:984-1021) asks Topics.Subscribers(pk.TopicName) once per publish,
// from many connection goroutines at once. Here those calls are accumulated and matched as one
// GPU batch: producers Submit() a topic and get() its ticket; a dispatcher thread seals a batch
// and matches it with one engine call. The results are exactly those of Subscribers(topic) on
// the index state the batch was matched against (readers take no root lock in the reference
// either, topics.go:583, Q11); the OnSelectSubscribers hook, SelectShared / MergeSharedSelected
// and the fan-out stay with the caller, as in the reference (hooks.go:360-367).
//
// Submission is sharded: a producer appends to one of kShards queues (picked per thread), each
// with its own lock, so thousands of submitters do not serialise on one mutex; a ticket names
// its queue's segment of the batch (one shared, reference-counted record per queue and batch,
// not one promise per topic), and a batch is completed by one notification per segment.
//
// Sealing policy: the dispatcher takes everything queued when the previous batch is done — so
// under load a batch holds what arrived while the last one was matched — and, when fewer than
// min_fill topics are queued and the previous batch held more than one (there is concurrent
// load), waits up to max_delay for more; a lone topic on an idle stage is matched at once.
// max_batch bounds a batch.
//
// Errors: a match call that throws is tried again after 0, 1, 4, 16, 64 and 256 ms (kRetryDelays:
// a transient failure — a kernel guard tripped by one batch, a device reset — costs retries, not
// the batch's deliveries); if every attempt throws, every ticket of the batch rethrows the error
// from get(): the callers see it, nothing is answered empty (there is no CPU matching path), and
// the stage goes on with the next batch. The Go shim's batcher does the same (go/topics_gpu.go).
//   PublishBatcher      tickets of Subscribers (the Go-shaped maps, TopicsIndex::SubscribersBatch)
//   PublishViewBatcher  tickets of TopicView (the recipients as a view over the batch's span
//                       result, TopicsIndex::SubscribersViews: no maps are built)
#pragma once

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <utility>
#include <vector>

#include "topics_index.h"

namespace mq {
namespace host {

// Policy: Batch — one match call's result; Item — what a ticket's get() gives;
// item(batch, i) — topic i's Item; match(index, packed topics) — the engine call.
template <class Policy>
class BasicBatcher {
  using Batch = typename Policy::Batch;
  using Item = typename Policy::Item;
  // One queue's part of one batch: its topics are the batch's [base, base + n).
  struct Segment {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
    std::shared_ptr<const Batch> results;  // the batch's results (null: it failed)
    std::exception_ptr err;
    uint32_t base = 0;
    std::chrono::steady_clock::time_point done_at;  // when the batch completed
  };
  // A submission queue: its topics packed as they come (bytes + offsets: sealing swaps the
  // buffers out, it does not move strings one by one).
  struct alignas(64) Shard {
    std::mutex mu;
    PackedTopics q;
    std::shared_ptr<Segment> seg;  // the segment the queued topics belong to
  };
  static constexpr uint32_t kShards = 64;  // (as many as typical submitters: each thread its own lock)

 public:
  struct Stats {
    uint64_t batches = 0;     // match calls
    uint64_t retried = 0;     // batches whose first match call failed
    uint64_t attempts = 0;    // match calls that failed and were tried again
    uint64_t failed = 0;      // batches whose every attempt failed (their tickets throw)
    uint64_t topics = 0;      // topics matched
    uint64_t largest = 0;     // largest batch
    // the dispatcher's time (ns): waiting for topics, sealing, in the match call, completing
    uint64_t wait_ns = 0, seal_ns = 0, match_ns = 0, complete_ns = 0;
  };
  using MatchFn = std::function<std::shared_ptr<const Batch>(const PackedTopics&)>;

  // A submitted topic: get() waits for its batch and returns its result (throws EngineError if
  // the batch's match failed). Valid until destroyed; copies share the result.
  class Ticket {
   public:
    Ticket() = default;
    Item get() const {
      wait();
      if (seg_->err) std::rethrow_exception(seg_->err);
      return Policy::item(seg_->results, seg_->base + idx_);
    }
    void wait() const {
      std::unique_lock<std::mutex> lk(seg_->mu);
      seg_->cv.wait(lk, [&] { return seg_->done; });
    }
    bool ready() const {
      std::lock_guard<std::mutex> lk(seg_->mu);
      return seg_->done;
    }
    bool valid() const { return seg_ != nullptr; }
    // when the ticket's batch completed (valid once ready()): for latency measurements
    std::chrono::steady_clock::time_point done_at() const {
      std::lock_guard<std::mutex> lk(seg_->mu);
      return seg_->done_at;
    }

   private:
    friend class BasicBatcher;
    Ticket(std::shared_ptr<Segment> s, uint32_t i) : seg_(std::move(s)), idx_(i) {}
    std::shared_ptr<Segment> seg_;
    uint32_t idx_ = 0;
  };

  BasicBatcher(MatchFn match, size_t max_batch, std::chrono::microseconds max_delay, size_t min_fill = 1024)
      : match_(std::move(match)), max_batch_(max_batch ? max_batch : 1), max_delay_(max_delay),
        min_fill_(std::min(min_fill, max_batch_)), th_([this] { run(); }) {}
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

  // Thread-safe.
  Ticket Submit(std::string_view topic) {
    static std::atomic<uint32_t> next_shard{0};
    thread_local const uint32_t my = next_shard.fetch_add(1, std::memory_order_relaxed);
    Shard& sh = shards_[my % kShards];
    Ticket t;
    uint64_t q;
    {
      std::lock_guard<std::mutex> lk(sh.mu);
      if (!sh.seg) sh.seg = std::make_shared<Segment>();
      t = Ticket(sh.seg, sh.q.size());
      sh.q.add(topic);
      // counted under the queue's lock: the dispatcher subtracts only topics it took, so the
      // count never runs below what is queued
      q = queued_.fetch_add(1, std::memory_order_acq_rel) + 1;
    }
    if (q == 1 || q == min_fill_ || q == max_batch_) {  // the dispatcher may be waiting for this
      std::lock_guard<std::mutex> lk(mu_);
      cv_.notify_one();
    }
    return t;
  }
  Stats stats() const {
    std::lock_guard<std::mutex> lk(mu_);
    return st_;
  }

 private:
  void run() {
    PackedTopics batch;
    PackedTopics spare[kShards];  // emptied buffers, swapped into the queues at the next seal
    std::vector<std::pair<std::shared_ptr<Segment>, uint32_t>> segs;  // (segment, its first topic)
    std::vector<uint32_t> taken;                                       // queues sealed into the batch
    using Clock = std::chrono::steady_clock;
    auto ns = [](Clock::time_point a, Clock::time_point b) {
      return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count();
    };
    for (;;) {
      const auto c0 = Clock::now();
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || queued_.load(std::memory_order_acquire) != 0; });
        if (stop_ && queued_.load() == 0) return;
        // a small batch waits up to max_delay for more (the clock starts at its first topic)
        if (!stop_ && last_n_ > 1 && queued_.load() < min_fill_) {
          const auto until = std::chrono::steady_clock::now() + max_delay_;
          cv_.wait_until(lk, until, [&] { return stop_ || queued_.load() >= min_fill_; });
        }
      }
      const auto c1 = Clock::now();
      // seal: every queue's topics, in queue order (at most max_batch; a queue that would
      // overflow the batch keeps its topics and its segment for the next one). Under a queue's
      // lock only its buffers are swapped for empty ones; the packing happens after.
      segs.clear();
      taken.clear();
      uint64_t n = 0;
      for (uint32_t k = 0; k < kShards; k++) {
        const uint32_t s = (k + rr_) % kShards;
        Shard& sh = shards_[s];
        std::lock_guard<std::mutex> lk(sh.mu);
        if (sh.q.empty()) continue;
        if (n && n + sh.q.size() > max_batch_) continue;
        segs.emplace_back(std::move(sh.seg), (uint32_t)n);
        n += sh.q.size();
        std::swap(sh.q, spare[s]);
        taken.push_back(s);
      }
      rr_++;  // the next batch starts at another queue (none waits behind the others for ever)
      if (!n) continue;
      queued_.fetch_sub(n, std::memory_order_acq_rel);
      batch.clear();
      size_t nb = 0;
      for (uint32_t s : taken) nb += spare[s].bytes.size();
      batch.bytes.reserve(nb + 16);
      batch.offs.reserve(n + 1);
      for (uint32_t s : taken) {
        PackedTopics& q = spare[s];
        const uint64_t b0 = batch.bytes.size();
        batch.bytes.append(q.bytes);
        for (uint32_t i = 1; i < q.offs.size(); i++) batch.offs.push_back(b0 + q.offs[i]);
        q.clear();
      }
      batch.finish();
      std::shared_ptr<const Batch> res;
      std::exception_ptr err;
      const auto c2 = Clock::now();
      bool retried = false;
      uint64_t again = 0;
      for (size_t attempt = 0; attempt <= kRetryDelays.size() && !res; attempt++) {
        if (attempt) {
          again++;
          if (kRetryDelays[attempt - 1].count()) std::this_thread::sleep_for(kRetryDelays[attempt - 1]);
        }
        try {
          err = nullptr;
          res = match_(batch);
        } catch (...) {
          err = std::current_exception();
          if (attempt == 0) retried = true;
        }
      }
      last_n_ = n;
      const auto c3 = Clock::now();
      for (auto& sg : segs) {
        {
          std::lock_guard<std::mutex> lk(sg.first->mu);
          sg.first->done_at = c3;
          sg.first->results = res;
          sg.first->err = err;
          sg.first->base = sg.second;
          sg.first->done = true;
        }
        sg.first->cv.notify_all();
      }
      segs.clear();  // (the last ticket of a segment frees it, and with it the batch)
      res.reset();
      const auto c4 = Clock::now();
      std::lock_guard<std::mutex> lk(mu_);
      st_.batches++;
      st_.retried += retried;
      st_.attempts += again;
      st_.failed += err != nullptr;
      st_.topics += n;
      st_.largest = std::max<uint64_t>(st_.largest, n);
      st_.wait_ns += ns(c0, c1);
      st_.seal_ns += ns(c1, c2);
      st_.match_ns += ns(c2, c3);
      st_.complete_ns += ns(c3, c4);
    }
  }

  // the waits before a failed batch's further attempts (about a third of a second in all)
  static constexpr std::array<std::chrono::milliseconds, 6> kRetryDelays = {
      std::chrono::milliseconds(0), std::chrono::milliseconds(1),  std::chrono::milliseconds(4),
      std::chrono::milliseconds(16), std::chrono::milliseconds(64), std::chrono::milliseconds(256)};
  MatchFn match_;
  const size_t max_batch_;
  const std::chrono::microseconds max_delay_;
  const size_t min_fill_;
  Shard shards_[kShards];
  std::atomic<uint64_t> queued_{0};
  uint32_t rr_ = 0;
  uint64_t last_n_ = 0;  // the previous batch's topics (dispatcher thread)
  mutable std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
  Stats st_;
  std::thread th_;
};

// Tickets of Subscribers (the Go-shaped maps, TopicsIndex::SubscribersBatch)
struct MapsPolicy {
  using Batch = std::vector<Subscribers>;
  using Item = const Subscribers&;
  static Item item(const std::shared_ptr<const Batch>& b, uint32_t i) { return (*b)[i]; }
};
// Tickets of TopicView: each view is made by the thread that takes it (one reference count per
// get()), so the dispatcher does no per-topic work after the match
struct ViewsPolicy {
  using Batch = SpanBatch;
  using Item = TopicView;
  static Item item(const std::shared_ptr<const Batch>& b, uint32_t i) { return TopicView(b, i); }
};

class PublishBatcher : public BasicBatcher<MapsPolicy> {
 public:
  explicit PublishBatcher(TopicsIndex& ix, size_t max_batch = 16384,
                          std::chrono::microseconds max_delay = std::chrono::microseconds(200),
                          size_t min_fill = 1024)
      : BasicBatcher(
            [&ix](const PackedTopics& t) {
              return std::make_shared<const std::vector<Subscribers>>(ix.SubscribersBatch(t));
            },
            max_batch, max_delay, min_fill) {}
};

class PublishViewBatcher : public BasicBatcher<ViewsPolicy> {
 public:
  explicit PublishViewBatcher(TopicsIndex& ix, size_t max_batch = 16384,
                              std::chrono::microseconds max_delay = std::chrono::microseconds(200),
                              size_t min_fill = 1024)
      : BasicBatcher([&ix](const PackedTopics& t) { return ix.SubscribersSpans(t); }, max_batch, max_delay,
                     min_fill) {}
};

}  // namespace host
}  // namespace mq
