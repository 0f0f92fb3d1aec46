// The reference's TopicsIndex tests (/root/reference/topics_test.go) restated against the C++
// host mirror (mqtt-server_amd/csrc/host/topics_index.h) over the GPU engine. White-box checks
// of index.root.particles are restated through the public API. Run by
// tests/test_gpu_parity.py::test_cpp_host_mirror (needs a GPU).
#include <algorithm>
#include <map>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "publish_batcher.h"
#include "topics_index.h"

#include <atomic>
#include <mutex>
#include <chrono>
#include <future>
#include <random>
#include <thread>

using mq::host::InlineSubscription;
using mq::host::Subscription;
using mq::host::TopicsIndex;

static int g_fail = 0;
#define REQUIRE(c)                                                        \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "%s:%d: REQUIRE(%s) failed\n", __FILE__, __LINE__, #c); \
      g_fail++;                                                           \
    }                                                                     \
  } while (0)

static Subscription S(const std::string& f, uint8_t qos = 0, int id = 0, bool nolocal = false) {
  Subscription s;
  s.Filter = f;
  s.Qos = qos;
  s.Identifier = id;
  s.NoLocal = nolocal;
  return s;
}

static int ident(const Subscription& s, const std::string& f) {  // Go map zero value
  auto it = s.Identifiers.find(f);
  return it == s.Identifiers.end() ? 0 : it->second;
}

static void TestSubscribe() {  // topics_test.go:170-226
  TopicsIndex x;
  REQUIRE(x.Subscribe("cl1", S("a/b/c", 2)));
  REQUIRE(!x.Subscribe("cl1", S("a/b/c", 1)));
  REQUIRE(x.Subscribe("cl1", S("A/B/c", 1)));
  REQUIRE(x.Subscribe("cl1", S("d/+")));
  REQUIRE(x.Subscribe("cl1", S("d/e/#")));
  REQUIRE(x.Subscribers_("a/b/c").Subscriptions.at("cl1").Qos == 1);
}

static void TestUnsubscribe() {  // topics_test.go:254-297
  TopicsIndex x;
  x.Subscribe("cl1", S("a/b/c/d", 1));
  x.Subscribe("cl1", S("a/b/+/d", 1));
  x.Subscribe("cl1", S("d/e/f", 1));
  x.Subscribe("cl2", S("d/e/f", 1));
  x.Subscribe("cl3", S("#", 2));
  REQUIRE(x.Unsubscribe("a/b/c/d", "cl1"));
  auto s = x.Subscribers_("a/b/c/d");
  REQUIRE(s.Subscriptions.size() == 2 && s.Subscriptions.at("cl1").Filter == "a/b/+/d");
  REQUIRE(x.Unsubscribe("d/e/f", "cl1"));
  s = x.Subscribers_("d/e/f");
  REQUIRE(s.Subscriptions.count("cl2") && s.Subscriptions.count("cl3") && !s.Subscriptions.count("cl1"));
  REQUIRE(!x.Unsubscribe("fdasfdas/dfsfads/sa", "nobody"));
}

static void TestRetainMessage() {  // topics_test.go:408-443
  TopicsIndex x;
  REQUIRE(x.RetainMessage("a/b/c", 1, 5, true) == 1);
  REQUIRE(x.RetainedLen() == 1);
  REQUIRE(x.RetainMessage("a/b/d/f", 2, 5, true) == 1);
  REQUIRE(x.RetainMessage("a/b/d/f", 3, 5, true) == 1);
  REQUIRE(x.RetainMessage("a/b/c", 4, 0, false) == -1);
  REQUIRE(x.RetainMessage("a/b/c", 5, 0, false) == 0);
}

static void TestScanSubscribers() {  // topics_test.go:490-528
  TopicsIndex x;
  x.Subscribe("cl1", S("a/b/c", 1, 22));
  x.Subscribe("cl1", S("a/b/c/d/e/f", 1));
  x.Subscribe("cl1", S("a/b/c/d/+/f", 2));
  x.Subscribe("cl2", S("a/#", 0));
  x.Subscribe("cl2", S("a/b/c", 1));
  x.Subscribe("cl2", S("a/b/+", 2, 77));
  x.Subscribe("cl2", S("d/e/f", 2, 7237));
  x.Subscribe("cl2", S("$SYS/uptime", 2, 3));
  x.Subscribe("cl3", S("+/b", 1, 234));
  x.Subscribe("cl4", S("#", 0, 5));
  x.Subscribe("cl2", S("$SYS/test", 0, 2));
  auto s = x.Subscribers_("a/b/c").Subscriptions;
  REQUIRE(s.size() == 3 && s.count("cl1") && s.count("cl2") && s.count("cl4"));
  REQUIRE(s.at("cl1").Qos == 1 && s.at("cl2").Qos == 2 && s.at("cl4").Qos == 0);
  REQUIRE(ident(s.at("cl1"), "a/b/c") == 22);
  REQUIRE(ident(s.at("cl2"), "a/#") == 0);
  REQUIRE(ident(s.at("cl2"), "a/b/+") == 77);
  REQUIRE(ident(s.at("cl2"), "a/b/c") == 0);
  REQUIRE(ident(s.at("cl4"), "#") == 5);
  s = x.Subscribers_("d/e/f/g").Subscriptions;
  REQUIRE(s.size() == 1 && s.count("cl4"));
  REQUIRE(x.Subscribers_("").Subscriptions.empty());
}

static void TestScanSubscribersShared() {  // topics_test.go:539-566
  TopicsIndex x;
  x.Subscribe("cl1", S("$SHARE/tmp/a/b/c", 1, 111));
  x.Subscribe("cl2", S("$SHARE/tmp/a/b/c", 0, 112));
  x.Subscribe("cl3", S("$SHARE/tmp2/a/b/c", 0, 113));
  x.Subscribe("cl2", S("$SHARE/tmp/a/b/+", 0, 10));
  x.Subscribe("cl3", S("$SHARE/tmp/a/b/+", 1, 200));
  x.Subscribe("cl4", S("$SHARE/tmp/a/b/+", 0, 201));
  x.Subscribe("cl5", S("$SHARE/tmp/a/b/c/#", 0));
  auto s = x.Subscribers_("a/b/c");
  REQUIRE(s.Shared.size() == 4);
  s.SelectShared();
  REQUIRE(s.SharedSelected.size() == 4 || s.SharedSelected.size() == 3);  // one pick per group/filter
}

// The same subscriptions with SelectShared on the device: one member (the smallest client id)
// per shared filter; the broker flow then picks it (topics.go:320-347).
static void TestScanSubscribersSharedSelected() {
  TopicsIndex x(0, true);
  x.Subscribe("cl1", S("$SHARE/tmp/a/b/c", 1, 111));
  x.Subscribe("cl2", S("$SHARE/tmp/a/b/c", 0, 112));
  x.Subscribe("cl3", S("$SHARE/tmp2/a/b/c", 0, 113));
  x.Subscribe("cl2", S("$SHARE/tmp/a/b/+", 0, 10));
  x.Subscribe("cl3", S("$SHARE/tmp/a/b/+", 1, 200));
  x.Subscribe("cl4", S("$SHARE/tmp/a/b/+", 0, 201));
  x.Subscribe("cl5", S("$SHARE/tmp/a/b/c/#", 0));
  auto s = x.Subscribers_("a/b/c");
  REQUIRE(s.Shared.size() == 4);
  for (const auto& f : s.Shared) REQUIRE(f.second.size() == 1);
  REQUIRE(s.Shared.at("$SHARE/tmp/a/b/c").count("cl1"));  // client ids interned in order
  REQUIRE(s.Shared.at("$SHARE/tmp/a/b/+").count("cl2"));
  s.SelectShared();
  s.MergeSharedSelected();
  REQUIRE(s.SharedSelected.size() == 4 && s.Subscriptions.size() == 4);
}

static void TestSubscribersFind() {  // topics_test.go:590-625
  struct Row {
    const char *f, *t;
    bool m;
  } rows[] = {
      {"a", "a", true}, {"a/", "a", false}, {"a/", "a/", true}, {"/a", "/a", true},
      {"path/to/my/mqtt", "path/to/my/mqtt", true}, {"path/to/+/mqtt", "path/to/my/mqtt", true},
      {"+/to/+/mqtt", "path/to/my/mqtt", true}, {"#", "path/to/my/mqtt", true},
      {"+/+/+/+", "path/to/my/mqtt", true}, {"+/+/+/#", "path/to/my/mqtt", true},
      {"zen/#", "zen", true}, {"trailing-end/#", "trailing-end/", true},
      {"+/prefixed", "/prefixed", true}, {"+/+/#", "path/to/my/mqtt", true},
      {"path/to/", "path/to/my/mqtt", false}, {"#/stuff", "path/to/my/mqtt", false},
      {"#", "$SYS/info", false}, {"$SYS/#", "$SYS/info", true}, {"+/info", "$SYS/info", false},
  };
  for (const Row& r : rows) {
    TopicsIndex x;
    x.Subscribe("cl1", S(r.f));
    const bool got = x.Subscribers_(r.t).Subscriptions.size() == 1;
    if (got != r.m) std::fprintf(stderr, "find: filter %s topic %s\n", r.f, r.t);
    REQUIRE(got == r.m);
  }
}

static void TestMessagesPattern() {  // topics_test.go:640-685
  TopicsIndex x;
  const char* topics[] = {"$SYS/uptime", "$SYS/info", "a/b/c/d", "a/b/c/e", "a/b/d/f",
                          "q/w/e/r/t/y", "q/x/e/r/t/o", "asdf"};
  uint64_t h = 1;
  for (const char* t : topics) x.RetainMessage(t, h++, 5, true);
  struct Row {
    const char* f;
    size_t n;
  } rows[] = {{"a/b/c/d", 1}, {"$SYS/+", 2}, {"$SYS/#", 2}, {"#", 6}, {"a/b/c/+", 2},
              {"a/+/c/+", 2}, {"+/+/+/d", 1}, {"q/w/e/#", 1}, {"+/+/+/+", 3}, {"q/#", 2},
              {"asdf", 1}, {"", 0}, {"#", 6}};
  for (const Row& r : rows) {
    const size_t got = x.Messages(r.f).size();
    if (got != r.n) std::fprintf(stderr, "messages %s: %zu != %zu\n", r.f, got, r.n);
    REQUIRE(got == r.n);
  }
}

static void TestInline() {  // topics_test.go:946-1067
  TopicsIndex x;
  InlineSubscription a;
  a.Sub = S("a/b/c", 0, 1);
  REQUIRE(x.InlineSubscribe(a));
  REQUIRE(!x.InlineSubscribe(a));
  a.Sub.Identifier = 2;
  REQUIRE(x.InlineSubscribe(a));
  InlineSubscription b;
  b.Sub = S("#", 0, 1);
  x.InlineSubscribe(b);
  auto s = x.Subscribers_("a/b/c");
  REQUIRE(s.InlineSubscriptions.size() == 2 && s.InlineSubscriptions.at(1).Sub.Filter == "#");
  REQUIRE(x.InlineUnsubscribe(1, "a/b/c"));
  REQUIRE(!x.InlineUnsubscribe(1, "not/exist"));
}

static void TestPublishToSubscribersIdentifiers() {  // server_test.go:1973-1999
  TopicsIndex x;
  REQUIRE(x.Subscribe("cl", S("a/b/+", 0, 2)));
  REQUIRE(x.Subscribe("cl", S("a/#", 0, 3)));
  REQUIRE(x.Subscribe("cl", S("d/e/f", 0, 4)));
  auto sub = x.Subscribers_("a/b/c").Subscriptions.at("cl");
  std::vector<int> ids;
  for (auto& kv : sub.Identifiers)
    if (kv.second > 0) ids.push_back(kv.second);
  std::sort(ids.begin(), ids.end());
  REQUIRE((ids == std::vector<int>{2, 3}));  // packets/tpackets.go:1848-1872: 11,2, 11,3
}

static void TestMergeSharedSelected() {  // topics_test.go:568-588
  mq::host::Subscribers s;
  s.SharedSelected["cl1"] = S("$SHARE/tmp/a/b/c", 1, 110);
  s.SharedSelected["cl2"] = S("$SHARE/tmp2/a/b/c", 1, 111);
  s.Subscriptions["cl2"] = S("a/b/c", 1, 112);
  s.MergeSharedSelected();
  REQUIRE(s.Subscriptions.size() == 2);
  REQUIRE((s.Subscriptions.at("cl2").Identifiers == std::map<std::string, int>{{"$SHARE/tmp2/a/b/c", 111}, {"a/b/c", 112}}));
}

static bool same_sub(const Subscription& a, const Subscription& b) {
  return a.Filter == b.Filter && a.Identifier == b.Identifier && a.HasIdentifiers == b.HasIdentifiers &&
         a.Identifiers == b.Identifiers && a.RetainHandling == b.RetainHandling && a.Qos == b.Qos &&
         a.RetainAsPublished == b.RetainAsPublished && a.NoLocal == b.NoLocal;
}

template <class M>
static bool same_map(const M& a, const M& b) {
  if (a.size() != b.size()) return false;
  for (auto ia = a.begin(), ib = b.begin(); ia != a.end(); ++ia, ++ib)
    if (ia->first != ib->first || !same_sub(ia->second, ib->second)) return false;
  return true;
}

static bool same(const mq::host::Subscribers& a, const mq::host::Subscribers& b) {
  if (!same_map(a.Subscriptions, b.Subscriptions) || a.Shared.size() != b.Shared.size() ||
      a.InlineSubscriptions.size() != b.InlineSubscriptions.size())
    return false;
  for (auto ia = a.Shared.begin(), ib = b.Shared.begin(); ia != a.Shared.end(); ++ia, ++ib)
    if (ia->first != ib->first || !same_map(ia->second, ib->second)) return false;
  for (auto ia = a.InlineSubscriptions.begin(), ib = b.InlineSubscriptions.begin(); ia != a.InlineSubscriptions.end();
       ++ia, ++ib)
    if (ia->first != ib->first || !same_sub(ia->second.Sub, ib->second.Sub)) return false;
  return true;
}

// The publish batching stage: 8 producer threads submit topics concurrently; every future holds
// exactly what Subscribers(topic) returns, and the stage really batched them.
static void TestPublishBatcher() {
  TopicsIndex ix;
  std::mt19937 r(7);
  const char* segs[] = {"a", "b", "c", "d", "+", "#"};
  std::vector<std::string> filters;
  for (int i = 0; i < 400; i++) {
    std::string f;
    const int n = 1 + (int)(r() % 4);
    for (int k = 0; k < n; k++) {
      std::string sg = segs[r() % (k + 1 == n ? 6 : 5)];
      f += (k ? "/" : "") + sg;
    }
    if (i % 10 == 0) f = "$share/g" + std::to_string(i % 3) + "/" + f;
    ix.Subscribe("c" + std::to_string(r() % 50), S(f, (uint8_t)(r() % 3), (int)(r() % 4)));
  }
  InlineSubscription in;
  in.Sub.Filter = "a/#";
  in.Sub.Identifier = 9;
  ix.InlineSubscribe(in);
  std::vector<std::string> topics;
  for (int i = 0; i < 64; i++) {
    std::string t;
    const int n = 1 + (int)(r() % 4);
    for (int k = 0; k < n; k++) t += (k ? "/" : "") + std::string(segs[r() % 4]);
    topics.push_back(t);
  }
  std::vector<std::vector<mq::host::PublishBatcher::Ticket>> futs(8);
  {
    mq::host::PublishBatcher b(ix, 4096, std::chrono::microseconds(2000));
    std::vector<std::thread> th;
    for (int w = 0; w < 8; w++)
      th.emplace_back([&, w] {
        for (int i = 0; i < 500; i++) futs[w].push_back(b.Submit(topics[(w * 7 + i) % topics.size()]));
      });
    for (auto& t : th) t.join();
    for (auto& fv : futs)
      for (auto& f : fv) f.wait();
    const auto st = b.stats();
    REQUIRE(st.topics == 4000);
    REQUIRE(st.batches < st.topics);  // publishes were matched in batches
    std::printf("publish batcher: %llu topics in %llu batches (largest %llu)\n",
                (unsigned long long)st.topics, (unsigned long long)st.batches, (unsigned long long)st.largest);
  }
  for (int w = 0; w < 8; w++)
    for (int i = 0; i < 500; i++) {
      const std::string& t = topics[(w * 7 + i) % topics.size()];
      REQUIRE(same(futs[w][i].get(), ix.Subscribers_(t)));
    }
}

// Client churn: ids of clients and filters with no subscription left are released
// and reused; Unsubscribe of an unknown client interns nothing but still answers whether the
// particle exists (topics.go:434-437).
static void TestChurnRecyclesIds() {
  TopicsIndex ix;
  ix.Subscribe("keep", S("k/+"));
  const size_t c0 = ix.live_clients(), f0 = ix.live_filters();
  for (int round = 0; round < 50; round++) {
    for (int i = 0; i < 20; i++) {
      const std::string c = "cl" + std::to_string(round * 100 + i);
      REQUIRE(ix.Subscribe(c, S("a/" + std::to_string(i % 5) + "/#", 1)));
    }
    REQUIRE(ix.Unsubscribe("a/0/#", "never-seen"));  // the particle exists: true
    REQUIRE(!ix.Unsubscribe("zz/top", "never-seen"));          // no particle: false
    for (int i = 0; i < 20; i++) {
      const std::string c = "cl" + std::to_string(round * 100 + i);
      REQUIRE(ix.Unsubscribe("a/" + std::to_string(i % 5) + "/#", c));
    }
  }
  REQUIRE(ix.live_clients() == c0);
  REQUIRE(ix.live_filters() == f0);
  REQUIRE(ix.Subscribers_("k/x").Subscriptions.count("keep") == 1);
  REQUIRE(ix.Subscribers_("a/1/x").Subscriptions.empty());
}

// Readers and updates at once: matches run while other threads subscribe, unsubscribe and
// churn client ids; every result names only strings the index has held, and the final state
// matches exactly. Liveness: three readers match back to back (their span results overlap all
// the time), yet every update must finish within kUpdateDeadline: updates copy what a live result
// may see instead of waiting for it (capi.cpp IndexLock), so an update waits at most for the one
// match whose GPU round trip holds the handle lock. A watchdog prints every thread's progress and
// fails the run if the test has not finished after kWatchdog.
static void TestConcurrentReadersAndUpdates() {
  using clk = std::chrono::steady_clock;
  constexpr auto kUpdateDeadline = std::chrono::milliseconds(10);
  constexpr auto kWatchdog = std::chrono::seconds(20);
  TopicsIndex ix;
  for (int i = 0; i < 200; i++) ix.Subscribe("base" + std::to_string(i % 40), S("s/" + std::to_string(i % 10) + "/+", 1));
  // device set-up outside the timing: the first batches allocate the device buffers and both
  // host-result stages (one-time costs, not update latency)
  for (int k = 0; k < 6; k++) ix.SubscribersBatch(std::vector<std::string>{"s/" + std::to_string(k) + "/x", "t/0"});
  std::atomic<bool> stop{false}, done{false};
  std::atomic<int> bad{0}, late{0};
  std::atomic<long> progress[5];
  std::atomic<long> worst_us{0};
  std::atomic<long> worst_warm_us{0};  // updates that started once every reader had matched a batch
  std::atomic<int> readers_warm{0};
  std::mutex slow_mu;
  std::vector<std::pair<long, long>> slow;  // (us, ms since the start) of updates over 2 ms
  std::vector<std::pair<long, long>> slow_reads;  //   and of matches
  const auto t_start = clk::now();
  for (auto& p : progress) p = 0;
  std::thread watchdog([&] {
    const auto t0 = clk::now();
    while (!done) {
      if (clk::now() - t0 > kWatchdog) {
        std::fprintf(stderr, "TestConcurrentReadersAndUpdates: stalled after %lld s; progress: readers %ld %ld %ld, "
                             "updaters %ld %ld of 400\n",
                     (long long)std::chrono::duration_cast<std::chrono::seconds>(kWatchdog).count(),
                     progress[0].load(), progress[1].load(), progress[2].load(), progress[3].load(),
                     progress[4].load());
        std::fflush(stderr);
        std::_Exit(3);
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
  });
  std::vector<std::thread> th;
  // the readers start cold, on fresh threads, as the updates start: a thread's first HIP calls set
  // up its per-thread runtime state (~10 ms), which the engine does before taking the handle lock
  // (capi.cpp thread_warm), so an update never waits for it
  for (int w = 0; w < 3; w++)
    th.emplace_back([&, w] {
      for (int k = 0; !stop; k++) {
        const auto r0 = clk::now();
        auto res = ix.SubscribersBatch(std::vector<std::string>{"s/" + std::to_string(k % 10) + "/x", "t/" + std::to_string(k % 7)});
        const long rus = (long)std::chrono::duration_cast<std::chrono::microseconds>(clk::now() - r0).count();
        if (rus > 2000) {
          std::lock_guard<std::mutex> g(slow_mu);
          slow_reads.emplace_back(rus, (long)std::chrono::duration_cast<std::chrono::milliseconds>(r0 - t_start).count());
        }
        for (auto& kv : res[0].Subscriptions)
          if (kv.first.rfind("base", 0) != 0 && kv.first.rfind("tmp", 0) != 0) bad++;
        for (auto& kv : res[1].Subscriptions)
          if (kv.first.rfind("tmp", 0) != 0) bad++;
        if (progress[w]++ == 0) readers_warm++;
      }
    });
  for (int u = 0; u < 2; u++)
    th.emplace_back([&, u] {
      auto timed = [&](auto&& f) {
        const bool warm = readers_warm.load() == 3;
        const auto t0 = clk::now();
        f();
        const auto dt = clk::now() - t0;
        const long us = (long)std::chrono::duration_cast<std::chrono::microseconds>(dt).count();
        for (long w = worst_us.load(); us > w && !worst_us.compare_exchange_weak(w, us);) {
        }
        if (warm)
          for (long w = worst_warm_us.load(); us > w && !worst_warm_us.compare_exchange_weak(w, us);) {
          }
        if (us > 2000) {
          std::lock_guard<std::mutex> g(slow_mu);
          slow.emplace_back(us, (long)std::chrono::duration_cast<std::chrono::milliseconds>(t0 - t_start).count());
        }
        if (dt > kUpdateDeadline) late++;
      };
      auto matched = [&] { return progress[0].load() + progress[1].load() + progress[2].load(); };
      for (int i = 0; i < 400; i++) {
        const long m0 = matched();
        const std::string c = "tmp" + std::to_string(u) + "_" + std::to_string(i);
        timed([&] { ix.Subscribe(c, S("t/" + std::to_string(i % 7))); });
        timed([&] { ix.Subscribe(c, S("s/" + std::to_string(i % 10) + "/+")); });
        timed([&] { ix.Unsubscribe("t/" + std::to_string(i % 7), c); });
        timed([&] { ix.Unsubscribe("s/" + std::to_string(i % 10) + "/+", c); });
        progress[3 + u]++;
        // the updates are fast (they wait for no match): pace them with the readers, so that
        // matches run all through the update phase (at least one per round, 20 ms at most)
        const auto t0 = clk::now();
        while (matched() == m0 && clk::now() - t0 < std::chrono::milliseconds(20)) std::this_thread::yield();
      }
    });
  // a third updater on the engine handle itself (mq_subscribe / mq_unsubscribe, no mirror tables):
  // separates the engine's lock from the mirror's
  std::atomic<long> raw_worst_us{0};
  std::thread raw([&] {
    for (int i = 0; i < 400; i++) {
      const std::string f = "raw/" + std::to_string(i % 5);
      const auto t0 = clk::now();
      mq_subscribe(ix.handle(), f.data(), (uint32_t)f.size(), 900000u + (uint32_t)(i % 50), 900000u + (uint32_t)(i % 5), 0, 0, 0);
      mq_unsubscribe(ix.handle(), f.data(), (uint32_t)f.size(), 900000u + (uint32_t)(i % 50));
      const long us = (long)std::chrono::duration_cast<std::chrono::microseconds>(clk::now() - t0).count() / 2;
      if (us > raw_worst_us) raw_worst_us = us;
    }
  });
  raw.join();
  th[3].join();
  th[4].join();
  stop = true;
  for (int w = 0; w < 3; w++) th[w].join();
  done = true;
  watchdog.join();
  std::fprintf(stderr, "  readers matched %ld batches during 3200 updates; slowest update %.1f ms\n",
               progress[0].load() + progress[1].load() + progress[2].load(), worst_us.load() / 1000.0);
  std::sort(slow.begin(), slow.end(), std::greater<std::pair<long, long>>());
  std::fprintf(stderr, "  slowest update once every reader had matched a batch (its threads' first HIP calls done): %.2f ms\n",
               worst_warm_us.load() / 1000.0);
  std::fprintf(stderr, "  engine-handle updates (no mirror): slowest %.1f ms\n", raw_worst_us.load() / 1000.0);
  std::fprintf(stderr, "  updates' longest waits: update lock %.1f ms (longest hold %.1f ms), tables %.1f ms, engine call %.1f ms\n",
               ix.update_waits().upd.load() / 1e3, ix.update_waits().held.load() / 1e3,
               ix.update_waits().tables.load() / 1e3, ix.update_waits().engine.load() / 1e3);
  std::fprintf(stderr, "  updates over 2 ms: %zu;", slow.size());
  for (size_t i = 0; i < slow.size() && i < 8; i++) std::fprintf(stderr, " %.1f ms at +%ld ms;", slow[i].first / 1e3, slow[i].second);
  std::fprintf(stderr, "\n");
  std::sort(slow_reads.begin(), slow_reads.end(), std::greater<std::pair<long, long>>());
  std::fprintf(stderr, "  matches over 2 ms: %zu;", slow_reads.size());
  for (size_t i = 0; i < slow_reads.size() && i < 8; i++)
    std::fprintf(stderr, " %.1f ms at +%ld ms;", slow_reads[i].first / 1e3, slow_reads[i].second);
  std::fprintf(stderr, "\n");
  REQUIRE(late == 0);
  REQUIRE(bad == 0);
  for (int k = 0; k < 10; k++) REQUIRE(ix.Subscribers_("s/" + std::to_string(k) + "/x").Subscriptions.size() == 4);
  REQUIRE(ix.Subscribers_("t/1").Subscriptions.empty());
}

// The restore path: LoadSubscriptions answers as Subscribe would, in order (duplicates: the
// last entry wins), and the Go-shaped results carry the stored subscriptions.
static void TestLoadSubscriptions() {
  TopicsIndex a, b;
  std::vector<std::pair<std::string, Subscription>> subs;
  std::mt19937 r(3);
  for (int i = 0; i < 6000; i++)
    subs.emplace_back("c" + std::to_string(r() % 300),
                      S((i % 9 == 0 ? "$share/g/" : "") + std::string("l/") + std::to_string(r() % 40) + (i % 3 ? "/+" : "/#"),
                        (uint8_t)(r() % 3), (int)(r() % 5)));
  const std::vector<bool> got = a.LoadSubscriptions(subs);
  for (size_t i = 0; i < subs.size(); i++) REQUIRE(got[i] == b.Subscribe(subs[i].first, subs[i].second));
  for (int k = 0; k < 40; k++) {
    const std::string t = "l/" + std::to_string(k) + "/x";
    REQUIRE(same(a.Subscribers_(t), b.Subscribers_(t)));
  }
}

// Retained.Add outside RetainMessage after an expiry sweep (Q12 re-add): found again.
static void TestRetainedAddAfterExpiry() {
  TopicsIndex ix;
  ix.RetainMessage("a/b", 7, 3, true);
  ix.RetainMessage("a/c", 8, 3, true);
  ix.RetainedDelete("a/b");
  REQUIRE(ix.Messages("a/+") == std::vector<uint64_t>{8});
  ix.RetainedAdd("a/b", 9, 3, true);
  std::vector<uint64_t> m = ix.Messages("a/+");
  std::sort(m.begin(), m.end());
  REQUIRE((m == std::vector<uint64_t>{8, 9}));
  REQUIRE(ix.RetainMessage("a/b", 10, 0, true) == -1);  // the re-added packet had Retain and a payload
}

// The view batcher: each future's TopicView names exactly the recipients of Subscribers(topic)
// (client rows with their merged Qos, shared members, inline identifiers).
static void TestPublishViewBatcher() {
  TopicsIndex ix;
  std::mt19937 r(11);
  for (int i = 0; i < 300; i++) {
    const std::string f = std::string(i % 7 == 0 ? "$share/g/" : "") + "v/" + std::to_string(r() % 20) + (i % 2 ? "/+" : "/#");
    ix.Subscribe("c" + std::to_string(r() % 40), S(f, (uint8_t)(r() % 3), (int)(r() % 3)));
  }
  std::vector<mq::host::PublishViewBatcher::Ticket> futs;
  {
    mq::host::PublishViewBatcher b(ix, 256, std::chrono::microseconds(1000));
    for (int i = 0; i < 400; i++) futs.push_back(b.Submit("v/" + std::to_string(i % 20) + "/x"));
    for (auto& f : futs) f.wait();
  }
  for (int i = 0; i < 400; i++) {
    const mq::host::TopicView& v = futs[i].get();
    const mq::host::Subscribers want = ix.Subscribers_("v/" + std::to_string(i % 20) + "/x");
    std::map<std::string, int> qos;
    v.for_each_row([&](const mq_client_row& cr) {
      if ((cr.meta & MQ_ROW_KIND_MASK) == 0) qos[v.client(cr.client_id)] = cr.meta & MQ_META_QOS_MASK;
    });
    REQUIRE(qos.size() == want.Subscriptions.size());
    for (auto& kv : want.Subscriptions) REQUIRE(qos.count(kv.first) && qos[kv.first] == kv.second.Qos);
    size_t shared = 0;
    v.for_each_shared([&](const mq_shared_row&) { shared++; });
    size_t want_shared = 0;
    for (auto& g : want.Shared) want_shared += g.second.size();
    REQUIRE(shared == want_shared);
  }
}

// A view held across updates and later batches: a consumer keeps batch N's TopicView while
// another thread subscribes and a later batch is matched; the update does not wait for the view
// (capi.cpp IndexLock: the index copies what a live result may see), the held view still names
// exactly the recipients it was matched with, and the later batch sees the new subscription.
static void TestViewHeldAcrossUpdates() {
  using clk = std::chrono::steady_clock;
  TopicsIndex ix;
  for (int i = 0; i < 64; i++) ix.Subscribe("h" + std::to_string(i), S(i % 2 ? "w/+" : "w/x", 1));
  auto recipients = [](const mq::host::TopicView& v) {
    std::map<std::string, int> q;
    v.for_each_row([&](const mq_client_row& cr) {
      if ((cr.meta & MQ_ROW_KIND_MASK) == 0) q[v.client(cr.client_id)] = cr.meta & MQ_META_QOS_MASK;
    });
    return q;
  };
  mq::host::PublishViewBatcher b(ix, 256, std::chrono::microseconds(200));
  const mq::host::TopicView held = b.Submit("w/x").get();
  const auto before = recipients(held);
  REQUIRE(before.size() == 64);
  std::atomic<long> worst_us{0};
  std::thread upd([&] {
    for (int i = 0; i < 200; i++) {
      const auto t0 = clk::now();
      ix.Subscribe("n" + std::to_string(i), S("w/x", 2));
      if (i % 3 == 0) ix.Unsubscribe(i % 2 ? "w/+" : "w/x", "h" + std::to_string(i % 64));
      const long us = (long)std::chrono::duration_cast<std::chrono::microseconds>(clk::now() - t0).count();
      if (us > worst_us) worst_us = us;
    }
  });
  upd.join();
  const mq::host::TopicView later = b.Submit("w/x").get();  // batch N+1, while `held` lives
  REQUIRE(recipients(held) == before);
  const auto after = recipients(later);
  REQUIRE(after.count("n199") && after.at("n199") == 2);
  REQUIRE(after.size() == ix.Subscribers_("w/x").Subscriptions.size());
  std::fprintf(stderr, "  200 updates while a view was held: slowest %.2f ms\n", worst_us.load() / 1000.0);
  REQUIRE(worst_us.load() < 10000);
}

// The batching stage's failure path: a match call that fails (an injected MQ_EIO, as a kernel
// guard would raise) is retried once; when the retry fails as well, that batch's tickets throw
// the EngineError and the stage goes on with the next batch.
// The batching stage under many submitters, checked against the ORACLE (the CPU restatement of
// the Go TopicsIndex, oracle/liboracle.so, test infrastructure): 32 threads keep 64 topics each
// in flight through PublishBatcher; a sample of the tickets is compared with the oracle's
// Subscribers(topic), as canonical JSON (sorted keys: Go map order is irrelevant).
extern "C" {
void* orc_new();
void orc_free(void*);
int orc_subscribe(void* h, const char* client, uint32_t clen, const char* filter, uint32_t flen, uint32_t client_id,
                  uint32_t filter_id, uint8_t qos, uint8_t flags, int64_t identifier);
int orc_inline_subscribe(void* h, const char* filter, uint32_t flen, int64_t id, uint32_t filter_id);
uint64_t orc_subscribers_json(void* h, const char* topic, uint32_t tlen, char* buf, uint64_t cap);
}

static std::string jesc(const std::string& s) {
  std::string o;
  for (unsigned char ch : s) {
    if (ch == '"' || ch == '\\') {
      o += '\\';
      o += (char)ch;
    } else if (ch < 0x20) {
      char b[8];
      std::snprintf(b, sizeof b, "\\u%04x", ch);
      o += b;
    } else {
      o += (char)ch;
    }
  }
  return o;
}

static void sub_json(std::string& o, const Subscription& s, bool with_idents) {
  char b[160];
  o += "{\"filter\":\"" + jesc(s.Filter) + "\"";
  std::snprintf(b, sizeof b, ",\"identifier\":%lld,\"qos\":%u,\"no_local\":%s,\"rap\":%s,\"rh\":%u",
                (long long)s.Identifier, s.Qos, s.NoLocal ? "true" : "false", s.RetainAsPublished ? "true" : "false",
                s.RetainHandling);
  o += b;
  if (with_idents) {
    o += ",\"identifiers\":";
    if (!s.HasIdentifiers) {
      o += "null";
    } else {
      o += "{";
      bool first = true;
      for (auto& kv : s.Identifiers) {
        if (!first) o += ",";
        first = false;
        o += "\"" + jesc(kv.first) + "\":" + std::to_string(kv.second);
      }
      o += "}";
    }
  }
  o += "}";
}

static std::string subscribers_json(const mq::host::Subscribers& s) {
  std::string o = "{\"subscriptions\":{";
  bool first = true;
  for (auto& kv : s.Subscriptions) {
    if (!first) o += ",";
    first = false;
    o += "\"" + jesc(kv.first) + "\":";
    sub_json(o, kv.second, true);
  }
  o += "},\"shared\":{";
  first = true;
  for (auto& g : s.Shared) {
    if (!first) o += ",";
    first = false;
    o += "\"" + jesc(g.first) + "\":{";
    bool f2 = true;
    for (auto& kv : g.second) {
      if (!f2) o += ",";
      f2 = false;
      o += "\"" + jesc(kv.first) + "\":";
      sub_json(o, kv.second, true);
    }
    o += "}";
  }
  o += "},\"inline\":{";
  first = true;
  for (auto& kv : s.InlineSubscriptions) {
    if (!first) o += ",";
    first = false;
    o += "\"" + std::to_string(kv.first) + "\":";
    sub_json(o, kv.second.Sub, false);
  }
  o += "}}";
  return o;
}

static std::string oracle_json(void* orc, const std::string& t) {
  std::string buf(orc_subscribers_json(orc, t.data(), (uint32_t)t.size(), nullptr, 0), '\0');
  orc_subscribers_json(orc, t.data(), (uint32_t)t.size(), &buf[0], buf.size());
  return buf;
}

static void TestBatcherManySubmittersVsOracle() {
  TopicsIndex ix;
  void* orc = orc_new();
  std::mt19937 r(23);
  const char* segs[] = {"a", "b", "c", "d", "e", "+", "#"};
  std::map<std::string, uint32_t> fids, cids;
  for (int i = 0; i < 6000; i++) {
    std::string f;
    const int n = 1 + (int)(r() % 5);
    for (int k = 0; k < n; k++) f += (k ? "/" : "") + std::string(segs[r() % (k + 1 == n ? 7 : 6)]);
    if (i % 9 == 0) f = std::string(i % 2 ? "$share" : "$SHARE") + "/g" + std::to_string(i % 4) + "/" + f;
    const std::string c = "c" + std::to_string(r() % 400);
    Subscription s = S(f, (uint8_t)(r() % 3), (int)(r() % 5), r() % 11 == 0);
    s.RetainAsPublished = r() % 2;
    s.RetainHandling = (uint8_t)(r() % 3);
    ix.Subscribe(c, s);
    const uint32_t fid = fids.emplace(f, (uint32_t)fids.size()).first->second;
    const uint32_t cid = cids.emplace(c, (uint32_t)cids.size()).first->second;
    orc_subscribe(orc, c.data(), (uint32_t)c.size(), f.data(), (uint32_t)f.size(), cid, fid, s.Qos,
                  (uint8_t)((s.NoLocal ? 1 : 0) | (s.RetainAsPublished ? 2 : 0) | (s.RetainHandling << 2)),
                  s.Identifier);
  }
  for (int id = 1; id <= 3; id++) {  // inline subscriptions (last write wins, Q8)
    InlineSubscription in;
    in.Sub.Filter = id == 1 ? "a/#" : id == 2 ? "+/b" : "a/b";
    in.Sub.Identifier = id;
    ix.InlineSubscribe(in);
    const uint32_t fid = fids.emplace(in.Sub.Filter, (uint32_t)fids.size()).first->second;
    orc_inline_subscribe(orc, in.Sub.Filter.data(), (uint32_t)in.Sub.Filter.size(), id, fid);
  }
  std::vector<std::string> topics;
  for (int i = 0; i < 512; i++) {
    std::string t = i % 53 == 0 ? "$SYS" : std::string(segs[r() % 5]);
    const int n = (int)(r() % 5);
    for (int k = 0; k < n; k++) t += "/" + std::string(segs[r() % 5]);
    topics.push_back(t);
  }
  constexpr int kThreads = 32, kPer = 600, kWindow = 64;
  std::atomic<int> bad{0}, checked{0};
  mq::host::PublishBatcher::Stats st;
  {
    mq::host::PublishBatcher b(ix, 4096, std::chrono::microseconds(500), 512);
    std::vector<std::thread> th;
    std::mutex omu;  // the oracle is not thread-safe
    for (int w = 0; w < kThreads; w++)
      th.emplace_back([&, w] {
        std::vector<std::pair<int, mq::host::PublishBatcher::Ticket>> q;
        size_t head = 0;
        for (int i = 0; i < kPer || head < q.size();) {
          while (i < kPer && (int)(q.size() - head) < kWindow) {
            const int k = (w * 131 + i * 7) % (int)topics.size();
            q.emplace_back(k, b.Submit(topics[k]));
            i++;
          }
          const auto& [k, tk] = q[head];
          const mq::host::Subscribers& got = tk.get();
          if (head % 5 == 0) {
            const std::string mine = subscribers_json(got);
            std::string want;
            {
              std::lock_guard<std::mutex> lk(omu);
              want = oracle_json(orc, topics[k]);
            }
            if (mine != want) {
              if (bad++ < 3) std::fprintf(stderr, "batcher vs oracle, topic %s:\n  got  %s\n  want %s\n",
                                          topics[k].c_str(), mine.c_str(), want.c_str());
            }
            checked++;
          }
          q[head].second = mq::host::PublishBatcher::Ticket();
          head++;
        }
      });
    for (auto& t : th) t.join();
    st = b.stats();
  }
  std::printf("batcher, %d submitters: %llu topics in %llu batches (largest %llu); %d checked against the oracle\n",
              kThreads, (unsigned long long)st.topics, (unsigned long long)st.batches,
              (unsigned long long)st.largest, checked.load());
  REQUIRE(bad == 0);
  REQUIRE(checked > 1000);
  REQUIRE(st.topics == (uint64_t)kThreads * kPer);
  REQUIRE(st.largest > 64);  // submitters' topics were matched together
  orc_free(orc);
}

// A failing engine (MQ_EIO injected into the batch's match call, as a tripped kernel guard
// returns it): the batch is tried again with backoff, and its callers get the ORACLE's answer, not
// an empty one, while the failures last no longer than the retries; a batch that fails every
// attempt makes its tickets throw (nothing is delivered as an empty Subscribers), and the next
// batch is matched as usual (server.go:1000-1020).
static void TestBatcherEngineError() {
  TopicsIndex ix;
  void* orc = orc_new();
  for (int i = 0; i < 20; i++) {
    const std::string c = "e" + std::to_string(i), f = i % 3 ? "e/+" : "e/#";
    ix.Subscribe(c, S(f, (uint8_t)(i % 3)));
    orc_subscribe(orc, c.data(), (uint32_t)c.size(), f.data(), (uint32_t)f.size(), (uint32_t)i, i % 3 ? 1u : 2u,
                  (uint8_t)(i % 3), 0, 0);
  }
  ix.Subscribe("e0", S("e/a", 2, 7));
  orc_subscribe(orc, "e0", 2, "e/a", 3, 0, 3, 2, 0, 7);
  std::atomic<int> fail_next{0};
  mq::host::BasicBatcher<mq::host::MapsPolicy> b(
      [&](const mq::host::PackedTopics& t) {
        if (fail_next > 0) {
          fail_next--;
          throw mq::host::EngineError(MQ_EIO, "injected MQ_EIO");
        }
        return std::make_shared<const std::vector<mq::host::Subscribers>>(ix.SubscribersBatch(t));
      },
      64, std::chrono::microseconds(100));
  for (int k : {1, 3, 6}) {  // k failures in a row: the retries outlast them
    fail_next = k;
    for (const char* t : {"e/a", "e/b"}) {
      auto tk = b.Submit(t);
      REQUIRE(subscribers_json(tk.get()) == oracle_json(orc, t));
      REQUIRE(!tk.get().Subscriptions.empty());
    }
  }
  fail_next = 7;  // more than the retries: the ticket throws
  bool threw = false;
  try {
    b.Submit("e/c").get();
  } catch (const mq::host::EngineError& e) {
    threw = e.code == MQ_EIO;
  }
  REQUIRE(threw);
  REQUIRE(subscribers_json(b.Submit("e/d").get()) == oracle_json(orc, "e/d"));  // the next batch
  auto st = b.stats();  // (a batch's stats are recorded just after its tickets complete)
  for (int i = 0; i < 1000 && st.batches < 8; i++) {
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
    st = b.stats();
  }
  REQUIRE(st.batches == 8 && st.retried == 4 && st.failed == 1 && st.attempts == 1 + 3 + 6 + 6);
  orc_free(orc);
}


// progress on stderr: a test that does not return is named by the last line
#define RUN(f)                             \
  do {                                     \
    std::fprintf(stderr, "%s\n", #f);      \
    std::fflush(stderr);                   \
    f();                                   \
  } while (0)

int main() {
  try {
    RUN(TestSubscribe);
    RUN(TestUnsubscribe);
    RUN(TestRetainMessage);
    RUN(TestScanSubscribers);
    RUN(TestScanSubscribersShared);
    RUN(TestScanSubscribersSharedSelected);
    RUN(TestSubscribersFind);
    RUN(TestMessagesPattern);
    RUN(TestInline);
    RUN(TestPublishToSubscribersIdentifiers);
    RUN(TestMergeSharedSelected);
    RUN(TestPublishBatcher);
    RUN(TestChurnRecyclesIds);
    RUN(TestConcurrentReadersAndUpdates);
    RUN(TestLoadSubscriptions);
    RUN(TestRetainedAddAfterExpiry);
    RUN(TestPublishViewBatcher);
    RUN(TestViewHeldAcrossUpdates);
    RUN(TestBatcherEngineError);
    RUN(TestBatcherManySubmittersVsOracle);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "exception: %s\n", e.what());
    return 2;
  }
  if (g_fail) {
    std::fprintf(stderr, "%d checks failed\n", g_fail);
    return 1;
  }
  std::printf("cpp host mirror: all reference test cases passed\n");
  return 0;
}
