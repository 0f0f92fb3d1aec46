// Host-only (no GPU) update latency of the C++ mirror: the updaters of
// TestConcurrentReadersAndUpdates without the readers, so any slow update is host work.
//   g++ -O2 -std=c++17 -Iinclude -Imqtt-server_amd/csrc/host tools/upd_latency.cpp -Lmqtt-server_amd/lib -lmqhost -lmqmatch ...
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <string>
#include <thread>
#include <vector>

#include "topics_index.h"

using mq::host::Subscription;
using mq::host::TopicsIndex;
using clk = std::chrono::steady_clock;

static Subscription S(const std::string& f, uint8_t qos = 0) {
  Subscription s;
  s.Filter = f;
  s.Qos = qos;
  return s;
}

int main() {
  TopicsIndex ix;
  for (int i = 0; i < 200; i++) ix.Subscribe("base" + std::to_string(i % 40), S("s/" + std::to_string(i % 10) + "/+", 1));
  const auto t_start = clk::now();
  std::vector<std::pair<long, long>> slow[2];
  std::vector<std::thread> th;
  for (int u = 0; u < 2; u++)
    th.emplace_back([&, u] {
      auto timed = [&](auto&& f) {
        const auto t0 = clk::now();
        f();
        const long us = (long)std::chrono::duration_cast<std::chrono::microseconds>(clk::now() - t0).count();
        if (us > 1000) slow[u].emplace_back(us, (long)std::chrono::duration_cast<std::chrono::milliseconds>(t0 - t_start).count());
      };
      for (int i = 0; i < 400; i++) {
        const std::string c = "tmp" + std::to_string(u) + "_" + std::to_string(i);
        timed([&] { ix.Subscribe(c, S("t/" + std::to_string(i % 7))); });
        timed([&] { ix.Subscribe(c, S("s/" + std::to_string(i % 10) + "/+")); });
        timed([&] { ix.Unsubscribe("t/" + std::to_string(i % 7), c); });
        timed([&] { ix.Unsubscribe("s/" + std::to_string(i % 10) + "/+", c); });
      }
    });
  for (auto& t : th) t.join();
  const long total = (long)std::chrono::duration_cast<std::chrono::milliseconds>(clk::now() - t_start).count();
  std::vector<std::pair<long, long>> all(slow[0]);
  all.insert(all.end(), slow[1].begin(), slow[1].end());
  std::sort(all.begin(), all.end(), std::greater<std::pair<long, long>>());
  std::printf("3200 updates in %ld ms; over 1 ms: %zu;", total, all.size());
  for (size_t i = 0; i < all.size() && i < 10; i++) std::printf(" %.1f ms at +%ld;", all[i].first / 1e3, all[i].second);
  std::printf("\n");
  return 0;
}
