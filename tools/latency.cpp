// Batch latency sweep: on an index of N subscriptions (default
// 10M, config-3 mix, restored through TopicsIndex::LoadSubscriptions), for batch sizes 1, 64,
// 1k, 16k and 64k:
//   match   one mq_match_spans call (host span result) per batch: call latency p50 / p99
//   batcher PublishViewBatcher(max_batch = B >= 1024): 64 submitter threads (connection
//           goroutines) keep 2B topics in flight together; latency of each Submit until its
//           ticket is ready (p50 / p99), throughput, batches formed, and the recipients per
//           topic of the views read (one in 64: the fan-out reads them on the connection
//           goroutines, not on the submitting thread)
//   open    PublishViewBatcher(max_batch = 16k) under an open-loop offered load (publishes
//           arriving at a fixed rate, as at a broker, whatever the stage's latency): 64 submitters
//           each submit on their share of the schedule; latency from each Submit until its batch
//           completed (p50 / p99), achieved rate, batches formed
// Prints one JSON object per line. Built by mqtt-server_amd/Makefile (build/latency).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <atomic>
#include <future>
#include <string>
#include <thread>
#include <vector>

#include "publish_batcher.h"
#include "topics_index.h"

extern "C" {
void* mqgen_subs(uint64_t n, uint32_t clients, uint64_t seed, int mix);
uint64_t mqgen_subs_n(void*);
uint64_t mqgen_subs_nbytes(void*);
void mqgen_subs_copy(void*, uint8_t*, uint64_t*, uint32_t*, uint32_t*, uint8_t*, uint8_t*, int32_t*);
void mqgen_subs_free(void*);
void* mqgen_topics(void* subs, uint64_t n, uint64_t seed, int mix);
uint64_t mqgen_batch_n(void*);
uint64_t mqgen_batch_nbytes(void*);
void mqgen_batch_copy(void*, uint8_t*, uint64_t*, uint64_t*);
void mqgen_batch_free(void*);
}

using Clock = std::chrono::steady_clock;

static double pct(std::vector<double>& v, double p) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, (size_t)(p * (v.size() - 1) + 0.5))];
}

int main(int argc, char** argv) {
  const uint64_t n_subs = argc > 1 ? strtoull(argv[1], nullptr, 10) : 10000000ull;
  const double secs = argc > 2 ? atof(argv[2]) : 3.0;
  const int kSubmitters = argc > 3 ? atoi(argv[3]) : 64;  // connection goroutines
  const uint64_t seed = 0x6D716D61;
  void* g = mqgen_subs(n_subs, (uint32_t)std::max<uint64_t>(1, n_subs / 10), seed, 0);
  const uint64_t n = mqgen_subs_n(g);
  std::vector<uint8_t> bytes(mqgen_subs_nbytes(g) + 16), qos(n), flags(n);
  std::vector<uint64_t> offs(n + 1);
  std::vector<uint32_t> cid(n), fid(n);
  std::vector<int32_t> ident(n);
  mqgen_subs_copy(g, bytes.data(), offs.data(), cid.data(), fid.data(), qos.data(), flags.data(), ident.data());
  mq::host::TopicsIndex ix;
  {
    std::vector<std::pair<std::string, mq::host::Subscription>> subs(n);
    char cb[32];
    for (uint64_t i = 0; i < n; i++) {
      snprintf(cb, sizeof cb, "c%07u", cid[i]);
      mq::host::Subscription& s = subs[i].second;
      subs[i].first = cb;
      s.Filter.assign((const char*)bytes.data() + offs[i], offs[i + 1] - offs[i]);
      s.Qos = qos[i];
      s.Identifier = ident[i];
      s.NoLocal = flags[i] & 1;
      s.RetainAsPublished = flags[i] & 2;
      s.RetainHandling = (flags[i] >> 2) & 3;
    }
    const auto t0 = Clock::now();
    ix.LoadSubscriptions(subs);
    std::printf("{\"load_subscriptions_s\": %.3f, \"subs\": %llu}\n",
                std::chrono::duration<double>(Clock::now() - t0).count(), (unsigned long long)n);
    std::fflush(stdout);
  }
  const uint64_t n_topics = 1 << 20;
  void* tb = mqgen_topics(g, n_topics, seed + 1, 0);
  std::vector<uint8_t> tbytes(mqgen_batch_nbytes(tb) + 16);
  std::vector<uint64_t> toffs(mqgen_batch_n(tb) + 1);
  mqgen_batch_copy(tb, tbytes.data(), toffs.data(), nullptr);
  std::vector<std::string> topics(toffs.size() - 1);
  for (size_t i = 0; i < topics.size(); i++)
    topics[i].assign((const char*)tbytes.data() + toffs[i], toffs[i + 1] - toffs[i]);
  mqgen_batch_free(tb);
  mqgen_subs_free(g);
  (void)ix.Subscribers_(topics[0]);  // first sync

  // open loop: offered rates (topics/s) at max_batch 16k
  auto open_loop = [&](double rate, size_t B) {
    mq::host::PublishViewBatcher pb(ix, B, std::chrono::microseconds(200), std::min<size_t>(B, 1024));
    using Ticket = mq::host::PublishViewBatcher::Ticket;
    std::vector<std::vector<double>> wl(kSubmitters);
    std::vector<uint64_t> done(kSubmitters, 0);
    std::atomic<bool> stop{false};
    const auto b0 = Clock::now() + std::chrono::milliseconds(5);
    const double period = kSubmitters / rate;  // seconds between one submitter's topics
    std::vector<std::thread> th;
    for (int w = 0; w < kSubmitters; w++)
      th.emplace_back([&, w] {
        std::deque<std::pair<Clock::time_point, Ticket>> q;
        size_t at_w = (size_t)w * 9973;
        uint64_t k = 0;
        auto harvest = [&](bool all) {
          while (!q.empty() && (all || q.front().second.ready())) {
            q.front().second.wait();
            wl[w].push_back(std::chrono::duration<double, std::micro>(q.front().second.done_at() - q.front().first).count());
            q.pop_front();
            done[w]++;
          }
        };
        while (!stop) {
          const auto now = Clock::now();
          // every topic due by now (the schedule, not this thread's wake-ups, sets the load)
          while (!stop) {
            const auto due = b0 + std::chrono::duration_cast<Clock::duration>(
                                      std::chrono::duration<double>((k + (double)w / kSubmitters) * period));
            if (due > now) break;
            q.emplace_back(Clock::now(), pb.Submit(topics[at_w % topics.size()]));
            at_w += 7;
            k++;
          }
          harvest(false);
          std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
        harvest(true);
      });
    std::this_thread::sleep_for(std::chrono::duration<double>(secs));
    stop = true;
    for (auto& t : th) t.join();
    const double bt = std::chrono::duration<double>(Clock::now() - b0).count();
    const auto st = pb.stats();
    std::vector<double> all;
    uint64_t n_done = 0;
    for (int w = 0; w < kSubmitters; w++) {
      all.insert(all.end(), wl[w].begin(), wl[w].end());
      n_done += done[w];
    }
    const double w50 = pct(all, 0.50), w99 = pct(all, 0.99);
    std::printf("{\"path\": \"PublishViewBatcher open loop\", \"offered_per_s\": %.0f, \"max_batch\": %zu, "
                "\"submitters\": %d, \"topics\": %llu, \"topics_per_s\": %.0f, \"p50_us\": %.1f, \"p99_us\": %.1f, "
                "\"mean_batch\": %.1f, \"largest_batch\": %llu, \"dispatcher_ms_per_batch\": {\"wait\": %.3f, "
                "\"seal\": %.3f, \"match\": %.3f, \"complete\": %.3f}}\n",
                rate, B, kSubmitters, (unsigned long long)n_done, n_done / bt, w50, w99,
                (double)st.topics / std::max<uint64_t>(st.batches, 1), (unsigned long long)st.largest,
                st.wait_ns / 1e6 / std::max<uint64_t>(st.batches, 1), st.seal_ns / 1e6 / std::max<uint64_t>(st.batches, 1),
                st.match_ns / 1e6 / std::max<uint64_t>(st.batches, 1),
                st.complete_ns / 1e6 / std::max<uint64_t>(st.batches, 1));
    std::fflush(stdout);
  };
  for (const double rate : {1e6, 2e6, 5e6, 10e6}) open_loop(rate, 16384);

  for (const size_t B : {(size_t)1, (size_t)64, (size_t)1024, (size_t)16384, (size_t)65536}) {
    // match: one call per batch
    std::vector<double> lat;
    size_t at = 0;
    uint64_t rows = 0;
    const auto m0 = Clock::now();
    while (lat.size() < 20 || std::chrono::duration<double>(Clock::now() - m0).count() < secs) {
      std::string b;
      std::vector<uint64_t> o(1, 0);
      for (size_t k = 0; k < B; k++, at = (at + 1) % topics.size()) {
        b += topics[at];
        o.push_back(b.size());
      }
      b.resize(b.size() + 16, '\0');
      mq_span_result* r = nullptr;
      const auto t0 = Clock::now();
      if (mq_match_spans(ix.handle(), (const uint8_t*)b.data(), o.data(), (uint32_t)B, &r) < 0) {
        std::fprintf(stderr, "mq_match_spans: %s\n", mq_last_error());
        return 1;
      }
      lat.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
      for (uint32_t t = 0; t < r->n_topics; t++) rows += r->topics[t].n_rows;
      mq_result_free(r);
      if (lat.size() >= 100000) break;
    }
    const double mt = std::chrono::duration<double>(Clock::now() - m0).count();
    const size_t calls = lat.size();
    const double p50 = pct(lat, 0.50), p99 = pct(lat, 0.99);
    std::printf("{\"path\": \"mq_match_spans\", \"batch\": %zu, \"calls\": %zu, \"p50_us\": %.1f, \"p99_us\": %.1f, "
                "\"topics_per_s\": %.0f, \"records_per_topic\": %.1f}\n",
                B, calls, p50, p99, calls * B / mt, (double)rows / (calls * B));
    std::fflush(stdout);

    // batcher: kSubmitters threads (connection goroutines) keep 2B topics in flight together
    if (B < 1024) continue;  // (the stage is measured at the batch sizes a broker would run)
    const size_t window = std::max<size_t>(1, 2 * B / kSubmitters);
    std::vector<std::vector<double>> wl(kSubmitters);
    std::vector<uint64_t> recipients(kSubmitters, 0), sampled(kSubmitters, 0), done(kSubmitters, 0);
    {
      mq::host::PublishViewBatcher pb(ix, B, std::chrono::microseconds(200), std::min<size_t>(B, 1024));
      const auto b0 = Clock::now();
      std::atomic<bool> stop{false};
      std::vector<std::thread> th;
      for (int w = 0; w < kSubmitters; w++)
        th.emplace_back([&, w] {
          std::deque<std::pair<Clock::time_point, mq::host::PublishViewBatcher::Ticket>> q;
          size_t at_w = (size_t)w * 9973;
          for (;;) {
            while (!stop && q.size() < window) {
              q.emplace_back(Clock::now(), pb.Submit(topics[at_w % topics.size()]));
              at_w += 7;
            }
            if (q.empty()) break;
            auto& f = q.front();
            const mq::host::TopicView& v = f.second.get();
            wl[w].push_back(std::chrono::duration<double, std::micro>(Clock::now() - f.first).count());
            // the fan-out reads every view on the broker's connection goroutines; one in 64 is
            // read here, so that the stage, not the readers, is measured
            if (done[w] % 64 == 0) {
              v.for_each_row([&](const mq_client_row&) { recipients[w]++; });
              sampled[w]++;
            }
            q.pop_front();
            done[w]++;
          }
        });
      std::this_thread::sleep_for(std::chrono::duration<double>(secs));
      stop = true;
      for (auto& t : th) t.join();
      const double bt = std::chrono::duration<double>(Clock::now() - b0).count();
      const auto st = pb.stats();
      std::vector<double> all;
      uint64_t n_done = 0, n_rec = 0, n_smp = 0;
      for (int w = 0; w < kSubmitters; w++) {
        all.insert(all.end(), wl[w].begin(), wl[w].end());
        n_done += done[w];
        n_rec += recipients[w];
        n_smp += sampled[w];
      }
      const double w50 = pct(all, 0.50), w99 = pct(all, 0.99);
      std::printf("{\"path\": \"PublishViewBatcher\", \"max_batch\": %zu, \"submitters\": %d, \"in_flight\": %zu, "
                  "\"topics\": %llu, \"p50_us\": %.1f, \"p99_us\": %.1f, \"topics_per_s\": %.0f, \"mean_batch\": %.1f, "
                  "\"largest_batch\": %llu, \"recipients_per_topic\": %.1f, \"dispatcher_ms_per_batch\": "
                  "{\"wait\": %.3f, \"seal\": %.3f, \"match\": %.3f, \"complete\": %.3f}}\n",
                  B, kSubmitters, window * kSubmitters, (unsigned long long)n_done, w50, w99, n_done / bt,
                  (double)st.topics / std::max<uint64_t>(st.batches, 1), (unsigned long long)st.largest,
                  (double)n_rec / std::max<uint64_t>(n_smp, 1), st.wait_ns / 1e6 / std::max<uint64_t>(st.batches, 1),
                  st.seal_ns / 1e6 / std::max<uint64_t>(st.batches, 1), st.match_ns / 1e6 / std::max<uint64_t>(st.batches, 1),
                  st.complete_ns / 1e6 / std::max<uint64_t>(st.batches, 1));
      std::fflush(stdout);
    }
  }
  return 0;
}
