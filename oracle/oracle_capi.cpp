// ORACLE — TEST INFRASTRUCTURE ONLY. extern "C" surface of the CPU restatement for ctypes
// (tests/, __graft_entry__.smoke(), bench.py's cpu_baseline leg). Never linked by the engine.
//
// Clients and filters carry caller-chosen u32 ids next to their strings so that batch digests
// can be compared with the engine's id-based rows (include/mqmatch.h).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "topics_fast.h"
#include "topics_oracle.h"

using namespace oracle;

namespace {

struct Handle {
  TopicsIndex idx;
  std::unordered_map<std::string, uint32_t> client_ids;
  std::unordered_map<std::string, uint32_t> filter_ids;
};

uint32_t id_of(const std::unordered_map<std::string, uint32_t>& m, const std::string& s) {
  auto it = m.find(s);
  return it == m.end() ? 0xFFFFFFFFu : it->second;
}

inline uint64_t mix64(uint64_t x) {
  x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27; x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}

// Canonical digest of one sorted row list: order-sensitive fold of mixed rows.
inline uint64_t fold(uint64_t h, uint64_t v) { return mix64(h ^ mix64(v + 0x9e3779b97f4a7c15ull)); }

std::string json_escape(const std::string& s) {
  std::string o;
  for (unsigned char ch : s) {
    if (ch == '"' || ch == '\\') { o += '\\'; o += (char)ch; }
    else if (ch < 0x20) { char b[8]; snprintf(b, sizeof b, "\\u%04x", ch); o += b; }
    else o += (char)ch;
  }
  return o;
}

void sub_json(std::string& o, const Subscription& s, bool with_idents) {
  char b[160];
  o += "{\"filter\":\"" + json_escape(s.filter) + "\"";
  snprintf(b, sizeof b, ",\"identifier\":%lld,\"qos\":%u,\"no_local\":%s,\"rap\":%s,\"rh\":%u",
           (long long)s.identifier, s.qos, s.no_local ? "true" : "false",
           s.retain_as_published ? "true" : "false", s.retain_handling);
  o += b;
  if (with_idents) {
    o += ",\"identifiers\":";
    if (!s.has_identifiers) {
      o += "null";
    } else {
      o += "{";
      bool first = true;
      for (auto& kv : s.identifiers) {
        if (!first) o += ",";
        first = false;
        snprintf(b, sizeof b, "%lld", (long long)kv.second);
        o += "\"" + json_escape(kv.first) + "\":" + b;
      }
      o += "}";
    }
  }
  o += "}";
}

// Per-topic canonical digest over ids, order-independent (Go maps have no order): for each
// row category, fold in (count, wrapping sum of row hashes). Rows mirror the engine layout
// (include/mqmatch.h): client rows (client, base filter, base identifier, meta), ident rows
// (Identifiers entries other than the base filter), shared rows (filter, client), inline rows
// (identifier, filter). tests/digest.py computes the same from the engine's rows.
inline uint64_t row_hash(uint64_t cat, uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
  return fold(fold(fold(fold(cat, a), b), c), d);
}

uint64_t digest_subscribers(const Handle& h, const Subscribers& s, uint64_t counts[4]) {
  uint64_t n[4] = {0, 0, 0, 0}, sum[4] = {0, 0, 0, 0};
  for (auto& kv : s.subscriptions) {
    const Subscription& sub = kv.second;
    uint64_t c = id_of(h.client_ids, kv.first), f = id_of(h.filter_ids, sub.filter);
    uint32_t meta = (sub.qos & 3u) | (sub.no_local ? 0x100u : 0u) |
                    (sub.retain_as_published ? 0x200u : 0u) | ((sub.retain_handling & 3u) << 10);
    n[0]++;
    sum[0] += row_hash(1, c, f, (uint32_t)sub.identifier, meta);
    if (sub.has_identifiers)
      for (auto& e : sub.identifiers)
        if (e.first != sub.filter) {
          n[1]++;
          sum[1] += row_hash(2, c, id_of(h.filter_ids, e.first), (uint32_t)e.second, 0);
        }
  }
  for (auto& g : s.shared)
    for (auto& kv : g.second) {
      n[2]++;
      sum[2] += row_hash(3, id_of(h.filter_ids, g.first), id_of(h.client_ids, kv.first), 0, 0);
    }
  for (auto& kv : s.inline_subscriptions) {
    n[3]++;
    sum[3] += row_hash(4, (uint32_t)kv.first, id_of(h.filter_ids, kv.second.sub.filter), 0, 0);
  }
  if (counts)
    for (int k = 0; k < 4; k++) counts[k] = n[k];
  uint64_t d = 0x6d716d61ull;
  for (int k = 0; k < 4; k++) d = fold(fold(d, n[k]), sum[k]);
  return d;
}

}  // namespace

extern "C" {

void* orc_new() { return new Handle(); }
void orc_free(void* h) { delete (Handle*)h; }

int orc_subscribe(void* hp, const char* client, uint32_t clen, const char* filter, uint32_t flen,
                  uint32_t client_id, uint32_t filter_id, uint8_t qos, uint8_t flags,
                  int64_t identifier) {
  Handle* h = (Handle*)hp;
  Subscription s;
  s.filter.assign(filter, flen);
  s.qos = qos;
  s.identifier = identifier;
  s.no_local = flags & 1;
  s.retain_as_published = (flags >> 1) & 1;
  s.retain_handling = (flags >> 2) & 3;
  std::string c(client, clen);
  h->client_ids[c] = client_id;
  h->filter_ids[s.filter] = filter_id;
  return h->idx.subscribe(c, s) ? 1 : 0;
}

int orc_unsubscribe(void* hp, const char* filter, uint32_t flen, const char* client, uint32_t clen) {
  return ((Handle*)hp)->idx.unsubscribe(std::string(filter, flen), std::string(client, clen)) ? 1 : 0;
}

int orc_inline_subscribe(void* hp, const char* filter, uint32_t flen, int64_t id, uint32_t filter_id) {
  Handle* h = (Handle*)hp;
  InlineSubscription s;
  s.sub.filter.assign(filter, flen);
  s.sub.identifier = id;
  h->filter_ids[s.sub.filter] = filter_id;
  return h->idx.inline_subscribe(s) ? 1 : 0;
}

int orc_inline_unsubscribe(void* hp, int64_t id, const char* filter, uint32_t flen) {
  return ((Handle*)hp)->idx.inline_unsubscribe(id, std::string(filter, flen)) ? 1 : 0;
}

int64_t orc_retain_message(void* hp, const char* topic, uint32_t tlen, uint64_t handle,
                           uint32_t payload_len, uint8_t retain) {
  RetainedPacket pk{handle, payload_len, retain != 0};
  return ((Handle*)hp)->idx.retain_message(std::string(topic, tlen), pk);
}

void orc_retained_delete(void* hp, const char* topic, uint32_t tlen) {
  ((Handle*)hp)->idx.retained_delete(std::string(topic, tlen));
}

void orc_retained_add(void* hp, const char* topic, uint32_t tlen, uint64_t handle, uint32_t payload_len,
                      uint8_t retain) {
  ((Handle*)hp)->idx.retained_add(std::string(topic, tlen), RetainedPacket{handle, payload_len, retain != 0});
}

uint64_t orc_retained_len(void* hp) { return ((Handle*)hp)->idx.retained_len(); }
uint64_t orc_particle_count(void* hp) { return ((Handle*)hp)->idx.particle_count(); }

// Bulk subscribe, columnar (restore path analogue, server.go:1624-1640). Client strings are
// "c%07d" of the id, as in the synthetic workload.
int orc_subscribe_bulk(void* hp, const uint8_t* bytes, const uint64_t* offs,
                       const uint32_t* client_ids, const uint32_t* filter_ids, const uint8_t* qos,
                       const uint8_t* flags, const int32_t* idents, uint64_t n, uint8_t* out_new) {
  Handle* h = (Handle*)hp;
  char cb[32];
  for (uint64_t i = 0; i < n; i++) {
    int cl = snprintf(cb, sizeof cb, "c%07u", client_ids[i]);
    int r = orc_subscribe(hp, cb, (uint32_t)cl, (const char*)bytes + offs[i],
                          (uint32_t)(offs[i + 1] - offs[i]), client_ids[i], filter_ids[i], qos[i],
                          flags[i], idents[i]);
    if (out_new) out_new[i] = (uint8_t)r;
  }
  (void)h;
  return 0;
}

int orc_retain_bulk(void* hp, const uint8_t* bytes, const uint64_t* offs, const uint64_t* handles,
                    uint64_t n) {
  for (uint64_t i = 0; i < n; i++)
    orc_retain_message(hp, (const char*)bytes + offs[i], (uint32_t)(offs[i + 1] - offs[i]),
                       handles[i], 1, 1);
  return 0;
}

// Canonical JSON of Subscribers(topic) (topics.go:583) — string-keyed, for small KATs.
// Returns the needed length; writes at most cap bytes.
uint64_t orc_subscribers_json(void* hp, const char* topic, uint32_t tlen, char* buf, uint64_t cap) {
  Handle* h = (Handle*)hp;
  Subscribers s = h->idx.subscribers(std::string(topic, tlen));
  std::string o = "{\"subscriptions\":{";
  bool first = true;
  for (auto& kv : s.subscriptions) {
    if (!first) o += ",";
    first = false;
    o += "\"" + json_escape(kv.first) + "\":";
    sub_json(o, kv.second, true);
  }
  o += "},\"shared\":{";
  first = true;
  for (auto& g : s.shared) {
    if (!first) o += ",";
    first = false;
    o += "\"" + json_escape(g.first) + "\":{";
    bool f2 = true;
    for (auto& kv : g.second) {
      if (!f2) o += ",";
      f2 = false;
      o += "\"" + json_escape(kv.first) + "\":";
      sub_json(o, kv.second, true);
    }
    o += "}";
  }
  o += "},\"inline\":{";
  first = true;
  for (auto& kv : s.inline_subscriptions) {
    if (!first) o += ",";
    first = false;
    o += "\"" + std::to_string(kv.first) + "\":";
    sub_json(o, kv.second.sub, false);
  }
  o += "}}";
  if (buf && cap) {
    size_t n = o.size() < cap ? o.size() : cap;
    memcpy(buf, o.data(), n);
  }
  return o.size();
}

// Messages(filter) (topics.go:525): handles, sorted (Go returns them in map order).
uint64_t orc_messages(void* hp, const char* filter, uint32_t flen, uint64_t* out, uint64_t cap) {
  auto pks = ((Handle*)hp)->idx.messages(std::string(filter, flen));
  std::vector<uint64_t> hs;
  for (auto& p : pks) hs.push_back(p.handle);
  std::sort(hs.begin(), hs.end());
  for (uint64_t i = 0; i < hs.size() && i < cap; i++) out[i] = hs[i];
  return hs.size();
}

// Per-topic canonical digests + row counts + roofline counters (L, P, S, O summed).
int orc_digest_batch(void* hp, const uint8_t* bytes, const uint64_t* offs, uint64_t n,
                     uint32_t nthreads, uint64_t* digests, uint32_t* row_counts /*n*4 or null*/,
                     uint64_t* totals /*4: L,P,S,O*/) {
  Handle* h = (Handle*)hp;
  if (nthreads == 0) nthreads = 1;
  std::vector<Counters> cs(nthreads);
  std::vector<std::thread> th;
  for (uint32_t t = 0; t < nthreads; t++) {
    th.emplace_back([&, t] {
      for (uint64_t i = t; i < n; i += nthreads) {
        std::string topic((const char*)bytes + offs[i], offs[i + 1] - offs[i]);
        Subscribers s = h->idx.subscribers(topic, &cs[t]);
        uint64_t cnt[4];
        digests[i] = digest_subscribers(*h, s, cnt);
        if (row_counts)
          for (int k = 0; k < 4; k++) row_counts[i * 4 + k] = (uint32_t)cnt[k];
      }
    });
  }
  for (auto& x : th) x.join();
  if (totals) {
    memset(totals, 0, 4 * sizeof(uint64_t));
    for (auto& c : cs) {
      totals[0] += c.levels; totals[1] += c.lookups; totals[2] += c.scanned; totals[3] += c.out_rows;
    }
  }
  return 0;
}

// Messages digests: per filter, fold of the sorted handle list; totals L, P, O.
int orc_messages_digest_batch(void* hp, const uint8_t* bytes, const uint64_t* offs, uint64_t n,
                              uint32_t nthreads, uint64_t* digests, uint32_t* counts,
                              uint64_t* totals /*4*/) {
  Handle* h = (Handle*)hp;
  if (nthreads == 0) nthreads = 1;
  std::vector<Counters> cs(nthreads);
  std::vector<std::thread> th;
  for (uint32_t t = 0; t < nthreads; t++) {
    th.emplace_back([&, t] {
      for (uint64_t i = t; i < n; i += nthreads) {
        std::string f((const char*)bytes + offs[i], offs[i + 1] - offs[i]);
        auto pks = h->idx.messages(f, &cs[t]);
        std::vector<uint64_t> hs;
        for (auto& p : pks) hs.push_back(p.handle);
        std::sort(hs.begin(), hs.end());
        uint64_t d = 0x6d716d61ull;
        d = fold(d, hs.size());
        for (uint64_t x : hs) d = fold(d, x);
        digests[i] = d;
        if (counts) counts[i] = (uint32_t)hs.size();
      }
    });
  }
  for (auto& x : th) x.join();
  if (totals) {
    memset(totals, 0, 4 * sizeof(uint64_t));
    for (auto& c : cs) { totals[0] += c.levels; totals[1] += c.lookups; totals[2] += c.scanned; totals[3] += c.out_rows; }
  }
  return 0;
}

// The same per-filter digest of an engine's Messages result (filter i's handles at
// handles[base[i], + count[i]), any order): the checker's side of a comparison with the digests
// above, for results too large to digest in numpy.
int orc_handle_digests(const uint64_t* base, const uint32_t* count, const uint64_t* handles, uint64_t n,
                       uint32_t nthreads, uint64_t* digests) {
  if (nthreads == 0) nthreads = 1;
  std::vector<std::thread> th;
  for (uint32_t t = 0; t < nthreads; t++) {
    th.emplace_back([&, t] {
      std::vector<uint64_t> hs;
      for (uint64_t i = t; i < n; i += nthreads) {
        hs.assign(handles + base[i], handles + base[i] + count[i]);
        std::sort(hs.begin(), hs.end());
        uint64_t d = 0x6d716d61ull;
        d = fold(d, hs.size());
        for (uint64_t x : hs) d = fold(d, x);
        digests[i] = d;
      }
    });
  }
  for (auto& x : th) x.join();
  return 0;
}

// The same digest of an engine Messages runs result (mq_messages_runs_*): filter i's handles are
// handles[r.first, + r.count) over its runs runs[run_base[i], + n_runs[i]) (runs: first u32,
// count u32, at u64 — mq_msg_run), any order.
int orc_run_digests(const uint64_t* run_base, const uint32_t* n_runs, const uint32_t* runs, const uint64_t* handles,
                    uint64_t n, uint32_t nthreads, uint64_t* digests) {
  if (nthreads == 0) nthreads = 1;
  std::vector<std::thread> th;
  for (uint32_t t = 0; t < nthreads; t++) {
    th.emplace_back([&, t] {
      std::vector<uint64_t> hs;
      for (uint64_t i = t; i < n; i += nthreads) {
        hs.clear();
        for (uint64_t k = run_base[i]; k < run_base[i] + n_runs[i]; k++)
          hs.insert(hs.end(), handles + runs[4 * k], handles + runs[4 * k] + runs[4 * k + 1]);
        std::sort(hs.begin(), hs.end());
        uint64_t d = 0x6d716d61ull;
        d = fold(d, hs.size());
        for (uint64_t x : hs) d = fold(d, x);
        digests[i] = d;
      }
    });
  }
  for (auto& x : th) x.join();
  return 0;
}

// CPU baseline: `nthreads` std::threads each call Subscribers(topic) on the
// frozen shared index, as Go connection goroutines do (topics.go:583 takes no writer lock).
// Returns wall seconds; *sink receives a value derived from every result.
double orc_bench_subscribers(void* hp, const uint8_t* bytes, const uint64_t* offs, uint64_t n,
                             uint32_t nthreads, uint64_t* sink) {
  Handle* h = (Handle*)hp;
  if (nthreads == 0) nthreads = 1;
  std::atomic<uint64_t> acc{0};
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (uint32_t t = 0; t < nthreads; t++) {
    th.emplace_back([&, t] {
      uint64_t local = 0;
      for (uint64_t i = t; i < n; i += nthreads) {
        std::string topic((const char*)bytes + offs[i], offs[i + 1] - offs[i]);
        Subscribers s = h->idx.subscribers(topic);
        local += s.subscriptions.size() + s.shared.size() + s.inline_subscriptions.size();
      }
      acc += local;
    });
  }
  for (auto& x : th) x.join();
  auto t1 = std::chrono::steady_clock::now();
  if (sink) *sink = acc.load();
  return std::chrono::duration<double>(t1 - t0).count();
}

double orc_bench_messages(void* hp, const uint8_t* bytes, const uint64_t* offs, uint64_t n,
                          uint32_t nthreads, uint64_t* sink) {
  Handle* h = (Handle*)hp;
  if (nthreads == 0) nthreads = 1;
  std::atomic<uint64_t> acc{0};
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (uint32_t t = 0; t < nthreads; t++) {
    th.emplace_back([&, t] {
      uint64_t local = 0;
      for (uint64_t i = t; i < n; i += nthreads)
        local += h->idx.messages(std::string((const char*)bytes + offs[i], offs[i + 1] - offs[i])).size();
      acc += local;
    });
  }
  for (auto& x : th) x.join();
  auto t1 = std::chrono::steady_clock::now();
  if (sink) *sink = acc.load();
  return std::chrono::duration<double>(t1 - t0).count();
}

// ---- the fast Messages restatement (topics_fast.h): bench_messages.py's cpu_baseline ----
void* orc_fast_msg_build(void* hp) { return fast_msg_build(((Handle*)hp)->idx); }
void orc_fast_msg_free(void* fp) { fast_msg_free((FastMsgIndex*)fp); }

int orc_fast_msg_digest_batch(void* fp, const uint8_t* bytes, const uint64_t* offs, uint64_t n, uint32_t nthreads,
                              uint64_t* digests, uint32_t* counts) {
  const FastMsgIndex& f = *(FastMsgIndex*)fp;
  if (nthreads == 0) nthreads = 1;
  std::vector<std::thread> th;
  for (uint32_t t = 0; t < nthreads; t++) {
    th.emplace_back([&, t] {
      std::vector<uint64_t> hs;
      for (uint64_t i = t; i < n; i += nthreads) {
        fast_messages(f, (const char*)bytes + offs[i], (uint32_t)(offs[i + 1] - offs[i]), hs);
        std::sort(hs.begin(), hs.end());
        uint64_t d = 0x6d716d61ull;
        d = fold(d, hs.size());
        for (uint64_t x : hs) d = fold(d, x);
        digests[i] = d;
        if (counts) counts[i] = (uint32_t)hs.size();
      }
    });
  }
  for (auto& x : th) x.join();
  return 0;
}

double orc_fast_msg_bench(void* fp, const uint8_t* bytes, const uint64_t* offs, uint64_t n, uint32_t nthreads,
                          uint64_t* sink) {
  const FastMsgIndex& f = *(FastMsgIndex*)fp;
  if (nthreads == 0) nthreads = 1;
  std::atomic<uint64_t> acc{0};
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (uint32_t t = 0; t < nthreads; t++) {
    th.emplace_back([&, t] {
      std::vector<uint64_t> hs;
      uint64_t local = 0;
      for (uint64_t i = t; i < n; i += nthreads)
        local += fast_messages(f, (const char*)bytes + offs[i], (uint32_t)(offs[i + 1] - offs[i]), hs);
      acc += local;
    });
  }
  for (auto& x : th) x.join();
  auto t1 = std::chrono::steady_clock::now();
  if (sink) *sink = acc.load();
  return std::chrono::duration<double>(t1 - t0).count();
}

// ---- the fast CPU restatement (topics_fast.h): bench.py's cpu_baseline, checked against the
// oracle's digests in the tests ----
void* orc_fast_build(void* hp) {
  Handle* h = (Handle*)hp;
  return fast_build(h->idx, h->client_ids, h->filter_ids);
}
void orc_fast_free(void* fp) { fast_free((FastIndex*)fp); }

int orc_fast_digest_batch(void* fp, const uint8_t* bytes, const uint64_t* offs, uint64_t n, uint32_t nthreads,
                          uint64_t* digests, uint32_t* row_counts) {
  const FastIndex& f = *(FastIndex*)fp;
  if (nthreads == 0) nthreads = 1;
  std::vector<std::thread> th;
  for (uint32_t t = 0; t < nthreads; t++) {
    th.emplace_back([&, t] {
      std::unique_ptr<FastScratch, void (*)(FastScratch*)> s(fast_scratch(f), fast_scratch_free);
      for (uint64_t i = t; i < n; i += nthreads) {
        uint64_t cnt[4];
        fast_subscribers(f, *s, (const char*)bytes + offs[i], (uint32_t)(offs[i + 1] - offs[i]), &digests[i], cnt);
        if (row_counts)
          for (int k = 0; k < 4; k++) row_counts[i * 4 + k] = (uint32_t)cnt[k];
      }
    });
  }
  for (auto& x : th) x.join();
  return 0;
}

// CPU baseline: `nthreads` std::threads each run Subscribers(topic) on the shared frozen index
// (topics.go:583 takes no writer lock). Scratch tables are set up before the clock starts.
double orc_fast_bench(void* fp, const uint8_t* bytes, const uint64_t* offs, uint64_t n, uint32_t nthreads,
                      uint64_t* sink) {
  const FastIndex& f = *(FastIndex*)fp;
  if (nthreads == 0) nthreads = 1;
  std::vector<std::unique_ptr<FastScratch, void (*)(FastScratch*)>> sc;
  for (uint32_t t = 0; t < nthreads; t++) sc.emplace_back(fast_scratch(f), fast_scratch_free);
  std::atomic<uint64_t> acc{0};
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (uint32_t t = 0; t < nthreads; t++) {
    th.emplace_back([&, t] {
      uint64_t local = 0;
      for (uint64_t i = t; i < n; i += nthreads)
        local += fast_subscribers(f, *sc[t], (const char*)bytes + offs[i], (uint32_t)(offs[i + 1] - offs[i]), nullptr,
                                  nullptr);
      acc += local;
    });
  }
  for (auto& x : th) x.join();
  auto t1 = std::chrono::steady_clock::now();
  if (sink) *sink = acc.load();
  return std::chrono::duration<double>(t1 - t0).count();
}

// ---- white-box / helper surface for the transcribed tests ----
int orc_isolate_particle(const char* f, uint32_t flen, int d, uint32_t* start, uint32_t* len) {
  bool hn;
  std::string_view v = isolate_particle(std::string_view(f, flen), d, &hn);
  *start = v.data() ? (uint32_t)(v.data() - f) : 0;
  *len = (uint32_t)v.size();
  return hn ? 1 : 0;
}
int orc_is_valid_filter(const char* f, uint32_t flen, int for_publish) {
  return is_valid_filter(std::string_view(f, flen), for_publish != 0) ? 1 : 0;
}
// auth.MatchTopic: returns matched; elems (cap pairs of start, len in the topic) and *n_elems
int orc_match_topic(const char* f, uint32_t flen, const char* t, uint32_t tlen, uint32_t* elems, uint32_t cap,
                    uint32_t* n_elems) {
  std::vector<std::pair<uint32_t, uint32_t>> el;
  const bool m = match_topic(std::string_view(f, flen), std::string_view(t, tlen), &el);
  *n_elems = (uint32_t)el.size();
  for (size_t i = 0; i < el.size() && i < cap; i++) {
    elems[2 * i] = el[i].first;
    elems[2 * i + 1] = el[i].second;
  }
  return m ? 1 : 0;
}
int orc_is_shared_filter(const char* f, uint32_t flen) {
  return is_shared_filter(std::string_view(f, flen)) ? 1 : 0;
}
int orc_equal_fold_ascii(const char* s, uint32_t slen, const char* t, uint32_t tlen) {
  return equal_fold_ascii(std::string_view(s, slen), std::string_view(t, tlen)) ? 1 : 0;
}
// seek(filter, d) != nil (topics.go:499)
int orc_path_exists(void* hp, const char* f, uint32_t flen, int d) {
  return ((Handle*)hp)->idx.seek(std::string(f, flen), d) ? 1 : 0;
}
// Number of entries in a particle's containers; -1 if the path does not exist.
int64_t orc_node_counts(void* hp, const char* f, uint32_t flen, int d, int64_t* out /*5*/) {
  Particle* p = ((Handle*)hp)->idx.seek(std::string(f, flen), d);
  if (!p) return -1;
  out[0] = (int64_t)p->particles.size();
  out[1] = (int64_t)p->subscriptions.size();
  out[2] = (int64_t)p->shared_len();
  out[3] = (int64_t)p->inline_subscriptions.size();
  out[4] = p->retain_path.empty() ? 0 : 1;
  return 0;
}
uint64_t orc_root_children(void* hp) { return ((Handle*)hp)->idx.root()->particles.size(); }

}  // extern "C"
