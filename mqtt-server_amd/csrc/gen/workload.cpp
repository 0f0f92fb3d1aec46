// Deterministic synthetic workload generator for bench.py and the parity tests.
// Input generation only: it neither matches nor merges anything.
//
// Vocabulary: level 0 has 256 tokens, every level >= 1 its own 4096 tokens; tokens are
// [a-z0-9_-] strings of length 3..12, drawn Zipf(s=1.0) per level. Seeds: base 0x6D716D61,
// subscriptions seed+1, topics seed+2, retained topics seed+3, wildcard filters seed+4.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

constexpr int kMaxLevels = 16;

struct Rng {  // xoshiro256** seeded by splitmix64
  uint64_t s[4];
  explicit Rng(uint64_t seed) {
    for (int i = 0; i < 4; i++) {
      seed += 0x9e3779b97f4a7c15ull;
      uint64_t z = seed;
      z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
      z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
      s[i] = z ^ (z >> 31);
    }
  }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
    return r;
  }
  double uniform() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  uint64_t below(uint64_t n) { return (uint64_t)(uniform() * (double)n) % n; }
  bool chance(double p) { return uniform() < p; }
};

struct Vocab {
  std::vector<std::vector<std::string>> tokens;  // per level
  std::vector<std::vector<double>> cdf;          // Zipf(1.0) per level

  explicit Vocab(uint64_t seed) {
    static const char alpha[] = "abcdefghijklmnopqrstuvwxyz0123456789_-";
    Rng r(seed ^ 0x766f636162ull);
    tokens.resize(kMaxLevels);
    cdf.resize(kMaxLevels);
    for (int l = 0; l < kMaxLevels; l++) {
      size_t v = l == 0 ? 256 : 4096;
      std::unordered_set<std::string> seen;
      while (tokens[l].size() < v) {
        int len = 3 + (int)r.below(10);
        std::string t;
        for (int i = 0; i < len; i++) t += alpha[r.below(sizeof(alpha) - 1)];
        if (seen.insert(t).second) tokens[l].push_back(t);
      }
      double acc = 0;
      for (size_t i = 0; i < v; i++) acc += 1.0 / (double)(i + 1);
      double run = 0;
      for (size_t i = 0; i < v; i++) {
        run += 1.0 / (double)(i + 1) / acc;
        cdf[l].push_back(run);
      }
      cdf[l].back() = 1.0;
    }
  }
  const std::string& draw(int level, Rng& r) const {
    int l = level < kMaxLevels ? level : kMaxLevels - 1;
    double u = r.uniform();
    const auto& c = cdf[l];
    size_t lo = 0, hi = c.size() - 1;
    while (lo < hi) {
      size_t mid = (lo + hi) / 2;
      if (c[mid] < u) lo = mid + 1; else hi = mid;
    }
    return tokens[l][lo];
  }
};

struct Strings {
  std::vector<uint8_t> bytes;
  std::vector<uint64_t> offs{0};
  void push(const std::string& s) {
    bytes.insert(bytes.end(), s.begin(), s.end());
    offs.push_back(bytes.size());
  }
  size_t size() const { return offs.size() - 1; }
  std::string at(size_t i) const {
    return std::string((const char*)bytes.data() + offs[i], offs[i + 1] - offs[i]);
  }
};

struct Subs {
  Strings filters;
  std::vector<uint32_t> client_ids, filter_ids;
  std::vector<uint8_t> qos, flags;
  std::vector<int32_t> idents;
  uint64_t n_unique_filters = 0;
};

struct Batch {
  Strings s;
  std::vector<uint64_t> handles;
};

std::string join(const std::vector<std::string>& v) {
  std::string o;
  for (size_t i = 0; i < v.size(); i++) {
    if (i) o += '/';
    o += v[i];
  }
  return o;
}

// Split a filter on '/', keeping empty segments.
std::vector<std::string> split(const std::string& f) {
  std::vector<std::string> out;
  size_t s = 0;
  for (;;) {
    size_t e = f.find('/', s);
    if (e == std::string::npos) { out.push_back(f.substr(s)); break; }
    out.push_back(f.substr(s, e - s));
    s = e + 1;
  }
  return out;
}

}  // namespace

extern "C" {

// mix: 0 = config-2/3 mix (depth 4-8, 30% '+', 10% '#', 5% $share, 0.1% top-level wildcards);
//      1 = IoT fan-in (config 4): exact dev/r{0..63}/s{0..4095}/d{u32}/telemetry + 1% dashboards.
void* mqgen_subs(uint64_t n_subs, uint32_t n_clients, uint64_t seed, int mix) {
  Vocab voc(seed);
  Rng r(seed + 1);
  Subs* out = new Subs();
  std::unordered_map<std::string, uint32_t> intern;
  intern.reserve(n_subs * 2);
  static const char* share_case[3] = {"$share", "$SHARE", "$Share"};
  for (uint64_t i = 0; i < n_subs; i++) {
    std::vector<std::string> seg;
    uint32_t client;
    if (mix == 1) {
      if (r.chance(0.01)) {
        unsigned rr = (unsigned)r.below(64);
        if (r.chance(0.5))
          seg = {"dev", "r" + std::to_string(rr), "+", "+", "telemetry"};
        else
          seg = {"dev", "r" + std::to_string(rr), "s" + std::to_string(r.below(4096)), "#"};
        client = (uint32_t)r.below(n_clients);
      } else {
        seg = {"dev", "r" + std::to_string(r.below(64)), "s" + std::to_string(r.below(4096)),
               "d" + std::to_string((uint32_t)r.next()), "telemetry"};
        client = (uint32_t)(i % n_clients);  // one unique client per device filter
      }
    } else {
      client = (uint32_t)r.below(n_clients);
      int k = 4 + (int)r.below(5);
      for (int l = 0; l < k; l++) seg.push_back(voc.draw(l, r));
      if (r.chance(0.30)) {
        int nplus = 1 + (int)r.below(2);
        for (int j = 0; j < nplus; j++) seg[1 + r.below(k - 1)] = "+";
      }
      if (r.chance(0.10)) {
        int j = 1 + (int)r.below(k - 1);
        seg.resize(j);
        seg.push_back("#");
      }
      if (r.chance(0.001)) {  // top-level wildcard
        if (r.chance(0.5)) seg = {"#"};
        else seg[0] = "+";
      }
      if (r.chance(0.05)) {
        std::vector<std::string> sh{share_case[r.below(3)], "g" + std::to_string(r.below(16))};
        sh.insert(sh.end(), seg.begin(), seg.end());
        seg.swap(sh);
      }
    }
    std::string f = join(seg);
    auto it = intern.find(f);
    uint32_t fid;
    if (it == intern.end()) {
      fid = (uint32_t)intern.size();
      intern.emplace(f, fid);
    } else {
      fid = it->second;
    }
    out->filters.push(f);
    out->client_ids.push_back(client);
    out->filter_ids.push_back(fid);
    out->qos.push_back((uint8_t)r.below(3));
    int32_t ident = r.chance(0.5) ? 0 : (int32_t)(1 + r.below(268435455));
    out->idents.push_back(ident);
    uint8_t fl = 0;
    if (r.chance(0.05)) fl |= 1;
    if (r.chance(0.5)) fl |= 2;
    fl |= (uint8_t)(r.below(3) << 2);
    out->flags.push_back(fl);
  }
  out->n_unique_filters = intern.size();
  return out;
}

uint64_t mqgen_subs_n(void* h) { return ((Subs*)h)->filters.size(); }
uint64_t mqgen_subs_nbytes(void* h) { return ((Subs*)h)->filters.bytes.size(); }
uint64_t mqgen_subs_unique_filters(void* h) { return ((Subs*)h)->n_unique_filters; }
void mqgen_subs_copy(void* h, uint8_t* bytes, uint64_t* offs, uint32_t* client_ids,
                     uint32_t* filter_ids, uint8_t* qos, uint8_t* flags, int32_t* idents) {
  Subs* s = (Subs*)h;
  size_t n = s->filters.size();
  memcpy(bytes, s->filters.bytes.data(), s->filters.bytes.size());
  memcpy(offs, s->filters.offs.data(), (n + 1) * 8);
  memcpy(client_ids, s->client_ids.data(), n * 4);
  memcpy(filter_ids, s->filter_ids.data(), n * 4);
  memcpy(qos, s->qos.data(), n);
  memcpy(flags, s->flags.data(), n);
  memcpy(idents, s->idents.data(), n * 4);
}
void mqgen_subs_free(void* h) { delete (Subs*)h; }

// Publish topics: 70% instantiate a random existing filter ('+' -> token,
// '#' -> 0..3 tokens), 30% fresh with depth 1..10; 1% $SYS/..., 0.5% $<token>/...
// Never empty, never containing '+' or '#'.
void* mqgen_topics(void* subs_h, uint64_t n_topics, uint64_t seed, int mix) {
  Subs* subs = (Subs*)subs_h;
  Vocab voc(seed);
  Rng r(seed + 2);
  Batch* out = new Batch();
  out->s.bytes.reserve(n_topics * 56);
  out->s.offs.reserve(n_topics + 1);
  size_t ns = subs ? subs->filters.size() : 0;
  for (uint64_t i = 0; i < n_topics; i++) {
    std::vector<std::string> seg;
    double u = r.uniform();
    if (u < 0.01) {
      seg = {"$SYS", "broker", voc.draw(2, r)};
      int extra = (int)r.below(3);
      for (int l = 0; l < extra; l++) seg.push_back(voc.draw(3 + l, r));
    } else if (u < 0.015) {
      seg = {"$" + voc.draw(0, r)};
      int extra = 1 + (int)r.below(4);
      for (int l = 0; l < extra; l++) seg.push_back(voc.draw(1 + l, r));
    } else if (ns && u < 0.015 + 0.70) {
      std::vector<std::string> fs = split(subs->filters.at(r.below(ns)));
      size_t start = 0;
      if (fs.size() >= 3) {
        // strip a $share/<group>/ prefix (the shared path starts at segment 2)
        const std::string& p = fs[0];
        if (p.size() == 6 && (p[0] == '$') && (p[1] | 32) == 's' && (p[2] | 32) == 'h' &&
            (p[3] | 32) == 'a' && (p[4] | 32) == 'r' && (p[5] | 32) == 'e')
          start = 2;
      }
      for (size_t l = start; l < fs.size(); l++) {
        size_t lvl = l - start;
        if (fs[l] == "+") {
          if (mix == 1) seg.push_back("s" + std::to_string(r.below(4096)));
          else seg.push_back(voc.draw((int)lvl, r));
        } else if (fs[l] == "#") {
          int extra = (int)r.below(4);
          for (int e = 0; e < extra; e++) seg.push_back(voc.draw((int)(lvl + e), r));
        } else {
          seg.push_back(fs[l]);
        }
      }
      if (seg.empty()) seg.push_back(voc.draw(0, r));
    } else {
      if (mix == 1) {
        seg = {"dev", "r" + std::to_string(r.below(64)), "s" + std::to_string(r.below(4096)),
               "d" + std::to_string((uint32_t)r.next()), "telemetry"};
      } else {
        int k = 1 + (int)r.below(10);
        for (int l = 0; l < k; l++) seg.push_back(voc.draw(l, r));
      }
    }
    out->s.push(join(seg));
  }
  return out;
}

// Retained topics (config 5): topic names generated like fresh config-2 topics (mix 0) or IoT
// device topics (mix 1), plus n_sys `$SYS/...` topics; handle = index + 1.
void* mqgen_retained(uint64_t n, uint64_t n_sys, uint64_t seed, int mix) {
  Vocab voc(seed);
  Rng r(seed + 3);
  Batch* out = new Batch();
  const uint64_t want = n + n_sys;
  out->s.bytes.reserve(want * 48);
  out->s.offs.reserve(want + 1);
  out->handles.reserve(want);
  // Exact de-duplication (same topics, same order as a set of strings would give): an
  // open-addressing table of (hash tag, topic index + 1) over the batch's own bytes, load <= 1/2.
  uint64_t cap = 1024;
  while (cap < 2 * want) cap <<= 1;
  std::vector<uint64_t> table(cap, 0);
  auto hash = [](const char* p, size_t len) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ len;
    for (size_t i = 0; i < len; i++) h = (h ^ (uint8_t)p[i]) * 0x100000001B3ull;
    return h ^ (h >> 29);
  };
  std::string t;
  while (out->s.size() < want) {
    t.clear();
    auto add = [&](const std::string& s) {
      if (!t.empty()) t += '/';
      t += s;
    };
    if (out->s.size() < n_sys) {
      add("$SYS"); add("broker"); add(voc.draw(2, r)); add(voc.draw(3, r));
    } else if (mix == 1) {
      add("dev"); add("r" + std::to_string(r.below(64))); add("s" + std::to_string(r.below(4096)));
      add("d" + std::to_string((uint32_t)r.next())); add("telemetry");
    } else {
      int k = 2 + (int)r.below(7);
      for (int l = 0; l < k; l++) add(voc.draw(l, r));
    }
    const uint64_t h = hash(t.data(), t.size());
    const uint64_t tag = h & 0xFFFFFFFF00000000ull;
    bool dup = false;
    uint64_t i = h & (cap - 1);
    for (;; i = (i + 1) & (cap - 1)) {
      const uint64_t e = table[i];
      if (!e) break;
      if ((e & 0xFFFFFFFF00000000ull) != tag) continue;
      const uint64_t k = (e & 0xFFFFFFFFull) - 1;
      const uint64_t o = out->s.offs[k], len = out->s.offs[k + 1] - o;
      if (len == t.size() && !memcmp(out->s.bytes.data() + o, t.data(), len)) { dup = true; break; }
    }
    if (dup) continue;
    table[i] = tag | (out->s.size() + 1);
    out->s.push(t);
    out->handles.push_back(out->s.size());
  }
  return out;
}

// Wildcard filters for the Messages path (config 5): mostly '+' at depth >= 2 and '#' at
// depth >= 3, plus a few literal filters; derived from the retained topics so they hit.
void* mqgen_msg_filters(void* retained_h, uint64_t n, uint64_t seed) {
  Batch* ret = (Batch*)retained_h;
  Rng r(seed + 4);
  Batch* out = new Batch();
  size_t nr = ret->s.size();
  for (uint64_t i = 0; i < n; i++) {
    std::vector<std::string> seg = split(ret->s.at(r.below(nr)));
    double u = r.uniform();
    if (u < 0.45 && seg.size() >= 3) {
      seg[2 + r.below(seg.size() - 2)] = "+";
    } else if (u < 0.90 && seg.size() >= 4) {
      size_t j = 3 + r.below(seg.size() - 3);
      seg.resize(j);
      seg.push_back("#");
    } else if (u < 0.95 && seg.size() >= 2) {
      seg[1] = "+";
      if (seg.size() >= 3) seg[seg.size() - 1] = "+";
    }
    out->s.push(join(seg));
  }
  return out;
}

uint64_t mqgen_batch_n(void* h) { return ((Batch*)h)->s.size(); }
uint64_t mqgen_batch_nbytes(void* h) { return ((Batch*)h)->s.bytes.size(); }
void mqgen_batch_copy(void* h, uint8_t* bytes, uint64_t* offs, uint64_t* handles) {
  Batch* b = (Batch*)h;
  memcpy(bytes, b->s.bytes.data(), b->s.bytes.size());
  memcpy(offs, b->s.offs.data(), b->s.offs.size() * 8);
  if (handles && !b->handles.empty()) memcpy(handles, b->handles.data(), b->handles.size() * 8);
}
void mqgen_batch_free(void* h) { delete (Batch*)h; }

}  // extern "C"
