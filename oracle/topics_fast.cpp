// CPU BASELINE — TEST / MEASUREMENT INFRASTRUCTURE ONLY (see topics_fast.h).
#include "topics_fast.h"

#include <algorithm>
#include <string_view>
#include <vector>

namespace oracle {

namespace {

constexpr uint32_t kNone = 0xFFFFFFFFu;

inline uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}
inline uint64_t fold(uint64_t h, uint64_t v) { return mix64(h ^ mix64(v + 0x9e3779b97f4a7c15ull)); }
inline uint64_t row_hash(uint64_t cat, uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
  return fold(fold(fold(fold(cat, a), b), c), d);
}

struct FSub {
  uint32_t client, filter;
  int32_t ident;
  uint32_t meta;  // qos | nolocal << 8 | rap << 9 | rh << 10 (the engine's row meta)
  bool wild0;     // filter starts with '+' / '#': dropped for '$' topics (topics.go:637)
};
struct FShr {
  uint32_t filter, client;
};
struct FInl {
  int64_t id;
  uint32_t filter;
};
struct FNode {
  std::unordered_map<std::string, uint32_t> kids;  // particles, keyed by segment (topics.go:772)
  uint32_t plus = kNone, hash = kNone;              // the "+" and "#" children
  uint32_t sub_off = 0, sub_cnt = 0, shr_off = 0, shr_cnt = 0, inl_off = 0, inl_cnt = 0;
};

}  // namespace

struct FastIndex {
  std::vector<FNode> nodes;
  std::vector<FSub> subs;
  std::vector<FShr> shr;
  std::vector<FInl> inl;
  uint32_t n_clients = 0;
};

struct FastScratch {
  struct Merged {
    uint32_t client, base, meta;  // base: index of the first gathered FSub; meta: merged
  };
  std::vector<uint32_t> epoch, slot;  // per client id: result stamp, index into res
  uint32_t cur = 0;
  std::vector<Merged> res;                     // Subscriptions
  std::vector<FSub> idents;                    // Identifiers entries beyond the base's
  std::vector<FShr> shared;                    // Shared[filter][client]
  std::vector<FInl> inl;                       // InlineSubscriptions, in gather order
  std::unordered_map<int64_t, uint32_t> inl_last;
  std::vector<std::string_view> segs;
  std::string key;
  bool dollar = false;
};

void fast_free(FastIndex* f) { delete f; }
void fast_scratch_free(FastScratch* s) { delete s; }

FastIndex* fast_build(const TopicsIndex& idx, const std::unordered_map<std::string, uint32_t>& client_ids,
                      const std::unordered_map<std::string, uint32_t>& filter_ids) {
  FastIndex* f = new FastIndex();
  std::unordered_map<std::string, uint32_t> extra_c, extra_f;
  uint32_t max_c = 0, max_f = 0;
  for (auto& kv : client_ids) max_c = std::max(max_c, kv.second + 1);
  for (auto& kv : filter_ids) max_f = std::max(max_f, kv.second + 1);
  auto cid = [&](const std::string& c) {
    auto it = client_ids.find(c);
    if (it != client_ids.end()) return it->second;
    auto e = extra_c.emplace(c, max_c + (uint32_t)extra_c.size());
    return e.first->second;
  };
  auto fid = [&](const std::string& s) {
    auto it = filter_ids.find(s);
    if (it != filter_ids.end()) return it->second;
    auto e = extra_f.emplace(s, max_f + (uint32_t)extra_f.size());
    return e.first->second;
  };
  // iterative DFS over the particle tree; node ids in visit order
  std::vector<std::pair<const Particle*, uint32_t>> stack{{idx.root(), 0u}};
  f->nodes.emplace_back();
  while (!stack.empty()) {
    const Particle* p = stack.back().first;
    const uint32_t id = stack.back().second;
    stack.pop_back();
    {
      FNode& n = f->nodes[id];
      n.sub_off = (uint32_t)f->subs.size();
      for (auto& kv : p->subscriptions) {
        const Subscription& s = kv.second;
        const uint32_t meta = (s.qos & 3u) | (s.no_local ? 0x100u : 0u) | (s.retain_as_published ? 0x200u : 0u) |
                              ((s.retain_handling & 3u) << 10);
        const bool w0 = !s.filter.empty() && (s.filter[0] == '+' || s.filter[0] == '#');
        f->subs.push_back(FSub{cid(kv.first), fid(s.filter), (int32_t)s.identifier, meta, w0});
      }
      n.sub_cnt = (uint32_t)f->subs.size() - n.sub_off;
      n.shr_off = (uint32_t)f->shr.size();
      for (auto& g : p->shared)
        for (auto& kv : g.second) f->shr.push_back(FShr{fid(kv.second.filter), cid(kv.first)});
      n.shr_cnt = (uint32_t)f->shr.size() - n.shr_off;
      n.inl_off = (uint32_t)f->inl.size();
      for (auto& kv : p->inline_subscriptions) f->inl.push_back(FInl{kv.first, fid(kv.second.sub.filter)});
      n.inl_cnt = (uint32_t)f->inl.size() - n.inl_off;
    }
    for (auto& kv : p->particles) {
      const uint32_t c = (uint32_t)f->nodes.size();
      f->nodes.emplace_back();  // may reallocate: index, do not hold references across
      f->nodes[id].kids.emplace(kv.first, c);
      if (kv.first == "+") f->nodes[id].plus = c;
      if (kv.first == "#") f->nodes[id].hash = c;
      stack.emplace_back(kv.second.get(), c);
    }
  }
  f->n_clients = max_c + (uint32_t)extra_c.size();
  return f;
}

FastScratch* fast_scratch(const FastIndex& f) {
  FastScratch* s = new FastScratch();
  s->epoch.assign(f.n_clients, 0);
  s->slot.assign(f.n_clients, 0);
  return s;
}

namespace {

// gatherSubscriptions (topics.go:631-648) + Subscription.Merge (packets/packets.go:254-274)
inline void gather_subs(const FastIndex& f, FastScratch& s, const FNode& n) {
  for (uint32_t i = n.sub_off; i < n.sub_off + n.sub_cnt; i++) {
    const FSub& r = f.subs[i];
    if (s.dollar && r.wild0) continue;
    if (s.epoch[r.client] != s.cur) {
      s.epoch[r.client] = s.cur;
      s.slot[r.client] = (uint32_t)s.res.size();
      s.res.push_back(FastScratch::Merged{r.client, i, r.meta});
      continue;
    }
    FastScratch::Merged& m = s.res[s.slot[r.client]];
    const uint32_t q = std::max(m.meta & 3u, r.meta & 3u);
    m.meta = (m.meta & ~3u) | q | (r.meta & 0x100u);
    if (r.ident > 0) s.idents.push_back(r);
  }
}

inline void gather_shared(const FastIndex& f, FastScratch& s, const FNode& n) {  // topics.go:651-665
  for (uint32_t i = n.shr_off; i < n.shr_off + n.shr_cnt; i++) s.shared.push_back(f.shr[i]);
}

inline void gather_inline(const FastIndex& f, FastScratch& s, const FNode& n) {  // topics.go:668-676
  for (uint32_t i = n.inl_off; i < n.inl_off + n.inl_cnt; i++) s.inl.push_back(f.inl[i]);
}

inline void gather_all(const FastIndex& f, FastScratch& s, const FNode& n) {
  gather_subs(f, s, n);
  gather_shared(f, s, n);
  gather_inline(f, s, n);
}

// scanSubscribers (topics.go:593-628) over the pre-split segments
void scan(const FastIndex& f, FastScratch& s, uint32_t d, uint32_t node) {
  const std::string_view seg = s.segs[d];
  const bool has_next = d + 1 < s.segs.size();
  const FNode& n = f.nodes[node];
  for (int pk = 0; pk < 2; pk++) {
    uint32_t p = kNone;
    if (pk == 0) {
      if (seg == "+") continue;  // a literal "+" visits the '+' child twice, identically
      s.key.assign(seg.data(), seg.size());
      auto it = n.kids.find(s.key);
      if (it != n.kids.end()) p = it->second;
    } else {
      p = n.plus;
    }
    if (p == kNone) continue;
    if (has_next) {
      scan(f, s, d + 1, p);
      continue;
    }
    const FNode& pn = f.nodes[p];
    gather_all(f, s, pn);
    if (pk == 0 && pn.hash != kNone) {  // filter/# matches filter; inline: the particle's again (Q2)
      gather_subs(f, s, f.nodes[pn.hash]);
      gather_shared(f, s, f.nodes[pn.hash]);
      gather_inline(f, s, pn);
    }
  }
  if (n.hash != kNone) gather_all(f, s, f.nodes[n.hash]);
}

}  // namespace

uint64_t fast_subscribers(const FastIndex& f, FastScratch& s, const char* topic, uint32_t len,
                          uint64_t* digest, uint64_t counts[4]) {
  if (++s.cur == 0) {  // epoch wrap: restamp
    std::fill(s.epoch.begin(), s.epoch.end(), 0);
    s.cur = 1;
  }
  s.res.clear();
  s.idents.clear();
  s.shared.clear();
  s.inl.clear();
  if (len) {  // Subscribers("") is empty (topics.go:598-600)
    s.segs.clear();
    uint32_t b = 0;
    for (uint32_t i = 0; i <= len; i++)
      if (i == len || topic[i] == '/') {
        s.segs.emplace_back(topic + b, i - b);
        b = i + 1;
      }
    s.dollar = topic[0] == '$';
    scan(f, s, 0, 0);
  }
  uint64_t n_inl = s.inl.size();
  if (!s.inl.empty()) {  // InlineSubscriptions[id]: the last write wins
    s.inl_last.clear();
    for (uint32_t i = 0; i < s.inl.size(); i++) s.inl_last[s.inl[i].id] = i;
    n_inl = s.inl_last.size();
  }
  if (digest) {
    uint64_t n[4] = {s.res.size(), s.idents.size(), s.shared.size(), n_inl}, sum[4] = {0, 0, 0, 0};
    for (const FastScratch::Merged& m : s.res) {
      const FSub& b = f.subs[m.base];
      sum[0] += row_hash(1, m.client, b.filter, (uint32_t)b.ident, m.meta);
    }
    for (const FSub& r : s.idents) sum[1] += row_hash(2, r.client, r.filter, (uint32_t)r.ident, 0);
    for (const FShr& r : s.shared) sum[2] += row_hash(3, r.filter, r.client, 0, 0);
    if (!s.inl.empty())
      for (auto& kv : s.inl_last) sum[3] += row_hash(4, (uint32_t)kv.first, s.inl[kv.second].filter, 0, 0);
    uint64_t d = 0x6d716d61ull;
    for (int k = 0; k < 4; k++) d = fold(fold(d, n[k]), sum[k]);
    *digest = d;
    if (counts)
      for (int k = 0; k < 4; k++) counts[k] = n[k];
  }
  return s.res.size() + s.shared.size() + n_inl;
}

// ---- Messages ----

namespace {
struct FMNode {
  std::unordered_map<std::string, uint32_t> kids;  // particles, keyed by segment
  std::vector<uint32_t> list;                      // the same children, for '+' / '#' (getAll)
  int64_t h = -1;          // Retained.Get(retain_path) at build time (-1: none)
  bool path = false;       // retain_path != "" (the enumerations' check, topics.go:558)
  bool sys = false;        // key == "$SYS" (skipped at level 0, topics.go:549)
};
}  // namespace

struct FastMsgIndex {
  const TopicsIndex* idx = nullptr;  // Retained.Get(filter) of a filter without wildcards
  std::vector<FMNode> nodes;
  bool empty = true;                 // Retained.Len() == 0
};

FastMsgIndex* fast_msg_build(const TopicsIndex& idx) {
  FastMsgIndex* f = new FastMsgIndex();
  f->idx = &idx;
  f->empty = idx.retained_len() == 0;
  std::vector<std::pair<const Particle*, uint32_t>> stack{{idx.root(), 0u}};
  f->nodes.emplace_back();
  while (!stack.empty()) {
    const Particle* p = stack.back().first;
    const uint32_t id = stack.back().second;
    stack.pop_back();
    RetainedPacket pk;
    if (idx.retained_get(p->retain_path, &pk)) f->nodes[id].h = (int64_t)pk.handle;
    f->nodes[id].path = !p->retain_path.empty();
    f->nodes[id].sys = p->key == "$SYS";
    for (auto& kv : p->particles) {
      const uint32_t c = (uint32_t)f->nodes.size();
      f->nodes.emplace_back();
      f->nodes[id].kids.emplace(kv.first, c);
      f->nodes[id].list.push_back(c);
      stack.emplace_back(kv.second.get(), c);
    }
  }
  return f;
}

void fast_msg_free(FastMsgIndex* f) { delete f; }

namespace {
// scanMessages (topics.go:546-578) over pre-split segments
void scan_msg(const FastMsgIndex& f, const std::vector<std::string_view>& segs, std::string& key, uint32_t d,
              uint32_t node, std::vector<uint64_t>& out) {
  // isolateParticle past the last segment gives the last one again ('#' recurses below itself)
  const std::string_view seg = segs[std::min<size_t>(d, segs.size() - 1)];
  const bool has_next = d + 1 < segs.size();
  const FMNode& n = f.nodes[node];
  if (seg == "+" || seg == "#") {
    for (uint32_t c : n.list) {
      const FMNode& a = f.nodes[c];
      if (d == 0 && a.sys) continue;
      if (!has_next && a.path && a.h >= 0) out.push_back((uint64_t)a.h);
      if (has_next || seg == "#") scan_msg(f, segs, key, d + 1, c, out);
    }
    return;
  }
  key.assign(seg.data(), seg.size());
  auto it = n.kids.find(key);
  if (it == n.kids.end()) return;
  if (has_next) {
    scan_msg(f, segs, key, d + 1, it->second, out);
    return;
  }
  const FMNode& p = f.nodes[it->second];
  if (p.h >= 0) out.push_back((uint64_t)p.h);  // Q6: no emptiness check
}
}  // namespace

uint64_t fast_messages(const FastMsgIndex& f, const char* filter, uint32_t len, std::vector<uint64_t>& out) {
  out.clear();
  if (!len || f.empty) return 0;  // topics.go:535
  bool wild = false;
  for (uint32_t i = 0; i < len && !wild; i++) wild = filter[i] == '+' || filter[i] == '#';
  if (!wild) {  // Retained.Get(filter) (topics.go:539-544)
    RetainedPacket pk;
    if (f.idx->retained_get(std::string(filter, len), &pk)) out.push_back(pk.handle);
    return out.size();
  }
  thread_local std::vector<std::string_view> segs;
  thread_local std::string key;
  segs.clear();
  uint32_t b = 0;
  for (uint32_t i = 0; i <= len; i++)
    if (i == len || filter[i] == '/') {
      segs.emplace_back(filter + b, i - b);
      b = i + 1;
    }
  scan_msg(f, segs, key, 0, 0, out);
  return out.size();
}

}  // namespace oracle
