// ORACLE — TEST INFRASTRUCTURE ONLY (see topics_oracle.h). A line-by-line CPU restatement of
// /root/reference/topics.go; each function cites the Go lines it follows.
#include "topics_oracle.h"

#include <algorithm>

namespace oracle {

static const char* kSharePrefix = "$SHARE";  // topics.go:16
static const char* kSysPrefix = "$SYS";      // topics.go:17

// packets/packets.go:254-274
Subscription Subscription::merge(const Subscription& n) const {
  Subscription s = *this;
  if (!s.has_identifiers) {
    s.has_identifiers = true;
    s.identifiers.clear();
    s.identifiers[s.filter] = s.identifier;
  }
  if (n.identifier > 0) s.identifiers[n.filter] = n.identifier;
  if (n.qos > s.qos) s.qos = n.qos;  // [MQTT-3.3.4-2]
  if (n.no_local) s.no_local = true;  // [MQTT-3.8.3-3]
  return s;
}

// topics.go:679-698. `next` is always 0 in the Go code because `filter` is re-sliced.
std::string_view isolate_particle(std::string_view filter, int d, bool* has_next) {
  std::string_view particle;
  bool hn = false;
  long end = 0;
  for (int i = 0; end > -1 && i <= d; i++) {
    size_t pos = filter.find('/');
    end = pos == std::string_view::npos ? -1 : (long)pos;
    if (d > -1 && i == d && end > -1) {
      hn = true;
      particle = filter.substr(0, (size_t)end);
    } else if (end > -1) {
      hn = false;
      filter = filter.substr((size_t)end + 1);
    } else {
      hn = false;
      particle = filter;
    }
  }
  if (has_next) *has_next = hn;
  return particle;
}

// Go utf8.DecodeRuneInString: invalid encodings decode as U+FFFD of width 1.
static uint32_t decode_rune(std::string_view s, size_t i, size_t* width) {
  const unsigned char c0 = (unsigned char)s[i];
  if (c0 < 0x80) { *width = 1; return c0; }
  auto cont = [&](size_t k) { return i + k < s.size() && ((unsigned char)s[i + k] & 0xC0) == 0x80; };
  if (c0 >= 0xC2 && c0 <= 0xDF && cont(1)) {
    *width = 2;
    return ((c0 & 0x1Fu) << 6) | ((unsigned char)s[i + 1] & 0x3Fu);
  }
  if (c0 >= 0xE0 && c0 <= 0xEF && cont(1) && cont(2)) {
    uint32_t r = ((c0 & 0x0Fu) << 12) | (((unsigned char)s[i + 1] & 0x3Fu) << 6) |
                 ((unsigned char)s[i + 2] & 0x3Fu);
    if (r >= 0x800 && !(r >= 0xD800 && r <= 0xDFFF)) { *width = 3; return r; }
  }
  if (c0 >= 0xF0 && c0 <= 0xF4 && cont(1) && cont(2) && cont(3)) {
    uint32_t r = ((c0 & 0x07u) << 18) | (((unsigned char)s[i + 1] & 0x3Fu) << 12) |
                 (((unsigned char)s[i + 2] & 0x3Fu) << 6) | ((unsigned char)s[i + 3] & 0x3Fu);
    if (r >= 0x10000 && r <= 0x10FFFF) { *width = 4; return r; }
  }
  *width = 1;
  return 0xFFFD;
}

// strings.EqualFold(s, t) for an ASCII `t`. Under Go's unicode.SimpleFold the only non-ASCII
// runes whose fold orbit contains an ASCII letter are U+017F (ſ ~ s/S) and U+212A (K ~ k/K).
static bool fold_eq_ascii(uint32_t r, unsigned char t) {
  if (r == t) return true;
  unsigned char lt = (t >= 'A' && t <= 'Z') ? (unsigned char)(t + 32) : t;
  if (lt < 'a' || lt > 'z') return false;
  if (r < 0x80) {
    uint32_t lr = (r >= 'A' && r <= 'Z') ? r + 32 : r;
    return lr == lt;
  }
  if (r == 0x017F) return lt == 's';
  if (r == 0x212A) return lt == 'k';
  return false;
}

bool equal_fold_ascii(std::string_view s, std::string_view t) {
  size_t i = 0, j = 0;
  while (i < s.size()) {
    if (j >= t.size()) return false;
    size_t w;
    uint32_t r = decode_rune(s, i, &w);
    if (!fold_eq_ascii(r, (unsigned char)t[j])) return false;
    i += w;
    j++;
  }
  return j == t.size();
}

bool is_shared_filter(std::string_view filter) {  // topics.go:701-704
  bool hn;
  return equal_fold_ascii(isolate_particle(filter, 0, &hn), kSharePrefix);
}

static std::vector<std::string_view> split_slash(std::string_view s) {  // strings.Split(s, "/")
  std::vector<std::string_view> out;
  size_t b = 0;
  for (;;) {
    const size_t e = s.find('/', b);
    if (e == std::string_view::npos) {
      out.push_back(s.substr(b));
      return out;
    }
    out.push_back(s.substr(b, e - b));
    b = e + 1;
  }
}

bool match_topic(std::string_view filter, std::string_view topic,  // hooks/auth/ledger.go:90-118
                 std::vector<std::pair<uint32_t, uint32_t>>* elements) {
  const std::vector<std::string_view> fp = split_slash(filter), tp = split_slash(topic);
  if (elements) elements->clear();
  auto span = [&](std::string_view v) {
    return std::make_pair((uint32_t)(v.data() - topic.data()), (uint32_t)v.size());
  };
  for (size_t i = 0; i < fp.size(); i++) {
    if (i >= tp.size()) return false;  // ledger.go:95-98
    if (fp[i] == "+") {                // ledger.go:100-103
      if (elements) elements->push_back(span(tp[i]));
      continue;
    }
    if (fp[i] == "#") {  // ledger.go:105-109: the rest of the topic, joined
      if (elements) {
        const uint32_t b = (uint32_t)(tp[i].data() - topic.data());
        elements->push_back(std::make_pair(b, (uint32_t)topic.size() - b));
      }
      return true;
    }
    if (fp[i] != tp[i]) return false;  // ledger.go:111-114
  }
  return true;  // ledger.go:117
}

bool is_valid_filter(std::string_view filter, bool for_publish) {  // topics.go:707-745
  if (!for_publish && filter.empty()) return false;
  if (for_publish) {
    const size_t sl = std::char_traits<char>::length(kSysPrefix);
    if (filter.size() >= sl && equal_fold_ascii(filter.substr(0, sl), kSysPrefix)) return false;
    if (filter.find('+') != std::string_view::npos || filter.find('#') != std::string_view::npos)
      return false;
  }
  size_t wildhash = filter.find('#');
  if (wildhash != std::string_view::npos && wildhash != filter.size() - 1) return false;
  bool has_next;
  std::string_view prefix = isolate_particle(filter, 0, &has_next);
  if (!has_next && equal_fold_ascii(prefix, kSharePrefix)) return false;
  if (has_next && equal_fold_ascii(prefix, kSharePrefix)) {
    bool hn2;
    std::string_view group = isolate_particle(filter, 1, &hn2);
    if (!hn2) return false;
    if (group.find('+') != std::string_view::npos || group.find('#') != std::string_view::npos)
      return false;
  }
  return true;
}

TopicsIndex::TopicsIndex() : root_(new Particle()) {}  // topics.go:356-364

static Particle* new_particle(const std::string& key, Particle* parent) {  // topics.go:760-769
  Particle* p = new Particle();
  p->key = key;
  p->parent = parent;
  return p;
}

// topics.go:479-496
Particle* TopicsIndex::set(const std::string& topic, int d) {
  bool has_next = true;
  Particle* n = root_.get();
  while (has_next) {
    std::string key(isolate_particle(topic, d, &has_next));
    d++;
    Particle* p = n->get(key);
    if (!p) {
      p = new_particle(key, n);
      n->particles[key].reset(p);
    }
    n = p;
  }
  return n;
}

// topics.go:499-513
Particle* TopicsIndex::seek(const std::string& filter, int d) const {
  bool has_next = true;
  Particle* n = root_.get();
  while (has_next) {
    std::string key(isolate_particle(filter, d, &has_next));
    n = n->get(key);
    d++;
    if (!n) return nullptr;
  }
  return n;
}

// topics.go:516-522
void TopicsIndex::trim(Particle* n) {
  while (n->parent != nullptr && n->retain_path.empty() &&
         n->particles.size() + n->subscriptions.size() + n->shared_len() +
                 n->inline_subscriptions.size() == 0) {
    std::string key = n->key;
    n = n->parent;
    n->particles.erase(key);
  }
}

// topics.go:368-378
bool TopicsIndex::inline_subscribe(const InlineSubscription& s) {
  Particle* n = set(s.sub.filter, 0);
  bool existed = n->inline_subscriptions.count(s.sub.identifier) > 0;
  n->inline_subscriptions[s.sub.identifier] = s;
  return !existed;
}

// topics.go:382-397
bool TopicsIndex::inline_unsubscribe(int64_t id, const std::string& filter) {
  Particle* p = seek(filter, 0);
  if (!p) return false;
  p->inline_subscriptions.erase(id);
  if (p->inline_subscriptions.empty()) trim(p);
  return true;
}

// topics.go:401-419
bool TopicsIndex::subscribe(const std::string& client, const Subscription& s) {
  bool existed;
  bool hn;
  std::string prefix(isolate_particle(s.filter, 0, &hn));
  if (equal_fold_ascii(prefix, kSharePrefix)) {
    std::string group(isolate_particle(s.filter, 1, &hn));
    Particle* n = set(s.filter, 2);
    auto g = n->shared.find(group);
    existed = g != n->shared.end() && g->second.count(client) > 0;
    n->shared[group][client] = s;
  } else {
    Particle* n = set(s.filter, 0);
    existed = n->subscriptions.count(client) > 0;
    n->subscriptions[client] = s;
  }
  return !existed;
}

// topics.go:423-448
bool TopicsIndex::unsubscribe(const std::string& filter, const std::string& client) {
  int d = 0;
  bool hn;
  std::string prefix(isolate_particle(filter, 0, &hn));
  bool share_sub = equal_fold_ascii(prefix, kSharePrefix);
  if (share_sub) d = 2;
  Particle* p = seek(filter, d);
  if (!p) return false;
  if (share_sub) {
    std::string group(isolate_particle(filter, 1, &hn));
    // SharedSubscriptions.Delete (topics.go:132-139)
    auto g = p->shared.find(group);
    if (g != p->shared.end()) {
      g->second.erase(client);
      if (g->second.empty()) p->shared.erase(g);
    }
  } else {
    p->subscriptions.erase(client);
  }
  trim(p);
  return true;
}

bool TopicsIndex::retained_get(const std::string& topic, RetainedPacket* out) const {
  auto it = retained_.find(topic);
  if (it == retained_.end()) return false;
  if (out) *out = it->second;
  return true;
}

// topics.go:453-476
int64_t TopicsIndex::retain_message(const std::string& topic, const RetainedPacket& pk) {
  Particle* n = set(topic, 0);
  if (pk.payload_len > 0) {
    n->retain_path = topic;
    retained_[topic] = pk;
    return 1;
  }
  int64_t out = 0;
  auto it = retained_.find(topic);
  if (it != retained_.end() && it->second.payload_len > 0 && it->second.retain) out = -1;
  n->retain_path.clear();
  retained_.erase(topic);  // [MQTT-3.3.1-6] [MQTT-3.3.1-7]
  trim(n);
  return out;
}

// topics.go:525-527
std::vector<RetainedPacket> TopicsIndex::messages(const std::string& filter, Counters* c) const {
  std::vector<RetainedPacket> pks;
  if (c) {
    bool hn = true;
    for (int d = 0; hn; d++) isolate_particle(filter, d, &hn), c->levels++;
  }
  scan_messages(filter, 0, root_.get(), pks, c);
  if (c) c->out_rows += pks.size();
  return pks;
}

// topics.go:530-579
void TopicsIndex::scan_messages(const std::string& filter, int d, const Particle* n,
                                std::vector<RetainedPacket>& pks, Counters* c) const {
  if (filter.empty() || retained_.empty()) return;
  if (filter.find('#') == std::string::npos && filter.find('+') == std::string::npos) {
    RetainedPacket pk;
    if (retained_get(filter, &pk)) pks.push_back(pk);
    return;
  }
  bool has_next;
  std::string key(isolate_particle(filter, d, &has_next));
  if (key == "+" || key == "#" || d == -1) {
    if (c) c->lookups += n->particles.size();  // getAll copies every child (topics.go:792-800)
    for (auto& kv : n->particles) {
      const Particle* adjacent = kv.second.get();
      if (d == 0 && adjacent->key == kSysPrefix) continue;
      if (!has_next) {
        if (!adjacent->retain_path.empty()) {
          RetainedPacket pk;
          if (retained_get(adjacent->retain_path, &pk)) pks.push_back(pk);
        }
      }
      if (has_next || (d >= 0 && key == "#")) scan_messages(filter, d + 1, adjacent, pks, c);
    }
    return;
  }
  if (c) c->lookups++;
  if (const Particle* p = n->get(key)) {
    if (has_next) {
      scan_messages(filter, d + 1, p, pks, c);
      return;
    }
    RetainedPacket pk;
    if (retained_get(p->retain_path, &pk)) pks.push_back(pk);  // Q6: no emptiness check
  }
}

// topics.go:583-590
Subscribers TopicsIndex::subscribers(const std::string& topic, Counters* c) const {
  Subscribers subs;
  if (c) {
    bool hn = true;
    for (int d = 0; hn && !topic.empty(); d++) isolate_particle(topic, d, &hn), c->levels++;
  }
  scan_subscribers(topic, 0, root_.get(), subs, c);
  if (c) {
    for (auto& kv : subs.subscriptions)
      c->out_rows += kv.second.has_identifiers ? kv.second.identifiers.size() : 1;
    for (auto& kv : subs.shared) c->out_rows += kv.second.size();
    c->out_rows += subs.inline_subscriptions.size();
  }
  return subs;
}

// topics.go:593-628
void TopicsIndex::scan_subscribers(const std::string& topic, int d, const Particle* n,
                                   Subscribers& subs, Counters* c) const {
  if (topic.empty()) return;
  bool has_next;
  std::string key(isolate_particle(topic, d, &has_next));
  const std::string part_keys[2] = {key, "+"};
  for (const std::string& part_key : part_keys) {
    if (c) c->lookups++;
    if (const Particle* p = n->get(part_key)) {  // [MQTT-3.3.2-3]
      if (has_next) {
        scan_subscribers(topic, d + 1, p, subs, c);
      } else {
        gather_subscriptions(topic, p, subs, c);
        gather_shared(p, subs, c);
        gather_inline(p, subs, c);
        if (c) c->lookups++;
        const Particle* wild = p->get("#");
        if (wild && part_key != "+") {
          gather_subscriptions(topic, wild, subs, c);  // filter/# matches filter (4.7.1.2)
          gather_shared(wild, subs, c);
          gather_inline(p, subs, c);  // Q2: the literal particle's inline subs, again
        }
      }
    }
  }
  if (c) c->lookups++;
  if (const Particle* p = n->get("#")) {
    gather_subscriptions(topic, p, subs, c);
    gather_shared(p, subs, c);
    gather_inline(p, subs, c);
  }
}

// topics.go:631-648
void TopicsIndex::gather_subscriptions(const std::string& topic, const Particle* p,
                                       Subscribers& subs, Counters* c) const {
  if (c) c->scanned += p->subscriptions.size();
  for (auto& kv : p->subscriptions) {
    const Subscription& sub = kv.second;
    // [MQTT-4.7.1-1] [MQTT-4.7.1-2]: no top-level wildcard delivery of $ topics (Q3)
    if (!sub.filter.empty() && topic[0] == '$' && (sub.filter[0] == '+' || sub.filter[0] == '#'))
      continue;
    auto it = subs.subscriptions.find(kv.first);
    Subscription cls = it == subs.subscriptions.end() ? sub : it->second;
    subs.subscriptions[kv.first] = cls.merge(sub);
  }
}

// topics.go:651-665
void TopicsIndex::gather_shared(const Particle* p, Subscribers& subs, Counters* c) const {
  if (c) c->scanned += p->shared_len();
  for (auto& g : p->shared)
    for (auto& kv : g.second) subs.shared[kv.second.filter][kv.first] = kv.second;
}

// topics.go:668-676
void TopicsIndex::gather_inline(const Particle* p, Subscribers& subs, Counters* c) const {
  if (c) c->scanned += p->inline_subscriptions.size();
  for (auto& kv : p->inline_subscriptions) subs.inline_subscriptions[kv.first] = kv.second;
}

static size_t count_particles(const Particle* p) {
  size_t n = 1;
  for (auto& kv : p->particles) n += count_particles(kv.second.get());
  return n;
}
size_t TopicsIndex::particle_count() const { return count_particles(root_.get()) - 1; }

// topics.go:320-333; the Go pick is the first client of each group in (random) map order —
// here the first in sorted order, which is one of the orders Go may produce.
void select_shared_first(Subscribers& s) {
  s.shared_selected.clear();
  for (auto& g : s.shared) {
    for (auto& kv : g.second) {
      auto it = s.shared_selected.find(kv.first);
      Subscription cls = it == s.shared_selected.end() ? kv.second : it->second;
      s.shared_selected[kv.first] = cls.merge(kv.second);
      break;
    }
  }
}

// topics.go:338-347
void merge_shared_selected(Subscribers& s) {
  for (auto& kv : s.shared_selected) {
    auto it = s.subscriptions.find(kv.first);
    Subscription cls = it == s.subscriptions.end() ? kv.second : it->second;
    s.subscriptions[kv.first] = cls.merge(kv.second);
  }
}

}  // namespace oracle
