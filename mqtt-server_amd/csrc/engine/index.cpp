// Host side of the engine: incremental updates of the flat trie image (index.h).
// Each public operation restates the reference semantics it replaces (topics.go:368-522).
#include "index.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>

namespace mq {

// ---- HashU64 ------------------------------------------------------------------------------------
void HashU64::rehash(size_t cap) {
  size_t c = 16;
  while (c < cap) c <<= 1;
  std::vector<uint64_t> ok;
  std::vector<uint32_t> ov;
  ok.swap(keys_);
  ov.swap(vals_);
  keys_.assign(c, kEmpty);
  vals_.assign(c, 0);
  n_ = tombs_ = 0;
  for (size_t i = 0; i < ok.size(); i++)
    if (ok[i] != kEmpty && ok[i] != kTomb) put(ok[i], ov[i]);
}

bool HashU64::get(uint64_t k, uint32_t* v) const {
  size_t m = keys_.size() - 1, i = slot(k);
  for (;;) {
    uint64_t x = keys_[i];
    if (x == kEmpty) return false;
    if (x == k) {
      *v = vals_[i];
      return true;
    }
    i = (i + 1) & m;
  }
}

void HashU64::put(uint64_t k, uint32_t v) {
  if ((n_ + tombs_ + 1) * 2 > keys_.size()) rehash(n_ * 4 > keys_.size() ? keys_.size() * 2 : keys_.size());
  size_t m = keys_.size() - 1, i = slot(k), tomb = SIZE_MAX;
  for (;;) {
    uint64_t x = keys_[i];
    if (x == k) {
      vals_[i] = v;
      return;
    }
    if (x == kTomb && tomb == SIZE_MAX) tomb = i;
    if (x == kEmpty) {
      if (tomb != SIZE_MAX) {
        i = tomb;
        tombs_--;
      }
      keys_[i] = k;
      vals_[i] = v;
      n_++;
      return;
    }
    i = (i + 1) & m;
  }
}

void HashU64::build_parallel(const uint64_t* keys, const uint32_t* vals, size_t n, unsigned threads) {
  rehash(std::max<size_t>(n * 2 + 16, 16));
  const size_t m = keys_.size() - 1;
  parallel_for(n, threads, [&](size_t b, size_t e) {
    for (size_t j = b; j < e; j++) {
      size_t i = slot(keys[j]);
      for (;;) {
        uint64_t expect = kEmpty;
        if (__atomic_compare_exchange_n(&keys_[i], &expect, keys[j], false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
          vals_[i] = vals[j];
          break;
        }
        i = (i + 1) & m;
      }
    }
  });
  n_ = n;
  tombs_ = 0;
}

bool HashU64::erase(uint64_t k) {
  size_t m = keys_.size() - 1, i = slot(k);
  for (;;) {
    uint64_t x = keys_[i];
    if (x == kEmpty) return false;
    if (x == k) {
      keys_[i] = kTomb;
      n_--;
      tombs_++;
      return true;
    }
    i = (i + 1) & m;
  }
}

// ---- string helpers -------------------------------------------------------------------------

// strings.EqualFold(s, "$SHARE") (topics.go:407, Q9). Go decodes s rune by rune (invalid
// bytes become U+FFFD); under unicode.SimpleFold the runes equal to the ASCII target are the
// ASCII letter in either case, plus U+017F (LATIN SMALL LETTER LONG S, UTF-8 C5 BF) for 'S'.
bool is_share_prefix(std::string_view s) {
  static const char* up = "$SHARE";
  size_t i = 0;
  for (int j = 0; j < 6; j++) {
    if (i >= s.size()) return false;
    unsigned char c = (unsigned char)s[i];
    if (c == 0xC5 && i + 1 < s.size() && (unsigned char)s[i + 1] == 0xBF) {  // U+017F
      if (up[j] != 'S') return false;
      i += 2;
      continue;
    }
    if (c >= 0x80) return false;
    unsigned char lc = (c >= 'A' && c <= 'Z') ? (unsigned char)(c + 32) : c;
    unsigned char lt = (up[j] >= 'A' && up[j] <= 'Z') ? (unsigned char)(up[j] + 32) : (unsigned char)up[j];
    if (lc != lt) return false;
    i++;
  }
  return i == s.size();
}

// isolateParticle(filter, d) for every d from `d` on (topics.go:679-698): the segments
// from index d, or — when d is past the last '/' — the last segment alone.
void Index::path_of(std::string_view filter, int d, std::vector<std::string_view>& out) {
  out.clear();
  thread_local std::vector<std::string_view> segs;
  segs.clear();
  size_t s = 0;
  for (;;) {
    size_t e = filter.find('/', s);
    if (e == std::string_view::npos) {
      segs.push_back(filter.substr(s));
      break;
    }
    segs.push_back(filter.substr(s, e - s));
    s = e + 1;
  }
  if ((size_t)d < segs.size())
    out.assign(segs.begin() + d, segs.end());
  else
    out.push_back(segs.back());
}

std::string_view segment_at(std::string_view filter, int d) {  // isolateParticle value
  size_t s = 0;
  for (int i = 0;; i++) {
    size_t e = filter.find('/', s);
    if (e == std::string_view::npos) return filter.substr(s);
    if (i == d) return filter.substr(s, e - s);
    s = e + 1;
  }
}

uint64_t StrTable::hash(std::string_view s) {
  uint64_t h = 0xcbf29ce484222325ull ^ s.size();
  for (unsigned char c : s) h = (h ^ c) * 0x100000001b3ull;
  return mix64(h);
}

void StrTable::grow() {
  slots_.assign(slots_.size() * 2, kNone);
  const size_t m = slots_.size() - 1;
  for (uint32_t id = 0; id < hashes_.size(); id++) {
    size_t i = hashes_[id] & m;
    while (slots_[i] != kNone) i = (i + 1) & m;
    slots_[i] = id;
  }
}

uint32_t StrTable::find(std::string_view s) const {
  const uint64_t h = hash(s);
  const size_t m = slots_.size() - 1;
  for (size_t i = h & m;; i = (i + 1) & m) {
    const uint32_t id = slots_[i];
    if (id == kNone) return kNone;
    if (hashes_[id] == h && at(id) == s) return id;
  }
}

uint32_t StrTable::intern(std::string_view s) {
  const uint64_t h = hash(s);
  const size_t m = slots_.size() - 1;
  size_t i = h & m;
  for (;; i = (i + 1) & m) {
    const uint32_t id = slots_[i];
    if (id == kNone) break;
    if (hashes_[id] == h && at(id) == s) return id;
  }
  const uint32_t id = (uint32_t)hashes_.size();
  arena_.insert(arena_.end(), s.begin(), s.end());
  offs_.push_back(arena_.size());
  hashes_.push_back(h);
  slots_[i] = id;
  if (hashes_.size() * 2 > slots_.size()) grow();
  return id;
}

uint32_t Index::intern_str(std::string_view s) { return strs_.intern(s); }

// ---- sharding ------------------------------------------------------------------
uint32_t Index::shard_hash(std::string_view key) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (unsigned char c : key) h = (h ^ c) * 0x100000001b3ull;
  return (uint32_t)(mix64(h ^ key.size()) >> 32);
}

void Index::set_shard(uint32_t shard, uint32_t n_shards) {
  shard_ = shard;
  n_shards_ = n_shards ? n_shards : 1;
  if (n_shards_ > 1) {
    xinfo.grow_to(nh_.size(), XInfo{kNone, 0, 0});
    for (uint32_t n = 1; n < nh_.size(); n++)
      if (nh_[n].live) set_rank(n, walk.h[n].parent_flags & kParentMask, strs_.at(nh_[n].str));
  }
}

// rank key of node n from its parent's (layout.h XInfo)
void Index::set_rank(uint32_t n, uint32_t parent, std::string_view seg, bool mark) {
  const XInfo& P = xinfo.h[parent];
  XInfo x{kNone, P.deep, P.rank};
  const uint32_t d = nh_[n].depth;  // 1-based
  const uint64_t code = seg == "+" ? 2 : (seg == "#" ? 3 : 1);
  if (d <= 32) x.rank |= code << (64 - 2 * d);
  else x.deep = 1;
  if (mark) xinfo.at_w(n) = x;
  else xinfo.h[n] = x;
}

// The order of two deep paths whose rank keys tie (layout.h DeepTail): filter fid's codes for its
// levels 33.., kept for the device's tie-break (merge.hip deep_before). Entries are overwritten
// when a filter id is seen again (a filter id names one filter while it is subscribed).
size_t Index::deep_find(uint32_t fid) const {
  const size_t mask = deep.size() - 1;
  size_t sl = mix64(fid) & mask;
  while (deep.h[sl].fid != kNone && deep.h[sl].fid != fid) sl = (sl + 1) & mask;
  return sl;
}

void Index::deep_rebuild(size_t slots) {
  std::vector<DeepTail> old;
  old.swap(deep.h);
  std::vector<uint32_t> codes;
  codes.swap(deep_codes.h);
  deep.h.assign(slots, DeepTail{kNone, 0, 0, 0});
  deep_codes.h.clear();
  for (const DeepTail& e : old) {
    if (e.fid == kNone || e.fid == kDeepTomb) continue;
    const uint32_t off = (uint32_t)deep_codes.h.size();
    deep_codes.h.insert(deep_codes.h.end(), codes.begin() + e.off, codes.begin() + e.off + e.n);
    deep.h[deep_find(e.fid)] = DeepTail{e.fid, off, e.n, 0};
  }
  n_deep_ = n_deep_live_;
  deep_garbage_ = 0;
  deep.epoch++;
  deep.all_dirty = true;
  deep_codes.epoch++;
  deep_codes.all_dirty = true;
  version_++;
}

void Index::note_deep(uint32_t fid, const uint32_t* segs, uint32_t depth) {
  if (depth <= 32 || fid == kNone) return;
  deep_refs_[fid]++;
  const uint32_t n = (depth - 32 + 15) / 16;
  thread_local std::vector<uint32_t> w;
  w.assign(n, 0u);
  for (uint32_t i = 32; i < depth; i++) {
    const uint32_t code = segs[i] == 0 ? 2u : (segs[i] == 1 ? 3u : 1u);  // '+' 2, '#' 3, literal 1
    const uint32_t j = i - 32;
    w[j / 16] |= code << (30 - 2 * (j % 16));
  }
  if (deep.size()) {
    const DeepTail& e = deep.h[deep_find(fid)];
    if (e.fid == fid && e.n == n && std::equal(w.begin(), w.end(), deep_codes.h.begin() + e.off)) return;
  }
  if ((n_deep_ + 1) * 2 > deep.size()) {  // at most half full (tombstones count): rehash
    size_t slots = 64;
    while (slots < 4 * (size_t)(n_deep_live_ + 1)) slots *= 2;
    deep_rebuild(slots);
  }
  const size_t sl = deep_find(fid);
  if (deep.h[sl].fid == kNone) {
    n_deep_++;
    n_deep_live_++;
  } else {
    deep_garbage_ += deep.h[sl].n;  // (an id reused for another deep path while still referenced)
  }
  const uint32_t off = (uint32_t)deep_codes.size();
  deep_codes.grow_to(off + n, 0u);
  for (uint32_t k = 0; k < n; k++) deep_codes.at_w(off + k) = w[k];
  deep.at_w(sl) = DeepTail{fid, off, n, 0};
  version_++;
}

void Index::deep_unref(uint32_t fid) {
  auto it = deep_refs_.find(fid);
  if (it == deep_refs_.end() || --it->second) return;
  deep_refs_.erase(it);
  if (!deep.size()) return;
  const size_t sl = deep_find(fid);
  if (deep.h[sl].fid != fid) return;
  deep_garbage_ += deep.h[sl].n;
  deep.at_w(sl) = DeepTail{kDeepTomb, 0, 0, 0};  // (probes for other ids pass over it)
  n_deep_live_--;
  version_++;
  if (deep_garbage_ > 4096 && deep_garbage_ > deep_codes.size() / 2) deep_rebuild(deep.size());
}

void Index::note_deep_node(uint32_t n, uint32_t fid) {
  if (nh_[n].depth <= 32) return;
  thread_local std::vector<uint32_t> pa;
  pa.resize(nh_[n].depth);
  int la;
  path_strs(n, pa.data(), &la);
  note_deep(fid, pa.data(), (uint32_t)la);
}

// Qos | NoLocal of partner `p` (a node of this shard, or kForeign | fid) of `client`'s slot
uint32_t Index::partner_meta(uint32_t p, uint32_t client) const {
  uint32_t i = kNone;
  if (p & kForeign) {
    if (!fsub_pos_.get((uint64_t)(p & ~kForeign) << 32 | client, &i))
      throw std::logic_error("partner_meta: foreign partner missing");
    return fsubs_[i].meta;
  }
  if (!sub_pos_.get((uint64_t)p << 32 | client, &i))  // partners are symmetric
    throw std::logic_error("flush_merge: partner subscription missing");
  return subs.m.h[i].meta & (kMetaQos | kMetaNoLocal);
}

// ---- construction ----------------------------------------------------------------------------
Index::Index(uint64_t expected_subs, uint64_t expected_nodes) {
  intern_str("+");
  intern_str("#");
  size_t cap = 1024;
  uint64_t want = expected_nodes ? expected_nodes : expected_subs * 3;
  while (cap < want * 2) cap <<= 1;
  edges.h.assign(cap, EdgeSlot{0, 0, kEdgeEmpty, kNone, kNone, kNone});
  edges.epoch++;
  if (want) {
    walk.h.reserve(want);
    lists.h.reserve(want);
    msg.h.reserve(want);
    nh_.reserve(want);
    sub_pos_.reserve(expected_subs);
    subs.m.h.reserve(expected_subs + expected_subs / 2);
  }
  // root particle (topics.go:359-362)
  nh_.push_back(NodeHost{});
  nh_[0].live = true;
  walk.grow_to(1, NodeWalk{kNone, kNone, kParentMask, kNone});
  lists.grow_to(1, kEmptyLists);
  inls.grow_to(1, NodeInl{0, 0});
  msg.grow_to(1, NodeMsg{});
  seginfo.grow_to(1, SegInfo{0, 0});
  segbytes.grow_to(1, 0);
  subp_.resize(1, PartList{0, 0, 0});
  parts.m.grow_to(1, 0);
  mpart.m.grow_to(1, MergePart{kNone, 0});
  npair.grow_to(1, NodePair{0, kNone, 0, 0});
  pent.m.grow_to(1, PairEnt{kNone, 0, 0, 0});
  plist.m.grow_to(1, PairSlot{0, 0, 0, 0});
}

// ---- edge table -------------------------------------------------------------------------------
uint32_t Index::find_child(uint32_t parent, const SegKey& k, std::string_view seg) const {
  const uint64_t m = edges.size() - 1;
  uint64_t i = edge_hash(parent, k) & m;
  for (;;) {
    const EdgeSlot& e = edges.h[i];
    if (e.parent == kEdgeEmpty) return kNone;
    if (e.parent == parent && e.k0 == k.k0 && e.k1 == k.k1) {
      if (!seg_is_long(k)) return e.child;
      const SegInfo& si = seginfo.h[walk.h[e.child].seg];
      if (si.len == seg.size() && memcmp(&segbytes.h[si.off], seg.data(), si.len) == 0) return e.child;
    }
    i = (i + 1) & m;
  }
}

void Index::edge_rehash(size_t cap, unsigned threads) {
  std::vector<EdgeSlot> old, fresh;
  reserve_resident(fresh, cap, threads);
  old.swap(edges.h);
  edges.h.swap(fresh);
  edges.h.assign(cap, EdgeSlot{0, 0, kEdgeEmpty, kNone, kNone, kNone});
  edges.epoch++;
  edges.all_dirty = true;
  n_edges_ = n_tombs_ = 0;
  for (const EdgeSlot& e : old)
    if (e.parent != kEdgeEmpty && e.parent != kEdgeTomb) edge_insert(e.parent, SegKey{e.k0, e.k1}, e.child, e.plus, e.hash);
}

void Index::edge_walk_sync(uint32_t n) {
  if (n == kRoot) return;  // the walk reads the root's NodeWalk itself
  const uint32_t p = walk.h[n].parent_flags & kParentMask;
  const SegKey& k = nh_[n].key;
  const uint64_t m = edges.size() - 1;
  for (uint64_t i = edge_hash(p, k) & m;; i = (i + 1) & m) {
    EdgeSlot& e = edges.h[i];
    if (e.parent == kEdgeEmpty) throw std::logic_error("edge_walk_sync: particle without an edge");
    if (e.parent == p && e.child == n) {
      e.plus = walk.h[n].plus_child;
      e.hash = walk.h[n].hash_child;
      edges.mark(i);
      return;
    }
  }
}

void Index::edge_insert(uint32_t parent, const SegKey& k, uint32_t child, uint32_t plus, uint32_t hash) {
  if ((n_edges_ + n_tombs_ + 1) * edge_load_at(edges.size()) > edges.size()) {
    size_t cap = edges.size();
    if ((n_edges_ + 1) * 2 * edge_load_at(cap) > cap) cap <<= 1;  // double unless mostly tombstones
    while ((n_edges_ + 1) * edge_load_at(cap) > cap) cap <<= 1;   // (the bound was lowered)
    edge_rehash(cap);
  }
  const uint64_t m = edges.size() - 1;
  uint64_t i = edge_hash(parent, k) & m;
  for (;;) {
    EdgeSlot& e = edges.h[i];
    if (e.parent == kEdgeEmpty || e.parent == kEdgeTomb) {
      if (e.parent == kEdgeTomb) n_tombs_--;
      e = EdgeSlot{k.k0, k.k1, parent, child, plus, hash};
      edges.mark(i);
      n_edges_++;
      return;
    }
    i = (i + 1) & m;
  }
}

// Backward-shift deletion: the slots after the erased one that probed past it move back, so the
// table never holds tombstones — churn (unsubscribe + subscribe) does not lengthen the walk's
// probe chains (a tombstone is probed like a full slot) nor force a whole-table rehash and upload.
void Index::edge_erase(uint32_t parent, const SegKey& k, uint32_t child) {
  const uint64_t m = edges.size() - 1;
  uint64_t i = edge_hash(parent, k) & m;
  for (;;) {
    const EdgeSlot& e = edges.h[i];
    if (e.parent == kEdgeEmpty) return;
    if (e.parent == parent && e.child == child) break;
    i = (i + 1) & m;
  }
  n_edges_--;
  for (uint64_t j = (i + 1) & m;; j = (j + 1) & m) {
    const EdgeSlot& e = edges.h[j];
    if (e.parent == kEdgeEmpty) break;
    if (e.parent == kEdgeTomb) continue;  // (none are made; one would stay, occupied)
    const uint64_t h = edge_hash(e.parent, SegKey{e.k0, e.k1}) & m;
    // the entry at j may move to the hole at i iff its home is not cyclically in (i, j]
    const bool stays = i <= j ? (h > i && h <= j) : (h > i || h <= j);
    if (stays) continue;
    edges.at_w(i) = e;
    i = j;
  }
  edges.at_w(i).parent = kEdgeEmpty;
}

// ---- nodes ---------------------------------------------------------------------------------------
template <class T, class Rec>
void Index::list_push(SlabPool<T>& pool, uint32_t& off, uint32_t& cnt, uint32_t& cap, const Rec& r) {
  constexpr bool kShared = std::is_same<T, ShrRec>::value;  // (live host results point into shr)
  if (cnt + 1 > cap) {
    uint32_t nc = cap ? cap * 2 : 1;
    if constexpr (kShared) guard_growth(pool.m, pool.m.size() + nc, retired_shr_);
    uint32_t no = pool.alloc(nc);
    for (uint32_t i = 0; i < cnt; i++) pool.m.at_w(no + i) = pool.m.h[off + i];
    if constexpr (kShared) retire(1, off, cap);
    else pool.release(off, cap);
    off = no;
    cap = nc;
  }
  pool.m.at_w(off + cnt) = r;
  cnt++;
  pool.live++;
}

uint32_t Index::new_node(uint32_t parent, std::string_view seg, const SegKey& k) {
  uint32_t id;
  if (!free_nodes_.empty()) {
    id = free_nodes_.back();
    free_nodes_.pop_back();
  } else {
    id = (uint32_t)nh_.size();
    nh_.push_back(NodeHost{});
    walk.grow_to(id + 1, NodeWalk{kNone, kNone, 0, kNone});
    lists.grow_to(id + 1, kEmptyLists);
    inls.grow_to(id + 1, NodeInl{0, 0});
    msg.grow_to(id + 1, NodeMsg{});
    npair.grow_to(id + 1, NodePair{0, kNone, 0, 0});
  }
  NodeHost& h = nh_[id];
  h = NodeHost{};
  h.key = k;
  h.str = intern_str(seg);
  h.depth = (uint16_t)(nh_[parent].depth + 1);
  h.seg0 = parent == kRoot ? h.str : nh_[parent].seg0;
  h.live = true;
  max_depth_ = std::max<uint32_t>(max_depth_, h.depth);

  uint32_t flags = 0;
  if (h.str == 0) flags |= kFlagPlusKey;
  if (parent == kRoot) {
    if (!seg.empty() && (seg[0] == '+' || seg[0] == '#')) flags |= kFlagSeg0Wild;
  } else {
    flags |= walk.h[parent].parent_flags & kFlagSeg0Wild;
  }
  uint32_t segref = kNone;
  if (seg_is_long(k)) {
    auto it = long_segs_.find(std::string(seg));
    if (it == long_segs_.end()) {
      segref = (uint32_t)seginfo.size();
      uint32_t off = (uint32_t)segbytes.size();
      segbytes.grow_to(off + seg.size(), 0);
      memcpy(&segbytes.h[off], seg.data(), seg.size());
      seginfo.grow_to(segref + 1, SegInfo{off, (uint32_t)seg.size()});
      long_segs_.emplace(std::string(seg), segref);
    } else {
      segref = it->second;
    }
  }
  walk.at_w(id) = NodeWalk{kNone, kNone, parent | flags, segref};
  NodeLists L = kEmptyLists;
  L.flags = flags & kFlagSeg0Wild;
  lists.at_w(id) = L;
  NodeMsg M{};
  M.parent = parent;
  M.flags = (parent == kRoot && seg == "$SYS") ? kChildSys : 0u;
  msg.at_w(id) = M;

  if (sharded()) {
    xinfo.grow_to(id + 1, XInfo{kNone, 0, 0});
    set_rank(id, parent, seg);
  }
  edge_insert(parent, k, id);
  if (h.str == 0) walk.at_w(parent).plus_child = id;
  if (h.str == 1) walk.at_w(parent).hash_child = id;
  if (h.str <= 1) edge_walk_sync(parent);
  NodeMsg& pm = msg.at_w(parent);
  h.child_pos = pm.child_cnt;
  msg.h[id].child_pos = pm.child_cnt;
  list_push(children, pm.child_off, pm.child_cnt, nh_[parent].child_cap,
            ChildRec{id, 0, 0, M.flags, 0});
  child_rec_sync(parent);  // the parent's slab may have moved
  nh_[parent].n_children++;
  n_live_nodes_++;
  n_wild_nodes_ += h.str <= 1;
  return id;
}

// A live retained topic at n counts in below_live of every strict ancestor (root included).
void Index::add_below_live(uint32_t n, int delta) {
  for (uint32_t a = n; a != kRoot;) {
    a = msg.h[a].parent;
    msg.at_w(a).below_live += (uint32_t)delta;
  }
}

void Index::child_rec_sync(uint32_t n) {
  if (n == kRoot) return;
  const NodeMsg& M = msg.h[n];
  const uint32_t p = M.parent;
  children.m.at_w(msg.h[p].child_off + M.child_pos) =
      ChildRec{n, M.child_off, M.child_cnt, M.flags, M.handle};
}

void Index::remove_node(uint32_t n) {
  NodeHost& h = nh_[n];
  uint32_t p = walk.h[n].parent_flags & kParentMask;
  edge_erase(p, h.key, n);
  if (h.str == 0) walk.at_w(p).plus_child = kNone;
  if (h.str == 1) walk.at_w(p).hash_child = kNone;
  if (h.str <= 1) edge_walk_sync(p);
  NodeMsg& pm = msg.at_w(p);
  const ChildRec last = children.m.h[pm.child_off + pm.child_cnt - 1];
  children.m.at_w(pm.child_off + h.child_pos) = last;
  nh_[last.node].child_pos = h.child_pos;
  msg.at_w(last.node).child_pos = h.child_pos;
  pm.child_cnt--;
  children.live--;
  child_rec_sync(p);
  nh_[p].n_children--;
  // release the node's (empty) slabs
  retire(0, lists.h[n].sub_off, h.sub_cap);
  retire(1, lists.h[n].shr_off, h.shr_cap);
  inl.release(inls.h[n].off, h.inl_cap);
  children.release(msg.h[n].child_off, h.child_cap);
  merge_release(n);
  walk.at_w(n) = NodeWalk{kNone, kNone, 0, kNone};
  lists.at_w(n) = kEmptyLists;
  if (inls.h[n].cnt || inls.h[n].off) inls.at_w(n) = NodeInl{0, 0};
  msg.at_w(n) = NodeMsg{};
  if (sharded()) {
    if (xinfo.h[n].fid != kNone && h.depth > 32) deep_unref(xinfo.h[n].fid);
    xinfo.at_w(n) = XInfo{kNone, 0, 0};
  }
  n_wild_nodes_ -= h.str <= 1;
  h = NodeHost{};
  free_nodes_.push_back(n);
  n_live_nodes_--;
}

uint32_t Index::set(std::string_view filter, int d) {  // topics.go:479-496
  thread_local std::vector<std::string_view> path;
  path_of(filter, d, path);
  uint32_t n = kRoot;
  for (std::string_view seg : path) {
    SegKey k = seg_key((const uint8_t*)seg.data(), (uint32_t)seg.size());
    uint32_t c = find_child(n, k, seg);
    if (c == kNone) c = new_node(n, seg, k);
    n = c;
  }
  return n;
}

uint32_t Index::seek(std::string_view filter, int d) const {  // topics.go:499-513
  thread_local std::vector<std::string_view> path;
  path_of(filter, d, path);
  uint32_t n = kRoot;
  for (std::string_view seg : path) {
    SegKey k = seg_key((const uint8_t*)seg.data(), (uint32_t)seg.size());
    n = find_child(n, k, seg);
    if (n == kNone) return kNone;
  }
  return n;
}

void Index::trim(uint32_t n) {  // topics.go:516-522
  while (n != kRoot && !nh_[n].retain_path && nh_[n].n_children == 0 && sub_count(n) == 0 &&
         lists.h[n].shr_cnt == 0 && inls.h[n].cnt == 0) {
    uint32_t p = walk.h[n].parent_flags & kParentMask;
    remove_node(n);
    n = p;
  }
}

// ---- subscription lists ----------------------------------------------------------------------------
// A slot is the SubRec plus its partner list; they always move together, and the
// (node, client) -> slot map follows. A move changes this node's device merge records (its
// partner links sit at slot positions, its pair lists name slots); the partners' records name
// this node and the subscription's Qos / NoLocal, not its position, so they stay as they are.
void Index::move_slot(uint32_t n, uint32_t from, uint32_t to, bool mark) {
  const SubRec r = subs.m.h[from];
  subs.m.at_w(to) = r;
  subp_[to] = subp_[from];
  sub_pos_.put((uint64_t)n << 32 | r.client, to);
  if (mark) {
    merge_dirty_slot(n, from);
    merge_dirty_slot(n, to);
  }
}

void Index::merge_release(uint32_t n) {
  NodeHost& h = nh_[n];
  const NodePair& P = npair.h[n];
  auto it = minc_.find(n);
  if (it != minc_.end()) {  // slabs the in-place updates allocated outside the base slabs
    for (const MergeInc::Slot& sl : it->second.slot)
      if (sl.mp_cap && !(sl.mp_cap & kPairBase)) {
        mpart.release(sl.mp_off, sl.mp_cap);
        mpart.live -= sl.mp_cap;
      }
    if (P.ent_mask != kNone)
      for (uint32_t i = 0; i <= P.ent_mask; i++) {
        const PairEnt& e = pent.m.h[P.ent_off + i];
        if (e.h != kNone && !(e.cap & kPairBase)) plist.release(e.off, e.cap);
      }
    minc_.erase(it);
  }
  if (h.mpart_cap) {
    mpart.release(h.mpart_off, h.mpart_cap);
    mpart.live -= h.mpart_cap;
  }
  h.mpart_off = h.mpart_cap = 0;
  if (P.ent_mask != kNone) {
    pent.live -= P.n_lists;
    uint32_t links = 0;
    for (uint32_t i = 0; i <= P.ent_mask; i++)
      if (pent.m.h[P.ent_off + i].h != kNone) links += pent.m.h[P.ent_off + i].cnt;
    plist.live -= links;
    pent.release(P.ent_off, h.pent_cap);
    if (h.plist_cap) plist.release(P.list_off, h.plist_cap);
  }
  h.pent_cap = h.plist_cap = 0;
  if (P.ent_mask != kNone || P.n_lists) set_pair_header(n, NodePair{0, kNone, 0, 0});
}

void Index::flush_merge() {
  if (mref.size() < subs.m.size()) mref.grow_to(subs.m.size(), MergeRef{0, 0});
  for (uint32_t n : merge_dirty_) {
    merge_dirty_flag_[n] = 0;
    auto it = minc_.find(n);
    // in place while the base slabs' unused records stay below the ones in use
    if (it != minc_.end() && nh_[n].live && it->second.garbage <= 2 * it->second.links + 4096) {
      merge_patch(n, it->second);
      continue;
    }
    merge_release(n);
    if (nh_[n].live) merge_rebuild(n);
  }
  merge_dirty_.clear();
}

// The node's merge records from scratch: every may-merge slot's partner links (one base slab),
// and the pair block — a hash table of partner nodes, each with the list of slots whose client
// also subscribes there (one base slab of lists). A node with kIncLinks links or more is then
// updated in place (merge_patch).
void Index::merge_rebuild(uint32_t n) {
  const NodeLists& L = lists.h[n];
  uint32_t links = 0, xs = 0;
  for (uint32_t k = 0; k < L.n_merge; k++) {
    const PartList& p = subp_[L.sub_off + L.n_direct + k];
    links += p.cnt;
    bool x = false;
    for (uint32_t i = 0; i < p.cnt && !x; i++) x = (parts.m.h[p.off + i] & kForeign) != 0;
    xs += x;
  }
  if ((xs != 0) != ((L.flags & kFlagXNode) != 0)) {
    NodeLists& W = lists.at_w(n);
    W.flags = xs ? (W.flags | kFlagXNode) : (W.flags & ~kFlagXNode);
  }
  nh_[n].x_slots = xs;
  if (!links) return;
  uint32_t cap = 1;
  while (cap < links) cap <<= 1;
  const uint32_t off = mpart.alloc(cap);
  uint32_t at = off;
  for (uint32_t k = 0; k < L.n_merge; k++) {
    const uint32_t pos = L.sub_off + L.n_direct + k;
    const PartList& p = subp_[pos];
    const uint32_t client = subs.m.h[pos].client;
    mref.at_w(pos) = MergeRef{at, p.cnt};
    for (uint32_t i = 0; i < p.cnt; i++) {
      const uint32_t m = parts.m.h[p.off + i];
      mpart.m.at_w(at++) = MergePart{m, partner_meta(m, client)};
    }
  }
  nh_[n].mpart_off = off;
  nh_[n].mpart_cap = cap;
  mpart.live += cap;

  // pair block: partner node h -> g's slots (their places k in g's list) whose client also
  // subscribes at h
  thread_local std::vector<std::pair<uint32_t, uint32_t>> hk;
  hk.clear();
  for (uint32_t k = L.n_direct; k < L.n_direct + L.n_merge; k++) {
    const PartList& p = subp_[L.sub_off + k];
    for (uint32_t i = 0; i < p.cnt; i++) hk.emplace_back(parts.m.h[p.off + i], k);
  }
  std::sort(hk.begin(), hk.end());
  uint32_t lists_n = 0;
  for (size_t i = 0; i < hk.size(); i++) lists_n += i == 0 || hk[i].first != hk[i - 1].first;
  uint32_t ecap = 2, lcap = 1;
  while (ecap < 4 * lists_n) ecap <<= 1;  // load <= 1/4: k_merge probes four slots per load round
  while (lcap < hk.size()) lcap <<= 1;
  const uint32_t eo = pent.alloc(ecap), lo = plist.alloc(lcap), mask = ecap - 1;
  for (uint32_t i = 0; i < ecap; i++) pent.m.at_w(eo + i) = PairEnt{kNone, 0, 0, 0};
  for (size_t i = 0; i < hk.size(); i++) {
    const uint32_t pos = L.sub_off + hk[i].second;
    const MergeRef r = mref.h[pos];
    const SubRec& rec = subs.m.h[pos];
    plist.m.at_w(lo + i) = PairSlot{hk[i].second, r.off, r.cnt,
                                    rec.meta | (rec.ident > 0 ? kSlotIdentPos : 0u) |
                                        slot_partner_bits(partner_meta(hk[i].first, rec.client))};
  }
  const bool inc = links >= kIncLinks;
  MergeInc* I = nullptr;
  if (inc) {
    I = &minc_[n];
    I->slot.assign(L.n_direct + L.n_merge, MergeInc::Slot{});
    for (uint32_t k = L.n_direct; k < L.n_direct + L.n_merge; k++) {
      const MergeRef r = mref.h[L.sub_off + k];
      I->slot[k] = MergeInc::Slot{r.off, r.cnt, r.cnt | kPairBase};
    }
    I->where.reserve(hk.size());
    I->links = links;
  }
  for (size_t b = 0; b < hk.size();) {
    size_t e = b + 1;
    while (e < hk.size() && hk[e].first == hk[b].first) e++;
    uint32_t sl = pair_hash(hk[b].first) & mask;
    while (pent.m.h[eo + sl].h != kNone) sl = (sl + 1) & mask;
    const uint32_t cnt = (uint32_t)(e - b);
    pent.m.at_w(eo + sl) = PairEnt{hk[b].first, lo + (uint32_t)b, cnt, cnt | kPairBase};
    if (inc)
      for (size_t i = b; i < e; i++) I->where.put((uint64_t)hk[i].first << 32 | hk[i].second, (uint32_t)(i - b));
    b = e;
  }
  pent.live += lists_n;
  plist.live += hk.size();
  set_pair_header(n, NodePair{eo, mask, lo, lists_n});
  nh_[n].pent_cap = ecap;
  nh_[n].plist_cap = lcap;
}

// In place: every changed slot (by its place k) comes off the pair lists of its old partners
// and its old links are dropped; then every slot that is a may-merge slot now gets new links
// and goes onto the lists of its partners. A list or links slab that outgrows its room moves
// to a slab of its own; emptied lists leave the table (backward shift).
void Index::merge_patch(uint32_t n, MergeInc& I) {
  std::sort(I.dirty.begin(), I.dirty.end());
  I.dirty.erase(std::unique(I.dirty.begin(), I.dirty.end()), I.dirty.end());
  int32_t xs = 0;
  for (uint32_t k : I.dirty) {
    if (k >= I.slot.size() || !I.slot[k].mp_cnt) continue;
    const MergeInc::Slot S = I.slot[k];
    bool x = false;
    for (uint32_t e = 0; e < S.mp_cnt; e++) {
      const uint32_t h = mpart.m.h[S.mp_off + e].node;
      x |= (h & kForeign) != 0;
      pair_remove(n, I, h, k);
    }
    xs -= x;
    if (S.mp_cap & kPairBase) {
      I.garbage += S.mp_cnt;
    } else {
      mpart.release(S.mp_off, S.mp_cap);
      mpart.live -= S.mp_cap;
    }
    I.links -= S.mp_cnt;
    I.slot[k] = MergeInc::Slot{};
  }
  const NodeLists& L = lists.h[n];
  for (uint32_t k : I.dirty) {
    if (k < L.n_direct || k >= L.n_direct + L.n_merge) continue;
    const uint32_t pos = L.sub_off + k;
    const PartList p = subp_[pos];
    if (!p.cnt) continue;
    uint32_t cap = 1;
    while (cap < p.cnt) cap <<= 1;
    const uint32_t off = mpart.alloc(cap);
    mpart.live += cap;
    const SubRec rec = subs.m.h[pos];
    bool x = false;
    for (uint32_t i = 0; i < p.cnt; i++) {
      const uint32_t m = parts.m.h[p.off + i];
      mpart.m.at_w(off + i) = MergePart{m, partner_meta(m, rec.client)};
      x |= (m & kForeign) != 0;
    }
    xs += x;
    mref.at_w(pos) = MergeRef{off, p.cnt};
    if (k >= I.slot.size()) I.slot.resize(k + 1);
    I.slot[k] = MergeInc::Slot{off, p.cnt, cap};
    I.links += p.cnt;
    const uint32_t own = rec.meta | (rec.ident > 0 ? kSlotIdentPos : 0u);
    for (uint32_t i = 0; i < p.cnt; i++)
      pair_add(n, I, parts.m.h[p.off + i], PairSlot{k, off, p.cnt, own | slot_partner_bits(mpart.m.h[off + i].meta)});
  }
  I.dirty.clear();
  if (xs) {
    nh_[n].x_slots = (uint32_t)((int32_t)nh_[n].x_slots + xs);
    const bool want = nh_[n].x_slots != 0;
    if (want != ((L.flags & kFlagXNode) != 0)) {
      NodeLists& W = lists.at_w(n);
      W.flags = want ? (W.flags | kFlagXNode) : (W.flags & ~kFlagXNode);
    }
  }
}

uint32_t Index::pair_find(const NodePair& P, uint32_t h) const {
  if (P.ent_mask == kNone) return kNone;
  uint32_t sl = pair_hash(h) & P.ent_mask;
  for (uint32_t i = 0; i <= P.ent_mask; i++, sl = (sl + 1) & P.ent_mask) {
    const PairEnt& e = pent.m.h[P.ent_off + sl];
    if (e.h == h) return P.ent_off + sl;
    if (e.h == kNone) return kNone;
  }
  return kNone;
}

void Index::pair_rehash(uint32_t n, uint32_t ecap) {
  NodePair P = npair.h[n];
  const uint32_t eo = pent.alloc(ecap), mask = ecap - 1;
  for (uint32_t i = 0; i < ecap; i++) pent.m.at_w(eo + i) = PairEnt{kNone, 0, 0, 0};
  if (P.ent_mask != kNone) {
    for (uint32_t i = 0; i <= P.ent_mask; i++) {
      const PairEnt e = pent.m.h[P.ent_off + i];
      if (e.h == kNone) continue;
      uint32_t sl = pair_hash(e.h) & mask;
      while (pent.m.h[eo + sl].h != kNone) sl = (sl + 1) & mask;
      pent.m.at_w(eo + sl) = e;
    }
    pent.release(P.ent_off, nh_[n].pent_cap);
  }
  nh_[n].pent_cap = ecap;
  P.ent_off = eo;
  P.ent_mask = mask;
  set_pair_header(n, P);
}

void Index::pair_add(uint32_t n, MergeInc& I, uint32_t h, const PairSlot& ps) {
  NodePair P = npair.h[n];
  uint32_t ei = pair_find(P, h);
  if (ei == kNone) {  // a new partner node: a list of its own in the table (load <= 1/4)
    if (P.ent_mask == kNone || (P.n_lists + 1) * 4 > P.ent_mask + 1) {
      pair_rehash(n, P.ent_mask == kNone ? 4u : 2 * (P.ent_mask + 1));
      P = npair.h[n];
    }
    uint32_t sl = pair_hash(h) & P.ent_mask;
    while (pent.m.h[P.ent_off + sl].h != kNone) sl = (sl + 1) & P.ent_mask;
    ei = P.ent_off + sl;
    pent.m.at_w(ei) = PairEnt{h, plist.alloc(1), 0, 1};
    P.n_lists++;
    set_pair_header(n, P);
    pent.live++;
  }
  PairEnt e = pent.m.h[ei];
  const uint32_t cap = e.cap & ~kPairBase;
  if (e.cnt == cap) {  // full: the list moves to a slab twice as large
    uint32_t nc = 1;
    while (nc < e.cnt + 1) nc <<= 1;
    if (nc < 2 * cap && !(e.cap & kPairBase)) nc = 2 * cap;
    const uint32_t no = plist.alloc(nc);
    for (uint32_t i = 0; i < e.cnt; i++) plist.m.at_w(no + i) = plist.m.h[e.off + i];
    if (e.cap & kPairBase) I.garbage += cap;
    else plist.release(e.off, cap);
    e.off = no;
    e.cap = nc;
  }
  plist.m.at_w(e.off + e.cnt) = ps;
  I.where.put((uint64_t)h << 32 | ps.k, e.cnt);
  e.cnt++;
  plist.live++;
  pent.m.at_w(ei) = e;
}

void Index::pair_remove(uint32_t n, MergeInc& I, uint32_t h, uint32_t k) {
  NodePair P = npair.h[n];
  const uint32_t ei = pair_find(P, h);
  const uint64_t key = (uint64_t)h << 32 | k;
  uint32_t idx = kNone;
  if (ei == kNone || !I.where.get(key, &idx)) throw std::logic_error("flush_merge: pair-list entry missing");
  PairEnt e = pent.m.h[ei];
  const uint32_t last = e.cnt - 1;
  if (idx != last) {
    const PairSlot mv = plist.m.h[e.off + last];
    plist.m.at_w(e.off + idx) = mv;
    I.where.put((uint64_t)h << 32 | mv.k, idx);
  }
  I.where.erase(key);
  e.cnt--;
  plist.live--;
  if (e.cnt) {
    pent.m.at_w(ei) = e;
    return;
  }
  // the list is empty: its slab goes, and its entry leaves the table by backward shift (the
  // kernels' probes stop at an empty entry)
  if (e.cap & kPairBase) I.garbage += e.cap & ~kPairBase;
  else plist.release(e.off, e.cap);
  const uint32_t m = P.ent_mask;
  uint32_t i = ei - P.ent_off;
  for (uint32_t j = (i + 1) & m;; j = (j + 1) & m) {
    const PairEnt f = pent.m.h[P.ent_off + j];
    if (f.h == kNone) break;
    const uint32_t home = pair_hash(f.h) & m;
    const bool stays = i <= j ? (home > i && home <= j) : (home > i || home <= j);
    if (stays) continue;
    pent.m.at_w(P.ent_off + i) = f;
    i = j;
  }
  pent.m.at_w(P.ent_off + i) = PairEnt{kNone, 0, 0, 0};
  P.n_lists--;
  set_pair_header(n, P);
  pent.live--;
}

bool Index::check(std::string* why) {
  flush_merge();
  auto bad = [&](const std::string& m) {
    *why = m;
    return false;
  };
  uint64_t wild = 0;
  for (uint32_t n = 0; n < nh_.size(); n++) wild += nh_[n].live && n != kRoot && nh_[n].str <= 1;
  if (wild != n_wild_nodes_) return bad("wildcard particle count stale");
  for (uint32_t n = 0; n < nh_.size(); n++) {
    if (!nh_[n].live) continue;
    const NodeLists& L = lists.h[n];
    const std::string at = "node " + std::to_string(n);
    if (n != kRoot) {  // the incoming edge carries the node's '+' / '#' children
      const uint32_t par = walk.h[n].parent_flags & kParentMask;
      const uint64_t m = edges.size() - 1;
      uint64_t i = edge_hash(par, nh_[n].key) & m;
      while (edges.h[i].parent != kEdgeEmpty && !(edges.h[i].parent == par && edges.h[i].child == n)) i = (i + 1) & m;
      const EdgeSlot& e = edges.h[i];
      if (e.parent != par) return bad(at + ": no incoming edge");
      if (e.plus != walk.h[n].plus_child || e.hash != walk.h[n].hash_child) return bad(at + ": edge '+'/'#' copy stale");
    }
    if ((uint64_t)L.sub_off + L.n_direct + L.n_merge > subs.m.size() || L.n_direct + L.n_merge > nh_[n].sub_cap)
      return bad(at + ": subscription list out of bounds");
    if ((uint64_t)L.shr_off + L.shr_cnt > shr.m.size() || (uint64_t)inls.h[n].off + inls.h[n].cnt > inl.m.size() ||
        ((L.flags & kFlagInline) != 0) != (inls.h[n].cnt != 0) || L.ent_off != npair.h[n].ent_off ||
        L.ent_mask != npair.h[n].ent_mask)
      return bad(at + ": shared/inline list out of bounds");
    for (uint32_t k = 0; k < L.n_direct + L.n_merge; k++) {
      const uint32_t pos = L.sub_off + k;
      const uint32_t client = subs.m.h[pos].client;
      uint32_t p = kNone;
      if (!sub_pos_.get((uint64_t)n << 32 | client, &p) || p != pos) return bad(at + ": slot map stale");
      const PartList& pl = subp_[pos];
      if (k < L.n_direct) {
        if (pl.cnt) return bad(at + ": direct slot with partners");
        continue;
      }
      if (!pl.cnt) return bad(at + ": may-merge slot without partners");
      const MergeRef r = mref.h[pos];
      if (r.cnt != pl.cnt || (uint64_t)r.off + r.cnt > mpart.m.size()) return bad(at + ": partner ref stale");
      for (uint32_t e = 0; e < r.cnt; e++) {
        const MergePart mp = mpart.m.h[r.off + e];
        if (mp.node != parts.m.h[pl.off + e]) return bad(at + ": partner link stale");
        if (mp.node & kForeign) {  // another shard's subscription of the client
          uint32_t fi = kNone;
          if (!fsub_pos_.get((uint64_t)(mp.node & ~kForeign) << 32 | client, &fi)) return bad(at + ": foreign partner missing");
          if (mp.meta != fsubs_[fi].meta) return bad(at + ": foreign partner meta stale");
          if (!compatible_foreign(n, fsubs_[fi])) return bad(at + ": foreign partner not co-matchable");
          if (!(L.flags & kFlagXNode)) return bad(at + ": foreign partner but no X flag");
          continue;
        }
        if (mp.node >= nh_.size() || !nh_[mp.node].live) return bad(at + ": partner node stale");
        uint32_t ppos = kNone;
        if (!sub_pos_.get((uint64_t)mp.node << 32 | client, &ppos)) return bad(at + ": partner missing");
        const NodeLists& M = lists.h[mp.node];
        if (ppos < M.sub_off + M.n_direct || ppos >= M.sub_off + M.n_direct + M.n_merge)
          return bad(at + ": partner outside the partner's may-merge slots");
        if (mp.meta != (subs.m.h[ppos].meta & (kMetaQos | kMetaNoLocal))) return bad(at + ": partner meta stale");
        if (!compatible(n, mp.node)) return bad(at + ": partner not co-matchable");
        // the pair block of n lists slot k under partner node mp.node
        const NodePair& P = npair.h[n];
        if (P.ent_mask == kNone) return bad(at + ": may-merge slots without a pair block");
        uint32_t sl = pair_hash(mp.node) & P.ent_mask;
        while (pent.m.h[P.ent_off + sl].h != kNone && pent.m.h[P.ent_off + sl].h != mp.node)
          sl = (sl + 1) & P.ent_mask;
        const PairEnt& pe = pent.m.h[P.ent_off + sl];
        if (pe.h != mp.node) return bad(at + ": pair block misses a partner node");
        bool listed = false;
        const SubRec& rec = subs.m.h[pos];
        const uint32_t want_meta = rec.meta | (rec.ident > 0 ? kSlotIdentPos : 0u) | slot_partner_bits(mp.meta);
        for (uint32_t i = 0; i < pe.cnt && !listed; i++) {
          const PairSlot& ps = plist.m.h[pe.off + i];
          listed = ps.k == k && ps.mp_off == r.off && ps.mp_cnt == r.cnt && ps.meta == want_meta;
        }
        if (!listed) return bad(at + ": pair list misses a slot");
      }
    }
    // and the pair block lists nothing else: one entry per partner link, n_lists lists
    const NodePair& P = npair.h[n];
    if (P.ent_mask != kNone) {
      uint64_t want = 0, have = 0;
      uint32_t nl = 0;
      for (uint32_t k = L.n_direct; k < L.n_direct + L.n_merge; k++) want += mref.h[L.sub_off + k].cnt;
      for (uint32_t i = 0; i <= P.ent_mask; i++) {
        const PairEnt& e = pent.m.h[P.ent_off + i];
        if (e.h == kNone) continue;
        if (!e.cnt || e.cnt > (e.cap & ~kPairBase)) return bad(at + ": pair list count out of bounds");
        have += e.cnt;
        nl++;
      }
      if (have != want || nl != P.n_lists) return bad(at + ": pair block holds stale entries");
    }
  }
  for (uint32_t n = 0; n < nh_.size(); n++) {  // children slabs: each particle once, in its parent's
    if (!nh_[n].live) continue;
    const NodeMsg& M = msg.h[n];
    if (M.child_cnt != nh_[n].n_children || M.child_cnt > nh_[n].child_cap ||
        (uint64_t)M.child_off + nh_[n].child_cap > children.m.size())
      return bad("node " + std::to_string(n) + ": children slab out of bounds");
    if (n == kRoot) continue;
    const NodeMsg& P = msg.h[M.parent];
    if (M.child_pos >= P.child_cnt || children.m.h[P.child_off + M.child_pos].node != n)
      return bad("node " + std::to_string(n) + ": not at its position in the parent's children slab");
  }
  {  // below_live == live retained particles strictly below, recomputed bottom-up
    std::vector<uint32_t> below(nh_.size(), 0);
    for (uint32_t n = 0; n < nh_.size(); n++) {
      if (!nh_[n].live || n == kRoot || !(msg.h[n].flags & kRetainLive)) continue;
      for (uint32_t a = n; a != kRoot;) {
        a = msg.h[a].parent;
        below[a]++;
      }
    }
    for (uint32_t n = 0; n < nh_.size(); n++)
      if ((nh_[n].live || n == kRoot) && below[n] != msg.h[n].below_live)
        return bad("node " + std::to_string(n) + ": below_live stale");
  }
  return true;
}

// ---- copy-on-write against live host results (ViewTracker) ------------------------------------
void Index::begin_op() {
  if (!views_) return;
  uint64_t min_live = 0;
  {
    std::lock_guard<std::mutex> g(views_->mu);
    op_gen_ = views_->gen;
    op_max_ = views_->live.empty() ? 0 : *views_->live.rbegin();
    min_live = views_->live.empty() ? 0 : *views_->live.begin();
  }
  // what was retired at generation `tag` is seen only by live results of that generation or older
  // (the tags grow along the queues)
  auto unseen = [&](uint64_t tag) { return min_live == 0 || min_live > tag; };
  while (!retired_.empty() && unseen(retired_.front().tag)) {
    const Retired r = retired_.front();
    retired_.pop_front();
    if (r.pool == 0) subs.release(r.off, r.cap);
    else shr.release(r.off, r.cap);
  }
  while (!retired_subs_.empty() && unseen(retired_subs_.front().first)) retired_subs_.pop_front();
  while (!retired_shr_.empty() && unseen(retired_shr_.front().first)) retired_shr_.pop_front();
}

uint32_t Index::fresh_gen() {
  if (op_gen_ + 1 - gen_base_ >= 0xFFFFFFF0ull) {  // the 32-bit generations run out: every slab is old
    for (size_t n = 0; n < nh_.size(); n++) nh_[n].sub_gen = nh_[n].shr_gen = 0;
    gen_base_ = op_gen_;
  }
  return (uint32_t)(op_gen_ + 1 - gen_base_);  // seen by results published from now on
}

void Index::retire(int pool, uint32_t off, uint32_t cap) {
  if (!cap) return;
  if (!op_max_) {  // no live result
    if (pool == 0) subs.release(off, cap);
    else shr.release(off, cap);
    return;
  }
  retired_.push_back(Retired{op_gen_, pool, off, cap});
}

template <class T>
void Index::guard_growth(Mirror<T>& m, size_t need, std::deque<std::pair<uint64_t, std::vector<T>>>& keep) {
  if (!op_max_ || need <= m.h.capacity()) return;
  // a live result points into this buffer: the pool moves to a new one, the old one stays for it
  std::vector<T> fresh;
  fresh.reserve(std::max(need, 2 * m.h.capacity()));
  fresh.assign(m.h.begin(), m.h.end());
  keep.emplace_back(op_gen_, std::move(m.h));
  m.h = std::move(fresh);
  m.epoch++;
  m.all_dirty = true;
}

void Index::sub_cow(uint32_t n) {
  if (nh_[n].sub_cap && seen(nh_[n].sub_gen)) sub_move(n, nh_[n].sub_cap);
}

void Index::shr_cow(uint32_t n) {
  const uint32_t cap = nh_[n].shr_cap;
  if (!cap || !seen(nh_[n].shr_gen)) return;
  guard_growth(shr.m, shr.m.size() + cap, retired_shr_);
  NodeLists& L = lists.at_w(n);
  const uint32_t no = shr.alloc(cap), old = L.shr_off;
  if (shr_group_.size() < shr.m.size()) shr_group_.resize(shr.m.size());
  for (uint32_t i = 0; i < L.shr_cnt; i++) {
    shr.m.at_w(no + i) = shr.m.h[old + i];
    shr_group_[no + i] = shr_group_[old + i];
    shr_pos_[ShrKey{n, shr_group_[no + i], shr.m.h[no + i].client}] = no + i;
  }
  retire(1, old, cap);
  L.shr_off = no;
  nh_[n].shr_gen = fresh_gen();
}

void Index::sub_ensure(uint32_t n, uint32_t need) {
  uint32_t cap = nh_[n].sub_cap;
  if (need <= cap) return;
  uint32_t nc = cap ? cap : 1;
  while (nc < need) nc *= 2;
  sub_move(n, nc);
}

// n's subscription list to a new slab of nc records (the slots keep their places k)
void Index::sub_move(uint32_t n, uint32_t nc) {
  const uint32_t cap = nh_[n].sub_cap;
  guard_growth(subs.m, subs.m.size() + nc, retired_subs_);
  NodeLists& L = lists.at_w(n);
  uint32_t no = subs.alloc(nc), cnt = L.n_direct + L.n_merge;
  subp_.resize(subs.m.size(), PartList{0, 0, 0});
  for (uint32_t i = 0; i < cnt; i++) move_slot(n, L.sub_off + i, no + i, false);
  if (L.n_merge) {  // the merge refs follow their slots (pair slots name places, not positions)
    if (mref.size() < subs.m.size()) mref.grow_to(subs.m.size(), MergeRef{0, 0});
    for (uint32_t i = L.n_direct; i < cnt; i++) mref.at_w(no + i) = mref.h[L.sub_off + i];
  }
  retire(0, L.sub_off, cap);
  L.sub_off = no;
  nh_[n].sub_cap = nc;
  max_sub_cap_ = std::max(max_sub_cap_, nc);
  nh_[n].sub_gen = fresh_gen();
}

uint32_t Index::cow_pos(uint32_t n, uint32_t pos) {
  const uint32_t k = pos - lists.h[n].sub_off;
  sub_cow(n);
  return lists.h[n].sub_off + k;
}

uint32_t Index::sub_add(uint32_t n, const SubRec& r, bool merge) {
  sub_ensure(n, sub_count(n) + 1);
  if (!merge && lists.h[n].n_merge) sub_cow(n);  // (the first may-merge slot moves behind the others)
  NodeLists& L = lists.at_w(n);
  uint32_t base = L.sub_off, pos;
  if (merge) {
    pos = base + L.n_direct + L.n_merge;
    L.n_merge++;
    n_merge_++;
    merge_dirty_slot(n, pos);
  } else {
    pos = base + L.n_direct;
    if (L.n_merge) move_slot(n, pos, base + L.n_direct + L.n_merge);
    L.n_direct++;
  }
  subs.m.at_w(pos) = r;
  subp_[pos] = PartList{0, 0, 0};
  sub_pos_.put((uint64_t)n << 32 | r.client, pos);
  subs.live++;
  return pos;
}

void Index::sub_remove(uint32_t n, uint32_t pos) {
  pos = cow_pos(n, pos);
  NodeLists& L = lists.at_w(n);
  uint32_t base = L.sub_off;
  if (pos < base + L.n_direct) {
    uint32_t last_d = base + L.n_direct - 1;
    if (pos != last_d) move_slot(n, last_d, pos);
    if (L.n_merge) move_slot(n, base + L.n_direct + L.n_merge - 1, last_d);
    L.n_direct--;
  } else {
    uint32_t last = base + L.n_direct + L.n_merge - 1;
    merge_dirty_slot(n, pos);
    merge_dirty_slot(n, last);
    if (pos != last) move_slot(n, last, pos);
    L.n_merge--;
    n_merge_--;
  }
  subs.live--;
}

void Index::sub_set_merge(uint32_t n, uint32_t pos, bool merge) {
  if (merge == (pos >= lists.h[n].sub_off + lists.h[n].n_direct)) return;
  pos = cow_pos(n, pos);
  NodeLists& L = lists.at_w(n);
  uint32_t base = L.sub_off;
  uint32_t other = merge ? base + L.n_direct - 1 : base + L.n_direct;
  const SubRec a = subs.m.h[pos];
  const PartList ap = subp_[pos];
  if (other != pos) move_slot(n, other, pos);
  if (merge) {
    L.n_direct--;
    L.n_merge++;
    n_merge_++;
  } else {
    L.n_direct++;
    L.n_merge--;
    n_merge_--;
  }
  merge_dirty_slot(n, pos);
  merge_dirty_slot(n, other);
  subs.m.at_w(other) = a;
  subp_[other] = ap;
  sub_pos_.put((uint64_t)n << 32 | a.client, other);
}

void Index::part_set(uint32_t pos, const std::vector<uint32_t>& nodes) {
  uint32_t cap = 1;
  while (cap < nodes.size()) cap *= 2;
  const uint32_t off = parts.alloc(cap);
  for (size_t i = 0; i < nodes.size(); i++) parts.m.at_w(off + i) = nodes[i];
  subp_[pos] = PartList{off, (uint32_t)nodes.size(), cap};
  parts.live += nodes.size();
}

void Index::part_add(uint32_t pos, uint32_t node) {
  PartList& p = subp_[pos];
  list_push(parts, p.off, p.cnt, p.cap, node);
}

uint32_t Index::part_remove(uint32_t pos, uint32_t node) {
  PartList& p = subp_[pos];
  for (uint32_t i = 0; i < p.cnt; i++) {
    if (parts.m.h[p.off + i] != node) continue;
    parts.m.at_w(p.off + i) = parts.m.h[p.off + p.cnt - 1];
    p.cnt--;
    parts.live--;
    break;
  }
  return p.cnt;
}

void Index::part_release(uint32_t pos) {
  PartList& p = subp_[pos];
  parts.release(p.off, p.cap);
  parts.live -= p.cnt;
  p = PartList{0, 0, 0};
}

void Index::path_strs(uint32_t n, uint32_t* out, int* len) const {
  int d = nh_[n].depth;
  *len = d;
  while (n != kRoot) {
    out[--d] = nh_[n].str;
    n = walk.h[n].parent_flags & kParentMask;
  }
}

// Could one publish topic match both node paths a and b (A.2 rules A/B/C)? A sound
// over-approximation: '#' matches any suffix (including none), '+' any one level, and a
// path may be one level longer than the other only through a trailing '#'.
bool Index::compatible_strs(const uint32_t* pa, int la, const uint32_t* pb, int lb) {
  const int m = std::min(la, lb);
  for (int i = 0; i < m; i++) {
    const uint32_t x = pa[i], y = pb[i];
    if (x == 1 || y == 1) return true;  // '#'
    if (x == 0 || y == 0) continue;     // '+'
    if (x != y) return false;
  }
  if (la == lb) return true;
  const uint32_t* lo = la > lb ? pa : pb;
  return std::max(la, lb) == m + 1 && lo[m] == 1;
}

bool Index::compatible(uint32_t a, uint32_t b) const {
  const uint32_t s0 = nh_[a].seg0, s1 = nh_[b].seg0;
  if (s0 > 1 && s1 > 1 && s0 != s1) return false;  // different literal first levels
  thread_local std::vector<uint32_t> pa, pb;
  pa.resize(nh_[a].depth);
  pb.resize(nh_[b].depth);
  int la, lb;
  path_strs(a, pa.data(), &la);
  path_strs(b, pb.data(), &lb);
  return compatible_strs(pa.data(), la, pb.data(), lb);
}

bool Index::compatible_foreign(uint32_t a, const ForeignSub& f) const {
  const uint32_t s0 = nh_[a].seg0, s1 = fpaths_[f.path_off];
  if (s0 > 1 && s1 > 1 && s0 != s1) return false;
  thread_local std::vector<uint32_t> pa;
  pa.resize(nh_[a].depth);
  int la;
  path_strs(a, pa.data(), &la);
  return compatible_strs(pa.data(), la, fpaths_.data() + f.path_off, (int)f.depth);
}

// A non-shared subscription owned by another shard (sharded index): recorded as a foreign
// partner of this shard's co-matchable subscriptions of the same client.
int Index::foreign_subscribe(std::string_view filter, uint32_t client, uint32_t fid, uint32_t meta) {
  if (fid & kForeign) throw std::invalid_argument("sharded index: filter ids must be < 2^31");
  const uint32_t sid = ffilt_.intern(filter);
  if (sid >= ffid_.size()) ffid_.resize(sid + 1, kNone);
  ffid_[sid] = fid;
  uint32_t i = kNone;
  const uint64_t key = (uint64_t)fid << 32 | client;
  auto cn = client_nodes_.find(client);
  if (fsub_pos_.get(key, &i)) {  // re-Subscribe: the partners' links carry its meta
    if (fsubs_[i].meta != meta && cn != client_nodes_.end())
      for (uint32_t m : cn->second) touch_partner(m, client);
    fsubs_[i].meta = meta;
    return 0;
  }
  thread_local std::vector<std::string_view> path;
  path_of(filter, 0, path);
  ForeignSub f{client, fid, meta, (uint32_t)fpaths_.size(), (uint32_t)path.size()};
  for (std::string_view seg : path) fpaths_.push_back(intern_str(seg));
  if (f.depth > 32) note_deep(fid, fpaths_.data() + f.path_off, f.depth);
  if (!fsub_free_.empty()) {
    i = fsub_free_.back();
    fsub_free_.pop_back();
    fsubs_[i] = f;
  } else {
    i = (uint32_t)fsubs_.size();
    fsubs_.push_back(f);
  }
  fsub_pos_.put(key, i);
  client_foreign_[client].push_back(i);
  if (cn != client_nodes_.end())
    for (uint32_t m : cn->second) {
      if (!compatible_foreign(m, f)) continue;
      uint32_t mp;
      if (!sub_pos_.get((uint64_t)m << 32 | client, &mp)) continue;
      if (!sub_is_merge(m, mp)) {
        sub_set_merge(m, mp, true);
        sub_pos_.get((uint64_t)m << 32 | client, &mp);
      }
      part_add(mp, kForeign | fid);
      merge_dirty_slot(m, mp);
    }
  return 0;
}

void Index::foreign_unsubscribe(uint32_t client, uint32_t fid) {
  uint32_t i = kNone;
  const uint64_t key = (uint64_t)fid << 32 | client;
  if (!fsub_pos_.get(key, &i)) return;
  auto cn = client_nodes_.find(client);
  if (cn != client_nodes_.end())
    for (uint32_t m : cn->second) {
      uint32_t mp;
      if (!sub_pos_.get((uint64_t)m << 32 | client, &mp)) continue;
      const PartList& p = subp_[mp];
      bool linked = false;
      for (uint32_t k = 0; k < p.cnt && !linked; k++) linked = parts.m.h[p.off + k] == (kForeign | fid);
      if (!linked) continue;
      merge_dirty_slot(m, mp);
      if (part_remove(mp, kForeign | fid) == 0) {
        part_release(mp);
        sub_set_merge(m, mp, false);
      }
    }
  fsub_pos_.erase(key);
  auto cf = client_foreign_.find(client);
  if (cf != client_foreign_.end()) {
    auto& v = cf->second;
    v.erase(std::find(v.begin(), v.end(), i));
    if (v.empty()) client_foreign_.erase(cf);
  }
  if (fsubs_[i].depth > 32) deep_unref(fid);
  fsubs_[i].depth = 0;
  fsub_free_.push_back(i);
}

// ---- TopicsIndex operations ----------------------------------------------------------------------

// topics.go:401-419
// Owner shard of a subscription. A shared one is keyed by (particle, group, client)
// (topics.go:406-411): its owner hashes the group and the particle's path — "$share/g/a" and
// "$SHARE/g/a" are one key, and so are "$share/g" and "$share/g/g" (Q13: a short filter's
// particle is its last segment, isolateParticle beyond range). Others hash the filter.
std::string shard_key(std::string_view filter, bool share) {
  if (!share) return std::string(filter);
  std::string k(segment_at(filter, 1));
  k.push_back('\0');
  std::vector<std::string_view> path;
  size_t s = 0;
  std::vector<std::string_view> segs;
  for (;;) {
    const size_t e = filter.find('/', s);
    segs.push_back(filter.substr(s, e == std::string_view::npos ? std::string_view::npos : e - s));
    if (e == std::string_view::npos) break;
    s = e + 1;
  }
  if (segs.size() > 2) path.assign(segs.begin() + 2, segs.end());
  else path.push_back(segs.back());
  for (std::string_view p : path) {
    k.append(p.data(), p.size());
    k.push_back('/');
  }
  return k;
}

int Index::subscribe(std::string_view filter, uint32_t client, uint32_t filter_id, uint8_t qos,
                     uint8_t flags, int32_t ident) {
  version_++;
  begin_op();
  const bool share = is_share_prefix(segment_at(filter, 0));
  if (sharded() && shard_hash(shard_key(filter, share)) % n_shards_ != shard_) {
    if (share) return 0;  // the owner answers
    return foreign_subscribe(filter, client, filter_id, (uint32_t)(qos & 3) | ((flags & 1) ? kMetaNoLocal : 0));
  }
  if (share) {
    std::string group(segment_at(filter, 1));
    auto git = group_ids_.find(group);
    uint32_t gid;
    if (git == group_ids_.end()) {
      gid = (uint32_t)group_ids_.size();
      group_ids_.emplace(group, gid);
    } else {
      gid = git->second;
    }
    uint32_t n = set(filter, 2);
    ShrKey key{n, gid, client};
    auto it = shr_pos_.find(key);
    ShrRec rec{filter_id, client};
    if (it != shr_pos_.end()) {
      shr_cow(n);
      shr.m.at_w(shr_pos_[key]) = rec;
      return 0;
    }
    NodeLists& L = lists.at_w(n);
    uint32_t old_off = L.shr_off, cnt = L.shr_cnt;
    list_push(shr, L.shr_off, L.shr_cnt, nh_[n].shr_cap, rec);
    if (shr_group_.size() < shr.m.size()) shr_group_.resize(shr.m.size());
    if (L.shr_off != old_off) {  // slab moved: carry the group ids and re-point the records
      for (uint32_t i = 0; i < cnt; i++) {
        uint32_t g = shr_group_[old_off + i];
        shr_group_[L.shr_off + i] = g;
        shr_pos_[ShrKey{n, g, shr.m.h[L.shr_off + i].client}] = L.shr_off + i;
      }
      nh_[n].shr_gen = fresh_gen();
    }
    shr_pos_[key] = L.shr_off + cnt;
    shr_group_[L.shr_off + cnt] = gid;
    return 1;
  }
  uint32_t n = set(filter, 0);
  SubRec rec{client, filter_id, ident,
             (uint32_t)(qos & 3) | ((flags & 1) ? kMetaNoLocal : 0) | ((flags & 2) ? kMetaRap : 0) |
                 ((uint32_t)((flags >> 2) & 3) << kMetaRhShift)};
  uint32_t pos;
  if (sub_pos_.get((uint64_t)n << 32 | client, &pos)) {
    pos = cow_pos(n, pos);
    const SubRec old = subs.m.h[pos];
    subs.m.at_w(pos) = rec;
    const PartList& p = subp_[pos];  // the partners' links carry this subscription's Qos / NoLocal,
    if ((old.meta ^ rec.meta) & (kMetaQos | kMetaNoLocal))
      for (uint32_t i = 0; i < p.cnt; i++) touch_partner(parts.m.h[p.off + i], client);
    // and n's pair slots copy its meta and whether its identifier is > 0
    if (sub_is_merge(n, pos) && (old.meta != rec.meta || (old.ident > 0) != (rec.ident > 0))) merge_dirty_slot(n, pos);
    return 0;
  }
  // Partners: the client's other subscriptions that could match the same topic (the merge
  // candidates of gatherSubscriptions / Subscription.Merge, topics.go:641-646), on this shard
  // and (sharded index) on the others.
  if (sharded() && xinfo.h[n].fid == kNone) {
    if (filter_id & kForeign) throw std::invalid_argument("sharded index: filter ids must be < 2^31");
    xinfo.at_w(n).fid = filter_id;
    note_deep_node(n, filter_id);
  }
  std::vector<uint32_t>& mine = client_nodes_[client];
  thread_local std::vector<uint32_t> comp, all;
  comp.clear();
  for (uint32_t m : mine)
    if (compatible(n, m)) comp.push_back(m);
  all = comp;
  auto cf = client_foreign_.find(client);
  if (cf != client_foreign_.end())
    for (uint32_t i : cf->second)
      if (compatible_foreign(n, fsubs_[i])) all.push_back(kForeign | fsubs_[i].fid);
  pos = sub_add(n, rec, !all.empty());
  if (!all.empty()) part_set(pos, all);
  for (uint32_t m : comp) {
    uint32_t mp;
    if (!sub_pos_.get((uint64_t)m << 32 | client, &mp)) continue;
    if (!sub_is_merge(m, mp)) {
      sub_set_merge(m, mp, true);
      sub_pos_.get((uint64_t)m << 32 | client, &mp);
    }
    part_add(mp, n);
    merge_dirty_slot(m, mp);
  }
  mine.push_back(n);
  return 1;
}

// topics.go:423-448
int Index::unsubscribe(std::string_view filter, uint32_t client) {
  version_++;
  begin_op();
  bool share = is_share_prefix(segment_at(filter, 0));
  if (sharded() && shard_hash(shard_key(filter, share)) % n_shards_ != shard_) {
    if (!share) {  // the owner drops the subscription; here it stops being a foreign partner
      const uint32_t sid = ffilt_.find(filter);
      if (sid != kNone && sid < ffid_.size()) foreign_unsubscribe(client, ffid_[sid]);
    }
    return seek(filter, share ? 2 : 0) != kNone ? 1 : 0;  // this shard's part of "particle exists"
  }
  uint32_t n = seek(filter, share ? 2 : 0);
  if (n == kNone) return 0;
  if (share) {
    auto git = group_ids_.find(std::string(segment_at(filter, 1)));
    if (git != group_ids_.end()) {
      auto it = shr_pos_.find(ShrKey{n, git->second, client});
      if (it != shr_pos_.end()) {
        shr_cow(n);
        it = shr_pos_.find(ShrKey{n, git->second, client});
        NodeLists& L = lists.at_w(n);
        uint32_t pos = it->second, last = L.shr_off + L.shr_cnt - 1;
        shr_pos_.erase(it);
        if (pos != last) {
          shr.m.at_w(pos) = shr.m.h[last];
          shr_group_[pos] = shr_group_[last];
          shr_pos_[ShrKey{n, shr_group_[pos], shr.m.h[pos].client}] = pos;
        }
        L.shr_cnt--;
        shr.live--;
      }
    }
  } else {
    uint32_t pos;
    uint64_t key = (uint64_t)n << 32 | client;
    if (sub_pos_.get(key, &pos)) {
      const PartList pl = subp_[pos];
      std::vector<uint32_t> partners(parts.m.h.begin() + pl.off, parts.m.h.begin() + pl.off + pl.cnt);
      part_release(pos);
      sub_remove(n, pos);
      sub_pos_.erase(key);
      auto cit = client_nodes_.find(client);
      if (cit != client_nodes_.end()) {
        auto& v = cit->second;
        v.erase(std::find(v.begin(), v.end(), n));
        if (v.empty()) client_nodes_.erase(cit);
      }
      for (uint32_t m : partners) {  // the partners lose this one; unflag those left alone
        if (m & kForeign) continue;  // another shard's subscription: no link back on this shard
        uint32_t mp;
        if (!sub_pos_.get((uint64_t)m << 32 | client, &mp)) continue;
        merge_dirty_slot(m, mp);
        if (part_remove(mp, n) == 0) {
          part_release(mp);
          sub_set_merge(m, mp, false);
        }
      }
    }
  }
  trim(n);
  return 1;
}

// topics.go:368-378
static std::string_view inline_key(const int32_t& ident) {
  return std::string_view(reinterpret_cast<const char*>(&ident), sizeof(ident));
}

int Index::inline_subscribe(std::string_view filter, int32_t ident, uint32_t filter_id) {
  version_++;
  begin_op();
  if (sharded() && shard_hash(inline_key(ident)) % n_shards_ != shard_) return 0;  // by identifier
  uint32_t n = set(filter, 0);
  uint64_t key = (uint64_t)n << 32 | (uint32_t)ident;
  InlRec rec{ident, filter_id};
  uint32_t pos;
  if (inl_pos_.get(key, &pos)) {
    inl.m.at_w(pos) = rec;
    return 0;
  }
  NodeInl& I = inls.at_w(n);
  uint32_t old_off = I.off, cnt = I.cnt;
  list_push(inl, I.off, I.cnt, nh_[n].inl_cap, rec);
  if (I.off != old_off)
    for (uint32_t i = 0; i < cnt; i++)
      inl_pos_.put((uint64_t)n << 32 | (uint32_t)inl.m.h[I.off + i].ident, I.off + i);
  inl_pos_.put(key, I.off + cnt);
  if (!(lists.h[n].flags & kFlagInline)) lists.at_w(n).flags |= kFlagInline;
  return 1;
}

// topics.go:382-397
int Index::inline_unsubscribe(std::string_view filter, int32_t ident) {
  version_++;
  begin_op();
  uint32_t n = seek(filter, 0);
  if (n == kNone) return 0;
  if (sharded() && shard_hash(inline_key(ident)) % n_shards_ != shard_) return 1;  // exists here
  uint64_t key = (uint64_t)n << 32 | (uint32_t)ident;
  uint32_t pos;
  if (inl_pos_.get(key, &pos)) {
    NodeInl& I = inls.at_w(n);
    uint32_t last = I.off + I.cnt - 1;
    inl_pos_.erase(key);
    if (pos != last) {
      inl.m.at_w(pos) = inl.m.h[last];
      inl_pos_.put((uint64_t)n << 32 | (uint32_t)inl.m.h[pos].ident, pos);
    }
    I.cnt--;
    inl.live--;
    if (!I.cnt) lists.at_w(n).flags &= ~kFlagInline;
  }
  if (inls.h[n].cnt == 0) trim(n);
  return 1;
}

// topics.go:453-476. The Retained map (packets.Packets, topics.go:351) is kept on the particles:
// a non-empty topic's particle is unique (its path spells the topic), so the map entry is the
// particle's kRetainLive bit (with the packet's Retain flag, which the -1 answer reads) and the
// entry of topic "" (retainPath "" is no path, Q6) is kept apart.
int64_t Index::retain_message(std::string_view topic, uint64_t handle, uint32_t payload_len,
                              bool retain) {
  version_++;
  begin_op();
  retained_version_++;
  if (sharded() && shard_hash(topic) % n_shards_ != shard_) return 0;  // retained: by topic
  const uint32_t n = set(topic, 0);
  const bool path = !topic.empty();  // retainPath = pk.TopicName; "" means no path
  NodeMsg& M = msg.at_w(n);
  const bool node_live = (M.flags & kRetainLive) != 0;
  if (payload_len > 0) {
    nh_[n].retain_path = path;
    M.flags = (M.flags & kChildSys) | (path ? (kRetainPath | kRetainLive | (retain ? kRetainFlag : 0u)) : 0u);
    M.handle = path ? handle : 0;
    child_rec_sync(n);
    if (path && !node_live) {
      add_below_live(n, 1);
      n_retained_++;
    }
    if (!path) {
      if (!empty_topic_live) n_retained_++;
      empty_topic_live = true;
      empty_topic_handle = handle;
      empty_topic_retain = retain;
    }
    return 1;
  }
  // -1: the replaced entry had a payload (every stored one has) and its Retain flag
  const bool was_live = path ? node_live : empty_topic_live;
  const bool was_retain = path ? (M.flags & kRetainFlag) != 0 : empty_topic_retain;
  const int64_t out = was_live && was_retain ? -1 : 0;
  nh_[n].retain_path = false;
  M.flags &= kChildSys;
  M.handle = 0;
  child_rec_sync(n);
  if (node_live) add_below_live(n, -1);
  if (was_live) n_retained_--;
  if (!path) empty_topic_live = false;
  trim(n);
  return out;
}

// Retained.Delete (server.go:1726): the map entry only; the particle keeps retainPath (Q12).
int Index::retained_delete(std::string_view topic) {
  version_++;
  begin_op();
  retained_version_++;
  if (sharded() && shard_hash(topic) % n_shards_ != shard_) return 0;
  if (topic.empty()) {
    if (!empty_topic_live) return 0;
    empty_topic_live = false;
    n_retained_--;
    return 1;
  }
  const uint32_t n = seek(topic, 0);
  if (n == kNone || !(msg.h[n].flags & kRetainLive)) return 0;
  msg.at_w(n).flags &= ~(kRetainLive | kRetainFlag);
  child_rec_sync(n);
  add_below_live(n, -1);
  n_retained_--;
  return 1;
}

// Retained.Add outside RetainMessage (mq_retained_set): the entry of a particle whose retain path
// is the topic becomes live again (Q12 re-add); the "" entry is kept apart (Q6).
int Index::retained_set(std::string_view topic, uint64_t handle, uint32_t payload_len, bool retain) {
  version_++;
  begin_op();
  retained_version_++;
  if (sharded() && shard_hash(topic) % n_shards_ != shard_) return 0;
  const bool flag = retain && payload_len > 0;  // what RetainMessage's -1 answer reads (topics.go:467)
  if (topic.empty()) {
    if (!empty_topic_live) n_retained_++;
    empty_topic_live = true;
    empty_topic_handle = handle;
    empty_topic_retain = flag;
    return 1;
  }
  const uint32_t n = seek(topic, 0);
  if (n == kNone || !nh_[n].retain_path) return 0;
  NodeMsg& M = msg.at_w(n);
  if (!(M.flags & kRetainLive)) {
    add_below_live(n, 1);
    n_retained_++;
  }
  M.flags = (M.flags & (kChildSys | kRetainPath)) | kRetainLive | (flag ? kRetainFlag : 0u);
  M.handle = handle;
  child_rec_sync(n);
  return 1;
}

}  // namespace mq

namespace mq {
// used by the bulk build (index_bulk.cpp)
template void Index::list_push<ShrRec, ShrRec>(SlabPool<ShrRec>&, uint32_t&, uint32_t&, uint32_t&, const ShrRec&);
}  // namespace mq
