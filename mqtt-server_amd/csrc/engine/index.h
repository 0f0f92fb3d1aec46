// Host side of the engine: the authoritative, incrementally updated trie image.
//
// The reference keeps a pointer trie of particles with per-node Go maps (topics.go:748-822).
// Here the same trie is held as flat arrays in exactly the device layout (layout.h): an
// open-addressing edge table, node records, and slab-allocated subscription lists. Updates
// (Subscribe/Unsubscribe/RetainMessage...) edit these host arrays in place and mark dirty
// pages; Device::sync() uploads only those pages, so the HBM image is updated incrementally
// rather than rebuilt.
#pragma once

#include <sys/mman.h>

#include <algorithm>
#include <cstdlib>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <new>
#include <set>
#include <type_traits>
#include <cstdint>
#include <string>
#include <thread>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "layout.h"

namespace mq {

// Grows v's capacity to at least n elements and makes the unused capacity resident — huge
// pages where the kernel allows them, faulted in by `threads` threads — so that a bulk build's
// first touch of a multi-GB array is not one thread's page-fault storm. Contents are unchanged.
template <class T>
void reserve_resident(std::vector<T>& v, size_t n, unsigned threads) {
  if (n > v.capacity()) v.reserve(n);
  constexpr uintptr_t kPage = 4096;
  const uintptr_t b = ((uintptr_t)(v.data() + v.size()) + kPage - 1) & ~(kPage - 1);
  const uintptr_t e = (uintptr_t)(v.data() + v.capacity()) & ~(kPage - 1);
  if (e <= b || e - b < (64u << 20)) return;  // small: the ordinary faults are cheap
  madvise((void*)b, e - b, MADV_HUGEPAGE);
  constexpr uintptr_t kHuge = 2u << 20;
  const unsigned t = std::max(1u, std::min<unsigned>(threads, (unsigned)((e - b) / (32u << 20))));
  const uintptr_t per = ((e - b) / t + kHuge - 1) & ~(kHuge - 1);
  std::vector<std::thread> th;
  for (unsigned k = 0; k < t; k++) {
    const uintptr_t lo = b + k * per, hi = std::min(e, lo + per);
    if (lo < hi) th.emplace_back([lo, hi] { madvise((void*)lo, hi - lo, MADV_POPULATE_WRITE); });  // best effort
  }
  for (auto& x : th) x.join();
}

// Grows v's capacity to at least n elements and advises huge pages for the unused part (no
// touch): a bulk build that then fills it takes 2 MiB faults instead of 4 KiB ones.
template <class T>
void reserve_huge(std::vector<T>& v, size_t n) {
  if (n > v.capacity()) v.reserve(n);
  constexpr uintptr_t kHuge = 2u << 20;
  const uintptr_t b = ((uintptr_t)(v.data() + v.size()) + kHuge - 1) & ~(kHuge - 1);
  const uintptr_t e = (uintptr_t)(v.data() + v.capacity()) & ~(kHuge - 1);
  if (e > b) madvise((void*)b, e - b, MADV_HUGEPAGE);
}

// A host vector mirrored into device memory; tracks which pages changed since the last sync.
template <class T>
struct Mirror {
  // Dirty tracking granule: an update touches single records at random places, and each
  // touched page is uploaded whole, so pages are small (64 B: a power of two elements, at least
  // one; page starts are 16-byte aligned); the device applies them by scatter (Device::sync). The
  // bitmap's non-zero words are also listed, so a sync visits only those (a 10M-subscription
  // edge table has a million bitmap words).
  static constexpr size_t kPageBytes = 64;
  std::vector<T> h;
  std::vector<uint64_t> dirty;        // bitmap of pages
  std::vector<uint32_t> dirty_words;  // its non-zero words, in marking order
  size_t dirty_pages = 0;
  bool all_dirty = true;
  uint64_t epoch = 0;  // bumped when the host array is reallocated (device must realloc too)

  static constexpr size_t per_page() {
    size_t p = 1;
    while (p * 2 * sizeof(T) <= kPageBytes) p *= 2;
    return p;
  }
  size_t size() const { return h.size(); }
  T& operator[](size_t i) { return h[i]; }
  const T& operator[](size_t i) const { return h[i]; }
  void mark_page(size_t p) {  // (not thread-safe: parallel bulk builds write h directly, all_dirty)
    if (all_dirty) return;     // the whole array is uploaded anyway
    const size_t w = p / 64;
    if (w >= dirty.size()) dirty.resize(std::max(w + 1, dirty.size() + dirty.size() / 2), 0);
    const uint64_t bit = 1ull << (p % 64);
    if (dirty[w] & bit) return;
    if (!dirty[w]) dirty_words.push_back((uint32_t)w);
    dirty[w] |= bit;
    dirty_pages++;
  }
  void mark(size_t i) { mark_page(i / per_page()); }
  void mark_range(size_t i, size_t n) {
    if (!n) return;
    const size_t p0 = i / per_page(), p1 = (i + n - 1) / per_page();
    for (size_t p = p0; p <= p1; p++) mark_page(p);
  }
  T& at_w(size_t i) {  // write access
    mark(i);
    return h[i];
  }
  void reserve_resident(size_t n, unsigned threads) {  // capacity for n, resident (bulk builds)
    if (n > h.capacity()) {
      epoch++;
      all_dirty = true;
    }
    mq::reserve_resident(h, n, threads);
  }
  void grow_to(size_t n, const T& fill) {
    if (n <= h.size()) return;
    size_t old = h.size();
    if (n > h.capacity()) {
      h.reserve(n < 2 * h.capacity() ? 2 * h.capacity() : n);
      epoch++;
      all_dirty = true;
    }
    h.resize(n, fill);
    if (!all_dirty) mark_range(old, n - old);  // (a whole upload is coming anyway)
  }
  void clear_dirty() {
    all_dirty = false;
    for (uint32_t w : dirty_words) dirty[w] = 0;
    dirty_words.clear();
    dirty_pages = 0;
  }
};

// Power-of-two size-class slab allocator over a mirrored pool.
template <class T>
struct SlabPool {
  Mirror<T> m;
  std::vector<std::vector<uint32_t>> free_lists = std::vector<std::vector<uint32_t>>(33);
  uint64_t live = 0;  // elements in use

  static uint32_t cls_of(uint32_t cap) {
    uint32_t c = 0;
    while ((1u << c) < cap) c++;
    return c;
  }
  uint32_t alloc(uint32_t cap) {  // cap must be a power of two
    uint32_t c = cls_of(cap);
    auto& fl = free_lists[c];
    if (!fl.empty()) {
      uint32_t off = fl.back();
      fl.pop_back();
      return off;
    }
    uint32_t off = (uint32_t)m.size();
    m.grow_to(m.size() + (1u << c), T{});
    return off;
  }
  void release(uint32_t off, uint32_t cap) {
    if (cap) free_lists[cls_of(cap)].push_back(off);
  }
};

// Runs f(begin, end) over [0, n) split into contiguous pieces on up to `threads` threads.
template <class F>
void parallel_for(size_t n, unsigned threads, F&& f) {
  threads = std::max(1u, std::min<unsigned>(threads, (unsigned)((n + 4095) / 4096)));
  if (threads <= 1) {
    if (n) f((size_t)0, n);
    return;
  }
  std::vector<std::thread> th;
  const size_t per = (n + threads - 1) / threads;
  for (unsigned t = 0; t < threads; t++) {
    const size_t b = std::min(n, t * per), e = std::min(n, b + per);
    if (b < e) th.emplace_back([&f, b, e] { f(b, e); });
  }
  for (auto& x : th) x.join();
}

// Growable array of trivially copyable records (the host-only particle table): like a
// std::vector, but a bulk build's growth is filled on many threads (resize) and its reservation
// can be huge-page advised before the first touch (reserve_huge).
template <class T>
class PodVec {
  static_assert(std::is_trivially_copyable<T>::value, "PodVec holds trivially copyable records");

 public:
  PodVec() = default;
  ~PodVec() { std::free(p_); }
  PodVec(const PodVec&) = delete;
  PodVec& operator=(const PodVec&) = delete;
  size_t size() const { return n_; }
  size_t capacity() const { return cap_; }
  T* data() { return p_; }
  T& operator[](size_t i) { return p_[i]; }
  const T& operator[](size_t i) const { return p_[i]; }
  void reserve(size_t n) {
    if (n <= cap_) return;
    T* q = static_cast<T*>(std::realloc(p_, n * sizeof(T)));
    if (!q) throw std::bad_alloc();
    p_ = q;
    cap_ = n;
  }
  void reserve_huge(size_t n) {  // reserve, then advise huge pages for the untouched part
    reserve(n);
    constexpr uintptr_t kHuge = 2u << 20;
    const uintptr_t b = ((uintptr_t)(p_ + n_) + kHuge - 1) & ~(kHuge - 1);
    const uintptr_t e = (uintptr_t)(p_ + cap_) & ~(kHuge - 1);
    if (e > b) madvise((void*)b, e - b, MADV_HUGEPAGE);
  }
  void push_back(const T& v) {
    if (n_ == cap_) reserve(std::max<size_t>(16, cap_ * 2));
    p_[n_++] = v;
  }
  void resize(size_t n, unsigned threads = 1) {  // new records are T{}
    if (n > cap_) reserve(std::max(n, cap_ + cap_ / 2));
    if (n > n_)
      parallel_for(n - n_, threads, [&](size_t b, size_t e) {
        for (size_t i = b; i < e; i++) new (p_ + n_ + i) T{};
      });
    n_ = n;
  }

 private:
  T* p_ = nullptr;
  size_t n_ = 0, cap_ = 0;
};

// Open-addressing u64 -> u32 map (linear probing), used for (node, client) positions.
class HashU64 {
 public:
  explicit HashU64(size_t cap = 1024) { rehash(cap); }
  bool get(uint64_t k, uint32_t* v) const;
  void put(uint64_t k, uint32_t v);
  // Replace the contents with n distinct keys (bulk build; threads insert with CAS).
  void build_parallel(const uint64_t* keys, const uint32_t* vals, size_t n, unsigned threads);
  bool erase(uint64_t k);
  size_t size() const { return n_; }
  void reserve(size_t n) {
    if (n * 2 > keys_.size()) rehash(n * 2);
  }

 private:
  void rehash(size_t cap);
  size_t slot(uint64_t k) const { return (size_t)(mix64(k) & (keys_.size() - 1)); }
  static constexpr uint64_t kEmpty = ~0ull, kTomb = ~0ull - 1;
  std::vector<uint64_t> keys_;
  std::vector<uint32_t> vals_;
  size_t n_ = 0, tombs_ = 0;
};

// Interned strings: an arena plus an open-addressing table keyed by the bytes (no std::string
// per lookup).
class StrTable {
 public:
  StrTable() { slots_.assign(1024, kNone); }
  uint32_t intern(std::string_view s);  // id of s, inserting it if new
  uint32_t find(std::string_view s) const;  // id or kNone
  std::string_view at(uint32_t id) const {
    return std::string_view(arena_.data() + offs_[id], offs_[id + 1] - offs_[id]);
  }
  size_t size() const { return offs_.size() - 1; }

 private:
  static uint64_t hash(std::string_view s);
  void grow();
  std::vector<char> arena_;
  std::vector<uint64_t> offs_{0};
  std::vector<uint64_t> hashes_;
  std::vector<uint32_t> slots_;
};

// Host span results alive (mq_match_spans results point into the subscription pools; capi.cpp).
// Each gets a generation when published; the index copies a slab before it changes one that a live
// result may see, and keeps released slabs and outgrown pool buffers until no live result can see
// them (Index::begin_op) — so updates never wait for results (the reference's writers never wait
// for a reader's maps either, topics.go:270-277, 401-419). Owned by the handle's lock record, so a
// result freed after the index is destroyed still finds it.
struct ViewTracker {
  std::mutex mu;
  std::multiset<uint64_t> live;  // generations of the live results
  uint64_t gen = 0;              // generations handed out
  uint64_t publish() {
    std::lock_guard<std::mutex> g(mu);
    live.insert(++gen);
    return gen;
  }
  std::condition_variable cv;  // new matches wait on it while updates are announced
  uint64_t writers = 0;         // updates announced (a new match waits for them: capi.cpp)
  void release(uint64_t v) {
    std::lock_guard<std::mutex> g(mu);
    auto it = live.find(v);
    if (it != live.end()) live.erase(it);
    cv.notify_all();
  }
};

struct NodeHost {
  SegKey key{0, 0};
  uint32_t str = 0;        // interned segment string id (0 = "+", 1 = "#")
  uint32_t seg0 = 0;       // str of the path's first segment (quick compatibility reject)
  uint32_t n_children = 0;
  uint32_t child_pos = 0;  // position in the parent's children slab
  uint32_t sub_cap = 0, shr_cap = 0, inl_cap = 0, child_cap = 0;
  uint32_t mpart_off = 0, mpart_cap = 0;  // the node's slab of device partner links
  uint32_t pent_cap = 0, plist_cap = 0;    // its pair block slabs
  uint32_t x_slots = 0;                    // sharded: may-merge slots with a foreign partner
  uint32_t sub_gen = 0, shr_gen = 0;       // when its subs / shared slab was filled (Index::fresh_gen;
                                           //   0: before the generation base)
  uint16_t depth = 0;
  bool live = false;
  bool retain_path = false;
};

// A subscription held by another shard, as this shard sees it (sharded index): what its
// partner links need — the filter's path, for co-matchability with this shard's filters.
struct ForeignSub {
  uint32_t client, fid, meta;  // meta: Qos | NoLocal (the bits Subscription.Merge takes)
  uint32_t path_off, depth;    // segment string ids in Index::fpaths_ (depth 0: a free entry)
};

class Index {
 public:
  explicit Index(uint64_t expected_subs = 0, uint64_t expected_nodes = 0);

  // Sharded index: this index holds shard `shard` of `n_shards`. Every update is
  // issued to every shard; each applies the part it owns — non-shared and shared subscriptions
  // by a hash of the full filter, inline subscriptions by identifier, retained messages by
  // topic — and records the other shards' non-shared subscriptions of its clients as foreign
  // partners (cross-shard merges). Returns the shard's own answer: the reference's return value
  // is the owner's (Subscribe, InlineSubscribe, RetainMessage: others return 0) or the OR over
  // shards (Unsubscribe / InlineUnsubscribe: particle exists, Q10). Call before any update.
  void set_shard(uint32_t shard, uint32_t n_shards);
  // The live host results (ViewTracker): set by the C-ABI when the index is created.
  void set_views(ViewTracker* v) { views_ = v; }
  bool views_live() const {  // a host span result is live (it may read the pools)
    if (!views_) return false;
    std::lock_guard<std::mutex> g(views_->mu);
    return !views_->live.empty();
  }
  uint64_t retired_slabs() const { return retired_.size(); }
  uint32_t shard() const { return shard_; }
  uint32_t n_shards() const { return n_shards_; }
  bool sharded() const { return n_shards_ > 1; }
  static uint32_t shard_hash(std::string_view key);  // owner = shard_hash(key) % n_shards

  // TopicsIndex API (topics.go:368-476); semantics and return values as the reference.
  int subscribe(std::string_view filter, uint32_t client, uint32_t filter_id, uint8_t qos,
                uint8_t flags, int32_t ident);
  int unsubscribe(std::string_view filter, uint32_t client);
  int inline_subscribe(std::string_view filter, int32_t ident, uint32_t filter_id);
  int inline_unsubscribe(std::string_view filter, int32_t ident);
  int64_t retain_message(std::string_view topic, uint64_t handle, uint32_t payload_len,
                         bool retain);
  // Restore path (server.go:1624-1640 loadSubscriptions, 1688-1692 loadRetained): the same as
  // calling subscribe / retain_message per entry, in order. On an empty index the image is
  // built directly in parallel passes (index_bulk.cpp); otherwise entry by entry.
  void subscribe_bulk(const uint8_t* bytes, const uint64_t* offs, const uint32_t* client_ids,
                      const uint32_t* filter_ids, const uint8_t* qos, const uint8_t* flags,
                      const int32_t* idents, uint64_t n, uint8_t* out_new);
  void retain_bulk(const uint8_t* bytes, const uint64_t* offs, const uint64_t* handles, uint64_t n);
  bool empty_image() const;
  int retained_delete(std::string_view topic);
  int retained_set(std::string_view topic, uint64_t handle, uint32_t payload_len, bool retain);
  uint64_t retained_len() const { return n_retained_; }

  // Device image (layout.h); the Device uploads dirty pages of these.
  Mirror<EdgeSlot> edges;
  Mirror<NodeWalk> walk;
  Mirror<NodeLists> lists;
  Mirror<NodeInl> inls;       // per node: its inline subscriptions (NodeLists kFlagInline)
  Mirror<NodeMsg> msg;
  Mirror<SegInfo> seginfo;
  Mirror<uint8_t> segbytes;
  SlabPool<SubRec> subs;
  SlabPool<uint32_t> parts;   // host only: partner node ids of each may-merge slot
  Mirror<MergeRef> mref;      // device partner links (layout.h), parallel to subs, and
  SlabPool<MergePart> mpart;  // pair blocks, rebuilt per node by flush_merge()
  Mirror<NodePair> npair;
  SlabPool<PairEnt> pent;
  SlabPool<PairSlot> plist;
  SlabPool<ShrRec> shr;
  SlabPool<InlRec> inl;
  SlabPool<ChildRec> children;  // per node: its children (NodeMsg.child_off/child_cnt)
  Mirror<XInfo> xinfo;          // sharded only (empty otherwise): per node fid + rank key
  Mirror<DeepTail> deep;        // sharded only: deep filters' codes beyond 32 levels, by fid
  Mirror<uint32_t> deep_codes;  //   (layout.h DeepTail; empty while no filter is that deep)
  // Retained packet stored on topic "" (retainPath "" is "no path", Q6): literal-final
  // lookups of particles without a retain path read this entry (topics.go:573).
  bool empty_topic_live = false;
  bool empty_topic_retain = false;
  uint64_t empty_topic_handle = 0;

  uint64_t edge_mask() const { return edges.size() - 1; }
  uint64_t n_nodes() const { return n_live_nodes_; }
  uint64_t n_wild_nodes() const { return n_wild_nodes_; }  // '+' / '#' particles
  uint32_t max_sub_cap() const { return max_sub_cap_; }     // the largest subscription slab ever
  bool deep_live() const { return n_deep_live_ != 0; }       // a filter deeper than 32 levels is known
  uint64_t n_edges() const { return n_edges_; }
  // edge table: at most 1/load of its slots used (MQ_OPT_EDGE_LOAD); from the next growth. A
  // table of 2^30 slots or more keeps load <= 1/2 (32 GB of slots at 2^30).
  void set_edge_load(uint32_t load) { edge_load_ = load; }
  // HBM the edge table may take at a load sparser than 1/4 (0: no limit); mq_index_create sets it
  // from the device's memory, so that several indexes on one GPU, or one far larger than config 3,
  // fall back to 1/4 instead of running out
  void set_edge_budget(uint64_t bytes) { edge_budget_ = bytes; }
  uint32_t edge_load_at(size_t cap) const {  // (non-increasing in cap: the growth loops converge)
    if (cap >= (size_t(1) << 30)) return 2u;
    if (edge_budget_ && edge_load_ > 4 && cap * sizeof(EdgeSlot) > edge_budget_) return 4u;
    return edge_load_;
  }
  uint64_t n_subs_merge() const { return n_merge_; }
  uint32_t max_depth() const { return max_depth_; }
  uint64_t version() const { return version_; }
  // bumped by every change of the retained state (live set or handles): the device's Messages
  // image is rebuilt when it moved
  uint64_t retained_version() const { return retained_version_; }
  uint32_t node_slots() const { return (uint32_t)nh_.size(); }  // node ids are below this
  // Rebuild the device partner links of nodes whose may-merge slots, partner lists or
  // partners' positions changed since the last call (the Device calls this before uploading).
  // O(partner links of those nodes).
  void flush_merge();
  uint64_t merge_links() const { return mpart.live; }
  uint64_t foreign_subs() const { return fsub_pos_.size(); }
  // Flush, then verify the device-bound invariants (mq_index_check); false + reason on the
  // first violation.
  bool check(std::string* why);

 private:
  // path of `filter` from isolateParticle depth d on (topics.go:479-496 / 499-513)
  static void path_of(std::string_view filter, int d, std::vector<std::string_view>& out);
  uint32_t set(std::string_view filter, int d);           // create path, return node
  uint32_t seek(std::string_view filter, int d) const;    // find path or kNone
  void trim(uint32_t n);                                  // topics.go:516-522
  uint32_t find_child(uint32_t parent, const SegKey& k, std::string_view seg) const;
  uint32_t new_node(uint32_t parent, std::string_view seg, const SegKey& k);
  void remove_node(uint32_t n);
  // Refresh n's entry in its parent's children slab from msg[n] (after any NodeMsg change).
  void child_rec_sync(uint32_t n);
  void add_below_live(uint32_t n, int delta);
  void edge_insert(uint32_t parent, const SegKey& k, uint32_t child, uint32_t plus = kNone, uint32_t hash = kNone);
  // Copy n's '+' / '#' children (NodeWalk) into n's incoming edge slot (EdgeSlot.plus / hash).
  void edge_walk_sync(uint32_t n);
  void edge_erase(uint32_t parent, const SegKey& k, uint32_t child);
  void edge_rehash(size_t cap, unsigned threads = 1);
  uint32_t intern_str(std::string_view s);

  // subscription list primitives (positions are absolute pool indices)
  void sub_ensure(uint32_t n, uint32_t need);
  uint32_t sub_add(uint32_t n, const SubRec& r, bool merge);
  void sub_remove(uint32_t n, uint32_t pos);
  void sub_set_merge(uint32_t n, uint32_t pos, bool merge);
  bool compatible(uint32_t a, uint32_t b) const;
  bool compatible_foreign(uint32_t a, const ForeignSub& f) const;
  static bool compatible_strs(const uint32_t* pa, int la, const uint32_t* pb, int lb);
  void path_strs(uint32_t n, uint32_t* out, int* len) const;
  // bulk build helpers (index_bulk.cpp)
  struct BulkItem;
  void bulk_trie(std::vector<BulkItem>& items, const uint8_t* bytes, unsigned threads);
  void bulk_children(uint32_t first_new, unsigned threads);
  // sharded: a non-shared subscription owned by another shard (Subscribe / Unsubscribe)
  int foreign_subscribe(std::string_view filter, uint32_t client, uint32_t fid, uint32_t meta);
  void foreign_unsubscribe(uint32_t client, uint32_t fid);
  uint32_t partner_meta(uint32_t partner, uint32_t client) const;  // Qos | NoLocal of a partner
  // client's slot at partner node p carries a changed Qos / NoLocal in its partner links
  void touch_partner(uint32_t p, uint32_t client) {
    uint32_t pos;
    if (!(p & kForeign) && sub_pos_.get((uint64_t)p << 32 | client, &pos)) merge_dirty_slot(p, pos);
  }
  // (mark = false: a parallel bulk build, which marks the whole array dirty itself)
  void set_rank(uint32_t n, uint32_t parent, std::string_view seg, bool mark = true);
  // a deep filter's DeepTail from its segment string ids (path_strs / fpaths_: 0 '+', 1 '#')
  // Each call is one reference to fid's entry (a node that took fid, or a foreign subscription);
  // deep_unref drops one, and the entry goes (a tombstone) with the last, so a filter id that is
  // reused for another filter never finds a stale entry.
  void note_deep(uint32_t fid, const uint32_t* segs, uint32_t depth);
  void note_deep_node(uint32_t n, uint32_t fid);
  void deep_unref(uint32_t fid);
  void deep_rebuild(size_t slots);  // live entries only into `slots` slots, codes compacted
  size_t deep_find(uint32_t fid) const;  // fid's slot, or the free slot that ends its probe
  uint32_t n_deep_ = 0;       // used slots, tombstones included (the table's load)
  uint32_t n_deep_live_ = 0;  // entries
  size_t deep_garbage_ = 0;   // words of deep_codes no entry names
  std::unordered_map<uint32_t, uint32_t> deep_refs_;
  // (mark = false: the whole list moves to a new slab; no slot changes its place k)
  void move_slot(uint32_t n, uint32_t from, uint32_t to, bool mark = true);
  void part_set(uint32_t pos, const std::vector<uint32_t>& nodes);
  void part_add(uint32_t pos, uint32_t node);
  uint32_t part_remove(uint32_t pos, uint32_t node);
  void part_release(uint32_t pos);

  template <class T, class Rec>
  void list_push(SlabPool<T>& pool, uint32_t& off, uint32_t& cnt, uint32_t& cap, const Rec& r);
  // copy-on-write against live host results (ViewTracker)
  void begin_op();  // an update starts: snapshot the live results; free what none of them can see
  bool seen(uint32_t g) const { return op_max_ && (g == 0 || op_max_ >= gen_base_ + g); }
  uint32_t fresh_gen();  // the generation of a slab filled now
  void retire(int pool, uint32_t off, uint32_t cap);  // pool 0 subs, 1 shr: free now or once unseen
  void sub_cow(uint32_t n);  // n's subs slab moves to a copy if a live result may see it
  void sub_move(uint32_t n, uint32_t nc);
  uint32_t cow_pos(uint32_t n, uint32_t pos);  // sub_cow, then pos's place in the (new) slab
  void shr_cow(uint32_t n);
  template <class T>
  void guard_growth(Mirror<T>& m, size_t need, std::deque<std::pair<uint64_t, std::vector<T>>>& keep);

  bool sub_is_merge(uint32_t n, uint32_t pos) const { return pos >= lists.h[n].sub_off + lists.h[n].n_direct; }
  void merge_dirty(uint32_t n) {
    if (n >= merge_dirty_flag_.size()) merge_dirty_flag_.resize(nh_.size() > n ? nh_.size() : n + 1, 0);
    if (!merge_dirty_flag_[n]) {
      merge_dirty_flag_[n] = 1;
      merge_dirty_.push_back(n);
    }
  }
  // the slot at pool position pos of n changed (its record, partners or place): n's merge records
  // are stale; a node updated incrementally also notes the slot's place
  void merge_dirty_slot(uint32_t n, uint32_t pos) {
    merge_dirty(n);
    auto it = minc_.find(n);
    if (it != minc_.end()) it->second.dirty.push_back(pos - lists.h[n].sub_off);
  }
  void merge_release(uint32_t n);
  // npair[n] = P, and the copy of its header in lists[n] (the walk's epilogue reads that one)
  void set_pair_header(uint32_t n, const NodePair& P) {
    npair.at_w(n) = P;
    if (lists.h[n].ent_off != P.ent_off || lists.h[n].ent_mask != P.ent_mask) {
      NodeLists& L = lists.at_w(n);
      L.ent_off = P.ent_off;
      L.ent_mask = P.ent_mask;
    }
  }
  // Merge records of a node with many partner links, updated in place (flush_merge): the
  // changed slots are taken off the pair lists and put back, instead of rebuilding the node's
  // links and pair block (a hot node's block is megabytes). Host only.
  struct MergeInc {
    struct Slot {
      uint32_t mp_off = 0, mp_cnt = 0, mp_cap = 0;  // its MergePart records; mp_cap | kPairBase: in the base slab
    };
    std::vector<Slot> slot;       // by place k in the node's subscription list
    std::vector<uint32_t> dirty;  // places changed since the last flush
    HashU64 where{64};            // (h << 32 | k) -> index of slot k on the list of partner node h
    uint64_t links = 0;           // MergePart records in use (= pair-list entries)
    uint64_t garbage = 0;         // records of the base slabs no longer in use
  };
  static constexpr uint64_t kIncLinks = 256;  // nodes with this many partner links update in place
  void merge_rebuild(uint32_t n);
  void merge_patch(uint32_t n, MergeInc& I);
  uint32_t pair_find(const NodePair& P, uint32_t h) const;  // pent index of partner h, or kNone
  void pair_add(uint32_t n, MergeInc& I, uint32_t h, const PairSlot& ps);
  void pair_remove(uint32_t n, MergeInc& I, uint32_t h, uint32_t k);
  void pair_rehash(uint32_t n, uint32_t ecap);
  uint32_t sub_count(uint32_t n) const { return lists[n].n_direct + lists[n].n_merge; }

  ViewTracker* views_ = nullptr;
  uint64_t op_gen_ = 0, op_max_ = 0;  // this update's snapshot: generations handed out, newest live (0: none)
  uint64_t gen_base_ = 0;             // NodeHost gens count from here
  struct Retired {
    uint64_t tag;  // freed once no live result is this old
    int pool;
    uint32_t off, cap;
  };
  std::deque<Retired> retired_;
  std::deque<std::pair<uint64_t, std::vector<SubRec>>> retired_subs_;  // outgrown pool buffers
  std::deque<std::pair<uint64_t, std::vector<ShrRec>>> retired_shr_;
  PodVec<NodeHost> nh_;
  std::vector<uint32_t> free_nodes_;
  uint64_t n_live_nodes_ = 0, n_edges_ = 0, n_tombs_ = 0, n_merge_ = 0;
  uint64_t n_wild_nodes_ = 0;
  uint32_t max_sub_cap_ = 0;
  // sparser than 1/2: shorter probe chains (r02 k_walk at 10M: 1/2 1.90 ms, 1/4 1.64 ms; round 4,
  // the frontier walk with the fused desc: 1/4 1.204 ms, 1/8 1.079 ms, 1/16 1.027 ms — 17 GB of
  // HBM at 10M subscriptions, profiles/r04/y/, r04/yb/)
  uint32_t edge_load_ = 16;
  uint64_t edge_budget_ = 0;
  uint32_t max_depth_ = 0;
  uint64_t version_ = 0;
  uint64_t retained_version_ = 0;

  StrTable strs_;
  std::unordered_map<std::string, uint32_t> long_segs_;  // long segment -> SegInfo index
  std::unordered_map<std::string, uint32_t> group_ids_;

  HashU64 sub_pos_{1024};  // (node << 32 | client) -> pool position
  HashU64 inl_pos_{64};    // (node << 32 | ident) -> pool position
  struct ShrKey {
    uint32_t node, group, client;
    bool operator==(const ShrKey& o) const {
      return node == o.node && group == o.group && client == o.client;
    }
  };
  struct ShrKeyHash {
    size_t operator()(const ShrKey& k) const {
      return (size_t)mix64(((uint64_t)k.node << 32 | k.client) ^ ((uint64_t)k.group * 0x9e3779b97f4a7c15ull));
    }
  };
  std::unordered_map<ShrKey, uint32_t, ShrKeyHash> shr_pos_;
  std::vector<uint32_t> shr_group_;  // group id per shared pool position
  struct PartList {
    uint32_t off, cnt, cap;
  };
  std::vector<PartList> subp_;       // each slot's partner slab
  std::vector<uint32_t> merge_dirty_;  // nodes whose device partner links are stale
  std::vector<uint8_t> merge_dirty_flag_;
  std::unordered_map<uint32_t, MergeInc> minc_;  // nodes whose merge records update in place
  std::unordered_map<uint32_t, std::vector<uint32_t>> client_nodes_;  // non-shared subs
  uint64_t n_retained_ = 0;  // live Retained entries (topic "" included)
  // sharding
  uint32_t shard_ = 0, n_shards_ = 1;
  std::vector<ForeignSub> fsubs_;
  std::vector<uint32_t> fsub_free_;
  HashU64 fsub_pos_{64};  // (fid << 32 | client) -> fsubs_ index
  std::unordered_map<uint32_t, std::vector<uint32_t>> client_foreign_;  // client -> fsubs_ indices
  std::vector<uint32_t> fpaths_;                                         // foreign filters' segment ids
  StrTable ffilt_;                   // foreign non-shared filter strings -> ffid_ index
  std::vector<uint32_t> ffid_;       // their caller filter ids
};

// strings.EqualFold(s, "$SHARE") under Go's Unicode simple folding (Q9: U+017F ~ 's').
bool is_share_prefix(std::string_view s);
// isolateParticle(filter, d)'s value (topics.go:679-698)
std::string_view segment_at(std::string_view filter, int d);
// the key a sharded index owns a subscription by (index.cpp)
std::string shard_key(std::string_view filter, bool share);

}  // namespace mq
