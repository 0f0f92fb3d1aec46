// Bulk build of the host image for the restore path (server.go:1624-1640
// loadSubscriptions, server.go:1688-1692 loadRetained): the stored subscriptions / retained
// messages are replayed into an empty index. Instead of one Subscribe / RetainMessage per entry
// (each a root-to-leaf walk creating particles one at a time), the trie is built level by
// level — every entry's next segment is keyed, the (parent, segment) pairs are de-duplicated in
// hash partitions on all threads, and the new particles get consecutive ids (BFS order) — and
// the subscription lists, partner links and children slabs are laid out by sorting and
// counting. The result is the image the per-entry path would build (node ids aside), with the
// same answers (out_new) and the same invariants (mq_index_check); an index that is not empty
// takes the per-entry path.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <stdexcept>

#include "index.h"

namespace mq {

namespace {

unsigned build_threads() {
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  return std::min(16u, hw);
}

constexpr uint32_t kParts = 64;  // hash partitions of a level's (parent, segment) keys

// Sort v by `less` on `threads` threads: a stable partition into nb buckets by bucket(x) < nb
// (which must not decrease along `less`), then every bucket sorted on its own.
template <class T, class Bucket, class Less>
void bucket_sort(std::vector<T>& v, unsigned threads, uint32_t nb, Bucket&& bucket, Less&& less) {
  const size_t n = v.size();
  if (n < 65536) {
    std::sort(v.begin(), v.end(), less);
    return;
  }
  const unsigned chunks = std::max(1u, std::min<unsigned>(threads * 4, (unsigned)(n / 65536)));
  std::vector<uint64_t> cnt((size_t)chunks * nb, 0), at((size_t)chunks * nb);
  parallel_for(chunks, chunks, [&](size_t cb, size_t ce) {
    for (size_t c = cb; c < ce; c++)
      for (size_t i = n * c / chunks; i < n * (c + 1) / chunks; i++) cnt[c * nb + bucket(v[i])]++;
  });
  std::vector<uint64_t> off(nb + 1);
  uint64_t run = 0;
  for (uint32_t b = 0; b < nb; b++) {
    off[b] = run;
    for (unsigned c = 0; c < chunks; c++) {
      at[(size_t)c * nb + b] = run;
      run += cnt[(size_t)c * nb + b];
    }
  }
  off[nb] = run;
  std::vector<T> tmp(n);
  parallel_for(chunks, chunks, [&](size_t cb, size_t ce) {
    for (size_t c = cb; c < ce; c++)
      for (size_t i = n * c / chunks; i < n * (c + 1) / chunks; i++) tmp[at[c * nb + bucket(v[i])]++] = v[i];
  });
  std::atomic<uint32_t> next{0};
  std::vector<std::thread> th;
  for (unsigned t = 0; t < threads; t++)
    th.emplace_back([&] {
      for (uint32_t b; (b = next.fetch_add(1)) < nb;) std::sort(tmp.begin() + off[b], tmp.begin() + off[b + 1], less);
    });
  for (auto& x : th) x.join();
  v.swap(tmp);
}

// Buckets for keys below `limit`: a power-of-two count (about 64 per thread) and the shift that
// maps a key to its bucket.
inline uint32_t bucket_shift(uint64_t limit, unsigned threads, uint32_t* nb) {
  uint32_t bits = 1;
  while ((1ull << bits) < limit) bits++;
  uint32_t want = 1;
  while (want < threads * 64) want <<= 1;
  uint32_t wb = 0;
  while ((1u << wb) < want) wb++;
  const uint32_t shift = bits > wb ? bits - wb : 0;
  *nb = (uint32_t)(((limit - 1) >> shift) + 1);
  return shift;
}

// Stable partition of 0..n-1 by part(i) < nparts on `threads` threads (count, prefix, scatter):
// the members of part p are flat[offs[p] .. offs[p + 1]), in increasing order.
template <class Part>
void partition_ids(uint32_t n, uint32_t nparts, unsigned threads, Part&& part, std::vector<uint32_t>& flat,
                   std::vector<uint64_t>& offs) {
  const unsigned chunks = std::max(1u, std::min<unsigned>(threads * 4, (n + 65535) / 65536));
  std::vector<uint8_t> pid(n);  // nparts <= 256
  std::vector<uint64_t> cnt((size_t)chunks * nparts, 0);
  parallel_for(chunks, chunks, [&](size_t cb, size_t ce) {
    for (size_t c = cb; c < ce; c++)
      for (uint64_t i = (uint64_t)n * c / chunks; i < (uint64_t)n * (c + 1) / chunks; i++) {
        pid[i] = (uint8_t)part((uint32_t)i);
        cnt[c * nparts + pid[i]]++;
      }
  });
  offs.assign(nparts + 1, 0);
  std::vector<uint64_t> at((size_t)chunks * nparts);
  uint64_t run = 0;
  for (uint32_t p = 0; p < nparts; p++) {
    offs[p] = run;
    for (unsigned c = 0; c < chunks; c++) {
      at[(size_t)c * nparts + p] = run;
      run += cnt[(size_t)c * nparts + p];
    }
  }
  offs[nparts] = run;
  flat.resize(n);
  parallel_for(chunks, chunks, [&](size_t cb, size_t ce) {
    for (size_t c = cb; c < ce; c++)
      for (uint64_t i = (uint64_t)n * c / chunks; i < (uint64_t)n * (c + 1) / chunks; i++)
        flat[at[c * nparts + pid[i]]++] = (uint32_t)i;
  });
}

// f(p) for every partition p on up to `threads` threads, partitions handed out one at a time
// (parallel_for's 4096-item grain would run 64 partitions on one thread).
template <class F>
void for_parts(unsigned threads, F&& f) {
  std::atomic<uint32_t> next{0};
  std::vector<std::thread> th;
  for (unsigned t = 0; t < std::min<unsigned>(threads, kParts); t++)
    th.emplace_back([&] {
      for (uint32_t p; (p = next.fetch_add(1)) < kParts;) f(p);
    });
  for (auto& x : th) x.join();
}

}  // namespace

// One path being built: its next segment starts at `cur` (absolute offset into the bytes),
// the path ends at `end`; `node` is the particle reached so far.
struct Index::BulkItem {
  uint64_t cur, end;
  uint32_t node;
  bool done;
};

bool Index::empty_image() const {
  return n_live_nodes_ == 0 && subs.live == 0 && shr.live == 0 && inl.live == 0 && n_retained_ == 0 &&
         fsub_pos_.size() == 0;
}

// Level-synchronous trie build for items[] on an empty index: on return every item's `node` is
// its path's particle (Index::set semantics, topics.go:479-496), and every new particle has its
// records, edge and children slab.
void Index::bulk_trie(std::vector<BulkItem>& items, const uint8_t* bytes, unsigned threads) {
  const uint32_t first_new = (uint32_t)nh_.size();
  std::vector<uint64_t> rep_off;  // per new node: its segment's bytes (a representative item's)
  std::vector<uint32_t> rep_len, node_parent, level_end;
  std::vector<uint32_t> active(items.size());
  for (uint32_t i = 0; i < items.size(); i++) active[i] = i;
  std::vector<SegKey> key;
  std::vector<uint64_t> seg_beg;
  std::vector<uint32_t> seg_len, part, order, local;
  {  // every particle this build can create, reserved once (no reallocation per level)
    std::atomic<uint64_t> segs{0};
    parallel_for(items.size(), threads, [&](size_t b, size_t e) {
      uint64_t c = 0;
      for (size_t j = b; j < e; j++) {
        const uint8_t* p = bytes + items[j].cur;
        const uint8_t* end = bytes + items[j].end;
        c++;
        while ((p = (const uint8_t*)memchr(p, '/', end - p)) != nullptr) c++, p++;
      }
      segs += c;
    });
    nh_.reserve_huge(nh_.size() + segs.load());  // an upper bound: reserved, not touched
    reserve_huge(rep_off, segs.load());
    reserve_huge(rep_len, segs.load());
    reserve_huge(node_parent, segs.load());
  }
  struct Slot {  // a partition's dedup table entry
    uint64_t k0, k1;
    uint32_t parent, j;  // j = kNone: empty
  };
  while (!active.empty()) {
    const size_t na = active.size();
    key.resize(na);
    seg_beg.resize(na);
    seg_len.resize(na);
    part.resize(na);
    local.resize(na);
    // 1. every active item's next segment and its key
    parallel_for(na, threads, [&](size_t b, size_t e) {
      for (size_t j = b; j < e; j++) {
        const BulkItem& it = items[active[j]];
        const uint8_t* p = bytes + it.cur;
        const void* sl = memchr(p, '/', it.end - it.cur);
        const uint64_t se = sl ? (uint64_t)((const uint8_t*)sl - bytes) : it.end;
        seg_beg[j] = it.cur;
        seg_len[j] = (uint32_t)(se - it.cur);
        key[j] = seg_key(p, seg_len[j]);
        part[j] = (uint32_t)(edge_hash(it.node, key[j]) >> 40) % kParts;
      }
    });
    // 2. group by partition (stable), then de-duplicate each partition's (parent, key) pairs on
    // its own thread; a new pair's local id is its first appearance's rank
    std::vector<uint32_t> pcnt(kParts + 1, 0);
    for (size_t j = 0; j < na; j++) pcnt[part[j] + 1]++;
    for (uint32_t p = 0; p < kParts; p++) pcnt[p + 1] += pcnt[p];
    order.resize(na);
    {
      std::vector<uint32_t> at(pcnt.begin(), pcnt.end() - 1);
      for (size_t j = 0; j < na; j++) order[at[part[j]]++] = (uint32_t)j;
    }
    std::vector<uint32_t> uniq(kParts, 0);
    std::vector<std::vector<uint32_t>> reps(kParts);  // per partition: the first item of each new pair
    for_parts(threads, [&](uint32_t p) {
      std::vector<Slot> table;
      {
        const uint32_t lo = pcnt[p], hi = pcnt[p + 1];
        size_t cap = 16;
        while (cap < 2 * (size_t)(hi - lo)) cap <<= 1;
        table.assign(cap, Slot{0, 0, 0, kNone});
        reps[p].reserve(hi - lo);
        for (uint32_t q = lo; q < hi; q++) {
          const uint32_t j = order[q];
          const uint32_t parent = items[active[j]].node;
          const SegKey& k = key[j];
          size_t s = edge_hash(parent, k) & (cap - 1);
          for (;;) {
            Slot& e = table[s];
            if (e.j == kNone) {
              e = Slot{k.k0, k.k1, parent, j};
              local[j] = uniq[p]++;
              reps[p].push_back(j);
              break;
            }
            if (e.parent == parent && e.k0 == k.k0 && e.k1 == k.k1 &&
                (!seg_is_long(k) ||
                 (seg_len[e.j] == seg_len[j] && memcmp(bytes + seg_beg[e.j], bytes + seg_beg[j], seg_len[j]) == 0))) {
              local[j] = local[e.j];
              break;
            }
            s = (s + 1) & (cap - 1);
          }
        }
      }
    });
    // 3. ids: partitions in order, pairs in first-appearance order within each
    std::vector<uint32_t> base(kParts + 1, (uint32_t)nh_.size());
    for (uint32_t p = 0; p < kParts; p++) base[p + 1] = base[p] + uniq[p];
    const uint32_t n1 = base[kParts];
    nh_.resize(n1, threads);
    rep_off.resize(n1 - first_new);
    rep_len.resize(n1 - first_new);
    node_parent.resize(n1 - first_new);
    for_parts(threads, [&](uint32_t p) {
        for (uint32_t k = 0; k < uniq[p]; k++) {
          const uint32_t j = reps[p][k], id = base[p] + k;
          rep_off[id - first_new] = seg_beg[j];
          rep_len[id - first_new] = seg_len[j];
          node_parent[id - first_new] = items[active[j]].node;
          nh_[id].key = key[j];
        }
    });
    level_end.push_back(n1);
    // 4. advance the items; drop the finished ones
    parallel_for(na, threads, [&](size_t b, size_t e) {
      for (size_t j = b; j < e; j++) {
        BulkItem& it = items[active[j]];
        it.node = base[part[j]] + local[j];
        const uint64_t se = seg_beg[j] + seg_len[j];
        if (se >= it.end) it.done = true;
        else it.cur = se + 1;
      }
    });
    size_t w = 0;
    for (size_t j = 0; j < na; j++)
      if (!items[active[j]].done) active[w++] = active[j];
    active.resize(w);
  }

  const uint32_t n_end = (uint32_t)nh_.size(), n_new = n_end - first_new;
  // The particles' device-mirrored records and the edge table, grown on threads of their own
  // (first touch of a few hundred MB each) while the strings are resolved.
  std::vector<std::thread> grow;
  grow.emplace_back([&] {
    walk.reserve_resident(n_end, threads);
    walk.grow_to(n_end, NodeWalk{kNone, kNone, 0, kNone});
  });
  grow.emplace_back([&] {
    lists.reserve_resident(n_end, threads);
    lists.grow_to(n_end, kEmptyLists);
    inls.grow_to(n_end, NodeInl{0, 0});
  });
  grow.emplace_back([&] {
    msg.reserve_resident(n_end, threads);
    msg.grow_to(n_end, NodeMsg{});
  });
  grow.emplace_back([&] {
    npair.reserve_resident(n_end, threads);
    npair.grow_to(n_end, NodePair{0, kNone, 0, 0});
    if (sharded()) xinfo.grow_to(n_end, XInfo{kNone, 0, 0});
  });
  grow.emplace_back([&] {  // sized for every particle at load <= 1/edge_load_ (default 1/16; 2^30+ slots keep 1/2)
    size_t cap = 1024;
    while (cap < edge_load_at(cap) * ((size_t)n_edges_ + n_new + 1)) cap <<= 1;
    if (cap > edges.size()) edge_rehash(cap, threads);
  });
  // Segment strings: interned once per distinct segment (a level holds few: the topic
  // vocabulary), found by every particle through a key -> string id table.
  std::vector<uint32_t> str(n_new, kNone);
  {
    struct KS {
      uint64_t k0, k1;
      uint32_t str;
    };
    // inline keys by hash into kParts partitions, long ones into partition kParts
    std::vector<uint32_t> pk;
    std::vector<uint64_t> po;
    partition_ids(n_new, kParts + 1, threads, [&](uint32_t k) {
      const SegKey& sk = nh_[first_new + k].key;
      return seg_is_long(sk) ? kParts : (uint32_t)(mix64(sk.k0 ^ (sk.k1 * 0x9e3779b97f4a7c15ull)) % kParts);
    }, pk, po);
    std::vector<std::vector<uint32_t>> firsts(kParts);  // per partition: keys seen first, to intern
    std::vector<std::vector<KS>> tabs(kParts);
    auto slot = [&](const std::vector<KS>& t, const SegKey& sk) {
      size_t i = mix64(sk.k0 + sk.k1) & (t.size() - 1);
      while (t[i].str != kNone && !(t[i].k0 == sk.k0 && t[i].k1 == sk.k1)) i = (i + 1) & (t.size() - 1);
      return i;
    };
    auto grow = [&](std::vector<KS>& t) {  // a level holds few distinct segments: tables start small
      std::vector<KS> old(t.size() * 2, KS{0, 0, kNone});
      old.swap(t);
      for (const KS& e : old)
        if (e.str != kNone) t[slot(t, SegKey{e.k0, e.k1})] = e;
    };
    auto seg_of = [&](uint32_t k) { return std::string_view((const char*)bytes + rep_off[k], rep_len[k]); };
    for_parts(threads, [&](uint32_t p) {
      std::vector<KS>& t = tabs[p];
      t.assign(1024, KS{0, 0, kNone});
      size_t used = 0;
      for (uint64_t q = po[p]; q < po[p + 1]; q++) {
        const uint32_t k = pk[q];
        const SegKey& sk = nh_[first_new + k].key;
        if (t[slot(t, sk)].str != kNone) continue;
        if (2 * ++used > t.size()) grow(t);
        KS& e = t[slot(t, sk)];
        e = KS{sk.k0, sk.k1, strs_.find(seg_of(k))};  // first particle with this segment
        if (e.str == kNone) {
          e.str = kNone - 1;  // to intern below (serially)
          firsts[p].push_back(k);
        }
      }
    });
    for (uint32_t p = 0; p < kParts; p++)
      for (uint32_t k : firsts[p]) tabs[p][slot(tabs[p], nh_[first_new + k].key)].str = intern_str(seg_of(k));
    for_parts(threads, [&](uint32_t p) {
      const std::vector<KS>& t = tabs[p];
      for (uint64_t q = po[p]; q < po[p + 1]; q++) str[pk[q]] = t[slot(t, nh_[first_new + pk[q]].key)].str;
    });
    for (uint64_t q = po[kParts]; q < po[kParts + 1]; q++) str[pk[q]] = intern_str(seg_of(pk[q]));
  }
  // Node records, level by level (a level's parents are complete), each level on all threads.
  for (auto& t : grow) t.join();
  std::vector<uint32_t> segref(n_new, kNone);  // long segments' SegInfo (serial: rare)
  for (uint32_t k = 0; k < n_new; k++) {
    if (!seg_is_long(nh_[first_new + k].key)) continue;
    const std::string seg((const char*)bytes + rep_off[k], rep_len[k]);
    auto it = long_segs_.find(seg);
    if (it == long_segs_.end()) {
      const uint32_t ref = (uint32_t)seginfo.size(), off = (uint32_t)segbytes.size();
      segbytes.grow_to(off + seg.size(), 0);
      memcpy(&segbytes.h[off], seg.data(), seg.size());
      seginfo.grow_to(ref + 1, SegInfo{off, (uint32_t)seg.size()});
      it = long_segs_.emplace(seg, ref).first;
    }
    segref[k] = it->second;
  }
  uint32_t lo = first_new;
  for (uint32_t hi : level_end) {
    parallel_for(hi - lo, threads, [&](size_t b, size_t e) {
      uint32_t depth_max = 0;
      uint64_t wild = 0;
      for (size_t q = b; q < e; q++) {
        const uint32_t id = lo + (uint32_t)q, k = id - first_new, parent = node_parent[k];
        NodeHost& h = nh_[id];
        const std::string_view seg((const char*)bytes + rep_off[k], rep_len[k]);
        h.str = str[k];
        h.depth = (uint16_t)(nh_[parent].depth + 1);
        h.seg0 = parent == kRoot ? h.str : nh_[parent].seg0;
        h.live = true;
        wild += h.str <= 1;
        depth_max = std::max<uint32_t>(depth_max, h.depth);
        uint32_t flags = 0;
        if (h.str == 0) flags |= kFlagPlusKey;
        if (parent == kRoot) {
          if (!seg.empty() && (seg[0] == '+' || seg[0] == '#')) flags |= kFlagSeg0Wild;
        } else {
          flags |= walk.h[parent].parent_flags & kFlagSeg0Wild;
        }
        walk.h[id] = NodeWalk{kNone, kNone, parent | flags, segref[k]};
        NodeLists L = kEmptyLists;
        L.flags = flags & kFlagSeg0Wild;
        lists.h[id] = L;
        NodeMsg M{};
        M.parent = parent;
        M.flags = (parent == kRoot && seg == "$SYS") ? kChildSys : 0u;
        msg.h[id] = M;
        if (h.str == 0) walk.h[parent].plus_child = id;  // a parent has one "+" and one "#" child
        if (h.str == 1) walk.h[parent].hash_child = id;
        __atomic_fetch_add(&nh_[parent].n_children, 1u, __ATOMIC_RELAXED);
        if (sharded()) set_rank(id, parent, seg, false);
      }
      __atomic_fetch_add(&n_wild_nodes_, wild, __ATOMIC_RELAXED);
      uint32_t cur = __atomic_load_n(&max_depth_, __ATOMIC_RELAXED);
      while (depth_max > cur && !__atomic_compare_exchange_n(&max_depth_, &cur, depth_max, true, __ATOMIC_RELAXED,
                                                             __ATOMIC_RELAXED)) {
      }
    });
    lo = hi;
  }
  n_live_nodes_ += n_new;
  // the edges, inserted by all threads (CAS)
  EdgeSlot* E = edges.h.data();
  const uint64_t em = edges.size() - 1;
  parallel_for(n_new, threads, [&](size_t b, size_t e) {
    for (size_t k = b; k < e; k++) {
      const uint32_t id = first_new + (uint32_t)k, parent = node_parent[k];
      const SegKey sk = nh_[id].key;
      uint64_t i = edge_hash(parent, sk) & em;
      for (;;) {
        uint32_t expect = kEdgeEmpty;
        if (__atomic_compare_exchange_n(&E[i].parent, &expect, parent, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
          E[i].k0 = sk.k0;
          E[i].k1 = sk.k1;
          E[i].child = id;
          E[i].plus = walk.h[id].plus_child;  // final: every level is built before the edges
          E[i].hash = walk.h[id].hash_child;
          break;
        }
        i = (i + 1) & em;
      }
    }
  });
  n_edges_ += n_new;
  edges.all_dirty = true;
  walk.all_dirty = lists.all_dirty = inls.all_dirty = msg.all_dirty = npair.all_dirty = true;
  if (sharded()) xinfo.all_dirty = true;
  bulk_children(first_new, threads);
}

// Children slabs of every particle that gained children in a bulk build: power-of-two slabs
// bump-allocated in id order (the image starts empty), positions taken atomically (Messages
// enumerates children in no particular order), ChildRec copies written once the particles'
// own slabs are known (retained state is copied again by retain_bulk).
void Index::bulk_children(uint32_t first_new, unsigned threads) {
  const uint32_t n_end = (uint32_t)nh_.size();
  // candidates: the root and every new particle; slab sizes, then offsets by a prefix sum
  const size_t m = (size_t)(n_end - first_new) + 1;
  auto cand = [&](size_t k) { return k == 0 ? kRoot : first_new + (uint32_t)(k - 1); };
  std::vector<uint64_t> off(m + 1, 0);
  parallel_for(m, threads, [&](size_t b, size_t e) {
    for (size_t k = b; k < e; k++) {
      const NodeHost& h = nh_[cand(k)];
      uint32_t c = 0;
      if (h.n_children && !h.child_cap) {
        c = 1;
        while (c < h.n_children) c <<= 1;
      }
      off[k + 1] = c;
    }
  });
  for (size_t k = 0; k < m; k++) off[k + 1] += off[k];
  const uint64_t base = children.m.size();
  if (base + off.back() >= (1ull << 32)) throw std::length_error("children pool beyond 2^32 entries");
  children.m.reserve_resident(base + off.back(), threads);
  children.m.grow_to(base + off.back(), ChildRec{0, 0, 0, 0, 0});
  parallel_for(m, threads, [&](size_t b, size_t e) {
    for (size_t k = b; k < e; k++) {
      if (off[k + 1] == off[k]) continue;
      const uint32_t v = cand(k);
      msg.h[v].child_off = (uint32_t)(base + off[k]);
      msg.h[v].child_cnt = 0;
      nh_[v].child_cap = (uint32_t)(off[k + 1] - off[k]);
    }
  });
  parallel_for(n_end - first_new, threads, [&](size_t b, size_t e) {
    for (size_t q = b; q < e; q++) {
      const uint32_t v = first_new + (uint32_t)q, p = msg.h[v].parent;
      const uint32_t pos = __atomic_fetch_add(&msg.h[p].child_cnt, 1u, __ATOMIC_RELAXED);
      nh_[v].child_pos = pos;
      msg.h[v].child_pos = pos;
    }
  });
  children.live += n_end - first_new;
  parallel_for(n_end - first_new, threads, [&](size_t b, size_t e) {
    for (size_t q = b; q < e; q++) {
      const uint32_t n = first_new + (uint32_t)q;
      const NodeMsg& M = msg.h[n];
      children.m.h[msg.h[M.parent].child_off + M.child_pos] = ChildRec{n, M.child_off, M.child_cnt, M.flags, M.handle};
    }
  });
  children.m.all_dirty = true;
  msg.all_dirty = true;
}

void Index::subscribe_bulk(const uint8_t* bytes, const uint64_t* offs, const uint32_t* client_ids,
                           const uint32_t* filter_ids, const uint8_t* qos, const uint8_t* flags,
                           const int32_t* idents, uint64_t n, uint8_t* out_new) {
  auto one = [&](uint64_t i) {
    const int r = subscribe(std::string_view((const char*)bytes + offs[i], offs[i + 1] - offs[i]), client_ids[i],
                            filter_ids[i], qos[i], flags[i], idents[i]);
    if (out_new) out_new[i] = (uint8_t)r;
  };
  // The per-entry path (copy-on-write against live results, as every update) unless the image is
  // empty and no result is live: the parallel build below lays the pools out afresh, over slabs
  // that a result from before the image emptied might still read.
  if (!empty_image() || n < 4096 || views_live()) {
    for (uint64_t i = 0; i < n; i++) one(i);
    return;
  }
  version_++;
  begin_op();
  const unsigned threads = build_threads();
  // 0. classify: this shard's non-shared / shared entries and their paths (Index::set(f, 0) /
  // set(f, 2), isolateParticle semantics for short shared filters, Q13); the rest is foreign
  std::vector<uint8_t> kind(n);  // 0 non-shared, 1 shared, 2 another shard's
  std::vector<BulkItem> items(n);
  parallel_for(n, threads, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; i++) {
      const std::string_view f((const char*)bytes + offs[i], offs[i + 1] - offs[i]);
      const bool share = is_share_prefix(segment_at(f, 0));
      kind[i] = share ? 1 : 0;
      if (sharded() && shard_hash(shard_key(f, share)) % n_shards_ != shard_) kind[i] = 2;
      BulkItem it{offs[i], offs[i + 1], kRoot, false};
      if (share) {
        const size_t s1 = f.find('/');
        const size_t s2 = s1 == std::string_view::npos ? s1 : f.find('/', s1 + 1);
        if (s2 != std::string_view::npos) it.cur = offs[i] + s2 + 1;  // segments 2..
        else {                                                        // the last segment
          const size_t l = f.rfind('/');
          it.cur = offs[i] + (l == std::string_view::npos ? 0 : l + 1);
        }
      }
      items[i] = it;
    }
  });
  std::vector<uint64_t> loc;  // this shard's entries
  for (uint64_t i = 0; i < n; i++)
    if (kind[i] != 2) loc.push_back(i);
  {
    std::vector<BulkItem> li(loc.size());
    for (size_t k = 0; k < loc.size(); k++) li[k] = items[loc[k]];
    bulk_trie(li, bytes, threads);
    for (size_t k = 0; k < loc.size(); k++) items[loc[k]].node = li[k].node;
  }
  if (out_new) memset(out_new, 0, n);

  // 1. non-shared: (particle, client) keeps its last entry (topics.go:413-415); out_new marks
  // the first. Sorted by (particle, client, entry).
  struct Ent {
    uint32_t node, client;
    uint64_t i;
  };
  std::vector<Ent> ns;
  for (uint64_t i : loc)
    if (kind[i] == 0) ns.push_back(Ent{items[i].node, client_ids[i], i});
  {
    uint32_t nb;
    const uint32_t sh = bucket_shift(nh_.size(), threads, &nb);
    bucket_sort(ns, threads, nb, [sh](const Ent& e) { return e.node >> sh; }, [](const Ent& a, const Ent& b) {
      return a.node != b.node ? a.node < b.node : (a.client != b.client ? a.client < b.client : a.i < b.i);
    });
  }
  std::vector<Ent> slots;  // one per (particle, client): the last entry
  slots.reserve(ns.size());
  for (size_t k = 0; k < ns.size(); k++) {
    const bool first = k == 0 || ns[k - 1].node != ns[k].node || ns[k - 1].client != ns[k].client;
    if (first && out_new) out_new[ns[k].i] = 1;
    const bool last = k + 1 == ns.size() || ns[k + 1].node != ns[k].node || ns[k + 1].client != ns[k].client;
    if (last) slots.push_back(ns[k]);
  }
  std::vector<Ent>().swap(ns);
  // 2. partners: per client, its particles pairwise (Index::compatible)
  std::vector<uint64_t> cn(slots.size());  // client << 32 | node
  for (size_t k = 0; k < slots.size(); k++) cn[k] = (uint64_t)slots[k].client << 32 | slots[k].node;
  {
    uint64_t max_c = 0;
    for (const Ent& e : slots) max_c = std::max<uint64_t>(max_c, e.client);
    uint32_t nb;
    const uint32_t sh = bucket_shift(max_c + 1, threads, &nb) + 32;
    bucket_sort(cn, threads, nb, [sh](uint64_t x) { return (uint32_t)(x >> sh); }, std::less<uint64_t>());
  }
  std::vector<size_t> cstart;  // client groups in cn
  for (size_t k = 0; k < cn.size(); k++)
    if (k == 0 || (cn[k] >> 32) != (cn[k - 1] >> 32)) cstart.push_back(k);
  cstart.push_back(cn.size());
  const size_t n_clients = cstart.size() - 1;
  std::vector<std::vector<std::pair<uint64_t, uint32_t>>> plinks(threads);  // (node << 32 | client, partner)
  {
    std::atomic<size_t> next{0};
    std::vector<std::thread> th;
    for (unsigned t = 0; t < threads; t++)
      th.emplace_back([&, t] {
        for (;;) {
          const size_t g0 = next.fetch_add(256);
          if (g0 >= n_clients) break;
          for (size_t g = g0; g < std::min(n_clients, g0 + 256); g++) {
            const size_t b = cstart[g], e = cstart[g + 1];
            if (e - b < 2) continue;
            const uint32_t c = (uint32_t)(cn[b] >> 32);
            for (size_t x = b; x < e; x++)
              for (size_t y = x + 1; y < e; y++) {
                const uint32_t a = (uint32_t)cn[x], d = (uint32_t)cn[y];
                if (!compatible(a, d)) continue;
                plinks[t].emplace_back((uint64_t)a << 32 | c, d);
                plinks[t].emplace_back((uint64_t)d << 32 | c, a);
              }
          }
        }
      });
    for (auto& x : th) x.join();
  }
  std::vector<std::pair<uint64_t, uint32_t>> links;
  for (auto& v : plinks) links.insert(links.end(), v.begin(), v.end());
  std::vector<std::vector<std::pair<uint64_t, uint32_t>>>().swap(plinks);
  {
    uint32_t nb;
    const uint32_t sh = bucket_shift(nh_.size(), threads, &nb) + 32;
    bucket_sort(links, threads, nb, [sh](const std::pair<uint64_t, uint32_t>& x) { return (uint32_t)(x.first >> sh); },
                [](const std::pair<uint64_t, uint32_t>& a, const std::pair<uint64_t, uint32_t>& b) {
                  return a.first != b.first ? a.first < b.first : a.second < b.second;
                });
  }
  // 3. subscription slabs: per particle [direct slots][may-merge slots], slots in client order
  std::vector<uint8_t> is_merge(slots.size(), 0);
  {
    size_t l = 0;
    for (size_t k = 0; k < slots.size(); k++) {
      const uint64_t key = (uint64_t)slots[k].node << 32 | slots[k].client;
      while (l < links.size() && links[l].first < key) l++;
      is_merge[k] = l < links.size() && links[l].first == key;
    }
  }
  std::vector<uint32_t> pos(slots.size());
  for (size_t b = 0; b < slots.size();) {
    size_t e = b;
    while (e < slots.size() && slots[e].node == slots[b].node) e++;
    const uint32_t node = slots[b].node, cnt = (uint32_t)(e - b);
    uint32_t c = 1;
    while (c < cnt) c <<= 1;
    NodeLists& L = lists.h[node];
    L.sub_off = subs.alloc(c);
    nh_[node].sub_cap = c;
    max_sub_cap_ = std::max(max_sub_cap_, c);
    uint32_t nd = 0;
    for (size_t k = b; k < e; k++) nd += !is_merge[k];
    L.n_direct = nd;
    L.n_merge = cnt - nd;
    uint32_t di = 0, mi = nd;
    for (size_t k = b; k < e; k++) pos[k] = L.sub_off + (is_merge[k] ? mi++ : di++);
    if (L.n_merge) merge_dirty(node);
    n_merge_ += L.n_merge;
    if (sharded() && xinfo.h[node].fid == kNone) {
      xinfo.h[node].fid = filter_ids[slots[b].i];
      note_deep_node(node, xinfo.h[node].fid);
    }
    b = e;
  }
  subp_.resize(subs.m.size(), PartList{0, 0, 0});
  parallel_for(slots.size(), threads, [&](size_t b, size_t e) {
    for (size_t k = b; k < e; k++) {
      const uint64_t i = slots[k].i;
      subs.m.h[pos[k]] = SubRec{client_ids[i], filter_ids[i], idents[i],
                                (uint32_t)(qos[i] & 3) | ((flags[i] & 1) ? kMetaNoLocal : 0) |
                                    ((flags[i] & 2) ? kMetaRap : 0) | ((uint32_t)((flags[i] >> 2) & 3) << kMetaRhShift)};
    }
  });
  subs.live += slots.size();
  {
    std::vector<uint64_t> keys(slots.size());
    for (size_t k = 0; k < slots.size(); k++) keys[k] = (uint64_t)slots[k].node << 32 | slots[k].client;
    sub_pos_.build_parallel(keys.data(), pos.data(), keys.size(), threads);
  }
  for (size_t l = 0; l < links.size();) {  // partner lists of the may-merge slots
    size_t e = l;
    while (e < links.size() && links[e].first == links[l].first) e++;
    uint32_t p;
    sub_pos_.get(links[l].first, &p);
    std::vector<uint32_t> part(e - l);
    for (size_t k = l; k < e; k++) part[k - l] = links[k].second;
    part_set(p, part);
    l = e;
  }
  client_nodes_.reserve(n_clients);
  for (size_t g = 0; g < n_clients; g++) {
    std::vector<uint32_t>& v = client_nodes_[(uint32_t)(cn[cstart[g]] >> 32)];
    for (size_t k = cstart[g]; k < cstart[g + 1]; k++) v.push_back((uint32_t)cn[k]);
  }
  // 4. shared: (particle, group, client) keeps its last entry
  for (uint64_t i : loc) {
    if (kind[i] != 1) continue;
    const std::string_view f((const char*)bytes + offs[i], offs[i + 1] - offs[i]);
    std::string group(segment_at(f, 1));
    auto git = group_ids_.find(group);
    uint32_t gid;
    if (git == group_ids_.end()) {
      gid = (uint32_t)group_ids_.size();
      group_ids_.emplace(group, gid);
    } else {
      gid = git->second;
    }
    const uint32_t node = items[i].node;
    ShrKey key{node, gid, client_ids[i]};
    const ShrRec rec{filter_ids[i], client_ids[i]};
    auto it = shr_pos_.find(key);
    if (it != shr_pos_.end()) {
      shr.m.h[it->second] = rec;
      continue;
    }
    if (out_new) out_new[i] = 1;
    NodeLists& L = lists.h[node];
    const uint32_t old_off = L.shr_off, cnt = L.shr_cnt;
    list_push(shr, L.shr_off, L.shr_cnt, nh_[node].shr_cap, rec);
    if (shr_group_.size() < shr.m.size()) shr_group_.resize(shr.m.size());
    if (L.shr_off != old_off)
      for (uint32_t k = 0; k < cnt; k++) {
        const uint32_t g = shr_group_[old_off + k];
        shr_group_[L.shr_off + k] = g;
        shr_pos_[ShrKey{node, g, shr.m.h[L.shr_off + k].client}] = L.shr_off + k;
      }
    shr_pos_[key] = L.shr_off + cnt;
    shr_group_[L.shr_off + cnt] = gid;
  }
  lists.all_dirty = subs.m.all_dirty = shr.m.all_dirty = true;
  if (sharded()) xinfo.all_dirty = true;
  // 5. the other shards' subscriptions, in order: this shard's foreign partners
  for (uint64_t i = 0; i < n; i++)
    if (kind[i] == 2) one(i);
}

void Index::retain_bulk(const uint8_t* bytes, const uint64_t* offs, const uint64_t* handles, uint64_t n) {
  if (!empty_image() || n < 4096) {
    for (uint64_t i = 0; i < n; i++)
      retain_message(std::string_view((const char*)bytes + offs[i], offs[i + 1] - offs[i]), handles[i], 1, true);
    return;
  }
  version_++;
  retained_version_++;
  const unsigned threads = build_threads();
  std::vector<uint8_t> mine(n, 1);
  std::vector<BulkItem> items;
  std::vector<uint64_t> idx;
  for (uint64_t i = 0; i < n; i++) {
    const std::string_view t((const char*)bytes + offs[i], offs[i + 1] - offs[i]);
    if (sharded() && shard_hash(t) % n_shards_ != shard_) continue;  // retained: by topic
    items.push_back(BulkItem{offs[i], offs[i + 1], kRoot, false});
    idx.push_back(i);
  }
  bulk_trie(items, bytes, threads);
  // RetainMessage with a payload, in order: the particle's last entry is live (topic "": the
  // Retained entry without a retain path, Q6)
  for (size_t k = 0; k < items.size(); k++) {
    const uint64_t i = idx[k];
    const uint32_t node = items[k].node;
    if (offs[i + 1] == offs[i]) {
      if (!empty_topic_live) n_retained_++;
      empty_topic_live = true;
      empty_topic_handle = handles[i];
      empty_topic_retain = true;
      continue;
    }
    NodeMsg& M = msg.h[node];
    if (!(M.flags & kRetainLive)) n_retained_++;
    M.flags = (M.flags & kChildSys) | kRetainPath | kRetainLive | kRetainFlag;
    M.handle = handles[i];
    nh_[node].retain_path = true;
  }
  // below_live, bottom-up: children have larger ids than their parents (BFS)
  for (uint32_t v = (uint32_t)nh_.size() - 1; v > kRoot; v--) {
    if (!nh_[v].live) continue;
    const NodeMsg& M = msg.h[v];
    msg.h[M.parent].below_live += M.below_live + ((M.flags & kRetainLive) ? 1u : 0u);
  }
  parallel_for(nh_.size() - 1, threads, [&](size_t b, size_t e) {  // the children slabs' copies
    for (size_t k = b; k < e; k++) {
      const uint32_t v = (uint32_t)k + 1;
      if (!nh_[v].live) continue;
      const NodeMsg& M = msg.h[v];
      children.m.h[msg.h[M.parent].child_off + M.child_pos] = ChildRec{v, M.child_off, M.child_cnt, M.flags, M.handle};
    }
  });
  msg.all_dirty = children.m.all_dirty = true;
}

}  // namespace mq
