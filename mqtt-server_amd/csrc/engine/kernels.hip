// gfx950 kernels of the topic-matching engine.
//
//   k_walk<false>   one thread per publish topic: tokenises the topic and walks the trie in the
//                   reference's exact DFS order (scanSubscribers, topics.go:593-628) with no
//                   stack — parent pointers in the node records replace recursion. Counts the
//                   gathers and the rows each topic will emit.
//   k_scan_*        exclusive scan of the per-topic counts into output offsets.
//   k_walk<true>    the same walk again, writing the gather list (node + what to gather).
//   k_emit          one wavefront (64 lanes) per topic: streams the gathered subscription
//                   lists into the output rows (coalesced 16-byte rows), merges subscriptions of
//                   clients with several matching filters through a per-wave LDS hash table
//                   (gatherSubscriptions + Subscription.Merge, topics.go:631-648,
//                   packets/packets.go:254-274), copies shared rows and applies the inline
//                   last-write rule (topics.go:668-676) with ballot/mbcnt compaction.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace mq {

// ---------------------------------------------------------------------------------------------
// byte-level helpers over the topic buffer
// ---------------------------------------------------------------------------------------------
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Byte reader with a one-chunk register cache: one 16-byte load serves 16 sequential byte
// reads. The topic buffer must be readable up to its next 16-byte boundary (include/mqmatch.h).
struct ByteReader {
  const uint8_t* base;
  uint64_t ci;
  u32x4 c;
  __device__ __forceinline__ explicit ByteReader(const uint8_t* b) : base(b), ci(~0ull) {}
  __device__ __forceinline__ uint32_t at(uint64_t i) {
    const uint64_t k = i >> 4;
    if (k != ci) {
      c = *reinterpret_cast<const u32x4*>(base + (k << 4));
      ci = k;
    }
    const uint32_t w = ((uint32_t)i >> 2) & 3;
    const uint32_t word = w == 0 ? c.x : (w == 1 ? c.y : (w == 2 ? c.z : c.w));
    return (word >> (((uint32_t)i & 3) * 8)) & 0xffu;
  }
};

// Scan the segment that starts at s: returns the position of its terminating '/' (or end) and
// its key (layout.h) in the same pass.
__device__ __forceinline__ uint64_t scan_segment(ByteReader& R, uint64_t s, uint64_t end, SegKey* key) {
  SegKeyBuilder kb;
  uint64_t i = s;
  for (; i < end; i++) {
    const uint32_t ch = R.at(i);
    if (ch == '/') break;
    kb.push(ch);
  }
  *key = kb.finish();
  return i;
}

__device__ __forceinline__ uint64_t seg_start_before(ByteReader& R, uint64_t b0, uint64_t e) {
  while (e > b0 && R.at(e - 1) != '/') e--;
  return e;
}

// particles.get(key) (topics.go:803-807) through the global edge table.
__device__ __forceinline__ uint32_t lookup(const DevIndex& ix, uint32_t parent, const SegKey& k,
                                          const uint8_t* seg, uint32_t len) {
  uint64_t i = edge_hash(parent, k) & ix.edge_mask;
  for (uint64_t probes = 0; probes <= ix.edge_mask; probes++) {
    const EdgeSlot e = ix.edges[i];
    if (e.parent == kEdgeEmpty) return kNone;
    if (e.parent == parent && e.k0 == k.k0 && e.k1 == k.k1) {
      if (!seg_is_long(k)) return e.child;
      const SegInfo si = ix.seginfo[ix.walk[e.child].seg];
      bool eq = si.len == len;
      for (uint32_t j = 0; eq && j < len; j++) eq = ix.segbytes[si.off + j] == seg[j];
      if (eq) return e.child;
    }
    i = (i + 1) & ix.edge_mask;
  }
  return kNone;
}

// ---------------------------------------------------------------------------------------------
// k_walk: the match walk (thread per topic)
// ---------------------------------------------------------------------------------------------
// FILL=false: count pass; also writes the first kGatherCap gathers of each topic to its slot
// of `gathers` (stride kGatherCap) and flags a topic with more. FILL=true: writes every gather
// compactly at off[t].g (run only when some topic overflowed its slot).
template <bool FILL>
__global__ __launch_bounds__(256) void k_walk(const uint8_t* __restrict__ tb,
                                              const uint64_t* __restrict__ to, uint32_t n,
                                              DevIndex ix, TopicCount* __restrict__ cnt,
                                              const TopicOff* __restrict__ off,
                                              uint32_t* __restrict__ gathers) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint64_t b0 = to[t], b1 = to[t + 1];
  uint32_t ng = 0, rows = 0, shared = 0, inl = 0, merge = 0;
  uint32_t* gout = FILL ? gathers + off[t].g : gathers + (uint64_t)t * kGatherCap;

  if (b1 > b0) {  // Subscribers("") matches nothing (topics.go:598-600)
    ByteReader R(tb);
    const bool dollar = R.at(b0) == '$';
    // gather{Subscriptions,SharedSubscriptions,InlineSubscriptions} of one particle
    auto gather = [&](uint32_t node, bool with_inline) {
      const NodeLists L = ix.lists[node];
      // [MQTT-4.7.1-1]: '$' topics skip subscriptions whose filter starts with '+'/'#' (Q3)
      const bool subs_ok = !(dollar && (L.flags & kFlagSeg0Wild));
      const uint32_t gw = node | (subs_ok ? kGatherSubs : 0u) | (with_inline ? kGatherInline : 0u);
      if (FILL || ng < kGatherCap) gout[ng] = gw;
      if (!FILL) {
        if (subs_ok) {
          rows += L.n_direct + L.n_merge;
          merge += L.n_merge;
        }
        shared += L.shr_cnt;
        if (with_inline) inl += L.inl_cnt;
      }
      ng++;
    };

    uint32_t node = kRoot;
    SegKey key;
    uint64_t s = b0, e = scan_segment(R, b0, b1, &key);
    int state = 0;  // 0: literal child next, 1: '+' child next, 2: '#' gather and return
    for (uint64_t guard = 0;; guard++) {
      if (guard > kWalkGuard) {  // never reached on a well-formed image; fail loudly, not hang
        atomicOr(ix.err, kErrWalkGuard);
        break;
      }
      const bool has_next = e < b1;
      if (state == 0) {
        state = 1;
        const uint32_t len = (uint32_t)(e - s);
        // A literal "+" segment makes the reference visit the '+' child twice with identical
        // results (topics.go:603); the '+' branch below covers it.
        if (!(len == 1 && R.at(s) == '+')) {
          const uint32_t p = lookup(ix, node, key, tb + s, len);
          if (p != kNone) {
            if (has_next) {
              node = p;
              s = e + 1;
              e = scan_segment(R, s, b1, &key);
              state = 0;
              continue;
            }
            gather(p, true);
            const uint32_t w = ix.walk[p].hash_child;  // filter/# matches filter (topics.go:612)
            if (w != kNone) gather(w, false);          // inline: the particle's own again (Q2)
          }
        }
      }
      if (state == 1) {
        state = 2;
        const uint32_t p = ix.walk[node].plus_child;
        if (p != kNone) {
          if (has_next) {
            node = p;
            s = e + 1;
            e = scan_segment(R, s, b1, &key);
            state = 0;
            continue;
          }
          gather(p, true);
        }
      }
      const NodeWalk nw = ix.walk[node];
      if (nw.hash_child != kNone) gather(nw.hash_child, true);  // topics.go:621-625
      if (node == kRoot) break;
      // return to the parent: restore its segment window and continue after this branch
      node = nw.parent_flags & kParentMask;
      e = s - 1;
      s = seg_start_before(R, b0, e);
      state = (nw.parent_flags & kFlagPlusKey) ? 2 : 1;
    }
  }
  if (!FILL) {
    TopicCount c;
    c.gathers = ng;
    c.rows = rows;
    c.shared = shared;
    c.inlines = inl;
    uint32_t tab = 0;
    if (merge > kLdsTab / 2) {
      tab = 1;
      while (tab < 2 * merge) tab <<= 1;
    }
    c.table = tab;
    cnt[t] = c;
    if (ng > kGatherCap) atomicOr(ix.err + 1, 1u);
  }
}

// ---------------------------------------------------------------------------------------------
// exclusive scan of TopicCount -> TopicOff (1024 topics per block)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void add_count(TopicOff& a, const TopicCount& c) {
  a.g += c.gathers;
  a.rows += c.rows;
  a.shr += c.shared;
  a.inl += c.inlines;
  a.tab += c.table;
}
__device__ __forceinline__ void add_off(TopicOff& a, const TopicOff& b) {
  a.g += b.g;
  a.rows += b.rows;
  a.shr += b.shr;
  a.inl += b.inl;
  a.tab += b.tab;
}
__device__ __forceinline__ TopicOff shfl_up_off(const TopicOff& v, int d) {
  TopicOff r;
  r.g = __shfl_up(v.g, d, 64);
  r.rows = __shfl_up(v.rows, d, 64);
  r.shr = __shfl_up(v.shr, d, 64);
  r.inl = __shfl_up(v.inl, d, 64);
  r.tab = __shfl_up(v.tab, d, 64);
  return r;
}

// Block-wide inclusive scan of one TopicOff per thread (256 threads).
__device__ TopicOff block_scan_incl(TopicOff v, TopicOff* wave_tot /*4*/) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int d = 1; d < 64; d <<= 1) {
    TopicOff u = shfl_up_off(v, d);
    if (lane >= d) add_off(v, u);
  }
  if (lane == 63) wave_tot[wv] = v;
  __syncthreads();
  for (int w = 0; w < wv; w++) add_off(v, wave_tot[w]);
  __syncthreads();
  return v;
}

__global__ __launch_bounds__(256) void k_scan_reduce(const TopicCount* __restrict__ cnt, uint32_t n,
                                                     TopicOff* __restrict__ bsum) {
  __shared__ TopicOff wt[4];
  TopicOff v{0, 0, 0, 0, 0};
  const uint64_t base = (uint64_t)blockIdx.x * kScanBlock + threadIdx.x * 4;
  for (int k = 0; k < 4; k++)
    if (base + k < n) add_count(v, cnt[base + k]);
  v = block_scan_incl(v, wt);
  if (threadIdx.x == 255) bsum[blockIdx.x] = v;
}

// Single workgroup: exclusive scan of the block sums; bpre[nb] = total.
__global__ __launch_bounds__(256) void k_scan_blocks(const TopicOff* __restrict__ bsum, uint32_t nb,
                                                     TopicOff* __restrict__ bpre) {
  __shared__ TopicOff wt[4];
  __shared__ TopicOff carry;
  if (threadIdx.x == 0) carry = TopicOff{0, 0, 0, 0, 0};
  __syncthreads();
  for (uint32_t b0 = 0; b0 < nb; b0 += 256) {
    const uint32_t b = b0 + threadIdx.x;
    TopicOff v = b < nb ? bsum[b] : TopicOff{0, 0, 0, 0, 0};
    TopicOff incl = block_scan_incl(v, wt);
    TopicOff c = carry;
    TopicOff ex = incl;
    ex.g -= v.g; ex.rows -= v.rows; ex.shr -= v.shr; ex.inl -= v.inl; ex.tab -= v.tab;
    add_off(ex, c);
    if (b < nb) bpre[b] = ex;
    __syncthreads();
    if (threadIdx.x == 255) add_off(carry, incl);
    __syncthreads();
  }
  if (threadIdx.x == 0) bpre[nb] = carry;
}

__global__ __launch_bounds__(256) void k_scan_apply(const TopicCount* __restrict__ cnt, uint32_t n,
                                                    const TopicOff* __restrict__ bpre,
                                                    TopicOff* __restrict__ off) {
  __shared__ TopicOff wt[4];
  const uint64_t base = (uint64_t)blockIdx.x * kScanBlock + threadIdx.x * 4;
  TopicCount c[4];
  TopicOff v{0, 0, 0, 0, 0};
  for (int k = 0; k < 4; k++) {
    c[k] = base + k < n ? cnt[base + k] : TopicCount{0, 0, 0, 0, 0};
    add_count(v, c[k]);
  }
  TopicOff incl = block_scan_incl(v, wt);
  TopicOff ex = bpre[blockIdx.x];
  add_off(ex, incl);
  ex.g -= v.g; ex.rows -= v.rows; ex.shr -= v.shr; ex.inl -= v.inl; ex.tab -= v.tab;
  for (int k = 0; k < 4; k++) {
    if (base + k < n) off[base + k] = ex;
    add_count(ex, c[k]);
  }
  if (base + 3 >= (uint64_t)n - 1 && base < n) off[n] = bpre[gridDim.x];
}

// ---------------------------------------------------------------------------------------------
// k_emit: expand + merge + emit (one wavefront per topic)
// ---------------------------------------------------------------------------------------------
constexpr uint32_t kTabEmpty = 0xFFFFFFFFu;
constexpr uint32_t kMetaDirty = 0x80000000u;

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint32_t prefix_before(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
}

// Exclusive wave-wide prefix sum (64 lanes); *total receives the sum.
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t lane, uint32_t* total) {
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  *total = __shfl(x, 63, 64);
  return x - v;
}

// Copy the concatenation of up to 64 record lists (list j at src + off[j], exclusive prefix
// pre[j], pre[64] = total) to dst[0, total): 64 consecutive rows per wave-instruction, four
// loads in flight per lane. Each lane keeps a cursor j that only advances. The rows are
// written once and never re-read here, so they are stored non-temporally and do not evict
// the hot subscription lists from L2 / the Infinity Cache.
template <class V>
__device__ __forceinline__ void copy_lists(V* __restrict__ dst, const V* __restrict__ src,
                                           const uint32_t* __restrict__ off,
                                           const uint32_t* __restrict__ pre, uint32_t total,
                                           uint32_t lane) {
  // Loads are issued unconditionally (idle lanes re-read the last row) so the four stay in
  // flight together: a load inside a divergent branch makes the compiler wait for it at the
  // branch join.
  uint32_t j = 0;
  for (uint32_t r0 = 0; r0 < total; r0 += 256) {
    uint32_t src_i[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t r = min(r0 + k * 64 + lane, total - 1);
      while (pre[j + 1] <= r) j++;
      src_i[k] = off[j] + (r - pre[j]);
    }
    V v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = src[src_i[k]];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t r = r0 + k * 64 + lane;
      if (r < total) __builtin_nontemporal_store(v[k], dst + r);
    }
  }
}

constexpr uint32_t kGroup = 64;  // gathers staged per pass: one per lane

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int d = 32; d; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

__global__ __launch_bounds__(256) void k_emit(EmitArgs a) {
  __shared__ uint32_t lds_key[4][kLdsTab];
  __shared__ uint32_t lds_row[4][kLdsTab];
  __shared__ uint32_t lds_meta[4][kLdsTab];
  __shared__ uint32_t gwl[4][kPairMax];          // the topic's gather words (pair analysis)
  __shared__ uint32_t ghit[4][kPairMax];         // gather has table-bound records
  __shared__ uint32_t hit_g[4][kHitMax];         // hits: gather index, list offset, list length
  __shared__ uint32_t hit_off[4][kHitMax];
  __shared__ uint32_t hit_cnt[4][kHitMax];
  __shared__ uint32_t bm[4][kBitWin / 32];       // table-bound bitmap of a may-merge window
  __shared__ uint32_t tlist[4][kTList];          // table-bound records queued for the table
  __shared__ uint32_t g_off[3][4][kGroup];       // direct-sub / shared / inline list offsets
  __shared__ uint32_t g_pre[3][4][kGroup + 1];   // their exclusive prefixes (+ total)
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t w = blockIdx.x * 4 + wv;
  uint32_t t;
  if (a.list) {
    if (w >= a.n_list) return;  // wave-uniform
    t = a.list[2 * w];
  } else {
    t = a.t0 + w;
    if (t >= a.t1) return;  // wave-uniform
  }
  const bool global_tab = a.list != nullptr;
  // Diagnosis only (MQ_EMIT_PROF): per-phase wave cycles and work counts.
  const bool wp = a.wprof != nullptr;
  const long long wp_t0 = wp ? clock64() : 0;
  long long wp_copy = 0, wp_merge = 0, wp_drain = 0, wp_setup = 0;
  uint32_t wp_mrecs = 0, wp_chunks = 0, wp_look = 0, wp_probe = 0;
  auto wp_flush = [&](uint32_t tab_recs) {
    if (!wp) return;
    const uint32_t lk = wave_sum(wp_look), pr = wave_sum(wp_probe);
    if (lane == 0) {
      unsigned long long* q = a.wprof;
      atomicAdd(q + kWpWaves, 1ull);
      atomicAdd(q + kWpTotal, (unsigned long long)(clock64() - wp_t0));
      atomicAdd(q + kWpSetup, (unsigned long long)wp_setup);
      atomicAdd(q + kWpCopy, (unsigned long long)wp_copy);
      atomicAdd(q + kWpMerge, (unsigned long long)wp_merge);
      atomicAdd(q + kWpDrain, (unsigned long long)wp_drain);
      atomicAdd(q + kWpMergeRecs, (unsigned long long)wp_mrecs);
      atomicAdd(q + kWpTabRecs, (unsigned long long)tab_recs);
      atomicAdd(q + kWpLookups, (unsigned long long)lk);
      atomicAdd(q + kWpProbes, (unsigned long long)pr);
      atomicAdd(q + kWpChunks, (unsigned long long)wp_chunks);
    }
  };

  const TopicOff o0 = a.off[t], o1 = a.off[t + 1];
  const uint64_t rb = o0.rows - a.base.rows;
  const uint32_t cap = (uint32_t)(o1.rows - o0.rows);
  const uint64_t sb = o0.shr - a.base.shr, ib = o0.inl - a.base.inl;
  SubRec* __restrict__ rows = a.rows + rb;
  const uint32_t n_g = (uint32_t)(o1.g - o0.g);
  auto gword = [&](uint32_t i) {
    return a.gather_stride ? a.gathers[(uint64_t)t * a.gather_stride + i] : a.gathers[o0.g + i];
  };

  // ---- Pair analysis: which may-merge records need the merge table. For every ordered pair
  // (g, h) of gathered nodes with subscriptions, g's pair block lists g's may-merge slots whose
  // client also subscribes at h (layout.h). The union of the hit lists of g is exactly g's
  // table-bound records; every other record of the topic is its client's only match and is
  // emitted as is. Beyond kPairMax gathers or kHitMax hits every may-merge record is
  // table-bound (correct, slower; not seen in the SURVEY.md §8d workloads).
  bool pair_ok = n_g <= kPairMax;
  uint32_t n_hit = 0, ub = 0;  // hits; upper bound of the table-bound records
  if (pair_ok) {
    for (uint32_t i = lane; i < n_g; i += 64) {
      gwl[wv][i] = gword(i);
      ghit[wv][i] = 0;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const uint32_t np = n_g * n_g;
    uint32_t ub_l = 0;
    for (uint32_t p0 = 0; p0 < np; p0 += 64) {
      const uint32_t p = p0 + lane;
      bool hit = false;
      uint32_t gi = 0, e_off = 0, e_cnt = 0;
      if (p < np) {
        gi = p / n_g;
        const uint32_t hi = p - gi * n_g;
        const uint32_t gg = gwl[wv][gi], gh = gwl[wv][hi];
        if (gi != hi && (gg & gh & kGatherSubs)) {
          const NodePair P = a.ix.npair[gg & kGatherNode];
          if (P.ent_mask != kNone) {
            const uint32_t h = gh & kGatherNode;
            uint32_t sl = pair_hash(h) & P.ent_mask;
            if (wp) wp_look++;
            for (;;) {
              if (wp) wp_probe++;
              const PairEnt e = a.ix.pent[P.ent_off + sl];
              if (e.h == h) {
                hit = true;
                e_off = e.off;
                e_cnt = e.cnt;
                break;
              }
              if (e.h == kNone) break;
              sl = (sl + 1) & P.ent_mask;
            }
          }
        }
      }
      const uint64_t bh = __ballot(hit);
      if (hit) {
        const uint32_t x = n_hit + prefix_before(bh);
        if (x < kHitMax) {
          hit_g[wv][x] = gi;
          hit_off[wv][x] = e_off;
          hit_cnt[wv][x] = e_cnt;
        }
        ghit[wv][gi] = 1;
      }
      n_hit += __popcll(bh);
      ub_l += e_cnt;
    }
    ub = wave_sum(ub_l);
    if (n_hit > kHitMax) pair_ok = false;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  if (!pair_ok) {  // every may-merge record is table-bound
    uint32_t ub_l = 0;
    for (uint32_t i = lane; i < n_g; i += 64) {
      const uint32_t gw = gword(i);
      if (gw & kGatherSubs) ub_l += a.ix.lists[gw & kGatherNode].n_merge;
    }
    ub = wave_sum(ub_l);
  }
  if (wp) wp_setup = clock64() - wp_t0;

  // A topic whose table would outgrow LDS goes to the overflow pass, which gives it a global
  // table of >= 2 * ub slots.
  if (!global_tab && ub > kLdsTabMax) {
    if (lane == 0) {
      uint32_t slots = 1;
      while (slots < 2 * ub) slots <<= 1;
      const uint32_t i = atomicAdd(a.ovf, 1u);
      a.ovf[4 + 2 * i] = t;
      a.ovf[4 + 2 * i + 1] = slots;
      atomicAdd(a.ovf + 1, slots);
    }
    wp_flush(ub);
    return;
  }

  // Merge table: LDS on the fast pass, a global slice on the overflow pass. Accesses branch on
  // the (wave-uniform) kind so each compiles to typed ds_* / global_* instructions.
  uint32_t* gk = nullptr;
  uint32_t* gr = nullptr;
  uint32_t* gm = nullptr;
  uint32_t tmask = kLdsTab - 1;
  if (global_tab) {
    const uint32_t slots = a.list[2 * w + 1];
    uint32_t tb = 0;
    if (lane == 0) tb = atomicAdd(a.ovf + 2, slots);
    tb = __builtin_amdgcn_readfirstlane(tb);
    gk = a.tab + tb;
    gr = a.tab + a.tab_cap + tb;
    gm = a.tab + 2 * a.tab_cap + tb;
    tmask = slots - 1;
  }
  auto tk_load = [&](uint32_t i) -> uint32_t {
    return global_tab ? __hip_atomic_load(gk + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                      : __hip_atomic_load(&lds_key[wv][i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  auto tk_cas = [&](uint32_t i, uint32_t v) -> uint32_t {
    return global_tab ? atomicCAS(gk + i, kTabEmpty, v) : atomicCAS(&lds_key[wv][i], kTabEmpty, v);
  };
  auto tk_store = [&](uint32_t i, uint32_t v) {
    if (global_tab) gk[i] = v; else lds_key[wv][i] = v;
  };
  auto tr_load = [&](uint32_t i) -> uint32_t { return global_tab ? gr[i] : lds_row[wv][i]; };
  auto tr_store = [&](uint32_t i, uint32_t v) {
    if (global_tab) gr[i] = v; else lds_row[wv][i] = v;
  };
  auto tm_load = [&](uint32_t i) -> uint32_t { return global_tab ? gm[i] : lds_meta[wv][i]; };
  auto tm_store = [&](uint32_t i, uint32_t v) {
    if (global_tab) gm[i] = v; else lds_meta[wv][i] = v;
  };
  // Insert `key` (distinct across the active lanes); returns the slot and whether it was new.
  auto tab_insert = [&](uint32_t key, bool* is_new) -> uint32_t {
    uint32_t sl = hash32(key) & tmask;
    for (uint32_t probes = 0; probes <= tmask; probes++) {
      const uint32_t k = tk_load(sl);
      if (k == key) {
        *is_new = false;
        return sl;
      }
      if (k == kTabEmpty) {
        const uint32_t old = tk_cas(sl, key);
        if (old == kTabEmpty) {
          *is_new = true;
          return sl;
        }
        if (old == key) {
          *is_new = false;
          return sl;
        }
      }
      sl = (sl + 1) & tmask;
    }
    atomicOr(a.ix.err, kErrTableFull);  // sized at <= 3/4 load: unreachable
    *is_new = false;
    return 0;
  };
  bool tab_ready = false;
  uint32_t tab_recs = 0;

  uint32_t n_cli = 0, n_ext = 0, n_shr = 0, n_inl = 0;
  for (uint64_t g0 = o0.g; g0 < o1.g; g0 += kGroup) {
    // Stage up to 64 gathers at once (one per lane): the gather word and the node's lists. A
    // node without table-bound records this topic is copied whole (direct and may-merge
    // slots are contiguous); the others copy their direct part and stream the rest below.
    const uint32_t gbase = (uint32_t)(g0 - o0.g);
    const uint32_t ng = (uint32_t)min<uint64_t>(kGroup, o1.g - g0);
    uint32_t dn = 0, mn = 0, sn = 0, in = 0, sub_off = 0, shr_off = 0, inl_off = 0;
    if (lane < ng) {
      const uint32_t gw = pair_ok ? gwl[wv][gbase + lane] : gword(gbase + lane);
      const NodeLists L = a.ix.lists[gw & kGatherNode];
      if (gw & kGatherSubs) {
        const bool tb = pair_ok ? ghit[wv][gbase + lane] != 0 : L.n_merge != 0;
        dn = tb ? L.n_direct : L.n_direct + L.n_merge;
        mn = tb ? L.n_merge : 0;
      }
      sub_off = L.sub_off;
      sn = L.shr_cnt;
      shr_off = L.shr_off;
      if (gw & kGatherInline) {
        in = L.inl_cnt;
        inl_off = L.inl_off;
      }
    }
    uint32_t dt, st, it;
    const uint32_t dp = wave_excl_scan(dn, lane, &dt);
    const uint32_t sp = wave_excl_scan(sn, lane, &st);
    const uint32_t ip = wave_excl_scan(in, lane, &it);
    g_off[0][wv][lane] = sub_off;
    g_off[1][wv][lane] = shr_off;
    g_off[2][wv][lane] = inl_off;
    g_pre[0][wv][lane] = dp;
    g_pre[1][wv][lane] = sp;
    g_pre[2][wv][lane] = ip;
    if (lane == 0) {
      g_pre[0][wv][kGroup] = dt;
      g_pre[1][wv][kGroup] = st;
      g_pre[2][wv][kGroup] = it;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();

    const long long wp_c = wp ? clock64() : 0;
    // Records that are their client's only match: one flat coalesced copy into client rows.
    copy_lists(reinterpret_cast<u32x4*>(rows + n_cli), reinterpret_cast<const u32x4*>(a.ix.subs),
               g_off[0][wv], g_pre[0][wv], dt, lane);
    n_cli += dt;
    // Shared[sub.Filter][client] = sub (topics.go:656-663)
    copy_lists(reinterpret_cast<u32x2*>(a.shr_rows + sb + n_shr), reinterpret_cast<const u32x2*>(a.ix.shr),
               g_off[1][wv], g_pre[1][wv], st, lane);
    n_shr += st;
    // Inline subscriptions in gather order; the last write per id is kept below.
    copy_lists(reinterpret_cast<u32x2*>(a.inl_rows + ib + n_inl), reinterpret_cast<const u32x2*>(a.ix.inl),
               g_off[2][wv], g_pre[2][wv], it, lane);
    n_inl += it;
    if (wp) wp_copy += clock64() - wp_c;
    const long long wp_m = wp ? clock64() : 0;

    // Nodes with table-bound records, in gather (rank) order.
    uint64_t mm = __ballot(mn > 0);
    while (mm) {
      const uint32_t j = (uint32_t)__builtin_ctzll(mm);
      mm &= mm - 1;
      const uint32_t gidx = gbase + j;
      const uint32_t m_cnt = __builtin_amdgcn_readlane(mn, j);
      const uint32_t m_off = __builtin_amdgcn_readlane(sub_off + dn, j);
      const SubRec* __restrict__ ms = a.ix.subs + m_off;
      wp_mrecs += m_cnt;
      uint32_t nt = 0;  // table-bound records queued in tlist
      // Table pass over the queue (the clients with several matches). Records of one gather
      // belong to distinct clients, so their order within the gather does not matter.
      auto drain = [&]() {
        const long long wp_d = wp ? clock64() : 0;
        if (!tab_ready) {
          for (uint32_t q = lane; q <= tmask; q += 64) tk_store(q, kTabEmpty);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          tab_ready = true;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        tab_recs += nt;
        for (uint32_t c0 = 0; c0 < nt; c0 += 64) {
          const bool vt = c0 + lane < nt;
          SubRec r{0, 0, 0, 0};
          uint32_t slot = 0;
          bool is_new = false;
          if (vt) {
            r = ms[tlist[wv][c0 + lane]];
            slot = tab_insert(r.client, &is_new);
          }
          const uint64_t bn = __ballot(vt && is_new);
          if (vt && is_new) {  // first (minimum-rank) subscription of this client: the base
            const uint32_t pos = n_cli + prefix_before(bn);
            rows[pos] = r;
            tr_store(slot, pos);
            tm_store(slot, r.meta);
          }
          n_cli += __popcll(bn);
          const bool dup = vt && !is_new;
          if (dup) {  // Subscription.Merge: max Qos, OR NoLocal (packets/packets.go:264-271)
            const uint32_t mt = tm_load(slot);
            const uint32_t q = max(mt & kMetaQos, r.meta & kMetaQos);
            const uint32_t nm = (mt & ~kMetaQos) | q | (r.meta & kMetaNoLocal);
            if ((nm & ~kMetaDirty) != (mt & ~kMetaDirty)) tm_store(slot, nm | kMetaDirty);
          }
          const uint64_t be = __ballot(dup && r.ident > 0);
          if (dup && r.ident > 0) {  // Identifiers[n.Filter] = n.Identifier (id > 0)
            const uint32_t e = n_ext + prefix_before(be);
            SubRec x{r.client, r.filter_id, r.ident, 0};
            rows[cap - 1 - e] = x;
          }
          n_ext += __popcll(be);
        }
        nt = 0;
        if (wp) wp_drain += clock64() - wp_d;
      };

      if (!pair_ok) {  // all of them
        for (uint32_t i0 = 0; i0 < m_cnt; i0 += 64) {
          if (i0 + lane < m_cnt) tlist[wv][nt + lane] = i0 + lane;
          nt += min(64u, m_cnt - i0);
          if (nt + 64 > kTList) drain();
        }
        if (nt) drain();
        continue;
      }
      for (uint32_t w0 = 0; w0 < m_cnt; w0 += kBitWin) {
        const uint32_t wn = min(kBitWin, m_cnt - w0);
        // Mark this window's table-bound slots (union of the gather's hit lists) and queue
        // each once for the table.
        for (uint32_t q = lane; q < kBitWin / 32; q += 64) bm[wv][q] = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        for (uint32_t x = 0; x < n_hit; x++) {
          if (hit_g[wv][x] != gidx) continue;  // wave-uniform
          const uint32_t off = hit_off[wv][x], cnt = hit_cnt[wv][x];
          for (uint32_t c0 = 0; c0 < cnt; c0 += 64) {
            bool own = false;
            uint32_t k = 0;
            if (c0 + lane < cnt) {
              k = a.ix.plist[off + c0 + lane] - w0;
              if (k < wn) {
                const uint32_t bit = 1u << (k & 31);
                own = !(atomicOr(&bm[wv][k >> 5], bit) & bit);
              }
            }
            const uint64_t bo = __ballot(own);
            if (own) tlist[wv][nt + prefix_before(bo)] = w0 + k;
            nt += __popcll(bo);
            if (nt + 64 > kTList) drain();
          }
        }
        if (nt) drain();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        // Stream the window: everything not marked goes straight to client rows. Four
        // 64-record chunks in flight; loads are unconditional (see copy_lists).
        for (uint32_t i0 = 0; i0 < wn; i0 += 256) {
          wp_chunks++;
          SubRec rr[4];
#pragma unroll
          for (int u = 0; u < 4; u++) rr[u] = ms[w0 + min(i0 + u * 64 + lane, wn - 1)];
#pragma unroll
          for (int u = 0; u < 4; u++) {
            const uint32_t k = i0 + u * 64 + lane;
            const bool v = k < wn && !((bm[wv][min(k, wn - 1) >> 5] >> (k & 31)) & 1);
            const uint64_t bd = __ballot(v);
            if (v)
              __builtin_nontemporal_store(*reinterpret_cast<const u32x4*>(&rr[u]),
                                          reinterpret_cast<u32x4*>(rows + n_cli + prefix_before(bd)));
            n_cli += __popcll(bd);
          }
        }
      }
    }
    if (wp) wp_merge += clock64() - wp_m;
  }

  if (tab_ready) {  // write back merged Qos/NoLocal of bases that absorbed later matches
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (uint32_t k = lane; k <= tmask; k += 64) {
      if (tk_load(k) != kTabEmpty) {
        const uint32_t m = tm_load(k);
        if (m & kMetaDirty) rows[tr_load(k)].meta = m & ~kMetaDirty;
      }
    }
  }

  if (n_inl) {  // InlineSubscriptions[id] = last gathered (topics.go:673-675)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    InlRec* __restrict__ ir = a.inl_rows + ib;
    uint32_t kept = 0;
    for (uint32_t i0 = 0; i0 < n_inl; i0 += 64) {
      const uint32_t i = i0 + lane;
      bool keep = false;
      InlRec r{0, 0};
      if (i < n_inl) {
        r = ir[i];
        keep = true;
        for (uint32_t j = i + 1; j < n_inl && keep; j++) keep = ir[j].ident != r.ident;
      }
      const uint64_t bk = __ballot(keep);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (keep) ir[kept + prefix_before(bk)] = r;
      kept += __popcll(bk);
    }
    n_inl = kept;
  }

  if (lane == 0) {
    mq_topic_result_dev res;
    res.sub_base = rb;
    res.shared_base = sb;
    res.inline_base = ib;
    res.sub_cap = cap;
    res.n_client = n_cli;
    res.n_ident = n_ext;
    res.n_shared = n_shr;
    res.n_inline = n_inl;
    res.reserved = 0;
    a.res[t - a.t0] = res;
  }
  wp_flush(tab_recs);
}

}  // namespace mq

namespace mq {

void launch_walk(bool fill, const uint8_t* tb, const uint64_t* to, uint32_t n, const DevIndex& ix,
                 TopicCount* cnt, const TopicOff* off, uint32_t* gathers, hipStream_t s) {
  if (!n) return;
  dim3 grid((n + 255) / 256);
  if (fill)
    hipLaunchKernelGGL(k_walk<true>, grid, dim3(256), 0, s, tb, to, n, ix, cnt, off, gathers);
  else
    hipLaunchKernelGGL(k_walk<false>, grid, dim3(256), 0, s, tb, to, n, ix, cnt, off, gathers);
}

void launch_scan(const TopicCount* cnt, uint32_t n, TopicOff* bsum, TopicOff* bpre, TopicOff* off,
                 hipStream_t s) {
  if (!n) return;
  const uint32_t nb = (n + kScanBlock - 1) / kScanBlock;
  hipLaunchKernelGGL(k_scan_reduce, dim3(nb), dim3(256), 0, s, cnt, n, bsum);
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(256), 0, s, bsum, nb, bpre);
  hipLaunchKernelGGL(k_scan_apply, dim3(nb), dim3(256), 0, s, cnt, n, bpre, off);
}

void launch_emit(const EmitArgs& a, hipStream_t s) {
  const uint32_t waves = a.list ? a.n_list : (a.t1 > a.t0 ? a.t1 - a.t0 : 0);
  if (!waves) return;
  hipLaunchKernelGGL(k_emit, dim3((waves + 3) / 4), dim3(256), 0, s, a);
}


// ---------------------------------------------------------------------------------------------
// k_msg: Messages(filter), the reverse retained scan (topics.go:525-579). One thread per filter.
// The recursion is a depth-first walk without a stack: a frame is (node, level d); a '+'/'#'
// level enumerates the node's children slab and, after returning from child c, resumes at
// c's slab position + 1 (NodeMsg.child_pos). Levels past the last segment repeat it
// (isolateParticle, topics.go:679-698), which is how a trailing '#' covers the subtree.
// FILL=false counts the packets per filter; FILL=true writes their handles.
// ---------------------------------------------------------------------------------------------
template <bool FILL>
__global__ __launch_bounds__(256) void k_msg(const uint8_t* __restrict__ fb,
                                             const uint64_t* __restrict__ fo, uint32_t n,
                                             DevIndex ix, TopicCount* __restrict__ cnt,
                                             const TopicOff* __restrict__ off,
                                             uint64_t* __restrict__ handles,
                                             uint64_t* __restrict__ base_out,
                                             uint32_t* __restrict__ count_out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint64_t b0 = fo[t], b1 = fo[t + 1];
  uint32_t c = 0;
  uint64_t* out = FILL ? handles + off[t].rows : nullptr;
  auto emit = [&](uint64_t h) {
    if (FILL) out[c] = h;
    c++;
  };
  // len(filter) == 0 || Retained.Len() == 0 (topics.go:535)
  if (b1 > b0 && ix.retained_len != 0) {
    ByteReader R(fb);
    bool wild = false;
    for (uint64_t i = b0; i < b1; i++) {
      const uint32_t ch = R.at(i);
      wild |= (ch == '+') | (ch == '#');
    }
    if (!wild) {
      // no wildcard: Retained.Get(filter) (topics.go:539-544)
      uint32_t node = kRoot;
      uint64_t s = b0;
      for (;;) {
        SegKey key;
        const uint64_t e = scan_segment(R, s, b1, &key);
        node = lookup(ix, node, key, fb + s, (uint32_t)(e - s));
        if (node == kNone || e >= b1) break;
        s = e + 1;
      }
      if (node != kNone) {
        const NodeMsg m = ix.msg[node];
        if (m.flags & kRetainLive) emit(m.handle);
      }
    } else {
      uint32_t node = kRoot, d = 0, wd = 0;  // wd: level of the segment in the window
      SegKey key;  // key of the window's segment (valid after every forward move)
      uint64_t s = b0, e = scan_segment(R, b0, b1, &key);
      uint32_t cursor = 0;
      bool resume = false;  // re-entering an enumeration frame after a child returned
      for (uint64_t guard = 0;; guard++) {
        if (guard > kWalkGuard * 64) {
          atomicOr(ix.err, kErrWalkGuard);
          break;
        }
        const bool has_next = (wd == d) && (e < b1);
        const uint32_t len = (uint32_t)(e - s);
        const uint32_t c0 = len == 1 ? R.at(s) : 0;
        const bool plus = c0 == '+';
        const bool hash = c0 == '#';
        bool descended = false;
        if (plus || hash) {  // topics.go:547-565
          const NodeMsg nm = ix.msg[node];
          if (!resume) cursor = 0;
          while (cursor < nm.child_cnt) {
            const uint32_t ch = ix.children[nm.child_off + cursor];
            cursor++;
            const NodeMsg cm = ix.msg[ch];
            if (d == 0 && cm.key_sys) continue;  // only the exact $SYS particle, level 0 (Q4)
            if (!has_next && (cm.flags & kRetainPath) && (cm.flags & kRetainLive)) emit(cm.handle);
            if (has_next || hash) {
              node = ch;
              d++;
              if (e < b1) {
                s = e + 1;
                e = scan_segment(R, s, b1, &key);
                wd++;
              }
              descended = true;
              break;
            }
          }
        } else if (!resume) {  // literal level (topics.go:568-576)
          const uint32_t p = lookup(ix, node, key, fb + s, len);
          if (p != kNone) {
            if (has_next) {
              node = p;
              d++;
              s = e + 1;
              e = scan_segment(R, s, b1, &key);
              wd++;
              descended = true;
            } else {
              const NodeMsg m = ix.msg[p];
              if (m.flags & kRetainPath) {
                if (m.flags & kRetainLive) emit(m.handle);
              } else if (ix.empty_topic_live) {
                emit(ix.empty_topic_handle);  // Retained.Get("") on a particle without a path (Q6)
              }
            }
          }
        }
        if (descended) {
          resume = false;
          continue;
        }
        // frame finished: return to the parent frame (its key is not needed again: a literal
        // frame is done, an enumeration frame resumes after this child)
        if (d == 0) break;
        const NodeMsg cm = ix.msg[node];
        node = ix.walk[node].parent_flags & kParentMask;
        if (wd == d) {
          e = s - 1;
          s = seg_start_before(R, b0, e);
          wd--;
        }
        d--;
        cursor = cm.child_pos + 1;
        resume = true;
      }
    }
  }
  if (!FILL) {
    cnt[t] = TopicCount{0, c, 0, 0, 0};
  } else {
    base_out[t] = off[t].rows;
    count_out[t] = c;
  }
}

void launch_msg(bool fill, const uint8_t* fb, const uint64_t* fo, uint32_t n, const DevIndex& ix,
                TopicCount* cnt, const TopicOff* off, uint64_t* handles, uint64_t* base,
                uint32_t* count, hipStream_t s) {
  if (!n) return;
  dim3 grid((n + 255) / 256);
  if (fill)
    hipLaunchKernelGGL(k_msg<true>, grid, dim3(256), 0, s, fb, fo, n, ix, cnt, off, handles, base, count);
  else
    hipLaunchKernelGGL(k_msg<false>, grid, dim3(256), 0, s, fb, fo, n, ix, cnt, off, handles, base, count);
}

}  // namespace mq
