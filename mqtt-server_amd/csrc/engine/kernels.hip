// gfx950 kernels of the topic-matching engine.
//
//   k_walk<false>   one thread per publish topic: tokenises the topic and walks the trie in the
//                   reference's exact DFS order (scanSubscribers, topics.go:593-628) with no
//                   stack — parent pointers in the node records replace recursion. Counts the
//                   gathers and the rows each topic will emit.
//   k_scan_*        exclusive scan of the per-topic counts into output offsets.
//   k_walk<true>    the same walk again, writing the gather list (node + what to gather).
//   k_desc          per output chunk, thread per topic: flattens the gathers into descriptors
//                   and marks where each k_copy tile starts.
//   k_copy          load-balanced streaming copy of every gathered list into output rows
//                   (coalesced 16-byte rows, eight loads in flight per lane).
//   k_merge         one wavefront (64 lanes) per topic: resolves the subscriptions of clients
//                   with several matching filters through their partner links
//                   (gatherSubscriptions + Subscription.Merge, topics.go:631-648,
//                   packets/packets.go:254-274) and applies the inline last-write rule
//                   (topics.go:668-676), with ballot/mbcnt compaction.
#include <hip/hip_runtime.h>

#include "kernels.h"

#include <algorithm>
#include <cstring>

namespace mq {

// ---------------------------------------------------------------------------------------------
// byte-level helpers over the topic buffer
// ---------------------------------------------------------------------------------------------
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Byte reader with a one-chunk register cache: one 16-byte load serves 16 sequential byte
// reads. The topic buffer must be readable up to its next 16-byte boundary (include/mqmatch.h):
// every chunk this reader loads holds at least one byte of the buffer. P: the position type —
// 32-bit positions (relative to a 16-byte-aligned base) save registers in the walk.
template <class P = uint64_t>
struct ByteReaderT {
  const uint8_t* base;
  P ci;
  u32x4 c;
  __device__ __forceinline__ explicit ByteReaderT(const uint8_t* b) : base(b), ci((P)~(P)0) {}
  __device__ __forceinline__ u32x4 chunk(P k) {
    if (k != ci) {
      c = *reinterpret_cast<const u32x4*>(base + ((uint64_t)k << 4));
      ci = k;
    }
    return c;
  }
  __device__ __forceinline__ uint32_t at(P i) {
    const u32x4 v = chunk(i >> 4);
    const uint32_t w = ((uint32_t)i >> 2) & 3;
    const uint32_t word = w == 0 ? v.x : (w == 1 ? v.y : (w == 2 ? v.z : v.w));
    return (word >> (((uint32_t)i & 3) * 8)) & 0xffu;
  }
};
using ByteReader = ByteReaderT<uint64_t>;

// SWAR segment scanning: a 16-byte chunk is searched for '/' with exact per-byte zero tests, so
// the walk does per-chunk rather than per-byte work; only segments longer than 15 bytes (hashed
// keys) are read byte by byte.
__device__ __forceinline__ uint32_t slash_nibble(uint32_t w) {  // bit i: byte i of w is '/'
  const uint32_t x = w ^ 0x2F2F2F2Fu;
  const uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);  // 0x80 where byte == 0
  return ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
}
__device__ __forceinline__ uint32_t slash_mask(const u32x4& c) {  // bit i: byte i of the chunk is '/'
  return slash_nibble(c.x) | (slash_nibble(c.y) << 4) | (slash_nibble(c.z) << 8) | (slash_nibble(c.w) << 12);
}

// First '/' in [s, end), or end. Bytes past `end` belong to the next topic.
template <class P>
__device__ __forceinline__ P find_slash(ByteReaderT<P>& R, P s, P end) {
  if (s >= end) return end;
  P k = s >> 4;
  uint32_t m = slash_mask(R.chunk(k)) & (0xFFFFu << (s & 15));
  for (;;) {
    if (m) return min((P)((k << 4) + (P)(__ffs(m) - 1)), end);
    k++;
    if ((k << 4) >= end) return end;
    m = slash_mask(R.chunk(k));
  }
}

// Start of the segment that ends at e: one past the last '/' in [b0, e), or b0.
template <class P>
__device__ __forceinline__ P seg_start_before(ByteReaderT<P>& R, P b0, P e) {
  if (e <= b0) return b0;
  P k = (e - 1) >> 4;
  const uint32_t top = (uint32_t)((e - 1) & 15);
  uint32_t m = slash_mask(R.chunk(k)) & (top == 15 ? 0xFFFFu : ((2u << top) - 1u));
  for (;;) {
    if (m) return max((P)((k << 4) + (P)(31 - __clz(m)) + 1), b0);
    if ((k << 4) <= b0) return b0;
    k--;
    m = slash_mask(R.chunk(k));
  }
}

// Key (layout.h) of the segment [s, e): inline segments (<= 15 bytes) are cut out of at most two
// chunks with funnel shifts; longer ones take the byte-wise hash of SegKeyBuilder.
template <class P>
__device__ __forceinline__ SegKey key_of(ByteReaderT<P>& R, P s, P e) {
  const uint32_t len = (uint32_t)(e - s);
  if (len > kInlineSegMax) {
    SegKeyBuilder kb;
    for (P i = s; i < e; i++) kb.push(R.at(i));
    return kb.finish();
  }
  if (len == 0) return SegKey{0, 0};
  const P k = s >> 4;
  const u32x4 c0 = R.chunk(k);
  const u32x4 c1 = ((e - 1) >> 4) != k ? R.chunk(k + 1) : u32x4{0u, 0u, 0u, 0u};
  const uint64_t q0 = c0.x | (uint64_t)c0.y << 32, q1 = c0.z | (uint64_t)c0.w << 32;
  const uint64_t q2 = c1.x | (uint64_t)c1.y << 32, q3 = c1.z | (uint64_t)c1.w << 32;
  const uint32_t o = (uint32_t)(s & 15);
  const uint64_t a = o >= 8 ? q1 : q0, b = o >= 8 ? q2 : q1, c = o >= 8 ? q3 : q2;
  const uint32_t sh = (o & 7) * 8;
  uint64_t v0 = sh ? (a >> sh) | (b << (64 - sh)) : a;
  uint64_t v1 = sh ? (b >> sh) | (c << (64 - sh)) : b;
  if (len < 8) v0 &= (1ull << (8 * len)) - 1;
  const uint32_t lb = len > 8 ? len - 8 : 0;  // <= 7 bytes in k1
  v1 = lb ? v1 & ((1ull << (8 * lb)) - 1) : 0ull;
  return SegKey{v0, v1 | ((uint64_t)len << 56)};
}

// Scan the segment that starts at s: returns the position of its terminating '/' (or end) and
// its key (layout.h).
template <class P>
__device__ __forceinline__ P scan_segment(ByteReaderT<P>& R, P s, P end, SegKey* key) {
  const P e = find_slash(R, s, end);
  *key = key_of(R, s, e);
  return e;
}

// wavefront helpers
__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

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

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int d = 32; d; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// Index of the calling wavefront in its workgroup, as a wave-uniform (scalar) value: the
// compiler cannot prove threadIdx.x >> 6 uniform, and per-wave work indexed by it would
// otherwise run as vector code under exec masks.
__device__ __forceinline__ uint32_t wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// particles.get(key) (topics.go:803-807) through the global edge table. The slot that names the
// child also carries the child's '+' and '#' children (EdgeSlot.plus / hash).
struct EdgeHit {
  uint32_t child, plus, hash;
};
__device__ __forceinline__ EdgeHit lookup_edge(const DevIndex& ix, uint32_t parent, const SegKey& k,
                                               const uint8_t* seg, uint32_t len) {
  uint64_t i = edge_hash(parent, k) & ix.edge_mask;
  for (uint64_t probes = 0; probes <= ix.edge_mask; probes++) {
    const EdgeSlot e = ix.edges[i];
    if (e.parent == kEdgeEmpty) break;
    if (e.parent == parent && e.k0 == k.k0 && e.k1 == k.k1) {
      if (!seg_is_long(k)) return EdgeHit{e.child, e.plus, e.hash};
      const SegInfo si = ix.seginfo[ix.walk[e.child].seg];
      bool eq = si.len == len;
      for (uint32_t j = 0; eq && j < len; j++) eq = ix.segbytes[si.off + j] == seg[j];
      if (eq) return EdgeHit{e.child, e.plus, e.hash};
    }
    i = (i + 1) & ix.edge_mask;
  }
  return EdgeHit{kNone, kNone, kNone};
}

__device__ __forceinline__ uint32_t lookup(const DevIndex& ix, uint32_t parent, const SegKey& k,
                                          const uint8_t* seg, uint32_t len) {
  return lookup_edge(ix, parent, k, seg, len).child;
}

// ---------------------------------------------------------------------------------------------
// k_walk: the match walk (thread per topic)
// ---------------------------------------------------------------------------------------------
// The reference's DFS (topics.go:603-625): at a particle, the literal child's subtree, then the
// '+' child's, then the '#' child's gather. A particle found by an edge probe comes with its '+'
// and '#' children (EdgeSlot.plus / hash), so going down costs one probe. Coming back up needs
// only the parent's '+' / '#' children (its literal child is done): for the first kWalkPath
// levels they wait in LDS (8 B per level and thread), deeper levels return through the parent
// pointers of the NodeWalk records (the stackless form).
// FILL=false: count pass; also writes the first kGatherCap gathers of each topic to its slot
// of `gathers` (stride kGatherCap) and flags a topic with more. FILL=true: writes every gather
// compactly at off[t].g (run only when some topic overflowed its slot).
// LISTS=true: the count pass reads each gathered particle's lists (rows, shared, inline and
// may-merge counts); LISTS=false: gathers only (k_desc<true> reads the lists).
constexpr uint32_t kWalkPath = 8;
// WPE: minimum waves per SIMD asked of the register allocator (1: no constraint).
template <bool FILL, bool LISTS>
__device__ __forceinline__ void walk_topic(uint32_t t, const uint8_t* __restrict__ tb, const uint64_t* __restrict__ to,
                                           const DevIndex& ix, TopicCount* __restrict__ cnt,
                                           const TopicOff* __restrict__ off, uint32_t* __restrict__ gathers,
                                           uint32_t* __restrict__ ovf, uint2 (*path)[256], bool clamp) {
  const uint64_t a0 = to[t], a1 = to[t + 1];
  uint32_t ng = 0, rows = 0, shared = 0, inl = 0, merge = 0;
  uint32_t* gout = FILL ? gathers + off[t].g : gathers + (uint64_t)t * kGatherCap;

  if (a1 > a0) {  // Subscribers("") matches nothing (topics.go:598-600)
    // positions relative to the 16-byte chunk that holds the topic's first byte (a topic is far
    // shorter than 4 GB: MQTT caps it at 65,535 bytes)
    const uint8_t* tbase = tb + (a0 & ~15ull);
    const uint32_t b0 = (uint32_t)(a0 & 15), b1 = b0 + (uint32_t)(a1 - a0);
    ByteReaderT<uint32_t> R(tbase);
    const bool dollar = R.at(b0) == '$';
    // gather{Subscriptions,SharedSubscriptions,InlineSubscriptions} of one particle; wild: the
    // particle's path starts with a '+'/'#' segment (kFlagSeg0Wild)
    auto gather = [&](uint32_t node, bool with_inline, bool wild) __attribute__((always_inline)) {
      if (LISTS) {
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
          if (with_inline && (L.flags & kFlagInline)) inl += ix.inls[node].cnt;
        }
      } else {
        const bool subs_ok = !(dollar && wild);
        const uint32_t gw = node | (subs_ok ? kGatherSubs : 0u) | (with_inline ? kGatherInline : 0u);
        if (FILL || ng < kGatherCap) gout[ng] = gw;
      }
      ng++;
    };

    uint2* my_path = &path[0][threadIdx.x];  // level d at my_path[d * 256]
    uint32_t p_isplus = 0;                   // bit d: the particle at depth d + 1 is a '+' child
    const NodeWalk rw = ix.walk[kRoot];
    uint32_t node = kRoot, plus = rw.plus_child, hash = rw.hash_child, depth = 0;
    bool wild0 = false;  // segment 0 of the path is '+'/'#'
    SegKey key;
    uint32_t s = b0, e = scan_segment(R, b0, b1, &key);
    int state = 0;  // 0: literal child next, 1: '+' child next, 2: '#' gather and return
    // go down to child c (its '+' / '#' children known), to match the next segment
    auto descend = [&](uint32_t c, uint32_t cp, uint32_t ch, bool isplus) __attribute__((always_inline)) {
      if (depth < kWalkPath) my_path[depth * 256] = make_uint2(plus, hash);
      if (depth < 32) p_isplus = isplus ? (p_isplus | (1u << depth)) : (p_isplus & ~(1u << depth));
      depth++;
      node = c;
      plus = cp;
      hash = ch;
      s = e + 1;
      e = scan_segment(R, s, b1, &key);
      state = 0;
    };
    for (uint32_t guard = 0;; guard++) {
      if (guard > kWalkGuard) {  // never reached on a well-formed image; fail loudly, not hang
        atomicOr(ix.err, kErrWalkGuard);
        break;
      }
      const bool has_next = e < b1;
      const bool at_root = depth == 0;
      if (state == 0) {
        state = 1;
        const uint32_t len = (uint32_t)(e - s);
        const uint32_t c0 = len ? R.at(s) : 0u;  // an empty last segment may end the buffer
        // A literal "+" segment makes the reference visit the '+' child twice with identical
        // results (topics.go:603); the '+' branch below covers it.
        if (!(len == 1 && c0 == '+')) {
          const EdgeHit h = lookup_edge(ix, node, key, tbase + s, len);
          if (h.child != kNone) {
            const bool cw = at_root ? (c0 == '+' || c0 == '#') : wild0;
            if (has_next) {
              if (at_root) wild0 = cw;
              descend(h.child, h.plus, h.hash, false);
              continue;
            }
            gather(h.child, true, cw);
            if (h.hash != kNone) gather(h.hash, false, cw);  // filter/# matches filter (topics.go:612)
          }                                                   // inline: the particle's own again (Q2)
        }
      }
      if (state == 1) {
        state = 2;
        if (plus != kNone) {
          if (has_next) {
            const NodeWalk pw = ix.walk[plus];
            if (at_root) wild0 = true;
            descend(plus, pw.plus_child, pw.hash_child, true);
            continue;
          }
          gather(plus, true, at_root || wild0);
        }
      }
      if (hash != kNone) gather(hash, true, at_root || wild0);  // topics.go:621-625
      if (at_root) break;
      // return to the parent: its '+' / '#' children, and continue after this branch
      const bool was_plus = depth - 1 < 32 ? ((p_isplus >> (depth - 1)) & 1u) != 0
                                           : (ix.walk[node].parent_flags & kFlagPlusKey) != 0;
      state = was_plus ? 2 : 1;
      depth--;
      if (depth < kWalkPath) {
        const uint2 ph = my_path[depth * 256];
        plus = ph.x;
        hash = ph.y;
        // `node` is not needed above kWalkPath: the parent's literal child is done, and every
        // return from here on reads the path
      } else {
        node = ix.walk[node].parent_flags & kParentMask;
        const NodeWalk pw = ix.walk[node];
        plus = pw.plus_child;
        hash = pw.hash_child;
      }
      e = s - 1;
      s = seg_start_before(R, b0, e);
    }
  }
  if (!FILL) {
    TopicCount c;
    c.gathers = clamp ? min(ng, kGatherCap) : ng;
    c.rows = rows;
    c.shared = shared;
    c.inlines = inl;
    c.merge = merge;
    cnt[t] = c;
    if (ng > kGatherCap) atomicOr(ovf, 1u);
  }
}

// list == null: thread per topic t < n. Else the topics list[0, *n_list), grid-stride (the
// frontier walk's fallback: its length is known on the device only).
template <bool FILL, bool LISTS, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_walk(const uint8_t* __restrict__ tb,
                                              const uint64_t* __restrict__ to, uint32_t n,
                                              DevIndex ix, TopicCount* __restrict__ cnt,
                                              const TopicOff* __restrict__ off,
                                              uint32_t* __restrict__ gathers, uint32_t* __restrict__ ovf,
                                              const uint32_t* __restrict__ list, const uint32_t* __restrict__ n_list,
                                              bool clamp) {
  __shared__ uint2 path[kWalkPath][256];  // level d: the '+' / '#' children of the particle at depth d
  const uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x;
  if (!list) {
    if (i0 < n) walk_topic<FILL, LISTS>(i0, tb, to, ix, cnt, off, gathers, ovf, path, clamp);
    return;
  }
  const uint32_t nl = *n_list;
  for (uint32_t i = i0; i < nl; i += gridDim.x * blockDim.x)
    walk_topic<FILL, LISTS>(list[i], tb, to, ix, cnt, off, gathers, ovf, path, clamp);
}

// ---------------------------------------------------------------------------------------------
// k_walkf: the match walk as a level-synchronous frontier expansion (the north-star design):
// G lanes per topic (64 / G topics per wavefront). The group tokenises its topic together —
// lane j takes 16-byte chunks j, j + G, ... (coalesced), finds the '/' bytes with SWAR masks
// and places them with a group prefix sum — then walks it level by level. The frontier (the
// particles that match the topic's first d segments, each with its '+' / '#' children and its
// path code) is held one particle per lane; at level d every lane probes its particle's literal
// child and reads its '+' child's walk record at once, so a topic costs about two dependent
// round trips per level instead of one per probe of the reference's recursion, and the
// wavefront's loads are issued together. Gathers are staged in LDS with their DFS rank — the
// path code of SURVEY.md App. A.3, two bits per level (literal 1, '+' 2, '#' 3), zero padded,
// so that comparing ranks is comparing positions in scanSubscribers' order (topics.go:603-625):
// the literal subtree, then the '+' subtree, then the '#' gather; at the final level the
// particle before its '#' child (topics.go:612). The group then sorts them by rank (each lane
// counts the smaller ranks) and writes them in the reference's order, exactly what k_walk
// writes. A topic the frontier cannot hold — more than kFrontLevels levels (the rank's 32 bits),
// more than G particles at one level, more than kGatherCap gathers — goes to `fb_list` and is
// walked by k_walk (thread per topic, stackless DFS) right after.
// ---------------------------------------------------------------------------------------------
constexpr uint32_t kFrontLevels = 15;  // levels a topic may have: its deepest gather rank needs 2 bits more

// Inclusive prefix sum over the G lanes of a group (G a power of two <= 64; sub = lane % G).
template <uint32_t G>
__device__ __forceinline__ uint32_t grp_incl(uint32_t v, uint32_t sub) {
#pragma unroll
  for (uint32_t d = 1; d < G; d <<= 1) {
    const uint32_t y = __shfl_up(v, d, G);
    if (sub >= d) v += y;
  }
  return v;
}
template <uint32_t G>
__device__ __forceinline__ uint32_t grp_sum(uint32_t v) {
#pragma unroll
  for (uint32_t d = 1; d < G; d <<= 1) v += __shfl_xor(v, d, G);
  return v;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
  for (int d = 32; d; d >>= 1) v = max(v, (uint32_t)__shfl_xor(v, d, 64));
  return v;
}

struct FrontEnt {  // one frontier particle: its '+' / '#' children and its path code
  uint32_t node, plus, hash, code;
};

// WPE: waves per SIMD asked of the register allocator (8: a few SGPRs spill to VGPR lanes; 1:
// no constraint, 7 waves).
template <uint32_t G, class GW>
__device__ __forceinline__ void desc_grp(const DescArgs& a, uint32_t t, uint32_t n_g, uint64_t g0, uint64_t ipos,
                                         uint32_t shr0, uint32_t sub, GW gw_at);

// DESC (G = 16, LISTS = false): k_desc fused into the epilogue — the gathers, placed in the
// reference's order in LDS, go straight to the topic's spans and merge lists (desc_g16 with the
// stride layout, da.g_stride); neither the gather slots nor the counts are written.
template <uint32_t G, bool LISTS, int WPE, bool DESC = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_walkf(const uint8_t* __restrict__ tb, const uint64_t* __restrict__ to,
                                               uint32_t n, DevIndex ix, TopicCount* __restrict__ cnt,
                                               uint32_t* __restrict__ gathers, uint32_t* __restrict__ fb_list,
                                               uint32_t* __restrict__ fb_count, DescArgs da) {
  static_assert(!DESC || ((G == 16 || G == 8) && !LISTS), "the fused desc runs on 8- or 16-lane groups of a gathers-only walk");
  constexpr uint32_t kTopics = 256 / G;  // topics per workgroup
  // levels and gathers a group holds: 8-lane groups keep 32 topics per workgroup within 20 KB of
  // LDS (8 workgroups per CU: twice the topics in flight of 16-lane groups); a topic beyond them
  // is walked by k_walk
  constexpr uint32_t kLv = G >= 16 ? kFrontLevels : 10u;
  constexpr uint32_t kStage = G >= 16 ? kGatherCap : 24u;
  __shared__ uint32_t sl[kTopics][kLv];      // '/' positions (relative to the topic's chunk base)
  __shared__ uint4 skey[kTopics][kLv];       // each level's segment key (SegKey)
  __shared__ uint2 sseg[kTopics][kLv];       // ... its start, and length | "+" segment << 31
  __shared__ uint2 gat[kTopics][kStage];     // staged gathers: (word, rank)
  __shared__ FrontEnt xf[kTopics][G];                 // next level's frontier, compacted
  const uint32_t q = threadIdx.x / G, sub = threadIdx.x % G;
  const uint32_t t = blockIdx.x * kTopics + q;
  const bool live = t < n;
  uint64_t a0 = 0, a1 = 0;
  if (live) {
    a0 = to[t];
    a1 = to[t + 1];
  }
  const uint8_t* tbase = tb + (a0 & ~15ull);
  const uint32_t b0 = (uint32_t)(a0 & 15), b1 = b0 + (uint32_t)(a1 - a0);
  ByteReaderT<uint32_t> R(tbase);
  // --- tokenise: the group's lanes over the topic's chunks -------------------------------------
  const uint32_t nch = a1 > a0 ? (b1 + 15) >> 4 : 0u;
  uint32_t nsl = 0;  // '/' found so far (group-uniform)
  const uint32_t rounds = wave_max((nch + G - 1) / G);
  for (uint32_t r = 0; r < rounds; r++) {
    const uint32_t k = r * G + sub;
    uint32_t m = 0;
    if (k < nch) {
      m = slash_mask(*reinterpret_cast<const u32x4*>(tbase + ((uint64_t)k << 4)));
      if (k == 0) m &= 0xFFFFu << b0;
      if (k == nch - 1 && (b1 & 15)) m &= (1u << (b1 & 15)) - 1u;
    }
    const uint32_t c = __popc(m);
    const uint32_t inc = grp_incl<G>(c, sub);
    uint32_t idx = nsl + inc - c;
    for (; m; m &= m - 1, idx++)
      if (idx < kLv) sl[q][idx] = (k << 4) + (uint32_t)(__ffs(m) - 1);
    nsl += __shfl(inc, G - 1, G);
  }
  const uint32_t L = nch ? nsl + 1 : 0u;  // levels (0: the empty topic, which matches nothing)
  bool fb = live && L > kLv;
  wave_sync_lds();
  // every level's key, lanes over the levels: the walk below then reads them from LDS instead of
  // loading topic bytes on each level's critical path
  if (live && !fb)
    for (uint32_t d = sub; d < L; d += G) {
      const uint32_t s = d ? sl[q][d - 1] + 1 : b0, e = d + 1 < L ? sl[q][d] : b1;
      const SegKey k = key_of(R, s, e);
      const bool plusseg = e - s == 1 && R.at(s) == '+';
      skey[q][d] = make_uint4((uint32_t)k.k0, (uint32_t)(k.k0 >> 32), (uint32_t)k.k1, (uint32_t)(k.k1 >> 32));
      sseg[q][d] = make_uint2(s, (e - s) | (plusseg ? 0x80000000u : 0u));
    }
  const bool dollar = L && R.at(b0) == '$';
  bool lit0wild = false;  // segment 0 starts with '+' / '#' (a literal child there is 'wild', Q3)
  if (L) {
    const uint32_t e0 = L > 1 ? sl[q][0] : b1;
    if (e0 > b0) {
      const uint32_t c0 = R.at(b0);
      lit0wild = c0 == '+' || c0 == '#';
    }
  }
  wave_sync_lds();
  // --- the frontier, level by level ------------------------------------------------------------
  FrontEnt fe{kNone, kNone, kNone, 0u};
  if (sub == 0) {
    const NodeWalk rw = ix.walk[kRoot];
    fe = FrontEnt{kRoot, rw.plus_child, rw.hash_child, 0u};
  }
  uint32_t F = 1, ng = 0;  // frontier size, gathers staged (group-uniform)
  const uint32_t levels = wave_max(live && !fb ? L : 0u);
  for (uint32_t d = 0; d < levels; d++) {
    const bool act = live && !fb && d < L && F != 0;
    const bool mine = act && sub < F;
    const bool has_next = d + 1 < L;
    const uint32_t sh = 30 - 2 * d;  // level d's two bits of the rank
    SegKey key{0, 0};
    uint32_t s = 0, len = 0;
    bool plusseg = false;
    if (act) {
      const uint4 kk = skey[q][d];
      const uint2 sg = sseg[q][d];
      key = SegKey{kk.x | (uint64_t)kk.y << 32, kk.z | (uint64_t)kk.w << 32};
      s = sg.x;
      len = sg.y & 0x7FFFFFFFu;
      plusseg = (sg.y >> 31) != 0;
    }
    NodeWalk pw{kNone, kNone, 0, 0};
    if (mine && has_next && fe.plus != kNone) pw = ix.walk[fe.plus];
    EdgeHit h{kNone, kNone, kNone};
    // a literal "+" segment: the reference visits the '+' child twice alike (topics.go:603)
    if (mine && !plusseg) h = lookup_edge(ix, fe.node, key, tbase + s, len);
    // this lane's gathers (at most four): the particle's '#' child (topics.go:621); at the last
    // level the literal child, its '#' child (filter/# matches filter, topics.go:612; inline: the
    // particle's own again, Q2) and the '+' child
    const bool gH = mine && fe.hash != kNone;
    const bool gL = mine && !has_next && h.child != kNone;
    const bool gC = gL && h.hash != kNone;
    const bool gP = mine && !has_next && fe.plus != kNone;
    const uint32_t gc = (uint32_t)gH + (uint32_t)gL + (uint32_t)gC + (uint32_t)gP;
    const uint32_t gi = grp_incl<G>(gc, sub);
    const uint32_t gtot = __shfl(gi, G - 1, G);
    if (act && ng + gtot > kStage) fb = true;
    if (act && !fb) {
      uint32_t p = ng + gi - gc;
      if (gH) gat[q][p++] = make_uint2(fe.hash | kGatherInline, fe.code | 3u << sh);
      if (gL) gat[q][p++] = make_uint2(h.child | kGatherInline, fe.code | 1u << sh);
      if (gC) gat[q][p++] = make_uint2(h.hash, fe.code | 1u << sh | 3u << (sh - 2));
      if (gP) gat[q][p++] = make_uint2(fe.plus | kGatherInline, fe.code | 2u << sh);
    }
    ng += gtot;
    // next level's frontier: the literal and '+' children, compacted over the group
    const bool fL = mine && has_next && h.child != kNone;
    const bool fP = mine && has_next && fe.plus != kNone;
    const uint32_t fc = (uint32_t)fL + (uint32_t)fP;
    const uint32_t fi = grp_incl<G>(fc, sub);
    const uint32_t ftot = __shfl(fi, G - 1, G);
    if (act && has_next && ftot > G) fb = true;
    if (act && !fb && has_next) {
      uint32_t p = fi - fc;
      if (fL) xf[q][p++] = FrontEnt{h.child, h.plus, h.hash, fe.code | 1u << sh};
      if (fP) xf[q][p] = FrontEnt{fe.plus, pw.plus_child, pw.hash_child, fe.code | 2u << sh};
    }
    wave_sync_lds();
    if (act) {
      F = has_next ? ftot : 0u;
      if (!fb && sub < F) fe = xf[q][sub];
    }
    wave_sync_lds();  // the frontier is read before the next level overwrites it
  }
  if (!live) return;
  if (fb) {
    if (sub == 0) fb_list[atomicAdd(fb_count, 1u)] = t;
    return;
  }
  // --- the gathers in the reference's order ------------------------------------------------------
  wave_sync_lds();
  if (DESC) {
    // each gather's place (the smaller ranks), then the words in place in LDS, then k_desc's work
    constexpr uint32_t kPer = (kStage + G - 1) / G;  // gathers per lane
    uint32_t pw[kPer], ww[kPer];
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
      const uint32_t i = sub + k * G;
      pw[k] = kNone;
      if (i < ng) {
        const uint2 gi = gat[q][i];
        uint32_t pos = 0;
        for (uint32_t j = 0; j < ng; j++) pos += gat[q][j].y < gi.y ? 1u : 0u;
        const uint32_t k0 = gi.y >> 30;  // how the path starts: literal 1, '+' 2, '#' 3
        const bool wild = k0 >= 2 || (k0 == 1 && lit0wild);
        pw[k] = pos;
        ww[k] = gi.x | (!(dollar && wild) ? kGatherSubs : 0u);
      }
    }
    wave_sync_lds();
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++)
      if (pw[k] != kNone) gat[q][pw[k]].x = ww[k];
    wave_sync_lds();
    desc_grp<G>(da, t, ng, (uint64_t)t * da.g_stride, 0ull, 0u, sub, [&](uint32_t i) { return gat[q][i].x; });
    return;
  }
  uint32_t rows = 0, shared = 0, inl = 0, merge = 0;
  uint32_t* gout = gathers + (uint64_t)t * kGatherCap;
  for (uint32_t i = sub; i < ng; i += G) {
    const uint2 gi = gat[q][i];
    uint32_t pos = 0;
    for (uint32_t j = 0; j < ng; j++) pos += gat[q][j].y < gi.y ? 1u : 0u;
    const uint32_t node = gi.x & kGatherNode;
    uint32_t gw = gi.x;
    if (LISTS) {
      const NodeLists Ls = ix.lists[node];
      // [MQTT-4.7.1-1]: '$' topics skip subscriptions whose filter starts with '+'/'#' (Q3)
      const bool subs_ok = !(dollar && (Ls.flags & kFlagSeg0Wild));
      if (subs_ok) {
        gw |= kGatherSubs;
        rows += Ls.n_direct + Ls.n_merge;
        merge += Ls.n_merge;
      }
      shared += Ls.shr_cnt;
      if ((gi.x & kGatherInline) && (Ls.flags & kFlagInline)) inl += ix.inls[node].cnt;
    } else {
      const uint32_t k0 = gi.y >> 30;  // how the path starts: literal 1, '+' 2, '#' 3
      const bool wild = k0 >= 2 || (k0 == 1 && lit0wild);
      if (!(dollar && wild)) gw |= kGatherSubs;
    }
    gout[pos] = gw;
  }
  if (LISTS) {
    rows = grp_sum<G>(rows);
    shared = grp_sum<G>(shared);
    inl = grp_sum<G>(inl);
    merge = grp_sum<G>(merge);
  }
  if (sub == 0) {
    TopicCount c;
    c.gathers = ng;
    c.rows = rows;
    c.shared = shared;
    c.inlines = inl;
    c.merge = merge;
    cnt[t] = c;
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
  a.merge += c.merge;
}
__device__ __forceinline__ void add_off(TopicOff& a, const TopicOff& b) {
  a.g += b.g;
  a.rows += b.rows;
  a.shr += b.shr;
  a.inl += b.inl;
  a.merge += b.merge;
}
__device__ __forceinline__ TopicOff shfl_up_off(const TopicOff& v, int d) {
  TopicOff r;
  r.g = __shfl_up(v.g, d, 64);
  r.rows = __shfl_up(v.rows, d, 64);
  r.shr = __shfl_up(v.shr, d, 64);
  r.inl = __shfl_up(v.inl, d, 64);
  r.merge = __shfl_up(v.merge, d, 64);
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
    ex.g -= v.g; ex.rows -= v.rows; ex.shr -= v.shr; ex.inl -= v.inl; ex.merge -= v.merge;
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
  ex.g -= v.g; ex.rows -= v.rows; ex.shr -= v.shr; ex.inl -= v.inl; ex.merge -= v.merge;
  for (int k = 0; k < 4; k++) {
    if (base + k < n) off[base + k] = ex;
    add_count(ex, c[k]);
  }
  if (base + 3 >= (uint64_t)n - 1 && base < n) off[n] = bpre[gridDim.x];
}

// ---------------------------------------------------------------------------------------------
// Emit: every gathered subscription list becomes output rows.
//   k_desc   thread per topic: flattens the topic's gathers into GDesc records and marks the
//            k_copy tiles that start inside each gather.
//   k_copy   load-balanced streaming copy: each wavefront moves kCopyTile consecutive rows of
//            one stream (direct client rows, shared rows, inline rows) of the whole chunk,
//            whatever topics and gathers they belong to — 64 consecutive rows per
//            wave-instruction, eight loads in flight per lane.
//   k_merge  wavefront per topic: resolves the may-merge records through their partner links
//            (gatherSubscriptions + Subscription.Merge, topics.go:631-648,
//            packets/packets.go:254-274), applies the inline last-write rule (topics.go:668-676)
//            and writes the topic's result record.
// ---------------------------------------------------------------------------------------------
// SPANS=false (row format): positions are relative to the topic's output chunk and the k_copy
// tiles starting in each gather are marked. SPANS=true: positions are topic-relative (k_merge
// patches name a topic's rows), every gather also becomes a SpanRec at its gather index, and
// the gathered inline rows are copied to off[t].inl for k_merge's last-write pass.
template <bool SPANS>
__global__ __launch_bounds__(256) void k_desc(DescArgs a) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= a.n) return;
  const TopicOff o0 = a.off[t], o1 = a.off[t + 1];
  ChunkPlan cp{0, 0, 0, 0, 0, 0, 0};
  if (!SPANS) cp = a.plan[a.chunk_of_block[t / kScanBlock]];
  uint32_t rpos = SPANS ? 0u : (uint32_t)(o0.rows - cp.rows);
  uint32_t spos = (uint32_t)(o0.shr - cp.shr);
  uint64_t ipos = o0.inl - cp.inl;
  const uint32_t n_g = (uint32_t)(o1.g - o0.g);
  uint32_t* tile_r = SPANS ? nullptr : a.tiles + cp.tile_off;
  uint32_t* tile_s = SPANS ? nullptr : tile_r + cp.n_tiles0;
  uint32_t* tile_i = SPANS ? nullptr : tile_s + cp.n_tiles1;
  const uint32_t* gw_src = a.gather_stride ? a.gathers + (uint64_t)t * a.gather_stride : a.gathers + o0.g;
  uint32_t n_merge = 0;
  uint64_t msig = 0x6D657267652D7365ull;  // merge-set signature (a.msig)
  uint32_t n_mg = 0;
  // four gathers per round: their gather words, lists and pair-block headers are loaded together
  // (one latency per round instead of per gather)
  constexpr uint32_t U = 4;
  for (uint32_t i0 = 0; i0 < n_g; i0 += U) {
    uint32_t gwv[U];
    NodeLists Lv[U];
#pragma unroll
    for (uint32_t u = 0; u < U; u++) gwv[u] = i0 + u < n_g ? gw_src[i0 + u] : 0u;
#pragma unroll
    for (uint32_t u = 0; u < U; u++) Lv[u] = a.ix.lists[gwv[u] & kGatherNode];
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
    const uint32_t i = i0 + u;
    if (i >= n_g) break;
    const uint32_t gw = gwv[u];
    const NodeLists& L = Lv[u];
    const uint32_t rn = (gw & kGatherSubs) ? L.n_direct + L.n_merge : 0u;
    const NodeInl I = ((gw & kGatherInline) && (L.flags & kFlagInline)) ? a.ix.inls[gw & kGatherNode] : NodeInl{0, 0};
    const uint32_t in = I.cnt;
    const uint64_t g = o0.g + i;
    GDesc d;
    d.r_pos = rpos;
    d.r_src = L.sub_off;
    d.s_pos = spos;
    d.s_src = L.shr_off;
    d.i_pos = (uint32_t)ipos;
    d.i_src = I.off;
    d.word = gw;
    d.mdir = L.n_direct | ((gw & kGatherSubs) && L.n_merge ? kDescMerge : 0u);
    if (SPANS) {  // k_merge reads the pair block's header (and the rank key) from here
      d.i_pos = 0;
      d.i_src = 0;
      if (d.mdir & kDescMerge) {
        d.s_pos = L.ent_off;
        d.s_src = L.ent_mask;
        if (a.ix.xinfo) {
          const uint64_t rk = a.ix.xinfo[gw & kGatherNode].rank;
          d.i_pos = (uint32_t)rk;
          d.i_src = (uint32_t)(rk >> 32);
        }
      }
    }
    if (!SPANS || !a.msig) a.desc[g] = d;  // dedup lists: GDesc only for a wide topic (below)
    if (SPANS) {
      if (gw & kGatherSubs) n_merge += L.n_merge;
      if (a.msig && (d.mdir & kDescMerge)) {
        msig = mix64(msig ^ (gw & kGatherNode)) + 0x9e3779b97f4a7c15ull;
        if (n_mg < kPairMax) {
          a.mlist[(uint64_t)t * kPairMax + n_mg] = gw & kGatherNode;
          a.mrow[(uint64_t)t * kPairMax + n_mg] = rpos;
          a.mpair[(uint64_t)t * kPairMax + n_mg] = make_uint2(d.s_pos, d.s_src);
        }
        // set-relative rows hold 26 bits of slot: a larger merge gather keeps the topic apart
        n_mg += L.n_direct + L.n_merge < (1u << kSetRowBits) ? 1u : kPairMax + 1;
      }
      a.spans[g] = SpanRec{L.sub_off, rn, L.shr_off, L.shr_cnt};
      for (uint32_t k = 0; k < in; k++) a.inl_out[ipos + k] = a.ix.inl[I.off + k];
    } else {
      // the k_copy tiles whose first row falls inside this gather start their cursor here
      for (uint32_t k = (rpos + kCopyTile - 1) / kCopyTile; k * kCopyTile < rpos + rn; k++) tile_r[k] = (uint32_t)g;
      for (uint32_t k = (spos + kCopyTile - 1) / kCopyTile; k * kCopyTile < spos + L.shr_cnt; k++) tile_s[k] = (uint32_t)g;
      for (uint64_t k = (ipos + kCopyTile - 1) / kCopyTile; k * kCopyTile < ipos + in; k++) tile_i[k] = (uint32_t)g;
    }
    rpos += rn;
    spos += L.shr_cnt;
    ipos += in;
    }
  }
  if (SPANS && a.tc_out) a.tc_out[t] = TopicCount{n_g, rpos, spos - (uint32_t)o0.shr, 0u, n_merge};
  if (SPANS && a.msig) {
    a.msig[t] = msig | 1ull;  // never 0 (the dedup table's empty key)
    a.mcount[t] = n_mg;
    if (n_mg > kPairMax) {  // k_merge maps this topic from its GDesc records: write them (rare)
      uint32_t rp = 0, sp = (uint32_t)o0.shr;
      for (uint32_t i = 0; i < n_g; i++) {
        const uint32_t gw = gw_src[i];
        const NodeLists L = a.ix.lists[gw & kGatherNode];
        const bool mg = (gw & kGatherSubs) && L.n_merge;
        a.desc[o0.g + i] = GDesc{rp, L.sub_off, mg ? L.ent_off : sp, mg ? L.ent_mask : L.shr_off, 0u, 0u, gw,
                                 L.n_direct | (mg ? kDescMerge : 0u)};
        rp += (gw & kGatherSubs) ? L.n_direct + L.n_merge : 0u;
        sp += L.shr_cnt;
      }
    }
  }
}

// 16-lane inclusive scan (lanes of a 16-lane group of the wavefront; sub = lane & 15)
__device__ __forceinline__ uint32_t g16_incl(uint32_t v, uint32_t sub) {
#pragma unroll
  for (uint32_t d = 1; d < 16; d <<= 1) {
    const uint32_t y = __shfl_up(v, d, 16);
    if (sub >= d) v += y;
  }
  return v;
}

// The GDesc records of one topic's gathers for k_merge's slow paths (a topic beyond the map):
// rows topic-relative, a merge gather's pair-block header in s_pos / s_src and, on a sharded
// index, its rank key in i_pos (low) / i_src (high).
__device__ __forceinline__ void write_gdesc(const DevIndex& ix, const uint32_t* gw_src, uint32_t n_g, uint32_t sp,
                                            GDesc* out) {
  uint32_t rp = 0;
  for (uint32_t i = 0; i < n_g; i++) {
    const uint32_t gw = gw_src[i];
    const NodeLists L = ix.lists[gw & kGatherNode];
    const bool mg = (gw & kGatherSubs) && L.n_merge;
    const uint64_t rk = mg && ix.xinfo ? ix.xinfo[gw & kGatherNode].rank : 0ull;
    out[i] = GDesc{rp, L.sub_off, mg ? L.ent_off : sp, mg ? L.ent_mask : L.shr_off, (uint32_t)rk, (uint32_t)(rk >> 32),
                   gw, L.n_direct | (mg ? kDescMerge : 0u)};
    rp += (gw & kGatherSubs) ? L.n_direct + L.n_merge : 0u;
    sp += L.shr_cnt;
  }
}

// k_desc for the span format with merge-set dedup lists (the default): 16 lanes per topic, four
// topics per wavefront, the lanes over the topic's gathers. A topic's gather words, spans and
// merge lists are contiguous, so its loads and stores coalesce; a thread per topic stores to 64
// scattered places per instruction (1.18 GB written per 1M topics at 10M subscriptions for
// 0.3 GB of records). Same outputs as k_desc<true> with dedup lists; the merge-set signature is
// position-keyed (a sum over the merge gathers of a hash of (particle, merge index)).
// desc_g16: one topic on its 16-lane group (sub = lane & 15; group-uniform control flow): n_g
// gathers, gw_at(i) the word of gather i, spans / GDesc at g0, inline rows copied to ipos, shared
// rows counted from shr0 (GDesc records only). Also run by the walk-fused k_walkf<..., DESC>.
__device__ __forceinline__ uint32_t dedup_insert(unsigned long long* keys, uint32_t* vals, uint64_t mask, uint32_t t,
                                                bool ok, unsigned long long k);

template <uint32_t G, class GW>
__device__ __forceinline__ void desc_grp(const DescArgs& a, uint32_t t, uint32_t n_g, uint64_t g0, uint64_t ipos,
                                         uint32_t shr0, uint32_t sub, GW gw_at) {
  // one-sync batch: spans past the buffer are not written (the batch runs again, host-sized)
  const bool fits = !a.unsafe || g0 + n_g <= a.spans_cap;
  if (!fits && sub == 0) atomicOr(a.unsafe, kUnsafeSpans);
  uint32_t rpos = 0, spos = 0, n_mg = 0, n_merge = 0;
  uint64_t sig = 0;
  for (uint32_t r0 = 0; r0 < n_g; r0 += G) {
    const uint32_t i = r0 + sub;
    const bool act = i < n_g;
    uint32_t gw = 0;
    NodeLists L = kEmptyLists;
    if (act) {  // one record per gathered particle: its lists and its pair-block header
      gw = gw_at(i);
      L = a.ix.lists[gw & kGatherNode];
    }
    const bool subs = act && (gw & kGatherSubs);
    const uint32_t rn = subs ? L.n_direct + L.n_merge : 0u;
    const NodeInl I = (act && (gw & kGatherInline) && (L.flags & kFlagInline)) ? a.ix.inls[gw & kGatherNode]
                                                                                 : NodeInl{0, 0};
    const uint32_t in = I.cnt;
    const bool ismg = subs && L.n_merge != 0;
    // set-relative rows hold 26 bits of slot: a larger merge gather keeps the topic apart
    const uint32_t inc = ismg ? (L.n_direct + L.n_merge < (1u << kSetRowBits) ? 1u : kPairMax + 1) : 0u;
    const uint32_t rn_i = grp_incl<G>(rn, sub), in_i = grp_incl<G>(in, sub), inc_i = grp_incl<G>(inc, sub);
    const uint32_t sh_i = grp_incl<G>(act ? L.shr_cnt : 0u, sub);
    const uint32_t rp = rpos + rn_i - rn, x = n_mg + inc_i - inc;
    const uint64_t ip = ipos + (in_i - in);
    if (act && fits) a.spans[g0 + i] = SpanRec{L.sub_off, rn, L.shr_off, L.shr_cnt};
    for (uint32_t k = 0; k < in; k++) a.inl_out[ip + k] = a.ix.inl[I.off + k];
    if (ismg) {
      sig += mix64(((uint64_t)x << 32 | (gw & kGatherNode)) + 0x9e3779b97f4a7c15ull);
      if (x < kPairMax) {
        const uint64_t q = (uint64_t)t * kPairMax + x;
        a.mlist[q] = gw & kGatherNode;
        a.mrow[q] = rp;
        a.mpair[q] = make_uint2(L.ent_off, L.ent_mask);
        if (a.mrank) a.mrank[q] = a.ix.xinfo[gw & kGatherNode].rank;
      }
    }
    if (subs) n_merge += L.n_merge;
    rpos += __shfl(rn_i, G - 1, G);
    spos += __shfl(sh_i, G - 1, G);
    ipos += __shfl(in_i, G - 1, G);
    n_mg += __shfl(inc_i, G - 1, G);
  }
#pragma unroll
  for (uint32_t d = 1; d < G; d <<= 1) {
    sig += __shfl_xor(sig, d, G);
    n_merge += __shfl_xor(n_merge, d, G);
  }
  const unsigned long long msig = mix64(sig + n_mg) | 1ull;  // never 0 (the dedup table's empty key)
  if (a.dd_keys) {  // k_dedup_insert's work, one lane per topic
    const uint32_t slot = dedup_insert(a.dd_keys, a.dd_vals, a.dd_mask, t, sub == 0 && n_mg != 0 && n_mg <= kPairMax,
                                       msig);
    if (sub == 0) a.dd_tslot[t] = slot;
  }
  if (sub != 0) return;
  if (a.tc_out) a.tc_out[t] = TopicCount{n_g, rpos, spos, 0u, n_merge};
  a.msig[t] = msig;
  a.mcount[t] = n_mg;
  // k_merge maps this topic from its GDesc records: write them (rare; gather words re-read)
  if (n_mg > kPairMax) {
    if (!a.unsafe || g0 + n_g <= a.desc_cap) {
      uint32_t rp = 0, sp = shr0;
      for (uint32_t i = 0; i < n_g; i++) {
        const uint32_t gw = gw_at(i);
        const NodeLists L = a.ix.lists[gw & kGatherNode];
        const bool mg = (gw & kGatherSubs) && L.n_merge;
        const uint64_t rk = mg && a.ix.xinfo ? a.ix.xinfo[gw & kGatherNode].rank : 0ull;
        a.desc[g0 + i] = GDesc{rp, L.sub_off, mg ? L.ent_off : sp, mg ? L.ent_mask : L.shr_off, (uint32_t)rk,
                               (uint32_t)(rk >> 32), gw, L.n_direct | (mg ? kDescMerge : 0u)};
        rp += (gw & kGatherSubs) ? L.n_direct + L.n_merge : 0u;
        sp += L.shr_cnt;
      }
    } else {
      atomicOr(a.unsafe, kUnsafeSpans);
    }
  }
}

// list == null: topic t = (global thread) / 16 < n, at off[t] (or at t * g_stride). Else the
// topics list[0, *n_list), group-strided (stride layout; their gathers counted in g_count).
__global__ __launch_bounds__(256) void k_desc_g16(DescArgs a) {
  const uint32_t sub = threadIdx.x & 15;
  const uint32_t gid = (blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  if (a.list) {
    const uint32_t nl = *a.n_list;
    for (uint32_t i = gid; i < nl; i += (gridDim.x * blockDim.x) >> 4) {
      const uint32_t t = a.list[i];
      const uint32_t n_g = min(a.g_count[t].gathers, kGatherCap);
      const uint32_t* gw_src = a.gathers + (uint64_t)t * a.gather_stride;
      desc_grp<16>(a, t, n_g, (uint64_t)t * a.g_stride, 0ull, 0u, sub, [&](uint32_t i) { return gw_src[i]; });
    }
    return;
  }
  const uint32_t t = gid;
  if (t >= a.n) return;  // (group-uniform)
  const TopicOff o0 = a.off[t], o1 = a.off[t + 1];
  const uint32_t n_g = (uint32_t)(o1.g - o0.g);
  const uint32_t* gw_src = a.gather_stride ? a.gathers + (uint64_t)t * a.gather_stride : a.gathers + o0.g;
  desc_grp<16>(a, t, n_g, o0.g, o0.inl, (uint32_t)o0.shr, sub, [&](uint32_t i) { return gw_src[i]; });
}

// k_dedup_insert: thread per topic with 1..kPairMax merge gathers; its signature's slot, whose
// value is the topic that inserted the signature. k_dedup_rep: the representative, verified list against list (a
// signature collision leaves the topic its own representative).
// The insert of topic t's signature k (ok: it is deduped) into the table; called by every active
// lane of the wavefront (the lanes with ok == false take part in the leader choice). One table
// operation per distinct signature in the wavefront: a hot signature (the topics under the same
// busy particles) would otherwise have every topic's CAS on one slot at once. Returns the slot
// (kNone when !ok).
__device__ __forceinline__ uint32_t dedup_insert(unsigned long long* keys, uint32_t* vals, uint64_t mask, uint32_t t,
                                                bool ok, unsigned long long k) {
  const uint32_t lane = threadIdx.x & 63;
  uint32_t leader = lane;
  for (uint64_t rem = __ballot(ok); rem;) {  // uniform over the active lanes: a leader per signature
    const uint32_t l = (uint32_t)__builtin_ctzll(rem);
    const unsigned long long kl = __shfl(k, (int)l, 64);
    const uint64_t same = __ballot(ok && k == kl) & rem;
    if ((same >> lane) & 1) leader = l;
    rem &= ~same;
  }
  uint32_t slot = kNone;
  if (ok && leader == lane) {
    uint64_t i = mix64(k) & mask;
    for (uint64_t probes = 0; probes <= mask; probes++) {
      // most leaders find their signature already in place: a plain load, no atomic on a hot
      // slot; the topic whose CAS fills a slot is the representative of its signature
      unsigned long long prev = __atomic_load_n(keys + i, __ATOMIC_RELAXED);
      if (prev == 0ull) {
        prev = atomicCAS(keys + i, 0ull, k);
        if (prev == 0ull) {
          vals[i] = t;
          slot = (uint32_t)i;
          break;
        }
      }
      if (prev == k) {
        slot = (uint32_t)i;
        break;
      }
      i = (i + 1) & mask;
    }  // slot stays kNone only for a full table (sized 2x the topics: cannot happen)
  }
  slot = __shfl(slot, (int)leader, 64);
  return ok ? slot : kNone;
}

__global__ __launch_bounds__(256) void k_dedup_insert(DedupArgs a) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = t < a.n;
  const uint32_t c = act ? a.mcount[t] : 0u;
  // (sharded: the merge gathers and the other shards' entries must fit k_merge's map)
  const bool ok = c != 0 && c <= kPairMax && (!a.fcount || c + a.fcount[t] < kMapSlots);
  const unsigned long long k = ok ? a.msig[t] : 0ull;
  const uint32_t slot = dedup_insert(a.keys, a.vals, a.table_mask, t, ok, k);
  if (act) a.tslot[t] = slot;
}

// k_dedup_rep also lists the topics that resolve a merge set (rep_list, n_sets of them): the
// merge's set pass walks that list instead of every topic.
__global__ __launch_bounds__(1024) void k_dedup_rep(DedupArgs a) {
  __shared__ uint32_t wcnt[3][16];
  __shared__ unsigned long long bbase[2];
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, lane = threadIdx.x & 63, wv = wave_id();
  const bool act = t < a.n;
  const uint32_t sl = act ? a.tslot[t] : kNone;
  uint32_t r = t;
  if (sl != kNone) {
    const uint32_t v = a.vals[sl];
    if (v != t) {
      const uint32_t c = a.mcount[t];
      bool eq = a.mcount[v] == c;
      // the lists, four nodes per load (rows of kPairMax u32 are 16-byte aligned; entries past c
      // are not compared)
      const uint4* x = reinterpret_cast<const uint4*>(a.mlist + (uint64_t)t * kPairMax);
      const uint4* y = reinterpret_cast<const uint4*>(a.mlist + (uint64_t)v * kPairMax);
      for (uint32_t j = 0; eq && j < c; j += 4) {
        const uint4 p = x[j >> 2], q = y[j >> 2];
        eq = p.x == q.x && (j + 1 >= c || p.y == q.y) && (j + 2 >= c || p.z == q.z) && (j + 3 >= c || p.w == q.w);
      }
      // sharded: the same cross-shard entries of every other shard, in the same order
      for (uint32_t f = 0; eq && f < a.n_xf; f++) {
        const XSrc src = a.xsrc[f];
        const uint64_t t0 = src.xoff[t].g, t1 = src.xoff[t + 1].g, v0 = src.xoff[v].g;
        eq = src.xoff[v + 1].g - v0 == t1 - t0;
        for (uint64_t k = 0; eq && k < t1 - t0; k++) {
          const XEnt p = src.xent[t0 + k], q = src.xent[v0 + k];
          eq = p.fid == q.fid && p.rank == q.rank;
        }
      }
      if (eq) r = v;
    }
  }
  if (act) a.rep[t] = r;
  const bool own = r == t && sl != kNone;
  const bool heavy = own && (a.tc ? a.tc[t].merge : (uint32_t)(a.off[t + 1].merge - a.off[t].merge)) >= a.heavy;
  // the batch's gathers (the walk-fused desc has no scan to total them)
  const uint32_t gsum = a.tc ? wave_sum(act ? a.tc[t].gathers : 0u) : 0u;
  const uint64_t bh = __ballot(heavy), bl = __ballot(own && !heavy);
  // one atomic per workgroup and list end on the counters (one per wavefront serialised ~16k
  // atomics on one address per 1M topics)
  if (lane == 0) {
    wcnt[0][wv] = (uint32_t)__popcll(bh);
    wcnt[1][wv] = (uint32_t)__popcll(bl);
    wcnt[2][wv] = gsum;
  }
  __syncthreads();
  if (a.tc && threadIdx.x == 64) {
    unsigned long long g = 0;
    for (uint32_t w = 0; w < blockDim.x / 64; w++) g += wcnt[2][w];
    if (g) atomicAdd(a.n_sets + 2, g);
  }
  if (threadIdx.x < 2) {
    const uint32_t e = threadIdx.x;
    uint32_t tot = 0;
    for (uint32_t w = 0; w < blockDim.x / 64; w++) {
      const uint32_t c = wcnt[e][w];
      wcnt[e][w] = tot;
      tot += c;
    }
    bbase[e] = tot ? atomicAdd(a.n_sets + e, (unsigned long long)tot) : 0ull;
  }
  __syncthreads();
  if (heavy) a.rep_list[bbase[0] + wcnt[0][wv] + prefix_before(bh)] = t;
  else if (own) a.rep_list[a.n - 1 - (bbase[1] + wcnt[1][wv] + prefix_before(bl))] = t;
}

__global__ __launch_bounds__(256) void k_finish(FinishArgs a) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, lane = threadIdx.x & 63;
  bool wave = false;
  if (t < a.n) {
    TopicOff o0, o1;
    if (a.g_stride) {  // the stride layout of the walk-fused desc (a.tc holds the counts)
      o0 = TopicOff{(uint64_t)t * a.g_stride, 0, 0, 0, 0};
      o1 = o0;
      o1.g += a.tc[t].gathers;
    } else {
      o0 = a.off[t];
      o1 = a.off[t + 1];
    }
    const TopicCount c = a.tc ? a.tc[t]
                              : TopicCount{(uint32_t)(o1.g - o0.g), (uint32_t)(o1.rows - o0.rows),
                                           (uint32_t)(o1.shr - o0.shr), (uint32_t)(o1.inl - o0.inl),
                                           (uint32_t)(o1.merge - o0.merge)};
    const uint32_t sl = a.tslot[t];
    const bool set = sl != kNone;
    wave = c.inlines != 0 || (c.merge != 0 && !set);
    if (!wave) {
      TopicSpansDev res;
      res.span_base = o0.g;
      res.patch_base = 0;
      res.inline_base = o0.inl;
      res.picked_base = o0.shr;
      res.n_spans = (uint32_t)(o1.g - o0.g);
      res.n_patches = 0;
      res.n_inline = 0;
      res.n_rows = c.rows;
      res.n_client = c.rows;
      res.n_ident = 0;
      res.n_shared = c.shared;
      res.flags = 0;
      if (set) {  // the representative's resolution (k_merge's set pass), by reference
        const SetInfo si = a.sets[a.rep[t]];
        res.patch_base = si.base;
        res.n_patches = si.n;
        res.n_client = c.rows - si.nonbase;
        res.n_ident = si.ext;
        res.flags = kTopicSetPatches;
      }
      a.sres[t] = res;
    }
  }
  const uint64_t b = __ballot(wave);
  unsigned long long base = 0;
  if (lane == 0 && b) base = atomicAdd(a.n_wave, (unsigned long long)__popcll(b));
  base = __shfl(base, 0, 64);
  if (wave) a.wave_list[base + prefix_before(b)] = t;
}

// Host span results (mq_match_spans): the merge rows of every topic that references its set's
// patches, packed (topics in any order; one atomic per wavefront). base[t]: where topic t's
// start (0 for a topic without a set); *total: the packed count. The wavefront copies its
// topics' rows one topic at a time, a lane per row (coalesced).
__global__ __launch_bounds__(256) void k_mrow_pack(uint32_t n, const uint32_t* __restrict__ tslot,
                                                   const uint32_t* __restrict__ mcount,
                                                   const uint32_t* __restrict__ mrow, uint32_t* __restrict__ base,
                                                   uint32_t* __restrict__ rows, unsigned long long* total) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, lane = threadIdx.x & 63, t0 = t - lane;
  const uint32_t c = t < n && tslot[t] != kNone ? mcount[t] : 0u;
  uint32_t sum;
  const uint32_t pre = wave_excl_scan(c, lane, &sum);
  unsigned long long b = 0;
  if (lane == 0 && sum) b = atomicAdd(total, (unsigned long long)sum);
  b = __shfl(b, 0, 64) + pre;
  if (t < n) base[t] = c ? (uint32_t)b : 0u;
  for (uint64_t m = __ballot(c != 0); m; m &= m - 1) {
    const int j = __builtin_ctzll(m);
    const uint32_t cj = __shfl(c, j, 64);
    const unsigned long long bj = __shfl(b, j, 64);
    if (lane < cj) rows[bj + lane] = mrow[(uint64_t)(t0 + j) * kPairMax + lane];
  }
}

// Host span results: the written patches of every merge set packed (the set pool holds each
// set's reservation, of which SetInfo.n are written); nbase[rep]: where the set's start.
// One atomic per wavefront; the wavefront copies its sets one at a time (coalesced).
__global__ __launch_bounds__(256) void k_set_pack(uint32_t n, const uint32_t* __restrict__ tslot,
                                                  const uint32_t* __restrict__ rep, const SetInfo* __restrict__ sets,
                                                  const PatchRec* __restrict__ pool, uint64_t* __restrict__ nbase,
                                                  PatchRec* __restrict__ out, unsigned long long* total) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, lane = threadIdx.x & 63;
  const bool own = t < n && tslot[t] != kNone && rep[t] == t;  // a set's representative
  SetInfo si{0, 0, 0, 0, 0};
  if (own) si = sets[t];
  const uint32_t c = own ? si.n : 0u;
  uint32_t sum;
  const uint32_t pre = wave_excl_scan(c, lane, &sum);
  unsigned long long b = 0;
  if (lane == 0 && sum) b = atomicAdd(total, (unsigned long long)sum);
  b = __shfl(b, 0, 64) + pre;
  if (own) nbase[t] = b;
  for (uint64_t m = __ballot(c != 0); m; m &= m - 1) {
    const int j = __builtin_ctzll(m);
    const uint32_t cj = __shfl(c, j, 64);
    const unsigned long long bj = __shfl(b, j, 64), sj = __shfl((unsigned long long)si.base, j, 64);
    for (uint32_t k = lane; k < cj; k += 64) out[bj + k] = pool[sj + k];
  }
}

// Host span results: every topic's patch_base into the packed arrays — its set's patches
// (nbase of its representative) or its own (the regions' packed offsets roff), 0 without patches.
__global__ __launch_bounds__(256) void k_host_rebase(uint32_t n, const uint32_t* __restrict__ rep,
                                                     const uint64_t* __restrict__ nbase,
                                                     const uint64_t* __restrict__ roff, uint64_t rcap,
                                                     TopicSpansDev* sres) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint32_t np = sres[t].n_patches, fl = sres[t].flags;
  const uint64_t pb = sres[t].patch_base;
  uint64_t b = 0;
  if (np && (fl & kTopicSetPatches)) b = nbase[rep[t]];
  else if (np) b = roff[pb / rcap] + pb % rcap;
  sres[t].patch_base = b;
}

void launch_mrow_pack(uint32_t n, const uint32_t* tslot, const uint32_t* mcount, const uint32_t* mrow,
                      uint32_t* base, uint32_t* rows, unsigned long long* total, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_mrow_pack, dim3((n + 255) / 256), dim3(256), 0, s, n, tslot, mcount, mrow, base, rows, total);
}

void launch_set_pack(uint32_t n, const uint32_t* tslot, const uint32_t* rep, const SetInfo* sets,
                     const PatchRec* pool, uint64_t* nbase, PatchRec* out, unsigned long long* total, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_set_pack, dim3((n + 255) / 256), dim3(256), 0, s, n, tslot, rep, sets, pool, nbase, out, total);
}

void launch_host_rebase(uint32_t n, const uint32_t* rep, const uint64_t* nbase, const uint64_t* roff, uint64_t rcap,
                        TopicSpansDev* sres, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_host_rebase, dim3((n + 255) / 256), dim3(256), 0, s, n, rep, nbase, roff, rcap, sres);
}

__global__ __launch_bounds__(256) void k_xsig(XSigArgs a) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= a.n) return;
  uint64_t sig = 0;
  uint32_t fc = 0;
  for (uint32_t f = 0; f < a.n_xf; f++) {
    const XSrc src = a.xsrc[f];
    const uint64_t x0 = src.xoff[t].g, x1 = src.xoff[t + 1].g;
    for (uint64_t k = x0; k < x1; k++) {
      const XEnt e = src.xent[k];
      sig = mix64(sig ^ ((uint64_t)f << 56 | (uint64_t)fc << 32 | e.fid)) + e.rank;
      fc++;
    }
  }
  a.fcount[t] = fc;
  const uint32_t mc = a.mcount[t];
  if (!fc || !mc) return;
  a.msig[t] = mix64(a.msig[t] ^ sig) | 1ull;
  if (mc <= kPairMax && mc + fc >= kMapSlots) {  // k_merge's slow path reads GDesc records
    const TopicOff o0 = a.off[t], o1 = a.off[t + 1];
    const uint32_t* gw_src = a.gather_stride ? a.gathers + (uint64_t)t * a.gather_stride : a.gathers + o0.g;
    write_gdesc(a.ix, gw_src, (uint32_t)(o1.g - o0.g), (uint32_t)o0.shr, a.desc + o0.g);
  }
}

void launch_xsig(const XSigArgs& a, hipStream_t s) {
  if (!a.n) return;
  hipLaunchKernelGGL(k_xsig, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
}

void launch_finish(const FinishArgs& a, hipStream_t s) {
  if (!a.n) return;
  hipLaunchKernelGGL(k_finish, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
}

void launch_dedup(const DedupArgs& a, hipStream_t s, bool insert) {
  if (!a.n) return;
  const dim3 g((a.n + 255) / 256), b(256);
  if (insert) hipLaunchKernelGGL(k_dedup_insert, g, b, 0, s, a);
  hipLaunchKernelGGL(k_dedup_rep, dim3((a.n + 1023) / 1024), dim3(1024), 0, s, a);
}

// Stream S of one tile: rows [x0, x1) of the chunk's stream S (0: client rows, 1: shared rows,
// 2: inline rows), starting at gather j. The gathers' (position, source) pairs are read as a
// register window of 64 consecutive GDesc records (one coalesced load: lane k holds gather
// wb + k) plus the start of gather wb + 64. Each lane keeps its own gather cursor and reads the
// window with ds_bpermute in wave-uniform loops (every lane executes every bpermute), so the
// inner loop issues no dependent global loads. The window slides to lane 0's gather (the lowest
// row) when a lane's row lies past it; rows past a window that cannot slide (more than 64
// gathers, empty ones included, between lane 0 and the lane) are found by a global scan.
template <int S, class V>
__device__ __forceinline__ void copy_tile(const EmitArgs& a, const V* __restrict__ src, V* __restrict__ dst,
                                          uint32_t x0, uint32_t x1, uint32_t j, uint32_t lane) {
  constexpr int U = 8;
  constexpr uint32_t kInf = 0xFFFFFFFFu;
  const uint32_t jend = (uint32_t)a.off[a.t1].g;
  auto pos_of = [&](uint32_t g) -> uint32_t {
    return S == 0 ? a.desc[g].r_pos : (S == 1 ? a.desc[g].s_pos : a.desc[g].i_pos);
  };
  auto src_of = [&](uint32_t g) -> uint32_t {
    return S == 0 ? a.desc[g].r_src : (S == 1 ? a.desc[g].s_src : a.desc[g].i_src);
  };
  uint32_t wb = j, wpos = kInf, wsrc = 0, wsent = kInf;
  auto load_window = [&]() {
    const uint32_t g = wb + lane;
    wpos = g < jend ? pos_of(g) : kInf;
    wsrc = g < jend ? src_of(g) : 0u;
    wsent = wb + 64 < jend ? pos_of(wb + 64) : kInf;
  };
  // start of gather ga + 1 for an in-window ga (kInf when ga is past the window: unknown)
  auto next_of = [&](uint32_t ga) -> uint32_t {
    const uint32_t k = ga - wb;
    const uint32_t v = __shfl(wpos, (int)min(k + 1, 63u), 64);
    return k < 63 ? v : (k == 63 ? wsent : kInf);
  };
  load_window();
  uint32_t ga = j;  // this lane's gather (absolute index)
  uint32_t nxt = next_of(ga);
  uint32_t sb = __shfl(wsrc, 0, 64) - __shfl(wpos, 0, 64);  // source index = sb + row
  for (uint32_t r0 = x0; r0 < x1; r0 += 64 * U) {
    uint32_t si[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t x = min(r0 + u * 64 + lane, x1 - 1);
      bool moved = false, slow = false;
      uint32_t sb_slow = 0;
      for (;;) {
        const bool adv = ga - wb < 64 && x >= nxt;
        if (__any(adv)) {
          if (adv) {
            ga++;
            moved = true;
          }
          nxt = next_of(ga);
          continue;
        }
        const bool out = ga - wb >= 64 || (ga - wb == 63 && x >= wsent);
        if (!__any(out)) break;
        const uint32_t nb = __shfl(ga, 0, 64);  // lane 0 holds the lowest row
        if (nb != wb) {
          wb = nb;
          load_window();
          nxt = next_of(ga);
          moved = true;
          continue;
        }
        if (out) {  // the window cannot reach this lane's row: scan the records
          uint32_t n2 = ga + 1 < jend ? pos_of(ga + 1) : kInf;
          while (x >= n2) {
            ga++;
            n2 = ga + 1 < jend ? pos_of(ga + 1) : kInf;
          }
          sb_slow = src_of(ga) - pos_of(ga);
          slow = true;
          nxt = kInf;
        }
        break;
      }
      if (__any(moved || slow)) {  // usually no lane changed gather: keep sb without bpermutes
        const uint32_t k = min(ga - wb, 63u);
        const uint32_t sp = __shfl(wpos, (int)k, 64), ss = __shfl(wsrc, (int)k, 64);
        if (slow) sb = sb_slow;
        else if (moved) sb = ss - sp;
      }
      si[u] = sb + x;
    }
    V v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = src[si[u]];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t x = r0 + u * 64 + lane;
      if (x < x1) __builtin_nontemporal_store(v[u], dst + x);
    }
  }
}

// Persistent: a.copy_waves wavefronts stride over the chunk's tiles, so the copy holds only the
// wave slots it needs to keep HBM busy and k_merge (side stream) gets the rest of every CU.
__global__ __launch_bounds__(256) void k_copy(EmitArgs a) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t n_all = a.n_tiles[0] + a.n_tiles[1] + a.n_tiles[2];
  for (uint32_t w0 = blockIdx.x * 4 + wave_id(); w0 < n_all; w0 += gridDim.x * 4) {
    uint32_t w = w0;
    const uint32_t j = a.tiles[w];
    if (w < a.n_tiles[0]) {
      const uint32_t x0 = w * kCopyTile, x1 = min(x0 + kCopyTile, a.total[0]);
      copy_tile<0>(a, reinterpret_cast<const u32x4*>(a.ix.subs), reinterpret_cast<u32x4*>(a.rows), x0, x1, j, lane);
      continue;
    }
    w -= a.n_tiles[0];
    if (w < a.n_tiles[1]) {
      const uint32_t x0 = w * kCopyTile, x1 = min(x0 + kCopyTile, a.total[1]);
      copy_tile<1>(a, reinterpret_cast<const u32x2*>(a.ix.shr), reinterpret_cast<u32x2*>(a.shr_rows), x0, x1, j, lane);
      continue;
    }
    w -= a.n_tiles[1];
    const uint32_t x0 = w * kCopyTile, x1 = min(x0 + kCopyTile, a.total[2]);
    copy_tile<2>(a, reinterpret_cast<const u32x2*>(a.ix.inl), reinterpret_cast<u32x2*>(a.inl_rows), x0, x1, j, lane);
  }
}

// Rank key of a span-format merge gather of a sharded index (k_desc<true>; else 0).
template <bool XS>
__device__ __forceinline__ uint64_t gdesc_rank(const GDesc& d) {
  return XS ? ((uint64_t)d.i_src << 32 | d.i_pos) : 0ull;
}

// SPANS=false: the records were copied to the chunk's rows by k_copy and are rewritten in
// place. SPANS=true: nothing was copied; each record whose row changes leaves a PatchRec (its
// topic-relative row, the new meta) in a range the topic reserves with one atomicAdd on its
// region's counter (a.pcount[t % kPatchRegions]: one shared counter serialised a million
// same-address atomics per batch), sized by the records its hit lists hold (the reservation is
// made before any record is resolved: when the hit lists do not fit in LDS the pair analysis
// runs twice, counting, then resolving). A reservation past the region's a.rcap writes
// nothing; the host reads the counters, grows the pool and runs the batch's k_merge again.
// WPE: minimum waves per SIMD asked of the register allocator (1 = no constraint; the kernel is
// latency-bound, so occupancy can pay for a few spills). MQ_OPT_MERGE_WAVES picks the variant.
// XS (span format of a sharded index): the other shards' exported nodes join the topic's map
// and DFS order compares rank keys first (SPANS must be true).
// SET (span format, merge-set dedup): the set pass (a.dd_phase 1), compiled apart so that the
// topic pass's copy, inline and result code does not weigh on its register allocation.
template <bool SPANS, bool XS, int WPE, bool SET = false, uint32_t PB = kPartBatch>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_merge(EmitArgs a) {
  constexpr uint32_t kEnt = XS ? kMapSlots : kPairMax;  // map entries
  __shared__ uint32_t map_key[4][kMapSlots];   // gathered node with may-merge records (or
                                               //   kForeign | fid: another shard's, XS)
  __shared__ uint32_t map_val[4][kMapSlots];   // its entry below
  __shared__ uint32_t mg_node[4][kEnt];        // entries: the topic's merge gathers in gather
  __shared__ uint32_t mg_gi[4][kEnt];          //   order (node, gather index), then (XS) the
  __shared__ uint64_t mg_rank[4][XS ? kEnt : 1];  // other shards' (kForeign | fid, kNone, rank)
  __shared__ uint32_t mg_row[4][kPairMax];     //   output row of its first record (pair slots name
                                               //   a record by its place k in the particle's list),
  __shared__ uint32_t mg_eoff[4][kPairMax];    //   its pair-block hash table (NodePair)
  __shared__ uint32_t mg_emask[4][kPairMax];
  __shared__ uint32_t h_ga[4][kHitMax];        // staged hit lists: merge gather of g,
  __shared__ uint32_t h_off[4][kHitMax];       //   pair-list offset,
  __shared__ uint32_t h_via[4][kHitMax];       //   partner node h,
  __shared__ uint32_t h_pre[4][kHitMax + 1];   //   exclusive prefix of their lengths (+ total)
  const uint32_t wv = wave_id(), lane = threadIdx.x & 63;
  auto rank_of = [](const GDesc& d) { return gdesc_rank<XS>(d); };
  // persistent: a.merge grid's waves stride over the chunk's topics (wave-uniform loop)
  // (dedup's set pass: the waves stride over the list of set representatives instead; its topic
  // pass after k_finish: over the topics k_finish left)
  const uint32_t* __restrict__ tlist = !(SPANS && a.rep) ? nullptr
                                     : SET ? a.rep_list : a.wave_list;
  const uint32_t n_front = SET && tlist ? (uint32_t)a.n_reps[0] : 0u;  // heavy sets, then the back
  const uint32_t i_end = tlist ? (SET ? n_front + (uint32_t)a.n_reps[1] : (uint32_t)*a.n_wave) : a.t1;
  for (uint32_t i = a.t0 + blockIdx.x * 4 + wv; i < i_end; i += gridDim.x * 4) {
  const uint32_t t = !tlist ? i : (SET && i >= n_front) ? tlist[a.t1 - 1 - (i - n_front)] : tlist[i];
  TopicOff o0, o1;
  if (SPANS && a.g_stride) {  // the stride layout of the walk-fused desc: no offsets
    o0 = TopicOff{(uint64_t)t * a.g_stride, 0, 0, 0, 0};
    o1 = o0;
    o1.g += a.tc[t].gathers;
  } else {
    o0 = a.off[t];
    o1 = a.off[t + 1];
  }
  const uint64_t rb = o0.rows - a.base.rows;
  const uint64_t ib = o0.inl - a.base.inl;
  const uint32_t n_g = (uint32_t)(o1.g - o0.g);
  // per-topic counts: the offsets' differences, or k_desc's counts (walk without lists)
  TopicCount tcn{n_g, (uint32_t)(o1.rows - o0.rows), (uint32_t)(o1.shr - o0.shr), (uint32_t)(o1.inl - o0.inl),
                 (uint32_t)(o1.merge - o0.merge)};
  if (SPANS && a.tc) tcn = a.tc[t];
  const GDesc* __restrict__ gd = a.desc + o0.g;
  SubRec* __restrict__ crow = a.rows;  // chunk-relative rows (GDesc positions), row format
  // merge-set dedup (wave-uniform): a representative resolves in phase 1, a deduped topic copies
  // in phase 2, a topic that is not deduped resolves itself in phase 2
  const uint32_t dslot = (SPANS && a.rep) ? a.tslot[t] : kNone;
  const uint32_t drep = dslot != kNone ? a.rep[t] : t;
  if (SET && (dslot == kNone || drep != t)) continue;
  const bool setrel = SET;
  // MQ_PROF_WORK: the set pass's phases in shader clocks (map, pair analysis, resolution)
  const bool stamp = SET && a.work != nullptr;
  uint64_t c_start = stamp ? clock64() : 0ull, c_map = c_start, c_pairs = c_start;
  const bool dcopy = !SET && SPANS && a.rep && dslot != kNone;
  PatchRec* __restrict__ ppool = setrel ? a.spatches : a.patches;
  unsigned long long* __restrict__ pcnt = setrel ? a.spcount : a.pcount;
  const uint64_t prcap = setrel ? a.srcap : a.rcap;
  uint32_t n_nonbase = 0, n_ext = 0;
  uint64_t pbase = 0;    // span format: the topic's patch range [pbase, pbase + reserved)
  uint32_t n_patch = 0;
  bool pfit = true;      // the reservation fits the pool
  uint32_t w_ent = 0, w_rec = 0, w_link = 0;  // this lane's work (MQ_PROF_WORK)
  uint32_t w_map = 0;  // bytes of the map's sources read (merge lists or GDesc records; wave-uniform)

  // reserve n patch slots for this topic in its region (wave-uniform). The atomic's answer is
  // taken only when the first patch is written (settle): by then the pair-slot loads issued
  // after it have returned, so the reservation costs no round trip of its own.
  unsigned long long resv = 0;  // lane 0: the region's counter before this topic's reservation
  uint64_t resv_n = 0;
  bool resv_pending = false;
  auto reserve = [&](uint64_t n) __attribute__((always_inline)) {
    if (lane == 0 && n) resv = atomicAdd(pcnt + (t & (kPatchRegions - 1)), (unsigned long long)n);
    resv_n = n;
    resv_pending = true;
  };
  auto settle = [&]() __attribute__((always_inline)) {
    if (resv_pending) {
      const unsigned long long b = __shfl(resv, 0, 64);
      pfit = b + resv_n <= prcap;
      if (!pfit && a.unsafe && lane == 0) atomicOr(a.unsafe, kUnsafePatches);
      pbase = (uint64_t)(t & (kPatchRegions - 1)) * prcap + b;
      resv_pending = false;
    }
  };
  // one patch per lane that wants one, compacted by ballot (wave-uniform)
  auto emit_patch = [&](bool want, uint32_t row, uint32_t meta) __attribute__((always_inline)) {
    settle();
    const uint64_t m = __ballot(want);
    if (want && pfit) ppool[pbase + n_patch + prefix_before(m)] = PatchRec{row, meta};
    n_patch += (uint32_t)__popcll(m);
  };

  uint32_t n_map = 0;
  const uint32_t cap = tcn.rows;

  uint32_t res_flags = 0;
  if (dcopy && a.set_ref) {
    // device result: the topic names its representative's set-relative patches (translated by the
    // consumer through the topic's merge rows, MQ_TOPIC_SET_PATCHES)
    const SetInfo si = a.sets[drep];
    pbase = si.base;
    n_patch = si.n;
    n_nonbase = si.nonbase;
    n_ext = si.ext;
    res_flags = kTopicSetPatches;
  } else if (dcopy) {
    // the representative's resolution: its set-relative patches, rows translated through this
    // topic's merge gathers (the same particles in the same order: k_dedup compared them)
    const SetInfo si = a.sets[drep];
    const uint32_t mc = a.mcount[t];
    const uint32_t my_row = lane < mc ? a.mrow[(uint64_t)t * kPairMax + lane] : 0u;
    reserve(si.n);
    for (uint32_t j0 = 0; j0 < si.n; j0 += 64) {
      const uint32_t j = j0 + lane;
      const bool want = j < si.n;
      PatchRec pr{0, 0};
      if (want) pr = a.spatches[si.base + j];
      const uint32_t base_row = __shfl(my_row, (int)(pr.row >> kSetRowBits), 64);
      emit_patch(want, base_row + (pr.row & ((1u << kSetRowBits) - 1)), pr.meta);
    }
    n_nonbase = si.nonbase;
    n_ext = si.ext;
  } else if (tcn.merge) {  // the topic gathers may-merge records
    // Map every gathered node that holds may-merge records (and whose subscriptions are
    // gathered, Q3) to its gather index, and list them in gather order. Nodes are distinct
    // within a topic.
    // merge-set dedup's lists (k_desc): the topic's merge gathers directly, x standing for the
    // gather index (the same order); a topic with more than kPairMax of them has GDesc records
    const uint32_t lc = (SPANS && a.mlist) ? a.mcount[t] : kNone;
    if (lc <= kPairMax) {
      for (uint32_t q = lane; q < kMapSlots; q += 64) map_key[wv][q] = kNone;
      wave_sync_lds();
      if (lane < lc) {
        const uint64_t k = (uint64_t)t * kPairMax + lane;
        const uint32_t node = a.mlist[k];
        const uint2 P = a.mpair[k];
        uint32_t sl = hash32(node) & (kMapSlots - 1);
        while (atomicCAS(&map_key[wv][sl], kNone, node) != kNone) sl = (sl + 1) & (kMapSlots - 1);
        map_val[wv][sl] = lane;
        mg_node[wv][lane] = node;
        mg_gi[wv][lane] = lane;
        if (XS) mg_rank[wv][lane] = a.mrank[k];
        mg_row[wv][lane] = a.mrow[k];
        mg_eoff[wv][lane] = P.x;
        mg_emask[wv][lane] = P.y;
      }
      n_map = lc;
      w_map = (XS ? 24u : 16u) * lc;
    } else {
    if (a.unsafe && o1.g > a.desc_cap) {  // one-sync batch: no GDesc records to read
      if (lane == 0) atomicOr(a.unsafe, kUnsafeDesc);
      continue;
    }
    for (uint32_t q = lane; q < kMapSlots; q += 64) map_key[wv][q] = kNone;
    wave_sync_lds();
    w_map = (uint32_t)sizeof(GDesc) * n_g;
    for (uint32_t i0 = 0; i0 < n_g; i0 += 64) {
      const uint32_t i = i0 + lane;
      bool ins = false;
      uint32_t node = 0, mrow = 0;
      NodePair P{0, kNone, 0, 0};
      if (i < n_g) {
        const GDesc d = gd[i];
        node = d.word & kGatherNode;
        ins = (d.mdir & kDescMerge) != 0;
        mrow = d.r_pos;  // (pair slots name records by their place in the particle's list)
        if (ins) {
          if (SPANS) P = NodePair{d.s_pos, d.s_src, 0, 0};  // folded in by k_desc<true>
          else P = a.ix.npair[node];
        }
      }
      const uint64_t bi = __ballot(ins);
      const uint32_t x = n_map + prefix_before(bi);
      if (ins && x < kPairMax) {
        uint32_t sl = hash32(node) & (kMapSlots - 1);
        while (atomicCAS(&map_key[wv][sl], kNone, node) != kNone) sl = (sl + 1) & (kMapSlots - 1);
        map_val[wv][sl] = x;
        mg_node[wv][x] = node;
        mg_gi[wv][x] = i;
        if (XS) mg_rank[wv][x] = rank_of(gd[i]);
        mg_row[wv][x] = mrow;
        mg_eoff[wv][x] = P.ent_off;
        mg_emask[wv][x] = P.ent_mask;
      }
      n_map += __popcll(bi);
    }
    }
    // sharded index: the other shards' gathered cross-shard nodes join the map as entries
    // n_map.. (their partner links name them kForeign | fid; their rank keys order them)
    uint32_t n_ent = n_map;
    for (uint32_t f = 0; XS && f < a.n_xf; f++) {
      const XSrc src = a.xsrc[f];
      const uint64_t x0 = src.xoff[t].g, x1 = src.xoff[t + 1].g;
      for (uint64_t k0 = x0; k0 < x1; k0 += 64) {
        const uint64_t k = k0 + lane;
        const uint32_t x = n_ent + (uint32_t)(k - x0);
        if (k < x1 && x < kEnt && n_map <= kPairMax) {
          const XEnt e = src.xent[k];
          const uint32_t key = kForeign | e.fid;
          uint32_t sl = hash32(key) & (kMapSlots - 1);
          while (atomicCAS(&map_key[wv][sl], kNone, key) != kNone) sl = (sl + 1) & (kMapSlots - 1);
          map_val[wv][sl] = x;
          mg_node[wv][x] = key;
          mg_gi[wv][x] = kNone;
          if (XS) mg_rank[wv][x] = e.rank;
        }
      }
      n_ent += (uint32_t)(x1 - x0);
    }
    wave_sync_lds();
    if (stamp) c_map = clock64();
    // beyond the map: linear lookups (the map's hash table keeps a free slot: kMapSlots - 1
    // entries at most, so a lookup of a node that is not there ends)
    const bool slow = n_map > kPairMax || n_ent > (XS ? kEnt - 1 : kEnt);
    if (slow && a.unsafe && o1.g > a.desc_cap) {  // one-sync batch: no GDesc records to read
      if (lane == 0) atomicOr(a.unsafe, kUnsafeDesc);
      continue;
    }
    // Is node h (or kForeign | fid) gathered for this topic? Its DFS position: rank key, then
    // gather index (kNone for another shard's node); found = false otherwise.
    struct Pos {
      uint64_t rk;
      uint32_t gi;
      bool found;
    };
    auto gathered = [&](uint32_t h) __attribute__((always_inline)) -> Pos {
      if (!slow) {
        uint32_t sl = hash32(h) & (kMapSlots - 1);
        for (;;) {
          const uint32_t k = map_key[wv][sl];
          if (k == h) {
            const uint32_t y = map_val[wv][sl];
            return Pos{XS ? mg_rank[wv][y] : 0ull, mg_gi[wv][y], true};
          }
          if (k == kNone) return Pos{0, kNone, false};
          sl = (sl + 1) & (kMapSlots - 1);
        }
      }
      if (XS && (h & kForeign)) {
        for (uint32_t f = 0; f < a.n_xf; f++) {
          const XSrc src = a.xsrc[f];
          for (uint64_t k = src.xoff[t].g; k < src.xoff[t + 1].g; k++)
            if ((kForeign | src.xent[k].fid) == h) return Pos{src.xent[k].rank, kNone, true};
        }
        return Pos{0, kNone, false};
      }
      for (uint32_t i = 0; i < n_g; i++) {
        const GDesc d = gd[i];
        if ((d.word & kGatherNode) == h && (d.word & kGatherSubs)) return Pos{rank_of(d), i, true};
      }
      return Pos{0, kNone, false};
    };
    // does the gathered node at (rh, gh) come before the record's own (rg, gg) in DFS order?
    auto before = [&](uint64_t rh, uint32_t gh, uint64_t rg, uint32_t gg) __attribute__((always_inline)) -> bool {
      if (!XS) return gh < gg;
      if (rh != rg) return rh < rg;
      if (gh != kNone) return gh < gg;  // both on this shard: gather order is DFS order
      atomicOr(a.ix.err, kErrDeepRank);  // another shard's node tied beyond the key's 32 levels
      return false;
    };

    // Resolve one record whose client may have other matches for this topic: its partners that
    // are gathered decide it (layout.h, MergePart). An earlier one makes it a non-base entry:
    // an Identifiers row when its identifier is > 0 (Subscription.Merge,
    // packets/packets.go:261-263), else dropped. Otherwise it is the base and takes the
    // partners' max Qos and OR'd NoLocal (packets/packets.go:265-271). A record may be reached
    // through several hit lists; only the visit through its first gathered partner (`via`, or
    // any when via == kNone) counts it, and only that visit leaves a patch (the row format
    // writes the same row on every visit). Called by all lanes (wave-uniform).
    // mw: the record's meta | kSlotIdentPos when its identifier is > 0 (PairSlot.meta); (rg, gi):
    // its gather's rank key and gather index.
    auto resolve = [&](bool active, uint32_t mw, uint32_t row, uint64_t rg, uint32_t gi, uint32_t via,
                       uint32_t mp_off, uint32_t mp_cnt) __attribute__((always_inline)) {
      bool counted = false, nonbase = false, want = false;
      uint32_t pmeta = 0;
      if (active) {
        const uint32_t rmeta = mw & ~kSlotIdentPos;
        const bool idpos = (mw & kSlotIdentPos) != 0;
        bool bound = false, base = true;
        // (span format) a visit through a partner that is not the record's first gathered one
        // counts and emits nothing: it stops at that first one (the row format rewrites the row on
        // every visit, so it reads every link)
        bool other = false;
        uint32_t first = kNone;
        uint32_t q = rmeta & kMetaQos, nl = rmeta & kMetaNoLocal;
        if (SET && (a.exp & 1u)) mp_cnt = 0;
        // partner links in batches of PB independent loads (one latency per batch)
        for (uint32_t e0 = 0; e0 < mp_cnt && base && !other; e0 += PB) {
          MergePart pb[PB];
#pragma unroll
          for (uint32_t u = 0; u < PB; u++)
            pb[u] = e0 + u < mp_cnt ? a.ix.mpart[mp_off + e0 + u] : MergePart{kNone, 0};
          w_link += min(PB, mp_cnt - e0);
#pragma unroll
          for (uint32_t u = 0; u < PB; u++) {
            if (!base || other || pb[u].node == kNone) continue;
            if (SET && (a.exp & 2u)) {
              q = max(q, pb[u].meta & kMetaQos);
              continue;
            }
            const Pos ph = gathered(pb[u].node);
            if (!ph.found) continue;
            if (!bound) {
              first = pb[u].node;
              other = SPANS && via != kNone && first != via && !(SET && (a.exp & 16u));
            }
            bound = true;
            if (before(ph.rk, ph.gi, rg, gi)) {
              base = false;
              continue;
            }
            q = max(q, pb[u].meta & kMetaQos);
            nl |= pb[u].meta & kMetaNoLocal;
          }
        }
        if (bound) {
          counted = via == kNone || via == first;
          nonbase = !base;
          pmeta = base ? (rmeta & ~(kMetaQos | kMetaNoLocal)) | q | nl : rmeta | (idpos ? kRowIdent : kRowDrop);
          if (SPANS) {
            want = counted && pmeta != rmeta;
          } else if (pmeta != rmeta) {
            crow[row].meta = pmeta;
          }
        }
      }
      if (SPANS) emit_patch(want && !(SET && (a.exp & 4u)), row, pmeta);
      const uint64_t bn = __ballot(counted && nonbase);
      const uint64_t bx = __ballot(counted && nonbase && (pmeta & kRowIdent));
      n_nonbase += __popcll(bn);
      n_ext += __popcll(bx);
    };


    if (!slow) {
      // Pair analysis over ordered pairs (g, h) of merge gathers: g's pair block lists the slots
      // whose client also subscribes at h. Hit lists are staged in LDS and their concatenation
      // is resolved 64 records per wave-instruction.
      uint32_t n_hit = 0, tot = 0;
      auto flush_hits = [&]() __attribute__((always_inline)) {
        if (lane == 0) h_pre[wv][n_hit] = tot;
        wave_sync_lds();
        // record r of the staged lists: its list (binary search of the prefix) and its pair slot
        auto locate = [&](uint32_t r, uint32_t& jj) __attribute__((always_inline)) -> PairSlot {
          const uint32_t rc = min(r, tot - 1);
          uint32_t lo = 0, hi = n_hit;  // h_pre[lo] <= rc < h_pre[hi] (lists are non-empty)
          if (SET && (a.exp & 8u)) {  // (a list's first slot: in bounds, not the record's)
            jj = rc % n_hit;
            return a.ix.plist[h_off[wv][jj]];
          }
          while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (h_pre[wv][mid] <= rc) lo = mid; else hi = mid;
          }
          jj = lo;
          return a.ix.plist[h_off[wv][lo] + (rc - h_pre[wv][lo])];
        };
        // software-pipelined by one round: the next 64 records' pair slots are loaded before
        // this round's partner links, so each round waits on one load latency, not two (two
        // rounds, with the next round's first links in flight too, spilled registers and was
        // slower: 1.15 -> 1.36 ms at 8 waves per SIMD, 1.24 ms at 6; profiles/r03/s2_hostsets/)
        uint32_t jj_next = 0;
        PairSlot e_next = locate(lane, jj_next);
        for (uint32_t r0 = 0; r0 < tot; r0 += 64) {
          const uint32_t r = r0 + lane;
          const uint32_t jj = jj_next;
          const PairSlot e = e_next;
          if (r0 + 64 < tot) e_next = locate(r0 + 64 + lane, jj_next);  // wave-uniform
          const uint32_t xa = h_ga[wv][jj];
          w_rec += r < tot;
          resolve(r < tot, e.meta, setrel ? (xa << kSetRowBits | e.k) : mg_row[wv][xa] + e.k,
                  XS ? mg_rank[wv][xa] : 0ull, mg_gi[wv][xa], h_via[wv][jj], e.mp_off, e.mp_cnt);
        }
        n_hit = 0;
        tot = 0;
        wave_sync_lds();
      };
      // counting = true: stage hit lists while they fit and add up every list's length
      // (tot_all); stop staging at the first batch that does not fit (staged_all = false).
      // counting = false: stage and resolve (flush) as the lists come.
      uint64_t tot_all = 0;
      bool staged_all = true;
      auto pairs = [&](bool counting) __attribute__((always_inline)) {
        const uint32_t np = n_map * n_ent;  // (g: a merge gather here, h: any entry)
        for (uint32_t p0 = 0; p0 < np; p0 += 64) {
          const uint32_t p = p0 + lane;
          bool hit = false;
          uint32_t ga = 0, e_off = 0, e_cnt = 0, hn = 0;
          if (p < np) {
            ga = p / n_ent;
            const uint32_t hb = p - ga * n_ent;
            if (ga != hb) {
              const uint32_t ent_mask = mg_emask[wv][ga], ent_off = mg_eoff[wv][ga];
              if (ent_mask != kNone) {
                hn = mg_node[wv][hb];
                // linear probing, four slots per round: one load latency covers most probes
                uint32_t sl = pair_hash(hn) & ent_mask;
                for (uint32_t probes = 0; probes <= ent_mask; probes += 4) {
                  PairEnt pe[4];
#pragma unroll
                  for (uint32_t u = 0; u < 4; u++) pe[u] = a.ix.pent[ent_off + ((sl + u) & ent_mask)];
                  w_ent += 4;
                  bool stop = false;
#pragma unroll
                  for (uint32_t u = 0; u < 4; u++) {
                    if (stop) continue;
                    if (pe[u].h == hn) {
                      hit = true;
                      e_off = pe[u].off;
                      e_cnt = pe[u].cnt;
                      stop = true;
                    } else if (pe[u].h == kNone) {
                      stop = true;
                    }
                  }
                  if (stop) break;
                  sl = (sl + 4) & ent_mask;
                }
              }
            }
          }
          const uint64_t bh = __ballot(hit);
          const uint32_t nh = __popcll(bh);
          uint32_t ct;
          const uint32_t cp = wave_excl_scan(hit ? e_cnt : 0u, lane, &ct);
          if (counting) {
            tot_all += ct;
            if (!staged_all || n_hit + nh > kHitMax) {  // wave-uniform
              staged_all = false;
              continue;
            }
          } else if (n_hit + nh > kHitMax) {
            flush_hits();
          }
          if (hit) {
            const uint32_t x = n_hit + prefix_before(bh);
            h_ga[wv][x] = ga;
            h_off[wv][x] = e_off;
            h_via[wv][x] = hn;
            h_pre[wv][x] = tot + cp;
          }
          n_hit += nh;
          tot += ct;
        }
      };
      if (SPANS) {
        pairs(true);
        if (stamp) c_pairs = clock64();
        reserve(tot_all);
        if (staged_all) {
          if (n_hit) flush_hits();
        } else {  // rare: more hit lists than LDS holds; probe again, resolving as they come
          n_hit = 0;
          tot = 0;
          wave_sync_lds();
          pairs(false);
          if (n_hit) flush_hits();
        }
      } else {
        pairs(false);
        if (n_hit) flush_hits();
      }
    } else {
      // Too many merge gathers for the pair analysis: resolve every may-merge record.
      if (SPANS) reserve(tcn.merge);
      for (uint32_t i = 0; i < n_g; i++) {
        const GDesc d = gd[i];
        if (!(d.word & kGatherSubs)) continue;
        const NodeLists L = a.ix.lists[d.word & kGatherNode];
        for (uint32_t c0 = 0; c0 < L.n_merge; c0 += 64) {
          const bool act = c0 + lane < L.n_merge;
          const uint32_t pos = L.sub_off + L.n_direct + min(c0 + lane, L.n_merge - 1);
          const MergeRef mr = a.ix.mref[pos];
          const SubRec rec = a.ix.subs[pos];
          w_rec += act;
          resolve(act, rec.meta | (rec.ident > 0 ? kSlotIdentPos : 0u), d.r_pos + L.n_direct + c0 + lane, rank_of(d),
                  i, kNone, mr.off, mr.cnt);
        }
      }
    }
  }

  if (setrel) {  // phase 1: the set's resolution; the topic itself is finished in phase 2
    settle();
    if (lane == 0) a.sets[t] = SetInfo{pbase, n_patch, n_nonbase, n_ext, pfit ? 1u : 0u};
    if (a.work) {  // MQ_PROF_WORK (the resolution work happens here, once per set)
      const uint32_t e = wave_sum(w_ent), rr = wave_sum(w_rec), l = wave_sum(w_link);
      if (a.set_rec && lane == 0) a.set_rec[t] = rr;
      unsigned long long* wc = a.work + (uint64_t)(t & (kPatchRegions - 1)) * kWork;
      if (lane == 0 && (e | rr | l)) {
        atomicAdd(wc + 0, (unsigned long long)e);
        atomicAdd(wc + 1, (unsigned long long)rr);
        atomicAdd(wc + 2, (unsigned long long)l);
        atomicAdd(wc + 3, (unsigned long long)n_patch);
      }
      if (lane == 0) {
        atomicAdd(wc + 8, 1ull);
        if (w_map) atomicAdd(wc + 9, (unsigned long long)w_map);
      }
      const uint64_t c_end = clock64();
      if (lane == 0 && c_pairs != c_start) {  // (the map / pair-analysis path)
        atomicAdd(wc + 4, (unsigned long long)(c_map - c_start));
        atomicAdd(wc + 5, (unsigned long long)(c_pairs - c_map));
        atomicAdd(wc + 6, (unsigned long long)(c_end - c_pairs));
        atomicAdd(wc + 7, (unsigned long long)(c_end - c_start));
      }
    }
    continue;
  }
  uint32_t n_inl = tcn.inlines;
  if (n_inl) {  // InlineSubscriptions[id] = last gathered (topics.go:673-675)
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

  if (SPANS && a.work) {  // MQ_PROF_WORK: one set of atomics per topic, spread over the regions
    const uint32_t e = wave_sum(w_ent), rr = wave_sum(w_rec), l = wave_sum(w_link);
    unsigned long long* wc = a.work + (uint64_t)(t & (kPatchRegions - 1)) * kWork;
    if (lane == 0 && (e | rr | l)) {
      atomicAdd(wc + 0, (unsigned long long)e);
      atomicAdd(wc + 1, (unsigned long long)rr);
      atomicAdd(wc + 2, (unsigned long long)l);
      atomicAdd(wc + 3, (unsigned long long)n_patch);
    }
    if (lane == 0) {
      atomicAdd(wc + 8, 1ull);
      if (w_map) atomicAdd(wc + 9, (unsigned long long)w_map);
    }
  }

  if (SPANS) settle();
  if (lane == 0) {
    if (SPANS) {
      TopicSpansDev res;
      res.span_base = o0.g;
      res.patch_base = pbase;
      res.inline_base = ib;
      res.picked_base = o0.shr;
      res.n_spans = n_g;
      res.n_patches = n_patch;
      res.n_inline = n_inl;
      res.n_rows = cap;
      res.n_client = cap - n_nonbase;
      res.n_ident = n_ext;
      res.n_shared = tcn.shared;
      res.flags = res_flags;
      a.sres[t] = res;
    } else {
      mq_topic_result_dev res;
      res.sub_base = rb;
      res.shared_base = o0.shr - a.base.shr;
      res.inline_base = ib;
      res.sub_cap = cap;
      res.n_client = cap - n_nonbase;
      res.n_ident = n_ext;
      res.n_shared = (uint32_t)(o1.shr - o0.shr);
      res.n_inline = n_inl;
      res.reserved = 0;
      a.res[t - a.t0] = res;
    }
  }
  }  // topic loop
}

}  // namespace mq

namespace mq {

void launch_walk(bool fill, bool lists, uint32_t wpe, const uint8_t* tb, const uint64_t* to, uint32_t n,
                 const DevIndex& ix, TopicCount* cnt, const TopicOff* off, uint32_t* gathers, uint32_t* ovf,
                 hipStream_t s, bool clamp) {
  if (!n) return;
  dim3 grid((n + 255) / 256);
#define MQ_WALK(F, L, W) \
  hipLaunchKernelGGL((k_walk<F, L, W>), grid, dim3(256), 0, s, tb, to, n, ix, cnt, off, gathers, ovf, nullptr, nullptr, clamp)
  if (fill) {
    if (lists) MQ_WALK(true, true, 1);
    else MQ_WALK(true, false, 1);
  } else if (wpe >= 8) {
    if (lists) MQ_WALK(false, true, 8);
    else MQ_WALK(false, false, 8);
  } else {
    if (lists) MQ_WALK(false, true, 1);
    else MQ_WALK(false, false, 1);
  }
#undef MQ_WALK
}

void launch_walk_front(uint32_t group, bool lists, uint32_t wpe, const uint8_t* tb, const uint64_t* to, uint32_t n,
                       const DevIndex& ix, TopicCount* cnt, uint32_t* gathers, uint32_t* ovf, uint32_t* fb_list,
                       uint32_t* fb_count, uint32_t fb_blocks, hipStream_t s, bool clamp) {
  if (!n) return;
  const dim3 grid((n + 256 / group - 1) / (256 / group));
  DescArgs nd;
  std::memset(&nd, 0, sizeof(nd));
#define MQ_WALKF(G, L)                                                                                              \
  if (wpe >= 8)                                                                                                  \
    hipLaunchKernelGGL((k_walkf<G, L, 8>), grid, dim3(256), 0, s, tb, to, n, ix, cnt, gathers, fb_list, fb_count, nd); \
  else                                                                                                           \
    hipLaunchKernelGGL((k_walkf<G, L, 1>), grid, dim3(256), 0, s, tb, to, n, ix, cnt, gathers, fb_list, fb_count, nd)
  if (group == 16) {
    if (lists) MQ_WALKF(16, true);
    else MQ_WALKF(16, false);
  } else {  // (narrower groups: more topics per workgroup, so LDS bounds them below 8 waves)
#define MQ_WALKF1(G, L) \
  hipLaunchKernelGGL((k_walkf<G, L, 1>), grid, dim3(256), 0, s, tb, to, n, ix, cnt, gathers, fb_list, fb_count, nd)
    if (group == 8) {
      if (lists) MQ_WALKF1(8, true);
      else MQ_WALKF1(8, false);
    } else {
      if (lists) MQ_WALKF1(4, true);
      else MQ_WALKF1(4, false);
    }
#undef MQ_WALKF1
  }
#undef MQ_WALKF
  // the topics the frontier could not hold: thread per topic, grid-stride over the list
  const dim3 fgrid(std::max<uint32_t>(1, std::min<uint32_t>((n + 255) / 256, fb_blocks)));
  if (lists)
    hipLaunchKernelGGL((k_walk<false, true, 1>), fgrid, dim3(256), 0, s, tb, to, n, ix, cnt, nullptr, gathers, ovf,
                       fb_list, fb_count, clamp);
  else
    hipLaunchKernelGGL((k_walk<false, false, 1>), fgrid, dim3(256), 0, s, tb, to, n, ix, cnt, nullptr, gathers, ovf,
                       fb_list, fb_count, clamp);
}

void launch_walk_desc(uint32_t group, uint32_t wpe, const uint8_t* tb, const uint64_t* to, uint32_t n, const DevIndex& ix,
                      TopicCount* cnt, uint32_t* gathers, uint32_t* ovf, uint32_t* fb_list, uint32_t* fb_count,
                      uint32_t fb_blocks, const DescArgs& da, hipStream_t s) {
  if (!n) return;
  if (group == 8)
    hipLaunchKernelGGL((k_walkf<8, false, 8, true>), dim3((n + 31) / 32), dim3(256), 0, s, tb, to, n, ix, cnt, gathers,
                       fb_list, fb_count, da);
  else if (wpe >= 8)
    hipLaunchKernelGGL((k_walkf<16, false, 8, true>), dim3((n + 15) / 16), dim3(256), 0, s, tb, to, n, ix, cnt, gathers,
                       fb_list, fb_count, da);
  else
    hipLaunchKernelGGL((k_walkf<16, false, 1, true>), dim3((n + 15) / 16), dim3(256), 0, s, tb, to, n, ix, cnt, gathers,
                       fb_list, fb_count, da);
  // the topics the frontier could not hold: k_walk's gather slots (clamped counts), then k_desc
  const dim3 fgrid(std::max<uint32_t>(1, std::min<uint32_t>((n + 255) / 256, fb_blocks)));
  hipLaunchKernelGGL((k_walk<false, false, 1>), fgrid, dim3(256), 0, s, tb, to, n, ix, cnt, nullptr, gathers, ovf,
                     fb_list, fb_count, true);
  DescArgs fa = da;
  fa.list = fb_list;
  fa.n_list = fb_count;
  fa.g_count = cnt;
  fa.gathers = gathers;
  fa.gather_stride = kGatherCap;
  hipLaunchKernelGGL(k_desc_g16, fgrid, dim3(256), 0, s, fa);
}

void launch_scan(const TopicCount* cnt, uint32_t n, TopicOff* bsum, TopicOff* bpre, TopicOff* off,
                 hipStream_t s) {
  if (!n) return;
  const uint32_t nb = (n + kScanBlock - 1) / kScanBlock;
  hipLaunchKernelGGL(k_scan_reduce, dim3(nb), dim3(256), 0, s, cnt, n, bsum);
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(256), 0, s, bsum, nb, bpre);
  hipLaunchKernelGGL(k_scan_apply, dim3(nb), dim3(256), 0, s, cnt, n, bpre, off);
}

void launch_desc(const DescArgs& a, bool spans, hipStream_t s) {
  if (!a.n) return;
  if (spans && a.msig)  // dedup lists: 16 lanes per topic
    hipLaunchKernelGGL(k_desc_g16, dim3((a.n + 15) / 16), dim3(256), 0, s, a);
  else if (spans)
    hipLaunchKernelGGL(k_desc<true>, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(k_desc<false>, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
}

void launch_copy(const EmitArgs& a, uint32_t max_blocks, hipStream_t s) {
  const uint32_t waves = a.n_tiles[0] + a.n_tiles[1] + a.n_tiles[2];
  if (!waves) return;
  const uint32_t blocks = max_blocks ? std::min((waves + 3) / 4, max_blocks) : (waves + 3) / 4;
  hipLaunchKernelGGL(k_copy, dim3(blocks), dim3(256), 0, s, a);
}

void launch_merge(const EmitArgs& a, bool spans, uint32_t wpe, uint32_t max_blocks, hipStream_t s) {
  const uint32_t waves = a.t1 - a.t0;
  if (!waves) return;
  const uint32_t blocks = max_blocks ? std::min((waves + 3) / 4, max_blocks) : (waves + 3) / 4;
  const dim3 g(blocks), b(256);
  if (spans && a.ix.xinfo && a.rep && a.dd_phase == 1) {  // sharded index, merge-set dedup: the set pass
    if (wpe >= 6) hipLaunchKernelGGL((k_merge<true, true, 6, true>), g, b, 0, s, a);
    else hipLaunchKernelGGL((k_merge<true, true, 1, true>), g, b, 0, s, a);
  } else if (spans && a.ix.xinfo) {  // sharded index
    if (wpe >= 6) hipLaunchKernelGGL((k_merge<true, true, 6>), g, b, 0, s, a);
    else hipLaunchKernelGGL((k_merge<true, true, 1>), g, b, 0, s, a);
  } else if (spans && a.rep && a.dd_phase == 1) {  // merge-set dedup: the set pass
    // (MQ_OPT_SET_EXP bits 5 / 6: partner links 3 / 4 per batch instead of kPartBatch)
    if (wpe >= 8 && (a.exp & 32u)) hipLaunchKernelGGL((k_merge<true, false, 8, true, 3>), g, b, 0, s, a);
    else if (wpe >= 8 && (a.exp & 64u)) hipLaunchKernelGGL((k_merge<true, false, 8, true, 4>), g, b, 0, s, a);
    else if (wpe >= 8) hipLaunchKernelGGL((k_merge<true, false, 8, true>), g, b, 0, s, a);
    else if (wpe == 7) hipLaunchKernelGGL((k_merge<true, false, 7, true>), g, b, 0, s, a);
    else if (wpe >= 6) hipLaunchKernelGGL((k_merge<true, false, 6, true>), g, b, 0, s, a);
    else hipLaunchKernelGGL((k_merge<true, false, 1, true>), g, b, 0, s, a);
  } else if (spans) {
    if (wpe >= 8) hipLaunchKernelGGL((k_merge<true, false, 8>), g, b, 0, s, a);
    else if (wpe >= 6) hipLaunchKernelGGL((k_merge<true, false, 6>), g, b, 0, s, a);
    else hipLaunchKernelGGL((k_merge<true, false, 1>), g, b, 0, s, a);
  } else {
    if (wpe >= 8) hipLaunchKernelGGL((k_merge<false, false, 8>), g, b, 0, s, a);
    else if (wpe >= 6) hipLaunchKernelGGL((k_merge<false, false, 6>), g, b, 0, s, a);
    else hipLaunchKernelGGL((k_merge<false, false, 1>), g, b, 0, s, a);
  }
}

// ---------------------------------------------------------------------------------------------
// k_msg: Messages(filter), the reverse retained scan (topics.go:525-579). One wavefront per
// filter. The literal prefix of the filter is walked first (all lanes alike) down to its first
// '+'/'#' level, whose children are the units of parallel work: lane k takes child k of that
// enumeration frame (and k + 64, ...), applies the frame's per-child rule (Q4 $SYS skip at level
// 0, emit at the last level, descend otherwise) and walks the child's subtree depth-first
// without a stack — a frame is (node, level d); a '+'/'#' level enumerates the node's children
// slab (ChildRec: each child's retained state and own slab, read sequentially; childless
// children are never entered) and, after returning from child c, resumes at c's slab position
// + 1 (NodeMsg.child_pos, NodeMsg.parent);
// levels past the last segment repeat it (isolateParticle, topics.go:679-698), which is how a
// trailing '#' covers the subtree. A lane stops when it returns to the enumeration frame.
// FILL=false counts the packets per filter; FILL=true walks again and appends them at the
// filter's offset through a per-wave LDS cursor (Messages' order is Go map order, i.e. none).
// ---------------------------------------------------------------------------------------------
// WPE: minimum waves per SIMD asked of the register allocator (1 = no constraint). The walk
// needs ~127 VGPRs (4 waves per SIMD); fewer registers with some spills buy occupancy for
// this latency-bound kernel (MQ_MSG_WPE picks the variant).
template <bool FILL, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_msg(const uint8_t* __restrict__ fb,
                                             const uint64_t* __restrict__ fo, uint32_t n,
                                             DevIndex ix, TopicCount* __restrict__ cnt,
                                             const TopicOff* __restrict__ off,
                                             uint64_t* __restrict__ handles,
                                             uint64_t* __restrict__ base_out,
                                             uint32_t* __restrict__ count_out,
                                             uint64_t* __restrict__ spec, uint32_t spec_cap) {
  __shared__ uint32_t cursor[4];  // FILL / speculative count: next free slot of the filter
  const uint32_t lane = threadIdx.x & 63, wv = wave_id();
  const uint32_t t = blockIdx.x * 4 + wv;
  if (t >= n) return;  // wave-uniform
  // FILL after a speculative count: only the filters k_msg_place could not place are walked
  if (FILL && spec && cnt[t].gathers == 0) return;
  const uint64_t b0 = fo[t], b1 = fo[t + 1];
  uint32_t total = 0;  // packets of this filter (wave-uniform)
  uint64_t* out = FILL ? handles + off[t].rows : nullptr;
  // speculative count: the handles also go to the filter's scratch slots (first spec_cap)
  uint64_t* sp = (!FILL && spec) ? spec + (uint64_t)t * spec_cap : nullptr;
  bool partial = false;  // a count shortcut (below_live) left the scratch incomplete
  // len(filter) == 0 || Retained.Len() == 0 (topics.go:535)
  if (b1 > b0 && ix.retained_len != 0) {
    ByteReader R(fb);
    bool w = false;
    for (uint64_t i = b0 + lane; i < b1; i += 64) {
      const uint32_t ch = fb[i];
      w |= (ch == '+') | (ch == '#');
    }
    const bool wild = __any(w);
    // the literal prefix, down to the first '+'/'#' level (all lanes alike)
    uint32_t node = kRoot, d = 0;
    SegKey key;
    uint64_t s = b0, e = scan_segment(R, b0, b1, &key);
    bool frame = false;  // an enumeration frame was reached at (node, d)
    if (!wild) {
      // no wildcard: Retained.Get(filter) (topics.go:539-544)
      for (;;) {
        node = lookup(ix, node, key, fb + s, (uint32_t)(e - s));
        if (node == kNone || e >= b1) break;
        s = e + 1;
        e = scan_segment(R, s, b1, &key);
      }
      if (node != kNone && (ix.msg[node].flags & kRetainLive)) {
        if (FILL && lane == 0) out[0] = ix.msg[node].handle;
        if (sp && lane == 0 && spec_cap) sp[0] = ix.msg[node].handle;
        total = 1;
      }
    } else {
      for (;;) {
        const uint32_t len = (uint32_t)(e - s);
        const uint32_t c0 = len == 1 ? R.at(s) : 0;
        if (c0 == '+' || c0 == '#') {
          frame = true;
          break;
        }
        const uint32_t p = lookup(ix, node, key, fb + s, len);  // literal level (topics.go:568-576)
        if (p == kNone) break;
        if (e < b1) {
          node = p;
          d++;
          s = e + 1;
          e = scan_segment(R, s, b1, &key);
          continue;
        }
        const NodeMsg m = ix.msg[p];
        uint64_t h = 0;
        bool hit = false;
        if (m.flags & kRetainPath) {
          hit = (m.flags & kRetainLive) != 0;
          h = m.handle;
        } else if (ix.empty_topic_live) {
          hit = true;
          h = ix.empty_topic_handle;  // Retained.Get("") on a particle without a path (Q6)
        }
        if (hit) {
          if (FILL && lane == 0) out[0] = h;
          if (sp && lane == 0 && spec_cap) sp[0] = h;
          total = 1;
        }
        break;
      }
    }
    if (frame) {  // topics.go:547-565 at (node, d), segment [s, e)
      const uint32_t fd = d;
      const uint64_t fs = s, fe = e;
      const SegKey fkey = key;
      const bool has_next = fe < b1;
      const bool hash = R.at(fs) == '#';
      const NodeMsg nm = ix.msg[node];
      // packets under child k of the frame (its own and its subtree's), counted or appended
      auto child = [&](uint32_t k) -> uint32_t {
        uint32_t c = 0;
        auto emit = [&](uint64_t h) {
          if (FILL) {
            out[atomicAdd(&cursor[wv], 1u)] = h;
          } else if (sp) {
            const uint32_t q = atomicAdd(&cursor[wv], 1u);
            if (q < spec_cap) sp[q] = h;
          }
          c++;
        };
        const ChildRec r0 = ix.children[nm.child_off + k];
        if (fd == 0 && (r0.flags & kChildSys)) return 0u;  // only the exact $SYS particle, level 0 (Q4)
        if (!has_next && (r0.flags & kRetainPath) && (r0.flags & kRetainLive)) emit(r0.handle);
        // a childless particle has nothing below it for any further level: not entered
        if (!(has_next || hash) || r0.child_cnt == 0) return c;
        // count pass, '#' frame: every live retained topic below the child, from its aggregate
        if (!FILL && hash) {
          partial = true;
          return c + ix.msg[r0.node].below_live;
        }
        uint32_t node = r0.node, d = fd + 1, wd = fd;  // wd: level of the segment in the window
        uint32_t coff = r0.child_off, ccnt = r0.child_cnt;  // node's children slab
        uint64_t s = fs, e = fe;
        SegKey key = fkey;
        if (e < b1) {
          s = e + 1;
          e = scan_segment(R, s, b1, &key);
          wd++;
        }
        uint32_t cursor = 0;
        bool resume = false;  // re-entering an enumeration frame after a child returned
        for (uint64_t guard = 0;; guard++) {
          if (guard > kWalkGuard * 64) {
            atomicOr(ix.err, kErrWalkGuard);
            break;
          }
          const bool has_nx = (wd == d) && (e < b1);
          const uint32_t len = (uint32_t)(e - s);
          const uint32_t c0 = len == 1 ? R.at(s) : 0;
          const bool plus = c0 == '+';
          const bool hsh = c0 == '#';
          bool descended = false;
          if (!FILL && hsh) {  // count pass: the subtree's live retained topics (below_live)
            c += ix.msg[node].below_live;
            partial = true;
          } else if (plus || hsh) {  // topics.go:547-565: the slab copy holds what each child needs
            if (!resume) cursor = 0;
            while (cursor < ccnt) {
              const ChildRec cr = ix.children[coff + cursor];
              cursor++;
              if (!has_nx && (cr.flags & kRetainPath) && (cr.flags & kRetainLive)) emit(cr.handle);
              if ((has_nx || hsh) && cr.child_cnt != 0) {
                node = cr.node;
                coff = cr.child_off;
                ccnt = cr.child_cnt;
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
              const NodeMsg m = ix.msg[p];
              if (has_nx) {
                if (m.child_cnt != 0) {
                  node = p;
                  coff = m.child_off;
                  ccnt = m.child_cnt;
                  d++;
                  s = e + 1;
                  e = scan_segment(R, s, b1, &key);
                  wd++;
                  descended = true;
                }
              } else if (m.flags & kRetainPath) {
                if (m.flags & kRetainLive) emit(m.handle);
              } else if (ix.empty_topic_live) {
                emit(ix.empty_topic_handle);  // Q6
              }
            }
          }
          if (descended) {
            resume = false;
            continue;
          }
          // frame finished: return to the parent frame; the child of the wave's enumeration
          // frame is done when we would return into it
          if (d == fd + 1) break;
          const NodeMsg cm = ix.msg[node];
          node = cm.parent;
          const NodeMsg pm = ix.msg[node];
          coff = pm.child_off;
          ccnt = pm.child_cnt;
          if (wd == d) {
            e = s - 1;
            s = seg_start_before(R, b0, e);
            wd--;
          }
          d--;
          cursor = cm.child_pos + 1;
          resume = true;
        }
        return c;
      };
      if ((FILL || sp) && lane == 0) cursor[wv] = total;
      wave_sync_lds();
      if (!FILL && hash && fd > 0) {
        // count pass, '#' below level 0 (no $SYS exclusion): the frame's aggregate
        total += nm.below_live;
        partial = true;
      } else
      for (uint32_t k0 = 0; k0 < nm.child_cnt; k0 += 64) {  // wave-uniform
        const uint32_t k = k0 + lane;
        total += wave_sum(k < nm.child_cnt ? child(k) : 0u);
      }
    }
  }
  const bool walk_again = __any(partial) || total > spec_cap;  // for the FILL pass
  if (lane == 0) {
    if (!FILL) {
      cnt[t] = TopicCount{(sp && !walk_again) ? 0u : 1u, total, 0, 0, 0};
    } else {
      base_out[t] = off[t].rows;
      count_out[t] = total;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// k_acl: auth.MatchTopic (hooks/auth/ledger.go:90-118) for (filter, topic) pairs — the ACL test
// the fan-out runs per recipient (server.go:1029 -> Ledger.ACLOk -> FilterMatches). One thread
// per pair; filter and topic are split on '/' as strings.Split does (an empty string is one empty
// part); '+' captures the topic part, '#' captures the rest of the topic (when a part exists at
// its position) and matches; a filter that runs out first matches (the reference's prefix rule).
// Captured elements are (start, len) spans into the topic, written from elem_base[pair].
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_acl(AclArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n_pairs) return;
  const uint32_t f = a.pair_filter[i], t = a.pair_topic[i];
  const uint64_t fb0 = a.filter_offs[f], fb1 = a.filter_offs[f + 1];
  const uint64_t tb0 = a.topic_offs[t], tb1 = a.topic_offs[t + 1];
  ByteReader RF(a.filter_bytes), RT(a.topic_bytes);
  uint32_t* el = a.elems + 2 * a.elem_base[i];
  uint32_t n_el = 0;
  bool matched = true;
  uint64_t fs = fb0, ts = tb0;
  bool topic_left = true;  // a topic part exists at this index
  for (;;) {
    const uint64_t fe = find_slash(RF, fs, fb1);
    if (!topic_left) {  // ledger.go:95-98
      matched = false;
      break;
    }
    const uint64_t te = find_slash(RT, ts, tb1);
    const uint64_t flen = fe - fs;
    const uint32_t c0 = flen == 1 ? RF.at(fs) : 0u;
    if (c0 == '+') {  // ledger.go:100-103
      el[2 * n_el] = (uint32_t)(ts - tb0);
      el[2 * n_el + 1] = (uint32_t)(te - ts);
      n_el++;
    } else if (c0 == '#') {  // ledger.go:105-109
      el[2 * n_el] = (uint32_t)(ts - tb0);
      el[2 * n_el + 1] = (uint32_t)(tb1 - ts);
      n_el++;
      break;
    } else {  // ledger.go:111-114
      bool eq = flen == te - ts;
      for (uint64_t k = 0; eq && k < flen; k++) eq = RF.at(fs + k) == RT.at(ts + k);
      if (!eq) {
        matched = false;
        break;
      }
    }
    if (fe >= fb1) break;  // the filter's parts are used up: ledger.go:117
    fs = fe + 1;
    topic_left = te < tb1;
    ts = topic_left ? te + 1 : tb1;
  }
  a.matched[i] = matched ? 1 : 0;
  a.n_elems[i] = n_el;
}

void launch_acl(const AclArgs& a, hipStream_t s) {
  if (!a.n_pairs) return;
  hipLaunchKernelGGL(k_acl, dim3((uint32_t)((a.n_pairs + 255) / 256)), dim3(256), 0, s, a);
}

// ---------------------------------------------------------------------------------------------
// k_pick — SelectShared on the device (topics.go:320-333). Go keeps the first
// member of each Shared[filter] map in random iteration order, so any one member is a conformant
// pick; this one is deterministic: the member with the smallest client id. One wavefront per
// topic: the topic's shared rows are inserted into a per-wave LDS hash table keyed by filter id
// (atomicMin of the client per slot), then streamed again in row order and each filter's picked
// row is compacted by ballot/mbcnt into `sel` at the topic's shared_base. A topic with more
// distinct filters than the table holds is re-run in hash partitions (2, 4, ... passes over its
// rows), each pass with the table to itself. (filter, client) pairs are unique within a topic
// (a filter lives at one node, keyed there by (group, client)), so exactly one row wins.
// ---------------------------------------------------------------------------------------------
constexpr uint32_t kPickSlots = 1024;       // per wave: 8 KB of LDS
constexpr uint32_t kPickProbe = 256;        // probe bound before a pass is split
constexpr uint32_t kPickMaxParts = 1u << 16;
constexpr uint32_t kPickBatch = 16;         // rows per lane in flight (1024 per wave)

__device__ __forceinline__ bool pick_in_part(uint32_t filter_id, uint32_t parts, uint32_t part) {
  return parts == 1 || hash32(filter_id ^ 0x5bd1e995u) % parts == part;
}

// One wavefront per workgroup: a topic's table is released as soon as its own wave ends.
// Row format: the topic's shared rows are one contiguous segment; span format: one segment per
// span (the shared-pool ranges of its gathered particles), picks written at picked_base.
template <bool SPANS>
__global__ __launch_bounds__(64) void k_pick(PickArgs a) {
  __shared__ uint32_t K[kPickSlots];  // filter id + 1 (0 = empty)
  __shared__ uint32_t V[kPickSlots];  // smallest client id seen
  const uint32_t lane = threadIdx.x;
  const uint32_t t = blockIdx.x;
  uint64_t base, span_base = 0;
  uint32_t cnt, n_seg = 1;
  if (SPANS) {
    const TopicSpansDev& r = a.sres[t];
    base = r.picked_base;
    cnt = r.n_shared;
    span_base = r.span_base;
    n_seg = r.n_spans;
  } else {
    base = a.res[t].shared_base;
    cnt = a.res[t].n_shared;
  }
  // segment k of the topic's shared rows (wave-uniform)
  auto segment = [&](uint32_t k, const ShrRec** p, uint32_t* c) {
    if (SPANS) {
      const SpanRec sp = a.spans[span_base + k];
      *p = a.pool + sp.shr_off;
      *c = sp.n_shr;
    } else {
      *p = a.rows + base;
      *c = cnt;
    }
  };
  constexpr uint32_t kSpan = 64 * kPickBatch;
  const bool resident = !SPANS && cnt <= kSpan;  // the mark pass reuses the rows held in registers
  ShrRec buf[kPickBatch];
  uint32_t picked = 0;
  uint32_t parts = 1;
  // table size: a power of two >= 2 * rows (64 .. kPickSlots), so small topics clear little
  uint32_t tsize = 64;
  while (tsize < kPickSlots && tsize < 2 * cnt) tsize *= 2;
  for (uint32_t part = 0; cnt && part < parts;) {
    const uint32_t tmask = tsize - 1;
    for (uint32_t i = lane; i < tsize; i += 64) {
      K[i] = 0;
      V[i] = 0xFFFFFFFFu;
    }
    wave_sync_lds();
    bool full = false;
    for (uint32_t sg = 0; sg < n_seg; sg++) {
      const ShrRec* rows;
      uint32_t sc;
      segment(sg, &rows, &sc);
      for (uint32_t rb = 0; rb < sc; rb += kSpan) {
#pragma unroll
        for (uint32_t j = 0; j < kPickBatch; j++) {  // all loads issued before any use
          const uint32_t r = rb + j * 64 + lane;
          buf[j] = r < sc ? rows[r] : ShrRec{0, 0};
        }
#pragma unroll
        for (uint32_t j = 0; j < kPickBatch; j++) {
          const uint32_t r = rb + j * 64 + lane;
          if (r >= sc || !pick_in_part(buf[j].filter_id, parts, part)) continue;
          const uint32_t key = buf[j].filter_id + 1;
          uint32_t slot = hash32(buf[j].filter_id) & tmask;
          for (uint32_t probe = 0;; probe++) {
            if (probe == kPickProbe || probe == tsize) {
              full = true;
              break;
            }
            // plain LDS reads first: a filter's later members mostly find their slot claimed
            // and the client beaten, and skip the atomics (same-slot atomics serialise)
            uint32_t k = K[slot];
            if (k == 0u) {
              k = atomicCAS(&K[slot], 0u, key);
              if (k == 0u) k = key;
            }
            if (k == key) {
              if (buf[j].client < V[slot]) atomicMin(&V[slot], buf[j].client);
              break;
            }
            slot = (slot + 1) & tmask;
          }
        }
      }
    }
    wave_sync_lds();
    if (__any(full)) {  // too many filters for the table: grow it, then split into partitions
      if (parts >= kPickMaxParts) {
        if (lane == 0) atomicOr(a.err, kErrPickGuard);
        picked = 0;
        break;
      }
      if (tsize < kPickSlots) tsize = kPickSlots;
      else parts *= 2;
      part = 0;
      picked = 0;
      continue;
    }
    for (uint32_t sg = 0; sg < n_seg; sg++) {
      const ShrRec* rows;
      uint32_t sc;
      segment(sg, &rows, &sc);
      for (uint32_t rb = 0; rb < sc; rb += kSpan) {
        if (!resident) {
#pragma unroll
          for (uint32_t j = 0; j < kPickBatch; j++) {
            const uint32_t r = rb + j * 64 + lane;
            buf[j] = r < sc ? rows[r] : ShrRec{0, 0};
          }
        }
#pragma unroll
        for (uint32_t j = 0; j < kPickBatch; j++) {
          if (rb + j * 64 >= sc) break;  // wave-uniform
          const uint32_t r = rb + j * 64 + lane;
          bool take = false;
          if (r < sc && pick_in_part(buf[j].filter_id, parts, part)) {
            const uint32_t key = buf[j].filter_id + 1;
            uint32_t slot = hash32(buf[j].filter_id) & tmask;
            while (K[slot] != key) slot = (slot + 1) & tmask;  // inserted above
            take = V[slot] == buf[j].client;
          }
          const uint64_t m = __ballot(take);
          if (take) a.sel[base + picked + prefix_before(m)] = buf[j];
          picked += (uint32_t)__popcll(m);
        }
      }
    }
    wave_sync_lds();  // the next pass clears the table
    part++;
  }
  if (lane == 0) a.n_out[(uint64_t)t * a.n_out_stride] = picked;
}

void launch_pick(const PickArgs& a, hipStream_t s) {
  if (!a.n) return;
  if (a.sres)
    hipLaunchKernelGGL(k_pick<true>, dim3(a.n), dim3(64), 0, s, a);
  else
    hipLaunchKernelGGL(k_pick<false>, dim3(a.n), dim3(64), 0, s, a);
}

// Sharded index: each topic's gathered cross-shard nodes (the exported list).
template <bool COUNT>
__global__ __launch_bounds__(256) void k_xlist(DevIndex ix, uint32_t n, const TopicOff* __restrict__ off,
                                               const uint32_t* __restrict__ gathers, uint32_t gather_stride,
                                               TopicCount* __restrict__ cnt, const TopicOff* __restrict__ xoff,
                                               XEnt* __restrict__ ents, uint32_t* __restrict__ counts) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint32_t n_g = (uint32_t)(off[t + 1].g - off[t].g);
  const uint32_t* gw_src = gather_stride ? gathers + (uint64_t)t * gather_stride : gathers + off[t].g;
  uint32_t k = 0;
  XEnt* out = COUNT ? nullptr : ents + xoff[t].g;
  for (uint32_t g = 0; g < n_g; g++) {
    const uint32_t gw = gw_src[g];
    if (!(gw & kGatherSubs)) continue;
    const uint32_t node = gw & kGatherNode;
    if (!(ix.lists[node].flags & kFlagXNode)) continue;
    if (!COUNT) {
      const XInfo x = ix.xinfo[node];
      out[k] = XEnt{x.fid, x.deep, x.rank};
    }
    k++;
  }
  if (COUNT) cnt[t] = TopicCount{k, 0, 0, 0, 0};
  else counts[t] = k;
}

void launch_xlist(bool count, const DevIndex& ix, uint32_t n, const TopicOff* off, const uint32_t* gathers,
                  uint32_t gather_stride, TopicCount* cnt, const TopicOff* xoff, XEnt* ents, uint32_t* counts,
                  hipStream_t s) {
  if (!n) return;
  if (count)
    hipLaunchKernelGGL(k_xlist<true>, dim3((n + 255) / 256), dim3(256), 0, s, ix, n, off, gathers, gather_stride, cnt,
                       xoff, ents, counts);
  else
    hipLaunchKernelGGL(k_xlist<false>, dim3((n + 255) / 256), dim3(256), 0, s, ix, n, off, gathers, gather_stride, cnt,
                       xoff, ents, counts);
}

__global__ __launch_bounds__(256) void k_counts(const uint32_t* __restrict__ counts, uint32_t n,
                                                TopicCount* __restrict__ cnt) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) cnt[t] = TopicCount{counts[t], 0, 0, 0, 0};
}

void launch_counts(const uint32_t* counts, uint32_t n, TopicCount* cnt, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_counts, dim3((n + 255) / 256), dim3(256), 0, s, counts, n, cnt);
}

__global__ __launch_bounds__(256) void k_patch_compact(const PatchRec* __restrict__ pool, uint64_t rcap,
                                                      const unsigned long long* __restrict__ pcount,
                                                      const uint64_t* __restrict__ roff, PatchRec* __restrict__ out) {
  const uint32_t r = blockIdx.x;
  const uint64_t n = pcount[r];
  const PatchRec* src = pool + (uint64_t)r * rcap;
  PatchRec* dst = out + roff[r];
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
}

void launch_patch_compact(const PatchRec* pool, uint64_t rcap, const unsigned long long* pcount,
                          const uint64_t* roff, PatchRec* out, hipStream_t s) {
  hipLaunchKernelGGL(k_patch_compact, dim3(kPatchRegions), dim3(256), 0, s, pool, rcap, pcount, roff, out);
}

template <int WPE>
static void launch_msg_wpe(bool fill, const uint8_t* fb, const uint64_t* fo, uint32_t n, const DevIndex& ix,
                           TopicCount* cnt, const TopicOff* off, uint64_t* handles, uint64_t* base,
                           uint32_t* count, uint64_t* spec, uint32_t spec_cap, hipStream_t s) {
  dim3 grid((n + 3) / 4);  // one wavefront per filter
  if (fill)
    hipLaunchKernelGGL((k_msg<true, WPE>), grid, dim3(256), 0, s, fb, fo, n, ix, cnt, off, handles, base, count,
                       spec, spec_cap);
  else
    hipLaunchKernelGGL((k_msg<false, WPE>), grid, dim3(256), 0, s, fb, fo, n, ix, cnt, off, handles, base,
                       count, spec, spec_cap);
}

void launch_msg(bool fill, const uint8_t* fb, const uint64_t* fo, uint32_t n, const DevIndex& ix,
                TopicCount* cnt, const TopicOff* off, uint64_t* handles, uint64_t* base,
                uint32_t* count, uint64_t* spec, uint32_t spec_cap, uint32_t wpe, hipStream_t s) {
  if (!n) return;
  if (wpe >= 8)
    launch_msg_wpe<8>(fill, fb, fo, n, ix, cnt, off, handles, base, count, spec, spec_cap, s);
  else if (wpe >= 6)
    launch_msg_wpe<6>(fill, fb, fo, n, ix, cnt, off, handles, base, count, spec, spec_cap, s);
  else
    launch_msg_wpe<1>(fill, fb, fo, n, ix, cnt, off, handles, base, count, spec, spec_cap, s);
}

// k_msg_place: after a speculative count, every filter whose handles all sit in its scratch
// slots is moved to its output range (one wavefront per filter, coalesced 8-byte rows); the
// others (more than spec_cap handles, or counted through a below_live shortcut) are left to
// k_msg<true>, which walks only them.
__global__ __launch_bounds__(256) void k_msg_place(uint32_t n, const TopicCount* __restrict__ cnt,
                                                   const TopicOff* __restrict__ off,
                                                   const uint64_t* __restrict__ spec, uint32_t spec_cap,
                                                   uint64_t* __restrict__ handles,
                                                   uint64_t* __restrict__ base_out,
                                                   uint32_t* __restrict__ count_out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t t = blockIdx.x * 4 + wave_id();
  if (t >= n) return;
  const TopicCount c = cnt[t];
  if (c.gathers != 0) return;  // walked again by the FILL pass
  const uint64_t o = off[t].rows;
  const uint64_t* src = spec + (uint64_t)t * spec_cap;
  for (uint32_t i = lane; i < c.rows; i += 64) handles[o + i] = src[i];
  if (lane == 0) {
    base_out[t] = o;
    count_out[t] = c.rows;
  }
}

void launch_msg_place(uint32_t n, const TopicCount* cnt, const TopicOff* off, const uint64_t* spec,
                      uint32_t spec_cap, uint64_t* handles, uint64_t* base, uint32_t* count, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_msg_place, dim3((n + 3) / 4), dim3(256), 0, s, n, cnt, off, spec, spec_cap, handles,
                     base, count);
}

// Workgroup per run: byte head up to 16-byte alignment (source and destination agree mod 16),
// 16-byte body, byte tail.
__global__ __launch_bounds__(256) void k_scatter(const ScatterRun* __restrict__ runs,
                                                 const uint8_t* __restrict__ stage) {
  const ScatterRun r = runs[blockIdx.x];
  uint8_t* d = reinterpret_cast<uint8_t*>(r.dst);
  const uint8_t* s = stage + r.src;
  const uint64_t head = min(r.bytes, (uint64_t)((16 - (r.dst & 15)) & 15));
  for (uint64_t i = threadIdx.x; i < head; i += 256) d[i] = s[i];
  const uint64_t body = (r.bytes - head) >> 4;
  const u32x4* s4 = reinterpret_cast<const u32x4*>(s + head);
  u32x4* d4 = reinterpret_cast<u32x4*>(d + head);
  for (uint64_t i = threadIdx.x; i < body; i += 256) d4[i] = s4[i];
  for (uint64_t i = head + (body << 4) + threadIdx.x; i < r.bytes; i += 256) d[i] = s[i];
}

void launch_scatter(const ScatterRun* runs, uint32_t n, const uint8_t* stage, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_scatter, dim3(n), dim3(256), 0, s, runs, stage);
}

// ---------------------------------------------------------------------------------------------
// Messages over the level-order retained image (kernels.h MsgImg): the reverse
// retained scan (topics.go:530-579) as run arithmetic. A '+' or '#' level with more segments
// after it takes every image child of the run (its particles' children that have live retained
// state at or below them: the others add nothing), a final '+' emits the children's live
// handles, a final '#' every level below (isolateParticle repeats the last segment past the end,
// topics.go:679-698), the root's "$SYS" child excluded at level 0 (topics.go:549, Q4). A literal
// level looks the segment up under each particle of the run (topics.go:568-576); under a run of
// more than one particle this is the only fan-out: the wave's lanes take the run's particles,
// and a lane keeps deeper fan-outs on a small frame stack.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t block_scan_incl32(uint32_t v, uint32_t* wt /*4*/) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t tot;
  const uint32_t ex = wave_excl_scan(v, lane, &tot);
  if (lane == 0) wt[wv] = tot;
  __syncthreads();
  uint32_t add = 0;
  for (uint32_t w = 0; w < wv; w++) add += wt[w];
  __syncthreads();
  return ex + v + add;
}

__global__ __launch_bounds__(256) void k_scan32_reduce(const uint32_t* __restrict__ in, uint64_t n,
                                                       uint32_t* __restrict__ bsum) {
  __shared__ uint32_t wt[4];
  const uint64_t base = (uint64_t)blockIdx.x * kScanBlock + threadIdx.x * 4;
  uint32_t v = 0;
  for (int k = 0; k < 4; k++)
    if (base + k < n) v += in[base + k];
  v = block_scan_incl32(v, wt);
  if (threadIdx.x == 255) bsum[blockIdx.x] = v;
}

// Single workgroup: exclusive scan of the block sums; bpre[nb] = total.
__global__ __launch_bounds__(256) void k_scan32_blocks(const uint32_t* __restrict__ bsum, uint32_t nb,
                                                       uint32_t* __restrict__ bpre) {
  __shared__ uint32_t wt[4];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t b0 = 0; b0 < nb; b0 += 256) {
    const uint32_t b = b0 + threadIdx.x;
    const uint32_t v = b < nb ? bsum[b] : 0u;
    const uint32_t incl = block_scan_incl32(v, wt);
    if (b < nb) bpre[b] = carry + incl - v;
    __syncthreads();
    if (threadIdx.x == 255) carry += incl;
    __syncthreads();
  }
  if (threadIdx.x == 0) bpre[nb] = carry;
}

// in and out may alias: every thread reads its four elements before any is written
__global__ __launch_bounds__(256) void k_scan32_apply(const uint32_t* in, uint64_t n,
                                                      const uint32_t* __restrict__ bpre, uint32_t* out) {
  __shared__ uint32_t wt[4];
  const uint64_t base = (uint64_t)blockIdx.x * kScanBlock + threadIdx.x * 4;
  uint32_t c[4], v = 0;
  for (int k = 0; k < 4; k++) {
    c[k] = base + k < n ? in[base + k] : 0u;
    v += c[k];
  }
  const uint32_t incl = block_scan_incl32(v, wt);
  uint32_t ex = bpre[blockIdx.x] + incl - v;
  for (int k = 0; k < 4; k++) {
    if (base + k < n) out[base + k] = ex;
    ex += c[k];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = bpre[gridDim.x];
}

void launch_scan32(const uint32_t* in, uint64_t n, uint32_t* bsum, uint32_t* bpre, uint32_t* out,
                   hipStream_t s) {
  if (n == 0) {
    (void)hipMemsetAsync(out, 0, sizeof(uint32_t), s);  // errors surface at the caller's next check
    return;
  }
  const uint32_t nb = (uint32_t)((n + kScanBlock - 1) / kScanBlock);
  hipLaunchKernelGGL(k_scan32_reduce, dim3(nb), dim3(256), 0, s, in, n, bsum);
  hipLaunchKernelGGL(k_scan32_blocks, dim3(1), dim3(256), 0, s, bsum, nb, bpre);
  hipLaunchKernelGGL(k_scan32_apply, dim3(nb), dim3(256), 0, s, in, n, bpre, out);
}

__global__ void k_img_root(uint32_t* node, uint32_t* pos, uint32_t* live) {
  if (threadIdx.x == 0) {
    node[0] = kRoot;
    pos[kRoot] = 0;
    live[0] = 0;  // the root has no retain path ("" is kept apart, Q6)
  }
}

// Wavefront per parent of the level: its children slab (ChildRec) in slab order; a child is in
// the image when its own retained message is live or one below it is (NodeMsg.below_live).
template <bool FILL>
// Grid-stride over the level's parents (a level of a 100M-topic index holds more parents than
// one wavefront each can launch: a grid is limited to 2^32 threads).
__global__ __launch_bounds__(256) void k_img_level(DevIndex ix, ImgLevelArgs a) {
  const uint32_t lane = threadIdx.x & 63, wv = wave_id();
  for (uint32_t p = blockIdx.x * 4 + wv; p < a.n; p += gridDim.x * 4) {  // wave-uniform
  const uint32_t v = a.node[a.lo + p];
  const NodeMsg m = ix.msg[v];
  const bool root = v == kRoot;
  const uint32_t base = FILL ? a.next + a.coff[p] : 0u;
  uint32_t run = 0;
  uint32_t sys_node = kNone, sys_live = 0;  // the root's "$SYS" child goes last
  if (m.below_live != 0) {
    for (uint32_t k0 = 0; k0 < m.child_cnt; k0 += 64) {  // wave-uniform
      const uint32_t k = k0 + lane;
      bool incl = false, live = false, sys = false;
      uint32_t c = kNone;
      if (k < m.child_cnt) {
        const ChildRec r = ix.children[m.child_off + k];
        c = r.node;
        live = (r.flags & kRetainPath) && (r.flags & kRetainLive);
        incl = live || ix.msg[c].below_live != 0;
        sys = root && (r.flags & kChildSys);
      }
      const uint64_t bm = __ballot(incl && !sys);
      if (FILL && incl && !sys) {
        const uint32_t q = base + run + prefix_before(bm);
        a.node[q] = c;
        a.pos[c] = q;
        a.live[q] = live ? 1u : 0u;
      }
      if (incl && sys) {
        sys_node = c;
        sys_live = live ? 1u : 0u;
      }
      run += (uint32_t)__popcll(bm);
    }
  }
  const bool has_sys = __ballot(sys_node != kNone) != 0;
  if (FILL && sys_node != kNone) {
    const uint32_t q = base + run;
    a.node[q] = sys_node;
    a.pos[sys_node] = q;
    a.live[q] = sys_live;
  }
  const uint32_t total = run + (has_sys ? 1u : 0u);
  if (lane == 0) {
    if (FILL) a.cl[a.lo + p] = make_uint2(base, base + total);
    else a.cnt[p] = total;
  }
  }
}

__global__ __launch_bounds__(256) void k_img_compact(DevIndex ix, const uint32_t* __restrict__ node,
                                                     const uint32_t* __restrict__ lp, uint32_t n,
                                                     uint64_t* __restrict__ h) {
  const uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= n) return;
  const uint32_t l = lp[q];
  if (lp[q + 1] != l) h[l] = ix.msg[node[q]].handle;
}

void launch_img_root(uint32_t* node, uint32_t* pos, uint32_t* live, hipStream_t s) {
  hipLaunchKernelGGL(k_img_root, dim3(1), dim3(64), 0, s, node, pos, live);
}

void launch_img_level(bool fill, const DevIndex& ix, const ImgLevelArgs& a, hipStream_t s) {
  if (!a.n) return;
  const dim3 g(std::min<uint32_t>((a.n + 3) / 4, kMaxWaveBlocks)), b(256);
  if (fill) hipLaunchKernelGGL(k_img_level<true>, g, b, 0, s, ix, a);
  else hipLaunchKernelGGL(k_img_level<false>, g, b, 0, s, ix, a);
}

void launch_img_compact(const DevIndex& ix, const uint32_t* node, const uint32_t* lp, uint32_t n,
                        uint64_t* h, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_img_compact, dim3((n + 255) / 256), dim3(256), 0, s, ix, node, lp, n, h);
}

// Image position of particle c, or kNone (not in the image: no live retained at or below it).
__device__ __forceinline__ uint32_t img_pos(const MsgImg& img, uint32_t c) {
  if (c >= img.n_pos) return kNone;  // kNone included
  const uint32_t q = img.pos[c];
  return (q < img.n && img.node[q] == c) ? q : kNone;
}

struct MsgFrame {  // a fan-out in progress: particles [cur, end) still to take segment s
  uint32_t cur, end, s;
};

// Wavefront per filter. MODE (kernels.h MsgMode): kMsgCount counts the filter's handles and copy
// pieces; kMsgFill writes short runs and piece records at the offsets of the count pass's scan;
// kMsgRuns counts and records the runs (their output and piece offsets fixed by the same LDS
// cursors the fill pass uses); kMsgPlace places recorded runs without walking again — the
// filter's walk then runs once per batch instead of twice.
template <int MODE>
__global__ __launch_bounds__(256) void k_msgq(const uint8_t* __restrict__ fb, const uint64_t* __restrict__ fo,
                                              uint32_t n, DevIndex ix, MsgImg img,
                                              TopicCount* __restrict__ cnt, const TopicOff* __restrict__ off,
                                              MsgPiece* __restrict__ pieces, uint64_t* __restrict__ handles,
                                              uint64_t* __restrict__ base_out, uint32_t* __restrict__ count_out,
                                              MsgRun* __restrict__ runs, uint32_t run_cap,
                                              uint32_t* __restrict__ n_runs, MsgWide w) {
  constexpr bool WIDE = MODE == kMsgWideCount || MODE == kMsgWideFill;  // exported work items
  constexpr bool FILL = MODE == kMsgFill || MODE == kMsgPlace || MODE == kMsgWideFill;  // the walk writes output
  constexpr bool RUNS = MODE == kMsgRuns;
  __shared__ uint32_t hcur[4], pcur[4], rcur[4];  // next handle / piece / run of the wave's filter
  __shared__ uint2 mfront[4][2][kMsgFront];       // fan-out frontier: runs of one level (two buffers)
  __shared__ uint32_t mpre[4][kMsgFront + 1];      // ... particles before each run
  const uint32_t lane = threadIdx.x & 63, wv = wave_id();
  uint32_t t = blockIdx.x * 4 + wv;  // (a work item's filter in the wide modes)
  if (!WIDE && t >= n) return;  // wave-uniform
  const uint64_t c_start = (!FILL && !WIDE && img.cyc) ? clock64() : 0ull;
  uint64_t b0 = 0, b1 = 0, obase = 0, pbase = 0;
  if (!WIDE) {
    b0 = fo[t];
    b1 = fo[t + 1];
    obase = FILL ? off[t].rows : 0;
    pbase = FILL ? off[t].g : 0;
  }
  // one piece record per kMsgPiece handles of a long run
  auto put_pieces = [&](uint32_t h0, uint32_t len, uint32_t dst, uint32_t slot) __attribute__((always_inline)) {
    const uint32_t npc = (len + kMsgPiece - 1) / kMsgPiece;
    for (uint32_t i = 0; i < npc; i++)
      pieces[pbase + slot + i] = MsgPiece{h0 + i * kMsgPiece, (uint32_t)min(kMsgPiece, len - i * kMsgPiece),
                                          obase + dst + (uint64_t)i * kMsgPiece};
  };
  if (MODE == kMsgPlace) {
    const uint32_t nr = n_runs[t];
    if (nr != kNone) {  // wave-uniform: the count pass recorded every run of this filter
      const MsgRun* __restrict__ fr = runs + (uint64_t)t * run_cap;
      for (uint32_t k = lane; k < nr; k += 64) {
        const MsgRun r = fr[k];
        if (r.len > kMsgDirect) put_pieces(r.h0, r.len, r.dst, r.pslot);
        else
          for (uint32_t j = 0; j < r.len; j++) handles[obase + r.dst + j] = img.h[r.h0 + j];
      }
      if (lane == 0) {
        base_out[t] = obase;
        count_out[t] = cnt[t].rows;
      }
      return;
    }
  }
  if (FILL || RUNS || WIDE) {
    if (lane == 0) hcur[wv] = pcur[wv] = rcur[wv] = 0;
    wave_sync_lds();
  }
  uint32_t nh = 0, np = 0;  // count pass: this lane's handles and pieces
  auto emit = [&](uint32_t h0, uint32_t len) __attribute__((always_inline)) {
    if (len == 0) return;
    const uint32_t npc = len > kMsgDirect ? (len + kMsgPiece - 1) / kMsgPiece : 0u;
    if (!FILL) {
      nh += len;
      np += npc;
      if (!RUNS && MODE != kMsgWideCount) return;
    }
    const uint32_t dst = atomicAdd(&hcur[wv], len);
    const uint32_t slot = npc ? atomicAdd(&pcur[wv], npc) : 0u;
    if (RUNS) {
      const uint32_t ri = atomicAdd(&rcur[wv], 1u);
      if (ri < run_cap) runs[(uint64_t)t * run_cap + ri] = MsgRun{h0, len, dst, slot};
      return;
    }
    if (MODE == kMsgWideCount) {  // into the wavefront's scratch (its cursor runs across items)
      const uint32_t ri = atomicAdd(&rcur[wv], 1u);
      if (ri < w.per_wave) w.scratch[(uint64_t)(blockIdx.x * 4 + wv) * w.per_wave + ri] = MsgRun{h0, len, dst, slot};
      return;
    }
    if (!npc) {
      for (uint32_t k = 0; k < len; k++) handles[obase + dst + k] = img.h[h0 + k];
      return;
    }
    put_pieces(h0, len, dst, slot);
  };
  // image children of the run [a, b) (a < b); at level 0 without "$SYS" (topics.go:549)
  auto desc = [&](uint32_t a, uint32_t b, uint32_t& x, uint32_t& y) __attribute__((always_inline)) {
    x = img.cl[a].x;
    y = img.cl[b - 1].y;
    if (a == 0 && y > x && (ix.msg[img.node[y - 1]].flags & kChildSys)) y--;
  };
  // a final '+' (one level) or '#' (every level below) over the children run [x, y)
  auto emit_final = [&](bool hash, uint32_t x, uint32_t y) __attribute__((always_inline)) {
    for (uint32_t guard = 0; x < y && guard < 4096; guard++) {
      emit(img.lp[x], img.lp[y] - img.lp[x]);
      if (!hash) break;
      const uint32_t nx = img.cl[x].x, ny = img.cl[y - 1].y;
      x = nx;
      y = ny;
    }
  };
  ByteReader R(fb);
  auto dfs_run = [&](uint32_t ra, uint32_t rb, uint64_t rs) __attribute__((always_inline)) {
    MsgFrame st[kMsgStack];
    for (uint32_t u = ra + lane; u < rb; u += 64) {
      uint32_t sp = 0, ua = u, ub = u + 1;
      uint64_t us = rs;
      for (uint64_t guard = 0;; guard++) {
        if (guard > kWalkGuard) {
          atomicOr(ix.err, kErrWalkGuard);
          break;
        }
        bool pop = false;
        const uint64_t e = find_slash(R, us, b1);
        const bool last = e >= b1;
        const uint32_t len = (uint32_t)(e - us);
        const uint32_t c0 = len == 1 ? R.at(us) : 0u;
        if (c0 == '+' || c0 == '#') {
          uint32_t x, y;
          desc(ua, ub, x, y);
          if (last) {
            emit_final(c0 == '#', x, y);
            pop = true;
          } else {
            ua = x;
            ub = y;
            us = e + 1;
            pop = ua >= ub;
          }
        } else if (ub - ua > 1) {  // a literal under a run: one particle now, the rest later
          if (sp == kMsgStack) {
            atomicOr(ix.err, kErrMsgNest);
            break;
          }
          st[sp++] = MsgFrame{ua + 1, ub, (uint32_t)(us - b0)};
          ub = ua + 1;
        } else {
          SegKey key = key_of(R, us, e);
          const uint32_t qc = img_pos(img, lookup(ix, img.node[ua], key, fb + us, len));
          if (qc == kNone) {
            pop = true;
          } else if (last) {
            emit(img.lp[qc], img.lp[qc + 1] - img.lp[qc]);
            pop = true;
          } else {
            ua = qc;
            ub = qc + 1;
            us = e + 1;
          }
        }
        if (pop) {
          if (sp == 0) break;
          MsgFrame& f = st[sp - 1];
          ua = f.cur;
          ub = ua + 1;
          us = b0 + f.s;
          if (++f.cur >= f.end) sp--;
        }
      }
    }
  };
  if (WIDE) {  // wavefront per exported item: its particles, lane by lane (dfs_run)
    const uint32_t ni = min(*w.n_items, w.cap);
    const uint32_t wbase = (blockIdx.x * 4 + wv) * w.per_wave;  // (wide count: this wavefront's scratch)
    for (uint32_t i = blockIdx.x * 4 + wv; i < ni; i += gridDim.x * 4) {
      const MsgWork it = w.items[i];
      t = it.t;
      b0 = fo[t];
      b1 = fo[t + 1];
      if (FILL && it.n_runs != kNone) {  // the count's runs, placed after the filter's own part
        obase = off[t].rows + it.dst;
        pbase = off[t].g + it.pslot;
        for (uint32_t k = lane; k < it.n_runs; k += 64) {
          const MsgRun r = w.scratch[(uint64_t)it.run_off + k];
          if (r.len > kMsgDirect) put_pieces(r.h0, r.len, r.dst, r.pslot);
          else
            for (uint32_t j = 0; j < r.len; j++) handles[obase + r.dst + j] = img.h[r.h0 + j];
        }
        continue;
      }
      uint32_t r0 = 0;
      if (lane == 0) {
        if (FILL) {
          hcur[wv] = it.dst;
          pcur[wv] = it.pslot;
        } else {
          hcur[wv] = pcur[wv] = 0;
          r0 = rcur[wv];
        }
      }
      if (FILL) {
        obase = off[t].rows;
        pbase = off[t].g;
      }
      wave_sync_lds();
      dfs_run(it.x, it.y, b0 + it.s);
      wave_sync_lds();
      if (!FILL && lane == 0) {  // the item's place in its filter's output: after the count pass's own part
        const uint32_t r1 = rcur[wv];
        w.items[i].dst = atomicAdd(&cnt[t].rows, hcur[wv]);
        w.items[i].pslot = atomicAdd(&cnt[t].gathers, pcur[wv]);
        w.items[i].run_off = wbase + r0;
        w.items[i].n_runs = r1 <= w.per_wave ? r1 - r0 : kNone;
      }
    }
    return;
  }
  bool exported = false;  // the count pass handed the filter's fan-out to work items (MsgWide)
  if (b1 > b0 && ix.retained_len != 0) {  // topics.go:535
    bool wild = false;
    for (uint64_t i = b0 + lane; i < b1; i += 64) {
      const uint32_t ch = fb[i];
      wild |= (ch == '+') | (ch == '#');
    }
    if (!__any(wild)) {  // Retained.Get(filter) (topics.go:539-544)
      uint32_t node = kRoot;
      SegKey key;
      uint64_t s = b0, e = scan_segment(R, b0, b1, &key);
      for (;;) {
        node = lookup(ix, node, key, fb + s, (uint32_t)(e - s));
        if (node == kNone || e >= b1) break;
        s = e + 1;
        e = scan_segment(R, s, b1, &key);
      }
      if (lane == 0 && node != kNone && (ix.msg[node].flags & kRetainLive)) {
        const uint32_t q = img_pos(img, node);
        if (q != kNone) emit(img.lp[q], 1u);
      }
    } else {
      // wave-uniform: the run [a, b) that segment s applies to, until a literal meets a longer run
      uint32_t a = 0, b = 1;
      uint64_t s = b0;
      bool fan = false;
      for (uint32_t guard = 0; guard < 4096; guard++) {
        const uint64_t e = find_slash(R, s, b1);
        const bool last = e >= b1;
        const uint32_t len = (uint32_t)(e - s);
        const uint32_t c0 = len == 1 ? R.at(s) : 0u;
        if (c0 == '+' || c0 == '#') {  // topics.go:547-565
          uint32_t x, y;
          desc(a, b, x, y);
          if (last) {
            if (lane == 0) emit_final(c0 == '#', x, y);
            break;
          }
          a = x;
          b = y;
          s = e + 1;
          if (a >= b) break;
          continue;
        }
        if (b - a > 1) {
          fan = true;
          break;
        }
        SegKey key = key_of(R, s, e);
        const uint32_t qc = img_pos(img, lookup(ix, img.node[a], key, fb + s, len));
        if (qc == kNone) break;
        if (last) {
          if (lane == 0) emit(img.lp[qc], img.lp[qc + 1] - img.lp[qc]);
          break;
        }
        a = qc;
        b = qc + 1;
        s = e + 1;
      }
      if (fan) {
        // A literal segment under a run of several particles. Level-synchronous fan-out: the
        // frontier is a list of runs [x, y) of one level, in LDS; every lane takes particles of
        // the same level, so a literal level's lookups are issued together with one key for the
        // wave, a '+' maps each run to its children's run, and a final '+' / '#' emits each run.
        // A frontier that outgrows its LDS falls back, run by run, to the per-lane walk
        // (dfs_run: lanes take a run's particles, each walks the rest of the filter alone with
        // deeper fan-outs on a frame stack).
        uint2* cur = mfront[wv][0];
        uint2* nxt = mfront[wv][1];
        uint32_t nr = 1;
        if (lane == 0) cur[0] = make_uint2(a, b);
        wave_sync_lds();
        uint64_t ls = s;  // the segment the frontier's runs take next
        for (uint32_t guard = 0; guard < 4096; guard++) {
          const uint64_t e = find_slash(R, ls, b1);
          const bool last = e >= b1;
          const uint32_t len = (uint32_t)(e - ls);
          const uint32_t c0 = len == 1 ? R.at(ls) : 0u;
          uint32_t nn = 0;  // the next frontier's runs (wave-uniform)
          if (c0 == '+' || c0 == '#') {
            for (uint32_t r0 = 0; r0 < nr; r0 += 64) {
              const uint32_t r = r0 + lane;
              uint32_t x = 0, y = 0;
              if (r < nr) {
                const uint2 ru = cur[r];
                desc(ru.x, ru.y, x, y);
              }
              if (last) {
                if (r < nr) emit_final(c0 == '#', x, y);
                continue;
              }
              const bool keep = r < nr && x < y;
              const uint64_t bk = __ballot(keep);
              const uint32_t at = nn + prefix_before(bk);
              if (keep && at < kMsgFront) nxt[at] = make_uint2(x, y);
              nn += (uint32_t)__popcll(bk);
            }
          } else {
            // literal: every particle of every run looks the segment up; particle p of the
            // frontier is found through the runs' prefix sums
            const SegKey key = key_of(R, ls, e);
            uint32_t tot = 0;
            for (uint32_t r0 = 0; r0 < nr; r0 += 64) {
              const uint32_t r = r0 + lane;
              const uint32_t v = r < nr ? cur[r].y - cur[r].x : 0u;
              uint32_t ct;
              const uint32_t ex = wave_excl_scan(v, lane, &ct);
              if (r < nr) mpre[wv][r] = tot + ex;
              tot += ct;
            }
            if (lane == 0) mpre[wv][nr] = tot;
            if (!FILL && img.work && lane == 0) atomicAdd(img.work + 0, (unsigned long long)tot);
            wave_sync_lds();
            if ((RUNS || MODE == kMsgFill || MODE == kMsgPlace) && w.min_tot && tot > w.min_tot) {
              if (FILL) {  // the count pass exported from here: its items write the rest
                if (cnt[t].shared) break;
              } else {
                // the runs as items of at most kMsgChunk particles (one reservation for all)
                uint32_t nit = 0;
                for (uint32_t r0 = 0; r0 < nr; r0 += 64) {
                  const uint32_t r = r0 + lane;
                  const uint32_t c = r < nr ? (cur[r].y - cur[r].x + kMsgChunk - 1) / kMsgChunk : 0u;
                  nit += wave_sum(c);
                }
                uint32_t ib = 0;
                if (lane == 0) ib = atomicAdd(w.n_items, nit);
                ib = __shfl(ib, 0, 64);
                if (ib + nit <= w.cap) {
                  for (uint32_t r0 = 0; r0 < nr; r0 += 64) {
                    const uint32_t r = r0 + lane;
                    uint32_t x = 0, y = 0;
                    if (r < nr) {
                      x = cur[r].x;
                      y = cur[r].y;
                    }
                    const uint32_t c = (y - x + kMsgChunk - 1) / kMsgChunk;
                    uint32_t ct;
                    const uint32_t ex = wave_excl_scan(c, lane, &ct);
                    for (uint32_t k = 0; k < c; k++)
                      w.items[ib + ex + k] = MsgWork{t, x + k * kMsgChunk, min(y, x + (k + 1) * kMsgChunk),
                                                     (uint32_t)(ls - b0), 0u, 0u, 0u, kNone};
                    ib += ct;
                  }
                  exported = true;
                  break;
                }  // (the queue is full: this filter walks alone, as a fill walk will)
              }
            }
            for (uint32_t p0 = 0; p0 < tot; p0 += 64) {
              const uint32_t p = p0 + lane;
              uint32_t qc = kNone;
              if (p < tot) {
                uint32_t lo = 0, hi = nr;  // mpre[lo] <= p < mpre[hi]
                while (hi - lo > 1) {
                  const uint32_t mid = (lo + hi) >> 1;
                  if (mpre[wv][mid] <= p) lo = mid;
                  else hi = mid;
                }
                const uint32_t u = cur[lo].x + (p - mpre[wv][lo]);
                qc = img_pos(img, lookup(ix, img.node[u], key, fb + ls, len));
              }
              if (last) {
                if (qc != kNone) emit(img.lp[qc], img.lp[qc + 1] - img.lp[qc]);
                continue;
              }
              const bool keep = qc != kNone;
              const uint64_t bk = __ballot(keep);
              const uint32_t at = nn + prefix_before(bk);
              if (keep && at < kMsgFront) nxt[at] = make_uint2(qc, qc + 1);
              nn += (uint32_t)__popcll(bk);
            }
          }
          if (last) break;
          if (nn > kMsgFront) {  // too wide for LDS: the per-lane walk from this level
            if (!FILL && img.work && lane == 0) {
              uint32_t np = 0;
              for (uint32_t r = 0; r < nr; r++) np += cur[r].y - cur[r].x;
              atomicAdd(img.work + 1, 1ull);
              atomicAdd(img.work + 2, (unsigned long long)np);
            }
            for (uint32_t r = 0; r < nr; r++) {
              const uint2 ru = cur[r];
              dfs_run(ru.x, ru.y, ls);
            }
            break;
          }
          wave_sync_lds();  // the next frontier is complete; the current one is free
          uint2* tmp = cur;
          cur = nxt;
          nxt = tmp;
          nr = nn;
          ls = e + 1;
          if (nr == 0) break;
        }
      }
    }
  }
  if (!FILL) {
    nh = wave_sum(nh);
    np = wave_sum(np);
    if (RUNS) wave_sync_lds();  // every lane's run reservations are in rcur
    if (lane == 0) {
      cnt[t] = TopicCount{np, nh, exported ? 1u : 0u, 0, 0};
      if (RUNS) n_runs[t] = rcur[wv] <= run_cap ? rcur[wv] : kNone;
      if (img.cyc) img.cyc[t] = (uint32_t)min((clock64() - c_start) >> 4, 0xFFFFFFFFull);
    }
  } else if (lane == 0) {
    base_out[t] = obase;
    count_out[t] = cnt[t].rows;
  }
}

void launch_msgq(int mode, const uint8_t* fb, const uint64_t* fo, uint32_t n, const DevIndex& ix,
                 const MsgImg& img, TopicCount* cnt, const TopicOff* off, MsgPiece* pieces,
                 uint64_t* handles, uint64_t* base, uint32_t* count, MsgRun* runs, uint32_t run_cap,
                 uint32_t* n_runs, const MsgWide& w, uint32_t wide_blocks, hipStream_t s) {
  if (!n) return;
  // the wide modes: persistent wavefronts over the items (their number is on the device)
  const dim3 g(mode == kMsgWideCount || mode == kMsgWideFill ? std::max(1u, wide_blocks) : (n + 3) / 4), b(256);
#define MQ_MSGQ(M) \
  hipLaunchKernelGGL(k_msgq<M>, g, b, 0, s, fb, fo, n, ix, img, cnt, off, pieces, handles, base, count, runs, run_cap, \
                     n_runs, w)
  switch (mode) {
    case kMsgCount: MQ_MSGQ(kMsgCount); break;
    case kMsgFill: MQ_MSGQ(kMsgFill); break;
    case kMsgRuns: MQ_MSGQ(kMsgRuns); break;
    case kMsgWideCount: MQ_MSGQ(kMsgWideCount); break;
    case kMsgWideFill: MQ_MSGQ(kMsgWideFill); break;
    default: MQ_MSGQ(kMsgPlace); break;
  }
#undef MQ_MSGQ
}

__global__ __launch_bounds__(256) void k_reset(ResetArgs a) {
  if (blockIdx.x == 0)
    for (uint32_t k = 0; k < a.n; k++) {
      uint32_t* p = static_cast<uint32_t*>(a.p[k]);
      for (uint32_t i = threadIdx.x; i < a.bytes[k] / 4; i += blockDim.x) p[i] = 0u;
    }
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.big_words; i += (uint64_t)gridDim.x * blockDim.x)
    a.big[i] = 0ull;
}

void launch_reset(const ResetArgs& a, hipStream_t s) {
  const uint64_t blocks = std::min<uint64_t>(std::max<uint64_t>(1, (a.big_words + 255) / 256), 2048);
  hipLaunchKernelGGL(k_reset, dim3((uint32_t)blocks), dim3(256), 0, s, a);
}

__global__ void k_readback(ReadbackArgs a) {
  if (threadIdx.x != 0) return;
  FastBackRec r;
  r.tot = a.tot ? *a.tot : TopicOff{0, 0, 0, 0, 0};
  r.ovf = *a.ovf;
  r.fallback = a.fallback ? *a.fallback : 0u;
  r.unsafe = *a.unsafe;
  r.err = *a.err;
  for (int k = 0; k < 3; k++) r.n_sets[k] = a.n_sets ? a.n_sets[k] : 0ull;
  *a.out = r;
  __threadfence_system();
}

void launch_readback(const ReadbackArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_readback, dim3(1), dim3(64), 0, s, a);
}

// Wavefront per piece: four 64-handle loads in flight per lane, then the stores.
__global__ __launch_bounds__(256) void k_msg_copy(const MsgPiece* __restrict__ pieces, uint64_t n,
                                                  const uint64_t* __restrict__ h, uint64_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t i = (uint64_t)blockIdx.x * 4 + wave_id(); i < n; i += (uint64_t)gridDim.x * 4) {
  const MsgPiece p = pieces[i];
  const uint64_t* src = h + p.h0;
  uint64_t* dst = out + p.dst;
  uint32_t k = lane;
  for (; k + 192 < p.len; k += 256) {
    const uint64_t v0 = src[k], v1 = src[k + 64], v2 = src[k + 128], v3 = src[k + 192];
    __builtin_nontemporal_store(v0, dst + k);
    __builtin_nontemporal_store(v1, dst + k + 64);
    __builtin_nontemporal_store(v2, dst + k + 128);
    __builtin_nontemporal_store(v3, dst + k + 192);
  }
  for (; k < p.len; k += 64) __builtin_nontemporal_store(src[k], dst + k);
  }
}

void launch_msg_copy(const MsgPiece* pieces, uint64_t n, const uint64_t* h, uint64_t* out, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_msg_copy, dim3((unsigned)std::min<uint64_t>((n + 3) / 4, kMaxWaveBlocks)), dim3(256), 0, s, pieces, n, h, out);
}

}  // namespace mq
