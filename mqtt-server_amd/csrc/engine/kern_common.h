// Device-side helpers shared by the gfx950 kernel files: the byte reader and
// SWAR segment scanning over topic buffers, segment keys, edge lookups, wave / group scans, the
// TopicCount scan arithmetic, and the per-topic desc (desc_grp), which both k_desc_g16 and the
// walk-fused k_walkf<..., DESC> run. Included by
//   walk.hip   the match walks (k_walk thread per topic, k_walkf frontier), scans, k_desc
//   merge.hip  merge-set dedup, the merge set and topic passes (k_merge), result packing, k_copy
//   msg.hip    Messages (the level-order image, k_msgq, the particle walk k_msg)
//   misc.hip   k_acl, k_pick, cross-shard export, staging scatter, batch reset / readback
#pragma once

#include <hip/hip_runtime.h>

#include "kernels.h"

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
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {  // lanes whose source is outside the row read 0
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
// (DPP: rows' prefix sums by row_shr, then row 0's total into rows 1 and 3 by row_bcast:15 and
// rows 0-1's into rows 2 and 3 by row_bcast:31; the total is lane 63's, read as a scalar)
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t lane, uint32_t* total) {
  (void)lane;
  uint32_t x = v;
  x += dpp<0x111>(x);
  x += dpp<0x112>(x);
  x += dpp<0x114>(x);
  x += dpp<0x118>(x);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
  *total = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
  return x - v;
}

// inclusive u32 scan over a 256-thread workgroup (wt: 4 words of LDS)
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

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int d = 32; d; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// A kernel parameter read from the kernarg segment where it is used. A by-value parameter (the
// 200-byte DevIndex, an argument struct) is loaded whole at the kernel's entry and its pointers
// held across the kernel, spilling scalar registers to vector lanes (v_readlane, a VALU
// instruction, in the hot loops); read through this reference, each field is loaded (s_load)
// where it is used. P: the kernel's parameters as a struct (same order: kernarg layout is the
// struct's, natural alignment), OFF: offsetof(P, the parameter).
template <class T>
__device__ __forceinline__ const T& kernarg_at(size_t off) {
  return *(const T*)((const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr() + off);
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
  uint64_t i = edge_slot(parent, k, ix.edge_mask);
  for (uint64_t probes = 0; probes <= ix.edge_mask; probes++) {
    // both halves of the slot in one round trip: left to itself the compiler loads the key half
    // only once the parent half has shown a full slot — a second, dependent load on every hit
    const uint4* sp = reinterpret_cast<const uint4*>(ix.edges + i);
    const uint4 q0 = sp[0], q1 = sp[1];
    __asm__ volatile("" ::"v"(q0.x), "v"(q1.x));
    const EdgeSlot e{q0.x | (uint64_t)q0.y << 32, q0.z | (uint64_t)q0.w << 32, q1.x, q1.y, q1.z, q1.w};
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

// Group collectives. A 16-lane group is a DPP row (8 lanes: half a row), so its prefix sums and
// sums are DPP moves folded into the adds — no LDS traffic, no lane-index arithmetic, no wait — and
// the broadcast of its last lane one ds_swizzle; other widths go through ds_bpermute (__shfl).
template <uint32_t G, int D = 1>
__device__ __forceinline__ uint32_t grp_incl_dpp(uint32_t v, uint32_t sub) {
  if constexpr (D >= (int)G) {
    return v;
  } else {
    const uint32_t y = dpp<0x110 + D>(v);  // row_shr:D
    if (G == 16 || sub >= (uint32_t)D) v += y;  // (8-lane groups: not across the group)
    return grp_incl_dpp<G, 2 * D>(v, sub);
  }
}
// Inclusive prefix sum over the G lanes of a group (G a power of two <= 64; sub = lane % G).
template <uint32_t G>
__device__ __forceinline__ uint32_t grp_incl(uint32_t v, uint32_t sub) {
  if constexpr (G == 16 || G == 8) {
    return grp_incl_dpp<G>(v, sub);
  } else {
#pragma unroll
    for (uint32_t d = 1; d < G; d <<= 1) {
      const uint32_t y = __shfl_up(v, d, G);
      if (sub >= d) v += y;
    }
    return v;
  }
}
// lane G-1's value, to every lane of the group (ds_swizzle bit mode: lane (lane & and) | or)
template <uint32_t G>
__device__ __forceinline__ uint32_t grp_last(uint32_t v) {
  if constexpr (G == 16 || G == 8) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (32 - G) | (G - 1) << 5);
  else return __shfl(v, G - 1, G);
}
template <uint32_t G>
__device__ __forceinline__ uint32_t grp_sum(uint32_t v) {
  if constexpr (G == 16 || G == 8) {
    v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]: quad sums
    v += dpp<0x141>(v);  // row_half_mirror: 8-lane sums
    if (G == 16) v += dpp<0x140>(v);  // row_mirror
    return v;
  } else {
#pragma unroll
    for (uint32_t d = 1; d < G; d <<= 1) v += __shfl_xor(v, d, G);
    return v;
  }
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
  return (uint64_t)dpp<CTRL>((uint32_t)v) | (uint64_t)dpp<CTRL>((uint32_t)(v >> 32)) << 32;
}
template <uint32_t G>
__device__ __forceinline__ uint64_t grp_sum64(uint64_t v) {
  if constexpr (G == 16 || G == 8) {
    v += dpp64<0xB1>(v);
    v += dpp64<0x4E>(v);
    v += dpp64<0x141>(v);
    if (G == 16) v += dpp64<0x140>(v);
    return v;
  } else {
#pragma unroll
    for (uint32_t d = 1; d < G; d <<= 1) v += __shfl_xor(v, d, G);
    return v;
  }
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
  for (int d = 32; d; d >>= 1) v = max(v, (uint32_t)__shfl_xor(v, d, 64));
  return v;
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


// 16-lane inclusive scan (lanes of a 16-lane group of the wavefront; sub = lane & 15)
__device__ __forceinline__ uint32_t g16_incl(uint32_t v, uint32_t sub) { return grp_incl<16>(v, sub); }

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
  uint32_t rpos = 0, spos = 0, n_mg = 0, n_merge = 0, n_x = 0;
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
    if (act && fits && a.gw_out) a.gw_out[g0 + i] = gw;
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
    if (a.xents) {  // sharded: the export (a gathered node whose subscriptions have a foreign partner)
      const bool isx = subs && (L.flags & kFlagXNode);
      const uint32_t xi = grp_incl<G>(isx ? 1u : 0u, sub);
      if (isx && fits) {
        const XInfo xn = a.ix.xinfo[gw & kGatherNode];
        a.xents[g0 + n_x + xi - 1] = XEnt{xn.fid, xn.deep, xn.rank};
      }
      n_x += grp_last<G>(xi);
    }
    rpos += grp_last<G>(rn_i);
    spos += grp_last<G>(sh_i);
    ipos += grp_last<G>(in_i);
    n_mg += grp_last<G>(inc_i);
  }
  sig = grp_sum64<G>(sig);
  n_merge = grp_sum<G>(n_merge);
  const unsigned long long msig = mix64(sig + n_mg) | 1ull;  // never 0 (the dedup table's empty key)
  if (a.dd_keys) {  // k_dedup_insert's work, one lane per topic
    const uint32_t slot = dedup_insert(a.dd_keys, a.dd_vals, a.dd_mask, t, sub == 0 && n_mg != 0 && n_mg <= kPairMax,
                                       msig);
    if (sub == 0) a.dd_tslot[t] = slot;
  }
  if (sub != 0) return;
  if (a.xcount) a.xcount[t] = n_x;
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

}  // namespace mq
