// gfx950 match walks: k_walk (thread per topic, stackless DFS) and k_walkf (16-lane frontier,
// k_desc fused), the TopicCount scans, k_desc / k_desc_g16.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "kern_common.h"

namespace mq {

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

// k_walk's parameters as they lie in the kernarg segment
struct WalkParams {
  const uint8_t* tb;
  const uint64_t* to;
  uint32_t n;
  DevIndex ix;
};

// list == null: thread per topic t < n. Else the topics list[0, *n_list), grid-stride (the
// frontier walk's fallback: its length is known on the device only).
template <bool FILL, bool LISTS, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_walk(const uint8_t* __restrict__ tb,
                                              const uint64_t* __restrict__ to, uint32_t n,
                                              DevIndex ix_, TopicCount* __restrict__ cnt,
                                              const TopicOff* __restrict__ off,
                                              uint32_t* __restrict__ gathers, uint32_t* __restrict__ ovf,
                                              const uint32_t* __restrict__ list, const uint32_t* __restrict__ n_list,
                                              bool clamp) {
  (void)ix_;
  const DevIndex& ix = kernarg_at<DevIndex>(offsetof(WalkParams, ix));
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


struct FrontEnt {  // one frontier particle: its '+' / '#' children and its path code
  uint32_t node, plus, hash, code;
};

// WPE: waves per SIMD asked of the register allocator (8: a few SGPRs spill to VGPR lanes; 1:
// no constraint, 7 waves).

// DESC (G = 16, LISTS = false): k_desc fused into the epilogue — the gathers, placed in the
// reference's order in LDS, go straight to the topic's spans and merge lists (desc_g16 with the
// stride layout, da.g_stride); neither the gather slots nor the counts are written.
// k_walkf's parameters as they lie in the kernarg segment (natural alignment, in order)
struct WalkfParams {
  const uint8_t* tb;
  const uint64_t* to;
  uint32_t n;
  DevIndex ix;
  TopicCount* cnt;
  uint32_t* gathers;
  uint32_t* fb_list;
  uint32_t* fb_count;
  DescArgs da;
};

template <uint32_t G, bool LISTS, int WPE, bool DESC = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_walkf(const uint8_t* __restrict__ tb, const uint64_t* __restrict__ to,
                                               uint32_t n, DevIndex ix, TopicCount* __restrict__ cnt,
                                               uint32_t* __restrict__ gathers, uint32_t* __restrict__ fb_list,
                                               uint32_t* __restrict__ fb_count, DescArgs da) {
  static_assert(!DESC || ((G == 16 || G == 8) && !LISTS), "the fused desc runs on 8- or 16-lane groups of a gathers-only walk");
  // the fused desc's arguments, read from the kernarg segment where the epilogue uses them: a
  // by-value parameter is loaded at the kernel's entry and held across the walk (~60 scalar
  // registers spilled to vector lanes, read back in the epilogue)
  const DescArgs& dk = kernarg_at<DescArgs>(offsetof(WalkfParams, da));
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
    nsl += grp_last<G>(inc);
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
    if (mine && !plusseg) {
      if (DESC && kDevBuild && dk.root_hint && d < dk.hint_levels) {  // (MQ_OPT_WALK_EXP: looked up before the walk)
        // level 0: the root's child; level 1 (bit 1): the literal child of the root's literal or
        // '+' child, by how the frontier entry's path starts
        const uint32_t k = dk.hint_levels == 1 ? t : 3 * t + (d == 0 ? 0u : (fe.code >> 30) == 1u ? 1u : 2u);
        const uint4 rh = dk.root_hint[k];
        h = EdgeHit{rh.x, rh.y, rh.z};
      } else {
        h = lookup_edge(ix, fe.node, key, tbase + s, len);
      }
    }
    // this lane's gathers (at most four): the particle's '#' child (topics.go:621); at the last
    // level the literal child, its '#' child (filter/# matches filter, topics.go:612; inline: the
    // particle's own again, Q2) and the '+' child
    const bool gH = mine && fe.hash != kNone;
    const bool gL = mine && !has_next && h.child != kNone;
    const bool gC = gL && h.hash != kNone;
    const bool gP = mine && !has_next && fe.plus != kNone;
    const uint32_t gc = (uint32_t)gH + (uint32_t)gL + (uint32_t)gC + (uint32_t)gP;
    // next level's frontier: the literal and '+' children, compacted over the group
    const bool fL = mine && has_next && h.child != kNone;
    const bool fP = mine && has_next && fe.plus != kNone;
    const uint32_t fc = (uint32_t)fL + (uint32_t)fP;
    // one group scan for both counts (at most 4 and 2 a lane: 16 bits each)
    const uint32_t gfi = grp_incl<G>(gc | fc << 16, sub);
    const uint32_t gft = grp_last<G>(gfi);
    const uint32_t gi = gfi & 0xFFFFu, gtot = gft & 0xFFFFu, fi = gfi >> 16, ftot = gft >> 16;
    if (act && ng + gtot > kStage) fb = true;
    if (act && !fb) {
      uint32_t p = ng + gi - gc;
      if (gH) gat[q][p++] = make_uint2(fe.hash | kGatherInline, fe.code | 3u << sh);
      if (gL) gat[q][p++] = make_uint2(h.child | kGatherInline, fe.code | 1u << sh);
      if (gC) gat[q][p++] = make_uint2(h.hash, fe.code | 1u << sh | 3u << (sh - 2));
      if (gP) gat[q][p++] = make_uint2(fe.plus | kGatherInline, fe.code | 2u << sh);
    }
    ng += gtot;
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
    desc_grp<G>(dk, t, ng, (uint64_t)t * dk.g_stride, 0ull, 0u, sub, [&](uint32_t i) { return gat[q][i].x; });
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
  // the product build: 16 lanes per topic at 8 waves per SIMD; narrower groups and other register
  // budgets (MQ_OPT_WALK_GROUP 8 / 4, MQ_OPT_WALK_WAVES) are measurement variants (DEV=1)
#define MQ_WALKF(G, L) \
  hipLaunchKernelGGL((k_walkf<G, L, 8>), grid, dim3(256), 0, s, tb, to, n, ix, cnt, gathers, fb_list, fb_count, nd)
  if (group == 16 && (!kDevBuild || wpe >= 8)) {
    if (lists) MQ_WALKF(16, true);
    else MQ_WALKF(16, false);
  }
#ifdef MQ_DEV_BUILD
  else {  // (narrower groups: more topics per workgroup, so LDS bounds them below 8 waves)
#define MQ_WALKF1(G, L) \
  hipLaunchKernelGGL((k_walkf<G, L, 1>), grid, dim3(256), 0, s, tb, to, n, ix, cnt, gathers, fb_list, fb_count, nd)
    if (group == 8) {
      if (lists) MQ_WALKF1(8, true);
      else MQ_WALKF1(8, false);
    } else if (group == 4) {
      if (lists) MQ_WALKF1(4, true);
      else MQ_WALKF1(4, false);
    } else {
      if (lists) MQ_WALKF1(16, true);
      else MQ_WALKF1(16, false);
    }
#undef MQ_WALKF1
  }
#endif
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
#ifdef MQ_DEV_BUILD
  if (group == 8)
    hipLaunchKernelGGL((k_walkf<8, false, 8, true>), dim3((n + 31) / 32), dim3(256), 0, s, tb, to, n, ix, cnt, gathers,
                       fb_list, fb_count, da);
  else if (wpe < 8)
    hipLaunchKernelGGL((k_walkf<16, false, 1, true>), dim3((n + 15) / 16), dim3(256), 0, s, tb, to, n, ix, cnt, gathers,
                       fb_list, fb_count, da);
  else
#else
  (void)group;
  (void)wpe;
#endif
    hipLaunchKernelGGL((k_walkf<16, false, 8, true>), dim3((n + 15) / 16), dim3(256), 0, s, tb, to, n, ix, cnt, gathers,
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

// MQ_OPT_WALK_EXP bit 0 (development builds): each topic's level-0 probe (the root's literal
// child of its first segment), thread per topic, ahead of the walk — the walk then reads it instead
// of probing, so the two kernels' times attribute the level-0 probes (the north star's "hot trie
// levels staged in LDS" would save at most that much)
// Bit 1 (round 6): levels 0 and 1 — also the level-1 probes of the frontier's two possible
// entries (the root's literal child and its '+' child), so that the walk's time without them bounds
// staging both hot levels in LDS.
__global__ __launch_bounds__(256) void k_root_hint(const uint8_t* __restrict__ tb, const uint64_t* __restrict__ to,
                                                   uint32_t n, DevIndex ix, uint4* __restrict__ out, uint32_t levels) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint64_t a0 = to[t], a1 = to[t + 1];
  const uint8_t* tbase = tb + (a0 & ~15ull);
  const uint32_t b0 = (uint32_t)(a0 & 15), b1 = b0 + (uint32_t)(a1 - a0);
  EdgeHit h{kNone, kNone, kNone}, hl{kNone, kNone, kNone}, hp{kNone, kNone, kNone};
  if (a1 > a0) {
    ByteReaderT<uint32_t> R(tbase);
    const uint32_t e = find_slash(R, b0, b1);
    const bool plusseg = e - b0 == 1 && R.at(b0) == '+';
    if (!plusseg) h = lookup_edge(ix, kRoot, key_of(R, b0, e), tbase + b0, e - b0);
    if (levels > 1 && e < b1) {
      const uint32_t s1 = e + 1, e1 = find_slash(R, s1, b1);
      const bool plus1 = e1 - s1 == 1 && R.at(s1) == '+';
      if (!plus1) {
        const SegKey k1 = key_of(R, s1, e1);
        if (h.child != kNone) hl = lookup_edge(ix, h.child, k1, tbase + s1, e1 - s1);
        const uint32_t rp = ix.walk[kRoot].plus_child;
        if (rp != kNone) hp = lookup_edge(ix, rp, k1, tbase + s1, e1 - s1);
      }
    }
  }
  if (levels > 1) {
    out[3 * t] = make_uint4(h.child, h.plus, h.hash, 0u);
    out[3 * t + 1] = make_uint4(hl.child, hl.plus, hl.hash, 0u);
    out[3 * t + 2] = make_uint4(hp.child, hp.plus, hp.hash, 0u);
  } else {
    out[t] = make_uint4(h.child, h.plus, h.hash, 0u);
  }
}

void launch_root_hint(const uint8_t* tb, const uint64_t* to, uint32_t n, const DevIndex& ix, uint4* out, uint32_t levels,
                      hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_root_hint, dim3((n + 255) / 256), dim3(256), 0, s, tb, to, n, ix, out, levels);
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

}  // namespace mq
