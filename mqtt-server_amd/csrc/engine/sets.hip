// gfx950 merge set pass, k_set: one wavefront per merge set of an index that is
// not sharded. The set pass of k_merge<spans, SET> holds the code of every k_merge path (the
// topic pass, the GDesc map, the linear lookups beyond the pair analysis, the sharded rank keys),
// and its wave-uniform state outgrew the scalar registers: ~180 SGPRs spilled to vector lanes and
// read back (v_readlane) all through the hot loops. On MI355X the pass was bound by instruction
// issue, not by memory: 2,750 VALU and 2,720 SALU wave-instructions per set (SQ counters,
// profiles/r05/pmcset/), the scalar unit ~67 % busy. k_set keeps only what a merge set needs — a
// set has 1..kPairMax merge gathers (k_dedup_insert admits no other), so its map is always the
// dedup lists' and the pair analysis always covers it — and its results are k_merge's exactly
// (Subscription.Merge, packets/packets.go:254-274, over gatherSubscriptions' order,
// topics.go:631-648).
#include <hip/hip_runtime.h>

#include "kern_common.h"

namespace mq {

// XS (a sharded index, round 5): a set's entries are its merge gathers and then the other shards'
// exported nodes of its representative (kForeign | fid, with their rank keys), the pair analysis
// covers pairs (merge gather, any entry), and DFS order between an entry of another shard and a
// merge gather here is the rank keys' (k_merge<spans, XS, SET>'s results; an index with filters
// deeper than 32 levels, whose keys can tie, keeps k_merge).
template <int WPE, bool XS = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_set(EmitArgs args) {
  // the arguments, read from the kernarg segment where they are used: a by-value parameter is
  // loaded whole at the kernel's entry, and its ~40 pointers and counts held across the kernel
  // spill to vector lanes (read back with v_readlane, a VALU instruction, in the hot loops)
  (void)args;
  const EmitArgs& a = kernarg_at<EmitArgs>(0);
  // per-wave LDS, one contiguous block: the node -> merge-gather map (links path only; the folds
  // use its words as their table, the record-keyed fold all kWsWords), then the merge gathers'
  // pair-block headers
  constexpr uint32_t kWsWords = 2 * kMapSlots + 3 * kPairMax;
  static_assert(kBigSlots <= kWsWords, "the record-keyed fold's table must fit the wave's words");
  // the record-keyed fold's table: the wave's words and kSetBigExtra more (eight workgroups of
  // four waves still fit a CU's 160 KB of LDS; XS, with its rank keys, six), so gathers of up to
  // kSetBigFill visits fold instead of resolving through their partner links
  constexpr uint32_t kSetBigExtra = 192;
  constexpr uint32_t kSetBigSlots = kWsWords + kSetBigExtra;
  constexpr uint32_t kEnt = XS ? kMapSlots : kPairMax;  // entries: merge gathers (+ XS: other shards' nodes)
  constexpr uint32_t kSetBigFill = kSetBigSlots * 3 / 4;
  // the hash fold's table: key and value words over the same block
  constexpr uint32_t kSetFoldSlots = (kSetBigSlots / 2) & ~63u;
  constexpr uint32_t kSetFoldCap = kSetFoldSlots * 2 / 3;
  static_assert(2 * kSetFoldSlots <= kSetBigSlots && kSetFoldSlots >= kFoldSlots, "the hash fold's table must fit the block");
  struct WaveLds {  // (one block per wave: every array an immediate offset from one base)
    uint32_t ws[kWsWords];
    uint32_t ws_big[kSetBigExtra];  // (contiguous with ws: the record-keyed fold's table continues here)
    uint32_t node[kEnt];         // entry x's particle: merge gathers in gather order (= DFS order), then
                                 //   (XS) other shards' nodes as kForeign | fid
    uint64_t rank[XS ? kEnt : 1];  // (XS) entry x's rank key
    uint32_t ga[kHitMax];        // staged hit lists (g, h): g's merge gather,
    uint32_t off[kHitMax];       //   the list's offset in the pair-list pool,
    uint32_t hb[kHitMax];        //   h's merge gather,
    uint32_t pre[kHitMax + 1];   //   exclusive prefix of the lists' lengths (+ total)
    uint8_t mark[64];            // locate_run: the list starts inside a window of 64 visits
  };
  __shared__ WaveLds lds[4];
  const uint32_t wv = wave_id(), lane = threadIdx.x & 63;
  WaveLds& W = lds[wv];
  uint32_t* const ws = W.ws;
  uint32_t* const map_key = ws;               // [kMapSlots]
  uint32_t* const map_val = ws + kMapSlots;   // [kMapSlots]
  uint32_t* const ent_off = ws + 2 * kMapSlots;              // [kPairMax]
  uint32_t* const ent_mask = ent_off + kPairMax;             // [kPairMax]
  uint32_t* const mg_node = W.node;
  uint32_t* const h_ga = W.ga;
  uint32_t* const h_off = W.off;
  uint32_t* const h_hb = W.hb;
  uint32_t* const h_pre = W.pre;
  const uint32_t exp_bits = kDevBuild ? a.exp : (a.exp & (256u | 512u | 1024u | 2048u | 16384u | 32768u | 65536u | 131072u));
  const bool small_fold = (exp_bits & 32768u) != 0;  // (MQ_OPT_SET_EXP bit 15: k_merge's 128-slot fold)
  const bool dense_fold = (exp_bits & 65536u) != 0;  // (bit 16: the hash fold up to 3/4 full, not 2/3)
  const bool sparse_fold = (exp_bits & 131072u) != 0;  // (bit 17: up to 3/5 full)
  const DevIndex& ix = a.ix;
  const uint32_t n_front = (uint32_t)a.n_reps[0];
  const uint32_t i_end = n_front + (uint32_t)a.n_reps[1];
  for (uint32_t i = blockIdx.x * 4 + wv; i < i_end; i += gridDim.x * 4) {
    // heavy sets from the front of the list, the others from its back (k_dedup_rep)
    const uint32_t t = i < n_front ? a.rep_list[i] : a.rep_list[a.t1 - 1 - (i - n_front)];
    const bool stamp = a.work != nullptr;
    const uint64_t c_start = stamp ? clock64() : 0ull;
    uint32_t w_ent = 0, w_rec = 0, w_link = 0;
    // --- the merge gathers (the dedup lists of k_desc, 1..kPairMax of them) ---------------------
    const uint32_t lc = a.mcount[t];
    if (lane < lc) {
      const uint64_t k = (uint64_t)t * kPairMax + lane;
      const uint2 P = a.mpair[k];
      mg_node[lane] = a.mlist[k];
      ent_off[lane] = P.x;
      ent_mask[lane] = P.y;
      if (XS) W.rank[lane] = a.mrank[k];
    }
    uint32_t n_ent = lc;  // (XS: the other shards' nodes of the set join as entries lc..; k_dedup
                          //  admitted the set only if they fit the map: n_ent < kMapSlots)
    for (uint32_t f = 0; XS && f < a.n_xf; f++) {
      const XSrc src = a.xsrc[f];
      const uint32_t x0 = src.xoff[t], x1 = src.xoff[t + 1];
      for (uint32_t k0 = x0; k0 < x1; k0 += 64) {
        const uint32_t k = k0 + lane, x = n_ent + (k - x0);
        if (k < x1 && x < kEnt) {
          const XEnt e = src.xent[k];
          mg_node[x] = kForeign | e.fid;
          W.rank[x] = e.rank;
        }
      }
      n_ent += x1 - x0;
    }
    wave_sync_lds();
    // does entry xh come before the set's merge gather xg in DFS order?
    auto before = [&](uint32_t xh, uint32_t xg) __attribute__((always_inline)) -> bool {
      if constexpr (!XS) {
        return xh < xg;
      } else {
        if (xh < lc) return xh < xg;  // both merge gathers here: gather order is DFS order
        const uint64_t rh = W.rank[xh], rg = W.rank[xg];
        if (rh != rg) return rh < rg;
        atomicOr(ix.err, kErrDeepRank);  // (not reached: an index with deep filters runs k_merge)
        return false;
      }
    };
    const uint64_t c_map = stamp ? clock64() : 0ull;
    // --- the patch range, reserved once the visits are counted -----------------------------------
    unsigned long long resv = 0;
    uint64_t resv_n = 0, pbase = 0;
    bool resv_pending = false, pfit = true;
    uint32_t n_patch = 0, n_nonbase = 0, n_ext = 0;
    auto settle = [&]() __attribute__((always_inline)) {
      if (resv_pending) {
        const unsigned long long b = __shfl(resv, 0, 64);
        pfit = b + resv_n <= a.srcap;
        if (!pfit && a.unsafe && lane == 0) atomicOr(a.unsafe, kUnsafePatches);
        pbase = (uint64_t)(t & (kPatchRegions - 1)) * a.srcap + b;
        resv_pending = false;
      }
    };
    auto emit_patch = [&](bool want, uint32_t row, uint32_t meta) __attribute__((always_inline)) {
      settle();
      const uint64_t m = __ballot(want);
      if (want && pfit) a.spatches[pbase + n_patch + prefix_before(m)] = PatchRec{row, meta};
      n_patch += (uint32_t)__popcll(m);
    };
    // --- pair analysis: ordered pairs (g, h), g a merge gather and h an entry; g's pair block lists
    // the slots whose client also subscribes at h. p = g * ne + h, g by a multiply: (p * inv) >> 24
    // == p / ne for p < 2^24 / ne (p < 64 * 127)
    const uint32_t ne = XS ? n_ent : lc;
    const uint32_t np = lc * ne;
    const uint32_t inv = (1u << 24) / ne + 1u;
    uint32_t n_hit = 0, tot = 0;
    uint64_t tot_all = 0;
    bool staged_all = true;
    auto pairs = [&](bool counting, auto&& flush) __attribute__((always_inline)) {
      for (uint32_t p0 = 0; p0 < np; p0 += 64) {
        const uint32_t p = p0 + lane;
        bool hit = false;
        uint32_t ga = 0, hb = 0, e_off = 0, e_cnt = 0;
        if (p < np) {
          ga = (p * inv) >> 24;
          hb = p - ga * ne;
          const uint32_t mask = ent_mask[ga];
          if (ga != hb && mask != kNone) {
            const uint32_t hn = mg_node[hb], eo = ent_off[ga];
            uint32_t sl = pair_hash(hn) & mask;
            for (uint32_t probes = 0; probes <= mask; probes += 4) {  // four slots per load round
              PairEnt pe[4];
#pragma unroll
              for (uint32_t u = 0; u < 4; u++) pe[u] = ix.pent[eo + ((sl + u) & mask)];
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
              sl = (sl + 4) & mask;
            }
          }
        }
        const uint64_t bh = __ballot(hit);
        const uint32_t nh = (uint32_t)__popcll(bh);
        uint32_t ct;
        const uint32_t cp = wave_excl_scan(hit ? e_cnt : 0u, lane, &ct);
        if (counting) {
          tot_all += ct;
          if (!staged_all || n_hit + nh > kHitMax) {  // wave-uniform
            staged_all = false;
            continue;
          }
        } else if (n_hit + nh > kHitMax) {
          flush();
        }
        if (hit) {
          const uint32_t x = n_hit + prefix_before(bh);
          h_ga[x] = ga;
          h_off[x] = e_off;
          h_hb[x] = hb;
          h_pre[x] = tot + cp;
        }
        n_hit += nh;
        tot += ct;
      }
    };
    // the visits [R, R + 64) of the staged lists [., j1), jb the list holding visit R, a lane
    // each: lane l reads list jb + 1 + l's start, the starts inside the window are marked in LDS,
    // and visit R + v's list is jb + the marks at or below v (lists are non-empty: one start per
    // place) — locate's result for 64 consecutive visits in two dependent LDS round trips where
    // the binary search takes log2(j1 - j0). jb_next: the list holding visit R + 64.
    auto locate_run = [&](uint32_t R, uint32_t jb, uint32_t j1, uint32_t& jj, uint32_t& jb_next)
        __attribute__((always_inline)) -> PairSlot {
      const uint32_t jl = jb + 1 + lane;
      const uint32_t pos = (jl < j1 ? h_pre[jl] : 0xFFFFFFFFu) - R;  // >= 1: list jb holds R
      W.mark[lane] = 0;
      if (pos < 64) W.mark[pos] = 1;
      wave_sync_lds();
      const uint64_t M = __ballot(W.mark[lane] != 0);
      jb_next = jb + (uint32_t)__popcll(__ballot(pos <= 64));
      jj = jb + (uint32_t)__popcll(M & (~0ull >> (63 - lane)));
      const uint32_t rc = min(R + lane, h_pre[j1] - 1);
      return ix.plist[h_off[jj] + (rc - h_pre[jj])];
    };
    // --- the partner-link path (a merge gather beyond the folds, or hit lists beyond the stage) --
    bool map_ok = false;
    auto map_rebuild = [&]() __attribute__((always_inline)) {
      for (uint32_t q = lane; q < kMapSlots; q += 64) map_key[q] = kNone;
      wave_sync_lds();
      for (uint32_t x = lane; x < n_ent; x += 64) {
        const uint32_t node = mg_node[x];
        uint32_t sl = hash32(node) & (kMapSlots - 1);
        while (atomicCAS(&map_key[sl], kNone, node) != kNone) sl = (sl + 1) & (kMapSlots - 1);
        map_val[sl] = x;
      }
      wave_sync_lds();
      map_ok = true;
    };
    auto gathered = [&](uint32_t h) __attribute__((always_inline)) -> uint32_t {  // its x, or kNone
      uint32_t sl = hash32(h) & (kMapSlots - 1);
      for (;;) {
        const uint32_t k = map_key[sl];
        if (k == h) return map_val[sl];
        if (k == kNone) return kNone;
        sl = (sl + 1) & (kMapSlots - 1);
      }
    };
    // a record resolved through its partner links (k_merge's resolve, one shard): the visit through
    // its first gathered partner (via) counts it; an earlier partner makes it a non-base entry,
    // else it is the merge base with the partners' max Qos and OR'd NoLocal
    auto resolve = [&](bool active, uint32_t mw, uint32_t row, uint32_t gx, uint32_t via, uint32_t mp_off,
                       uint32_t mp_cnt) __attribute__((always_inline)) {
      bool counted = false, nonbase = false, want = false;
      uint32_t pmeta = 0;
      if (active) {
        const uint32_t rmeta = mw & kSlotMetaMask;
        const bool idpos = (mw & kSlotIdentPos) != 0;
        bool bound = false, base = true, other = false;
        uint32_t first = kNone;
        uint32_t q = rmeta & kMetaQos, nl = rmeta & kMetaNoLocal;
        for (uint32_t e0 = 0; e0 < mp_cnt && base && !other; e0 += kPartBatch) {
          MergePart pb[kPartBatch];
#pragma unroll
          for (uint32_t u = 0; u < kPartBatch; u++)
            pb[u] = e0 + u < mp_cnt ? ix.mpart[mp_off + e0 + u] : MergePart{kNone, 0};
          w_link += min(kPartBatch, mp_cnt - e0);
#pragma unroll
          for (uint32_t u = 0; u < kPartBatch; u++) {
            if (!base || other || pb[u].node == kNone) continue;
            const uint32_t hx = gathered(pb[u].node);
            if (hx == kNone) continue;
            if (!bound) {
              first = pb[u].node;
              other = first != via;
            }
            bound = true;
            if (before(hx, gx)) {
              base = false;
              continue;
            }
            q = max(q, pb[u].meta & kMetaQos);
            nl |= pb[u].meta & kMetaNoLocal;
          }
        }
        if (bound) {
          counted = via == first;
          nonbase = !base;
          pmeta = base ? (rmeta & ~(kMetaQos | kMetaNoLocal)) | q | nl : rmeta | (idpos ? kRowIdent : kRowDrop);
          want = counted && pmeta != rmeta;
        }
      }
      emit_patch(want, row, pmeta);
      n_nonbase += (uint32_t)__popcll(__ballot(counted && nonbase));
      n_ext += (uint32_t)__popcll(__ballot(counted && nonbase && (pmeta & kRowIdent)));
    };
    // (pp, PP): only the records with hash32(k) % PP == pp
    auto resolve_lists = [&](uint32_t j0, uint32_t j1, uint32_t pp, uint32_t PP) __attribute__((always_inline)) {
      if (!map_ok) map_rebuild();
      const uint32_t v0 = h_pre[j0], v1 = h_pre[j1];
      uint32_t jj_next, jb = j0;
      PairSlot e_next = locate_run(v0, jb, j1, jj_next, jb);
      for (uint32_t r0 = v0; r0 < v1; r0 += 64) {
        const uint32_t r = r0 + lane;
        const uint32_t jj = jj_next;
        const PairSlot e = e_next;
        if (r0 + 64 < v1) e_next = locate_run(r0 + 64, jb, j1, jj_next, jb);  // wave-uniform
        const uint32_t xa = h_ga[jj];
        w_rec += r < v1;
        resolve(r < v1 && (PP == 1 || hash32(e.k) % PP == pp), e.meta, xa << kSetRowBits | e.k, xa,
                mg_node[h_hb[jj]], e.mp_off, e.mp_cnt);
      }
    };
    // --- the folds: a record's visits are exactly its gathered partners (one per hit list (g, h)
    // holding it), and each pair slot carries the partner's Qos / NoLocal, so no partner link is
    // read: the record is a non-base entry iff a visit's h comes before g, else the base with the
    // max Qos and OR'd NoLocal over its visits (k_merge's fold_lists / fold_big) ---------------------
    // small: lists [j0, j1) of whole merge gathers, at most kSetFoldCap visits, keyed x << 26 | k,
    // keys and values over the wave's whole block (the pair analysis is done with it), the table
    // sized to the chunk's visits (at most 2/3 full) so its clear and emission scan are too:
    // fewer, larger chunks, each paying its first pair-slot load's latency once
    auto fold_lists = [&](uint32_t j0, uint32_t j1) __attribute__((always_inline)) {
      const uint32_t v0 = h_pre[j0], v1 = h_pre[j1];
      const uint32_t nv = v1 - v0;
      const uint32_t ns = small_fold ? kFoldSlots : min(kSetFoldSlots, ((dense_fold ? nv * 4 / 3 : sparse_fold ? nv * 5 / 3 : nv * 3 / 2) + 63) & ~63u);
      uint32_t* __restrict__ f_key = ws;
      uint32_t* __restrict__ f_val = ws + ns;
      for (uint32_t q = lane; q < ns; q += 64) {
        f_key[q] = kNone;
        f_val[q] = 0;
      }
      map_ok = false;
      uint32_t jj_next, jb = j0;
      PairSlot e_next = locate_run(v0, jb, j1, jj_next, jb);
      wave_sync_lds();
      for (uint32_t r0 = v0; r0 < v1; r0 += 64) {
        const uint32_t r = r0 + lane;
        const uint32_t jj = jj_next;
        const PairSlot e = e_next;
        if (r0 + 64 < v1) e_next = locate_run(r0 + 64, jb, j1, jj_next, jb);  // wave-uniform
        if (r < v1) {
          const uint32_t xa = h_ga[jj], hb = h_hb[jj];
          const uint32_t key = xa << kSetRowBits | e.k;
          uint32_t sl = __umulhi(hash32(key), ns);
          for (;;) {
            const uint32_t prev = atomicCAS(&f_key[sl], kNone, key);
            if (prev == kNone || prev == key) break;
            sl = sl + 1 == ns ? 0u : sl + 1;
          }
          const uint32_t pm = e.meta >> kSlotPartShift;  // the partner's Qos | NoLocal << 2
          atomicOr(&f_val[sl], (e.meta & kSlotOwnMask) | (before(hb, xa) ? kFoldNonBase : 0u) |
                                   ((pm & 4u) ? kFoldNoLocal : 0u) | (kFoldQos0 << (pm & 3u)));
        }
        w_rec += r < v1;
      }
      wave_sync_lds();
      for (uint32_t s0 = 0; s0 < ns; s0 += 64) {
        const uint32_t key = f_key[s0 + lane], v = f_val[s0 + lane];
        const bool occ = key != kNone;
        const uint32_t rmeta = v & kSlotMetaMask;
        const bool nonbase = occ && (v & kFoldNonBase);
        uint32_t pmeta;
        if (v & kFoldNonBase) {
          pmeta = rmeta | ((v & kSlotIdentPos) ? kRowIdent : kRowDrop);
        } else {
          const uint32_t qv = (v & (kFoldQos0 << 2)) ? 2u : (v & (kFoldQos0 << 1)) ? 1u : 0u;
          pmeta = (rmeta & ~(kMetaQos | kMetaNoLocal)) | max(rmeta & kMetaQos, qv) | (rmeta & kMetaNoLocal) |
                  ((v & kFoldNoLocal) ? kMetaNoLocal : 0u);
        }
        emit_patch(occ && pmeta != rmeta, key, pmeta);
        n_nonbase += (uint32_t)__popcll(__ballot(nonbase));
        n_ext += (uint32_t)__popcll(__ballot(nonbase && (v & kSlotIdentPos)));
      }
      wave_sync_lds();
    };
    // big: one merge gather's lists [j0, j1), at most kSetBigFill visits, keyed by k alone:
    // (k + 1) << 5 | kBit* per record over the wave's kSetBigSlots words; the record's own meta and
    // identifier are read from the pool at the emission
    auto fold_big = [&](uint32_t j0, uint32_t j1) __attribute__((always_inline)) {
      map_ok = false;
      const uint32_t xa = h_ga[j0];
      const uint32_t sub_off = ix.lists[mg_node[xa]].sub_off;
      const uint32_t v0 = h_pre[j0], v1 = h_pre[j1];
      // the table sized to the visits (at most 2/3 full: short probe runs, and a short emission scan)
      const uint32_t ns = min(kSetBigSlots, ((v1 - v0) * 3 / 2 + 63) & ~63u);
      for (uint32_t q = lane; q < ns; q += 64) ws[q] = 0u;
      uint32_t jj_next, jb = j0;
      PairSlot e_next = locate_run(v0, jb, j1, jj_next, jb);
      wave_sync_lds();
      for (uint32_t r0 = v0; r0 < v1; r0 += 64) {
        const uint32_t r = r0 + lane;
        const uint32_t jj = jj_next;
        const PairSlot e = e_next;
        if (r0 + 64 < v1) e_next = locate_run(r0 + 64, jb, j1, jj_next, jb);  // wave-uniform
        if (r < v1) {
          const uint32_t pm = e.meta >> kSlotPartShift;
          const uint32_t bits = (before(h_hb[jj], xa) ? kBitNonBase : 0u) | ((pm & 4u) ? kBitNoLocal : 0u) |
                                ((pm & 3u) == 1u ? kBitQos1 : 0u) | ((pm & 3u) == 2u ? kBitQos2 : 0u);
          const uint32_t key = (e.k + 1u) << 5;
          uint32_t sl = __umulhi(hash32(e.k), ns);
          for (;;) {  // (at most kSetBigFill keys in ns >= 4/3 of them slots: a free slot is always found)
            const uint32_t prev = atomicCAS(&ws[sl], 0u, key | bits);
            if (prev == 0u) break;
            if ((prev & ~31u) == key) {
              if (bits & ~prev) atomicOr(&ws[sl], bits);
              break;
            }
            sl = sl + 1 == ns ? 0u : sl + 1;
          }
        }
        w_rec += r < v1;
      }
      wave_sync_lds();
      constexpr uint32_t kGroup = 4;
      for (uint32_t u0 = 0; u0 < ns; u0 += kGroup * 64) {
        uint32_t ent[kGroup];
        uint2 mi[kGroup];  // (identifier, meta) of the record
#pragma unroll
        for (uint32_t u = 0; u < kGroup; u++) {
          const uint32_t q = u0 + u * 64 + lane;
          ent[u] = q < ns ? ws[q] : 0u;
          mi[u] = make_uint2(0u, 0u);
          if (ent[u]) mi[u] = *reinterpret_cast<const uint2*>(&ix.subs[sub_off + (ent[u] >> 5) - 1u].ident);
        }
#pragma unroll
        for (uint32_t u = 0; u < kGroup; u++) {
          const uint32_t nib = ent[u] & 31u;
          const uint32_t rmeta = mi[u].y & kSlotMetaMask;
          const bool idpos = (int32_t)mi[u].x > 0;
          const bool nonbase = (nib & kBitNonBase) != 0;
          uint32_t pmeta;
          if (nonbase) {
            pmeta = rmeta | (idpos ? kRowIdent : kRowDrop);
          } else {
            const uint32_t qv = (nib & kBitQos2) ? 2u : (nib & kBitQos1) ? 1u : 0u;
            pmeta = (rmeta & ~(kMetaQos | kMetaNoLocal)) | max(rmeta & kMetaQos, qv) | (rmeta & kMetaNoLocal) |
                    ((nib & kBitNoLocal) ? kMetaNoLocal : 0u);
          }
          emit_patch(ent[u] != 0u && pmeta != rmeta, xa << kSetRowBits | ((ent[u] >> 5) - 1u), pmeta);
          n_nonbase += (uint32_t)__popcll(__ballot(nonbase));
          n_ext += (uint32_t)__popcll(__ballot(nonbase && idpos));
        }
      }
      wave_sync_lds();
    };
    auto flush_links = [&]() __attribute__((always_inline)) {  // the staged lists through the links
      if (lane == 0) h_pre[n_hit] = tot;
      wave_sync_lds();
      resolve_lists(0, n_hit, 0, 1);
      n_hit = 0;
      tot = 0;
      wave_sync_lds();
    };
    // the staged lists in chunks of whole merge gathers: up to kFoldCap visits folded together; a
    // gather beyond that alone in the record-keyed fold while kSetBigFill holds it (MQ_OPT_SET_EXP
    // bit 14: kBigFill, k_merge's table), else its links
    auto fold_hits = [&]() __attribute__((always_inline)) {
      if (lane == 0) h_pre[n_hit] = tot;
      wave_sync_lds();
      const uint32_t fcap = (exp_bits & 256u) ? 16u : small_fold ? kFoldCap : dense_fold ? kSetFoldSlots * 3 / 4 : sparse_fold ? kSetFoldSlots * 3 / 5 : kSetFoldCap;
      const uint32_t big_max = (exp_bits & 512u) ? 0u : (exp_bits & 16384u) ? kBigFill : kSetBigFill;
      uint32_t j0 = 0;
      while (j0 < n_hit) {  // wave-uniform
        const uint32_t b = h_pre[j0];
        uint32_t best = j0, next = n_hit;  // the furthest chunk end that fits; the next gather's start
        bool found = false;
        for (uint32_t c0 = j0 + 1; c0 <= n_hit; c0 += 64) {
          const uint32_t j = c0 + lane;
          bool bnd = false;
          if (j <= n_hit) bnd = j == n_hit || h_ga[j] != h_ga[j - 1];
          const uint64_t mb = __ballot(bnd), mf = __ballot(bnd && h_pre[min(j, n_hit)] - b <= fcap);
          if (mb && !found) {
            next = c0 + (uint32_t)__builtin_ctzll(mb);
            found = true;
          }
          if (mf) best = c0 + 63 - (uint32_t)__builtin_clzll(mf);
        }
        if (best > j0) {
          fold_lists(j0, best);
          j0 = best;
        } else {
          if (h_pre[next] - b <= big_max) fold_big(j0, next);
          else resolve_lists(j0, next, 0, 1);
          j0 = next;
        }
      }
      n_hit = 0;
      tot = 0;
      wave_sync_lds();
    };
    pairs(true, [] {});
    const uint64_t c_pairs = stamp ? clock64() : 0ull;
    const uint32_t n_hit_max = staged_all ? n_hit : kHitMax + 1;
    if (lane == 0 && tot_all) resv = atomicAdd(a.spcount + (t & (kPatchRegions - 1)), (unsigned long long)tot_all);
    resv_n = tot_all;
    resv_pending = true;
    if (staged_all) {
      if (n_hit) fold_hits();
    } else {  // rare: more hit lists than the stage holds; probe again, resolving as they come
      n_hit = 0;
      tot = 0;
      wave_sync_lds();
      pairs(false, flush_links);
      if (n_hit) flush_links();
    }
    settle();
    if (lane == 0) a.sets[t] = SetInfo{pbase, n_patch, n_nonbase, n_ext, pfit ? 1u : 0u};
    if (a.work) {  // MQ_PROF_WORK
      const uint32_t e = wave_sum(w_ent), rr = wave_sum(w_rec), l = wave_sum(w_link);
      if (a.set_rec && lane == 0) a.set_rec[t] = rr;
      unsigned long long* wc = a.work + (uint64_t)(t & (kPatchRegions - 1)) * kWork;
      if (lane == 0) {
        if (e | rr | l) {
          atomicAdd(wc + 0, (unsigned long long)e);
          atomicAdd(wc + 1, (unsigned long long)rr);
          atomicAdd(wc + 2, (unsigned long long)l);
          atomicAdd(wc + 3, (unsigned long long)n_patch);
        }
        atomicAdd(wc + 8, 1ull);
        atomicAdd(wc + 9, (unsigned long long)(16u * lc));
        const uint64_t c_end = clock64();
        atomicAdd(wc + 4, (unsigned long long)(c_map - c_start));
        atomicAdd(wc + 5, (unsigned long long)(c_pairs - c_map));
        atomicAdd(wc + 6, (unsigned long long)(c_end - c_pairs));
        atomicAdd(wc + 7, (unsigned long long)(c_end - c_start));
        atomicMax(wc + 24, (unsigned long long)(c_end - c_start));
        atomicMax(wc + 25, (unsigned long long)rr);
        atomicMax(wc + 26, (unsigned long long)(c_pairs - c_map));
        atomicMax(wc + 27, (unsigned long long)(c_end - c_pairs));
        atomicMax(wc + 28, (unsigned long long)lc);
        atomicMax(wc + 29, (unsigned long long)n_hit_max);
      }
    }
  }
}

void launch_set(const EmitArgs& a, uint32_t blocks, hipStream_t s) {
  if (!blocks) return;
  if (a.ix.xinfo) hipLaunchKernelGGL((k_set<6, true>), dim3(blocks), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(k_set<kMergeWavesPerEU>, dim3(blocks), dim3(256), 0, s, a);
}

}  // namespace mq
