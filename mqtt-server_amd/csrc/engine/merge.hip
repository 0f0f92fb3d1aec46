// gfx950 merge stage: merge-set dedup, k_finish, the merge set / topic passes (k_merge), host
// result packing and the row format's k_copy.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "kern_common.h"

namespace mq {


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
        const uint64_t t0 = src.xoff[t], t1 = src.xoff[t + 1], v0 = src.xoff[v];
        eq = src.xoff[v + 1] - v0 == t1 - t0;
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

// Host results' 4-byte patch codes (MQ_SPANS_PATCH_CODES): row << 3 | op, op from the new meta
// (1 + Qos + 3 NoLocal for a merge base, 7 for a later match); set rows x << 23 | k.
__device__ __forceinline__ uint32_t patch_op(uint32_t meta) {
  return (meta & (kRowIdent | kRowDrop)) ? 7u : 1u + (meta & kMetaQos) + ((meta & kMetaNoLocal) ? 3u : 0u);
}
__device__ __forceinline__ uint32_t set_patch_code(const PatchRec& p) {
  const uint32_t x = p.row >> kSetRowBits, k = p.row & ((1u << kSetRowBits) - 1u);
  return ((x << kCodeSetRowBits) | k) << 3 | patch_op(p.meta);
}

// Host span results: the written patches of every merge set packed (the set pool holds each
// set's reservation, of which SetInfo.n are written), as PatchRecs or (codes) patch codes;
// nbase[rep]: where the set's start. One atomic per wavefront; the wavefront copies its sets one
// at a time (coalesced).
__global__ __launch_bounds__(256) void k_set_pack(uint32_t n, const uint32_t* __restrict__ tslot,
                                                  const uint32_t* __restrict__ rep, const SetInfo* __restrict__ sets,
                                                  const PatchRec* __restrict__ pool, uint64_t* __restrict__ nbase,
                                                  PatchRec* __restrict__ out, uint32_t* __restrict__ codes,
                                                  unsigned long long* total) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, lane = threadIdx.x & 63;
  const bool own = t < n && tslot[t] != kNone && rep[t] == t;  // a set's representative
  SetInfo si{0, 0, 0, 0, 0};
  if (own) si = sets[t];
  // a set whose reservation did not fit its region (a one-sync batch that runs again) has no
  // patches in the pool: nothing to copy (its count would run past the pool and the stage)
  const uint32_t c = own && si.fit ? si.n : 0u;
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
    for (uint32_t k = lane; k < cj; k += 64) {
      if (codes) codes[bj + k] = set_patch_code(pool[sj + k]);
      else out[bj + k] = pool[sj + k];
    }
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

// Host span results: every topic's spans packed (one-sync batches leave them at t * 64, one
// atomic per wavefront places its topics' runs), span_base into the packed array.
__global__ __launch_bounds__(256) void k_span_pack(uint32_t n, TopicSpansDev* __restrict__ sres,
                                                   const SpanRec* __restrict__ src, SpanRec* __restrict__ dst,
                                                   unsigned long long* total) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, lane = threadIdx.x & 63;
  const uint32_t c = t < n ? sres[t].n_spans : 0u;
  const unsigned long long sb = t < n ? sres[t].span_base : 0ull;
  uint32_t sum;
  const uint32_t pre = wave_excl_scan(c, lane, &sum);
  unsigned long long b = 0;
  if (lane == 0 && sum) b = atomicAdd(total, (unsigned long long)sum);
  b = __shfl(b, 0, 64) + pre;
  if (t < n) sres[t].span_base = b;
  for (uint64_t m = __ballot(c != 0); m; m &= m - 1) {
    const int j = __builtin_ctzll(m);
    const uint32_t cj = __shfl(c, j, 64);
    const unsigned long long bj = __shfl(b, j, 64), sj = __shfl(sb, j, 64);
    for (uint32_t k = lane; k < cj; k += 64) dst[bj + k] = src[sj + k];
  }
}

void launch_span_pack(uint32_t n, TopicSpansDev* sres, const SpanRec* src, SpanRec* dst, unsigned long long* total,
                      hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_span_pack, dim3((n + 255) / 256), dim3(256), 0, s, n, sres, src, dst, total);
}

void launch_mrow_pack(uint32_t n, const uint32_t* tslot, const uint32_t* mcount, const uint32_t* mrow,
                      uint32_t* base, uint32_t* rows, unsigned long long* total, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_mrow_pack, dim3((n + 255) / 256), dim3(256), 0, s, n, tslot, mcount, mrow, base, rows, total);
}

void launch_set_pack(uint32_t n, const uint32_t* tslot, const uint32_t* rep, const SetInfo* sets,
                     const PatchRec* pool, uint64_t* nbase, PatchRec* out, uint32_t* codes, unsigned long long* total,
                     hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_set_pack, dim3((n + 255) / 256), dim3(256), 0, s, n, tslot, rep, sets, pool, nbase, out, codes,
                     total);
}

void launch_host_rebase(uint32_t n, const uint32_t* rep, const uint64_t* nbase, const uint64_t* roff, uint64_t rcap,
                        TopicSpansDev* sres, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_host_rebase, dim3((n + 255) / 256), dim3(256), 0, s, n, rep, nbase, roff, rcap, sres);
}

__global__ __launch_bounds__(256) void k_xsig(XSigArgs a) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = t < a.n;  // (no early exit: the dedup insert below is wave-cooperative)
  uint64_t sig = 0;
  uint32_t fc = 0, mc = 0;
  unsigned long long msig = 0;
  if (act) {
    for (uint32_t f = 0; f < a.n_xf; f++) {
      const XSrc src = a.xsrc[f];
      const uint64_t x0 = src.xoff[t], x1 = src.xoff[t + 1];
      for (uint64_t k = x0; k < x1; k++) {
        const XEnt e = src.xent[k];
        sig = mix64(sig ^ ((uint64_t)f << 56 | (uint64_t)fc << 32 | e.fid)) + e.rank;
        fc++;
      }
    }
    a.fcount[t] = fc;
    mc = a.mcount[t];
    if (mc) msig = a.msig[t];
    if (fc && mc) {
      msig = mix64(msig ^ sig) | 1ull;
      a.msig[t] = msig;
    }
  }
  if (a.dd_keys) {  // k_dedup_insert's work (the merge gathers and the other shards' entries must fit k_merge's map)
    const bool ok = act && mc != 0 && mc <= kPairMax && mc + fc < kMapSlots;
    const uint32_t slot = dedup_insert(a.dd_keys, a.dd_vals, a.dd_mask, t, ok, ok ? msig : 0ull);
    if (act) a.dd_tslot[t] = slot;
  }
  if (!act || !fc || !mc) return;
  if (mc <= kPairMax && mc + fc >= kMapSlots) {  // k_merge's slow path reads GDesc records
    if (a.g_stride) {  // the walk-fused layout (the gather words at the spans' positions)
      const uint64_t g0 = (uint64_t)t * a.g_stride;
      write_gdesc(a.ix, a.gathers + g0, a.tc[t].gathers, 0u, a.desc + g0);
    } else {
      const TopicOff o0 = a.off[t], o1 = a.off[t + 1];
      const uint32_t* gw_src = a.gather_stride ? a.gathers + (uint64_t)t * a.gather_stride : a.gathers + o0.g;
      write_gdesc(a.ix, gw_src, (uint32_t)(o1.g - o0.g), (uint32_t)o0.shr, a.desc + o0.g);
    }
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
// Sharded index: do filters fh and fg, whose rank keys tie, come in this DFS order? A tie means
// that their first 32 levels agree: both are deeper (their DeepTail codes decide, compared as the
// rank keys are, a proper prefix first), or one is exactly 32 levels deep — a proper prefix of
// the other, so first. A tie no entry explains trips kErrDeepRank.
__device__ __forceinline__ bool deep_before(const DevIndex& ix, uint32_t fh, uint32_t fg) {
  auto find = [&](uint32_t f) -> const DeepTail* {
    if (!ix.deep) return nullptr;
    uint64_t sl = mix64(f) & ix.deep_mask;
    for (;;) {
      const DeepTail* e = ix.deep + sl;
      if (e->fid == f) return e;
      if (e->fid == kNone) return nullptr;
      sl = (sl + 1) & ix.deep_mask;
    }
  };
  const DeepTail* h = find(fh);
  const DeepTail* g = find(fg);
  if (!h || !g) {
    if (!h && !g) atomicOr(ix.err, kErrDeepRank);
    return !h && g;
  }
  const uint32_t n = max(h->n, g->n);
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t wh = i < h->n ? ix.deep_codes[h->off + i] : 0u;
    const uint32_t wg = i < g->n ? ix.deep_codes[g->off + i] : 0u;
    if (wh != wg) return wh < wg;
  }
  return false;  // one path (a filter lives on one shard): not reached
}

// DEEP (a sharded index holding filters deeper than 32 levels, DevIndex.deep): rank-key ties are
// ordered by deep_before; without DEEP no tie can occur (the keys hold every level), and the
// tie-break's code and live values stay out of the kernel (the sharded set pass spills heavily
// already: 0.44 -> 1.7 ms per shard with the tie-break compiled in, profiles/r05/shard2/)
template <bool SPANS, bool XS, int WPE, bool SET = false, uint32_t PB = kPartBatch, bool DEEP = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_merge(EmitArgs args) {
  // the arguments, read from the kernarg segment where they are used (as in k_set: a by-value
  // parameter is loaded whole at the entry and its pointers spill to vector lanes)
  (void)args;
  const EmitArgs& a = kernarg_at<EmitArgs>(0);
  constexpr uint32_t kEnt = XS ? kMapSlots : kPairMax;  // map entries
  // per-wave words, one contiguous block (the set pass's record-keyed fold spans the map and the
  // merge gathers' three arrays): the map (gathered node with may-merge records, or kForeign | fid
  // of another shard's, XS -> its entry below), then per merge gather the output row of its first
  // record (pair slots name a record by its place k in the particle's list) and its pair-block hash
  // table (NodePair)
  __shared__ uint32_t wsm[4][2 * kMapSlots + 3 * kPairMax];
  uint32_t* const map_key = wsm[wave_id()];
  uint32_t* const map_val = map_key + kMapSlots;
  uint32_t* const mg_row = map_key + 2 * kMapSlots;
  uint32_t* const mg_eoff = mg_row + kPairMax;
  uint32_t* const mg_emask = mg_eoff + kPairMax;
  __shared__ uint32_t mg_node[4][kEnt];        // entries: the topic's merge gathers in gather
  __shared__ uint32_t mg_gi[4][kEnt];          //   order (node, gather index), then (XS) the
  __shared__ uint64_t mg_rank[4][XS ? kEnt : 1];  // other shards' (kForeign | fid, kNone, rank)
  __shared__ uint32_t h_ga[4][kHitMax];        // staged hit lists: merge gather of g,
  __shared__ uint32_t h_off[4][kHitMax];       //   pair-list offset,
  __shared__ uint32_t h_hb[4][kHitMax];        //   partner h's entry (mg_node[h_hb]: its node),
  __shared__ uint32_t h_pre[4][kHitMax + 1];   //   exclusive prefix of their lengths (+ total)
  const uint32_t wv = wave_id(), lane = threadIdx.x & 63;
  auto rank_of = [](const GDesc& d) { return gdesc_rank<XS>(d); };
  // MQ_OPT_SET_EXP: the exact variants (bit 7: partner links instead of the fold, bit 8: small fold
  // chunks) in every build; the attribution bits 0-4 in development builds only
  const uint32_t exp_bits = kDevBuild ? a.exp : (a.exp & (128u | 256u | 512u | 1024u | 2048u));
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
      for (uint32_t q = lane; q < kMapSlots; q += 64) map_key[q] = kNone;
      wave_sync_lds();
      if (lane < lc) {
        const uint64_t k = (uint64_t)t * kPairMax + lane;
        const uint32_t node = a.mlist[k];
        const uint2 P = a.mpair[k];
        uint32_t sl = hash32(node) & (kMapSlots - 1);
        while (atomicCAS(&map_key[sl], kNone, node) != kNone) sl = (sl + 1) & (kMapSlots - 1);
        map_val[sl] = lane;
        mg_node[wv][lane] = node;
        mg_gi[wv][lane] = lane;
        if (XS) mg_rank[wv][lane] = a.mrank[k];
        mg_row[lane] = a.mrow[k];
        mg_eoff[lane] = P.x;
        mg_emask[lane] = P.y;
      }
      n_map = lc;
      w_map = (XS ? 24u : 16u) * lc;
    } else {
    if (a.unsafe && o1.g > a.desc_cap) {  // one-sync batch: no GDesc records to read
      if (lane == 0) atomicOr(a.unsafe, kUnsafeDesc);
      continue;
    }
    for (uint32_t q = lane; q < kMapSlots; q += 64) map_key[q] = kNone;
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
        while (atomicCAS(&map_key[sl], kNone, node) != kNone) sl = (sl + 1) & (kMapSlots - 1);
        map_val[sl] = x;
        mg_node[wv][x] = node;
        mg_gi[wv][x] = i;
        if (XS) mg_rank[wv][x] = rank_of(gd[i]);
        mg_row[x] = mrow;
        mg_eoff[x] = P.ent_off;
        mg_emask[x] = P.ent_mask;
      }
      n_map += __popcll(bi);
    }
    }
    // sharded index: the other shards' gathered cross-shard nodes join the map as entries
    // n_map.. (their partner links name them kForeign | fid; their rank keys order them)
    uint32_t n_ent = n_map;
    for (uint32_t f = 0; XS && f < a.n_xf; f++) {
      const XSrc src = a.xsrc[f];
      const uint64_t x0 = src.xoff[t], x1 = src.xoff[t + 1];
      for (uint64_t k0 = x0; k0 < x1; k0 += 64) {
        const uint64_t k = k0 + lane;
        const uint32_t x = n_ent + (uint32_t)(k - x0);
        if (k < x1 && x < kEnt && n_map <= kPairMax) {
          const XEnt e = src.xent[k];
          const uint32_t key = kForeign | e.fid;
          uint32_t sl = hash32(key) & (kMapSlots - 1);
          while (atomicCAS(&map_key[sl], kNone, key) != kNone) sl = (sl + 1) & (kMapSlots - 1);
          map_val[sl] = x;
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
          const uint32_t k = map_key[sl];
          if (k == h) {
            const uint32_t y = map_val[sl];
            return Pos{XS ? mg_rank[wv][y] : 0ull, mg_gi[wv][y], true};
          }
          if (k == kNone) return Pos{0, kNone, false};
          sl = (sl + 1) & (kMapSlots - 1);
        }
      }
      if (XS && (h & kForeign)) {
        for (uint32_t f = 0; f < a.n_xf; f++) {
          const XSrc src = a.xsrc[f];
          for (uint64_t k = src.xoff[t]; k < src.xoff[t + 1]; k++)
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
    // hn / gn: the nodes (another shard's as kForeign | fid), read only on a tie
    auto before = [&](uint64_t rh, uint32_t gh, uint64_t rg, uint32_t gg, auto&& hn, auto&& gn)
        __attribute__((always_inline)) -> bool {
      if (!XS) return gh < gg;
      if (rh != rg) return rh < rg;
      if (gh != kNone) return gh < gg;  // both on this shard: gather order is DFS order
      // another shard's node tied with the record's beyond the key's 32 levels
      if constexpr (DEEP) {
        const uint32_t h = hn(), g = gn();
        return deep_before(a.ix, (h & kForeign) ? h & ~kForeign : a.ix.xinfo[h].fid,
                           (g & kForeign) ? g & ~kForeign : a.ix.xinfo[g].fid);
      } else {
        (void)hn;
        (void)gn;
        atomicOr(a.ix.err, kErrDeepRank);  // (no deep filters: not reached)
        return false;
      }
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
                       uint32_t mp_off, uint32_t mp_cnt, auto&& gnode) __attribute__((always_inline)) {
      bool counted = false, nonbase = false, want = false;
      uint32_t pmeta = 0;
      if (active) {
        const uint32_t rmeta = mw & kSlotMetaMask;
        const bool idpos = (mw & kSlotIdentPos) != 0;
        bool bound = false, base = true;
        // (span format) a visit through a partner that is not the record's first gathered one
        // counts and emits nothing: it stops at that first one (the row format rewrites the row on
        // every visit, so it reads every link)
        bool other = false;
        uint32_t first = kNone;
        uint32_t q = rmeta & kMetaQos, nl = rmeta & kMetaNoLocal;
        if (SET && (exp_bits & 1u)) mp_cnt = 0;
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
            if (SET && (exp_bits & 2u)) {
              q = max(q, pb[u].meta & kMetaQos);
              continue;
            }
            const Pos ph = gathered(pb[u].node);
            if (!ph.found) continue;
            if (!bound) {
              first = pb[u].node;
              other = SPANS && via != kNone && first != via && !(SET && (exp_bits & 16u));
            }
            bound = true;
            const uint32_t hnode = pb[u].node;
            if (before(ph.rk, ph.gi, rg, gi, [&] { return hnode; }, gnode)) {
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
      if (SPANS) emit_patch(want && !(SET && (exp_bits & 4u)), row, pmeta);
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
      bool map_ok = true;  // the node -> entry map is in place (a fold uses its LDS)
      // visit r of the staged lists [j0, j1): its list jj (binary search of the prefix) and its
      // pair slot
      auto locate = [&](uint32_t r, uint32_t j0, uint32_t j1, uint32_t& jj) __attribute__((always_inline)) -> PairSlot {
        const uint32_t rc = min(r, h_pre[wv][j1] - 1);
        uint32_t lo = j0, hi = j1;  // h_pre[lo] <= rc < h_pre[hi] (lists are non-empty)
        if (SET && (exp_bits & 8u)) {  // (a list's first slot: in bounds, not the record's)
          jj = j0 + rc % (j1 - j0);
          return a.ix.plist[h_off[wv][jj]];
        }
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (h_pre[wv][mid] <= rc) lo = mid; else hi = mid;
        }
        jj = lo;
        return a.ix.plist[h_off[wv][lo] + (rc - h_pre[wv][lo])];
      };
      // every visit of lists [j0, j1) resolves its record through the record's partner links
      // (wave-uniform; h_pre[j1] set). Software-pipelined by one round: the next 64 records' pair
      // slots are loaded before this round's partner links, so each round waits on one load
      // latency, not two (two rounds, with the next round's first links in flight too, spilled
      // registers and was slower: 1.15 -> 1.36 ms at 8 waves per SIMD, 1.24 ms at 6;
      // profiles/r03/s2_hostsets/)
      // (pp, PP): only the records with hash32(k) % PP == pp (fold_big's partitions)
      auto resolve_lists = [&](uint32_t j0, uint32_t j1, uint32_t pp = 0, uint32_t PP = 1) __attribute__((always_inline)) {
        const uint32_t v0 = h_pre[wv][j0], v1 = h_pre[wv][j1];
        uint32_t jj_next = j0;
        PairSlot e_next = locate(v0 + lane, j0, j1, jj_next);
        for (uint32_t r0 = v0; r0 < v1; r0 += 64) {
          const uint32_t r = r0 + lane;
          const uint32_t jj = jj_next;
          const PairSlot e = e_next;
          if (r0 + 64 < v1) e_next = locate(r0 + 64 + lane, j0, j1, jj_next);  // wave-uniform
          const uint32_t xa = h_ga[wv][jj];
          w_rec += r < v1;
          resolve(r < v1 && (PP == 1 || hash32(e.k) % PP == pp), e.meta, setrel ? (xa << kSetRowBits | e.k) : mg_row[xa] + e.k,
                  XS ? mg_rank[wv][xa] : 0ull, mg_gi[wv][xa], mg_node[wv][h_hb[wv][jj]], e.mp_off, e.mp_cnt,
                  [&] { return mg_node[wv][xa]; });
        }
      };
      auto flush_hits = [&]() __attribute__((always_inline)) {
        if (lane == 0) h_pre[wv][n_hit] = tot;
        wave_sync_lds();
        resolve_lists(0, n_hit);
        n_hit = 0;
        tot = 0;
        wave_sync_lds();
      };
      // Set pass, the fold (no partner links): a record's visits are exactly its gathered
      // partners (one visit per pair list (g, h) holding it, and every gathered h is probed), and
      // each pair slot carries its partner's Qos / NoLocal. So the record is a non-base entry iff
      // a visit's h comes before g, else the base with the max Qos and OR'd NoLocal over its
      // visits — folded per record in an LDS hash table keyed by its set-relative row, then one
      // patch per record. Lists [j0, j1) hold whole merge gathers (a record's visits are all in
      // its g's lists) and at most kFoldCap visits.
      auto fold_lists = [&](uint32_t j0, uint32_t j1) __attribute__((always_inline)) {
        uint32_t* __restrict__ f_key = map_key;  // (the table takes the map's place: the fold
        uint32_t* __restrict__ f_val = map_val;  //  does not look nodes up; map_rebuild restores it)
        const uint32_t v0 = h_pre[wv][j0], v1 = h_pre[wv][j1];
        for (uint32_t q = lane; q < kFoldSlots; q += 64) {
          f_key[q] = kNone;
          f_val[q] = 0;
        }
        map_ok = false;
        // software-pipelined by one round, as resolve_lists: the next round's pair slots are in
        // flight while this round folds
        uint32_t jj_next = j0;
        PairSlot e_next = locate(v0 + lane, j0, j1, jj_next);
        wave_sync_lds();
        for (uint32_t r0 = v0; r0 < v1; r0 += 64) {
          const uint32_t r = r0 + lane;
          const uint32_t jj = jj_next;
          const PairSlot e = e_next;
          if (r0 + 64 < v1) e_next = locate(r0 + 64 + lane, j0, j1, jj_next);  // wave-uniform
          if (r < v1) {
            const uint32_t xa = h_ga[wv][jj], hb = h_hb[wv][jj];
            const bool earlier = before(XS ? mg_rank[wv][hb] : 0ull, mg_gi[wv][hb], XS ? mg_rank[wv][xa] : 0ull,
                                        mg_gi[wv][xa], [&] { return mg_node[wv][hb]; }, [&] { return mg_node[wv][xa]; });
            const uint32_t key = xa << kSetRowBits | e.k;
            if (!(exp_bits & 4096u)) {  // (MQ_OPT_SET_EXP bit 12, development builds: no table inserts)
              uint32_t sl = hash32(key) & (kFoldSlots - 1);
              for (;;) {
                const uint32_t prev = atomicCAS(&f_key[sl], kNone, key);
                if (prev == kNone || prev == key) break;
                sl = (sl + 1) & (kFoldSlots - 1);
              }
              const uint32_t pm = e.meta >> kSlotPartShift;  // the partner's Qos | NoLocal << 2
              atomicOr(&f_val[sl], (e.meta & kSlotOwnMask) | (earlier ? kFoldNonBase : 0u) |
                                       ((pm & 4u) ? kFoldNoLocal : 0u) | (kFoldQos0 << (pm & 3u)));
            }
          }
          w_rec += r < v1;
        }
        wave_sync_lds();
        for (uint32_t s0 = 0; s0 < kFoldSlots; s0 += 64) {
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
          emit_patch(occ && pmeta != rmeta && !(exp_bits & 4u), key, pmeta);
          n_nonbase += __popcll(__ballot(nonbase));
          n_ext += __popcll(__ballot(nonbase && (v & kSlotIdentPos)));
        }
        wave_sync_lds();  // (before the table is cleared again)
      };
      // the node -> entry map again (after a fold took its place), for the partner-link path
      auto map_rebuild = [&]() __attribute__((always_inline)) {
        for (uint32_t q = lane; q < kMapSlots; q += 64) map_key[q] = kNone;
        wave_sync_lds();
        for (uint32_t x = lane; x < n_ent; x += 64) {
          const uint32_t node = mg_node[wv][x];
          uint32_t sl = hash32(node) & (kMapSlots - 1);
          while (atomicCAS(&map_key[sl], kNone, node) != kNone) sl = (sl + 1) & (kMapSlots - 1);
          map_val[sl] = x;
        }
        wave_sync_lds();
        map_ok = true;
      };
      // A merge gather whose lists hold more visits than the hash fold's chunk (the hot lists: root
      // '#', '+/...', 'x/#': ~10k may-merge records, ~200 of them visited per set): the same fold,
      // keyed by the record's place k in g's list alone (one gather), so a table entry is one word
      // — (k + 1) << 5 | kBit* — and kBigSlots of them fit in the map's LDS plus the merge gathers'
      // pair-block and row arrays (free once the pair analysis is done: the set pass names rows
      // set-relatively). The record's own meta and identifier are read from the pool at the
      // emission (one load per folded record, a group of rounds in flight), not carried in the
      // table. The caller folds a gather this way only while one pass holds its visits (more passes,
      // over partitions hash(k) mod P, each re-read every visit and cost more than the partner
      // links: profiles/r05/c/); a partition that still overflows the table resolves through the
      // links. No partner links otherwise.
      auto fold_big = [&](uint32_t j0, uint32_t j1) __attribute__((always_inline)) {
        auto slot_ptr = [&](uint32_t q) __attribute__((always_inline)) -> uint32_t* { return map_key + q; };
        map_ok = false;
        const uint32_t xa = h_ga[wv][j0];
        const uint32_t sub_off = a.ix.lists[mg_node[wv][xa]].sub_off;
        const uint32_t v0 = h_pre[wv][j0], v1 = h_pre[wv][j1];
        const uint64_t rg = XS ? mg_rank[wv][xa] : 0ull;
        const uint32_t gg = mg_gi[wv][xa];
        // the partitions: the records with hash(k) % PP == pp
        const uint32_t PP = max(1u, (v1 - v0 + kBigFill - 1) / kBigFill);
        for (uint32_t pp = 0; pp < PP; pp++) {  // wave-uniform
          for (uint32_t q = lane; q < kBigSlots; q += 64) *slot_ptr(q) = 0u;
          uint32_t jj_next = j0;
          PairSlot e_next = locate(v0 + lane, j0, j1, jj_next);
          wave_sync_lds();
          bool over = false;
          for (uint32_t r0 = v0; r0 < v1; r0 += 64) {
            const uint32_t r = r0 + lane;
            const uint32_t jj = jj_next;
            const PairSlot e = e_next;
            if (r0 + 64 < v1) e_next = locate(r0 + 64 + lane, j0, j1, jj_next);  // wave-uniform
            const uint32_t hk = hash32(e.k);
            if (r < v1 && hk % PP == pp) {
              const uint32_t hb = h_hb[wv][jj];
              const bool earlier = before(XS ? mg_rank[wv][hb] : 0ull, mg_gi[wv][hb], rg, gg,
                                          [&] { return mg_node[wv][hb]; }, [&] { return mg_node[wv][xa]; });
              const uint32_t pm = e.meta >> kSlotPartShift;  // the partner's Qos | NoLocal << 2
              const uint32_t bits = (earlier ? kBitNonBase : 0u) | ((pm & 4u) ? kBitNoLocal : 0u) |
                                    ((pm & 3u) == 1u ? kBitQos1 : 0u) | ((pm & 3u) == 2u ? kBitQos2 : 0u);
              const uint32_t key = (e.k + 1u) << 5;
              uint32_t sl = (hk >> 8) % kBigSlots;
              bool placed = (exp_bits & 4096u) != 0;  // (bit 12: no table inserts)
              for (uint32_t probes = 0; !placed && probes < kBigSlots; probes++) {
                const uint32_t prev = atomicCAS(slot_ptr(sl), 0u, key | bits);
                if (prev == 0u) {
                  placed = true;
                  break;
                }
                if ((prev & ~31u) == key) {
                  if (bits & ~prev) atomicOr(slot_ptr(sl), bits);
                  placed = true;
                  break;
                }
                sl = sl + 1 == kBigSlots ? 0u : sl + 1;
              }
              over |= !placed;
            }
            w_rec += r < v1;
          }
          wave_sync_lds();
          if (__ballot(over)) {  // (rare) this partition's records do not fit: through their links
            map_rebuild();
            resolve_lists(j0, j1, pp, PP);
            map_ok = false;
            continue;
          }
          // emission: every folded record, its own meta / identifier read from the pool (the
          // table's rounds loaded together)
          constexpr uint32_t kGroup = 4;
          for (uint32_t u0 = 0; u0 < kBigSlots / 64; u0 += kGroup) {
          uint32_t ent[kGroup];
          uint2 mi[kGroup];
#pragma unroll
          for (uint32_t u = 0; u < kGroup; u++) {
            ent[u] = (u0 + u) * 64 < kBigSlots ? *slot_ptr((u0 + u) * 64 + lane) : 0u;
            mi[u] = make_uint2(0u, 0u);
            if (ent[u]) mi[u] = *reinterpret_cast<const uint2*>(&a.ix.subs[sub_off + (ent[u] >> 5) - 1u].ident);
          }
#pragma unroll
          for (uint32_t u = 0; u < kGroup; u++) {
            const uint32_t nib = ent[u] & 31u;
            const uint32_t k = (ent[u] >> 5) - 1u;
            const uint32_t rmeta = mi[u].y & kSlotMetaMask;
            const bool idpos = (int32_t)mi[u].x > 0;
            const bool nonbase = ent[u] && (nib & kBitNonBase);
            uint32_t pmeta;
            if (nib & kBitNonBase) {
              pmeta = rmeta | (idpos ? kRowIdent : kRowDrop);
            } else {
              const uint32_t qv = (nib & kBitQos2) ? 2u : (nib & kBitQos1) ? 1u : 0u;
              pmeta = (rmeta & ~(kMetaQos | kMetaNoLocal)) | max(rmeta & kMetaQos, qv) | (rmeta & kMetaNoLocal) |
                      ((nib & kBitNoLocal) ? kMetaNoLocal : 0u);
            }
            emit_patch(ent[u] != 0u && pmeta != rmeta && !(exp_bits & 4u), xa << kSetRowBits | k, pmeta);
            n_nonbase += __popcll(__ballot(nonbase));
            n_ext += __popcll(__ballot(nonbase && idpos));
          }
          }
          wave_sync_lds();  // (before the table is cleared again)
        }
      };
      // the staged lists, folded in chunks of whole merge gathers; a merge gather whose lists
      // alone hold more than kFoldCap visits resolves through the partner links
      auto fold_hits = [&]() __attribute__((always_inline)) {
        if (lane == 0) h_pre[wv][n_hit] = tot;
        wave_sync_lds();
        const uint32_t fcap = (exp_bits & 256u) ? 16u : kFoldCap;  // (MQ_OPT_SET_EXP bit 8: small chunks)
        uint32_t j0 = 0;
        while (j0 < n_hit) {  // wave-uniform
          const uint32_t b = h_pre[wv][j0];
          uint32_t best = j0, next = n_hit;  // the furthest chunk end that fits; the next gather's start
          bool found = false;
          for (uint32_t c0 = j0 + 1; c0 <= n_hit; c0 += 64) {
            const uint32_t j = c0 + lane;
            bool bnd = false;
            if (j <= n_hit) bnd = j == n_hit || h_ga[wv][j] != h_ga[wv][j - 1];
            const uint64_t mb = __ballot(bnd), mf = __ballot(bnd && h_pre[wv][min(j, n_hit)] - b <= fcap);
            if (mb && !found) {
              next = c0 + (uint32_t)__builtin_ctzll(mb);
              found = true;
            }
            if (mf) best = c0 + 63 - (uint32_t)__builtin_clzll(mf);
          }
          if (best > j0) {
            if (a.work && lane == 0) {  // MQ_PROF_WORK: the fold's shape
              unsigned long long* wc = a.work + (uint64_t)(t & (kPatchRegions - 1)) * kWork;
              atomicAdd(wc + 10, (unsigned long long)(h_pre[wv][best] - h_pre[wv][j0]));
              uint64_t nm = 0;
              for (uint32_t j = j0; j < best; j++)
                if (j == j0 || h_ga[wv][j] != h_ga[wv][j - 1]) nm += a.ix.lists[mg_node[wv][h_ga[wv][j]]].n_merge;
              atomicAdd(wc + 14, (unsigned long long)nm);
              atomicAdd(wc + 15, 1ull);
            }
            fold_lists(j0, best);
            j0 = best;
          } else {
            if (a.work && lane == 0) {
              unsigned long long* wc = a.work + (uint64_t)(t & (kPatchRegions - 1)) * kWork;
              atomicAdd(wc + 11, (unsigned long long)(h_pre[wv][next] - h_pre[wv][j0]));
              atomicAdd(wc + 12, 1ull);
              atomicAdd(wc + 13, (unsigned long long)a.ix.lists[mg_node[wv][h_ga[wv][j0]]].n_merge);
              const uint32_t vb = h_pre[wv][next] - h_pre[wv][j0];
              const uint32_t bk = vb <= 192 ? 0u : vb <= 384 ? 1u : vb <= 1024 ? 2u : 3u;
              atomicAdd(wc + 16 + bk, 1ull);
              atomicAdd(wc + 20 + bk, (unsigned long long)vb);
            }
            // the bit fold while its passes stay few (a pass re-reads the gather's visits: many passes
            // cost more than the links); bits 10 / 11: up to two passes / any number (A/B)
            const uint32_t vbig = h_pre[wv][next] - h_pre[wv][j0];
            const uint32_t fold_max = (exp_bits & 2048u) ? ~0u : (exp_bits & 1024u) ? 2 * kBigFill : kBigFill;
            if (!(exp_bits & 512u) && vbig <= fold_max) {
              fold_big(j0, next);
            } else {  // (MQ_OPT_SET_EXP bit 9: through the partner links, as before round 5)
              if (!map_ok) map_rebuild();
              resolve_lists(j0, next);
            }
            j0 = next;
          }
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
          uint32_t ga = 0, e_off = 0, e_cnt = 0, hn = 0, hb = 0;
          if (p < np) {
            ga = p / n_ent;
            hb = p - ga * n_ent;
            if (ga != hb) {
              const uint32_t ent_mask = mg_emask[ga], ent_off = mg_eoff[ga];
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
            h_hb[wv][x] = hb;
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
          if (n_hit) {
            if (SET && !(exp_bits & 128u)) fold_hits();
            else flush_hits();
          }
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
                  i, kNone, mr.off, mr.cnt, [&] { return d.word & kGatherNode; });
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

void launch_copy(const EmitArgs& a, uint32_t max_blocks, hipStream_t s) {
  const uint32_t waves = a.n_tiles[0] + a.n_tiles[1] + a.n_tiles[2];
  if (!waves) return;
  const uint32_t blocks = max_blocks ? std::min((waves + 3) / 4, max_blocks) : (waves + 3) / 4;
  hipLaunchKernelGGL(k_copy, dim3(blocks), dim3(256), 0, s, a);
}

// The product build holds one register budget per pass (kMergeWavesPerEU; 6 for a sharded index,
// whose map holds rank keys); the other budgets and the set pass's 3 / 4 partner links per batch
// (MQ_OPT_MERGE_WAVES, MQ_OPT_SET_EXP bits 5 / 6) are measurement variants, built with DEV=1.
void launch_merge(const EmitArgs& a, bool spans, uint32_t wpe, uint32_t max_blocks, hipStream_t s) {
  const uint32_t waves = a.t1 - a.t0;
  if (!waves) return;
  const uint32_t blocks = max_blocks ? std::min((waves + 3) / 4, max_blocks) : (waves + 3) / 4;
  const dim3 g(blocks), b(256);
#ifdef MQ_DEV_BUILD
  if (spans && a.ix.xinfo && a.rep && a.dd_phase == 1 && wpe < 6) {
    hipLaunchKernelGGL((k_merge<true, true, 1, true>), g, b, 0, s, a);
    return;
  }
  if (spans && a.ix.xinfo && !(a.rep && a.dd_phase == 1) && wpe < 6) {
    hipLaunchKernelGGL((k_merge<true, true, 1>), g, b, 0, s, a);
    return;
  }
  if (spans && !a.ix.xinfo && a.rep && a.dd_phase == 1 && (wpe < 8 || (a.exp & 96u))) {
    if (wpe >= 8 && (a.exp & 32u)) hipLaunchKernelGGL((k_merge<true, false, 8, true, 3>), g, b, 0, s, a);
    else if (wpe >= 8) hipLaunchKernelGGL((k_merge<true, false, 8, true, 4>), g, b, 0, s, a);
    else if (wpe == 7) hipLaunchKernelGGL((k_merge<true, false, 7, true>), g, b, 0, s, a);
    else if (wpe >= 6) hipLaunchKernelGGL((k_merge<true, false, 6, true>), g, b, 0, s, a);
    else hipLaunchKernelGGL((k_merge<true, false, 1, true>), g, b, 0, s, a);
    return;
  }
  if (!(spans && a.ix.xinfo) && !(spans && a.rep && a.dd_phase == 1) && wpe < 8) {
    if (spans && wpe >= 6) hipLaunchKernelGGL((k_merge<true, false, 6>), g, b, 0, s, a);
    else if (spans) hipLaunchKernelGGL((k_merge<true, false, 1>), g, b, 0, s, a);
    else if (wpe >= 6) hipLaunchKernelGGL((k_merge<false, false, 6>), g, b, 0, s, a);
    else hipLaunchKernelGGL((k_merge<false, false, 1>), g, b, 0, s, a);
    return;
  }
#else
  (void)wpe;
#endif
  if (spans && a.ix.xinfo && a.rep && a.dd_phase == 1) {  // sharded index, merge-set dedup: the set pass
    if (a.ix.deep) hipLaunchKernelGGL((k_merge<true, true, 6, true, kPartBatch, true>), g, b, 0, s, a);
    else hipLaunchKernelGGL((k_merge<true, true, 6, true>), g, b, 0, s, a);
  } else if (spans && a.ix.xinfo) {  // sharded index
    if (a.ix.deep) hipLaunchKernelGGL((k_merge<true, true, 6, false, kPartBatch, true>), g, b, 0, s, a);
    else hipLaunchKernelGGL((k_merge<true, true, 6>), g, b, 0, s, a);
  }
  else if (spans && a.rep && a.dd_phase == 1)  // merge-set dedup: the set pass
    hipLaunchKernelGGL((k_merge<true, false, 8, true>), g, b, 0, s, a);
  else if (spans)
    hipLaunchKernelGGL((k_merge<true, false, 8>), g, b, 0, s, a);
  else
    hipLaunchKernelGGL((k_merge<false, false, 8>), g, b, 0, s, a);
}

__global__ __launch_bounds__(256) void k_patch_compact(const PatchRec* __restrict__ pool, uint64_t rcap,
                                                      const unsigned long long* __restrict__ pcount,
                                                      const uint64_t* __restrict__ roff, PatchRec* __restrict__ out,
                                                      uint32_t* __restrict__ codes) {
  const uint32_t r = blockIdx.x;
  const uint64_t n = pcount[r];
  const PatchRec* src = pool + (uint64_t)r * rcap;
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
    if (codes) codes[roff[r] + i] = src[i].row << 3 | patch_op(src[i].meta);
    else out[roff[r] + i] = src[i];
  }
}

void launch_patch_compact(const PatchRec* pool, uint64_t rcap, const unsigned long long* pcount,
                          const uint64_t* roff, PatchRec* out, uint32_t* codes, hipStream_t s) {
  hipLaunchKernelGGL(k_patch_compact, dim3(kPatchRegions), dim3(256), 0, s, pool, rcap, pcount, roff, out, codes);
}

}  // namespace mq
