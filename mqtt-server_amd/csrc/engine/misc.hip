// gfx950 kernels beside the match: k_acl, k_pick, the sharded export, staging scatter and the
// one-sync batch reset / readback.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "kern_common.h"

namespace mq {

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

__global__ __launch_bounds__(256) void k_xcounts(const uint32_t* __restrict__ xcount, const TopicCount* __restrict__ tc,
                                                 uint32_t n, TopicCount* __restrict__ cnt) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) cnt[t] = TopicCount{xcount[t], tc[t].gathers, 0, 0, 0};
}

void launch_xcounts(const uint32_t* xcount, const TopicCount* tc, uint32_t n, TopicCount* cnt, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_xcounts, dim3((n + 255) / 256), dim3(256), 0, s, xcount, tc, n, cnt);
}

__global__ __launch_bounds__(256) void k_xpack(uint32_t n, const TopicOff* __restrict__ off, uint32_t g_stride,
                                               const uint32_t* __restrict__ xcount, const TopicOff* __restrict__ xoff,
                                               const TopicOff* __restrict__ xtot, const XEnt* __restrict__ xents,
                                               XEnt* __restrict__ ents, uint64_t cap, uint32_t* unsafe,
                                               unsigned long long* total) {
  const uint64_t all = xtot->g;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t == 0) {
    total[0] = all;
    if (all > cap) atomicOr(unsafe, kUnsafeXEnts);
  }
  if (t >= n || all > cap) return;
  const uint32_t c = xcount[t];
  const uint64_t src = g_stride ? (uint64_t)t * g_stride : off[t].g, dst = xoff[t].g;
  for (uint32_t k = 0; k < c; k++) ents[dst + k] = xents[src + k];
}

void launch_xpack(uint32_t n, const TopicOff* off, uint32_t g_stride, const uint32_t* xcount, const TopicOff* xoff,
                  const TopicOff* xtot, const XEnt* xents, XEnt* ents, uint64_t cap, uint32_t* unsafe,
                  unsigned long long* total, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_xpack, dim3((n + 255) / 256), dim3(256), 0, s, n, off, g_stride, xcount, xoff, xtot, xents, ents,
                     cap, unsafe, total);
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
  const uint32_t lane = threadIdx.x;  // one wavefront
  unsigned long long np = 0;
  if (a.pcount) {  // the regions' exclusive prefix, kPatchRegions / 64 regions per lane
    constexpr uint32_t kPer = kPatchRegions / 64;
    unsigned long long c[kPer], sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
      c[k] = a.pcount[lane * kPer + k];
      sum += c[k];
    }
    unsigned long long x = sum;  // inclusive scan of the lanes' sums
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned long long y = __shfl_up(x, d, 64);
      if (lane >= (uint32_t)d) x += y;
    }
    unsigned long long off = x - sum;
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
      a.roff[lane * kPer + k] = off;
      off += c[k];
    }
    np = __shfl(x, 63, 64);
    if (lane == 63) a.roff[kPatchRegions] = np;
  }
  if (lane != 0) return;
  FastBackRec r;
  r.tot = a.tot ? *a.tot : TopicOff{0, 0, 0, 0, 0};
  r.ovf = *a.ovf;
  r.fallback = a.fallback ? *a.fallback : 0u;
  r.unsafe = *a.unsafe;
  r.err = *a.err;
  for (int k = 0; k < 3; k++) r.n_sets[k] = a.n_sets ? a.n_sets[k] : 0ull;
  r.n_patches = np;
  r.set_total = a.set_total ? *a.set_total : 0ull;
  r.mrow_total = a.mrow_total ? *a.mrow_total : 0ull;
  *a.out = r;
  __threadfence_system();
}

void launch_readback(const ReadbackArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_readback, dim3(1), dim3(64), 0, s, a);
}

// The imported lists' offsets (XScanArgs): the u32 scan of k_scan32_* with one row of blocks per
// foreign shard (blockIdx.y), so the import costs three launches for any number of shards, and 4
// bytes per topic and shard where a TopicOff scan wrote 40.
__global__ __launch_bounds__(256) void k_xscan_reduce(XScanArgs a, uint64_t n, uint32_t nb, uint32_t* __restrict__ bsum) {
  __shared__ uint32_t wt[4];
  const uint32_t* in = a.in[blockIdx.y];
  const uint64_t st = a.stride[blockIdx.y] ? a.stride[blockIdx.y] : 1u;
  const uint64_t base = (uint64_t)blockIdx.x * kScanBlock + threadIdx.x * 4;
  uint32_t v = 0;
  for (int k = 0; k < 4; k++)
    if (base + k < n) v += in[(base + k) * st];
  v = block_scan_incl32(v, wt);
  if (threadIdx.x == 255) bsum[(uint64_t)blockIdx.y * (nb + 1) + blockIdx.x] = v;
}

__global__ __launch_bounds__(256) void k_xscan_blocks(uint32_t nb, const uint32_t* __restrict__ bsum,
                                                      uint32_t* __restrict__ bpre) {
  __shared__ uint32_t wt[4];
  __shared__ uint32_t carry;
  const uint64_t row = (uint64_t)blockIdx.x * (nb + 1);
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t b0 = 0; b0 < nb; b0 += 256) {
    const uint32_t b = b0 + threadIdx.x;
    const uint32_t v = b < nb ? bsum[row + b] : 0u;
    const uint32_t incl = block_scan_incl32(v, wt);
    if (b < nb) bpre[row + b] = carry + incl - v;
    __syncthreads();
    if (threadIdx.x == 255) carry += incl;
    __syncthreads();
  }
  if (threadIdx.x == 0) bpre[row + nb] = carry;
}

__global__ __launch_bounds__(256) void k_xscan_apply(XScanArgs a, uint64_t n, uint32_t nb,
                                                     const uint32_t* __restrict__ bpre) {
  __shared__ uint32_t wt[4];
  const uint32_t* in = a.in[blockIdx.y];
  uint32_t* out = a.out[blockIdx.y];
  if (!out) return;  // (block-uniform: a row whose total alone is wanted)
  const uint64_t st = a.stride[blockIdx.y] ? a.stride[blockIdx.y] : 1u;
  const uint64_t row = (uint64_t)blockIdx.y * (nb + 1);
  const uint64_t base = (uint64_t)blockIdx.x * kScanBlock + threadIdx.x * 4;
  uint32_t c[4], v = 0;
  for (int k = 0; k < 4; k++) {
    c[k] = base + k < n ? in[(base + k) * st] : 0u;
    v += c[k];
  }
  const uint32_t incl = block_scan_incl32(v, wt);
  uint32_t ex = bpre[row + blockIdx.x] + incl - v;
  for (int k = 0; k < 4; k++) {
    if (base + k < n) out[base + k] = ex;
    ex += c[k];
  }
  if (blockIdx.x == nb - 1 && threadIdx.x == 0) out[n] = bpre[row + nb];
}

void launch_xscan(const XScanArgs& a, uint32_t nf, uint64_t n, uint32_t* bsum, uint32_t* bpre, hipStream_t s) {
  if (!nf || !n) return;
  const uint32_t nb = (uint32_t)((n + kScanBlock - 1) / kScanBlock);
  hipLaunchKernelGGL(k_xscan_reduce, dim3(nb, nf), dim3(256), 0, s, a, n, nb, bsum);
  hipLaunchKernelGGL(k_xscan_blocks, dim3(nf), dim3(256), 0, s, nb, bsum, bpre);
  hipLaunchKernelGGL(k_xscan_apply, dim3(nb, nf), dim3(256), 0, s, a, n, nb, bpre);
}

__global__ __launch_bounds__(256) void k_xpack32(uint32_t n, uint32_t g_stride, const uint32_t* __restrict__ xcount,
                                                 const uint32_t* __restrict__ xoff,
                                                 const XEnt* __restrict__ xents, XEnt* __restrict__ ents, uint64_t cap,
                                                 uint32_t* unsafe, unsigned long long* total,
                                                 const uint32_t* __restrict__ gathers, TopicOff* gt) {
  const uint64_t all = xoff[n];
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t == 0) {
    total[0] = all;
    *gt = TopicOff{all, *gathers, 0, 0, 0};
    if (all > cap) atomicOr(unsafe, kUnsafeXEnts);
  }
  if (t >= n || all > cap) return;
  const uint32_t c = xcount[t];
  const uint64_t src = (uint64_t)t * g_stride, dst = xoff[t];
  for (uint32_t k = 0; k < c; k++) ents[dst + k] = xents[src + k];
}

void launch_xpack32(uint32_t n, uint32_t g_stride, const uint32_t* xcount, const uint32_t* xoff, const XEnt* xents,
                    XEnt* ents, uint64_t cap, uint32_t* unsafe, unsigned long long* total, const uint32_t* gathers,
                    TopicOff* gt, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_xpack32, dim3((n + 255) / 256), dim3(256), 0, s, n, g_stride, xcount, xoff, xents, ents, cap,
                     unsafe, total, gathers, gt);
}

}  // namespace mq
