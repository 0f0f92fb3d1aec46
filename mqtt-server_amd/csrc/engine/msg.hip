// gfx950 Messages: the particle walk k_msg, the level-order retained image and k_msgq (DESIGN.md
// §4.8).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>

#include "kern_common.h"

namespace mq {

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

// Thread per slot of the index's edge table (a grid-stride loop): an edge whose parent and child
// are both in the image becomes the image's edge (parent's image position, the same key) -> the
// child's image position. Every image particle but the root has exactly one such edge (short
// segments live only in the edge slots: NodeWalk.seg names long ones). A parent's children have
// distinct keys, so a slot is claimed once (CAS on the position pair); the keys follow the claim
// (no reader runs until the kernel ends).
__global__ __launch_bounds__(256) void k_img_edges(DevIndex ix, const uint32_t* __restrict__ node,
                                                   const uint32_t* __restrict__ pos, uint32_t n, uint32_t n_pos,
                                                   ImgEdge* __restrict__ edges, uint64_t mask) {
  auto in_img = [&](uint32_t c) __attribute__((always_inline)) -> uint32_t {
    if (c >= n_pos) return kNone;
    const uint32_t q = pos[c];
    return (q < n && node[q] == c) ? q : kNone;
  };
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i <= ix.edge_mask; i += (uint64_t)gridDim.x * 256) {
    const EdgeSlot e = ix.edges[i];
    if (e.parent >= kEdgeTomb) continue;  // a free slot
    const uint32_t qc = in_img(e.child);
    if (qc == kNone) continue;
    const uint32_t qp = in_img(e.parent);
    if (qp == kNone) continue;  // (not reached: an image particle's parent is in the image)
    const SegKey k{e.k0, e.k1};
    const unsigned long long want = (unsigned long long)qp | ((unsigned long long)qc << 32);
    uint64_t j = edge_slot(qp, k, mask);
    bool put = false;
    for (uint64_t probes = 0; probes <= mask && !put; probes++) {
      unsigned long long* w = reinterpret_cast<unsigned long long*>(&edges[j]);
      if (atomicCAS(w, ~0ull, want) == ~0ull) {
        edges[j].k0 = k.k0;
        edges[j].k1 = k.k1;
        put = true;
      }
      j = (j + 1) & mask;
    }
    if (!put) atomicOr(ix.err, kErrWalkGuard);  // (the table holds twice the particles: not reached)
  }
}

void launch_img_edges(const DevIndex& ix, const uint32_t* node, const uint32_t* pos, uint32_t n, uint32_t n_pos,
                      ImgEdge* edges, uint64_t mask, hipStream_t s) {
  if (n <= 1) return;
  const uint64_t slots = ix.edge_mask + 1;
  const uint32_t g = (uint32_t)std::min<uint64_t>((slots + 255) / 256, 65536);
  hipLaunchKernelGGL(k_img_edges, dim3(g), dim3(256), 0, s, ix, node, pos, n, n_pos, edges, mask);
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

// The image child of image particle u for segment (key, seg, len), or kNone: one probe of the
// image's edge table (a long segment's bytes compared as the index's lookup does), or — without
// the table — the index's edge table, then the child's image position.
__device__ __forceinline__ uint32_t img_child(const MsgImg& img, const DevIndex& ix, uint32_t u, const SegKey& k,
                                              const uint8_t* seg, uint32_t len) {
  if (!img.edges) return img_pos(img, lookup(ix, img.node[u], k, seg, len));
  uint64_t i = edge_slot(u, k, img.edge_mask);
  for (uint64_t probes = 0; probes <= img.edge_mask; probes++) {
    const ImgEdge e = img.edges[i];
    if (e.parent == kImgEdgeEmpty) break;
    if (e.parent == u && e.k0 == k.k0 && e.k1 == k.k1) {
      if (!seg_is_long(k)) return e.child;
      const SegInfo si = ix.seginfo[ix.walk[img.node[e.child]].seg];
      bool eq = si.len == len;
      for (uint32_t j = 0; eq && j < len; j++) eq = ix.segbytes[si.off + j] == seg[j];
      if (eq) return e.child;
    }
    i = (i + 1) & img.edge_mask;
  }
  return kNone;
}

// ---- the image's key index (round 6) -----------------------------------------------------------
// Every edge of the index's edge table between image particles, as (parent and child image
// positions, the key, its hash), in any order (k_kx_collect), then stably sorted by parent
// position and by key hash (hipcub radix sorts, gathers), so that one key's entries are contiguous
// and ordered by parent position. A workgroup per chunk of edge slots, two passes over it: count,
// one atomic for the chunk's range, write (one atomic per wavefront on a single counter took
// 98 ms at 10M retained: ~4M same-address atomics; the edge slots are sparse)
__global__ __launch_bounds__(256) void k_kx_collect(DevIndex ix, const uint32_t* __restrict__ node,
                                                    const uint32_t* __restrict__ pos, uint32_t n, uint32_t n_pos,
                                                    uint64_t chunk, uint32_t* __restrict__ par,
                                                    uint32_t* __restrict__ chd, uint64_t* __restrict__ k0,
                                                    uint64_t* __restrict__ k1, uint64_t* __restrict__ h,
                                                    uint32_t* __restrict__ perm,
                                                    unsigned long long* __restrict__ count) {
  __shared__ uint32_t wcnt[4];
  __shared__ unsigned long long base_s;
  auto in_img = [&](uint32_t c) __attribute__((always_inline)) -> uint32_t {
    if (c >= n_pos) return kNone;
    const uint32_t q = pos[c];
    return (q < n && node[q] == c) ? q : kNone;
  };
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint64_t slots = ix.edge_mask + 1;
  const uint64_t c0 = (uint64_t)blockIdx.x * chunk, c1 = min(slots, c0 + chunk);
  auto look = [&](uint64_t i, EdgeSlot& e, uint32_t& qc, uint32_t& qp) __attribute__((always_inline)) -> bool {
    qc = qp = kNone;
    if (i >= c1) return false;
    e = ix.edges[i];
    if (e.parent >= kEdgeTomb) return false;  // a free slot
    qc = in_img(e.child);
    if (qc == kNone) return false;
    qp = in_img(e.parent);
    return qp != kNone;
  };
  uint32_t c = 0;
  for (uint64_t i = c0 + threadIdx.x; i < c1; i += 256) {
    EdgeSlot e;
    uint32_t qc, qp;
    c += look(i, e, qc, qp) ? 1u : 0u;
  }
  c = wave_sum(c);
  if (lane == 0) wcnt[wv] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t tot = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    base_s = tot ? atomicAdd(count, (unsigned long long)tot) : 0ull;
  }
  __syncthreads();
  unsigned long long off = base_s;
  for (uint64_t i0 = c0; i0 < c1; i0 += 256) {  // (workgroup-uniform trip count)
    EdgeSlot e{};
    uint32_t qc, qp;
    const bool take = look(i0 + threadIdx.x, e, qc, qp);
    const uint64_t m = __ballot(take);
    __syncthreads();  // (the last round's counts are read)
    if (lane == 0) wcnt[wv] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = 0, tot = 0;
    for (uint32_t k = 0; k < 4; k++) {
      before += k < wv ? wcnt[k] : 0u;
      tot += wcnt[k];
    }
    if (take) {
      const uint32_t j = (uint32_t)(off + before + prefix_before(m));
      par[j] = qp;
      chd[j] = qc;
      k0[j] = e.k0;
      k1[j] = e.k1;
      h[j] = kx_hash(e.k0, e.k1);
      perm[j] = j;
    }
    off += tot;
  }
}

void launch_kx_collect(const DevIndex& ix, const uint32_t* node, const uint32_t* pos, uint32_t n, uint32_t n_pos,
                       uint32_t* par, uint32_t* chd, uint64_t* k0, uint64_t* k1, uint64_t* h, uint32_t* perm,
                       unsigned long long* count, hipStream_t s) {
  const uint64_t slots = ix.edge_mask + 1;
  const uint64_t chunk = std::max<uint64_t>(256, ((slots + 4095) / 4096 + 255) & ~255ull);  // ~4k workgroups
  const uint32_t g = (uint32_t)((slots + chunk - 1) / chunk);
  hipLaunchKernelGGL(k_kx_collect, dim3(g), dim3(256), 0, s, ix, node, pos, n, n_pos, chunk, par, chd, k0, k1, h,
                     perm, count);
}

size_t kx_sort_u32(void* temp, size_t temp_bytes, const uint32_t* kin, uint32_t* kout, const uint32_t* vin,
                   uint32_t* vout, uint32_t n, hipStream_t s) {
  size_t b = temp_bytes;
  (void)hipcub::DeviceRadixSort::SortPairs(temp, b, kin, kout, vin, vout, (int)n, 0, 32, s);
  return b;
}

size_t kx_sort_u64(void* temp, size_t temp_bytes, const uint64_t* kin, uint64_t* kout, const uint32_t* vin,
                   uint32_t* vout, uint32_t n, hipStream_t s) {
  size_t b = temp_bytes;
  (void)hipcub::DeviceRadixSort::SortPairs(temp, b, kin, kout, vin, vout, (int)n, 0, 64, s);
  return b;
}

template <class T>
__global__ __launch_bounds__(256) void k_kx_gather(const T* __restrict__ src, const uint32_t* __restrict__ perm,
                                                   T* __restrict__ dst, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) dst[i] = src[perm[i]];
}

void launch_kx_gather32(const uint32_t* src, const uint32_t* perm, uint32_t* dst, uint32_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_kx_gather<uint32_t>, dim3((n + 255) / 256), dim3(256), 0, s, src, perm, dst, n);
}

void launch_kx_gather64(const uint64_t* src, const uint32_t* perm, uint64_t* dst, uint32_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_kx_gather<uint64_t>, dim3((n + 255) / 256), dim3(256), 0, s, src, perm, dst, n);
}

// distinct key hashes (run starts of the sorted hashes), one atomic per wavefront
__global__ __launch_bounds__(256) void k_kx_count_keys(const uint64_t* __restrict__ h, uint32_t n,
                                                       unsigned long long* __restrict__ keys) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  const bool st = i < n && (i == 0 || h[i] != h[i - 1]);
  const uint32_t c = (uint32_t)__popcll(__ballot(st));
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(keys, (unsigned long long)c);
}

void launch_kx_count_keys(const uint64_t* h, uint32_t n, unsigned long long* keys, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_kx_count_keys, dim3((n + 255) / 256), dim3(256), 0, s, h, n, keys);
}

// a run of equal hashes [i, j) becomes one slot; the thread at the run's start walks to its end
// (runs are short: one key's parents — a hot key's run is long, but there is one per key)
__global__ __launch_bounds__(256) void k_kx_table(const uint64_t* __restrict__ h, uint32_t n, KxSlot* __restrict__ tab,
                                                  uint64_t mask, uint32_t* __restrict__ err) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n || (i != 0 && h[i] == h[i - 1])) return;
  const uint64_t k = h[i];
  // the run's end: doubling, then a binary search (sorted hashes)
  uint32_t lo = i, step = 1;
  while (lo + step < n && h[lo + step] == k) {
    lo += step;
    step *= 2;
  }
  uint32_t hi = min(n, lo + step);  // h[lo] == k, h[hi] != k or hi == n
  while (hi - lo > 1) {
    const uint32_t m = (lo + hi) >> 1;
    if (h[m] == k) lo = m;
    else hi = m;
  }
  uint64_t sl = mix64(k) & mask;
  for (uint64_t probes = 0; probes <= mask; probes++) {
    if (atomicCAS(reinterpret_cast<unsigned long long*>(&tab[sl].h), 0ull, (unsigned long long)k) == 0ull) {
      tab[sl].start = i;
      tab[sl].count = hi - i;
      return;
    }
    sl = (sl + 1) & mask;
  }
  atomicOr(err, kErrWalkGuard);  // (the table holds twice the keys: not reached)
}

void launch_kx_table(const uint64_t* h, uint32_t n, KxSlot* tab, uint64_t mask, uint32_t* err, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_kx_table, dim3((n + 255) / 256), dim3(256), 0, s, h, n, tab, mask, err);
}

// the key's entries [x, y) (x == y: no image edge has that key)
__device__ __forceinline__ uint2 kx_range(const MsgImg& img, const SegKey& k) {
  const uint64_t h = kx_hash(k.k0, k.k1);
  uint64_t sl = mix64(h) & img.kx_mask;
  for (uint64_t probes = 0; probes <= img.kx_mask; probes++) {
    const KxSlot e = img.kx_tab[sl];
    if (e.h == h) return make_uint2(e.start, e.start + e.count);
    if (e.h == 0) break;
    sl = (sl + 1) & img.kx_mask;
  }
  return make_uint2(0u, 0u);
}

// the first entry of [a, b) whose parent position is >= x (entries of one key hash are sorted by it)
__device__ __forceinline__ uint32_t kx_lower(const uint32_t* __restrict__ par, uint32_t a, uint32_t b, uint32_t x) {
  while (a < b) {
    const uint32_t m = (a + b) >> 1;
    if (par[m] < x) a = m + 1;
    else b = m;
  }
  return a;
}

// the same, the wave together (a, b, x wave-uniform; every lane calls): 64 samples a step narrow
// [a, b) 64-fold, so a search is a few dependent loads instead of one per halving
__device__ __forceinline__ uint32_t kx_lower_wave(const uint32_t* __restrict__ par, uint32_t a, uint32_t b, uint32_t x,
                                                  uint32_t lane) {
  while (b - a > 64) {
    const uint32_t step = (b - a + 63) / 64;
    const uint32_t i = a + lane * step;
    const uint32_t c = (uint32_t)__popcll(__ballot(i < b && par[i] < x));  // samples below x: a prefix
    if (c == 0) return a;
    const uint32_t na = a + (c - 1) * step + 1;  // the sample before the bound is below x,
    b = min(b, a + c * step);                    // the next one (or b) is not
    a = na;
  }
  const uint32_t i = a + lane;
  return a + (uint32_t)__popcll(__ballot(i < b && par[i] < x));
}

// entry j's child if its key is the segment's (a hash shared by two keys interleaves their
// entries; a long segment's bytes are compared as the edge lookups do), else kNone
__device__ __forceinline__ uint32_t kx_hit(const MsgImg& img, const DevIndex& ix, uint32_t j, const SegKey& k,
                                           const uint8_t* seg, uint32_t len) {
  if (img.kx_k0[j] != k.k0 || img.kx_k1[j] != k.k1) return kNone;
  const uint32_t c = img.kx_chd[j];
  if (!seg_is_long(k)) return c;
  const SegInfo si = ix.seginfo[ix.walk[img.node[c]].seg];
  bool eq = si.len == len;
  for (uint32_t i = 0; eq && i < len; i++) eq = ix.segbytes[si.off + i] == seg[i];
  return eq ? c : kNone;
}

struct MsgFrame {  // a fan-out in progress: particles [cur, end) still to take segment s
  uint32_t cur, end, s;
};

// Wavefront per filter. MODE (kernels.h MsgMode): kMsgCount counts the filter's handles and copy
// pieces; kMsgFill writes short runs and piece records at the offsets of the count pass's scan;
// kMsgRuns counts and records the runs (their output and piece offsets fixed by the same LDS
// cursors the fill pass uses); kMsgPlace places recorded runs without walking again — the
// filter's walk then runs once per batch instead of twice.
// k_msgq's parameters as they lie in the kernarg segment
struct MsgqParams {
  const uint8_t* fb;
  const uint64_t* fo;
  uint32_t n;
  DevIndex ix;
  MsgImg img;
  TopicCount* cnt;
  const TopicOff* off;
  MsgPiece* pieces;
  uint64_t* handles;
  uint64_t* base_out;
  uint32_t* count_out;
  MsgRun* runs;
  uint32_t run_cap;
  uint32_t* n_runs;
  MsgWide w;
};

// waves per SIMD asked of the register allocator, per pass (MQ_MSGQ_WAVES_RUNS / _OTHER: build-time
// A/B); the passes are latency-bound probe rounds, so occupancy pays while nothing spills
#ifndef MQ_MSGQ_WAVES_RUNS
#define MQ_MSGQ_WAVES_RUNS 6  // (r06/v: 80 VGPRs with 28 spilled, against 96 at 5 waves: count 0.378 -> 0.356 ms)
#endif
#ifndef MQ_MSGQ_WAVES_OTHER
#define MQ_MSGQ_WAVES_OTHER 1
#endif
constexpr int msgq_waves(int mode) { return mode == kMsgRuns ? MQ_MSGQ_WAVES_RUNS : MQ_MSGQ_WAVES_OTHER; }

template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(msgq_waves(MODE)))) void k_msgq(const uint8_t* __restrict__ fb, const uint64_t* __restrict__ fo,
                                              uint32_t n, DevIndex ix_, MsgImg img_,
                                              TopicCount* __restrict__ cnt, const TopicOff* __restrict__ off,
                                              MsgPiece* __restrict__ pieces, uint64_t* __restrict__ handles,
                                              uint64_t* __restrict__ base_out, uint32_t* __restrict__ count_out,
                                              MsgRun* __restrict__ runs, uint32_t run_cap,
                                              uint32_t* __restrict__ n_runs, MsgWide w_) {
  (void)ix_;
  (void)img_;
  (void)w_;
  const DevIndex& ix = kernarg_at<DevIndex>(offsetof(MsgqParams, ix));
  const MsgImg& img = kernarg_at<MsgImg>(offsetof(MsgqParams, img));
  const MsgWide& w = kernarg_at<MsgWide>(offsetof(MsgqParams, w));
  constexpr bool WIDE = MODE == kMsgWideCount || MODE == kMsgWideFill;  // exported work items
  constexpr bool FILL = MODE == kMsgFill || MODE == kMsgPlace || MODE == kMsgWideFill;  // the walk writes output
  constexpr bool RUNS = MODE == kMsgRuns;
  if (FILL && img.gate && *img.gate == 0u) return;  // (block-uniform: the batch's outputs do not fit)
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
  // runs at the boundary: every run one piece record (uncut), no handle copied
  const bool run_out = img.run_base != nullptr;
  // one piece record per kMsgPiece handles of a long run
  auto put_pieces = [&](uint32_t h0, uint32_t len, uint32_t dst, uint32_t slot) __attribute__((always_inline)) {
    if (run_out) {
      pieces[pbase + slot] = MsgPiece{h0, len, obase + dst};
      return;
    }
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
        if (r.len > kMsgDirect || run_out) put_pieces(r.h0, r.len, r.dst, r.pslot);
        else
          for (uint32_t j = 0; j < r.len; j++) handles[obase + r.dst + j] = img.h[r.h0 + j];
      }
      if (lane == 0) {
        base_out[t] = obase;
        count_out[t] = cnt[t].rows;
        if (run_out) {
          img.run_base[t] = pbase;
          img.run_cnt[t] = cnt[t].gathers;
        }
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
    const uint32_t npc = run_out ? 1u : len > kMsgDirect ? (len + kMsgPiece - 1) / kMsgPiece : 0u;
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
  // ent: [ra, rb) are key-index entries of the literal segment (ek, at els, elen bytes) just before
  // rs; each lane starts from its entries' children instead of from particles
  auto dfs_run = [&](uint32_t ra, uint32_t rb, uint64_t rs, bool ent, const SegKey& ek, uint64_t els,
                     uint32_t elen) __attribute__((always_inline)) {
    MsgFrame st[kMsgStack];
    for (uint32_t u = ra + lane; u < rb; u += 64) {
      uint32_t ua = u;
      if (ent) {
        ua = kx_hit(img, ix, u, ek, fb + els, elen);
        if (ua == kNone) continue;
      }
      uint32_t sp = 0, ub = ua + 1;
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
          const uint32_t qc = img_child(img, ix, ua, key, fb + us, len);
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
  // A literal segment under a run of several particles: the level-synchronous fan-out from the run
  // [fa, fbnd) at segment fs. The frontier is a list of runs [x, y) of one level, in LDS; every lane
  // takes particles of the same level, so a literal level's lookups are issued together with one
  // key for the wave, a '+' maps each run to its children's run, and a final '+' / '#' emits each
  // run. A frontier that outgrows its LDS falls back, run by run, to the per-lane walk (dfs_run:
  // lanes take a run's particles, each walks the rest of the filter alone with deeper fan-outs on
  // a frame stack). The filter's own count pass may export the fan-out to work items (MsgWide)
  // instead; an item runs the same fan-out from its run (the wide modes).
  bool exported = false;  // the count pass handed the filter's fan-out to work items (MsgWide)
  // entries: [fa, fbnd) is a range of the key index's entries for the literal segment at fs (an item
  // exported from a literal level that took the key index), not a run of particles
  auto fan_out = [&](uint32_t fa, uint32_t fbnd, uint64_t fs, bool entries) __attribute__((always_inline)) {
    uint2* cur = mfront[wv][0];
    uint2* nxt = mfront[wv][1];
    uint32_t nr = 1;
    wave_sync_lds();  // (the frontier's LDS is free)
    if (lane == 0) cur[0] = make_uint2(fa, fbnd);
    wave_sync_lds();
    uint64_t ls = fs;  // the segment the frontier's runs take next
    bool ent = entries;
    for (uint32_t guard = 0; guard < 4096; guard++) {
      const uint64_t e = find_slash(R, ls, b1);
      const bool last = e >= b1;
      const uint32_t len = (uint32_t)(e - ls);
      const uint32_t c0 = len == 1 ? R.at(ls) : 0u;
      uint32_t nn = 0;  // the next frontier's runs (wave-uniform)
      bool kx = false;  // a literal level through the key index (below)
      bool ent_level = false;  // ... whose runs are entry ranges already (an exported item's first level)
      SegKey lit_key{0, 0};  // ... its key (a frontier too wide for LDS walks on from its entries)
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
        lit_key = key;
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
        // wide runs (round 6): the key index — one table probe, the key's entries narrowed to the
        // frontier's span by two wave-wide searches, then per run the entries whose parent lies in
        // it (wave-wide searches one run after another, or a binary search per lane); the level's
        // work is then its hits. Taken when those searches take fewer dependent rounds than the
        // probes of every particle (64 a round)
        uint32_t ri0[kMsgFront / 64], ri1[kMsgFront / 64];
#pragma unroll
        for (uint32_t k = 0; k < kMsgFront / 64; k++) ri0[k] = ri1[k] = 0;
        uint32_t hits = 0;
        ent_level = ent;
        ent = false;
        kx = ent_level;
        if (ent_level) hits = tot;
        const uint32_t probe_rounds = (tot + 63) / 64;
        if (!ent_level && img.kx_tab != nullptr && probe_rounds > img.kx_min_rounds) {
          const uint2 kr = kx_range(img, key);
          const uint32_t n0 = kx_lower_wave(img.kx_par, kr.x, kr.y, cur[0].x, lane);
          const uint32_t n1 = kx_lower_wave(img.kx_par, n0, kr.y, cur[nr - 1].y, lane);
          const uint32_t span = n1 - n0;
          uint32_t wave_steps = 1;  // a wave-wide search over the span: 64 samples a step
          for (uint32_t m = span; m > 64; m = (m + 63) / 64) wave_steps++;
          // dependent rounds: the searches, then a load per hit (at most the span's entries)
          const uint32_t hit_rounds = (span + 63) / 64;
          const uint32_t wave_cost = 2 * nr * wave_steps + hit_rounds;
          const uint32_t lane_cost = 2 * (32 - __clz(span)) * ((nr + 63) / 64) + hit_rounds;
          if (nr <= 64 && wave_cost <= lane_cost && wave_cost < probe_rounds) {
            kx = true;
            for (uint32_t r = 0; r < nr; r++) {
              const uint2 ru = cur[r];
              const uint32_t a = kx_lower_wave(img.kx_par, n0, n1, ru.x, lane);
              const uint32_t b = kx_lower_wave(img.kx_par, a, n1, ru.y, lane);
              if (lane == r) {
                ri0[0] = a;
                ri1[0] = b;
              }
              hits += b - a;
            }
          } else if (lane_cost < probe_rounds) {
            kx = true;
#pragma unroll
            for (uint32_t k = 0; k < kMsgFront / 64; k++) {
              const uint32_t r = k * 64 + lane;
              uint32_t a = 0, b = 0;
              if (r < nr) {
                a = kx_lower(img.kx_par, n0, n1, cur[r].x);
                b = kx_lower(img.kx_par, a, n1, cur[r].y);
              }
              ri0[k] = a;
              ri1[k] = b;
              hits += wave_sum(b - a);
            }
          }
        }
        if (!FILL && img.work && lane == 0)
          atomicAdd(img.work + 0, (unsigned long long)(kx ? hits + 2 * nr : tot));  // (edge-table probes, or
                                                                                   //  hits + searches)
        wave_sync_lds();
        if ((RUNS || MODE == kMsgFill || MODE == kMsgPlace) && w.min_tot && (kx ? hits > w.min_hits : tot > w.min_tot)) {
          if (FILL) {  // the count pass exported from here: its items write the rest
            if (cnt[t].shared) break;
          } else {
            // the runs as items of at most kMsgChunk particles — or, through the key index, the
            // runs' entry ranges as items of at most kMsgChunk entries (one reservation for all)
            uint32_t nit = 0;
#pragma unroll
            for (uint32_t k = 0; k < kMsgFront / 64; k++) {
              const uint32_t r = k * 64 + lane;
              const uint32_t x = r < nr ? (kx ? ri0[k] : cur[r].x) : 0u, y = r < nr ? (kx ? ri1[k] : cur[r].y) : 0u;
              nit += wave_sum((y - x + kMsgChunk - 1) / kMsgChunk);
            }
            uint32_t ib = 0;
            if (lane == 0) ib = atomicAdd(w.n_items, nit);
            ib = __shfl(ib, 0, 64);
            if (ib + nit <= w.cap) {
              const uint32_t s_item = (uint32_t)(ls - b0) | (kx ? kMsgWorkEntries : 0u);
#pragma unroll
              for (uint32_t k = 0; k < kMsgFront / 64; k++) {
                const uint32_t r = k * 64 + lane;
                const uint32_t x = r < nr ? (kx ? ri0[k] : cur[r].x) : 0u, y = r < nr ? (kx ? ri1[k] : cur[r].y) : 0u;
                const uint32_t c = (y - x + kMsgChunk - 1) / kMsgChunk;
                uint32_t ct;
                const uint32_t ex = wave_excl_scan(c, lane, &ct);
                for (uint32_t j = 0; j < c; j++)
                  w.items[ib + ex + j] = MsgWork{t, x + j * kMsgChunk, (uint32_t)min((uint32_t)y, (uint32_t)(x + (j + 1) * kMsgChunk)),
                                                 s_item, 0u, 0u, 0u, kNone};
                ib += ct;
              }
              exported = true;
              break;
            }  // (the queue is full: this filter walks alone, as a fill walk will)
          }
        }
        if (kx && !ent_level) {  // the runs become their entry ranges, the prefix counts their entries
          wave_sync_lds();
          uint32_t htot = 0;
#pragma unroll
          for (uint32_t k = 0; k < kMsgFront / 64; k++) {
            const uint32_t r = k * 64 + lane;
            uint32_t ct;
            const uint32_t ex = wave_excl_scan(r < nr ? ri1[k] - ri0[k] : 0u, lane, &ct);
            if (r < nr) {
              mpre[wv][r] = htot + ex;
              cur[r] = make_uint2(ri0[k], ri1[k]);
            }
            htot += ct;
          }
          if (lane == 0) mpre[wv][nr] = htot;
          tot = htot;
          wave_sync_lds();
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
            const uint32_t u = cur[lo].x + (p - mpre[wv][lo]);  // (a particle, or with the key index an entry)
            qc = kx ? kx_hit(img, ix, u, key, fb + ls, len) : img_child(img, ix, u, key, fb + ls, len);
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
        if (ent_level) {  // (not reached: an item's entries are at most kMsgChunk <= kMsgFront hits)
          if (lane == 0) atomicOr(ix.err, kErrMsgNest);
          break;
        }
        // (through the key index the runs are entry ranges: the lanes walk on from their hits)
        if (!FILL && img.work && lane == 0) {
          uint32_t np = 0;
          for (uint32_t r = 0; r < nr; r++) np += cur[r].y - cur[r].x;
          atomicAdd(img.work + 1, 1ull);
          atomicAdd(img.work + 2, (unsigned long long)np);
        }
        for (uint32_t r = 0; r < nr; r++) {
          const uint2 ru = cur[r];
          if (kx) dfs_run(ru.x, ru.y, e + 1, true, lit_key, ls, len);
          else dfs_run(ru.x, ru.y, ls, false, lit_key, ls, len);
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
  };
  if (WIDE) {  // wavefront per exported item: its run, level-synchronous (fan_out)
    const uint32_t ni = min(*w.n_items, w.cap);
    const uint32_t wbase = (blockIdx.x * 4 + wv) * w.per_wave;  // (wide count: this wavefront's scratch)
    // (a fixed stride over the items: taking them from one shared counter was slower — 8,192
    // wavefronts contending on one atomic, and the wavefronts that took many overflowed their run
    // scratch, so the fill walked those items again: 1.83 -> 3.48 ms at 10M retained)
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
          if (r.len > kMsgDirect || run_out) put_pieces(r.h0, r.len, r.dst, r.pslot);
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
      fan_out(it.x, it.y, b0 + (it.s & ~kMsgWorkEntries), (it.s & kMsgWorkEntries) != 0);
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
        const uint32_t qc = img_child(img, ix, a, key, fb + s, len);
        if (qc == kNone) break;
        if (last) {
          if (lane == 0) emit(img.lp[qc], img.lp[qc + 1] - img.lp[qc]);
          break;
        }
        a = qc;
        b = qc + 1;
        s = e + 1;
      }
      if (fan) fan_out(a, b, s, false);
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
    if (run_out) {
      img.run_base[t] = pbase;
      img.run_cnt[t] = cnt[t].gathers;
    }
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

// Wavefront per piece: four 64-handle loads in flight per lane, then the stores.
__global__ __launch_bounds__(256) void k_msg_copy(const MsgPiece* __restrict__ pieces, uint64_t n,
                                                  const uint64_t* __restrict__ h, uint64_t* __restrict__ out,
                                                  const uint64_t* __restrict__ n_dev) {
  const uint32_t lane = threadIdx.x & 63;
  if (n_dev) n = *n_dev;  // (one-sync batches: the count on the device, 0 when the gate is shut)
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
  hipLaunchKernelGGL(k_msg_copy, dim3((unsigned)std::min<uint64_t>((n + 3) / 4, kMaxWaveBlocks)), dim3(256), 0, s, pieces, n, h, out,
                     (const uint64_t*)nullptr);
}

void launch_msg_copy_dev(const MsgPiece* pieces, const uint64_t* n_pieces, uint64_t cap_g, const uint64_t* h,
                         uint64_t* out, hipStream_t s) {
  if (!cap_g) return;
  hipLaunchKernelGGL(k_msg_copy, dim3((unsigned)std::min<uint64_t>((cap_g + 3) / 4, kMaxWaveBlocks)), dim3(256), 0, s,
                     pieces, cap_g, h, out, n_pieces);
}

__global__ __launch_bounds__(256) void k_msg_runs_of(uint32_t n, const uint64_t* __restrict__ base,
                                                     const uint32_t* __restrict__ count, MsgPiece* __restrict__ runs,
                                                     uint64_t* __restrict__ run_base, uint32_t* __restrict__ run_cnt) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t >= n) return;
  runs[t] = MsgPiece{(uint32_t)base[t], count[t], base[t]};
  run_base[t] = t;
  run_cnt[t] = 1u;
}

void launch_msg_runs_of(uint32_t n, const uint64_t* base, const uint32_t* count, MsgPiece* runs, uint64_t* run_base,
                        uint32_t* run_cnt, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_msg_runs_of, dim3((n + 255) / 256), dim3(256), 0, s, n, base, count, runs, run_base, run_cnt);
}

__global__ void k_msg_gate(const TopicOff* tot, uint64_t cap_rows, uint64_t cap_g, uint32_t* gate, uint64_t* n_pieces) {
  if (threadIdx.x != 0) return;
  const TopicOff t = *tot;
  const bool ok = t.rows <= cap_rows && t.g <= cap_g;
  gate[0] = ok ? 1u : 0u;
  *n_pieces = ok ? t.g : 0ull;
}

void launch_msg_gate(const TopicOff* tot, uint64_t cap_rows, uint64_t cap_g, uint32_t* gate, uint64_t* n_pieces,
                     hipStream_t s) {
  hipLaunchKernelGGL(k_msg_gate, dim3(1), dim3(64), 0, s, tot, cap_rows, cap_g, gate, n_pieces);
}


}  // namespace mq
