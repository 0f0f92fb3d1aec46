// Device side of the engine (device.h): HBM mirror + batch pipeline.
#include "device.h"
#include "mqmatch_dev.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <vector>

static_assert(mq::kTopicSetPatches == MQ_TOPIC_SET_PATCHES && mq::kSetRowBits == MQ_SET_ROW_BITS &&
                  mq::kPairMax == MQ_MERGE_ROWS_STRIDE,
              "set patch layout (include/mqmatch.h)");

namespace mq {

void hip_check(hipError_t e, const char* where) {
  if (e != hipSuccess) throw HipError{e, std::string(where) + ": " + hipGetErrorString(e)};
}

// ---- pooled pinned host memory (PinnedAlloc) ------------------------------------------------------
namespace {
std::mutex g_pin_mu;
std::multimap<size_t, void*> g_pin_free;  // capacity -> block
size_t g_pin_pooled = 0;
// Pooled pinned blocks are kept up to 4 GiB per process (a broker holds this much page-locked
// memory at most after large host-result batches); larger frees go back to the system.
constexpr size_t kPinMin = 64 << 10, kPinPoolCap = 4ull << 30;
// Small blocks (a result's arrays for a few topics) are carved from 8 MiB slabs and always
// pooled: a host result holds up to eight of them, and page-locking each one on its own costs
// about half a millisecond, which readers meeting for the first time would pay inside a match.
constexpr size_t kPinSlab = 8 << 20, kPinSmall = 256 << 10;
uint8_t* g_slab = nullptr;
size_t g_slab_left = 0;
size_t pin_cap(size_t bytes) {
  size_t c = kPinMin;
  while (c < bytes) c <<= 1;
  return c;
}
}  // namespace

namespace {
struct SlowLog {
  std::chrono::steady_clock::time_point t0;
  char buf[512];
  size_t len = 0;
};
thread_local SlowLog g_slow;
const double g_slow_ms = [] {
  const char* e = getenv("MQ_SLOW_MS");
  return e ? atof(e) : 0.0;
}();
}  // namespace

bool slow_on() { return g_slow_ms > 0; }
void slow_begin() {
  if (!slow_on()) return;
  g_slow.t0 = std::chrono::steady_clock::now();
  g_slow.len = 0;
  g_slow.buf[0] = 0;
}
void slow_mark(const char* what) {
  if (!slow_on() || g_slow.len + 48 >= sizeof(g_slow.buf)) return;
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - g_slow.t0).count();
  g_slow.len += (size_t)snprintf(g_slow.buf + g_slow.len, sizeof(g_slow.buf) - g_slow.len, " %s@%.2f", what, ms);
}
void slow_report(const char* call, double) {
  if (!slow_on()) return;
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - g_slow.t0).count();
  if (ms > g_slow_ms) fprintf(stderr, "mq slow: %s %.2f ms:%s\n", call, ms, g_slow.buf);
}

void* pinned_alloc(size_t bytes) {
  const size_t cap = pin_cap(bytes);
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pin_free.find(cap);
    if (it != g_pin_free.end()) {
      void* p = it->second;
      g_pin_free.erase(it);
      if (cap > kPinSmall) g_pin_pooled -= cap;
      return p;
    }
    if (cap <= kPinSmall) {
      if (g_slab_left < cap) {
        void* sp = nullptr;
        if (hipHostMalloc(&sp, kPinSlab, hipHostMallocDefault) != hipSuccess || !sp) throw std::bad_alloc();
        g_slab = static_cast<uint8_t*>(sp);  // (the rest of the old slab is left unused)
        g_slab_left = kPinSlab;
      }
      void* p = g_slab;
      g_slab += cap;
      g_slab_left -= cap;
      return p;
    }
  }
  void* p = nullptr;
  slow_mark("hipHostMalloc");
  if (hipHostMalloc(&p, cap, hipHostMallocDefault) != hipSuccess || !p) throw std::bad_alloc();
  slow_mark("pinned");
  return p;
}

void pinned_free(void* p, size_t bytes) {
  if (!p) return;
  const size_t cap = pin_cap(bytes);
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    if (cap <= kPinSmall) {  // a slab's block: back to the pool, always
      g_pin_free.emplace(cap, p);
      return;
    }
    if (g_pin_pooled + cap <= kPinPoolCap) {
      g_pin_free.emplace(cap, p);
      g_pin_pooled += cap;
      return;
    }
  }
  slow_mark("hipHostFree");
  (void)hipHostFree(p);
  slow_mark("freed-pinned");
}

void DevBuf::ensure(size_t b) {
  if (b <= bytes && p) return;
  // a buffer that grows again takes half as much again as asked: results and scratch that follow
  // a growing index (a batch's rows, patches, spans) would otherwise be reallocated at every step
  // of it, and each hipFree / hipMalloc stalls the process's other threads for milliseconds
  const size_t grown = p ? b + b / 2 : b;
  release();
  size_t nb = std::max<size_t>(grown, 256);
  hip_check(hipMalloc(&p, nb), "hipMalloc");
  bytes = nb;
}

void DevBuf::release() {
  if (p) (void)hipFree(p);
  p = nullptr;
  bytes = 0;
}

template <class T>
void DevMirror<T>::release() {
  if (d) (void)hipFree(d);
  d = nullptr;
  cap = 0;
  if (spare) (void)hipFree(spare);
  spare = nullptr;
  spare_bytes = 0;
}

void Stager::add(void* dst, const void* src, size_t n) {
  for (size_t o = 0; o < n; o += kScatterRun)
    runs.push_back(Run{(uint8_t*)dst + o, (const uint8_t*)src + o, std::min<size_t>(kScatterRun, n - o)});
  bytes += n;
}

template <class T>
bool DevMirror<T>::sync(Mirror<T>& m, hipStream_t s, uint64_t* uploaded, Stager& st) {
  const size_t n = m.size();
  bool full = m.all_dirty;
  if (!d || m.epoch != epoch || cap < n) {
    if (d) st.frees.push_back(d);
    d = nullptr;
    cap = 0;
    cap = std::max<size_t>(std::max(m.h.capacity(), n), 1);
    if (spare && spare_bytes >= cap * sizeof(T)) {  // made ahead, outside the handle lock
      d = static_cast<T*>(spare);
      cap = spare_bytes / sizeof(T);
      spare = nullptr;
      spare_bytes = 0;
    } else {
      slow_mark("mirror-realloc");
      hip_check(hipMalloc(&d, cap * sizeof(T)), "hipMalloc(mirror)");
      slow_mark("mirror-malloc");
    }
    epoch = m.epoch;
    full = true;
  }
  const size_t pp = Mirror<T>::per_page();
  const size_t npages = (n + pp - 1) / pp;
  if (!full) full = m.dirty_pages * 4 > npages * 3;  // mostly dirty: one plain copy
  if (full && n * sizeof(T) <= kStageWhole) {
    // a small array whole through the pinned staging buffer (copied on the host now, uploaded and
    // scattered with the dirty pages): no pageable copy to wait for under the handle lock
    if (n) st.add(d, m.h.data(), n * sizeof(T));
    *uploaded += n * sizeof(T);
    full = false;
  } else if (full) {
    // pieces of at most 1 GiB: one pageable H2D copy of a multi-GiB array (the 100M-retained
    // image has 10 GB arrays) is not relied on
    const size_t bytes = n * sizeof(T), piece = 1ull << 30;
    for (size_t o = 0; o < bytes; o += piece)
      hip_check(hipMemcpyAsync(reinterpret_cast<uint8_t*>(d) + o, reinterpret_cast<const uint8_t*>(m.h.data()) + o,
                               std::min(piece, bytes - o), hipMemcpyHostToDevice, s),
                "H2D mirror");
    *uploaded += bytes;
  } else {
    // runs of consecutive dirty pages, from the listed bitmap words in address order
    std::sort(m.dirty_words.begin(), m.dirty_words.end());
    size_t ra = 0, rb = 0;  // the open run: pages [ra, rb)
    auto flush = [&] {
      const size_t a = ra * pp, b = std::min(n, rb * pp);
      if (a < b) {
        st.add(d + a, m.h.data() + a, (b - a) * sizeof(T));
        *uploaded += (b - a) * sizeof(T);
      }
      ra = rb = 0;
    };
    for (uint32_t w : m.dirty_words) {
      uint64_t bits = m.dirty[w];
      while (bits) {
        const uint32_t lo = (uint32_t)__builtin_ctzll(bits);
        const uint64_t x = bits >> lo;
        const uint32_t len = ~x ? (uint32_t)__builtin_ctzll(~x) : 64u - lo;
        const size_t pa = (size_t)w * 64 + lo, pb = pa + len;
        if (rb != 0 && pa == rb) {
          rb = pb;
        } else {
          flush();
          ra = pa;
          rb = pb;
        }
        bits = lo + len >= 64 ? 0ull : bits & ~(((1ull << len) - 1) << lo);
      }
    }
    flush();
  }
  m.clear_dirty();
  return full;
}

// ---- profiler ----------------------------------------------------------------------------------
void Profiler::begin(hipStream_t s, const char* name) {
  if (!on_) return;
  if (walk_only_ && strcmp(name, "walk") != 0) {  // MQ_PROF_WALK: the walk's launches only
    cur_ = nullptr;
    return;
  }
  if (free_.empty()) {
    hipEvent_t e;
    hip_check(hipEventCreate(&e), "hipEventCreate");
    free_.push_back(e);
  }
  cur_ = free_.back();
  free_.pop_back();
  hip_check(hipEventRecord(cur_, s), "hipEventRecord");
}

void Profiler::end(const char* name, hipStream_t s) {
  if (!on_ || !cur_) return;
  if (free_.empty()) {
    hipEvent_t e;
    hip_check(hipEventCreate(&e), "hipEventCreate");
    free_.push_back(e);
  }
  hipEvent_t b = free_.back();
  free_.pop_back();
  hip_check(hipEventRecord(b, s), "hipEventRecord");
  pending_.push_back(Pending{name, cur_, b});
  cur_ = nullptr;
  if (pending_.size() > 4096) drain();
}

void Profiler::drain() {
  for (auto& p : pending_) {
    hip_check(hipEventSynchronize(p.b), "hipEventSynchronize");
    float ms = 0;
    hip_check(hipEventElapsedTime(&ms, p.a, p.b), "hipEventElapsedTime");
    auto it = std::find_if(totals_.begin(), totals_.end(), [&](const Total& t) { return t.name == p.name; });
    if (it == totals_.end()) {
      totals_.push_back(Total{p.name, 0, 0});
      it = totals_.end() - 1;
    }
    it->launches++;
    it->ms += ms;
    free_.push_back(p.a);
    free_.push_back(p.b);
  }
  pending_.clear();
}

void Profiler::count(const char* name, uint64_t n) {
  if (!on_) return;
  auto it = std::find_if(totals_.begin(), totals_.end(), [&](const Total& t) { return t.name == name; });
  if (it == totals_.end()) {
    totals_.push_back(Total{name, 0, 0});
    it = totals_.end() - 1;
  }
  it->launches += n;
}

int Profiler::read(mq_kernel_time* out, uint32_t cap) {
  drain();
  uint32_t n = 0;
  for (auto& t : totals_) {
    if (n >= cap) break;
    // A name the record cannot hold whole would reach the caller under another key.
    if (t.name.size() >= sizeof(out[n].name)) throw std::runtime_error("profile name too long: " + t.name);
    memset(&out[n], 0, sizeof(out[n]));
    strncpy(out[n].name, t.name.c_str(), sizeof(out[n].name) - 1);
    out[n].launches = t.launches;
    out[n].total_ms = t.ms;
    n++;
  }
  return (int)n;
}

void Profiler::reset() {
  drain();
  totals_.clear();
}

// ---- device --------------------------------------------------------------------------------------
Device::Device(int dev) : dev_(dev) {
  hip_check(hipSetDevice(dev_), "hipSetDevice");
  int cus = 0;
  hip_check(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev_), "hipDeviceGetAttribute");
  n_cus_ = (uint32_t)std::max(1, cus);
  chunk_rows_budget_ = kChunkRows;
  chunk_tail_ = kChunkTail;
  chunk_min_ = kChunkMin;
  copy_blocks_ = n_cus_ * kCopyBlocksPerCU;    // persistent grid of that many workgroups per CU
  merge_blocks_ = n_cus_ * kMergeBlocksPerCU;  // 0: one wavefront per topic
  msg_spec_bytes_ = kMsgSpecMB << 20;
}

bool Device::set_option(uint32_t opt, uint64_t v) {
  switch (opt) {
    case MQ_OPT_CHUNK_ROWS: chunk_rows_budget_ = v ? std::min<uint64_t>(v, kChunkRows) : kChunkRows; return true;
    case MQ_OPT_SUBBATCH_TOPICS: subbatch_topics_ = v ? (uint32_t)std::min<uint64_t>(v, 1u << 30) : kSubBatchTopics; return true;
    case MQ_OPT_MSG_SPEC_MB: msg_spec_bytes_ = v << 20; return true;
    case MQ_OPT_MSG_WAVES: msg_wpe_opt_ = (uint32_t)v; return true;
    case MQ_OPT_SERIAL: serial_ = v != 0; return true;
    case MQ_OPT_PATCH_CAP: patch_cap_init_ = std::max<uint64_t>(v, 64); return true;
    case MQ_OPT_MERGE_WAVES: merge_wpe_opt_ = (uint32_t)v; return true;
    case MQ_OPT_WALK_WAVES: walk_wpe_ = (uint32_t)v; return true;
    case MQ_OPT_WALK_LISTS: walk_lists_ = v != 0; return true;
    case MQ_OPT_MERGE_DEDUP: dedup_ = (uint32_t)v; return true;
    case MQ_OPT_SET_GRID: set_grid_ = (uint32_t)v; return true;
    case MQ_OPT_ONE_SYNC: one_sync_ = v != 0; return true;
    case MQ_OPT_FUSE_DESC: fuse_desc_ = v != 0; return true;
    case MQ_OPT_SET_EXP:
#ifndef MQ_DEV_BUILD
      if (v & 0xFu) return false;  // (bits 0-3 make results wrong: development builds only)
#endif
      set_exp_ = (uint32_t)v;
      return true;
    case MQ_OPT_MSG_EXPORT: msg_export_ = (uint32_t)v; return true;
    case MQ_OPT_WALK_GROUP:
      if (v != 0 && v != 16 && !(kDevBuild && (v == 4 || v == 8))) return false;  // (8 / 4: DEV=1 builds)
      walk_group_ = (uint32_t)v;
      walk_auto_ = false;  // (a fixed choice: no trials)
      return true;
    case MQ_OPT_MSG_IMAGE: msg_img_on_ = v != 0; return true;
    case MQ_OPT_PATCH_CODES: patch_codes_ = v != 0; return true;
    case MQ_OPT_MSG_KEYIDX:
      msg_kx_on_ = v != 0;
      msg_kx_min_ = v >= 2 ? (uint32_t)v : kKxMinRounds;
      img_version_ = ~0ull;  // (rebuilt with or without it)
      return true;
    case MQ_OPT_MSG_EDGES:
      msg_edges_on_ = v != 0;
      img_version_ = ~0ull;  // (the image is rebuilt, with or without its table)
      return true;
    case MQ_OPT_MSG_EDGE_BUDGET:
      msg_edge_budget_ = v ? (v << 20) : (8ull << 30);
      img_version_ = ~0ull;
      return true;
    case MQ_OPT_FAIL_NEXT: fail_next_ = (uint32_t)v; return true;
    case MQ_OPT_WALK_EXP:
      if (!kDevBuild && v) return false;  // (development builds only)
      walk_exp_ = (uint32_t)v;
      return true;
    default: return false;
  }
}

// Device buffers and mirrors release themselves (DevBuf / DevMirror destructors, run after this
// body with the device still selected); streams, events and pinned host blocks are freed here.
Device::~Device() {
  (void)hipSetDevice(dev_);
  try {
    flush_host_copy();  // a pipelined result still waiting for its copy gets it
  } catch (...) {
  }
  (void)hipDeviceSynchronize();  // no kernel of this index still reads a buffer freed below
  release_retired();
  if (stage_done_) (void)hipEventDestroy(stage_done_);
  pinned_free(h_stage_, h_stage_bytes_);
  pinned_free(h_stage_spare_, h_stage_spare_bytes_);
  if (h_fast_) (void)hipHostFree(h_fast_);
  for (int k = 0; k < 2; k++) {
    if (copy_done_[k]) (void)hipEventDestroy(copy_done_[k]);
    if (merge_done_[k]) (void)hipEventDestroy(merge_done_[k]);
    if (sb_done_[k]) (void)hipEventDestroy(sb_done_[k]);
    if (walk_ev_[k]) (void)hipEventDestroy(walk_ev_[k]);
  }
  if (side_done_) (void)hipEventDestroy(side_done_);
  for (HostStage& h : hst_) {
    if (h.packed) (void)hipEventDestroy(h.packed);
    if (h.copied) (void)hipEventDestroy(h.copied);
  }
  if (hcopy_) (void)hipStreamDestroy(hcopy_);
  if (side_) (void)hipStreamDestroy(side_);
  if (hstream_) (void)hipStreamDestroy(hstream_);
  if (wstream_) (void)hipStreamDestroy(wstream_);
  if (ev_in_) (void)hipEventDestroy(ev_in_);
  for (hipEvent_t e : ev_scan_) (void)hipEventDestroy(e);
  if (h_plan_) (void)hipHostFree(h_plan_);
  if (h_pin_) (void)hipHostFree(h_pin_);
  if (h_xsrc_) (void)hipHostFree(h_xsrc_);
  if (xsrc_done_) (void)hipEventDestroy(xsrc_done_);
}

uint64_t Device::device_bytes() const {
  uint64_t b = edges_.cap * sizeof(EdgeSlot) + walk_.cap * sizeof(NodeWalk) +
               lists_.cap * sizeof(NodeLists) + inls_.cap * sizeof(NodeInl) + msg_.cap * sizeof(NodeMsg) +
               seginfo_.cap * sizeof(SegInfo) + segbytes_.cap + subs_.cap * sizeof(SubRec) +
               shr_.cap * sizeof(ShrRec) + inl_.cap * sizeof(InlRec) + children_.cap * sizeof(ChildRec) +
               mref_.cap * sizeof(MergeRef) + mpart_.cap * sizeof(MergePart) +
               npair_.cap * sizeof(NodePair) + pent_.cap * sizeof(PairEnt) + plist_.cap * sizeof(PairSlot);
  for (const DevBuf* x : {&in_bytes_, &in_offs_, &counts_, &offs_, &bsum_, &bpre_, &gathers_, &desc_[0], &desc_[1],
                          &tiles_[0], &tiles_[1], &sp_res_, &sp_spans_, &sp_inl_, &sp_picked_, &sp_patches_})
    b += x->bytes;
  for (int k = 0; k < 2; k++)
    for (const DevBuf* x : {&rows_[k], &shr_rows_[k], &inl_rows_[k], &res_[k], &sel_rows_[k]}) b += x->bytes;
  return b;
}

namespace {
template <class T>
std::string cmp_mirror(const DevMirror<T>& dm, const Mirror<T>& m, const char* name) {
  const size_t bytes = m.size() * sizeof(T);
  if (!bytes) return "";
  if (!dm.d) return std::string(name) + ": not on the device";
  std::vector<uint8_t> buf(std::min<size_t>(bytes, 256ull << 20));
  const uint8_t* h = reinterpret_cast<const uint8_t*>(m.h.data());
  for (size_t o = 0; o < bytes; o += buf.size()) {
    const size_t k = std::min(buf.size(), bytes - o);
    hip_check(hipMemcpy(buf.data(), reinterpret_cast<const uint8_t*>(dm.d) + o, k, hipMemcpyDeviceToHost), "D2H verify");
    if (memcmp(buf.data(), h + o, k) != 0) {
      size_t i = 0;
      while (buf[i] == h[o + i]) i++;
      return std::string(name) + ": device differs from the host mirror at byte " + std::to_string(o + i) + " of " +
             std::to_string(bytes);
    }
  }
  return "";
}
}  // namespace

std::string Device::verify(Index& ix) {
  sync(ix, nullptr);
  hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  std::string r;
  if (r.empty()) r = cmp_mirror(edges_, ix.edges, "edges");
  if (r.empty()) r = cmp_mirror(walk_, ix.walk, "walk");
  if (r.empty()) r = cmp_mirror(lists_, ix.lists, "lists");
  if (r.empty()) r = cmp_mirror(inls_, ix.inls, "inls");
  if (r.empty()) r = cmp_mirror(msg_, ix.msg, "msg");
  if (r.empty()) r = cmp_mirror(seginfo_, ix.seginfo, "seginfo");
  if (r.empty()) r = cmp_mirror(segbytes_, ix.segbytes, "segbytes");
  if (r.empty()) r = cmp_mirror(subs_, ix.subs.m, "subs");
  if (r.empty()) r = cmp_mirror(mref_, ix.mref, "mref");
  if (r.empty()) r = cmp_mirror(mpart_, ix.mpart.m, "mpart");
  if (r.empty()) r = cmp_mirror(npair_, ix.npair, "npair");
  if (r.empty()) r = cmp_mirror(pent_, ix.pent.m, "pent");
  if (r.empty()) r = cmp_mirror(plist_, ix.plist.m, "plist");
  if (r.empty()) r = cmp_mirror(shr_, ix.shr.m, "shr");
  if (r.empty()) r = cmp_mirror(inl_, ix.inl.m, "inl");
  if (r.empty()) r = cmp_mirror(children_, ix.children.m, "children");
  if (r.empty() && ix.sharded()) r = cmp_mirror(xinfo_, ix.xinfo, "xinfo");
  if (r.empty() && ix.deep.size()) r = cmp_mirror(deep_, ix.deep, "deep");
  if (r.empty() && ix.deep_codes.size()) r = cmp_mirror(deep_codes_, ix.deep_codes, "deep_codes");
  return r;
}

void Device::sync(Index& ix, hipStream_t s) {
  hip_check(hipSetDevice(dev_), "hipSetDevice");
  sync_ix(ix, s);
  issue_staged(s);
  release_retired();
}

void Device::issue_staged(hipStream_t s) {
  if (!staged_runs_) return;
  slow_mark("issue");
  hip_check(hipMemcpyAsync(d_stage_.p, h_stage_, staged_bytes_, hipMemcpyHostToDevice, s), "H2D staging");
  launch_scatter(d_stage_.as<ScatterRun>(), staged_runs_, d_stage_.as<uint8_t>(), s);
  hip_check(hipGetLastError(), "k_scatter");
  hip_check(hipEventRecord(stage_done_, s), "hipEventRecord(stage)");
  staged_runs_ = 0;
  staged_bytes_ = 0;
  staged_pending_ = true;
}

void Device::wait_staged() {
  if (staged_pending_ && stage_done_) hip_check(hipEventSynchronize(stage_done_), "hipEventSynchronize(stage)");
  staged_pending_ = false;
}

void Device::sync_ix(Index& ix, hipStream_t s) {
  if (ix.version() == synced_version_ && edges_.d) return;
  if (staged_runs_) issue_staged(s);  // (a batch that failed before issuing its upload: now)
  ix.flush_merge();
  slow_mark("flushed");
  Stager& st = stager_;
  st.runs.clear();
  st.bytes = 0;
  bool direct = false;
  direct |= edges_.sync(ix.edges, s, &uploaded_, st);
  direct |= walk_.sync(ix.walk, s, &uploaded_, st);
  direct |= lists_.sync(ix.lists, s, &uploaded_, st);
  direct |= inls_.sync(ix.inls, s, &uploaded_, st);
  direct |= msg_.sync(ix.msg, s, &uploaded_, st);
  direct |= seginfo_.sync(ix.seginfo, s, &uploaded_, st);
  direct |= segbytes_.sync(ix.segbytes, s, &uploaded_, st);
  direct |= subs_.sync(ix.subs.m, s, &uploaded_, st);
  direct |= mref_.sync(ix.mref, s, &uploaded_, st);
  direct |= mpart_.sync(ix.mpart.m, s, &uploaded_, st);
  direct |= npair_.sync(ix.npair, s, &uploaded_, st);
  direct |= pent_.sync(ix.pent.m, s, &uploaded_, st);
  direct |= plist_.sync(ix.plist.m, s, &uploaded_, st);
  direct |= shr_.sync(ix.shr.m, s, &uploaded_, st);
  direct |= inl_.sync(ix.inl.m, s, &uploaded_, st);
  direct |= children_.sync(ix.children.m, s, &uploaded_, st);
  if (ix.sharded()) direct |= xinfo_.sync(ix.xinfo, s, &uploaded_, st);
  if (ix.deep.size()) {
    direct |= deep_.sync(ix.deep, s, &uploaded_, st);
    direct |= deep_codes_.sync(ix.deep_codes, s, &uploaded_, st);
  }
  slow_mark("mirrors");
  if (!st.runs.empty()) {  // one staging buffer: the run table, then each run's bytes
    const size_t table = (st.runs.size() * sizeof(ScatterRun) + 15) & ~size_t(15);
    const size_t need = table + st.bytes + 16 * st.runs.size();
    // (the last upload finished reading the pinned buffer: wait_staged, before the handle lock;
    // the event is recorded only once a scatter has used it, before that waiting returns at once)
    if (!stage_done_) hip_check(hipEventCreateWithFlags(&stage_done_, hipEventDisableTiming), "hipEventCreate");
    if (staged_pending_) hip_check(hipEventSynchronize(stage_done_), "hipEventSynchronize(stage)");
    if (h_stage_bytes_ < need) {
      pinned_free(h_stage_, h_stage_bytes_);
      if (h_stage_spare_ && h_stage_spare_bytes_ >= need) {  // (made ahead: prealloc)
        h_stage_ = h_stage_spare_;
        h_stage_bytes_ = h_stage_spare_bytes_;
        h_stage_spare_ = nullptr;
        h_stage_spare_bytes_ = 0;
      } else {
        slow_mark("stage-alloc");
        h_stage_ = pinned_alloc(need);
        h_stage_bytes_ = need;
      }
    }
    if (d_stage_.bytes < need && d_stage_spare_.bytes >= need) {
      std::swap(d_stage_.p, d_stage_spare_.p);
      std::swap(d_stage_.bytes, d_stage_spare_.bytes);
    }
    d_stage_.ensure(need);
    uint8_t* hs = static_cast<uint8_t*>(h_stage_);
    ScatterRun* tab = reinterpret_cast<ScatterRun*>(hs);
    size_t o = table;
    for (size_t k = 0; k < st.runs.size(); k++) {
      const Stager::Run& r = st.runs[k];
      o += ((uintptr_t)r.dst - o) & 15;  // source and destination agree mod 16
      memcpy(hs + o, r.src, r.bytes);
      tab[k] = ScatterRun{(uint64_t)(uintptr_t)r.dst, o, r.bytes};
      o += r.bytes;
    }
    // the upload itself (H2D of the staging buffer, k_scatter) is issued by issue_staged: after
    // the handle lock, on the batch's stream, ahead of its kernels
    staged_bytes_ = o;
    staged_runs_ = (uint32_t)st.runs.size();
  }
  if (!h_stage_) {  // the first sync (a whole upload): the staging buffers for the updates' dirty
    // pages, sized for ordinary update bursts, so that the first update after it does not
    // page-lock host memory under the handle lock (a few ms)
    constexpr size_t kStageInit = 4u << 20;
    h_stage_ = pinned_alloc(kStageInit);
    h_stage_bytes_ = kStageInit;
    d_stage_.ensure(kStageInit);
    if (!stage_done_) hip_check(hipEventCreateWithFlags(&stage_done_, hipEventDisableTiming), "hipEventCreate");
    // ... and the scatter kernel loaded by one empty run, so that the first update's sync does
    // not load its code object under the handle lock
    *static_cast<ScatterRun*>(h_stage_) = ScatterRun{(uint64_t)(uintptr_t)d_stage_.p, 0, 0};
    hip_check(hipMemcpyAsync(d_stage_.p, h_stage_, sizeof(ScatterRun), hipMemcpyHostToDevice, s), "H2D staging");
    launch_scatter(d_stage_.as<ScatterRun>(), 1, d_stage_.as<uint8_t>(), s);
    hip_check(hipGetLastError(), "k_scatter");
    hip_check(hipEventRecord(stage_done_, s), "hipEventRecord(stage)");
    staged_pending_ = true;
  }
  retained_len_ = ix.retained_len();
  empty_live_ = ix.empty_topic_live;
  empty_handle_ = ix.empty_topic_handle;
  synced_version_ = ix.version();
  sync_direct_ = direct;
  syncs_++;
}

template <class F>
void Device::each_mirror(const Index& ix, F f) const {
  Device* me = const_cast<Device*>(this);  // (f gets the mirrors; plan reads, prealloc writes)
  f(0, me->edges_, ix.edges);
  f(1, me->walk_, ix.walk);
  f(2, me->lists_, ix.lists);
  f(3, me->inls_, ix.inls);
  f(4, me->msg_, ix.msg);
  f(5, me->seginfo_, ix.seginfo);
  f(6, me->segbytes_, ix.segbytes);
  f(7, me->subs_, ix.subs.m);
  f(8, me->mref_, ix.mref);
  f(9, me->mpart_, ix.mpart.m);
  f(10, me->npair_, ix.npair);
  f(11, me->pent_, ix.pent.m);
  f(12, me->plist_, ix.plist.m);
  f(13, me->shr_, ix.shr.m);
  f(14, me->inl_, ix.inl.m);
  f(15, me->children_, ix.children.m);
  if (ix.sharded()) f(16, me->xinfo_, ix.xinfo);
  if (ix.deep.size()) {
    f(17, me->deep_, ix.deep);
    f(18, me->deep_codes_, ix.deep_codes);
  }
}

Device::SyncPlan Device::sync_plan(Index& ix) const {
  SyncPlan p;
  if (ix.version() == synced_version_ && edges_.d) return p;
  slow_mark("plan");
  ix.flush_merge();  // (the deferred merge-record rebuilds grow arrays too: mref follows subs)
  slow_mark("plan-flushed");
  size_t dirty = 0;
  each_mirror(ix, [&](int k, auto& dm, const auto& m) {
    using T = typename std::decay_t<decltype(m.h)>::value_type;
    const size_t b = dm.need_bytes(m);
    p.mirror[k] = b;
    if (b && dm.spare_bytes < b) p.any = true;
    const size_t whole = m.size() * sizeof(T);
    if ((b || m.all_dirty) && whole <= kStageWhole) dirty += whole;  // (whole through the staging)
    else if (!b && !m.all_dirty) dirty += m.dirty_pages * std::max<size_t>(Mirror<T>::per_page() * sizeof(T), 16);
  });
  // the staging buffers: the dirty pages, a run record and 16 B of alignment per page at most
  // (a run record and 16 B of alignment per 64 B page, or per kScatterRun of a whole array)
  p.stage = dirty ? dirty + dirty / 16 * (sizeof(ScatterRun) + 16) + 4096 : 0;
  if (p.stage > h_stage_bytes_ && p.stage > h_stage_spare_bytes_) p.any = true;
  if (p.stage > d_stage_.bytes && p.stage > d_stage_spare_.bytes) p.any = true;
  return p;
}

void Device::prealloc(const SyncPlan& p) {
  hip_check(hipSetDevice(dev_), "hipSetDevice");
  auto one = [&](auto& dm, size_t b) {
    if (!b || dm.spare_bytes >= b) return;
    if (dm.spare) (void)hipFree(dm.spare);
    dm.spare = nullptr;
    dm.spare_bytes = 0;
    hip_check(hipMalloc(&dm.spare, b), "hipMalloc(mirror spare)");
    dm.spare_bytes = b;
  };
  one(edges_, p.mirror[0]);
  one(walk_, p.mirror[1]);
  one(lists_, p.mirror[2]);
  one(inls_, p.mirror[3]);
  one(msg_, p.mirror[4]);
  one(seginfo_, p.mirror[5]);
  one(segbytes_, p.mirror[6]);
  one(subs_, p.mirror[7]);
  one(mref_, p.mirror[8]);
  one(mpart_, p.mirror[9]);
  one(npair_, p.mirror[10]);
  one(pent_, p.mirror[11]);
  one(plist_, p.mirror[12]);
  one(shr_, p.mirror[13]);
  one(inl_, p.mirror[14]);
  one(children_, p.mirror[15]);
  one(xinfo_, p.mirror[16]);
  one(deep_, p.mirror[17]);
  one(deep_codes_, p.mirror[18]);
  if (p.stage > h_stage_bytes_ && p.stage > h_stage_spare_bytes_) {
    pinned_free(h_stage_spare_, h_stage_spare_bytes_);
    h_stage_spare_ = nullptr;
    h_stage_spare_bytes_ = 0;
    h_stage_spare_ = pinned_alloc(p.stage);
    h_stage_spare_bytes_ = p.stage;
  }
  if (p.stage > d_stage_.bytes && p.stage > d_stage_spare_.bytes) d_stage_spare_.ensure(p.stage);
}

void Device::release_retired() {
  if (stager_.frees.empty()) return;
  slow_mark("retire-free");
  for (void* p : stager_.frees) (void)hipFree(p);
  stager_.frees.clear();
  slow_mark("retired");
}

void Device::begin_prepare() {
  (void)host_stream();  // (sets the device; creates the host-result streams on first use)
  wait_staged();
}

void Device::prepare(Index& ix, hipStream_t s) {
  // (host work under the handle lock: the caller set the device and waited for the last staged
  // upload first — begin_prepare — so that no HIP call here waits behind another thread's)
  sync_ix(ix, s);  // (arrays it replaced are freed by the batch, outside the lock: spans_begin)
  // an upload straight from the host image (pageable memory) may still read it: done before an
  // update can touch it
  if (sync_direct_) {
    hip_check(hipStreamSynchronize(s), "hipStreamSynchronize(prepare)");
    sync_direct_ = false;
  }
  IndexSnap& x = snap_;
  x.version = ix.version();
  x.sharded = ix.sharded();
  x.shard = ix.shard();
  x.inl_live = ix.inl.live != 0;
  x.n_nodes = ix.n_nodes();
  x.n_wild = ix.n_wild_nodes();
  x.subs_len = ix.subs.m.size();
  x.shr_len = ix.shr.m.size();
  x.max_sub_cap = ix.max_sub_cap();
  x.deep_live = ix.sharded() && ix.deep_live();
  x.di = dev_index(ix);
}

DevIndex Device::dev_index(const Index& ix) const {
  DevIndex d;
  d.edges = edges_.d;
  d.edge_mask = ix.edge_mask();
  d.walk = walk_.d;
  d.lists = lists_.d;
  d.inls = inls_.d;
  d.msg = msg_.d;
  d.seginfo = seginfo_.d;
  d.segbytes = segbytes_.d;
  d.subs = subs_.d;
  d.mref = mref_.d;
  d.mpart = mpart_.d;
  d.npair = npair_.d;
  d.pent = pent_.d;
  d.plist = plist_.d;
  d.shr = shr_.d;
  d.inl = inl_.d;
  d.children = children_.d;
  d.xinfo = ix.sharded() ? xinfo_.d : nullptr;
  d.deep = ix.sharded() && ix.deep_live() ? deep_.d : nullptr;
  d.deep_codes = d.deep ? deep_codes_.d : nullptr;
  d.deep_mask = d.deep ? ix.deep.size() - 1 : 0;
  d.retained_len = retained_len_;
  d.empty_topic_handle = empty_handle_;
  d.empty_topic_live = empty_live_ ? 1u : 0u;
  d.pad = 0;
  d.err = err_.as<uint32_t>();
  return d;
}

void Device::check_err(hipStream_t s) {
  uint32_t e = 0;
  hip_check(hipMemcpyAsync(&e, err_.p, sizeof(e), hipMemcpyDeviceToHost, s), "D2H err");
  hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
  if (e) {
    hip_check(hipMemsetAsync(err_.p, 0, sizeof(uint32_t), s), "hipMemsetAsync(err)");
    throw HipError{hipErrorUnknown, std::string("device guard tripped: ") +
                                        ((e & kErrWalkGuard) ? "walk iteration bound " : "") +
                                        ((e & kErrTableFull) ? "merge table full " : "") +
                                        ((e & kErrPickGuard) ? "shared pick partitions " : "") +
                                        ((e & kErrDeepRank) ? "cross-shard rank tie without a deep-path entry" : "")};
  }
}

void Device::select_shared(const mq_match_result& r, hipStream_t s, ShrRec* d_sel, uint32_t* d_n) {
  if (!err_.p) throw HipError{hipErrorNotReady, "select_shared before any match"};
  PickArgs pa;
  pa.res = reinterpret_cast<const mq_topic_result_dev*>(r.topics);
  pa.rows = reinterpret_cast<const ShrRec*>(r.shared_rows);
  pa.sres = nullptr;
  pa.spans = nullptr;
  pa.pool = nullptr;
  pa.sel = d_sel;
  pa.n_out = d_n;
  pa.n_out_stride = 1;
  pa.n = r.n_topics;
  pa.err = err_.as<uint32_t>();
  launch_pick(pa, s);
  hip_check(hipGetLastError(), "k_pick");  // the guard flag is reported by the next match
}

void Device::stage_inputs(const uint8_t* tb, const uint64_t* to, uint32_t n, hipStream_t s,
                          const uint8_t** d_tb, const uint64_t** d_to) {
  hip_check(hipSetDevice(dev_), "hipSetDevice");
  const uint64_t nbytes = to[n];
  in_bytes_.ensure(nbytes + 16);
  in_offs_.ensure((n + 1) * sizeof(uint64_t));
  if (nbytes) hip_check(hipMemcpyAsync(in_bytes_.p, tb, nbytes, hipMemcpyHostToDevice, s), "H2D topics");
  hip_check(hipMemcpyAsync(in_offs_.p, to, (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, s),
            "H2D offsets");
  *d_tb = in_bytes_.as<uint8_t>();
  *d_to = in_offs_.as<uint64_t>();
}

// Grow a scratch buffer between launches of one batch: earlier launches may still read the old
// allocation, so the device drains first (rare: buffers only grow).
static void grow(DevBuf& b, size_t bytes) {
  if (bytes <= b.bytes && b.p) return;
  slow_mark("grow");
  if (b.p) hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize(grow)");
  b.ensure(bytes);
  slow_mark("grown");
}

hipStream_t Device::host_stream() {
  hip_check(hipSetDevice(dev_), "hipSetDevice");
  slow_mark("hs-setdev");
  if (!hstream_) {
    // the copy stream right after it: streams share the device's few hardware queues (4 by
    // default), and a copy stream on the host stream's queue would run each batch's result copy
    // in line with the next batch's kernels (measured: a pipelined submit waited for the previous
    // batch's whole copy when bench.py's other streams had been created between the two)
    hip_check(hipStreamCreateWithFlags(&hstream_, hipStreamNonBlocking), "hipStreamCreate");
    ensure_hcopy();
  }
  return hstream_;
}

void Device::issue_host_copy(const PendingCopy& c) {
  HostStage* hs = c.hs;
  HostSpans* host = c.host;
  hip_check(hipStreamWaitEvent(hcopy_, hs->packed, 0), "hipStreamWaitEvent");
  const size_t pw = c.codes ? sizeof(uint32_t) : sizeof(PatchRec);  // bytes per patch
  auto d2h = [&](void* dst, const DevBuf& src, size_t bytes) {
    if (bytes) hip_check(hipMemcpyAsync(dst, src.p, bytes, hipMemcpyDeviceToHost, hcopy_), "D2H");
  };
  d2h(host->topics.data(), hs->topics, (size_t)c.n * sizeof(TopicSpansDev));
  d2h(host->spans.data(), hs->spans, c.spans * sizeof(SpanRec));
  d2h(c.codes ? (void*)host->patch_codes.data() : (void*)host->patches.data(), hs->patches, c.patches * pw);
  d2h(host->inl.data(), hs->inl, c.inl * sizeof(InlRec));
  d2h(host->picked.data(), hs->picked, c.picked * sizeof(ShrRec));
  if (c.dedup) {  // the sets' written patches and the merge rows (packed by k_set_pack, k_mrow_pack)
    d2h(c.codes ? (void*)host->set_codes.data() : (void*)host->set_patches.data(), hs->set_patches, c.set * pw);
    d2h(host->merge_rows.data(), hs->merge_rows, c.mrows * sizeof(uint32_t));
    d2h(host->merge_base.data(), hs->merge_base, (size_t)c.n * sizeof(uint32_t));
  }
  hip_check(hipEventRecord(hs->copied, hcopy_), "hipEventRecord");
  if (c.ready) hip_check(hipEventRecord(c.ready, hcopy_), "hipEventRecord");
  if (c.issued) c.issued->store(true);
}

void Device::flush_host_copy() {
  if (!pc_.on) return;
  hip_check(hipSetDevice(dev_), "hipSetDevice");
  const PendingCopy c = pc_;
  pc_.on = false;
  issue_host_copy(c);
}

void Device::ensure_hcopy() {
  if (hcopy_) return;
  // the copy stream at the high priority: the runtime keeps separate hardware queues per priority,
  // so no kernel stream of this process (ours, or a framework's) shares the copies' queue
  int least = 0, greatest = 0;
  hip_check(hipDeviceGetStreamPriorityRange(&least, &greatest), "hipDeviceGetStreamPriorityRange");
  hip_check(hipStreamCreateWithPriority(&hcopy_, hipStreamNonBlocking, greatest), "hipStreamCreate");
  for (HostStage& h : hst_) {
    hip_check(hipEventCreateWithFlags(&h.packed, hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventCreateWithFlags(&h.copied, hipEventDisableTiming), "hipEventCreate");
  }
}

void Device::ensure_streams() {
  if (side_) return;
  hip_check(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking), "hipStreamCreate");
  hip_check(hipStreamCreateWithFlags(&wstream_, hipStreamNonBlocking), "hipStreamCreate");
  for (int k = 0; k < 2; k++) {
    hip_check(hipEventCreateWithFlags(&copy_done_[k], hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventCreateWithFlags(&merge_done_[k], hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventCreateWithFlags(&sb_done_[k], hipEventDisableTiming), "hipEventCreate");
  }
  hip_check(hipEventCreateWithFlags(&side_done_, hipEventDisableTiming), "hipEventCreate");
  hip_check(hipEventCreateWithFlags(&ev_in_, hipEventDisableTiming), "hipEventCreate");
}

void Device::pinned(size_t bytes) {
  if (bytes <= h_pin_bytes_) return;
  if (h_pin_) {
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize(pinned)");
    (void)hipHostFree(h_pin_);
  }
  h_pin_bytes_ = std::max<size_t>(bytes, 1 << 16);
  hip_check(hipHostMalloc(&h_pin_, h_pin_bytes_, hipHostMallocDefault), "hipHostMalloc");
}

// The batch is cut into scan-block aligned sub-batches. Walk + scan of every sub-batch are queued
// up front on the walk stream; the host plans sub-batch b's output chunks as soon as its scan
// lands and queues k_desc/k_copy (launch stream) and k_merge (side stream), so the walks of the
// later sub-batches run under the copies of the earlier ones.
void Device::match(Index& ix, const uint8_t* d_tb, const uint64_t* d_to, uint32_t n, hipStream_t s,
                   HostMatch* host, mq_match_result* out, mq_chunk_fn fn, void* user) {
  hip_check(hipSetDevice(dev_), "hipSetDevice");
  sync(ix, s);
  memset(out, 0, sizeof(*out));
  last_chunks_ = 0;
  if (host) *host = HostMatch{};
  if (!err_.p) {
    err_.ensure(2 * sizeof(uint32_t));
    hip_check(hipMemsetAsync(err_.p, 0, 2 * sizeof(uint32_t), s), "hipMemsetAsync(err)");
  }
  check_err(s);  // faults flagged by the previous batch's kernels
  if (n == 0) return;
  ensure_streams();
  const DevIndex di = dev_index(ix);

  struct Sub {
    uint32_t t0, n, nb, blk0;  // first topic, topics, scan blocks, first scan block of the batch
  };
  const uint32_t sbt = std::max(kScanBlock, subbatch_topics_ / kScanBlock * kScanBlock);
  const uint32_t S = (n + sbt - 1) / sbt;
  std::vector<Sub> sub(S);
  uint32_t nb_all = 0;
  for (uint32_t b = 0; b < S; b++) {
    sub[b].t0 = b * sbt;
    sub[b].n = std::min(n - b * sbt, sbt);
    sub[b].nb = (sub[b].n + kScanBlock - 1) / kScanBlock;
    sub[b].blk0 = nb_all;
    nb_all += sub[b].nb;
  }
  // sub-batch b: offsets at offs_ + t0 + b (n + 1 entries), block sums at blk0 + b (nb + 1)
  grow(counts_, (size_t)n * sizeof(TopicCount));
  grow(offs_, (size_t)(n + S) * sizeof(TopicOff));
  grow(bsum_, (size_t)(nb_all + S) * sizeof(TopicOff));
  grow(bpre_, (size_t)(nb_all + S) * sizeof(TopicOff));
  grow(gslots_, (size_t)n * kGatherCap * sizeof(uint32_t));
  grow(ovf_, (size_t)S * sizeof(uint32_t));
  pinned((size_t)(nb_all + S) * sizeof(TopicOff) + S * sizeof(uint32_t));
  const size_t plan_bytes = (size_t)nb_all * (sizeof(ChunkPlan) + sizeof(uint32_t));  // <= one chunk per block
  grow(plan_, plan_bytes);
  if (plan_bytes > h_plan_bytes_) {
    if (h_plan_) {
      hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize(plan)");
      (void)hipHostFree(h_plan_);
    }
    h_plan_bytes_ = std::max<size_t>(plan_bytes, 1 << 16);
    hip_check(hipHostMalloc(&h_plan_, h_plan_bytes_, hipHostMallocDefault), "hipHostMalloc");
  }
  TopicOff* h_bpre = static_cast<TopicOff*>(h_pin_);
  uint32_t* h_ovf = reinterpret_cast<uint32_t*>(h_bpre + nb_all + S);
  while (ev_scan_.size() < S) {
    hipEvent_t e;
    hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    ev_scan_.push_back(e);
  }
  hip_check(hipMemsetAsync(ovf_.p, 0, S * sizeof(uint32_t), s), "hipMemsetAsync(ovf)");
  hip_check(hipEventRecord(ev_in_, s), "hipEventRecord");  // inputs + the previous batch are done
  hip_check(hipStreamWaitEvent(wstream_, ev_in_, 0), "hipStreamWaitEvent");
  for (uint32_t b = 0; b < S; b++) {
    const Sub& q = sub[b];
    TopicOff* off_b = offs_.as<TopicOff>() + q.t0 + b;
    prof.begin(wstream_, "walk");
    launch_walk(false, true, walk_wpe_, d_tb, d_to + q.t0, q.n, di, counts_.as<TopicCount>() + q.t0, nullptr,
                gslots_.as<uint32_t>() + (size_t)q.t0 * kGatherCap, ovf_.as<uint32_t>() + b, wstream_);
    prof.end("walk", wstream_);
    hip_check(hipGetLastError(), "k_walk<count>");
    prof.begin(wstream_, "scan");
    launch_scan(counts_.as<TopicCount>() + q.t0, q.n, bsum_.as<TopicOff>() + q.blk0 + b,
                bpre_.as<TopicOff>() + q.blk0 + b, off_b, wstream_);
    prof.end("scan", wstream_);
    hip_check(hipGetLastError(), "k_scan");
    hip_check(hipMemcpyAsync(h_bpre + q.blk0 + b, bpre_.as<TopicOff>() + q.blk0 + b, (q.nb + 1) * sizeof(TopicOff),
                             hipMemcpyDeviceToHost, wstream_), "D2H block offsets");
    hip_check(hipMemcpyAsync(h_ovf + b, ovf_.as<uint32_t>() + b, sizeof(uint32_t), hipMemcpyDeviceToHost, wstream_),
              "D2H overflow");
    hip_check(hipEventRecord(ev_scan_[b], wstream_), "hipEventRecord");
  }

  // host results need every sub-batch's totals first (global row offsets)
  std::vector<TopicOff> base(S + 1, TopicOff{0, 0, 0, 0, 0});
  if (host) {
    hip_check(hipStreamSynchronize(wstream_), "hipStreamSynchronize");
    for (uint32_t b = 0; b < S; b++) {
      base[b + 1] = base[b];
      const TopicOff& t = h_bpre[sub[b].blk0 + b + sub[b].nb];
      base[b + 1].rows += t.rows;
      base[b + 1].shr += t.shr;
      base[b + 1].inl += t.inl;
    }
    host->topics.resize(n);
    host->rows.resize(base[S].rows);
    host->shr.resize(base[S].shr);
    host->inl.resize(base[S].inl);
  }

  struct Chunk {
    uint32_t sb, b0, b1;  // sub-batch, scan-block range within it
  };
  std::vector<Chunk> done;
  auto tiles_of = [](uint64_t rows) { return (rows + kCopyTile - 1) / kCopyTile; };
  size_t ci = 0;
  for (uint32_t sb = 0; sb < S; sb++) {
    const Sub& q = sub[sb];
    const uint32_t p = sb & 1;
    hip_check(hipEventSynchronize(ev_scan_[sb]), "hipEventSynchronize");
    const TopicOff* hb = h_bpre + q.blk0 + sb;
    const TopicOff tot = hb[q.nb];
    const TopicOff* off_b = offs_.as<TopicOff>() + q.t0 + sb;
    prof.count("topics", q.n);
    prof.count("gathers", tot.g);
    prof.count("reserved_rows", tot.rows);
    hip_check(hipStreamWaitEvent(s, ev_scan_[sb], 0), "hipStreamWaitEvent");
    // sub-batch sb reuses the desc / tile / plan buffers of sb - 2 once its merges are done
    if (sb >= 2) hip_check(hipStreamWaitEvent(s, sb_done_[p], 0), "hipStreamWaitEvent");

    // A topic with more gathers than its count-pass slots: write all gather lists compactly.
    const uint32_t* gathers = gslots_.as<uint32_t>() + (size_t)q.t0 * kGatherCap;
    uint32_t gstride = kGatherCap;
    if (h_ovf[sb]) {
      grow(gathers_, std::max<uint64_t>(tot.g, 1) * sizeof(uint32_t));
      prof.begin(s, "walk_fill");
      launch_walk(true, true, walk_wpe_, d_tb, d_to + q.t0, q.n, di, nullptr, off_b, gathers_.as<uint32_t>(), nullptr, s);
      prof.end("walk_fill", s);
      hip_check(hipGetLastError(), "k_walk<fill>");
      gathers = gathers_.as<uint32_t>();
      gstride = 0;
    }

    // Plan output chunks on scan-block boundaries, each within the row budget. The merge of the
    // last chunk runs alone after every copy, so the rows are cut into equal main chunks plus a
    // last one of about budget / chunk_tail rows: the exposed tail is that small chunk's merge.
    std::vector<Chunk> chunks;
    std::vector<ChunkPlan> plan;
    std::vector<uint32_t> chunk_of_block(q.nb);
    uint64_t max_rows = 1, max_shr = 1, max_inl = 1, max_topics = 1, total_tiles = 0;
    // at least chunk_min_ chunks (so merges overlap copies) unless chunks would get small
    uint64_t target = std::min<uint64_t>(chunk_rows_budget_,
                                         std::max<uint64_t>(tot.rows / std::max(1u, chunk_min_) + 1, kChunkRowsMin));
    if (tot.rows > target && chunk_tail_ > 1) {
      const uint64_t main_rows = tot.rows - target / chunk_tail_;
      const uint64_t n_main = (main_rows + target - 1) / target;
      target = (main_rows + n_main - 1) / n_main;
    }
    for (uint32_t b = 0; b < q.nb;) {
      uint32_t e = b + 1;
      const uint64_t remaining = tot.rows - hb[b].rows;
      const uint64_t cap = chunk_tail_ > 1 && remaining <= target + target / chunk_tail_
                               ? std::min<uint64_t>(remaining, chunk_rows_budget_)
                               : target;
      while (e < q.nb && hb[e + 1].rows - hb[b].rows <= cap) e++;
      const TopicOff &lo = hb[b], &hi = hb[e];
      for (uint32_t k = b; k < e; k++) chunk_of_block[k] = (uint32_t)chunks.size();
      chunks.push_back(Chunk{sb, b, e});
      ChunkPlan cp;
      cp.rows = lo.rows;
      cp.shr = lo.shr;
      cp.inl = lo.inl;
      cp.tile_off = (uint32_t)total_tiles;
      cp.n_tiles0 = (uint32_t)tiles_of(hi.rows - lo.rows);
      cp.n_tiles1 = (uint32_t)tiles_of(hi.shr - lo.shr);
      cp.pad = 0;
      plan.push_back(cp);
      max_rows = std::max(max_rows, hi.rows - lo.rows);
      max_shr = std::max(max_shr, hi.shr - lo.shr);
      max_inl = std::max(max_inl, hi.inl - lo.inl);
      total_tiles += tiles_of(hi.rows - lo.rows) + tiles_of(hi.shr - lo.shr) + tiles_of(hi.inl - lo.inl);
      max_topics = std::max<uint64_t>(max_topics, std::min<uint64_t>(q.n, (uint64_t)e * kScanBlock) - (uint64_t)b * kScanBlock);
      b = e;
    }
    if (max_rows >= (1ull << 32) || max_shr >= (1ull << 32) || max_inl >= (1ull << 32) || total_tiles >= (1ull << 32))
      throw HipError{hipErrorInvalidValue, "one scan block's output exceeds 2^32 rows"};
    for (size_t k = 0; k < 2; k++) {
      grow(rows_[k], max_rows * sizeof(SubRec));
      grow(shr_rows_[k], max_shr * sizeof(ShrRec));
      grow(inl_rows_[k], max_inl * sizeof(InlRec));
      grow(res_[k], max_topics * sizeof(mq_topic_result_dev));
    }
    grow(desc_[p], std::max<uint64_t>(tot.g, 1) * sizeof(GDesc));
    grow(tiles_[p], std::max<uint64_t>(total_tiles, 1) * sizeof(uint32_t));
    // plans of every sub-batch have their own slots (the host runs ahead of the launch stream,
    // so a pinned slot must not be rewritten before its H2D copy has run)
    ChunkPlan* hp = static_cast<ChunkPlan*>(h_plan_) + q.blk0;
    uint32_t* hc = reinterpret_cast<uint32_t*>(static_cast<ChunkPlan*>(h_plan_) + nb_all) + q.blk0;
    ChunkPlan* dp = plan_.as<ChunkPlan>() + q.blk0;
    uint32_t* dc = reinterpret_cast<uint32_t*>(plan_.as<ChunkPlan>() + nb_all) + q.blk0;
    memcpy(hp, plan.data(), plan.size() * sizeof(ChunkPlan));
    memcpy(hc, chunk_of_block.data(), q.nb * sizeof(uint32_t));
    hip_check(hipMemcpyAsync(dp, hp, plan.size() * sizeof(ChunkPlan), hipMemcpyHostToDevice, s), "H2D chunk plan");
    hip_check(hipMemcpyAsync(dc, hc, q.nb * sizeof(uint32_t), hipMemcpyHostToDevice, s), "H2D chunk map");

    // every topic's gathers become GDesc records and k_copy tile starts, in one launch
    DescArgs da;
    memset(&da, 0, sizeof(da));
    da.ix = di;
    da.n = q.n;
    da.gather_stride = gstride;
    da.off = off_b;
    da.gathers = gathers;
    da.plan = dp;
    da.chunk_of_block = dc;
    da.desc = desc_[p].as<GDesc>();
    da.tiles = tiles_[p].as<uint32_t>();
    da.spans = nullptr;
    da.inl_out = nullptr;
    da.tc_out = nullptr;
    da.msig = nullptr;
    da.mrank = nullptr;
    da.unsafe = nullptr;
    prof.begin(s, "desc");
    launch_desc(da, false, s);
    prof.end("desc", s);
    hip_check(hipGetLastError(), "k_desc");

    // Per chunk: k_copy on the launch stream, then k_merge (and, for host results, the D2H
    // copies) on the side stream. Chunk i + 2 reuses chunk i's buffers after its merge.
    hipStream_t ms = serial_ ? s : side_;
    for (size_t cj = 0; cj < chunks.size(); cj++, ci++) {
      const Chunk& c = chunks[cj];
      const size_t b = ci & 1;
      const TopicOff& lo = hb[c.b0];
      const TopicOff& hi = hb[c.b1];
      EmitArgs a;
      memset(&a, 0, sizeof(a));  // (every field the row format does not use: null / zero)
      a.ix = di;
      a.t0 = c.b0 * kScanBlock;
      a.t1 = std::min<uint64_t>(q.n, (uint64_t)c.b1 * kScanBlock);
      a.off = off_b;
      a.base = lo;
      a.desc = desc_[p].as<GDesc>();
      a.tiles = tiles_[p].as<uint32_t>() + plan[cj].tile_off;
      a.total[0] = (uint32_t)(hi.rows - lo.rows);
      a.total[1] = (uint32_t)(hi.shr - lo.shr);
      a.total[2] = (uint32_t)(hi.inl - lo.inl);
      for (int k = 0; k < 3; k++) a.n_tiles[k] = (uint32_t)tiles_of(a.total[k]);
      a.rows = rows_[b].as<SubRec>();
      a.shr_rows = shr_rows_[b].as<ShrRec>();
      a.inl_rows = inl_rows_[b].as<InlRec>();
      a.res = res_[b].as<mq_topic_result_dev>();
      a.sres = nullptr;
      a.patches = nullptr;
      a.pcount = nullptr;
      a.rcap = 0;
      a.work = nullptr;
      if (ci >= 2) hip_check(hipStreamWaitEvent(s, merge_done_[b], 0), "hipStreamWaitEvent");
      prof.begin(s, "copy");
      launch_copy(a, copy_blocks_, s);
      prof.end("copy", s);
      hip_check(hipGetLastError(), "k_copy");
      if (!serial_) {
        hip_check(hipEventRecord(copy_done_[b], s), "hipEventRecord");
        hip_check(hipStreamWaitEvent(side_, copy_done_[b], 0), "hipStreamWaitEvent");
      }
      prof.begin(ms, "merge");
      launch_merge(a, false, merge_wpe_opt_ ? merge_wpe_opt_ : 1u, merge_blocks_, ms);
      prof.end("merge", ms);
      hip_check(hipGetLastError(), "k_merge");
      const uint32_t nt = a.t1 - a.t0;
      const ShrRec* shr_out = a.shr_rows;
      if (select_shared_) {  // SelectShared on the device: the chunk's shared rows become the picks
        grow(sel_rows_[b], shr_rows_[b].bytes);
        PickArgs pa;
        pa.res = a.res;
        pa.rows = a.shr_rows;
        pa.sres = nullptr;
        pa.spans = nullptr;
        pa.pool = nullptr;
        pa.sel = sel_rows_[b].as<ShrRec>();
        pa.n_out = &a.res[0].n_shared;
        pa.n_out_stride = sizeof(mq_topic_result_dev) / sizeof(uint32_t);
        pa.n = nt;
        pa.err = err_.as<uint32_t>();
        prof.begin(ms, "pick");
        launch_pick(pa, ms);
        prof.end("pick", ms);
        hip_check(hipGetLastError(), "k_pick");
        shr_out = pa.sel;
      }
      prof.count("copy_rows", (uint64_t)a.total[0] + a.total[1] + a.total[2]);
      prof.count("copy_bytes", 16ull * a.total[0] + 8ull * a.total[1] + 8ull * a.total[2]);
      prof.count("merge_records", hi.merge - lo.merge);
      last_chunks_++;

      if (host) {
        const TopicOff& g = base[sb];
        hip_check(hipMemcpyAsync(host->rows.data() + g.rows + lo.rows, a.rows, (hi.rows - lo.rows) * sizeof(SubRec),
                                 hipMemcpyDeviceToHost, ms), "D2H rows");
        hip_check(hipMemcpyAsync(host->shr.data() + g.shr + lo.shr, shr_out, (hi.shr - lo.shr) * sizeof(ShrRec),
                                 hipMemcpyDeviceToHost, ms), "D2H shared rows");
        hip_check(hipMemcpyAsync(host->inl.data() + g.inl + lo.inl, a.inl_rows, (hi.inl - lo.inl) * sizeof(InlRec),
                                 hipMemcpyDeviceToHost, ms), "D2H inline rows");
        hip_check(hipMemcpyAsync(host->topics.data() + q.t0 + a.t0, a.res, nt * sizeof(mq_topic_result),
                                 hipMemcpyDeviceToHost, ms), "D2H topic results");
      }
      mq_match_result cr;
      memset(&cr, 0, sizeof(cr));
      cr.n_topics = nt;
      cr.topics = reinterpret_cast<const mq_topic_result*>(a.res);
      cr.sub_rows = reinterpret_cast<const mq_client_row*>(a.rows);
      cr.shared_rows = reinterpret_cast<const mq_shared_row*>(shr_out);
      cr.inline_rows = reinterpret_cast<const mq_inline_row*>(a.inl_rows);
      cr.n_sub_rows = hi.rows - lo.rows;
      cr.n_shared_rows = hi.shr - lo.shr;
      cr.n_inline_rows = hi.inl - lo.inl;
      if (fn) fn(user, &cr, q.t0 + a.t0, ms);  // the consumer's work precedes the buffer's reuse
      hip_check(hipEventRecord(merge_done_[b], ms), "hipEventRecord");
      *out = cr;
      done.push_back(c);
    }
    hip_check(hipEventRecord(sb_done_[p], ms), "hipEventRecord");
  }
  // the launch stream completes only after the side stream's work of this batch
  hip_check(hipEventRecord(side_done_, side_), "hipEventRecord");
  hip_check(hipStreamWaitEvent(s, side_done_, 0), "hipStreamWaitEvent");
  if (host) {
    hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
    for (const Chunk& c : done) {
      const Sub& q = sub[c.sb];
      const TopicOff& lo = h_bpre[q.blk0 + c.sb + c.b0];
      const TopicOff& g = base[c.sb];
      const uint32_t t0 = c.b0 * kScanBlock, t1 = (uint32_t)std::min<uint64_t>(q.n, (uint64_t)c.b1 * kScanBlock);
      for (uint32_t t = t0; t < t1; t++) {
        mq_topic_result& r = host->topics[q.t0 + t];
        r.sub_base += g.rows + lo.rows;
        r.shared_base += g.shr + lo.shr;
        r.inline_base += g.inl + lo.inl;
      }
    }
    check_err(s);
  } else if (fn) {
    // chunk consumers already used the rows: the batch's guard flags are read before returning,
    // so a tripped guard fails this call (MQ_EIO), not a later one
    hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
    check_err(s);
  }
}

TopicOff Device::walk_scan(const DevIndex& di, const uint8_t* d_tb, const uint64_t* d_to, uint32_t n, hipStream_t s,
                           const uint32_t** gathers, uint32_t* gstride, bool lists, bool one_sync,
                           const DescArgs* fused) {
  const uint32_t nb = (n + kScanBlock - 1) / kScanBlock;
  grow(counts_, (size_t)n * sizeof(TopicCount));
  grow(offs_, (size_t)(n + 1) * sizeof(TopicOff));
  grow(bsum_, (size_t)(nb + 1) * sizeof(TopicOff));
  grow(bpre_, (size_t)(nb + 1) * sizeof(TopicOff));
  grow(gslots_, (size_t)n * kGatherCap * sizeof(uint32_t));
  grow(ovf_, sizeof(uint32_t));
  pinned(sizeof(TopicOff) + 2 * sizeof(uint32_t));
  TopicOff* h_tot = static_cast<TopicOff*>(h_pin_);
  uint32_t* h_ovf = reinterpret_cast<uint32_t*>(h_tot + 1);
  if (!one_sync) hip_check(hipMemsetAsync(ovf_.p, 0, sizeof(uint32_t), s), "hipMemsetAsync(ovf)");
  const bool front = walk_group_ != 0;
  if (front) {
    grow(fb_list_, (size_t)n * sizeof(uint32_t));
    grow(fb_cnt_, sizeof(uint32_t));
    if (!one_sync) hip_check(hipMemsetAsync(fb_cnt_.p, 0, sizeof(uint32_t), s), "hipMemsetAsync(fb)");
  }  // (one-sync batches: zeroed by spans_begin's k_reset)
  prof.begin(s, "walk");
  if (fused) {  // one-sync batch, k_desc in the walk's epilogue: no scan (the dedup totals the gathers)
    launch_walk_desc(walk_group_, walk_wpe_, d_tb, d_to, n, di, counts_.as<TopicCount>(), gslots_.as<uint32_t>(), ovf_.as<uint32_t>(),
                     fb_list_.as<uint32_t>(), fb_cnt_.as<uint32_t>(), n_cus_ * 2, *fused, s);
    prof.end("walk", s);
    hip_check(hipGetLastError(), "k_walkf<desc>");
    *gathers = gslots_.as<uint32_t>();
    *gstride = kGatherCap;
    prof.count("topics", n);
    return TopicOff{0, 0, 0, 0, 0};
  }
  if (front)
    launch_walk_front(walk_group_, lists, walk_wpe_, d_tb, d_to, n, di, counts_.as<TopicCount>(), gslots_.as<uint32_t>(),
                      ovf_.as<uint32_t>(), fb_list_.as<uint32_t>(), fb_cnt_.as<uint32_t>(), n_cus_ * 2, s, one_sync);
  else
    launch_walk(false, lists, walk_wpe_, d_tb, d_to, n, di, counts_.as<TopicCount>(), nullptr, gslots_.as<uint32_t>(),
                ovf_.as<uint32_t>(), s, one_sync);
  prof.end("walk", s);
  hip_check(hipGetLastError(), "k_walk<count>");
  prof.begin(s, "scan");
  launch_scan(counts_.as<TopicCount>(), n, bsum_.as<TopicOff>(), bpre_.as<TopicOff>(), offs_.as<TopicOff>(), s);
  prof.end("scan", s);
  hip_check(hipGetLastError(), "k_scan");
  if (one_sync) {  // read at the batch's end (k_readback); the gather slots are the gather lists
    *gathers = gslots_.as<uint32_t>();
    *gstride = kGatherCap;
    prof.count("topics", n);
    return TopicOff{0, 0, 0, 0, 0};
  }
  hip_check(hipMemcpyAsync(h_tot, bpre_.as<TopicOff>() + nb, sizeof(TopicOff), hipMemcpyDeviceToHost, s), "D2H totals");
  hip_check(hipMemcpyAsync(h_ovf, ovf_.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s), "D2H overflow");
  if (front && prof.on())
    hip_check(hipMemcpyAsync(h_ovf + 1, fb_cnt_.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s), "D2H fallback");
  hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
  const TopicOff tot = *h_tot;
  if (front && prof.on()) prof.count("walk_fallback", h_ovf[1]);
  *gathers = gslots_.as<uint32_t>();
  *gstride = kGatherCap;
  if (*h_ovf) {  // a topic with more gathers than its count-pass slots: write all lists compactly
    grow(gathers_, std::max<uint64_t>(tot.g, 1) * sizeof(uint32_t));
    prof.begin(s, "walk_fill");
    launch_walk(true, lists, walk_wpe_, d_tb, d_to, n, di, nullptr, offs_.as<TopicOff>(), gathers_.as<uint32_t>(), nullptr, s);
    prof.end("walk_fill", s);
    hip_check(hipGetLastError(), "k_walk<fill>");
    *gathers = gathers_.as<uint32_t>();
    *gstride = 0;
  }
  prof.count("topics", n);
  prof.count("gathers", tot.g);
  prof.count("reserved_rows", tot.rows);
  return tot;
}

// Span format: walk + scan, then k_desc writes each topic's spans (and copies its inline rows)
// and k_merge resolves the co-matching records into patches; nothing is copied per row. The
// patch pool grows when a batch reserves more than it holds (the batch's k_merge then runs
// again); the call ends with the stream synchronised and the guard flags checked.
void Device::match_spans(const uint8_t* d_tb, const uint64_t* d_to, uint32_t n, hipStream_t s,
                         HostSpans* host, mq_span_result* out, hipEvent_t ready, std::atomic<bool>* issued) {
  mq_xlist x;
  trace_runs = 1;
  spans_begin(d_tb, d_to, n, s, &x, one_sync_);
  slow_mark("begin");
  if (spans_end(nullptr, 0, s, host, out, ready, issued)) {
    slow_mark("end");
    return;
  }
  slow_mark("end-rerun");
  trace_runs = 2;
  // the one-sync run's buffers did not hold the batch: again, sized by the host
  spans_begin(d_tb, d_to, n, s, &x, false);
  spans_end(nullptr, 0, s, host, out, ready, issued);
}

void Device::spans_begin(const uint8_t* d_tb, const uint64_t* d_to, uint32_t n, hipStream_t s,
                         mq_xlist* x, bool one_sync, bool shard_sync) {
  hip_check(hipSetDevice(dev_), "hipSetDevice");
  issue_staged(s);  // (the prepare phase's upload of the dirty pages, ahead of the kernels)
  release_retired();
  flush_host_copy();  // (a pipelined batch's copy: before this batch reuses any stage)
  slow_mark("flush");
  const IndexSnap& ix = snap_;  // (Device::prepare: the host image as synced)
  memset(x, 0, sizeof(*x));
  x->n_topics = n;
  x->shard = ix.shard;
  sb_ = SpanBatch{};
  if (!err_.p) {
    err_.ensure(2 * sizeof(uint32_t));
    hip_check(hipMemsetAsync(err_.p, 0, 2 * sizeof(uint32_t), s), "hipMemsetAsync(err)");
  }
  // The walk counts only gathers when nothing needs the lists' totals before k_desc: no inline
  // rows to place and no device share pick (k_desc<true> then counts rows / shared / merge).
  const bool lists = walk_lists_ || select_shared_ || ix.inl_live;
  // A sharded index's begin runs as a one-sync batch's does (k_reset, buffers as earlier batches
  // left them, the export written by k_desc and packed by k_xpack) and synchronises once, at its
  // end, for the export's size (the exchange needs it) and the guards; its spans_end is host-sized.
  const bool xsync = shard_sync && one_sync_ && ix.sharded && !lists && dedup_ != 0 && set_grid_;
  // One host synchronisation for the whole batch (at its end): device results of an index that is
  // not sharded, without inline rows or a device share pick (whose buffers the walk's totals size)
  one_sync = one_sync && !ix.sharded && !lists && dedup_ != 0 && set_grid_;
  const bool bsync = one_sync || xsync;  // the begin without host synchronisations
  sb_.trial = -1;
  if (one_sync && walk_auto_ && n >= kWalkTrialMin) {
    // Which walk suits this index (§4): the frontier walk with the fused desc, or the walk
    // thread per topic + scan + desc. The first batches of each index size try both (one batch
    // each, timed on the device); later batches take the faster per topic. A wildcard-heavy index
    // (config 3) favours the frontier (its DFS diverges), an exact-match one (config 4, 50M IoT
    // filters) the thread per topic (64 topics per wavefront in flight).
    // a new size, or a new wildcard mix (the share of '+' / '#' particles moved by more than a
    // quarter of itself and by more than 0.02 of all particles): try again
    const uint64_t nodes = ix.n_nodes;
    const double wild = nodes ? (double)ix.n_wild / (double)nodes : 0.0;
    const double dw = std::fabs(wild - walk_trial_wild_);
    if (nodes > 2 * walk_trial_nodes_ || 2 * nodes < walk_trial_nodes_ || (dw > 0.02 && dw > 0.25 * walk_trial_wild_)) {
      walk_trial_nodes_ = nodes;
      walk_trial_wild_ = wild;
      walk_trial_ns_[0] = walk_trial_ns_[1] = 0.0;
      walk_trial_step_ = 0;
    }
    const int k = walk_trial_step_ < 6 ? (int)kWalkTrialSeq[walk_trial_step_] : -1;
    if (k >= 0) {
      sb_.trial = k;
      if (!walk_ev_[0]) {
        hip_check(hipEventCreate(&walk_ev_[0]), "hipEventCreate");
        hip_check(hipEventCreate(&walk_ev_[1]), "hipEventCreate");
      }
      hip_check(hipEventRecord(walk_ev_[0], s), "hipEventRecord");
    }
    walk_group_ = (k == 1 || (k < 0 && walk_trial_ns_[1] < walk_trial_ns_[0])) ? 0u : 16u;
  }
  if (bsync) {
    if (!h_fast_) {
      void* hp = nullptr;  // (its own allocation, not a slab block: the device reads it by address)
      hip_check(hipHostMalloc(&hp, sizeof(FastBack), hipHostMallocDefault), "hipHostMalloc");
      h_fast_ = static_cast<FastBack*>(hp);
      void* dp = nullptr;
      hip_check(hipHostGetDevicePointer(&dp, h_fast_, 0), "hipHostGetDevicePointer");
      d_fast_ = static_cast<FastBack*>(dp);
    }
    if (!unsafe_.p) unsafe_.ensure(sizeof(uint32_t));
    memset(h_fast_, 0, sizeof(FastBack));
    // every counter of the batch, zeroed by one launch (k_reset): sized here, before the walk
    grow(counts_, (size_t)n * sizeof(TopicCount));
    grow(ovf_, sizeof(uint32_t));
    grow(fb_cnt_, sizeof(uint32_t));
    uint64_t slots = 1024;
    while (slots < 2ull * n) slots <<= 1;
    grow(dd_keys_, slots * sizeof(unsigned long long));
    grow(dd_vals_, slots * sizeof(uint32_t));
    grow(dd_slot_, (size_t)n * sizeof(uint32_t));
    if (!dd_nsets_.p) dd_nsets_.ensure(3 * sizeof(unsigned long long));
    if (!dd_spcount_.p) dd_spcount_.ensure(kPatchRegions * sizeof(unsigned long long));
    if (!sp_pcount_.p) sp_pcount_.ensure(kPatchRegions * sizeof(unsigned long long));
    if (!dd_nwave_.p) dd_nwave_.ensure(sizeof(unsigned long long));
    ResetArgs ra;
    memset(&ra, 0, sizeof(ra));
    void* ps[] = {unsafe_.p, ovf_.p, fb_cnt_.p, dd_nsets_.p, dd_spcount_.p, sp_pcount_.p, dd_nwave_.p};
    const uint32_t bs[] = {4, 4, 4, 3 * 8, kPatchRegions * 8, kPatchRegions * 8, 8};
    ra.n = 7;
    for (uint32_t k = 0; k < ra.n; k++) {
      ra.p[k] = ps[k];
      ra.bytes[k] = bs[k];
    }
    ra.big = dd_keys_.as<unsigned long long>();
    ra.big_words = slots;
    launch_reset(ra, s);
    hip_check(hipGetLastError(), "k_reset");
  } else {
    check_err(s);  // faults flagged by an earlier row-format batch (one-sync batches read it at their end)
  }
  snap_.di.err = err_.as<uint32_t>();  // (allocated above on the first batch)
  const DevIndex di = snap_.di;
  sb_.pending = true;
  sb_.n = n;
  sb_.version = ix.version;
  sb_.di = di;
  if (n == 0) return;
  ensure_streams();

  const uint32_t* gathers = nullptr;
  uint32_t gstride = 0;
  sb_.lists = lists;
  sb_.one_sync = one_sync;
  // k_desc in the frontier walk's epilogue (one-sync batches): spans and GDesc records at
  // t * kGatherCap, so nothing waits for a scan of the gather counts
  const bool fused = bsync && fuse_desc_ && (walk_group_ == 16 || walk_group_ == 8);
  sb_.fused = fused;
  sb_.walk_inserted = fused && !xsync;
  if (!sb_.lists) grow(sp_tc_, (size_t)n * sizeof(TopicCount));
  if (fused) {
    grow(desc_[0], (size_t)n * kGatherCap * sizeof(GDesc));
    grow(sp_spans_, (size_t)n * kGatherCap * sizeof(SpanRec));
  }
  if (xsync) {  // (k_desc's export at the spans' positions: as many as the spans hold)
    if (!fused) grow(sp_spans_, sizeof(SpanRec));
    grow(x_stride_, sp_spans_.bytes / sizeof(SpanRec) * sizeof(XEnt));
    grow(x_cnt_, (size_t)n * sizeof(uint32_t));
  }
  sb_.dedup = dedup_ != 0;
  if (sb_.dedup) {
    grow(dd_sig_, (size_t)n * sizeof(uint64_t));
    grow(dd_cnt_, (size_t)n * sizeof(uint32_t));
    grow(dd_list_, (size_t)n * kPairMax * sizeof(uint32_t));
    grow(dd_mrow_, (size_t)n * kPairMax * sizeof(uint32_t));
    grow(dd_mpair_, (size_t)n * kPairMax * sizeof(uint2));
    if (ix.sharded) grow(dd_mrank_, (size_t)n * kPairMax * sizeof(uint64_t));
  }
  // k_desc's arguments (the buffers are (re)sized below unless the batch is one-sync)
  auto desc_args = [&]() {
    DescArgs da;
    memset(&da, 0, sizeof(da));
    da.ix = di;
    da.n = n;
    da.gather_stride = gstride;
    da.off = offs_.as<TopicOff>();
    da.gathers = gathers;
    da.desc = desc_[0].as<GDesc>();
    da.spans = sp_spans_.as<SpanRec>();
    da.inl_out = sp_inl_.as<InlRec>();
    da.tc_out = sb_.lists ? nullptr : sp_tc_.as<TopicCount>();
    if (sb_.dedup) {  // merge-set dedup (on a sharded index too: a set is then also the other
                      // shards' entries, which spans_end knows after the exchange)
      da.mpair = dd_mpair_.as<uint2>();
      da.msig = dd_sig_.as<uint64_t>();
      da.mcount = dd_cnt_.as<uint32_t>();
      da.mlist = dd_list_.as<uint32_t>();
      da.mrow = dd_mrow_.as<uint32_t>();
      if (ix.sharded) da.mrank = dd_mrank_.as<uint64_t>();
    }
    da.spans_cap = sp_spans_.bytes / sizeof(SpanRec);
    da.desc_cap = desc_[0].bytes / sizeof(GDesc);
    da.unsafe = bsync ? unsafe_.as<uint32_t>() : nullptr;
    da.g_stride = fused ? kGatherCap : 0u;
    if (xsync) {
      da.xents = x_stride_.as<XEnt>();
      da.xcount = x_cnt_.as<uint32_t>();
      if (fused) da.gw_out = gslots_.as<uint32_t>();  // (walk_scan grew it; sized n * kGatherCap)
    }
    return da;
  };
  DescArgs fda;
  if (fused) {
    grow(sp_inl_, sizeof(InlRec));
    grow(gslots_, (size_t)n * kGatherCap * sizeof(uint32_t));
    fda = desc_args();
    // k_dedup_insert folded into the walk's epilogue (the table was zeroed by k_reset); not on a
    // sharded index, whose signatures take the other shards' entries after the exchange (k_xsig)
    fda.dd_keys = xsync ? nullptr : dd_keys_.as<unsigned long long>();
    fda.dd_vals = dd_vals_.as<uint32_t>();
    uint64_t slots = 1024;  // (as zeroed by k_reset above)
    while (slots < 2ull * n) slots <<= 1;
    fda.dd_mask = slots - 1;
    fda.dd_tslot = dd_slot_.as<uint32_t>();
    if (walk_exp_ & 3u) {  // MQ_OPT_WALK_EXP bit 0: the level-0 probes ahead of the walk; bit 1: levels 0, 1
      const uint32_t levels = (walk_exp_ & 2u) ? 2u : 1u;
      grow(root_hint_, (size_t)n * (levels == 2 ? 3 : 1) * sizeof(uint4));
      prof.begin(s, "root_hint");
      launch_root_hint(d_tb, d_to, n, di, root_hint_.as<uint4>(), levels, s);
      prof.end("root_hint", s);
      hip_check(hipGetLastError(), "k_root_hint");
      fda.root_hint = root_hint_.as<uint4>();
      fda.hint_levels = levels;
    }
  }
  TopicOff tot = walk_scan(di, d_tb, d_to, n, s, &gathers, &gstride, sb_.lists, bsync, fused ? &fda : nullptr);
  if (fail_next_) {  // MQ_OPT_FAIL_NEXT: as if a kernel guard had tripped in this batch
    fail_next_--;
    hip_check(hipMemsetD32Async((hipDeviceptr_t)err_.p, (int)kErrWalkGuard, 1, s), "hipMemsetD32Async(err)");
  }
  sb_.tot = tot;
  sb_.gathers = gathers;
  sb_.gstride = gstride;
  if (!bsync) {  // (one-sync: the buffers as earlier batches left them; the kernels check)
    grow(desc_[0], std::max<uint64_t>(tot.g, 1) * sizeof(GDesc));
    grow(sp_spans_, std::max<uint64_t>(tot.g, 1) * sizeof(SpanRec));
  }
  grow(sp_inl_, std::max<uint64_t>(tot.inl, 1) * sizeof(InlRec));
  grow(sp_res_, (size_t)n * sizeof(TopicSpansDev));
  if (select_shared_) grow(sp_picked_, std::max<uint64_t>(tot.shr, 1) * sizeof(ShrRec));
  if (!sp_pcount_.p) sp_pcount_.ensure(kPatchRegions * sizeof(unsigned long long));
  if (rcap_ * kPatchRegions < patch_cap_init_) {
    rcap_ = std::max<uint64_t>((patch_cap_init_ + kPatchRegions - 1) / kPatchRegions, 16);
    sp_patches_.release();
    sp_patches_.ensure(rcap_ * kPatchRegions * sizeof(PatchRec));
  }
  const DescArgs da = fused ? fda : desc_args();
  sb_.tc = da.tc_out;
  if (!fused) {
    prof.begin(s, "desc");
    launch_desc(da, true, s);
    prof.end("desc", s);
    hip_check(hipGetLastError(), "k_desc<spans>");
  }
  if (xsync) {  // export: packed from k_desc's, then the begin's one synchronisation
    const uint32_t nb = (n + kScanBlock - 1) / kScanBlock;
    grow(x_off_, (size_t)(n + 1) * sizeof(TopicOff));
    grow(xbsum_, (size_t)(nb + 1) * sizeof(TopicOff));
    grow(xbpre_, (size_t)(nb + 1) * sizeof(TopicOff));
    if (!x_tot_.p) x_tot_.ensure(3 * sizeof(unsigned long long));
    grow(x_ents_, sizeof(XEnt));
    auto pack = [&]() {
      prof.begin(s, "xpack");
      if (fused) {  // u32 scans: the export's counts, and (total only) the topics' gathers
        grow(x_off32_, (size_t)(n + 1) * sizeof(uint32_t));
        if (!x_gt_.p) x_gt_.ensure(sizeof(TopicOff));
        const uint32_t nb32 = (uint32_t)((n + kScanBlock - 1) / kScanBlock);
        grow(x_bsum_, 2 * (nb32 + 1) * sizeof(uint32_t));
        grow(x_bpre_, 2 * (nb32 + 1) * sizeof(uint32_t));
        XScanArgs xs;
        memset(&xs, 0, sizeof(xs));
        xs.in[0] = x_cnt_.as<uint32_t>();
        xs.out[0] = x_off32_.as<uint32_t>();
        xs.in[1] = reinterpret_cast<const uint32_t*>(sp_tc_.as<TopicCount>()) + offsetof(TopicCount, gathers) / 4;
        xs.stride[1] = sizeof(TopicCount) / 4;
        launch_xscan(xs, 2, n, x_bsum_.as<uint32_t>(), x_bpre_.as<uint32_t>(), s);
        launch_xpack32(n, kGatherCap, x_cnt_.as<uint32_t>(), x_off32_.as<uint32_t>(), x_stride_.as<XEnt>(),
                       x_ents_.as<XEnt>(), x_ents_.bytes / sizeof(XEnt), unsafe_.as<uint32_t>(),
                       x_tot_.as<unsigned long long>(), x_bpre_.as<uint32_t>() + (nb32 + 1) + nb32, x_gt_.as<TopicOff>(),
                       s);
      } else {
        launch_counts(x_cnt_.as<uint32_t>(), n, counts_.as<TopicCount>(), s);
        launch_scan(counts_.as<TopicCount>(), n, xbsum_.as<TopicOff>(), xbpre_.as<TopicOff>(), x_off_.as<TopicOff>(), s);
        launch_xpack(n, offs_.as<TopicOff>(), 0u, x_cnt_.as<uint32_t>(), x_off_.as<TopicOff>(), xbpre_.as<TopicOff>() + nb,
                     x_stride_.as<XEnt>(), x_ents_.as<XEnt>(), x_ents_.bytes / sizeof(XEnt), unsafe_.as<uint32_t>(),
                     x_tot_.as<unsigned long long>(), s);
      }
      prof.end("xpack", s);
      hip_check(hipGetLastError(), "k_xpack");
      ReadbackArgs rb;
      memset(&rb, 0, sizeof(rb));
      rb.tot = fused ? x_gt_.as<TopicOff>() : bpre_.as<TopicOff>() + nb;
      rb.ovf = ovf_.as<uint32_t>();
      rb.fallback = walk_group_ ? fb_cnt_.as<uint32_t>() : nullptr;
      rb.unsafe = unsafe_.as<uint32_t>();
      rb.err = err_.as<uint32_t>();
      rb.n_sets = x_tot_.as<unsigned long long>();
      rb.out = d_fast_;
      launch_readback(rb, s);
      hip_check(hipGetLastError(), "k_readback");
      hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
    };
    pack();
    if (h_fast_->err) check_err(s);  // throws with the tripped guard's name
    // (k_xsig writes GDesc records at the topics' gather offsets for k_merge's linear paths: the
    // records must hold every gather)
    const uint64_t gathers_total = fused ? h_fast_->tot.rows : h_fast_->tot.g;
    if (h_fast_->ovf || (h_fast_->unsafe & (kUnsafeSpans | kUnsafeDesc)) ||
        (!fused && gathers_total > desc_[0].bytes / sizeof(GDesc))) {
      // the walk or k_desc outgrew what earlier batches left: the begin again, host-sized
      prof.count("one_sync_retries", 1);
      spans_begin(d_tb, d_to, n, s, x, false, false);
      return;
    }
    if (h_fast_->unsafe & kUnsafeXEnts) {  // only the packed export outgrew its buffer: pack again
      x_ents_.release();
      x_ents_.ensure(std::max<uint64_t>(h_fast_->n_sets[0] + h_fast_->n_sets[0] / 4 + 1024, 1) * sizeof(XEnt));
      hip_check(hipMemsetAsync(unsafe_.p, 0, sizeof(uint32_t), s), "memset");
      pack();
      if (h_fast_->unsafe) throw HipError{hipErrorUnknown, "k_xpack: the export did not fit the grown buffer"};
    }
    sb_.tot = fused ? TopicOff{gathers_total, 0, 0, 0, 0} : h_fast_->tot;
    sb_.xsync = true;
    if (walk_group_ && prof.on()) prof.count("walk_fallback", h_fast_->fallback);
    x->counts = x_cnt_.as<uint32_t>();
    x->ents = reinterpret_cast<const mq_xent*>(x_ents_.p);
    x->n_ents = h_fast_->n_sets[0];
    prof.count("xents", x->n_ents);
    prof.count("topics", n);
  } else if (ix.sharded) {  // export: each topic's gathered cross-shard nodes
    const uint32_t nb = (n + kScanBlock - 1) / kScanBlock;
    grow(x_off_, (size_t)(n + 1) * sizeof(TopicOff));
    grow(x_cnt_, (size_t)n * sizeof(uint32_t));
    prof.begin(s, "xlist");
    launch_xlist(true, di, n, offs_.as<TopicOff>(), gathers, gstride, counts_.as<TopicCount>(), nullptr, nullptr,
                 nullptr, s);
    launch_scan(counts_.as<TopicCount>(), n, bsum_.as<TopicOff>(), bpre_.as<TopicOff>(), x_off_.as<TopicOff>(), s);
    TopicOff* h_tot = static_cast<TopicOff*>(h_pin_);
    hip_check(hipMemcpyAsync(h_tot, bpre_.as<TopicOff>() + nb, sizeof(TopicOff), hipMemcpyDeviceToHost, s), "D2H");
    hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
    const uint64_t n_ents = h_tot->g;
    grow(x_ents_, std::max<uint64_t>(n_ents, 1) * sizeof(XEnt));
    launch_xlist(false, di, n, offs_.as<TopicOff>(), gathers, gstride, nullptr, x_off_.as<TopicOff>(),
                 x_ents_.as<XEnt>(), x_cnt_.as<uint32_t>(), s);
    prof.end("xlist", s);
    hip_check(hipGetLastError(), "k_xlist");
    hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
    x->counts = x_cnt_.as<uint32_t>();
    x->ents = reinterpret_cast<const mq_xent*>(x_ents_.p);
    x->n_ents = n_ents;
    prof.count("xents", n_ents);
  }
}

bool Device::spans_end(const mq_xlist* xf, uint32_t nf, hipStream_t s, HostSpans* host,
                       mq_span_result* out, hipEvent_t ready, std::atomic<bool>* issued) {
  hip_check(hipSetDevice(dev_), "hipSetDevice");
  memset(out, 0, sizeof(*out));
  if (host) *host = HostSpans{};
  if (!sb_.pending) throw HipError{hipErrorInvalidValue, "spans_end without spans_begin"};
  sb_.pending = false;
  const IndexSnap& ix = snap_;
  const DevIndex di = sb_.di;
  const uint32_t n = sb_.n;
  TopicOff tot = sb_.tot;
  out->sub_pool = reinterpret_cast<const mq_client_row*>(di.subs);
  out->shared_pool = reinterpret_cast<const mq_shared_row*>(di.shr);
  out->sub_pool_len = ix.subs_len;
  out->shared_pool_len = ix.shr_len;
  out->flags = select_shared_ ? MQ_SPANS_PICKED : 0u;
  if (nf > kMaxShards - 1) throw HipError{hipErrorInvalidValue, "more foreign lists than kMaxShards - 1"};
  if (nf && !ix.sharded) throw HipError{hipErrorInvalidValue, "foreign lists for an index that is not sharded"};
  if (n == 0) {
    if (ready) hip_check(hipEventRecord(ready, s), "hipEventRecord");
    if (issued) issued->store(true);
    return true;
  }
  const bool one_sync = sb_.one_sync || sb_.xsync;
  // host results: this batch's stage, free once the copy of its last batch is done; 4-byte patch
  // codes while every subscription list is shorter than 2^23 (set rows) and the rows of a topic
  // fit 29 bits (MQ_SPANS_PATCH_CODES)
  HostStage* hs = nullptr;
  const bool codes = host && patch_codes_ && ix.max_sub_cap <= (1u << kCodeSetRowBits) &&
                     ix.subs_len < (1ull << 29);
  if (host) {
    host->codes = codes;
    ensure_hcopy();
    grow(sp_roff_, (kPatchRegions + 1) * sizeof(uint64_t));  // (written by k_readback in one-sync batches)
    hs = &hst_[hpar_];
    if (hs->used) hip_check(hipStreamWaitEvent(s, hs->copied, 0), "hipStreamWaitEvent");
  }

  EmitArgs a;
  memset(&a, 0, sizeof(a));
  a.n_xf = nf;
  if (nf && !h_xsrc_) {
    void* hp = nullptr;
    hip_check(hipHostMalloc(&hp, (kMaxShards - 1) * sizeof(XSrc), hipHostMallocDefault), "hipHostMalloc");
    h_xsrc_ = static_cast<XSrc*>(hp);
  }
  XSrc* const h_src = h_xsrc_;  // (pinned: its copy runs in order with the batch; the previous
                                //  batch's copy of it is waited for before it is written again —
                                //  a batch that threw after queueing the copy did not synchronise)
  if (nf && xsrc_done_) hip_check(hipEventSynchronize(xsrc_done_), "hipEventSynchronize(xsrc)");
  XScanArgs xs;  // import: per-topic offsets of every foreign list, one batched scan
  memset(&xs, 0, sizeof(xs));
  for (uint32_t f = 0; f < nf; f++) {
    if (xf[f].n_topics != n || (xf[f].n_ents && (!xf[f].counts || !xf[f].ents)))
      throw HipError{hipErrorInvalidValue, "foreign list does not match the batch"};
    grow(x_foff_[f], (size_t)(n + 1) * sizeof(uint32_t));
    if (!xf[f].counts && n) {  // (an export of nothing may come without counts: zeros)
      if (x_zero_.bytes < (size_t)n * sizeof(uint32_t)) {
        grow(x_zero_, (size_t)n * sizeof(uint32_t));
        hip_check(hipMemsetAsync(x_zero_.p, 0, x_zero_.bytes, s), "memset");
      }
    }
    xs.in[f] = xf[f].counts ? xf[f].counts : x_zero_.as<uint32_t>();
    xs.out[f] = x_foff_[f].as<uint32_t>();
    h_src[f] = XSrc{x_foff_[f].as<uint32_t>(), reinterpret_cast<const XEnt*>(xf[f].ents)};
  }
  if (nf && n) {
    const size_t rows = (size_t)nf * ((n + kScanBlock - 1) / kScanBlock + 1) * sizeof(uint32_t);
    grow(x_bsum_, rows);
    grow(x_bpre_, rows);
    launch_xscan(xs, nf, n, x_bsum_.as<uint32_t>(), x_bpre_.as<uint32_t>(), s);
    hip_check(hipGetLastError(), "import");
  }
  if (nf) {
    grow(x_src_, (kMaxShards - 1) * sizeof(XSrc));
    hip_check(hipMemcpyAsync(x_src_.p, h_src, nf * sizeof(XSrc), hipMemcpyHostToDevice, s), "H2D xsrc");
    if (!xsrc_done_) hip_check(hipEventCreateWithFlags(&xsrc_done_, hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventRecord(xsrc_done_, s), "hipEventRecord(xsrc)");
    a.xsrc = x_src_.as<XSrc>();
  }
  if (sb_.dedup) {  // merge-set dedup: each topic's representative (DedupArgs)
    uint64_t slots = 1024;
    while (slots < 2ull * n) slots <<= 1;
    grow(dd_keys_, slots * sizeof(unsigned long long));
    grow(dd_vals_, slots * sizeof(uint32_t));
    grow(dd_slot_, (size_t)n * sizeof(uint32_t));
    grow(dd_rep_, (size_t)n * sizeof(uint32_t));
    grow(dd_rlist_, (size_t)n * sizeof(uint32_t));
    if (!dd_nsets_.p) dd_nsets_.ensure(3 * sizeof(unsigned long long));
    if (!one_sync) {  // (one-sync batches: zeroed by spans_begin's k_reset)
      hip_check(hipMemsetAsync(dd_keys_.p, 0, slots * sizeof(unsigned long long), s), "memset");
      hip_check(hipMemsetAsync(dd_nsets_.p, 0, 3 * sizeof(unsigned long long), s), "memset");
    }
    DedupArgs dd;
    memset(&dd, 0, sizeof(dd));
    dd.n = n;
    dd.msig = dd_sig_.as<uint64_t>();
    dd.mcount = dd_cnt_.as<uint32_t>();
    dd.mlist = dd_list_.as<uint32_t>();
    dd.keys = dd_keys_.as<unsigned long long>();
    dd.vals = dd_vals_.as<uint32_t>();
    dd.table_mask = slots - 1;
    dd.tslot = dd_slot_.as<uint32_t>();
    dd.rep = dd_rep_.as<uint32_t>();
    dd.n_sets = dd_nsets_.as<unsigned long long>();
    dd.tc = sb_.tc;
    dd.off = offs_.as<TopicOff>();
    dd.heavy = kSetHeavy;
    dd.rep_list = dd_rlist_.as<uint32_t>();
    dd.fcount = nullptr;
    dd.n_xf = nf;
    dd.xsrc = a.xsrc;
    if (nf) {  // the other shards' entries join each topic's signature
      grow(dd_fcnt_, (size_t)n * sizeof(uint32_t));
      XSigArgs xa;
      xa.ix = di;
      xa.n = n;
      xa.n_xf = nf;
      xa.xsrc = a.xsrc;
      xa.msig = dd_sig_.as<uint64_t>();
      xa.mcount = dd_cnt_.as<uint32_t>();
      xa.fcount = dd_fcnt_.as<uint32_t>();
      xa.off = offs_.as<TopicOff>();
      xa.gathers = sb_.gathers;
      xa.gather_stride = sb_.gstride;
      xa.g_stride = sb_.fused ? kGatherCap : 0u;
      xa.tc = sb_.tc;
      xa.desc = desc_[0].as<GDesc>();
      xa.dd_keys = sb_.walk_inserted ? nullptr : dd.keys;  // (the insert on the finished signatures)
      xa.dd_vals = dd.vals;
      xa.dd_mask = dd.table_mask;
      xa.dd_tslot = dd.tslot;
      prof.begin(s, "xsig");
      launch_xsig(xa, s);
      prof.end("xsig", s);
      hip_check(hipGetLastError(), "k_xsig");
      dd.fcount = xa.fcount;
    }
    prof.begin(s, "dedup");
    launch_dedup(dd, s, !sb_.walk_inserted && !nf);
    prof.end("dedup", s);
    hip_check(hipGetLastError(), "k_dedup");
    sb_.n_sets = 0;
    if (one_sync) {  // the set count is read at the batch's end; the set pass strides over it
      // the grid: the last batch's count with room (the set pass strides over the true count);
      // with none yet, as many waves as topics (an unused one exits at once)
      sb_.n_sets = last_sets_ ? last_sets_ + last_sets_ / 8 + 256 : n;
    } else if (prof.on() || set_grid_) {
      unsigned long long two[2] = {0, 0};
      hip_check(hipMemcpyAsync(two, dd_nsets_.p, sizeof(two), hipMemcpyDeviceToHost, s), "D2H");
      hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
      const unsigned long long ns = two[0] + two[1];
      if (prof.on()) prof.count("dedup_sets", ns);
      sb_.n_sets = ns;
      last_sets_ = ns;
    }
  }


  a.ix = di;
  a.t0 = 0;
  a.t1 = n;
  a.off = offs_.as<TopicOff>();
  a.base = TopicOff{0, 0, 0, 0, 0};
  a.desc = desc_[0].as<GDesc>();
  a.inl_rows = sp_inl_.as<InlRec>();
  if (hs) grow(hs->topics, (size_t)n * sizeof(TopicSpansDev));
  a.sres = hs ? hs->topics.as<TopicSpansDev>() : sp_res_.as<TopicSpansDev>();
  a.pcount = sp_pcount_.as<unsigned long long>();
  a.tc = sb_.lists ? nullptr : sp_tc_.as<TopicCount>();
  a.work = nullptr;
  a.set_rec = nullptr;
  if (prof.work()) {  // [0]: the topics' pass, [1]: the merge sets' pass (dedup)
    grow(sp_work_, 2 * kPatchRegions * kWork * sizeof(unsigned long long));
    if (sb_.dedup) {
      grow(set_rec_, (size_t)n * sizeof(uint32_t));
      hip_check(hipMemsetAsync(set_rec_.p, 0, (size_t)n * sizeof(uint32_t), s), "memset");
      a.set_rec = set_rec_.as<uint32_t>();
    }
    a.work = sp_work_.as<unsigned long long>();
    hip_check(hipMemsetAsync(a.work + kPatchRegions * kWork, 0, kPatchRegions * kWork * sizeof(unsigned long long), s),
              "memset");
  }
  a.rep = nullptr;
  a.tslot = nullptr;
  a.dd_phase = 0;
  a.mrank = ix.sharded && sb_.dedup ? dd_mrank_.as<uint64_t>() : nullptr;
  a.desc_cap = desc_[0].bytes / sizeof(GDesc);
  a.unsafe = one_sync ? unsafe_.as<uint32_t>() : nullptr;
  a.g_stride = sb_.fused ? kGatherCap : 0u;
  a.exp = set_exp_;
  pinned((2 * kPatchRegions + 3) * sizeof(unsigned long long) + 2 * sizeof(uint32_t));
  unsigned long long* h_pc = static_cast<unsigned long long*>(h_pin_);        // [kPatchRegions]
  uint64_t* h_roff = reinterpret_cast<uint64_t*>(h_pc + kPatchRegions);       // [kPatchRegions + 1]
  uint32_t* h_err = reinterpret_cast<uint32_t*>(h_roff + kPatchRegions + 1);  // [2]
  unsigned long long* h_mrtot = reinterpret_cast<unsigned long long*>(h_err + 2);  // [1]
  unsigned long long* h_stot = h_mrtot + 1;                                         // [1]
  uint64_t n_patches = 0, max_region = 0;
  // k_merge register budget: the kernel waits on memory, and eight waves per SIMD (64 VGPRs, a
  // few spills) beat six (80 VGPRs) at 1M and 10M subscriptions (4.37 -> 4.17 ms and 1.37 -> 1.27
  // ms per 1M topics, profiles/r02/tune_walk_merge.jsonl). MQ_OPT_MERGE_WAVES overrides.
  const uint32_t merge_wpe = merge_wpe_opt_ ? merge_wpe_opt_ : kMergeWavesPerEU;
  if (sb_.dedup) {  // phase 1: one resolution per merge set, into the set pool (regions as below)
    grow(dd_sets_, (size_t)n * sizeof(SetInfo));
    if (!dd_spcount_.p) dd_spcount_.ensure(kPatchRegions * sizeof(unsigned long long));
    if (srcap_ * kPatchRegions < patch_cap_init_) {
      srcap_ = std::max<uint64_t>((patch_cap_init_ + kPatchRegions - 1) / kPatchRegions, 16);
      dd_spatches_.release();
      dd_spatches_.ensure(srcap_ * kPatchRegions * sizeof(PatchRec));
    }
    a.rep = dd_rep_.as<uint32_t>();
    a.tslot = dd_slot_.as<uint32_t>();
    a.mcount = dd_cnt_.as<uint32_t>();
    a.mrow = dd_mrow_.as<uint32_t>();
    a.mlist = dd_list_.as<uint32_t>();
    a.mpair = dd_mpair_.as<uint2>();
    a.sets = dd_sets_.as<SetInfo>();
    a.spcount = dd_spcount_.as<unsigned long long>();
    a.rep_list = dd_rlist_.as<uint32_t>();
    a.n_reps = dd_nsets_.as<unsigned long long>();
    a.dd_phase = 1;
    unsigned long long* work0 = a.work;
    if (a.work) a.work += kPatchRegions * kWork;
    for (int attempt = 0;; attempt++) {
      a.spatches = dd_spatches_.as<PatchRec>();
      a.srcap = srcap_;
      if (!one_sync) hip_check(hipMemsetAsync(a.spcount, 0, kPatchRegions * sizeof(unsigned long long), s), "memset");
      if (a.work) hip_check(hipMemsetAsync(a.work, 0, kPatchRegions * kWork * sizeof(unsigned long long), s), "memset");
      prof.begin(s, "merge_sets");
      // persistent: the waves stride over the representative list (its length is on the device)
      // MQ_OPT_SET_GRID 1: a wavefront per set (the dispatcher balances heavy sets); else
      // persistent waves striding over the list
      const uint32_t set_blocks = set_grid_ ? std::max<uint32_t>(1, (uint32_t)((sb_.n_sets + 3) / 4))
                                            : (merge_blocks_ ? merge_blocks_ : n_cus_ * 8);
      // k_set (sets.hip; a sharded index's with its rank keys) unless a sharded index holds filters
      // deeper than 32 levels (their keys can tie: k_merge's deep tie-break), a measurement variant
      // of k_merge's set pass is asked for (MQ_OPT_SET_EXP bit 7, the attribution bits 0-4), or bit 13
      if (!(ix.sharded && a.ix.deep) && !(set_exp_ & (0x1Fu | 128u | 8192u)) && merge_wpe == kMergeWavesPerEU)
        launch_set(a, set_blocks, s);
      else
        launch_merge(a, true, merge_wpe, set_blocks, s);
      prof.end("merge_sets", s);
      hip_check(hipGetLastError(), "k_merge<spans> (sets)");
      if (one_sync) break;  // a reservation past its region sets *unsafe (read at the end)
      hip_check(hipMemcpyAsync(h_pc, a.spcount, kPatchRegions * sizeof(unsigned long long), hipMemcpyDeviceToHost, s),
                "D2H");
      hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
      uint64_t mr = 0;
      for (uint32_t r = 0; r < kPatchRegions; r++) mr = std::max<uint64_t>(mr, h_pc[r]);
      if (mr <= srcap_) break;
      if (attempt) throw HipError{hipErrorUnknown, "k_merge<spans>: set patch reservations changed between runs"};
      srcap_ = mr + mr / 4 + 64;
      dd_spatches_.release();
      dd_spatches_.ensure(srcap_ * kPatchRegions * sizeof(PatchRec));
    }
    if (a.set_rec) {  // MQ_PROF_WORK: how the resolution work spreads over the sets
      std::vector<uint32_t> rec(n);
      hip_check(hipMemcpyAsync(rec.data(), a.set_rec, n * sizeof(uint32_t), hipMemcpyDeviceToHost, s), "D2H");
      hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
      std::sort(rec.begin(), rec.end(), std::greater<uint32_t>());
      uint64_t tot = 0, top = 0, sets = 0;
      for (uint32_t r : rec) tot += r, sets += r != 0;
      for (uint64_t i = 0; i < sets / 100; i++) top += rec[i];
      prof.count("set_records_max", rec.empty() ? 0 : rec[0]);
      prof.count("set_records_top1pct", top);
      prof.count("set_records_total", tot);
      prof.count("sets_over_4096_records", (uint64_t)std::count_if(rec.begin(), rec.end(), [](uint32_t r) { return r > 4096; }));
      a.set_rec = nullptr;
    }
    a.work = work0;
    a.dd_phase = 2;
    a.set_ref = 1u;  // a deduped topic references its set's patches (host results too: ABI v7)
    {  // results that need no wavefront: k_finish, thread per topic
      grow(dd_wlist_, (size_t)n * sizeof(uint32_t));
      if (!dd_nwave_.p) dd_nwave_.ensure(sizeof(unsigned long long));
      if (!one_sync) hip_check(hipMemsetAsync(dd_nwave_.p, 0, sizeof(unsigned long long), s), "memset");
      FinishArgs fa;
      fa.n = n;
      fa.off = a.off;
      fa.tc = a.tc;
      fa.tslot = a.tslot;
      fa.rep = a.rep;
      fa.sets = a.sets;
      fa.sres = a.sres;
      fa.wave_list = dd_wlist_.as<uint32_t>();
      fa.n_wave = dd_nwave_.as<unsigned long long>();
      fa.g_stride = a.g_stride;
      prof.begin(s, "finish");
      launch_finish(fa, s);
      prof.end("finish", s);
      hip_check(hipGetLastError(), "k_finish");
      a.wave_list = fa.wave_list;
      a.n_wave = fa.n_wave;
    }
    if (host) {  // the sets' written patches, packed (their total read with pcount)
      grow(set_nbase_, (size_t)n * sizeof(uint64_t));
      grow(hs->set_patches, srcap_ * kPatchRegions * sizeof(PatchRec));  // (at most every reservation)
      if (!set_total_.p) set_total_.ensure(sizeof(unsigned long long));
      hip_check(hipMemsetAsync(set_total_.p, 0, sizeof(unsigned long long), s), "memset");
      launch_set_pack(n, a.tslot, a.rep, a.sets, dd_spatches_.as<PatchRec>(), set_nbase_.as<uint64_t>(),
                      hs->set_patches.as<PatchRec>(), codes ? hs->set_patches.as<uint32_t>() : nullptr,
                      set_total_.as<unsigned long long>(), s);
      hip_check(hipGetLastError(), "k_set_pack");
      if (!one_sync)  // (one-sync: k_readback reads it)
        hip_check(hipMemcpyAsync(h_stot, set_total_.p, sizeof(unsigned long long), hipMemcpyDeviceToHost, s), "D2H");
    }
    if (host) {  // the merge rows of the topics with a set, packed (their total read with pcount)
      if ((uint64_t)n * kPairMax > UINT32_MAX) throw HipError{hipErrorInvalidValue, "host span batch too large"};
      grow(hs->merge_base, (size_t)n * sizeof(uint32_t));
      grow(hs->merge_rows, (size_t)n * kPairMax * sizeof(uint32_t));
      if (!mr_total_.p) mr_total_.ensure(sizeof(unsigned long long));
      hip_check(hipMemsetAsync(mr_total_.p, 0, sizeof(unsigned long long), s), "memset");
      launch_mrow_pack(n, a.tslot, a.mcount, a.mrow, hs->merge_base.as<uint32_t>(), hs->merge_rows.as<uint32_t>(),
                       mr_total_.as<unsigned long long>(), s);
      hip_check(hipGetLastError(), "k_mrow_pack");
      if (!one_sync)
        hip_check(hipMemcpyAsync(h_mrtot, mr_total_.p, sizeof(unsigned long long), hipMemcpyDeviceToHost, s), "D2H");
    }
  }
  for (int attempt = 0;; attempt++) {
    a.patches = sp_patches_.as<PatchRec>();
    a.rcap = rcap_;
    if (!one_sync)
      hip_check(hipMemsetAsync(a.pcount, 0, kPatchRegions * sizeof(unsigned long long), s), "hipMemsetAsync(pcount)");
    if (a.work) hip_check(hipMemsetAsync(a.work, 0, kPatchRegions * kWork * sizeof(unsigned long long), s), "memset");
    prof.begin(s, "merge");
    // after k_finish the waves stride over its list (its length is on the device)
    launch_merge(a, true, merge_wpe, a.wave_list && !merge_blocks_ ? n_cus_ * 8 : merge_blocks_, s);
    prof.end("merge", s);
    hip_check(hipGetLastError(), "k_merge<spans>");
    if (one_sync) break;  // as the set pass
    hip_check(hipMemcpyAsync(h_pc, a.pcount, kPatchRegions * sizeof(unsigned long long), hipMemcpyDeviceToHost, s),
              "D2H pcount");
    hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
    n_patches = max_region = 0;
    for (uint32_t r = 0; r < kPatchRegions; r++) {
      h_roff[r] = n_patches;
      n_patches += h_pc[r];
      max_region = std::max<uint64_t>(max_region, h_pc[r]);
    }
    h_roff[kPatchRegions] = n_patches;
    if (max_region <= rcap_) break;
    if (attempt) throw HipError{hipErrorUnknown, "k_merge<spans>: patch reservations changed between runs"};
    rcap_ = max_region + max_region / 4 + 64;  // every region of this batch, with slack
    sp_patches_.release();
    sp_patches_.ensure(rcap_ * kPatchRegions * sizeof(PatchRec));
  }
  if (select_shared_) {  // SelectShared on the device: picked members at each topic's picked_base
    PickArgs pa;
    pa.res = nullptr;
    pa.rows = nullptr;
    pa.sres = a.sres;
    pa.spans = sp_spans_.as<SpanRec>();
    pa.pool = di.shr;
    pa.sel = sp_picked_.as<ShrRec>();
    pa.n_out = &a.sres[0].n_shared;
    pa.n_out_stride = sizeof(TopicSpansDev) / sizeof(uint32_t);
    pa.n = n;
    pa.err = err_.as<uint32_t>();
    prof.begin(s, "pick");
    launch_pick(pa, s);
    prof.end("pick", s);
    hip_check(hipGetLastError(), "k_pick<spans>");
  }
  if (one_sync) {  // the batch's one synchronisation: totals, overflow, unsafe bits, errors
    ReadbackArgs rb;
    // (a sharded batch's totals were read by its begin: the imports' scans reused bpre_ since)
    rb.tot = sb_.fused || sb_.xsync ? nullptr : bpre_.as<TopicOff>() + (n + kScanBlock - 1) / kScanBlock;
    rb.ovf = ovf_.as<uint32_t>();
    rb.fallback = walk_group_ ? fb_cnt_.as<uint32_t>() : nullptr;
    rb.unsafe = unsafe_.as<uint32_t>();
    rb.err = err_.as<uint32_t>();
    rb.n_sets = sb_.dedup ? dd_nsets_.as<unsigned long long>() : nullptr;
    // host results: the topic pass's region offsets (on the device, for the packing below) and
    // the totals, with the rest
    rb.pcount = host ? a.pcount : nullptr;
    rb.roff = host ? sp_roff_.as<uint64_t>() : nullptr;
    rb.set_total = host && sb_.dedup ? set_total_.as<unsigned long long>() : nullptr;
    rb.mrow_total = host && sb_.dedup ? mr_total_.as<unsigned long long>() : nullptr;
    rb.out = d_fast_;
    launch_readback(rb, s);
    hip_check(hipGetLastError(), "k_readback");
    if (sb_.trial >= 0) hip_check(hipEventRecord(walk_ev_[1], s), "hipEventRecord");
    const auto ts0 = std::chrono::steady_clock::now();
    hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
    trace_sync_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ts0).count();
    if (sb_.trial >= 0 && !h_fast_->err && !h_fast_->ovf && !h_fast_->unsafe) {  // a walk trial: its time per topic
      if (walk_trial_step_ >= kWalkTrialWarm) {
        float ms = 0.f;
        hip_check(hipEventElapsedTime(&ms, walk_ev_[0], walk_ev_[1]), "hipEventElapsedTime");
        const double ns = std::max(1e-3, 1e6 * (double)ms / n);
        walk_trial_ns_[sb_.trial] += ns;
        prof.count(sb_.trial ? "trial_thread_ps_per_topic" : "trial_frontier_ps_per_topic",
                   std::max<uint64_t>(1, (uint64_t)(1e3 * ns)));
        prof.count(sb_.trial ? "trial_thread_batches" : "trial_frontier_batches", 1);
      }
      walk_trial_step_++;
      if (walk_trial_step_ == 6) prof.count(walk_trial_ns_[1] < walk_trial_ns_[0] ? "trial_chose_thread" : "trial_chose_frontier", 1);
    }
    if (h_fast_->err) check_err(s);  // throws with the tripped guard's name
    if (h_fast_->ovf || h_fast_->unsafe) {
      prof.count("one_sync_retries", 1);
      if (sb_.xsync) {  // sharded: the begin's results and the imported lists stand; the end again,
        sb_.pending = true;  // host-sized
        sb_.xsync = false;
        return spans_end(xf, nf, s, host, out, ready, issued);
      }
      return false;
    }
    tot = sb_.xsync ? sb_.tot : h_fast_->tot;
    if (sb_.fused) tot.g = h_fast_->n_sets[2];  // (no scan: k_dedup_rep totals the gathers)
    if (host) n_patches = h_fast_->n_patches;  // (the region offsets: sp_roff_, k_readback)
    sb_.tot = tot;
    last_sets_ = h_fast_->n_sets[0] + h_fast_->n_sets[1];
    if (prof.on()) {
      prof.count("gathers", tot.g);
      prof.count("dedup_sets", last_sets_);
      if (walk_group_) prof.count("walk_fallback", h_fast_->fallback);
    }
  }
  prof.count("patch_slots", n_patches);  // reserved; the written ones: merge_patches (MQ_PROF_WORK)
  prof.count("spans", tot.g);
  out->n_topics = n;
  out->topics = reinterpret_cast<const mq_topic_spans*>(a.sres);
  out->spans = reinterpret_cast<const mq_span*>(sp_spans_.p);
  out->patches = reinterpret_cast<const mq_patch*>(sp_patches_.p);
  out->inline_rows = reinterpret_cast<const mq_inline_row*>(sp_inl_.p);
  out->picked_rows = select_shared_ ? reinterpret_cast<const mq_shared_row*>(sp_picked_.p) : nullptr;
  out->n_spans = sb_.fused ? (uint64_t)n * kGatherCap : tot.g;  // (the stride layout's extent)
  out->n_patches = rcap_ * kPatchRegions;  // the pool's extent: topic ranges sit in regions
  out->n_inline_rows = tot.inl;
  out->n_picked_rows = select_shared_ ? tot.shr : 0;
  if (sb_.dedup && a.set_ref) {
    out->set_patches = reinterpret_cast<const mq_patch*>(dd_spatches_.p);
    out->merge_rows = dd_mrow_.as<uint32_t>();
    out->n_set_patches = srcap_ * kPatchRegions;
    out->n_merge_rows = (uint64_t)n * kPairMax;  // (MQ_MERGE_ROWS_STRIDE per topic)
  }
  if (a.work) {  // MQ_PROF_WORK: k_merge's work, for its algorithmic bytes (bench.py)
    std::vector<unsigned long long> w(2 * kPatchRegions * kWork);
    hip_check(hipMemcpyAsync(w.data(), a.work, w.size() * sizeof(w[0]), hipMemcpyDeviceToHost, s), "D2H work");
    hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
    uint64_t sum[kWork] = {};
    for (uint32_t r = 0; r < 2 * kPatchRegions; r++)
      for (uint32_t k = 0; k < kWork; k++) sum[k] = k >= 24 ? std::max<uint64_t>(sum[k], w[r * kWork + k]) : sum[k] + w[r * kWork + k];
    prof.count("merge_pair_entries", sum[0]);
    prof.count("merge_records", sum[1]);
    prof.count("merge_links", sum[2]);
    prof.count("merge_patches", sum[3]);
    prof.count("set_cycles_map", sum[4]);
    prof.count("set_cycles_pairs", sum[5]);
    prof.count("set_cycles_resolve", sum[6]);
    prof.count("set_cycles_total", sum[7]);
    prof.count("merge_topics_resolved", sum[8]);
    prof.count("merge_map_bytes", sum[9]);
    prof.count("merge_fold_visits", sum[10]);
    prof.count("merge_big_visits", sum[11]);
    prof.count("merge_big_gathers", sum[12]);
    prof.count("merge_big_nmerge", sum[13]);
    prof.count("merge_fold_nmerge", sum[14]);
    prof.count("merge_fold_chunks", sum[15]);
    static const char* const kBig[4] = {"192", "384", "1024", "more"};
    for (int b = 0; b < 4; b++) {
      prof.count((std::string("merge_big_gathers_v") + kBig[b]).c_str(), sum[16 + b]);
      prof.count((std::string("merge_big_visits_v") + kBig[b]).c_str(), sum[20 + b]);
    }
    prof.count("set_cycles_max", sum[24]);
    prof.count("set_records_max_wave", sum[25]);
    prof.count("set_pairs_cycles_max", sum[26]);
    prof.count("set_resolve_cycles_max", sum[27]);
    prof.count("set_gathers_max", sum[28]);
    prof.count("set_hit_lists_max", sum[29]);
    prof.count("merge_topics", n);
  }
  // A pipelined copy is armed (pc_) only when the batch has passed its error check: a batch that
  // throws frees the host arrays the copy would fill.
  PendingCopy arm;
  if (host) {  // pack the result into the stage, then copy it on the copy stream
    if (n_patches) {  // the regions' used parts, packed
      grow(hs->patches, n_patches * sizeof(PatchRec));
      if (!one_sync)  // (one-sync: k_readback wrote them)
        hip_check(hipMemcpyAsync(sp_roff_.p, h_roff, kPatchRegions * sizeof(uint64_t), hipMemcpyHostToDevice, s), "H2D");
      launch_patch_compact(sp_patches_.as<PatchRec>(), rcap_, a.pcount, sp_roff_.as<uint64_t>(),
                           hs->patches.as<PatchRec>(), codes ? hs->patches.as<uint32_t>() : nullptr, s);
      hip_check(hipGetLastError(), "k_patch_compact");
    }
    // every topic's patch_base into the packed arrays (its own patches' or its set's)
    launch_host_rebase(n, sb_.dedup ? a.rep : nullptr, sb_.dedup ? set_nbase_.as<uint64_t>() : nullptr,
                       n_patches ? sp_roff_.as<uint64_t>() : nullptr, rcap_, a.sres, s);
    hip_check(hipGetLastError(), "k_host_rebase");
    // the spans packed (one-sync batches leave them at t * 64), span_base into the packed array
    grow(hs->spans, std::max<uint64_t>(tot.g, 1) * sizeof(SpanRec));
    if (!hs->span_total.p) hs->span_total.ensure(sizeof(unsigned long long));
    hip_check(hipMemsetAsync(hs->span_total.p, 0, sizeof(unsigned long long), s), "memset");
    launch_span_pack(n, a.sres, sp_spans_.as<SpanRec>(), hs->spans.as<SpanRec>(),
                     hs->span_total.as<unsigned long long>(), s);
    hip_check(hipGetLastError(), "k_span_pack");
    if (tot.inl) {
      grow(hs->inl, tot.inl * sizeof(InlRec));
      hip_check(hipMemcpyAsync(hs->inl.p, sp_inl_.p, tot.inl * sizeof(InlRec), hipMemcpyDeviceToDevice, s), "D2D");
    }
    if (out->n_picked_rows) {
      grow(hs->picked, out->n_picked_rows * sizeof(ShrRec));
      hip_check(hipMemcpyAsync(hs->picked.p, sp_picked_.p, out->n_picked_rows * sizeof(ShrRec),
                               hipMemcpyDeviceToDevice, s), "D2D");
    }
    hip_check(hipEventRecord(hs->packed, s), "hipEventRecord");
    PendingCopy c;
    c.on = true;
    c.hs = hs;
    c.host = host;
    c.n = n;
    c.spans = tot.g;
    c.patches = n_patches;
    c.inl = tot.inl;
    c.picked = out->n_picked_rows;
    c.dedup = sb_.dedup;
    c.codes = codes;
    c.set = !sb_.dedup ? 0 : one_sync ? h_fast_->set_total : *h_stot;
    c.mrows = !sb_.dedup ? 0 : one_sync ? h_fast_->mrow_total : *h_mrtot;
    c.ready = ready;
    c.issued = issued;
    // the result's host arrays exist now (the caller publishes them); the copy fills them
    host->topics.resize(n);
    host->spans.resize(c.spans);
    if (codes) host->patch_codes.resize(c.patches);
    else host->patches.resize(c.patches);
    host->inl.resize(c.inl);
    host->picked.resize(c.picked);
    if (c.dedup) {
      if (codes) host->set_codes.resize(c.set);
      else host->set_patches.resize(c.set);
      host->merge_rows.resize(c.mrows);
      host->merge_base.resize(n);
    }
    hs->used = true;
    hpar_ ^= 1u;
    if (ready) {
      arm = c;  // pipelined: issued behind the next batch's upload (flush_host_copy)
    } else {
      issue_host_copy(c);
      hip_check(hipStreamSynchronize(hcopy_), "hipStreamSynchronize(copy)");
    }
  } else if (ready) {
    hip_check(hipEventRecord(ready, s), "hipEventRecord");
    if (issued) issued->store(true);
  }
  if (!one_sync) {  // (one-sync: checked above)
    hip_check(hipMemcpyAsync(h_err, err_.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s), "D2H err");
    hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
    if (*h_err) check_err(s);  // throws with the tripped guard's name
  }
  if (arm.on) pc_ = arm;
  return true;
}

void Device::acl(const uint8_t* fb, const uint64_t* fo, uint32_t nf, const uint8_t* tb, const uint64_t* to,
                 uint32_t nt, const uint32_t* pf, const uint32_t* pt, uint64_t n_pairs, HostAcl* out) {
  hip_check(hipSetDevice(dev_), "hipSetDevice");
  *out = HostAcl{};
  out->matched.resize(n_pairs);
  out->n_elems.resize(n_pairs);
  out->elem_base.resize(n_pairs);
  if (!n_pairs) return;
  // capacity of a pair = '+' / '#' parts of its filter (each captures at most one element)
  std::vector<uint32_t> cap(nf, 0);
  for (uint32_t f = 0; f < nf; f++) {
    uint64_t b = fo[f];
    for (uint64_t i = fo[f]; i <= fo[f + 1]; i++) {
      if (i == fo[f + 1] || fb[i] == '/') {
        if (i - b == 1 && (fb[b] == '+' || fb[b] == '#')) cap[f]++;
        b = i + 1;
      }
    }
  }
  uint64_t total = 0;
  for (uint64_t p = 0; p < n_pairs; p++) {
    if (pf[p] >= nf || pt[p] >= nt) throw HipError{hipErrorInvalidValue, "pair index out of range"};
    out->elem_base[p] = total;
    total += cap[pf[p]];
  }
  out->elems.resize(2 * std::max<uint64_t>(total, 1));
  auto up = [](uint64_t x) { return (x + 255) & ~255ull; };  // 256-byte aligned sub-buffers
  const uint64_t fbytes = fo[nf], tbytes = to[nt];
  const uint64_t o_fb = 0, o_fo = up(o_fb + fbytes + 16), o_tb = up(o_fo + 8 * (nf + 1)),
                 o_to = up(o_tb + tbytes + 16), o_pf = up(o_to + 8 * (nt + 1)), o_pt = up(o_pf + 4 * n_pairs),
                 o_eb = up(o_pt + 4 * n_pairs), o_m = up(o_eb + 8 * n_pairs), o_ne = up(o_m + n_pairs),
                 o_el = up(o_ne + 4 * n_pairs), o_end = up(o_el + 8 * std::max<uint64_t>(total, 1));
  acl_buf_.ensure(o_end);
  uint8_t* d = acl_buf_.as<uint8_t>();
  hipStream_t s = nullptr;
  hip_check(hipMemsetAsync(d, 0, o_fo, s), "memset");
  hip_check(hipMemsetAsync(d + o_tb, 0, o_to - o_tb, s), "memset");
  if (fbytes) hip_check(hipMemcpyAsync(d + o_fb, fb, fbytes, hipMemcpyHostToDevice, s), "H2D");
  hip_check(hipMemcpyAsync(d + o_fo, fo, 8 * (nf + 1), hipMemcpyHostToDevice, s), "H2D");
  if (tbytes) hip_check(hipMemcpyAsync(d + o_tb, tb, tbytes, hipMemcpyHostToDevice, s), "H2D");
  hip_check(hipMemcpyAsync(d + o_to, to, 8 * (nt + 1), hipMemcpyHostToDevice, s), "H2D");
  hip_check(hipMemcpyAsync(d + o_pf, pf, 4 * n_pairs, hipMemcpyHostToDevice, s), "H2D");
  hip_check(hipMemcpyAsync(d + o_pt, pt, 4 * n_pairs, hipMemcpyHostToDevice, s), "H2D");
  hip_check(hipMemcpyAsync(d + o_eb, out->elem_base.data(), 8 * n_pairs, hipMemcpyHostToDevice, s), "H2D");
  AclArgs a;
  a.filter_bytes = d + o_fb;
  a.filter_offs = reinterpret_cast<const uint64_t*>(d + o_fo);
  a.topic_bytes = d + o_tb;
  a.topic_offs = reinterpret_cast<const uint64_t*>(d + o_to);
  a.pair_filter = reinterpret_cast<const uint32_t*>(d + o_pf);
  a.pair_topic = reinterpret_cast<const uint32_t*>(d + o_pt);
  a.elem_base = reinterpret_cast<const uint64_t*>(d + o_eb);
  a.n_pairs = n_pairs;
  a.matched = d + o_m;
  a.n_elems = reinterpret_cast<uint32_t*>(d + o_ne);
  a.elems = reinterpret_cast<uint32_t*>(d + o_el);
  prof.begin(s, "acl");
  launch_acl(a, s);
  prof.end("acl", s);
  hip_check(hipGetLastError(), "k_acl");
  hip_check(hipMemcpyAsync(out->matched.data(), d + o_m, n_pairs, hipMemcpyDeviceToHost, s), "D2H");
  hip_check(hipMemcpyAsync(out->n_elems.data(), d + o_ne, 4 * n_pairs, hipMemcpyDeviceToHost, s), "D2H");
  if (total) hip_check(hipMemcpyAsync(out->elems.data(), d + o_el, 8 * total, hipMemcpyDeviceToHost, s), "D2H");
  hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
}

// The level-order retained image (kernels.h MsgImg): level by level from the root, a count pass
// (image children per parent), a scan (their positions), a fill pass; then the live handles are
// packed in image order. Rebuilt when the retained state changed since the last build.
void Device::ensure_img(const Index& ix, const DevIndex& di, hipStream_t s) {
  if (img_version_ == ix.retained_version()) return;
  const uint32_t slots = std::max<uint32_t>(ix.node_slots(), 1);
  img_node_.ensure((size_t)slots * sizeof(uint32_t));
  img_cl_.ensure((size_t)slots * sizeof(uint2));
  img_lp_.ensure(((size_t)slots + 1) * sizeof(uint32_t));
  img_pos_.ensure((size_t)slots * sizeof(uint32_t));
  img_cnt_.ensure(((size_t)slots + 1) * sizeof(uint32_t));
  img_coff_.ensure(((size_t)slots + 1) * sizeof(uint32_t));
  const size_t nb = ((size_t)slots + kScanBlock) / kScanBlock + 1;
  img_bsum_.ensure(nb * sizeof(uint32_t));
  img_bpre_.ensure(nb * sizeof(uint32_t));
  prof.begin(s, "msg_image");
  hip_check(hipMemsetAsync(img_pos_.p, 0xFF, (size_t)slots * sizeof(uint32_t), s), "hipMemsetAsync(img pos)");
  launch_img_root(img_node_.as<uint32_t>(), img_pos_.as<uint32_t>(), img_lp_.as<uint32_t>(), s);
  ImgLevelArgs a;
  a.node = img_node_.as<uint32_t>();
  a.pos = img_pos_.as<uint32_t>();
  a.cl = img_cl_.as<uint2>();
  a.live = img_lp_.as<uint32_t>();  // live flags, scanned in place into lp below
  a.cnt = img_cnt_.as<uint32_t>();
  a.coff = img_coff_.as<uint32_t>();
  uint32_t lo = 0, n = 1, levels = 0;
  while (n) {
    a.lo = lo;
    a.n = n;
    a.next = lo + n;
    launch_img_level(false, di, a, s);
    hip_check(hipGetLastError(), "k_img_level (count)");
    launch_scan32(a.cnt, n, img_bsum_.as<uint32_t>(), img_bpre_.as<uint32_t>(), img_coff_.as<uint32_t>(), s);
    uint32_t next_n = 0;
    hip_check(hipMemcpyAsync(&next_n, img_coff_.as<uint32_t>() + n, sizeof(uint32_t), hipMemcpyDeviceToHost, s),
              "D2H image level");
    hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
    if ((uint64_t)a.next + next_n > slots) throw HipError{hipErrorUnknown, "messages image beyond the node count"};
    launch_img_level(true, di, a, s);
    hip_check(hipGetLastError(), "k_img_level");
    lo += n;
    n = next_n;
    levels++;
  }
  launch_scan32(img_lp_.as<uint32_t>(), lo, img_bsum_.as<uint32_t>(), img_bpre_.as<uint32_t>(),
                img_lp_.as<uint32_t>(), s);
  uint32_t live = 0;
  hip_check(hipMemcpyAsync(&live, img_lp_.as<uint32_t>() + lo, sizeof(uint32_t), hipMemcpyDeviceToHost, s),
            "D2H image live");
  hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
  img_h_.ensure(std::max<size_t>(live, 1) * sizeof(uint64_t));
  launch_img_compact(di, img_node_.as<uint32_t>(), img_lp_.as<uint32_t>(), lo, img_h_.as<uint64_t>(), s);
  hip_check(hipGetLastError(), "k_img_compact");
  img_edge_mask_ = 0;
  if (msg_edges_on_) {
    // the image's edge table, sparse: most lookups miss (a literal under a wide run), and a miss
    // ends at the first free slot. At most a sixteenth full while that stays within 8 GiB, an
    // eighth within 32 GiB, else a quarter (10M retained: 1/8 -> 53.4M filters/s, 1/2 -> 37.9M)
    // (MQ_OPT_MSG_EDGE_BUDGET lowers the 8 GiB budget, and the 32 GiB one with it: the tier test)
    uint64_t slots2 = 1024;
    while (slots2 < 16ull * lo) slots2 <<= 1;
    while (slots2 > 4ull * lo && slots2 > 1024 &&
           slots2 * sizeof(ImgEdge) > (slots2 >= 16ull * lo ? msg_edge_budget_ : 4 * msg_edge_budget_))
      slots2 >>= 1;
    prof.count("msg_edge_slots", slots2);
    prof.count("msg_edge_particles", lo);
    img_edges_.ensure(slots2 * sizeof(ImgEdge));
    hip_check(hipMemsetAsync(img_edges_.p, 0xFF, slots2 * sizeof(ImgEdge), s), "hipMemsetAsync(image edges)");
    launch_img_edges(di, img_node_.as<uint32_t>(), img_pos_.as<uint32_t>(), lo, slots, img_edges_.as<ImgEdge>(), slots2 - 1, s);
    hip_check(hipGetLastError(), "k_img_edges");
    img_edge_mask_ = slots2 - 1;
  }
  kx_built_ = false;
  prof.end("msg_image", s);  // (the profiler does not nest: the key index is timed apart)
  if (msg_kx_on_) {
    prof.begin(s, "msg_kx_build");
    build_key_index(di, lo, slots, s);
    prof.end("msg_kx_build", s);
  }
  img_n_ = lo;
  img_n_pos_ = slots;
  img_levels_ = levels;
  img_live_ = live;
  img_version_ = ix.retained_version();
}

// The image's key index (kernels.h MsgImg.kx_*): its edges collected, sorted stably by parent
// position then by key hash (so one key's entries are contiguous and ordered by parent), and a
// table from key hash to the range. Skipped when its transient arrays (~90 B per image particle)
// would not fit a quarter of the device's free memory.
void Device::build_key_index(const DevIndex& di, uint32_t n_img, uint32_t n_pos, hipStream_t s) {
  kx_par_.release();
  kx_chd_.release();
  kx_k0_.release();
  kx_k1_.release();
  kx_tab_.release();
  kx_mask_ = 0;
  if (n_img < 2) return;
  size_t freeb = 0, total = 0;
  if (hipMemGetInfo(&freeb, &total) == hipSuccess && (uint64_t)n_img * 96 > freeb / 4) return;
  const uint32_t cap = n_img;
  DevBuf a_par, a_chd, a_k0, a_k1, a_h, perm0, t_par, perm1, t_h, perm2, s_h, cnt, temp;
  a_par.ensure((size_t)cap * 4);
  a_chd.ensure((size_t)cap * 4);
  a_k0.ensure((size_t)cap * 8);
  a_k1.ensure((size_t)cap * 8);
  a_h.ensure((size_t)cap * 8);
  perm0.ensure((size_t)cap * 4);
  cnt.ensure(2 * sizeof(unsigned long long));
  hip_check(hipMemsetAsync(cnt.p, 0, 2 * sizeof(unsigned long long), s), "memset");
  launch_kx_collect(di, img_node_.as<uint32_t>(), img_pos_.as<uint32_t>(), n_img, n_pos, a_par.as<uint32_t>(),
                    a_chd.as<uint32_t>(), a_k0.as<uint64_t>(), a_k1.as<uint64_t>(), a_h.as<uint64_t>(),
                    perm0.as<uint32_t>(), cnt.as<unsigned long long>(), s);
  hip_check(hipGetLastError(), "k_kx_collect");
  unsigned long long ne = 0;
  hip_check(hipMemcpyAsync(&ne, cnt.p, sizeof(ne), hipMemcpyDeviceToHost, s), "D2H kx count");
  hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
  if (ne == 0 || ne > cap) return;
  const uint32_t n = (uint32_t)ne;
  t_par.ensure((size_t)n * 4);
  perm1.ensure((size_t)n * 4);
  t_h.ensure((size_t)n * 8);
  perm2.ensure((size_t)n * 4);
  s_h.ensure((size_t)n * 8);
  const size_t tb = std::max(kx_sort_u32(nullptr, 0, a_par.as<uint32_t>(), t_par.as<uint32_t>(), perm0.as<uint32_t>(),
                                         perm1.as<uint32_t>(), n, s),
                             kx_sort_u64(nullptr, 0, t_h.as<uint64_t>(), s_h.as<uint64_t>(), perm1.as<uint32_t>(),
                                         perm2.as<uint32_t>(), n, s));
  temp.ensure(tb);
  kx_sort_u32(temp.p, tb, a_par.as<uint32_t>(), t_par.as<uint32_t>(), perm0.as<uint32_t>(), perm1.as<uint32_t>(), n, s);
  hip_check(hipGetLastError(), "kx sort (parents)");
  launch_kx_gather64(a_h.as<uint64_t>(), perm1.as<uint32_t>(), t_h.as<uint64_t>(), n, s);
  kx_sort_u64(temp.p, tb, t_h.as<uint64_t>(), s_h.as<uint64_t>(), perm1.as<uint32_t>(), perm2.as<uint32_t>(), n, s);
  hip_check(hipGetLastError(), "kx sort (keys)");
  kx_par_.ensure((size_t)n * 4);
  kx_chd_.ensure((size_t)n * 4);
  kx_k0_.ensure((size_t)n * 8);
  kx_k1_.ensure((size_t)n * 8);
  launch_kx_gather32(a_par.as<uint32_t>(), perm2.as<uint32_t>(), kx_par_.as<uint32_t>(), n, s);
  launch_kx_gather32(a_chd.as<uint32_t>(), perm2.as<uint32_t>(), kx_chd_.as<uint32_t>(), n, s);
  launch_kx_gather64(a_k0.as<uint64_t>(), perm2.as<uint32_t>(), kx_k0_.as<uint64_t>(), n, s);
  launch_kx_gather64(a_k1.as<uint64_t>(), perm2.as<uint32_t>(), kx_k1_.as<uint64_t>(), n, s);
  launch_kx_count_keys(s_h.as<uint64_t>(), n, cnt.as<unsigned long long>() + 1, s);
  hip_check(hipGetLastError(), "kx gathers");
  unsigned long long keys = 0;
  hip_check(hipMemcpyAsync(&keys, cnt.as<unsigned long long>() + 1, sizeof(keys), hipMemcpyDeviceToHost, s), "D2H kx keys");
  hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
  uint64_t slots = 1024;
  while (slots < 2 * keys) slots <<= 1;
  kx_tab_.ensure(slots * sizeof(KxSlot));
  hip_check(hipMemsetAsync(kx_tab_.p, 0, slots * sizeof(KxSlot), s), "memset kx table");
  launch_kx_table(s_h.as<uint64_t>(), n, kx_tab_.as<KxSlot>(), slots - 1, err_.as<uint32_t>(), s);
  hip_check(hipGetLastError(), "k_kx_table");
  hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");  // (the temporaries go at return)
  kx_mask_ = slots - 1;
  kx_built_ = true;
  prof.count("msg_kx_entries", n);
  prof.count("msg_kx_keys", keys);
}

MsgImg Device::msg_img() const {
  MsgImg m;
  m.node = img_node_.as<uint32_t>();
  m.pos = img_pos_.as<uint32_t>();
  m.cl = img_cl_.as<uint2>();
  m.lp = img_lp_.as<uint32_t>();
  m.h = img_h_.as<uint64_t>();
  m.edges = img_edge_mask_ ? img_edges_.as<ImgEdge>() : nullptr;
  m.edge_mask = img_edge_mask_;
  m.gate = nullptr;
  m.n = img_n_;
  m.n_pos = img_n_pos_;
  m.cyc = nullptr;
  m.work = nullptr;
  m.run_base = nullptr;
  m.run_cnt = nullptr;
  m.kx_tab = kx_built_ ? kx_tab_.as<KxSlot>() : nullptr;
  m.kx_mask = kx_mask_;
  m.kx_min_rounds = msg_kx_min_;
  m.kx_par = kx_par_.as<uint32_t>();
  m.kx_chd = kx_chd_.as<uint32_t>();
  m.kx_k0 = kx_k0_.as<uint64_t>();
  m.kx_k1 = kx_k1_.as<uint64_t>();
  return m;
}

// k_msgq count pass, scan, fill pass, k_msg_copy. Returns false (nothing written) when a filter's
// fan-out nesting exceeded kMsgStack: the batch then takes the particle walk.
bool Device::messages_img(const DevIndex& di, const uint8_t* d_fb, const uint64_t* d_fo, uint32_t n,
                          hipStream_t s, TopicOff* tot, bool run_out) {
  MsgImg img = msg_img();
  if (run_out) {  // runs at the boundary: a piece per run, nothing copied (k_msg_copy not launched)
    msg_rbase_.ensure((size_t)n * sizeof(uint64_t));
    msg_rcnt_.ensure((size_t)n * sizeof(uint32_t));
    img.run_base = msg_rbase_.as<uint64_t>();
    img.run_cnt = msg_rcnt_.as<uint32_t>();
  }
  const uint32_t nb = (n + kScanBlock - 1) / kScanBlock;
  if (prof.work()) {  // MQ_PROF_WORK: per-filter clocks and fan-out work of the count pass
    grow(msg_cyc_, (size_t)n * sizeof(uint32_t) + 4 * sizeof(unsigned long long));
    img.work = reinterpret_cast<unsigned long long*>(msg_cyc_.p);
    img.cyc = reinterpret_cast<uint32_t*>(img.work + 4);
    hip_check(hipMemsetAsync(msg_cyc_.p, 0, (size_t)n * sizeof(uint32_t) + 4 * sizeof(unsigned long long), s), "memset");
  }
  // One walk per filter: the count pass records each filter's runs (up to run_cap of them, from
  // the speculative-scratch budget) and the second pass places them; a filter with more runs
  // walks again in the second pass. Without the budget: count walk, then fill walk.
  const uint32_t run_cap = (uint32_t)std::min<uint64_t>(kMsgRunCap, msg_spec_bytes_ / ((uint64_t)n * sizeof(MsgRun)));
  const bool runs = run_cap >= 8;
  if (runs) {
    msg_runs_.ensure((size_t)n * run_cap * sizeof(MsgRun));
    msg_nruns_.ensure((size_t)n * sizeof(uint32_t));
  }
  MsgRun* d_runs = runs ? msg_runs_.as<MsgRun>() : nullptr;
  uint32_t* d_nruns = runs ? msg_nruns_.as<uint32_t>() : nullptr;
  // wide filters: the count pass exports a fan-out of more than kMsgExportMin particles as work
  // items that every wavefront of the grid can take (recorded-runs passes only)
  MsgWide wide;
  memset(&wide, 0, sizeof(wide));
  const bool exp = runs && msg_export_ != 0;
  if (exp) {
    msg_wq_.ensure(kMsgWorkCap * sizeof(MsgWork) + sizeof(uint32_t));
    wide.items = msg_wq_.as<MsgWork>();
    wide.n_items = reinterpret_cast<uint32_t*>(wide.items + kMsgWorkCap);
    wide.cap = kMsgWorkCap;
    wide.min_tot = msg_export_ > 1 ? msg_export_ : kMsgExportMin;
    wide.min_hits = msg_export_ > 1 ? msg_export_ : kMsgExportMinHits;
    msg_wscratch_.ensure((size_t)n_cus_ * 8 * 4 * kMsgWideRuns * sizeof(MsgRun));
    wide.scratch = msg_wscratch_.as<MsgRun>();
    wide.per_wave = kMsgWideRuns;
    hip_check(hipMemsetAsync(wide.n_items, 0, sizeof(uint32_t), s), "hipMemsetAsync(n_items)");
  }
  const uint32_t wide_blocks = n_cus_ * 8;
  prof.begin(s, "msgq_count");
  launch_msgq(runs ? kMsgRuns : kMsgCount, d_fb, d_fo, n, di, img, counts_.as<TopicCount>(), nullptr, nullptr,
              nullptr, nullptr, nullptr, d_runs, run_cap, d_nruns, wide, wide_blocks, s);
  prof.end("msgq_count", s);
  if (exp) {  // the exported items' counts
    prof.begin(s, "msgq_wide_count");
    launch_msgq(kMsgWideCount, d_fb, d_fo, n, di, img, counts_.as<TopicCount>(), nullptr, nullptr, nullptr, nullptr,
                nullptr, d_runs, run_cap, d_nruns, wide, wide_blocks, s);
    prof.end("msgq_wide_count", s);
  }
  hip_check(hipGetLastError(), "k_msgq<count>");
  launch_scan(counts_.as<TopicCount>(), n, bsum_.as<TopicOff>(), bpre_.as<TopicOff>(), offs_.as<TopicOff>(), s);
  hip_check(hipGetLastError(), "k_scan");
  // the fill and copy passes, given the output buffers as they are; true when they held the batch
  auto fill_copy = [&](const uint32_t* gate, const uint64_t* n_pieces) {
    img.gate = gate;
    prof.begin(s, "msgq_fill");
    launch_msgq(runs ? kMsgPlace : kMsgFill, d_fb, d_fo, n, di, img, counts_.as<TopicCount>(), offs_.as<TopicOff>(),
                msg_pieces_.as<MsgPiece>(), msg_handles_.as<uint64_t>(), msg_base_.as<uint64_t>(),
                msg_count_.as<uint32_t>(), d_runs, run_cap, d_nruns, wide, wide_blocks, s);
    prof.end("msgq_fill", s);
    if (exp) {
      prof.begin(s, "msgq_wide_fill");
      launch_msgq(kMsgWideFill, d_fb, d_fo, n, di, img, counts_.as<TopicCount>(), offs_.as<TopicOff>(),
                  msg_pieces_.as<MsgPiece>(), msg_handles_.as<uint64_t>(), msg_base_.as<uint64_t>(),
                  msg_count_.as<uint32_t>(), d_runs, run_cap, d_nruns, wide, wide_blocks, s);
      prof.end("msgq_wide_fill", s);
    }
    hip_check(hipGetLastError(), "k_msgq<fill>");
    if (run_out) return;
    prof.begin(s, "msg_copy");
    if (n_pieces)
      launch_msg_copy_dev(msg_pieces_.as<MsgPiece>(), n_pieces, msg_pieces_.bytes / sizeof(MsgPiece), img.h,
                          msg_handles_.as<uint64_t>(), s);
    else
      launch_msg_copy(msg_pieces_.as<MsgPiece>(), tot->g, img.h, msg_handles_.as<uint64_t>(), s);
    prof.end("msg_copy", s);
    hip_check(hipGetLastError(), "k_msg_copy");
  };
  if (!img.work) {
    // One host synchronisation per batch: the fill and copy passes run on the output buffers as
    // earlier batches left them, behind a gate (k_msg_gate: the totals fit); the totals, the error
    // word and the gate are read once at the end, and a batch that did not fit fills again into
    // buffers sized by the host (the counts stand). Errors flagged earlier surface here too.
    msg_base_.ensure((size_t)n * sizeof(uint64_t));
    msg_count_.ensure((size_t)n * sizeof(uint32_t));
    if (!msg_handles_.p) msg_handles_.ensure(sizeof(uint64_t));
    if (!msg_pieces_.p) msg_pieces_.ensure(sizeof(MsgPiece));
    if (!msg_gate_.p) msg_gate_.ensure(2 * sizeof(uint64_t));
    uint32_t* gate = msg_gate_.as<uint32_t>();
    uint64_t* n_pieces = msg_gate_.as<uint64_t>() + 1;
    launch_msg_gate(bpre_.as<TopicOff>() + nb, run_out ? ~0ull : msg_handles_.bytes / sizeof(uint64_t),
                    msg_pieces_.bytes / sizeof(MsgPiece), gate, n_pieces, s);
    hip_check(hipGetLastError(), "k_msg_gate");
    fill_copy(gate, n_pieces);
    uint32_t e = 0, g = 0;
    hip_check(hipMemcpyAsync(tot, bpre_.as<TopicOff>() + nb, sizeof(TopicOff), hipMemcpyDeviceToHost, s), "D2H total");
    hip_check(hipMemcpyAsync(&e, err_.p, sizeof(e), hipMemcpyDeviceToHost, s), "D2H err");
    hip_check(hipMemcpyAsync(&g, gate, sizeof(g), hipMemcpyDeviceToHost, s), "D2H gate");
    hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
    if (e == kErrMsgNest) {  // (the fill wrote within its buffers; the particle walk redoes the batch)
      hip_check(hipMemsetAsync(err_.p, 0, sizeof(uint32_t), s), "hipMemsetAsync(err)");
      return false;
    }
    if (e) check_err(s);  // throws with the tripped guard's name
    if (!g) {
      prof.count("msg_one_sync_retries", 1);
      if (!run_out) msg_handles_.ensure(std::max<uint64_t>(tot->rows, 1) * sizeof(uint64_t));
      msg_pieces_.ensure(std::max<uint64_t>(tot->g, 1) * sizeof(MsgPiece));
      fill_copy(nullptr, nullptr);
    }
    return true;
  }
  uint32_t e = 0;
  hip_check(hipMemcpyAsync(tot, bpre_.as<TopicOff>() + nb, sizeof(TopicOff), hipMemcpyDeviceToHost, s), "D2H total");
  hip_check(hipMemcpyAsync(&e, err_.p, sizeof(e), hipMemcpyDeviceToHost, s), "D2H err");
  hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
  if (e == kErrMsgNest) {
    hip_check(hipMemsetAsync(err_.p, 0, sizeof(uint32_t), s), "hipMemsetAsync(err)");
    return false;
  }
  check_err(s);
  if (img.work) {  // the count pass's cost over the filters: total, max, heaviest 1 % and 0.1 %
    std::vector<uint32_t> c(n);
    unsigned long long w[4];
    hip_check(hipMemcpy(w, img.work, sizeof(w), hipMemcpyDeviceToHost), "D2H");
    hip_check(hipMemcpy(c.data(), img.cyc, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost), "D2H");
    std::sort(c.begin(), c.end(), std::greater<uint32_t>());
    uint64_t tot_c = 0, top1 = 0, top01 = 0;
    for (uint32_t i = 0; i < n; i++) {
      tot_c += c[i];
      if (i < n / 100) top1 += c[i];
      if (i < n / 1000) top01 += c[i];
    }
    prof.count("msg_cyc16_total", tot_c);
    prof.count("msg_cyc16_max", n ? c[0] : 0);
    prof.count("msg_cyc16_p50", n ? c[n / 2] : 0);
    prof.count("msg_cyc16_p99", n ? c[n / 100] : 0);
    prof.count("msg_cyc16_top1pct", top1);
    prof.count("msg_cyc16_top01pct", top01);
    prof.count("msg_fanout_lookups", w[0]);
    prof.count("msg_lane_walk_filters", w[1]);
    prof.count("msg_lane_walk_particles", w[2]);
  }
  if (!run_out) msg_handles_.ensure(std::max<uint64_t>(tot->rows, 1) * sizeof(uint64_t));
  msg_base_.ensure((size_t)n * sizeof(uint64_t));
  msg_count_.ensure((size_t)n * sizeof(uint32_t));
  msg_pieces_.ensure(std::max<uint64_t>(tot->g, 1) * sizeof(MsgPiece));
  fill_copy(nullptr, nullptr);
  return true;
}

void Device::messages_walk(Index& ix, const DevIndex& di, const uint8_t* d_fb, const uint64_t* d_fo, uint32_t n,
                           hipStream_t s, TopicOff* tot) {
  const uint32_t nb = (n + kScanBlock - 1) / kScanBlock;
  // k_msg register budget: on a large retained index the walk waits on HBM far more often, and
  // 6 waves per SIMD (with spills) beat 4 (10M retained: 54.8 -> 50.2 ms per 100k filters); on
  // a small, cache-resident one the spills cost more (1M: 8.7 vs 9.2 ms). MQ_MSG_WPE overrides.
  const uint32_t msg_wpe = msg_wpe_opt_ ? msg_wpe_opt_ : (ix.retained_len() >= kMsgWpeMinRetained ? kMsgWavesPerEU : 1u);
  // Speculative count: the count pass also writes each filter's first `cap` handles to scratch,
  // so that only filters with more (or counted through below_live) are walked a second time.
  uint32_t cap = (uint32_t)std::min<uint64_t>(kMsgSpecCap, msg_spec_bytes_ / ((uint64_t)n * sizeof(uint64_t)));
  if (cap < 64) cap = 0;
  uint64_t* spec = nullptr;
  if (cap) {
    msg_spec_.ensure((size_t)n * cap * sizeof(uint64_t));
    spec = msg_spec_.as<uint64_t>();
  }
  prof.begin(s, "msg_count");
  launch_msg(false, d_fb, d_fo, n, di, counts_.as<TopicCount>(), nullptr, nullptr, nullptr, nullptr, spec, cap,
             msg_wpe, s);
  prof.end("msg_count", s);
  hip_check(hipGetLastError(), "k_msg<count>");
  launch_scan(counts_.as<TopicCount>(), n, bsum_.as<TopicOff>(), bpre_.as<TopicOff>(), offs_.as<TopicOff>(), s);
  hip_check(hipGetLastError(), "k_scan");
  hip_check(hipMemcpyAsync(tot, bpre_.as<TopicOff>() + nb, sizeof(TopicOff), hipMemcpyDeviceToHost, s), "D2H total");
  hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
  check_err(s);
  msg_handles_.ensure(std::max<uint64_t>(tot->rows, 1) * sizeof(uint64_t));
  msg_base_.ensure((size_t)n * sizeof(uint64_t));
  msg_count_.ensure((size_t)n * sizeof(uint32_t));
  if (cap) {
    prof.begin(s, "msg_place");
    launch_msg_place(n, counts_.as<TopicCount>(), offs_.as<TopicOff>(), spec, cap, msg_handles_.as<uint64_t>(),
                     msg_base_.as<uint64_t>(), msg_count_.as<uint32_t>(), s);
    prof.end("msg_place", s);
    hip_check(hipGetLastError(), "k_msg_place");
  }
  prof.begin(s, "msg_fill");
  launch_msg(true, d_fb, d_fo, n, di, counts_.as<TopicCount>(), offs_.as<TopicOff>(), msg_handles_.as<uint64_t>(),
             msg_base_.as<uint64_t>(), msg_count_.as<uint32_t>(), spec, cap, msg_wpe, s);
  prof.end("msg_fill", s);
  hip_check(hipGetLastError(), "k_msg<fill>");
}

void Device::messages(Index& ix, const uint8_t* d_fb, const uint64_t* d_fo, uint32_t n,
                      hipStream_t s, HostMsg* host, mq_msg_result* out, mq_msg_runs_result* runs,
                      HostMsgRuns* hruns) {
  hip_check(hipSetDevice(dev_), "hipSetDevice");
  sync(ix, s);
  mq_msg_result unused;
  if (!out) out = &unused;
  *out = mq_msg_result{};
  if (host) *host = HostMsg{};
  if (runs) *runs = mq_msg_runs_result{};
  if (hruns) *hruns = HostMsgRuns{};
  if (!err_.p) {
    err_.ensure(2 * sizeof(uint32_t));
    hip_check(hipMemsetAsync(err_.p, 0, 2 * sizeof(uint32_t), s), "hipMemsetAsync(err)");
  }
  // (one-sync image batches read the error word at their end instead, messages_img)
  const bool img_path = msg_img_on_ && !ix.empty_topic_live && ix.retained_len() != 0;
  if (!img_path || prof.work()) check_err(s);
  if (n == 0) return;
  // the Messages kernels launch a wavefront per filter (a grid is limited to 2^32 threads)
  if (n > kMaxWaveBlocks * 4) throw HipError{hipErrorInvalidValue, "more than 2^24 filters in one Messages batch"};
  const DevIndex di = dev_index(ix);
  const uint32_t nb = (n + kScanBlock - 1) / kScanBlock;
  counts_.ensure((size_t)n * sizeof(TopicCount));
  offs_.ensure((size_t)(n + 1) * sizeof(TopicOff));
  bsum_.ensure((size_t)(nb + 1) * sizeof(TopicOff));
  bpre_.ensure((size_t)(nb + 1) * sizeof(TopicOff));
  TopicOff tot{0, 0, 0, 0, 0};
  // The image path needs Retained.Get("") only on particles with a retain path; with the Q6
  // entry live, a literal level can emit on any particle, which the particle walk covers.
  bool done = false;
  if (img_path) {
    ensure_img(ix, di, s);
    done = messages_img(di, d_fb, d_fo, n, s, &tot, runs != nullptr);
  }
  if (!done) messages_walk(ix, di, d_fb, d_fo, n, s, &tot);
  if (runs) {
    if (!done) {  // the particle walk's own handles, one run per filter
      if (tot.rows >> 32) throw HipError{hipErrorInvalidValue, "Messages runs: a walked batch of 2^32 handles or more"};
      msg_rbase_.ensure((size_t)n * sizeof(uint64_t));
      msg_rcnt_.ensure((size_t)n * sizeof(uint32_t));
      msg_pieces_.ensure((size_t)n * sizeof(MsgPiece));
      launch_msg_runs_of(n, msg_base_.as<uint64_t>(), msg_count_.as<uint32_t>(), msg_pieces_.as<MsgPiece>(),
                         msg_rbase_.as<uint64_t>(), msg_rcnt_.as<uint32_t>(), s);
      hip_check(hipGetLastError(), "k_msg_runs_of");
      tot.g = n;
    }
    static_assert(sizeof(MsgPiece) == sizeof(mq_msg_run), "a piece is the ABI's run");
    runs->n_filters = n;
    runs->run_base = msg_rbase_.as<uint64_t>();
    runs->n_runs = msg_rcnt_.as<uint32_t>();
    runs->base = msg_base_.as<uint64_t>();
    runs->count = msg_count_.as<uint32_t>();
    runs->runs = msg_pieces_.as<mq_msg_run>();
    runs->n_runs_total = tot.g;
    runs->handles = done ? img_h_.as<uint64_t>() : msg_handles_.as<uint64_t>();
    runs->n_handles = done ? img_live_ : tot.rows;
    runs->n_expanded = tot.rows;
    if (hruns) {
      hruns->run_base.resize(n);
      hruns->n_runs.resize(n);
      hruns->base.resize(n);
      hruns->count.resize(n);
      hruns->runs.resize(tot.g);
      auto d2h = [&](void* dst, const void* src, size_t bytes) {
        if (bytes) hip_check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s), "D2H runs");
      };
      d2h(hruns->run_base.data(), runs->run_base, n * sizeof(uint64_t));
      d2h(hruns->n_runs.data(), runs->n_runs, n * sizeof(uint32_t));
      d2h(hruns->base.data(), runs->base, n * sizeof(uint64_t));
      d2h(hruns->count.data(), runs->count, n * sizeof(uint32_t));
      d2h(hruns->runs.data(), runs->runs, tot.g * sizeof(MsgPiece));
      if (done) {  // the image's handles: one host copy per image version, shared by the results
        if (!host_img_ || host_img_version_ != img_version_) {
          auto hv = std::make_shared<PinnedVec<uint64_t>>(img_live_);
          d2h(hv->data(), img_h_.p, img_live_ * sizeof(uint64_t));
          host_img_ = std::move(hv);
          host_img_version_ = img_version_;
        }
        hruns->handles = host_img_;
      } else {
        auto hv = std::make_shared<PinnedVec<uint64_t>>(tot.rows);
        d2h(hv->data(), msg_handles_.p, tot.rows * sizeof(uint64_t));
        hruns->handles = std::move(hv);
      }
      hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
      check_err(s);
    }
    return;
  }
  out->n_filters = n;
  out->base = msg_base_.as<uint64_t>();
  out->count = msg_count_.as<uint32_t>();
  out->handles = msg_handles_.as<uint64_t>();
  out->n_handles = tot.rows;
  if (host) {
    host->base.resize(n);
    host->count.resize(n);
    host->handles.resize(tot.rows);
    hip_check(hipMemcpyAsync(host->base.data(), msg_base_.p, n * sizeof(uint64_t), hipMemcpyDeviceToHost, s), "D2H");
    hip_check(hipMemcpyAsync(host->count.data(), msg_count_.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost, s), "D2H");
    if (tot.rows)
      hip_check(hipMemcpyAsync(host->handles.data(), msg_handles_.p, tot.rows * sizeof(uint64_t),
                               hipMemcpyDeviceToHost, s), "D2H handles");
    hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
    check_err(s);
  }
}

template struct DevMirror<EdgeSlot>;
template struct DevMirror<NodeWalk>;
template struct DevMirror<NodeLists>;
template struct DevMirror<NodeInl>;
template struct DevMirror<NodeMsg>;
template struct DevMirror<SegInfo>;
template struct DevMirror<uint8_t>;
template struct DevMirror<SubRec>;
template struct DevMirror<MergeRef>;
template struct DevMirror<MergePart>;
template struct DevMirror<NodePair>;
template struct DevMirror<PairEnt>;
template struct DevMirror<PairSlot>;
template struct DevMirror<ShrRec>;
template struct DevMirror<InlRec>;
template struct DevMirror<uint32_t>;
template struct DevMirror<ChildRec>;

}  // namespace mq
