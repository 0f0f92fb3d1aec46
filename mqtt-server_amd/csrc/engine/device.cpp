// Device side of the engine (device.h): HBM mirror + batch pipeline.
#include "device.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace mq {

void hip_check(hipError_t e, const char* where) {
  if (e != hipSuccess) throw HipError{e, std::string(where) + ": " + hipGetErrorString(e)};
}

void DevBuf::ensure(size_t b) {
  if (b <= bytes && p) return;
  release();
  size_t nb = std::max<size_t>(b, 256);
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
}

template <class T>
void DevMirror<T>::sync(Mirror<T>& m, hipStream_t s, uint64_t* uploaded) {
  const size_t n = m.size();
  bool full = m.all_dirty;
  if (!d || m.epoch != epoch || cap < n) {
    release();
    cap = std::max<size_t>(std::max(m.h.capacity(), n), 1);
    hip_check(hipMalloc(&d, cap * sizeof(T)), "hipMalloc(mirror)");
    epoch = m.epoch;
    full = true;
  }
  if (full) {
    if (n) hip_check(hipMemcpyAsync(d, m.h.data(), n * sizeof(T), hipMemcpyHostToDevice, s), "H2D mirror");
    *uploaded += n * sizeof(T);
  } else {
    const size_t pp = Mirror<T>::per_page();
    const size_t npages = (n + pp - 1) / pp;
    size_t p = 0;
    while (p < npages) {
      if (!(p / 64 < m.dirty.size() && (m.dirty[p / 64] >> (p % 64)) & 1)) {
        p++;
        continue;
      }
      size_t q = p;
      while (q < npages && q / 64 < m.dirty.size() && ((m.dirty[q / 64] >> (q % 64)) & 1)) q++;
      const size_t a = p * pp, b = std::min(n, q * pp);
      hip_check(hipMemcpyAsync(d + a, m.h.data() + a, (b - a) * sizeof(T), hipMemcpyHostToDevice, s),
                "H2D dirty pages");
      *uploaded += (b - a) * sizeof(T);
      p = q;
    }
  }
  m.clear_dirty();
}

// ---- profiler ----------------------------------------------------------------------------------
void Profiler::begin(hipStream_t s) {
  if (!on_) return;
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
  const char* e = getenv("MQ_CHUNK_ROWS");
  chunk_rows_budget_ = e ? strtoull(e, nullptr, 10) : (256ull << 20);  // 4 GiB of 16-B rows
  const char* ms = getenv("MQ_MERGE_STATS");  // diagnosis only
  merge_stats_ = ms != nullptr;
  if (ms && *ms) tstat_path_ = ms;
  int cus = 0;
  hip_check(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev_), "hipDeviceGetAttribute");
  n_cus_ = (uint32_t)std::max(1, cus);
  read_knobs();
}

// Tuning and diagnosis knobs, re-read per batch (development only; the defaults are the product).
void Device::read_knobs() {
  auto knob = [](const char* name, uint32_t def) {
    const char* v = getenv(name);
    return v ? (uint32_t)atoi(v) : def;
  };
  serial_ = getenv("MQ_SERIAL") != nullptr;                      // k_merge on the launch stream
  // 0: one wavefront per tile / topic; else a persistent grid of that many workgroups per CU
  copy_blocks_ = n_cus_ * knob("MQ_COPY_BLOCKS_PER_CU", kCopyBlocksPerCU);
  merge_blocks_ = n_cus_ * knob("MQ_MERGE_BLOCKS_PER_CU", kMergeBlocksPerCU);
  merge_diag_ = knob("MQ_MERGE_DIAG", 0);
}

Device::~Device() {
  (void)hipSetDevice(dev_);
  edges_.release(); walk_.release(); lists_.release(); msg_.release(); seginfo_.release();
  segbytes_.release(); subs_.release(); shr_.release(); inl_.release(); children_.release();
  mref_.release(); mpart_.release(); npair_.release(); pent_.release(); plist_.release();
  for (DevBuf* b : {&in_bytes_, &in_offs_, &counts_, &offs_, &bsum_, &bpre_, &gathers_, &err_, &desc_,
                    &msg_handles_, &msg_base_, &msg_count_, &gslots_, &mstats_, &tstat_, &tiles_, &plan_})
    b->release();
  for (int k = 0; k < 2; k++) {
    for (DevBuf* b : {&rows_[k], &shr_rows_[k], &inl_rows_[k], &res_[k]}) b->release();
    if (copy_done_[k]) (void)hipEventDestroy(copy_done_[k]);
    if (merge_done_[k]) (void)hipEventDestroy(merge_done_[k]);
  }
  if (side_done_) (void)hipEventDestroy(side_done_);
  if (side_) (void)hipStreamDestroy(side_);
}

uint64_t Device::device_bytes() const {
  uint64_t b = edges_.cap * sizeof(EdgeSlot) + walk_.cap * sizeof(NodeWalk) +
               lists_.cap * sizeof(NodeLists) + msg_.cap * sizeof(NodeMsg) +
               seginfo_.cap * sizeof(SegInfo) + segbytes_.cap + subs_.cap * sizeof(SubRec) +
               shr_.cap * sizeof(ShrRec) + inl_.cap * sizeof(InlRec) + children_.cap * 4 +
               mref_.cap * sizeof(MergeRef) + mpart_.cap * sizeof(MergePart) +
               npair_.cap * sizeof(NodePair) + pent_.cap * sizeof(PairEnt) + plist_.cap * sizeof(PairSlot);
  for (const DevBuf* x : {&in_bytes_, &in_offs_, &counts_, &offs_, &bsum_, &bpre_, &gathers_, &desc_, &tiles_})
    b += x->bytes;
  for (int k = 0; k < 2; k++)
    for (const DevBuf* x : {&rows_[k], &shr_rows_[k], &inl_rows_[k], &res_[k]}) b += x->bytes;
  return b;
}

void Device::sync(Index& ix, hipStream_t s) {
  hip_check(hipSetDevice(dev_), "hipSetDevice");
  if (ix.version() == synced_version_ && edges_.d) return;
  ix.flush_merge();
  edges_.sync(ix.edges, s, &uploaded_);
  walk_.sync(ix.walk, s, &uploaded_);
  lists_.sync(ix.lists, s, &uploaded_);
  msg_.sync(ix.msg, s, &uploaded_);
  seginfo_.sync(ix.seginfo, s, &uploaded_);
  segbytes_.sync(ix.segbytes, s, &uploaded_);
  subs_.sync(ix.subs.m, s, &uploaded_);
  mref_.sync(ix.mref, s, &uploaded_);
  mpart_.sync(ix.mpart.m, s, &uploaded_);
  npair_.sync(ix.npair, s, &uploaded_);
  pent_.sync(ix.pent.m, s, &uploaded_);
  plist_.sync(ix.plist.m, s, &uploaded_);
  shr_.sync(ix.shr.m, s, &uploaded_);
  inl_.sync(ix.inl.m, s, &uploaded_);
  children_.sync(ix.children.m, s, &uploaded_);
  retained_len_ = ix.retained_len();
  empty_live_ = ix.empty_topic_live;
  empty_handle_ = ix.empty_topic_handle;
  synced_version_ = ix.version();
  syncs_++;
}

DevIndex Device::dev_index(const Index& ix) const {
  DevIndex d;
  d.edges = edges_.d;
  d.edge_mask = ix.edge_mask();
  d.walk = walk_.d;
  d.lists = lists_.d;
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
                                        ((e & kErrTableFull) ? "merge table full" : "")};
  }
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

void Device::match(Index& ix, const uint8_t* d_tb, const uint64_t* d_to, uint32_t n, hipStream_t s,
                   HostMatch* host, mq_match_result* out) {
  hip_check(hipSetDevice(dev_), "hipSetDevice");
  read_knobs();
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
  const DevIndex di = dev_index(ix);
  const uint32_t nb = (n + kScanBlock - 1) / kScanBlock;

  counts_.ensure((size_t)n * sizeof(TopicCount));
  offs_.ensure((size_t)(n + 1) * sizeof(TopicOff));
  bsum_.ensure((size_t)(nb + 1) * sizeof(TopicOff));
  bpre_.ensure((size_t)(nb + 1) * sizeof(TopicOff));

  gslots_.ensure((size_t)n * kGatherCap * sizeof(uint32_t));
  prof.begin(s);
  launch_walk(false, d_tb, d_to, n, di, counts_.as<TopicCount>(), nullptr, gslots_.as<uint32_t>(), s);
  prof.end("walk", s);
  hip_check(hipGetLastError(), "k_walk<count>");
  prof.begin(s);
  launch_scan(counts_.as<TopicCount>(), n, bsum_.as<TopicOff>(), bpre_.as<TopicOff>(), offs_.as<TopicOff>(), s);
  prof.end("scan", s);
  hip_check(hipGetLastError(), "k_scan");

  h_bpre_.resize(nb + 1);
  hip_check(hipMemcpyAsync(h_bpre_.data(), bpre_.p, (nb + 1) * sizeof(TopicOff), hipMemcpyDeviceToHost, s),
            "D2H block offsets");
  uint32_t overflow = 0;
  hip_check(hipMemcpyAsync(&overflow, err_.as<uint32_t>() + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, s),
            "D2H overflow");
  hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
  check_err(s);
  const TopicOff tot = h_bpre_[nb];

  prof.count("topics", n);
  prof.count("gathers", tot.g);
  prof.count("reserved_rows", tot.rows);
  // A topic with more gathers than its count-pass slots: write all gather lists compactly.
  const uint32_t* gathers = gslots_.as<uint32_t>();
  uint32_t gstride = kGatherCap;
  if (overflow) {
    hip_check(hipMemsetAsync(err_.as<uint32_t>() + 1, 0, sizeof(uint32_t), s), "hipMemsetAsync");
    gathers_.ensure(std::max<uint64_t>(tot.g, 1) * sizeof(uint32_t));
    prof.begin(s);
    launch_walk(true, d_tb, d_to, n, di, nullptr, offs_.as<TopicOff>(), gathers_.as<uint32_t>(), s);
    prof.end("walk_fill", s);
    hip_check(hipGetLastError(), "k_walk<fill>");
    gathers = gathers_.as<uint32_t>();
    gstride = 0;
  }

  // plan output chunks on scan-block boundaries so each chunk's rows fit the budget
  struct Chunk {
    uint32_t b0, b1;
  };
  std::vector<Chunk> chunks;
  std::vector<ChunkPlan> plan;
  std::vector<uint32_t> chunk_of_block(nb);
  uint64_t max_rows = 1, max_shr = 1, max_inl = 1, max_topics = 1, total_tiles = 0;
  auto tiles_of = [](uint64_t rows) { return (rows + kCopyTile - 1) / kCopyTile; };
  for (uint32_t b = 0; b < nb;) {
    uint32_t e = b + 1;
    while (e < nb && h_bpre_[e + 1].rows - h_bpre_[b].rows <= chunk_rows_budget_) e++;
    const TopicOff &lo = h_bpre_[b], &hi = h_bpre_[e];
    for (uint32_t k = b; k < e; k++) chunk_of_block[k] = (uint32_t)chunks.size();
    chunks.push_back(Chunk{b, e});
    ChunkPlan p;
    p.rows = lo.rows;
    p.shr = lo.shr;
    p.inl = lo.inl;
    p.tile_off = (uint32_t)total_tiles;
    p.n_tiles0 = (uint32_t)tiles_of(hi.rows - lo.rows);
    p.n_tiles1 = (uint32_t)tiles_of(hi.shr - lo.shr);
    p.pad = 0;
    plan.push_back(p);
    max_rows = std::max(max_rows, hi.rows - lo.rows);
    max_shr = std::max(max_shr, hi.shr - lo.shr);
    max_inl = std::max(max_inl, hi.inl - lo.inl);
    total_tiles += tiles_of(hi.rows - lo.rows) + tiles_of(hi.shr - lo.shr) + tiles_of(hi.inl - lo.inl);
    max_topics = std::max<uint64_t>(max_topics, std::min<uint64_t>(n, (uint64_t)e * kScanBlock) - (uint64_t)b * kScanBlock);
    b = e;
  }
  if (max_rows >= (1ull << 32) || max_shr >= (1ull << 32) || max_inl >= (1ull << 32) || total_tiles >= (1ull << 32))
    throw HipError{hipErrorInvalidValue, "one scan block's output exceeds 2^32 rows"};
  const size_t nbuf = chunks.size() > 1 ? 2 : 1;
  for (size_t k = 0; k < nbuf; k++) {
    rows_[k].ensure(max_rows * sizeof(SubRec));
    shr_rows_[k].ensure(max_shr * sizeof(ShrRec));
    inl_rows_[k].ensure(max_inl * sizeof(InlRec));
    res_[k].ensure(max_topics * sizeof(mq_topic_result_dev));
  }
  desc_.ensure(std::max<uint64_t>(tot.g, 1) * sizeof(GDesc));
  tiles_.ensure(std::max<uint64_t>(total_tiles, 1) * sizeof(uint32_t));
  plan_.ensure(plan.size() * sizeof(ChunkPlan) + nb * sizeof(uint32_t));
  h_plan_.resize(plan.size() * sizeof(ChunkPlan) + nb * sizeof(uint32_t));
  memcpy(h_plan_.data(), plan.data(), plan.size() * sizeof(ChunkPlan));
  memcpy(h_plan_.data() + plan.size() * sizeof(ChunkPlan), chunk_of_block.data(), nb * sizeof(uint32_t));
  hip_check(hipMemcpyAsync(plan_.p, h_plan_.data(), h_plan_.size(), hipMemcpyHostToDevice, s), "H2D chunk plan");
  if (!side_) {
    hip_check(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking), "hipStreamCreate");
    for (int k = 0; k < 2; k++) {
      hip_check(hipEventCreateWithFlags(&copy_done_[k], hipEventDisableTiming), "hipEventCreate");
      hip_check(hipEventCreateWithFlags(&merge_done_[k], hipEventDisableTiming), "hipEventCreate");
    }
    hip_check(hipEventCreateWithFlags(&side_done_, hipEventDisableTiming), "hipEventCreate");
  }

  // every topic's gathers become GDesc records and k_copy tile starts, in one launch
  DescArgs da;
  da.ix = di;
  da.n = n;
  da.gather_stride = gstride;
  da.off = offs_.as<TopicOff>();
  da.gathers = gathers;
  da.plan = reinterpret_cast<const ChunkPlan*>(plan_.p);
  da.chunk_of_block = reinterpret_cast<const uint32_t*>(plan_.as<uint8_t>() + plan.size() * sizeof(ChunkPlan));
  da.desc = desc_.as<GDesc>();
  da.tiles = tiles_.as<uint32_t>();
  prof.begin(s);
  launch_desc(da, s);
  prof.end("desc", s);
  hip_check(hipGetLastError(), "k_desc");

  if (host) {
    host->topics.resize(n);
    host->rows.resize(tot.rows);
    host->shr.resize(tot.shr);
    host->inl.resize(tot.inl);
  }

  // Per chunk: k_desc + k_copy on the launch stream, then k_merge (and, for host results, the
  // D2H copies) on the side stream. Chunk i + 2 reuses chunk i's buffers after its merge.
  hipStream_t cs = s;  // k_copy stream
  for (size_t ci = 0; ci < chunks.size(); ci++) {
    const Chunk& c = chunks[ci];
    const size_t b = ci % nbuf;
    const TopicOff& lo = h_bpre_[c.b0];
    const TopicOff& hi = h_bpre_[c.b1];
    EmitArgs a;
    a.ix = di;
    a.t0 = c.b0 * kScanBlock;
    a.t1 = std::min<uint64_t>(n, (uint64_t)c.b1 * kScanBlock);
    a.off = offs_.as<TopicOff>();
    a.base = lo;
    a.desc = desc_.as<GDesc>();
    a.tiles = tiles_.as<uint32_t>() + plan[ci].tile_off;
    a.total[0] = (uint32_t)(hi.rows - lo.rows);
    a.total[1] = (uint32_t)(hi.shr - lo.shr);
    a.total[2] = (uint32_t)(hi.inl - lo.inl);
    for (int k = 0; k < 3; k++) a.n_tiles[k] = (uint32_t)tiles_of(a.total[k]);
    a.rows = rows_[b].as<SubRec>();
    a.shr_rows = shr_rows_[b].as<ShrRec>();
    a.inl_rows = inl_rows_[b].as<InlRec>();
    a.res = res_[b].as<mq_topic_result_dev>();
    a.stats = nullptr;
    a.tstat = nullptr;
    a.diag = merge_diag_;
    if (!tstat_path_.empty()) {
      if (ci == 0) tstat_.ensure((size_t)n * kTStat * sizeof(uint32_t));
      a.tstat = tstat_.as<uint32_t>();
    }
    if (merge_stats_) {
      if (!mstats_.p) {
        mstats_.ensure(4 * sizeof(unsigned long long));
        hip_check(hipMemsetAsync(mstats_.p, 0, 4 * sizeof(unsigned long long), s), "memset stats");
      }
      a.stats = mstats_.as<unsigned long long>();
    }
    if (ci >= nbuf) hip_check(hipStreamWaitEvent(cs, merge_done_[b], 0), "hipStreamWaitEvent");
    prof.begin(cs);
    launch_copy(a, copy_blocks_, cs);
    prof.end("copy", cs);
    hip_check(hipGetLastError(), "k_copy");
    hipStream_t ms = serial_ ? cs : side_;
    if (!serial_) {
      hip_check(hipEventRecord(copy_done_[b], cs), "hipEventRecord");
      hip_check(hipStreamWaitEvent(side_, copy_done_[b], 0), "hipStreamWaitEvent");
    }
    prof.begin(ms);
    launch_merge(a, merge_blocks_, ms);
    prof.end("merge", ms);
    hip_check(hipGetLastError(), "k_merge");
    prof.count("copy_rows", (uint64_t)a.total[0] + a.total[1] + a.total[2]);
    prof.count("copy_bytes", 16ull * a.total[0] + 8ull * a.total[1] + 8ull * a.total[2]);
    prof.count("merge_records", hi.merge - lo.merge);
    last_chunks_++;

    const uint32_t nt = a.t1 - a.t0;
    if (host) {
      hip_check(hipMemcpyAsync(host->rows.data() + lo.rows, a.rows, (hi.rows - lo.rows) * sizeof(SubRec),
                               hipMemcpyDeviceToHost, ms), "D2H rows");
      hip_check(hipMemcpyAsync(host->shr.data() + lo.shr, a.shr_rows, (hi.shr - lo.shr) * sizeof(ShrRec),
                               hipMemcpyDeviceToHost, ms), "D2H shared rows");
      hip_check(hipMemcpyAsync(host->inl.data() + lo.inl, a.inl_rows, (hi.inl - lo.inl) * sizeof(InlRec),
                               hipMemcpyDeviceToHost, ms), "D2H inline rows");
      hip_check(hipMemcpyAsync(host->topics.data() + a.t0, a.res, nt * sizeof(mq_topic_result),
                               hipMemcpyDeviceToHost, ms), "D2H topic results");
    }
    hip_check(hipEventRecord(merge_done_[b], ms), "hipEventRecord");
    if (merge_stats_) {  // diagnosis only: cumulative since the Device was created
      unsigned long long m[4];
      hip_check(hipMemcpyAsync(m, a.stats, sizeof(m), hipMemcpyDeviceToHost, ms), "D2H stats");
      hip_check(hipStreamSynchronize(ms), "hipStreamSynchronize");
      fprintf(stderr, "[merge] hit lists %llu records resolved %llu slow-path topics %llu\n", m[0], m[1], m[2]);
    }
    out->n_topics = nt;
    out->topics = reinterpret_cast<const mq_topic_result*>(a.res);
    out->sub_rows = reinterpret_cast<const mq_client_row*>(a.rows);
    out->shared_rows = reinterpret_cast<const mq_shared_row*>(a.shr_rows);
    out->inline_rows = reinterpret_cast<const mq_inline_row*>(a.inl_rows);
    out->n_sub_rows = hi.rows - lo.rows;
    out->n_shared_rows = hi.shr - lo.shr;
    out->n_inline_rows = hi.inl - lo.inl;
  }
  // the launch stream completes only after the side stream's work of this batch
  hip_check(hipEventRecord(side_done_, side_), "hipEventRecord");
  hip_check(hipStreamWaitEvent(s, side_done_, 0), "hipStreamWaitEvent");
  if (!tstat_path_.empty()) {  // diagnosis only: per-topic k_merge counters of this batch
    std::vector<uint32_t> h((size_t)n * kTStat);
    hip_check(hipMemcpyAsync(h.data(), tstat_.p, h.size() * 4, hipMemcpyDeviceToHost, s), "D2H tstat");
    hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
    if (FILE* f = fopen(tstat_path_.c_str(), "wb")) {
      fwrite(h.data(), 4, h.size(), f);
      fclose(f);
    }
  }
  if (host) {
    hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
    for (const Chunk& c : chunks) {
      const TopicOff& lo = h_bpre_[c.b0];
      const uint32_t t0 = c.b0 * kScanBlock, t1 = (uint32_t)std::min<uint64_t>(n, (uint64_t)c.b1 * kScanBlock);
      for (uint32_t t = t0; t < t1; t++) {
        mq_topic_result& r = host->topics[t];
        r.sub_base += lo.rows;
        r.shared_base += lo.shr;
        r.inline_base += lo.inl;
      }
    }
    check_err(s);
  }
}

void Device::messages(Index& ix, const uint8_t* d_fb, const uint64_t* d_fo, uint32_t n,
                      hipStream_t s, HostMsg* host, mq_msg_result* out) {
  hip_check(hipSetDevice(dev_), "hipSetDevice");
  sync(ix, s);
  *out = mq_msg_result{};
  if (host) *host = HostMsg{};
  if (!err_.p) {
    err_.ensure(2 * sizeof(uint32_t));
    hip_check(hipMemsetAsync(err_.p, 0, 2 * sizeof(uint32_t), s), "hipMemsetAsync(err)");
  }
  check_err(s);
  if (n == 0) return;
  const DevIndex di = dev_index(ix);
  const uint32_t nb = (n + kScanBlock - 1) / kScanBlock;
  counts_.ensure((size_t)n * sizeof(TopicCount));
  offs_.ensure((size_t)(n + 1) * sizeof(TopicOff));
  bsum_.ensure((size_t)(nb + 1) * sizeof(TopicOff));
  bpre_.ensure((size_t)(nb + 1) * sizeof(TopicOff));
  prof.begin(s);
  launch_msg(false, d_fb, d_fo, n, di, counts_.as<TopicCount>(), nullptr, nullptr, nullptr, nullptr, s);
  prof.end("msg_count", s);
  hip_check(hipGetLastError(), "k_msg<count>");
  launch_scan(counts_.as<TopicCount>(), n, bsum_.as<TopicOff>(), bpre_.as<TopicOff>(), offs_.as<TopicOff>(), s);
  hip_check(hipGetLastError(), "k_scan");
  TopicOff tot;
  hip_check(hipMemcpyAsync(&tot, bpre_.as<TopicOff>() + nb, sizeof(TopicOff), hipMemcpyDeviceToHost, s), "D2H total");
  hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
  check_err(s);
  msg_handles_.ensure(std::max<uint64_t>(tot.rows, 1) * sizeof(uint64_t));
  msg_base_.ensure((size_t)n * sizeof(uint64_t));
  msg_count_.ensure((size_t)n * sizeof(uint32_t));
  prof.begin(s);
  launch_msg(true, d_fb, d_fo, n, di, nullptr, offs_.as<TopicOff>(), msg_handles_.as<uint64_t>(),
             msg_base_.as<uint64_t>(), msg_count_.as<uint32_t>(), s);
  prof.end("msg_fill", s);
  hip_check(hipGetLastError(), "k_msg<fill>");
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

}  // namespace mq
