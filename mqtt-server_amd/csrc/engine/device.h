// Device side of the engine: the HBM-resident mirror of the index image and the batched match
// pipeline (walk-count -> scan -> [walk-fill] -> per output chunk: desc -> copy -> merge).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <memory>

#include <new>
#include <string>
#include <utility>
#include <vector>

#include "index.h"
#include "kernels.h"
#include "mqmatch.h"

namespace mq {

struct HipError {
  hipError_t code;
  std::string where;
};
void hip_check(hipError_t e, const char* where);

// Device allocation owned by its holder: released by the destructor (a buffer added to Device
// cannot leak on mq_index_destroy), never copied.
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void ensure(size_t b);
  void release();
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

// Dirty runs of the host mirrors collected by one Device::sync (host source, device target).
struct Stager {
  struct Run {
    void* dst;
    const void* src;
    size_t bytes;
  };
  std::vector<Run> runs;
  size_t bytes = 0;
  std::vector<void*> frees;  // device arrays a sync replaced: freed outside the handle lock
                             //   (hipFree waits for the device; Device::release_retired)
  void add(void* dst, const void* src, size_t n);  // split into runs of <= kScatterRun
};

// A reallocated or mostly dirty array this small goes whole through the pinned staging buffer
// (DevMirror::sync): no pageable copy, and no wait for one, under the handle lock.
constexpr size_t kStageWhole = 8u << 20;

template <class T>
struct DevMirror {
  T* d = nullptr;
  size_t cap = 0;
  uint64_t epoch = ~0ull;
  void* spare = nullptr;  // an allocation made ahead, outside the handle lock (Device::prealloc)
  size_t spare_bytes = 0;
  // bytes the next sync of m allocates (0: none)
  size_t need_bytes(const Mirror<T>& m) const {
    const size_t n = m.size();
    if (d && m.epoch == epoch && cap >= n) return 0;
    return std::max<size_t>(std::max(m.h.capacity(), n), 1) * sizeof(T);
  }
  DevMirror() = default;
  DevMirror(const DevMirror&) = delete;
  DevMirror& operator=(const DevMirror&) = delete;
  ~DevMirror() { release(); }
  // reallocated or mostly dirty: uploaded whole now (returns true); else its dirty pages go to `st`
  bool sync(Mirror<T>& m, hipStream_t s, uint64_t* uploaded, Stager& st);
  void release();
};

// Page-locked host memory for results copied to the host: D2H into pageable memory runs at a few
// GB/s, into pinned memory at PCIe rate. Blocks are pooled (page-locking is slow) and elements are
// default-initialised (resize does not zero gigabytes of rows that the D2H overwrites).
void* pinned_alloc(size_t bytes);
// MQ_SLOW_MS=<ms> (diagnosis): a C-ABI call that holds the handle lock longer than that prints the
// milestones its thread marked (slow_mark: the name and the ms since slow_begin) to stderr
bool slow_on();
void slow_begin();
void slow_mark(const char* what);
void slow_report(const char* call, double threshold_ms);
void pinned_free(void* p, size_t bytes);

template <class T>
struct PinnedAlloc {
  using value_type = T;
  PinnedAlloc() = default;
  template <class U>
  PinnedAlloc(const PinnedAlloc<U>&) {}
  T* allocate(size_t n) { return static_cast<T*>(pinned_alloc(n * sizeof(T))); }
  void deallocate(T* p, size_t n) { pinned_free(p, n * sizeof(T)); }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    if constexpr (sizeof...(A) == 0) ::new (static_cast<void*>(p)) U;
    else ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
  }
  template <class U>
  bool operator==(const PinnedAlloc<U>&) const { return true; }
  template <class U>
  bool operator!=(const PinnedAlloc<U>&) const { return false; }
};
template <class T>
using PinnedVec = std::vector<T, PinnedAlloc<T>>;

// Host-side destination of a Messages batch (mq_messages_batch).
struct HostMsg {
  PinnedVec<uint64_t> base;
  PinnedVec<uint32_t> count;
  PinnedVec<uint64_t> handles;
};

// Host-side destination of a Messages runs batch (mq_messages_runs_batch): the runs, and the
// array they index — a host copy of the retained image's handles, shared by every result of one
// image version, or the batch's own handles (particle walk).
struct HostMsgRuns {
  PinnedVec<uint64_t> run_base, base;
  PinnedVec<uint32_t> n_runs, count;
  PinnedVec<MsgPiece> runs;
  std::shared_ptr<const PinnedVec<uint64_t>> handles;
};

// Host-side destination of a batched MatchTopic (mq_acl_match_batch).
struct HostAcl {
  PinnedVec<uint8_t> matched;
  PinnedVec<uint32_t> n_elems;
  PinnedVec<uint64_t> elem_base;
  PinnedVec<uint32_t> elems;
};

// Host-side destination of a span-format batch (mq_match_spans).
struct HostSpans {
  PinnedVec<TopicSpansDev> topics;
  PinnedVec<SpanRec> spans;
  PinnedVec<PatchRec> patches;
  PinnedVec<InlRec> inl;
  PinnedVec<ShrRec> picked;
  PinnedVec<PatchRec> set_patches;  // merge-set patches, packed (set_patches of the result)
  PinnedVec<uint32_t> merge_rows;   // merge rows of the topics that reference a set, packed
  PinnedVec<uint32_t> merge_base;   //   and where each topic's start
  bool codes = false;               // patches / set patches as 4-byte codes (MQ_SPANS_PATCH_CODES):
  PinnedVec<uint32_t> patch_codes, set_codes;  //   then these instead of patches / set_patches
};

// Host-side destination of a batch's results (mq_match_batch).
struct HostMatch {
  PinnedVec<mq_topic_result> topics;
  PinnedVec<SubRec> rows;
  PinnedVec<ShrRec> shr;
  PinnedVec<InlRec> inl;
};

class Profiler {
 public:
  Profiler() = default;
  Profiler(const Profiler&) = delete;
  Profiler& operator=(const Profiler&) = delete;
  ~Profiler() {
    for (auto& p : pending_) {
      (void)hipEventDestroy(p.a);
      (void)hipEventDestroy(p.b);
    }
    for (hipEvent_t e : free_) (void)hipEventDestroy(e);
    if (cur_) (void)hipEventDestroy(cur_);
  }
  void enable(bool on, bool work = false, bool walk_only = false) {
    on_ = on;
    work_ = on && work;
    walk_only_ = on && walk_only;
  }
  bool on() const { return on_; }
  bool work() const { return work_; }  // MQ_PROF_WORK: kernel work counters
  void begin(hipStream_t s, const char* name);  // (name: the launch's, as end() gives it)
  void end(const char* name, hipStream_t s);
  int read(mq_kernel_time* out, uint32_t cap);
  // Event counters reported next to the kernels (launches = count, total_ms = 0).
  void count(const char* name, uint64_t n);
  void reset();

 private:
  struct Pending {
    std::string name;
    hipEvent_t a, b;
  };
  struct Total {
    std::string name;
    uint64_t launches = 0;
    double ms = 0;
  };
  void drain();
  bool on_ = false, work_ = false, walk_only_ = false;
  hipEvent_t cur_ = nullptr;
  std::vector<Pending> pending_;
  std::vector<hipEvent_t> free_;
  std::vector<Total> totals_;
};

// What a span batch reads of the host image, taken when the device image is synced
// (Device::prepare, under the handle lock): the batch's kernels then run without the lock while
// updates change the host image (capi.cpp Access::kMatch; topics.go:402 — writers serialise only
// with each other and with the sync, never with a match's GPU work).
struct IndexSnap {
  uint64_t version = ~0ull;
  bool sharded = false;
  uint32_t shard = 0;
  bool inl_live = false;        // inline subscriptions exist
  uint64_t n_nodes = 0, n_wild = 0;
  uint64_t subs_len = 0, shr_len = 0;  // the subscription pools' lengths (results name them)
  uint32_t max_sub_cap = 0;
  bool deep_live = false;       // a sharded index knows filters deeper than 32 levels
  DevIndex di{};
};

class Device {
 public:
  explicit Device(int dev);
  ~Device();
  int device() const { return dev_; }
  // The stream of host-buffer calls (mq_match_spans): its own, non-blocking.
  hipStream_t host_stream();
  hipStream_t host_stream_made() const { return hstream_; }  // (after begin_prepare: no HIP call)

  // Upload dirty pages of the index image (incremental device-side update).
  void sync(Index& ix, hipStream_t s);
  // Sync, then take the snapshot the next span batch runs on (under the handle lock; the batch
  // itself may then run without it). Uploads straight from the host image (a reallocated or
  // mostly dirty array) are waited for, so an update may change the image once this returns.
  void prepare(Index& ix, hipStream_t s);
  // Before the handle lock: the device set on this thread, the last staged upload done (prepare
  // then makes no HIP call that could wait behind another thread's).
  void begin_prepare();
  const IndexSnap& snap() const { return snap_; }
  // The allocations the next sync of ix would make (device arrays that grew, the staging buffers
  // for its dirty pages), read under the handle lock, so that prealloc makes them outside it:
  // hipMalloc and hipHostMalloc take milliseconds, which an update would otherwise wait for.
  struct SyncPlan {
    size_t mirror[19] = {};
    size_t stage = 0;
    bool any = false;  // something the spares do not cover yet
  };
  SyncPlan sync_plan(Index& ix) const;  // (runs the index's deferred merge-record rebuilds first)
  void prealloc(const SyncPlan& p);
  // Free the device arrays that syncs replaced (nothing on the device reads them any more: the
  // work that did ran under the device lock before the sync).
  void release_retired();
  // the index changed since the pending batch's spans_begin (the two-phase sharded calls)
  bool batch_stale(const Index& ix) const { return ix.version() != sb_.version; }
  // Diagnostic: sync, then read every device array back and compare it with the host mirror;
  // returns "" or the first difference.
  std::string verify(Index& ix);
  // Match n topics resident on the device. Fills `out` with device pointers of the last chunk;
  // when `host` is set every chunk's rows are also copied into it (global offsets).
  // fn (optional): per-chunk consumer (mq_match_device_chunks), called before the chunk's
  // buffers are released for reuse.
  void match(Index& ix, const uint8_t* d_tb, const uint64_t* d_to, uint32_t n, hipStream_t s,
             HostMatch* host, mq_match_result* out, mq_chunk_fn fn = nullptr, void* user = nullptr);
  // Span format (mq_match_spans*): spans + patches + inline rows of n topics on the device; the
  // call returns after the kernels completed and their guard flags were checked. `host`: also
  // copies every array into it (out's pointers then still name the device arrays).
  // ready (host results): the copy into `host` runs on the copy stream beside whatever the
  // device does next (the next batch's kernels), and `ready` is recorded when it is done; without
  // it the call returns after the copy. `issued` (with ready) is set when the deferred copy is queued:
  // a copy that was dropped (its flush failed) leaves it false, and the waiter reports MQ_EIO.
  // Runs on the snapshot of the last prepare().
  void match_spans(const uint8_t* d_tb, const uint64_t* d_to, uint32_t n, hipStream_t s,
                   HostSpans* host, mq_span_result* out, hipEvent_t ready = nullptr,
                   std::atomic<bool>* issued = nullptr);
  // Issue the pipelined host batch's copy that is still pending (match_spans with `ready` defers
  // it until the next batch's inputs are staged, or its result is waited for). Under the handle
  // lock.
  void flush_host_copy();
  // Forget the pending copy armed with this flag (its result was never published: the host arrays
  // it would fill are gone).
  void drop_pending_copy(const std::atomic<bool>* issued) {
    if (pc_.on && pc_.issued == issued) pc_.on = false;
  }
  // The same in two phases, for a sharded index: begin walks the batch and
  // exports the topics' gathered cross-shard nodes (device pointers in *x, valid until end);
  // the caller exchanges the lists between the shards; end merges with the other shards' lists.
  // shard_sync (mq_match_spans_begin): a sharded index's begin synchronises once, at its end
  // (MQ_OPT_ONE_SYNC); its spans_end is host-sized either way.
  // one_sync (match_spans only): the batch may run with one host synchronisation (at its end),
  // its buffers sized by earlier batches; spans_end then returns false when they did not hold it
  // and the caller runs the batch again without one_sync (host-sized buffers).
  void spans_begin(const uint8_t* d_tb, const uint64_t* d_to, uint32_t n, hipStream_t s, mq_xlist* x,
                   bool one_sync = false, bool shard_sync = false);
  bool spans_end(const mq_xlist* xf, uint32_t nf, hipStream_t s, HostSpans* host, mq_span_result* out,
                 hipEvent_t ready = nullptr, std::atomic<bool>* issued = nullptr);
  // Messages for n filters resident on the device (topics.go:525): handle sets per filter.
  // runs (mq_messages_runs_*): the runs instead of the handles (out then unused), into *runs
  // (device pointers) and, with hruns, copied to the host
  void messages(Index& ix, const uint8_t* d_fb, const uint64_t* d_fo, uint32_t n, hipStream_t s,
                HostMsg* host, mq_msg_result* out, mq_msg_runs_result* runs = nullptr,
                HostMsgRuns* hruns = nullptr);
  // auth.MatchTopic over (filter, topic) pairs of two host string tables (k_acl).
  void acl(const uint8_t* fb, const uint64_t* fo, uint32_t nf, const uint8_t* tb, const uint64_t* to,
           uint32_t nt, const uint32_t* pf, const uint32_t* pt, uint64_t n_pairs, HostAcl* out);
  // Copy host topics to the device input buffers and return their device pointers.
  void stage_inputs(const uint8_t* tb, const uint64_t* to, uint32_t n, hipStream_t s,
                    const uint8_t** d_tb, const uint64_t** d_to);

  // SelectShared on the device (k_pick) for a chunk of device results: picked rows to d_sel at
  // each topic's shared_base, picked counts to d_n (mq_select_shared_device).
  void select_shared(const mq_match_result& r, hipStream_t s, ShrRec* d_sel, uint32_t* d_n);
  // MQ_CFG_SELECT_SHARED: match results carry only the picked member of each shared filter.
  void set_select_shared(bool on) { select_shared_ = on; }
  bool select_shared() const { return select_shared_; }
  // mq_set_option (MQ_OPT_*); false for an unknown option.
  bool set_option(uint32_t opt, uint64_t value);

  uint32_t last_chunks() const { return last_chunks_; }
  uint64_t device_bytes() const;
  uint64_t upload_bytes() const { return uploaded_; }
  uint64_t syncs() const { return syncs_; }
  Profiler prof;

 private:
  DevIndex dev_index(const Index& ix) const;
  void sync_ix(Index& ix, hipStream_t s);  // sync() on the host: the upload is left to issue_staged
  void issue_staged(hipStream_t s);         // the staged dirty pages' H2D copy and k_scatter on s
  void wait_staged();                       // the last staged upload has read the pinned buffer
  uint64_t staged_bytes_ = 0;               // a staged upload not yet issued (bytes, runs)
  uint32_t staged_runs_ = 0;
  bool staged_pending_ = false;             // an issued upload may still read the pinned buffer
  void check_err(hipStream_t s);
  // walk (count) + scan of n topics; returns the batch totals (synchronises s)
  // (one_sync: the totals are not read back - the returned TopicOff is zero - and every topic's
  // gather count is clamped to its slot; the totals are read at the batch's end)
  TopicOff walk_scan(const DevIndex& di, const uint8_t* d_tb, const uint64_t* d_to, uint32_t n, hipStream_t s,
                     const uint32_t** gathers, uint32_t* gstride, bool lists, bool one_sync = false,
                     const DescArgs* fused = nullptr);
  // Messages: the level-order retained image (rebuilt when ix.retained_version() moved) and the
  // two query paths — run arithmetic over the image (k_msgq) and the particle walk (k_msg:
  // the Q6 state, nesting beyond kMsgStack, MQ_OPT_MSG_IMAGE = 0)
  void ensure_img(const Index& ix, const DevIndex& di, hipStream_t s);
  MsgImg msg_img() const;
  bool messages_img(const DevIndex& di, const uint8_t* d_fb, const uint64_t* d_fo, uint32_t n, hipStream_t s,
                    TopicOff* tot, bool run_out = false);
  void messages_walk(Index& ix, const DevIndex& di, const uint8_t* d_fb, const uint64_t* d_fo, uint32_t n,
                     hipStream_t s, TopicOff* tot);

  int dev_;
  uint64_t synced_version_ = ~0ull;
  IndexSnap snap_;
  bool sync_direct_ = false;  // the last sync uploaded from the host image directly (pageable)
  uint64_t uploaded_ = 0, syncs_ = 0;
  uint32_t last_chunks_ = 0;
  uint64_t chunk_rows_budget_;
  uint32_t chunk_tail_ = 0;  // > 1: last chunk ~ target / chunk_tail_ (MQ_CHUNK_TAIL)
  uint32_t chunk_min_ = 2;   // chunks a large batch is cut into at least (MQ_CHUNK_MIN)
  DevMirror<EdgeSlot> edges_;
  DevMirror<NodeWalk> walk_;
  DevMirror<NodeLists> lists_;
  DevMirror<NodeInl> inls_;
  DevMirror<NodeMsg> msg_;
  DevMirror<SegInfo> seginfo_;
  DevMirror<uint8_t> segbytes_;
  DevMirror<SubRec> subs_;
  DevMirror<MergeRef> mref_;
  DevMirror<MergePart> mpart_;
  DevMirror<NodePair> npair_;
  DevMirror<PairEnt> pent_;
  DevMirror<PairSlot> plist_;
  DevMirror<ShrRec> shr_;
  DevMirror<InlRec> inl_;
  DevMirror<ChildRec> children_;
  DevMirror<XInfo> xinfo_;
  DevMirror<DeepTail> deep_;
  DevMirror<uint32_t> deep_codes_;
  DevBuf in_bytes_, in_offs_;
  DevBuf counts_, offs_, bsum_, bpre_, gathers_;
  // Output chunks alternate between two buffer sets so that k_merge of chunk i (side stream)
  // overlaps k_desc/k_copy of chunk i + 1 (launch stream).
  DevBuf rows_[2], shr_rows_[2], inl_rows_[2], res_[2];
  DevBuf sel_rows_[2];          // k_pick output (MQ_CFG_SELECT_SHARED)
  bool select_shared_ = false;
  // per sub-batch parity: gather records and k_copy tile table
  DevBuf desc_[2], tiles_[2];
  // chunk plans + block -> chunk maps of every sub-batch ([nb_all] plans, then [nb_all] u32)
  DevBuf plan_;
  void* h_plan_ = nullptr;  // their pinned staging
  size_t h_plan_bytes_ = 0;
  void* h_pin_ = nullptr;  // pinned: block offsets + overflow flags of every sub-batch
  size_t h_pin_bytes_ = 0;
  DevBuf ovf_;             // per sub-batch gather-slot overflow flags
  DevBuf fb_list_, fb_cnt_;  // frontier walk: topics it handed to k_walk, and their number
  hipStream_t wstream_ = nullptr;  // walk + scan of the sub-batches
  hipEvent_t ev_in_ = nullptr, sb_done_[2] = {nullptr, nullptr};
  std::vector<hipEvent_t> ev_scan_;
  uint32_t subbatch_topics_ = kSubBatchTopics;
  void ensure_streams();
  void pinned(size_t bytes);
  DevBuf err_;
  Stager stager_;
  DevBuf d_stage_;                 // the staging buffer on the device
  void* h_stage_ = nullptr;        // ... and its pinned host side
  size_t h_stage_bytes_ = 0;
  DevBuf d_stage_spare_;           // larger staging buffers made ahead (prealloc)
  void* h_stage_spare_ = nullptr;
  size_t h_stage_spare_bytes_ = 0;
  template <class F>
  void each_mirror(const Index& ix, F f) const;  // f(k, DevMirror&, const Mirror&) for the synced arrays
  hipEvent_t stage_done_ = nullptr;  // the last scatter finished reading both
  hipStream_t side_ = nullptr;
  hipStream_t hstream_ = nullptr;  // host_stream()
  hipEvent_t copy_done_[2] = {nullptr, nullptr}, merge_done_[2] = {nullptr, nullptr}, side_done_ = nullptr;
  DevBuf msg_handles_, msg_base_, msg_count_, gslots_;
  // span format outputs
  DevBuf sp_res_, sp_spans_, sp_inl_, sp_picked_, sp_patches_, sp_pcount_;
  DevBuf sp_roff_, set_nbase_, set_total_, mr_total_;  // host results: packing offsets and totals
  // Host results, double-buffered: a batch's arrays are packed into a stage that the copy stream
  // then reads, while the next batch's kernels fill the other stage (copied: the copy that last
  // read it; the next use of the stage waits for it on the device).
  struct HostStage {
    DevBuf topics, spans, patches, set_patches, merge_rows, merge_base, inl, picked, span_total;
    hipEvent_t packed = nullptr, copied = nullptr;
    bool used = false;
  };
  HostStage hst_[2];
  uint32_t hpar_ = 0;              // the stage of the next host batch
  // A pipelined host batch's copy, not yet issued (flush_host_copy): it is queued behind the next
  // batch's input upload, so that upload does not wait for the copy on the DMA engine.
  struct PendingCopy {
    bool on = false;
    HostStage* hs = nullptr;
    HostSpans* host = nullptr;
    uint32_t n = 0;
    uint64_t spans = 0, patches = 0, inl = 0, picked = 0, set = 0, mrows = 0;
    bool dedup = false, codes = false;
    hipEvent_t ready = nullptr;
    std::atomic<bool>* issued = nullptr;  // the ticket's flag: set once the copy is queued
  };
  PendingCopy pc_;
  void issue_host_copy(const PendingCopy& c);
  bool patch_codes_ = true;        // MQ_OPT_PATCH_CODES
  hipStream_t hcopy_ = nullptr;    // the copy stream of host results
  void ensure_hcopy();
  DevBuf sp_work_;                   // MQ_PROF_WORK counters (kPatchRegions x kWork)
  // sharded: the exported list (offsets, entries, counts) and the imported lists' offsets
  DevBuf x_off_, x_ents_, x_cnt_, x_src_, x_foff_[kMaxShards - 1];
  DevBuf x_bsum_, x_bpre_;  // the import's batched scan (block sums, prefixes: a row per shard)
  DevBuf x_zero_;           // zero counts for an export that came without them
  DevBuf x_stride_, xbsum_, xbpre_, x_tot_;  // sharded one-sync begins: k_desc's export, its scan, total
  DevBuf x_off32_, x_gt_;  // walk-fused sharded begins: the export's u32 offsets; its totals (.g
                           //   entries, .rows gathers) for k_readback
  XSrc* h_xsrc_ = nullptr;                   // pinned: the imported lists' sources (no stack copy)
  hipEvent_t xsrc_done_ = nullptr;           // ... its last copy to the device is done
  struct SpanBatch {               // between spans_begin and spans_end
    bool pending = false;
    uint32_t n = 0;
    uint64_t version = 0;
    TopicOff tot{0, 0, 0, 0, 0};
    DevIndex di{};
    bool lists = true;             // the walk counted the lists (else k_desc did, into sp_tc_)
    bool dedup = false;            // merge-set dedup ran (dd_rep_ holds the representatives)
    uint64_t n_sets = 0;           // their number, when read back (profiling, MQ_OPT_SET_GRID)
    const uint32_t* gathers = nullptr;
    uint32_t gstride = 0;
    TopicCount* tc = nullptr;      // k_desc's per-topic counts (walk without lists), or null
    bool one_sync = false;         // one host synchronisation (spans_begin)
    bool xsync = false;            // a sharded index's one-sync begin: its end synchronises once too
                                   //   (and runs again, host-sized, if a pool overflowed)
    bool fused = false;            // k_desc ran in the walk's epilogue: spans at t * kGatherCap
    bool walk_inserted = false;    //   and k_dedup_insert with it (not on a sharded index)
    int trial = -1;                // a timed walk trial: 0 frontier, 1 thread per topic
  } sb_;
  // one-sync batches: values read back at the batch's end (pinned): the walk's totals, its
  // overflow and fallback counts, the *unsafe bits, the error word and the merge-set counts
  using FastBack = FastBackRec;     // (kernels.h: k_readback writes it)
  FastBack* h_fast_ = nullptr;
  FastBack* d_fast_ = nullptr;      // its device view
  DevBuf unsafe_;
  bool one_sync_ = true;      // MQ_OPT_ONE_SYNC
 public:
  double trace_sync_ms = 0.0;  // (MQ_TRACE_SUBMIT) the last one-sync batch's wait at its synchronisation
  int trace_runs = 0;          //   and how many runs the last match took
 private:
  bool fuse_desc_ = true;     // MQ_OPT_FUSE_DESC
  uint64_t msg_edge_budget_ = 8ull << 30;  // MQ_OPT_MSG_EDGE_BUDGET: the image edge table's 1/16 budget
  uint32_t fail_next_ = 0;    // MQ_OPT_FAIL_NEXT: span batches still to fail as if a guard tripped
  uint32_t walk_exp_ = 0;     // MQ_OPT_WALK_EXP (development builds)
  DevBuf root_hint_;
  uint32_t set_exp_ = 0;      // MQ_OPT_SET_EXP (timing experiments only)
  uint64_t last_sets_ = 0;    // merge sets of the last batch: the grid of the next set pass
  DevBuf sp_tc_;                     // per-topic counts from k_desc<true> (walk without lists)
  uint64_t rcap_ = 0;                // patches per region of sp_patches_ (kPatchRegions regions)
  uint64_t patch_cap_init_ = 1ull << 24;
  DevBuf img_node_, img_pos_, img_cl_, img_lp_, img_h_, img_cnt_, img_coff_, img_bsum_, img_bpre_;
  DevBuf img_edges_;                  // the image's edge table (MsgImg.edges)
  DevBuf kx_par_, kx_chd_, kx_k0_, kx_k1_, kx_tab_;  // the image's key index (MsgImg.kx_*)
  uint64_t kx_mask_ = 0;
  bool kx_built_ = false;
  bool msg_kx_on_ = true;             // MQ_OPT_MSG_KEYIDX
  uint32_t msg_kx_min_ = kKxMinRounds;  // ... its probe rounds below which a level does not try it
  void build_key_index(const DevIndex& di, uint32_t n_img, uint32_t n_pos, hipStream_t s);
  DevBuf msg_gate_;                   // one-sync Messages batches: the gate and the piece count (k_msg_gate)
  uint64_t img_edge_mask_ = 0;
  bool msg_edges_on_ = true;          // MQ_OPT_MSG_EDGES
  DevBuf msg_pieces_;               // k_msgq copy pieces of a batch
  DevBuf msg_runs_, msg_nruns_;     // k_msgq runs recorded by the count pass (kMsgRuns)
  DevBuf msg_rbase_, msg_rcnt_;     // runs at the boundary: each filter's first run, run count
  std::shared_ptr<PinnedVec<uint64_t>> host_img_;  // host copy of img_h_ (runs host results)
  uint64_t host_img_version_ = ~0ull;
  uint64_t img_version_ = ~0ull;    // ix.retained_version() the image was built at
  uint32_t img_n_ = 0, img_n_pos_ = 0, img_levels_ = 0;
  uint64_t img_live_ = 0;
  bool msg_img_on_ = true;          // MQ_OPT_MSG_IMAGE
  DevBuf msg_spec_;              // speculative-count scratch: spec_cap handles per filter
  uint64_t msg_spec_bytes_ = 0;  // its budget (MQ_MSG_SPEC_MB)
  uint32_t msg_wpe_opt_ = 0;     // k_msg variant (MQ_OPT_MSG_WAVES; 0: by index size)
  uint32_t merge_wpe_opt_ = 0;   // k_merge variant (MQ_OPT_MERGE_WAVES; 0: by index size)
  uint32_t walk_wpe_ = 8;        // k_walk count pass register budget (MQ_OPT_WALK_WAVES)
  bool walk_lists_ = false;      // span format: the walk counts the lists (MQ_OPT_WALK_LISTS)
  uint32_t walk_group_ = 16;     // frontier walk lanes per topic (MQ_OPT_WALK_GROUP; 0: k_walk)
  // one-sync batches choose the walk by trial (spans_begin) unless MQ_OPT_WALK_GROUP fixed it
  bool walk_auto_ = true;
  static constexpr uint32_t kWalkTrialMin = 65536;  // batches this large are timed for the trial
  uint64_t walk_trial_nodes_ = 0;                    // the index size the trials ran at
  double walk_trial_wild_ = 0.0;                     //   and its share of '+' / '#' particles
  // The trial schedule (walk per trial batch: 0 frontier, 1 thread per topic): one untimed batch of
  // each walk (caches, first-touch allocations), then two timed batches of each in ABBA order; the
  // faster mean per topic is kept. walk_trial_step_ counts the completed trial batches.
  static constexpr uint32_t kWalkTrialSeq[6] = {0, 1, 1, 0, 0, 1};
  static constexpr uint32_t kWalkTrialWarm = 2;
  uint32_t walk_trial_step_ = 0;
  double walk_trial_ns_[2] = {0.0, 0.0};             // timed batch time per topic, summed: frontier, thread
  hipEvent_t walk_ev_[2] = {nullptr, nullptr};
  uint32_t dedup_ = 1;           // span format: merge-set dedup (MQ_OPT_MERGE_DEDUP)
  uint32_t set_grid_ = 1;        // MQ_OPT_SET_GRID (10M: set pass 1.18 -> 1.05 ms against persistent waves)
  DevBuf dd_sig_, dd_cnt_, dd_list_, dd_mrow_, dd_keys_, dd_vals_, dd_slot_, dd_rep_, dd_nsets_, dd_rlist_;
  DevBuf dd_sets_, dd_spatches_, dd_spcount_;  // phase 1 of the dedup merge: SetInfo, set pool
  DevBuf dd_wlist_, dd_nwave_;                 // k_finish: topics left for k_merge's topic pass
  DevBuf dd_mpair_;                            // k_desc: merge gathers' pair-block headers
  DevBuf dd_mrank_;                            // ... and rank keys (sharded index)
  DevBuf dd_fcnt_;                             // k_xsig: cross-shard entries per topic
  DevBuf msg_wq_;                              // Messages: exported work items of wide filters (+ count)
  DevBuf msg_wscratch_;                        // ... the runs their count recorded (per wavefront)
  uint32_t msg_export_ = 1;                    // MQ_OPT_MSG_EXPORT (0 off, 1 kMsgExportMin, else the threshold)
  DevBuf msg_cyc_;                             // MQ_PROF_WORK: Messages count-pass clocks per filter
  DevBuf set_rec_;                             // MQ_PROF_WORK: records resolved per merge set
  uint64_t srcap_ = 0;                         // set patches per region of dd_spatches_
  uint32_t copy_blocks_ = 0, merge_blocks_ = 0;  // persistent k_copy / k_merge grids (workgroups)
  uint32_t n_cus_ = 1;
  bool serial_ = false;       // MQ_OPT_SERIAL: k_merge on the launch stream (isolated kernel times)
  DevBuf acl_buf_;  // k_acl inputs and outputs
  std::vector<TopicOff> h_bpre_;
  uint64_t retained_len_ = 0;
  uint64_t empty_handle_ = 0;
  bool empty_live_ = false;
};

}  // namespace mq
