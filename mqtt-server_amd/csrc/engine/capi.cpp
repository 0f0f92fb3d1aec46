// extern "C" surface of the engine (include/mqmatch.h). Each entry point serialises on the
// handle's mutex — the analogue of the reference's root.Lock() (topics.go:402) — and turns C++
// and HIP failures into negative errno codes with a thread-local message.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <cstring>
#include <new>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "device.h"
#include "index.h"
#include "mqmatch.h"
#include "mqmatch_dev.h"
#include <cstdlib>
#include <cstdio>
#include <chrono>
#include "fifo_mutex.h"

using namespace mq;

// The handle's locks (the reference's root lock, topics.go:402). `mu` guards the host image: updates
// take it, and a match takes it only while it syncs the device image and snapshots what its
// batch reads (Device::prepare) — the match's GPU work then runs without it, so an update never
// waits for a running match (round 6; before, every update queued behind the match in flight,
// which a stalled match made ~15 ms). `dev_mu` serialises the work on the handle's device
// (matches, Messages, syncs, checks) and is always taken before `mu`; updates never take it. `mu`
// prefers updates, as Go's sync.RWMutex prefers writers: an update announces itself
// (`views.writers`) before it takes `mu`, and a call that is not an update waits while one is
// announced. Host span results point into the host image's subscription pools until
// mq_result_free; `views` records them by generation — a match reserves its generation while it
// holds `mu`, before its kernels run — and the index copies a slab before it changes one that a
// live result may see and keeps what it frees until no live result can see it
// (Index::begin_op), so an update never waits for results either. `views` has its own mutex,
// never held across GPU work, so freeing a result never waits for a match in flight. Results
// hold a reference, so freeing one after mq_index_destroy is safe.
struct IndexLock {
  FifoMutex dev_mu;  // the device's work (taken before mu)
  FifoMutex mu;      // the host image (in arrival order: fifo_mutex.h)
  ViewTracker views;
  Device* dev = nullptr;  // the index's device, while it lives (pipelined results flush through it)
};

struct mq_index {
  std::shared_ptr<IndexLock> lk = std::make_shared<IndexLock>();
  mq_config cfg;
  std::unique_ptr<Index> ix;
  std::unique_ptr<Device> dev;
  std::atomic<bool> dev_ready{false};  // dev exists (read without the lock: thread warm-up)
  int profile = 0;  // MQ_PROF_*

  std::vector<std::pair<uint32_t, uint64_t>> options;  // mq_set_option, in call order

  Device& device() {
    if (!dev) {
      dev.reset(new Device(cfg.device));
      lk->dev = dev.get();
      dev->prof.enable(profile != 0, (profile & MQ_PROF_WORK) != 0, (profile & MQ_PROF_WALK) != 0);
      dev->set_select_shared((cfg.flags & MQ_CFG_SELECT_SHARED) != 0);
      for (auto& o : options) dev->set_option(o.first, o.second);
      dev_ready.store(true, std::memory_order_release);
    }
    return *dev;
  }
};

namespace {

thread_local std::string g_err;

struct MatchHolder {
  mq_match_result pub;  // first member: the pointer handed out
  HostMatch data;
};
struct SpanHolder {
  mq_span_result pub;
  HostSpans data;
  std::shared_ptr<IndexLock> lk;  // the index's lock (views)
  uint64_t gen = 0;                // this result's generation (ViewTracker)
};
struct MsgHolder {
  mq_msg_result pub;
  PinnedVec<uint64_t> base;
  PinnedVec<uint32_t> count;
  PinnedVec<uint64_t> handles;
};
struct MsgRunsHolder {
  mq_msg_runs_result pub;
  HostMsgRuns data;
};
struct AclHolder {
  mq_acl_result pub;
  HostAcl data;
};
std::mutex g_res_mu;
std::unordered_map<void*, int> g_results;  // 1 = match, 2 = messages, 3 = acl, 4 = spans, 5 = message runs

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// What a guarded call does to the host image (IndexLock).
// kUpdate: takes only `mu`; copy-on-write against the live results, never waits for them (a bulk
// subscribe too: it takes the per-entry path while a result is live). kRead: the device's work
// and the host image, for the whole call. Matches: guarded_match.
enum class Access { kRead, kUpdate };

// The calling thread's HIP runtime state for device dev, set up once per thread: a thread's first
// HIP calls cost ~10 ms, which a match must not pay while it holds the handle
// lock that updates wait for. (The Go batching stage also keeps its loop on one OS thread.) A
// thread that serves indexes on several devices keeps one bit per device; the warm-up's event is
// recorded on a non-blocking stream of the thread's own, not on the null stream (which would
// wait behind every blocking stream of the device).
void thread_warm(int dev) {
  static thread_local uint64_t warmed[4] = {0, 0, 0, 0};
  if (dev < 0 || dev >= 256) return;
  if (warmed[dev / 64] >> (dev % 64) & 1) return;
  if (hipSetDevice(dev) != hipSuccess) {
    (void)hipGetLastError();
    return;
  }
  hipStream_t st = nullptr;
  hipEvent_t e = nullptr;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess &&
      hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess) {
    (void)hipEventRecord(e, st);
    (void)hipEventSynchronize(e);
  }
  if (e) (void)hipEventDestroy(e);
  if (st) (void)hipStreamDestroy(st);
  (void)hipGetLastError();
  warmed[dev / 64] |= 1ull << (dev % 64);
}

// C++ and HIP failures as negative errno codes with the thread's message.
template <class F>
int caught(F&& f) {
  try {
    return f();
  } catch (const HipError& e) {
    return fail(e.code == hipErrorNoDevice || e.code == hipErrorInvalidDevice ? MQ_ENODEV : MQ_EIO, e.where);
  } catch (const std::bad_alloc&) {
    return fail(MQ_ENOMEM, "out of host memory");
  } catch (const std::exception& e) {
    return fail(MQ_EIO, e.what());
  }
}

// A call that is not an update waits while one is announced (updates are preferred).
void wait_for_writers(ViewTracker& V) {
  std::unique_lock<std::mutex> g(V.mu);
  V.cv.wait(g, [&] { return V.writers == 0; });
}

// Runs f under the handle's lock (IndexLock).
template <class F>
int guarded(mq_index* idx, F&& f, Access access = Access::kRead) {
  if (!idx) return fail(MQ_EINVAL, "null index");
  if (access != Access::kUpdate && idx->dev_ready.load(std::memory_order_acquire)) thread_warm(idx->cfg.device);
  IndexLock& L = *idx->lk;
  ViewTracker& V = L.views;
  struct Announce {  // an update's announcement, withdrawn however the call ends
    ViewTracker* V = nullptr;
    ~Announce() {
      if (!V) return;
      {
        std::lock_guard<std::mutex> g(V->mu);
        V->writers--;
      }
      V->cv.notify_all();
    }
  } ann;
  return caught([&] {
    std::unique_lock<FifoMutex> dlk(L.dev_mu, std::defer_lock);
    if (access == Access::kUpdate) {
      {
        std::lock_guard<std::mutex> g(V.mu);
        V.writers++;
      }
      ann.V = &V;
    } else {
      dlk.lock();
      wait_for_writers(V);
    }
    if (slow_on()) slow_begin();  // (the wait for the lock included)
    std::lock_guard<FifoMutex> lk(L.mu);
    if (!slow_on()) return f();
    slow_mark("locked");
    const int r = f();
    slow_report(access == Access::kUpdate ? "update" : "read", 0.0);
    return r;
  });
}

// A match in two phases (IndexLock): prep() under both locks — it syncs the device image and
// takes the batch's snapshot (Device::prepare), and for host results reserves their generation —
// then run() with the device's lock only, while updates change the host image. What the sync
// will allocate (arrays that grew, staging for the dirty pages) is allocated first, without `mu`
// (Device::sync_plan / prealloc). A match holds `mu` only for the sync itself, so it does not wait
// for announced updates (FifoMutex order is fair): with updates arriving back to back, waiting
// for none to be announced starved the readers (172 matches during 3,200 updates).
template <class P, class R>
int guarded_match(mq_index* idx, P&& prep, R&& run) {
  if (!idx) return fail(MQ_EINVAL, "null index");
  if (idx->dev_ready.load(std::memory_order_acquire)) thread_warm(idx->cfg.device);
  IndexLock& L = *idx->lk;
  return caught([&] {
    std::lock_guard<FifoMutex> dlk(L.dev_mu);
    if (slow_on()) slow_begin();
    idx->device().begin_prepare();  // (HIP calls before the host-image lock, none under it)
    slow_mark("begun");
    for (int round = 0;; round++) {
      Device::SyncPlan plan;
      {
        std::lock_guard<FifoMutex> lk(L.mu);
        plan = idx->device().sync_plan(*idx->ix);
        if (!plan.any || round == 2) {  // (still short after two rounds of updates: allocate under mu)
          prep();
          if (slow_on()) slow_report("match-prepare", 0.0);
          break;
        }
      }
      slow_mark("prealloc");
      idx->dev->prealloc(plan);
      slow_mark("preallocated");
    }
    slow_mark("unlocked");
    const int r = run();
    if (slow_on()) slow_report("match", 0.0);
    return r;
  });
}

// The host pools a host span result names, with its generation (reserved under `mu`, by the
// match's prepare phase). A result that is not published gives its generation back.
struct PoolView {
  const mq_client_row* sub = nullptr;
  const mq_shared_row* shr = nullptr;
  uint64_t sub_len = 0, shr_len = 0;
  ViewTracker* views = nullptr;
  uint64_t gen = 0;
  bool published = false;
  void reserve(mq_index* idx) {  // under mu
    sub = reinterpret_cast<const mq_client_row*>(idx->ix->subs.m.h.data());
    shr = reinterpret_cast<const mq_shared_row*>(idx->ix->shr.m.h.data());
    sub_len = idx->ix->subs.m.size();
    shr_len = idx->ix->shr.m.size();
    views = &idx->lk->views;
    gen = views->publish();
  }
  ~PoolView() {
    if (views && !published) views->release(gen);
  }
};

bool bad_str(const void* p, uint32_t len) { return p == nullptr && len != 0; }

}  // namespace

extern "C" {

uint32_t mq_abi_version(void) { return MQ_ABI_VERSION; }

int mq_thread_warm(mq_index* idx) {
  if (!idx) return fail(MQ_EINVAL, "null index");
  thread_warm(idx->cfg.device);
  return 0;
}
const char* mq_last_error(void) { return g_err.c_str(); }

int mq_index_create(const mq_config* cfg, mq_index** out) {
  if (!out) return fail(MQ_EINVAL, "null out");
  try {
    mq_index* idx = new mq_index();
    idx->cfg = cfg ? *cfg : mq_config{0, 0, 0, 0, 0, 0};
    if (idx->cfg.shard_count > kMaxShards || (idx->cfg.shard_count > 1 && idx->cfg.shard_index >= idx->cfg.shard_count)) {
      delete idx;
      return fail(MQ_EINVAL, "bad shard_index / shard_count");
    }
    idx->ix.reset(new Index(idx->cfg.expected_subs, idx->cfg.expected_nodes));
    idx->ix->set_views(&idx->lk->views);
    {  // the edge table's HBM budget at its sparse loads: an eighth of the device's memory
      int nd = 0;
      size_t freeb = 0, total = 0;
      if (hipGetDeviceCount(&nd) == hipSuccess && idx->cfg.device >= 0 && idx->cfg.device < nd) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        if (hipSetDevice(idx->cfg.device) == hipSuccess && hipMemGetInfo(&freeb, &total) == hipSuccess)
          idx->ix->set_edge_budget(total / 8);
        (void)hipSetDevice(cur);
      }
      (void)hipGetLastError();
    }
    if (idx->cfg.shard_count > 1) idx->ix->set_shard(idx->cfg.shard_index, idx->cfg.shard_count);
    *out = idx;
    return 0;
  } catch (const std::bad_alloc&) {
    return fail(MQ_ENOMEM, "out of host memory");
  }
}

void mq_index_destroy(mq_index* idx) {
  if (!idx) return;
  {
    std::lock_guard<FifoMutex> dg(idx->lk->dev_mu);
    std::lock_guard<FifoMutex> g(idx->lk->mu);
    idx->lk->dev = nullptr;  // (tickets still held flush through it no more; ~Device issues their copies)
  }
  delete idx;
}

int mq_subscribe(mq_index* idx, const char* filter, uint32_t flen, uint32_t client_id,
                 uint32_t filter_id, uint8_t qos, uint8_t flags, int32_t identifier) {
  if (bad_str(filter, flen)) return fail(MQ_EINVAL, "null filter");
  if (qos > 2) return fail(MQ_EINVAL, "qos > 2");
  return guarded(idx, [&] {
    return idx->ix->subscribe(std::string_view(filter, flen), client_id, filter_id, qos, flags, identifier);
  }, Access::kUpdate);
}

int mq_unsubscribe(mq_index* idx, const char* filter, uint32_t flen, uint32_t client_id) {
  if (bad_str(filter, flen)) return fail(MQ_EINVAL, "null filter");
  return guarded(idx, [&] { return idx->ix->unsubscribe(std::string_view(filter, flen), client_id); }, Access::kUpdate);
}

int mq_inline_subscribe(mq_index* idx, const char* filter, uint32_t flen, int32_t identifier,
                        uint32_t filter_id) {
  if (bad_str(filter, flen)) return fail(MQ_EINVAL, "null filter");
  return guarded(idx, [&] {
    return idx->ix->inline_subscribe(std::string_view(filter, flen), identifier, filter_id);
  }, Access::kUpdate);
}

int mq_inline_unsubscribe(mq_index* idx, const char* filter, uint32_t flen, int32_t identifier) {
  if (bad_str(filter, flen)) return fail(MQ_EINVAL, "null filter");
  return guarded(idx, [&] { return idx->ix->inline_unsubscribe(std::string_view(filter, flen), identifier); }, Access::kUpdate);
}

int mq_retain_message(mq_index* idx, const char* topic, uint32_t tlen, uint64_t handle,
                      uint32_t payload_len, uint8_t retain, int64_t* out) {
  if (bad_str(topic, tlen)) return fail(MQ_EINVAL, "null topic");
  return guarded(idx, [&] {
    int64_t r = idx->ix->retain_message(std::string_view(topic, tlen), handle, payload_len, retain != 0);
    if (out) *out = r;
    return 0;
  }, Access::kUpdate);
}

int mq_retained_delete(mq_index* idx, const char* topic, uint32_t tlen) {
  if (bad_str(topic, tlen)) return fail(MQ_EINVAL, "null topic");
  return guarded(idx, [&] { return idx->ix->retained_delete(std::string_view(topic, tlen)); }, Access::kUpdate);
}

int mq_retained_set(mq_index* idx, const char* topic, uint32_t tlen, uint64_t handle, uint32_t payload_len,
                    uint8_t retain) {
  if (bad_str(topic, tlen)) return fail(MQ_EINVAL, "null topic");
  return guarded(idx, [&] {
    return idx->ix->retained_set(std::string_view(topic, tlen), handle, payload_len, retain != 0);
  }, Access::kUpdate);
}

uint64_t mq_retained_len(const mq_index* idx) {
  if (!idx) return 0;
  std::lock_guard<FifoMutex> lk(idx->lk->mu);
  return idx->ix->retained_len();
}

int mq_subscribe_bulk(mq_index* idx, const uint8_t* bytes, const uint64_t* offs, const uint32_t* client_ids,
                      const uint32_t* filter_ids, const uint8_t* qos, const uint8_t* flags,
                      const int32_t* identifiers, uint64_t n, uint8_t* out_new) {
  if (n && (!bytes || !offs || !client_ids || !filter_ids || !qos || !flags || !identifiers))
    return fail(MQ_EINVAL, "null column");
  for (uint64_t i = 0; i < n; i++)
    if (qos[i] > 2) return fail(MQ_EINVAL, "qos > 2");
  return guarded(idx, [&] {
    idx->ix->subscribe_bulk(bytes, offs, client_ids, filter_ids, qos, flags, identifiers, n, out_new);
    return 0;
  }, Access::kUpdate);
}

int mq_unsubscribe_bulk(mq_index* idx, const uint8_t* bytes, const uint64_t* offs, const uint32_t* client_ids,
                        uint64_t n, uint8_t* out_existed) {
  if (n && (!bytes || !offs || !client_ids)) return fail(MQ_EINVAL, "null column");
  return guarded(idx, [&] {
    for (uint64_t i = 0; i < n; i++) {
      const int r = idx->ix->unsubscribe(std::string_view((const char*)bytes + offs[i], offs[i + 1] - offs[i]),
                                         client_ids[i]);
      if (out_existed) out_existed[i] = (uint8_t)r;
    }
    return 0;
  }, Access::kUpdate);
}

int mq_retain_bulk(mq_index* idx, const uint8_t* bytes, const uint64_t* offs, const uint64_t* handles,
                   uint64_t n) {
  if (n && (!bytes || !offs || !handles)) return fail(MQ_EINVAL, "null column");
  return guarded(idx, [&] {
    idx->ix->retain_bulk(bytes, offs, handles, n);
    return 0;
  }, Access::kUpdate);
}

int mq_match_batch(mq_index* idx, const uint8_t* tb, const uint64_t* to, uint32_t n, mq_match_result** out) {
  if (!out || (n && (!to || (!tb && to[n] != 0)))) return fail(MQ_EINVAL, "null argument");
  return guarded(idx, [&] {
    Device& d = idx->device();
    std::unique_ptr<MatchHolder> h(new MatchHolder());
    const uint8_t* dtb = nullptr;
    const uint64_t* dto = nullptr;
    mq_match_result dev_out;
    if (n) d.stage_inputs(tb, to, n, nullptr, &dtb, &dto);
    d.match(*idx->ix, dtb, dto, n, nullptr, &h->data, &dev_out);
    hip_check(hipStreamSynchronize(nullptr), "hipStreamSynchronize");
    mq_match_result& r = h->pub;
    r = mq_match_result{};
    r.n_topics = n;
    r.topics = h->data.topics.data();
    r.sub_rows = reinterpret_cast<const mq_client_row*>(h->data.rows.data());
    r.shared_rows = reinterpret_cast<const mq_shared_row*>(h->data.shr.data());
    r.inline_rows = reinterpret_cast<const mq_inline_row*>(h->data.inl.data());
    r.n_sub_rows = h->data.rows.size();
    r.n_shared_rows = h->data.shr.size();
    r.n_inline_rows = h->data.inl.size();
    *out = &h->pub;
    std::lock_guard<std::mutex> lk(g_res_mu);
    g_results[&h->pub] = 1;
    h.release();
    return 0;
  });
}

namespace {
// A host span result: the device arrays copied into h->data, the pools pointing at the host
// image as the match's prepare phase saw it (copy-on-write keeps what the result sees until
// mq_result_free).
int publish_host_spans(std::shared_ptr<IndexLock> lk, std::unique_ptr<SpanHolder> h, const mq_span_result& dev_out,
                       PoolView& pv, mq_span_result** out) {
  mq_span_result& r = h->pub;
  r = dev_out;  // counts and flags; pointers replaced by the host copies and host pools
  r.topics = reinterpret_cast<const mq_topic_spans*>(h->data.topics.data());
  r.spans = reinterpret_cast<const mq_span*>(h->data.spans.data());
  r.patches = reinterpret_cast<const mq_patch*>(h->data.patches.data());
  r.inline_rows = reinterpret_cast<const mq_inline_row*>(h->data.inl.data());
  r.picked_rows = reinterpret_cast<const mq_shared_row*>(h->data.picked.data());
  const bool codes = h->data.codes;  // 4-byte patch codes (MQ_SPANS_PATCH_CODES)
  if (codes) {
    r.flags |= MQ_SPANS_PATCH_CODES;
    r.patches = reinterpret_cast<const mq_patch*>(h->data.patch_codes.data());
  }
  r.n_patches = codes ? h->data.patch_codes.size() : h->data.patches.size();  // packed (the device pool has gaps)
  r.n_spans = h->data.spans.size();      // packed (a one-sync device batch leaves them at t * 64)
  r.n_inline_rows = h->data.inl.size();
  r.n_picked_rows = h->data.picked.size();
  const bool sets = !h->data.merge_base.empty();  // (topics with MQ_TOPIC_SET_PATCHES, ABI v7)
  r.set_patches = !sets ? nullptr
                  : codes ? reinterpret_cast<const mq_patch*>(h->data.set_codes.data())
                          : reinterpret_cast<const mq_patch*>(h->data.set_patches.data());
  r.n_set_patches = !sets ? 0 : codes ? h->data.set_codes.size() : h->data.set_patches.size();
  r.merge_rows = sets ? h->data.merge_rows.data() : nullptr;
  r.n_merge_rows = sets ? h->data.merge_rows.size() : 0;
  r.merge_row_base = sets ? h->data.merge_base.data() : nullptr;
  r.sub_pool = pv.sub;
  r.shared_pool = pv.shr;
  r.sub_pool_len = pv.sub_len;
  r.shared_pool_len = pv.shr_len;
  h->lk = std::move(lk);
  h->gen = pv.gen;
  pv.published = true;
  *out = &h->pub;
  std::lock_guard<std::mutex> g(g_res_mu);
  g_results[&h->pub] = 4;
  h.release();
  return 0;
}
}  // namespace

int mq_match_spans(mq_index* idx, const uint8_t* tb, const uint64_t* to, uint32_t n, mq_span_result** out) {
  if (!out || (n && (!to || (!tb && to[n] != 0)))) return fail(MQ_EINVAL, "null argument");
  Device* d = nullptr;
  hipStream_t hs = nullptr;
  PoolView pv;
  return guarded_match(idx, [&] {
    d = &idx->device();
    hs = d->host_stream_made();
    d->prepare(*idx->ix, hs);
    pv.reserve(idx);
  }, [&] {
    std::unique_ptr<SpanHolder> h(new SpanHolder());
    const uint8_t* dtb = nullptr;
    const uint64_t* dto = nullptr;
    if (n) d->stage_inputs(tb, to, n, hs, &dtb, &dto);
    mq_span_result dev_out;
    d->match_spans(dtb, dto, n, hs, &h->data, &dev_out);
    return publish_host_spans(idx->lk, std::move(h), dev_out, pv, out);
  });
}

// A submitted batch: its result, published (its arrays being filled by the copy stream), and the
// event recorded when the copy is done.
struct mq_spans_ticket {
  mq_span_result* res = nullptr;
  hipEvent_t ready = nullptr;
  std::shared_ptr<IndexLock> lk;  // the index's lock (its device issues the pending copy)
  std::atomic<bool> issued{false};  // the copy was queued (a dropped copy leaves it false)
};

int mq_match_spans_submit(mq_index* idx, const uint8_t* tb, const uint64_t* to, uint32_t n, mq_spans_ticket** out) {
  if (!out || (n && (!to || (!tb && to[n] != 0)))) return fail(MQ_EINVAL, "null argument");
  *out = nullptr;
  Device* d = nullptr;
  hipStream_t hs = nullptr;
  PoolView pv;
  return guarded_match(idx, [&] {
    d = &idx->device();
    hs = d->host_stream_made();
    d->prepare(*idx->ix, hs);
    pv.reserve(idx);
  }, [&] {
    std::unique_ptr<mq_spans_ticket> tk(new mq_spans_ticket());
    hip_check(hipEventCreateWithFlags(&tk->ready, hipEventDisableTiming), "hipEventCreate");
    struct EvGuard {  // the event goes if the submit fails
      mq_spans_ticket* t;
      ~EvGuard() {
        if (t && t->ready) (void)hipEventDestroy(t->ready);
      }
    } eg{tk.get()};
    std::unique_ptr<SpanHolder> h(new SpanHolder());
    const uint8_t* dtb = nullptr;
    const uint64_t* dto = nullptr;
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    if (n) d->stage_inputs(tb, to, n, hs, &dtb, &dto);  // (ahead of the last batch's copy: below)
    const auto t1 = clk::now();
    d->flush_host_copy();
    const auto t2 = clk::now();
    mq_span_result dev_out;
    struct Disarm {  // a result that is not published takes its armed copy with it
      Device* d;
      const std::atomic<bool>* f;
      ~Disarm() {
        if (d) d->drop_pending_copy(f);
      }
    } da{d, &tk->issued};
    d->match_spans(dtb, dto, n, hs, &h->data, &dev_out, tk->ready, &tk->issued);
    const auto t3 = clk::now();
    tk->lk = idx->lk;
    const int rc = publish_host_spans(idx->lk, std::move(h), dev_out, pv, &tk->res);
    static const bool trace = std::getenv("MQ_TRACE_SUBMIT") != nullptr;
    if (trace) {
      auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
      std::fprintf(stderr, "mq_match_spans_submit: upload %.3f flush %.3f match %.3f (runs %d, sync wait %.3f) publish %.3f ms\n",
                   ms(t0, t1), ms(t1, t2), ms(t2, t3), d->trace_runs, d->trace_sync_ms, ms(t3, clk::now()));
    }
    if (rc) return rc;
    da.d = nullptr;
    eg.t = nullptr;
    *out = tk.release();
    return 0;
  });
}

int mq_match_spans_wait(mq_spans_ticket* t, mq_span_result** out) {
  if (!t || !out) return fail(MQ_EINVAL, "null argument");
  *out = nullptr;
  if (t->lk) {  // the copy may still be pending (queued behind a next batch's upload)
    std::lock_guard<FifoMutex> g(t->lk->dev_mu);
    try {
      if (t->lk->dev) t->lk->dev->flush_host_copy();
    } catch (const HipError& he) {
      (void)hipEventDestroy(t->ready);
      mq_result_free(t->res);
      delete t;
      return fail(MQ_EIO, he.where);
    }
  }
  if (!t->issued.load()) {  // its copy was dropped: a later submit's flush of it failed
    (void)hipEventDestroy(t->ready);
    mq_result_free(t->res);
    delete t;
    return fail(MQ_EIO, "the result's copy into host memory was never issued (an earlier flush failed)");
  }
  const hipError_t e = hipEventSynchronize(t->ready);
  (void)hipEventDestroy(t->ready);
  mq_span_result* r = t->res;
  delete t;
  if (e != hipSuccess) {
    mq_result_free(r);
    return fail(MQ_EIO, std::string("hipEventSynchronize: ") + hipGetErrorString(e));
  }
  *out = r;
  return 0;
}

int mq_match_spans_end_host(mq_index* idx, const mq_xlist* foreign, uint32_t n_foreign, mq_span_result** out) {
  if (!out || (n_foreign && !foreign)) return fail(MQ_EINVAL, "null argument");
  return guarded(idx, [&] {
    Device& d = idx->device();
    if (d.batch_stale(*idx->ix)) throw HipError{hipErrorInvalidValue, "index updated between spans_begin and spans_end"};
    std::unique_ptr<SpanHolder> h(new SpanHolder());
    mq_span_result dev_out;
    d.spans_end(foreign, n_foreign, nullptr, &h->data, &dev_out);
    PoolView pv;
    pv.reserve(idx);
    return publish_host_spans(idx->lk, std::move(h), dev_out, pv, out);
  });
}

int mq_match_spans_device(mq_index* idx, const uint8_t* d_tb, const uint64_t* d_to, uint32_t n, void* stream,
                          mq_span_result* out) {
  if (!out || (n && !d_to)) return fail(MQ_EINVAL, "null argument");
  Device* d = nullptr;
  return guarded_match(idx, [&] {
    d = &idx->device();
    d->prepare(*idx->ix, (hipStream_t)stream);
  }, [&] {
    d->match_spans(d_tb, d_to, n, (hipStream_t)stream, nullptr, out);
    return 0;
  });
}

int mq_match_spans_begin(mq_index* idx, const uint8_t* d_tb, const uint64_t* d_to, uint32_t n, void* stream,
                         mq_xlist* exported) {
  if (!exported || (n && !d_to)) return fail(MQ_EINVAL, "null argument");
  return guarded(idx, [&] {
    Device& d = idx->device();
    d.prepare(*idx->ix, (hipStream_t)stream);
    d.spans_begin(d_tb, d_to, n, (hipStream_t)stream, exported, false, true);
    return 0;
  });
}

int mq_match_spans_end(mq_index* idx, const mq_xlist* foreign, uint32_t n_foreign, void* stream, mq_span_result* out) {
  if (!out || (n_foreign && !foreign)) return fail(MQ_EINVAL, "null argument");
  return guarded(idx, [&] {
    Device& d = idx->device();
    if (d.batch_stale(*idx->ix)) throw HipError{hipErrorInvalidValue, "index updated between spans_begin and spans_end"};
    d.spans_end(foreign, n_foreign, (hipStream_t)stream, nullptr, out);
    return 0;
  });
}

int mq_spans_expand(const mq_span_result* r, uint32_t first, uint32_t count, mq_client_row* rows,
                    uint64_t rows_cap, mq_shared_row* shared, uint64_t shared_cap, uint64_t* n_rows,
                    uint64_t* n_shared) {
  if (!r || (uint64_t)first + count > r->n_topics) return fail(MQ_EINVAL, "topic range out of bounds");
  {
    std::lock_guard<std::mutex> lk(g_res_mu);
    auto it = g_results.find((void*)r);
    if (it == g_results.end() || it->second != 4) return fail(MQ_EINVAL, "not a host span result (mq_match_spans)");
  }
  const bool picked = (r->flags & MQ_SPANS_PICKED) != 0;
  uint64_t nr = 0, ns = 0;
  for (uint32_t t = first; t < first + count; t++) {
    const mq_topic_spans& ts = r->topics[t];
    if (nr + ts.n_rows > rows_cap || ns + ts.n_shared > shared_cap) return fail(MQ_ERANGE, "output capacity");
    if ((ts.n_rows && !rows) || (ts.n_shared && !shared)) return fail(MQ_EINVAL, "null output");
    mq_client_row* out = rows + nr;
    uint64_t w = 0;
    for (uint32_t k = 0; k < ts.n_spans; k++) {
      const mq_span& sp = r->spans[ts.span_base + k];
      if (sp.n_sub) memcpy(out + w, r->sub_pool + sp.sub_off, (size_t)sp.n_sub * sizeof(mq_client_row));
      w += sp.n_sub;
      if (!picked && sp.n_shr) {
        memcpy(shared + ns, r->shared_pool + sp.shr_off, (size_t)sp.n_shr * sizeof(mq_shared_row));
        ns += sp.n_shr;
      }
    }
    if (w != ts.n_rows) return fail(MQ_EIO, "spans disagree with n_rows");
    const bool set = (ts.flags & MQ_TOPIC_SET_PATCHES) != 0;
    if (ts.n_patches && (set ? ts.patch_base + ts.n_patches > r->n_set_patches || !r->merge_row_base
                             : ts.patch_base + ts.n_patches > r->n_patches))
      return fail(MQ_EIO, "patch range out of bounds");
    const bool codes = (r->flags & MQ_SPANS_PATCH_CODES) != 0;
    for (uint32_t k = 0; k < ts.n_patches; k++) {
      const uint32_t x = !set ? 0u
                         : codes ? (reinterpret_cast<const uint32_t*>(r->set_patches)[ts.patch_base + k] >> 3) >>
                                       MQ_CODE_SET_ROW_BITS
                                 : r->set_patches[ts.patch_base + k].row >> MQ_SET_ROW_BITS;
      if (set && (uint64_t)r->merge_row_base[t] + x >= r->n_merge_rows) return fail(MQ_EIO, "merge row out of bounds");
      const mq_patch p = mq_topic_patch(r, t, k);
      if (p.row >= ts.n_rows) return fail(MQ_EIO, "patch row out of range");
      out[p.row].meta = mq_patch_apply(p.meta, out[p.row].meta, out[p.row].identifier);
    }
    if (picked && ts.n_shared) {
      memcpy(shared + ns, r->picked_rows + ts.picked_base, (size_t)ts.n_shared * sizeof(mq_shared_row));
      ns += ts.n_shared;
    }
    nr += ts.n_rows;
  }
  if (n_rows) *n_rows = nr;
  if (n_shared) *n_shared = ns;
  return 0;
}

int mq_match_device(mq_index* idx, const uint8_t* d_tb, const uint64_t* d_to, uint32_t n, void* stream,
                    mq_match_result* out) {
  if (!out || (n && !d_to)) return fail(MQ_EINVAL, "null argument");
  return guarded(idx, [&] {
    idx->device().match(*idx->ix, d_tb, d_to, n, (hipStream_t)stream, nullptr, out);
    return 0;
  });
}

int mq_match_device_chunks(mq_index* idx, const uint8_t* d_tb, const uint64_t* d_to, uint32_t n, void* stream,
                           mq_chunk_fn fn, void* user) {
  if (n && !d_to) return fail(MQ_EINVAL, "null argument");
  return guarded(idx, [&] {
    mq_match_result last;
    idx->device().match(*idx->ix, d_tb, d_to, n, (hipStream_t)stream, nullptr, &last, fn, user);
    return 0;
  });
}

int mq_select_shared_device(mq_index* idx, const mq_match_result* chunk, void* stream,
                            mq_shared_row* d_sel, uint32_t* d_n) {
  if (!chunk || (chunk->n_topics && (!chunk->topics || !d_n)) || (chunk->n_shared_rows && (!chunk->shared_rows || !d_sel)))
    return fail(MQ_EINVAL, "null argument");
  if (!idx) return fail(MQ_EINVAL, "null index");
  // No handle lock: this is called from inside mq_match_device_chunks' consumer, which runs
  // under it. It reads only the chunk and the device's guard flag, set up by that match.
  if (!idx->dev) return fail(MQ_EINVAL, "no match has run on this index");
  try {
    idx->dev->select_shared(*chunk, (hipStream_t)stream, reinterpret_cast<ShrRec*>(d_sel), d_n);
    return 0;
  } catch (const HipError& e) {
    return fail(MQ_EIO, e.where);
  }
}

uint32_t mq_match_chunks(const mq_index* idx) {
  return idx && idx->dev ? idx->dev->last_chunks() : 0;
}

int mq_messages_batch(mq_index* idx, const uint8_t* fb, const uint64_t* fo, uint32_t n, mq_msg_result** out) {
  if (!out || (n && (!fo || (!fb && fo[n] != 0)))) return fail(MQ_EINVAL, "null argument");
  return guarded(idx, [&] {
    Device& d = idx->device();
    std::unique_ptr<MsgHolder> h(new MsgHolder());
    const uint8_t* dfb = nullptr;
    const uint64_t* dfo = nullptr;
    if (n) d.stage_inputs(fb, fo, n, nullptr, &dfb, &dfo);
    mq_msg_result dev_out;
    HostMsg hm;
    d.messages(*idx->ix, dfb, dfo, n, nullptr, &hm, &dev_out);
    h->base.swap(hm.base);
    h->count.swap(hm.count);
    h->handles.swap(hm.handles);
    mq_msg_result& r = h->pub;
    r = mq_msg_result{};
    r.n_filters = n;
    r.base = h->base.data();
    r.count = h->count.data();
    r.handles = h->handles.data();
    r.n_handles = h->handles.size();
    *out = &h->pub;
    std::lock_guard<std::mutex> lk(g_res_mu);
    g_results[&h->pub] = 2;
    h.release();
    return 0;
  });
}

int mq_messages_device(mq_index* idx, const uint8_t* d_fb, const uint64_t* d_fo, uint32_t n, void* stream,
                       mq_msg_result* out) {
  if (!out || (n && !d_fo)) return fail(MQ_EINVAL, "null argument");
  return guarded(idx, [&] {
    idx->device().messages(*idx->ix, d_fb, d_fo, n, (hipStream_t)stream, nullptr, out);
    return 0;
  });
}

int mq_messages_runs_device(mq_index* idx, const uint8_t* d_fb, const uint64_t* d_fo, uint32_t n, void* stream,
                            mq_msg_runs_result* out) {
  if (!out || (n && !d_fo)) return fail(MQ_EINVAL, "null argument");
  return guarded(idx, [&] {
    idx->device().messages(*idx->ix, d_fb, d_fo, n, (hipStream_t)stream, nullptr, nullptr, out);
    return 0;
  });
}

int mq_messages_runs_batch(mq_index* idx, const uint8_t* fb, const uint64_t* fo, uint32_t n, mq_msg_runs_result** out) {
  if (!out || (n && (!fo || (!fb && fo[n] != 0)))) return fail(MQ_EINVAL, "null argument");
  return guarded(idx, [&] {
    Device& d = idx->device();
    std::unique_ptr<MsgRunsHolder> h(new MsgRunsHolder());
    const uint8_t* dfb = nullptr;
    const uint64_t* dfo = nullptr;
    if (n) d.stage_inputs(fb, fo, n, nullptr, &dfb, &dfo);
    mq_msg_runs_result dev_out;
    d.messages(*idx->ix, dfb, dfo, n, nullptr, nullptr, nullptr, &dev_out, &h->data);
    mq_msg_runs_result& r = h->pub;
    r = dev_out;  // counts; pointers replaced by the host copies
    r.run_base = h->data.run_base.data();
    r.n_runs = h->data.n_runs.data();
    r.base = h->data.base.data();
    r.count = h->data.count.data();
    r.runs = reinterpret_cast<const mq_msg_run*>(h->data.runs.data());
    r.handles = h->data.handles ? h->data.handles->data() : nullptr;
    *out = &h->pub;
    std::lock_guard<std::mutex> lk(g_res_mu);
    g_results[&h->pub] = 5;
    h.release();
    return 0;
  });
}

int mq_msg_runs_expand(const mq_msg_runs_result* r, uint32_t first, uint32_t count, uint64_t* out, uint64_t cap,
                       uint64_t* n_out) {
  if (!r || (uint64_t)first + count > r->n_filters) return fail(MQ_EINVAL, "filter range out of bounds");
  {
    std::lock_guard<std::mutex> lk(g_res_mu);
    auto it = g_results.find((void*)r);
    if (it == g_results.end() || it->second != 5) return fail(MQ_EINVAL, "not a host runs result (mq_messages_runs_batch)");
  }
  // filter i at out[base[i] - base[first]] (the expanded layout: a batch the particle walk answered
  // may leave gaps between filters, where its count pass reserved more than the filter holds)
  uint64_t end = 0;
  const uint64_t b0 = count ? r->base[first] : 0;
  for (uint32_t i = first; i < first + count; i++) {
    if (r->run_base[i] + r->n_runs[i] > r->n_runs_total) return fail(MQ_EIO, "run range out of bounds");
    if (r->base[i] < b0) return fail(MQ_EIO, "filter bases out of order");
    const uint64_t w = r->base[i] - b0;
    if (w + r->count[i] > cap) return fail(MQ_ERANGE, "output capacity");
    if (r->count[i] && !out) return fail(MQ_EINVAL, "null output");
    uint64_t got = 0;
    for (uint64_t k = r->run_base[i]; k < r->run_base[i] + r->n_runs[i]; k++) {
      const mq_msg_run& run = r->runs[k];
      if ((uint64_t)run.first + run.count > r->n_handles || got + run.count > r->count[i])
        return fail(MQ_EIO, "run out of bounds");
      memcpy(out + w + got, r->handles + run.first, (size_t)run.count * sizeof(uint64_t));
      got += run.count;
    }
    if (got != r->count[i]) return fail(MQ_EIO, "runs disagree with the filter's count");
    end = std::max(end, w + got);
  }
  if (n_out) *n_out = end;
  return 0;
}

int mq_acl_match_batch(mq_index* idx, const uint8_t* fb, const uint64_t* fo, uint32_t nf, const uint8_t* tb,
                       const uint64_t* to, uint32_t nt, const uint32_t* pf, const uint32_t* pt, uint64_t n_pairs,
                       mq_acl_result** out) {
  if (!out || !fo || !to || (n_pairs && (!pf || !pt)) || (fo[nf] && !fb) || (to[nt] && !tb))
    return fail(MQ_EINVAL, "null argument");
  return guarded(idx, [&] {
    std::unique_ptr<AclHolder> h(new AclHolder());
    idx->device().acl(fb, fo, nf, tb, to, nt, pf, pt, n_pairs, &h->data);
    mq_acl_result& r = h->pub;
    r.n_pairs = n_pairs;
    r.matched = h->data.matched.data();
    r.n_elems = h->data.n_elems.data();
    r.elem_base = h->data.elem_base.data();
    r.elems = h->data.elems.data();
    *out = &h->pub;
    std::lock_guard<std::mutex> lk(g_res_mu);
    g_results[&h->pub] = 3;
    h.release();
    return 0;
  });
}

void mq_result_free(void* r) {
  if (!r) return;
  int kind = 0;
  {
    std::lock_guard<std::mutex> lk(g_res_mu);
    auto it = g_results.find(r);
    if (it == g_results.end()) return;
    kind = it->second;
    g_results.erase(it);
  }
  if (kind == 1) delete reinterpret_cast<MatchHolder*>(r);
  if (kind == 2) delete reinterpret_cast<MsgHolder*>(r);
  if (kind == 3) delete reinterpret_cast<AclHolder*>(r);
  if (kind == 5) delete reinterpret_cast<MsgRunsHolder*>(r);
  if (kind == 4) {
    SpanHolder* h = reinterpret_cast<SpanHolder*>(r);
    std::shared_ptr<IndexLock> lk = h->lk;
    const uint64_t gen = h->gen;
    delete h;
    lk->views.release(gen);
  }
}

int mq_sync(mq_index* idx, void* stream) {
  return guarded(idx, [&] {
    idx->device().sync(*idx->ix, (hipStream_t)stream);
    return 0;
  });
}

int mq_index_stats(const mq_index* cidx, mq_stats* out) {
  mq_index* idx = const_cast<mq_index*>(cidx);
  if (!out) return fail(MQ_EINVAL, "null out");
  return guarded(idx, [&] {
    const Index& x = *idx->ix;
    *out = mq_stats{};
    out->nodes = x.n_nodes();
    out->edges = x.n_edges();
    out->edge_capacity = x.edges.size();
    out->subs = x.subs.live;
    out->subs_merge = x.n_subs_merge();
    out->shared = x.shr.live;
    out->inlines = x.inl.live;
    out->retained = x.retained_len();
    out->retained_live = x.msg.h[kRoot].below_live;  // live retained particles (every one is below the root)
    out->max_depth = x.max_depth();
    out->edge_load = x.edge_load_at(x.edges.size());
    out->partners = x.parts.live;
    out->foreign = x.foreign_subs();
    if (idx->dev) {
      out->device_bytes = idx->dev->device_bytes();
      out->upload_bytes_total = idx->dev->upload_bytes();
      out->syncs = idx->dev->syncs();
    }
    return 0;
  });
}

int mq_index_check(mq_index* idx) {
  return guarded(idx, [&]() -> int {
    std::string why;
    if (!idx->ix->check(&why)) return fail(MQ_EIO, "index check: " + why);
    return 0;
  });
}

int mq_device_check(mq_index* idx) {
  return guarded(idx, [&]() -> int {
    const std::string why = idx->device().verify(*idx->ix);
    if (!why.empty()) return fail(MQ_EIO, "device check: " + why);
    return 0;
  });
}

int mq_set_option(mq_index* idx, uint32_t option, uint64_t value) {
  if (option < MQ_OPT_CHUNK_ROWS || option > MQ_OPT_MAX || option == 11) return fail(MQ_EINVAL, "unknown option");
  return guarded(idx, [&] {
    if (option == MQ_OPT_EDGE_LOAD) {  // the host image's option
      if (value != 2 && value != 4 && value != 8 && value != 16) throw std::invalid_argument("MQ_OPT_EDGE_LOAD: 2, 4, 8 or 16");
      idx->ix->set_edge_load((uint32_t)value);
      return 0;
    }
    idx->options.emplace_back(option, value);  // applied when the device is first touched
    if (idx->dev) idx->dev->set_option(option, value);
    return 0;
  });
}

int mq_profile_enable(mq_index* idx, int enable) {
  return guarded(idx, [&] {
    idx->profile = enable;
    if (idx->dev) idx->dev->prof.enable(enable != 0, (enable & MQ_PROF_WORK) != 0, (enable & MQ_PROF_WALK) != 0);
    return 0;
  });
}

int mq_profile_read(const mq_index* cidx, mq_kernel_time* out, uint32_t cap) {
  mq_index* idx = const_cast<mq_index*>(cidx);
  return guarded(idx, [&] { return idx->dev ? idx->dev->prof.read(out, cap) : 0; });
}

int mq_profile_reset(mq_index* idx) {
  return guarded(idx, [&] {
    if (idx->dev) idx->dev->prof.reset();
    return 0;
  });
}

}  // extern "C"
