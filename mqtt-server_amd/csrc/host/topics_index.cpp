// C++ host mirror of the Go TopicsIndex over the C-ABI (topics_index.h).
#include "topics_index.h"

#include <chrono>

#include <climits>
#include <cstring>

namespace mq {
namespace host {

static void check(int rc, const char* what) {
  if (rc < 0) throw EngineError(rc, std::string(what) + ": " + mq_last_error());
}

// An id no subscription uses: Unsubscribe for a client the index never saw still answers
// whether the filter's particle exists (topics.go:434-437).
static constexpr uint32_t kNoClient = UINT32_MAX;

uint64_t Epochs::begin() {
  std::lock_guard<std::mutex> lk(mu_);
  active_.insert(++clock_);
  return clock_;
}

void Epochs::end(uint64_t stamp) {
  std::lock_guard<std::mutex> lk(mu_);
  active_.erase(active_.find(stamp));
}

uint64_t Epochs::now() {
  std::lock_guard<std::mutex> lk(mu_);
  return ++clock_;
}

uint64_t Epochs::oldest_active() const {
  std::lock_guard<std::mutex> lk(mu_);
  return active_.empty() ? UINT64_MAX : *active_.begin();
}

uint32_t IdTable::intern(const std::string& s) {
  auto it = ids_.find(s);
  if (it != ids_.end()) return it->second;
  uint32_t id;
  if (!free_.empty() && free_.front().second < ep_.oldest_active()) {
    id = free_.front().first;
    free_.pop_front();
    strs_[id] = s;
  } else {
    id = (uint32_t)strs_.size();
    if (id == kNoClient) throw EngineError(MQ_ENOMEM, "id space exhausted");
    strs_.push_back(s);
    refs_.push_back(0);
  }
  ids_.emplace(s, id);
  return id;
}

bool IdTable::find(const std::string& s, uint32_t* id) const {
  auto it = ids_.find(s);
  if (it == ids_.end()) return false;
  *id = it->second;
  return true;
}

void IdTable::unref(uint32_t id, uint64_t now) {
  if (--refs_[id] != 0) return;
  ids_.erase(strs_[id]);
  free_.emplace_back(id, now);  // strs_[id] stays readable for batches still in flight
}

void IdTable::tidy(uint32_t id, uint64_t now) {
  if (refs_[id] != 0) return;
  auto it = ids_.find(strs_[id]);
  if (it == ids_.end() || it->second != id) return;  // already released
  ids_.erase(it);
  free_.emplace_back(id, now);
}

void TopicsIndex::fail_tidy(int rc, const char* what, const uint32_t* clients, size_t nc, const uint32_t* filters,
                            size_t nf) {
  {
    std::unique_lock<WriterPreferringMutex> lk(tables_mu_);
    const uint64_t now = epochs_.now();
    for (size_t i = 0; i < nc; i++) clients_.tidy(clients[i], now);
    for (size_t i = 0; i < nf; i++) filters_.tidy(filters[i], now);
  }
  check(rc, what);
  throw EngineError(rc, what);  // rc < 0 here: check threw
}

TopicsIndex::TopicsIndex(int device, bool select_shared) {
  mq_config cfg{device, select_shared ? MQ_CFG_SELECT_SHARED : 0u, 0, 0, 0, 0};
  check(mq_index_create(&cfg, &idx_), "mq_index_create");
}

TopicsIndex::~TopicsIndex() { mq_index_destroy(idx_); }

static uint8_t sub_flags(const Subscription& sub) {
  return (sub.NoLocal ? MQ_SUB_NOLOCAL : 0) | (sub.RetainAsPublished ? MQ_SUB_RAP : 0) |
         (uint8_t)((sub.RetainHandling & 3) << MQ_SUB_RH_SHIFT);
}

void TopicsIndex::store(uint32_t c, uint32_t f, const Subscription& sub) {
  Subscription stored = sub;
  stored.HasIdentifiers = false;
  stored.Identifiers.clear();
  auto it = stored_.find({c, f});
  if (it != stored_.end()) {
    it->second = stored;
    return;
  }
  stored_.emplace(std::make_pair(c, f), stored);
  clients_.ref(c);
  filters_.ref(f);
}

namespace {
using WClock = std::chrono::steady_clock;
void note_max(std::atomic<uint64_t>& m, WClock::time_point a, WClock::time_point b) {
  const uint64_t us = (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(b - a).count();
  for (uint64_t v = m.load(); us > v && !m.compare_exchange_weak(v, us);) {
  }
}
// the update lock, with its wait and hold times noted (UpdateWaits)
struct UpdLock {
  FifoMutex& mu;
  std::atomic<uint64_t>& held;
  WClock::time_point t;
  UpdLock(FifoMutex& m, std::atomic<uint64_t>& wait_max, std::atomic<uint64_t>& held_max) : mu(m), held(held_max) {
    const auto t0 = WClock::now();
    mu.lock();
    t = WClock::now();
    note_max(wait_max, t0, t);
  }
  ~UpdLock() {
    note_max(held, t, WClock::now());
    mu.unlock();
  }
};
}  // namespace

#define MQ_UPDATE_LOCK UpdLock up(upd_mu_, waits_.upd, waits_.held)

bool TopicsIndex::Subscribe(const std::string& client, const Subscription& sub) {
  MQ_UPDATE_LOCK;
  const auto t1 = WClock::now();
  uint32_t c, f;
  {
    std::unique_lock<WriterPreferringMutex> lk(tables_mu_);
    note_max(waits_.tables, t1, WClock::now());
    c = clients_.intern(client);
    f = filters_.intern(sub.Filter);
  }
  const auto t2 = WClock::now();
  const int rc = mq_subscribe(idx_, sub.Filter.data(), (uint32_t)sub.Filter.size(), c, f, sub.Qos,
                              sub_flags(sub), sub.Identifier);
  const auto t3 = WClock::now();
  note_max(waits_.engine, t2, t3);
  if (rc < 0) fail_tidy(rc, "mq_subscribe", &c, 1, &f, 1);
  std::unique_lock<WriterPreferringMutex> lk(tables_mu_);
  note_max(waits_.tables, t3, WClock::now());
  store(c, f, sub);
  return rc == 1;
}

bool TopicsIndex::Unsubscribe(const std::string& filter, const std::string& client) {
  MQ_UPDATE_LOCK;
  uint32_t c = kNoClient, f = 0;
  bool known_f;
  const auto t1 = WClock::now();
  {
    std::shared_lock<WriterPreferringMutex> lk(tables_mu_);
    note_max(waits_.tables, t1, WClock::now());
    if (!clients_.find(client, &c)) c = kNoClient;  // looked up, never interned
    known_f = filters_.find(filter, &f);
  }
  const auto t2 = WClock::now();
  const int rc = mq_unsubscribe(idx_, filter.data(), (uint32_t)filter.size(), c);
  const auto t3 = WClock::now();
  note_max(waits_.engine, t2, t3);
  check(rc, "mq_unsubscribe");
  if (c != kNoClient && known_f) {
    std::unique_lock<WriterPreferringMutex> lk(tables_mu_);
    note_max(waits_.tables, t3, WClock::now());
    auto it = stored_.find({c, f});
    if (it != stored_.end()) {
      stored_.erase(it);
      const uint64_t now = epochs_.now();
      clients_.unref(c, now);
      filters_.unref(f, now);
    }
  }
  return rc == 1;
}

bool TopicsIndex::InlineSubscribe(const InlineSubscription& sub) {
  MQ_UPDATE_LOCK;
  uint32_t f;
  {
    std::unique_lock<WriterPreferringMutex> lk(tables_mu_);
    f = filters_.intern(sub.Sub.Filter);
  }
  const int rc = mq_inline_subscribe(idx_, sub.Sub.Filter.data(), (uint32_t)sub.Sub.Filter.size(),
                                     sub.Sub.Identifier, f);
  if (rc < 0) fail_tidy(rc, "mq_inline_subscribe", nullptr, 0, &f, 1);
  std::unique_lock<WriterPreferringMutex> lk(tables_mu_);
  auto it = inline_.find({sub.Sub.Identifier, f});
  if (it != inline_.end()) {
    it->second = sub;
  } else {
    inline_.emplace(std::make_pair(sub.Sub.Identifier, f), sub);
    filters_.ref(f);
  }
  return rc == 1;
}

bool TopicsIndex::InlineUnsubscribe(int id, const std::string& filter) {
  MQ_UPDATE_LOCK;
  const int rc = mq_inline_unsubscribe(idx_, filter.data(), (uint32_t)filter.size(), id);
  check(rc, "mq_inline_unsubscribe");
  std::unique_lock<WriterPreferringMutex> lk(tables_mu_);
  uint32_t f;
  if (filters_.find(filter, &f)) {
    auto it = inline_.find({id, f});
    if (it != inline_.end()) {
      inline_.erase(it);
      filters_.unref(f, epochs_.now());
    }
  }
  return rc == 1;
}

std::vector<bool> TopicsIndex::LoadSubscriptions(const std::vector<std::pair<std::string, Subscription>>& subs) {
  MQ_UPDATE_LOCK;
  const size_t n = subs.size();
  std::string bytes;
  std::vector<uint64_t> offs(1, 0);
  std::vector<uint32_t> cids(n), fids(n);
  std::vector<uint8_t> qos(n), flags(n), out_new(std::max<size_t>(n, 1));
  std::vector<int32_t> idents(n);
  {
    std::unique_lock<WriterPreferringMutex> lk(tables_mu_);
    for (size_t i = 0; i < n; i++) {
      const Subscription& s = subs[i].second;
      cids[i] = clients_.intern(subs[i].first);
      fids[i] = filters_.intern(s.Filter);
      qos[i] = s.Qos;
      flags[i] = sub_flags(s);
      idents[i] = s.Identifier;
      bytes += s.Filter;
      offs.push_back(bytes.size());
    }
  }
  bytes.resize(bytes.size() + 16, '\0');
  const int rc = mq_subscribe_bulk(idx_, (const uint8_t*)bytes.data(), offs.data(), cids.data(), fids.data(),
                                   qos.data(), flags.data(), idents.data(), n, out_new.data());
  if (rc < 0) fail_tidy(rc, "mq_subscribe_bulk", cids.data(), n, fids.data(), n);
  std::unique_lock<WriterPreferringMutex> lk(tables_mu_);
  std::vector<bool> out(n);
  for (size_t i = 0; i < n; i++) {
    store(cids[i], fids[i], subs[i].second);
    out[i] = out_new[i] != 0;
  }
  return out;
}

int64_t TopicsIndex::RetainMessage(const std::string& topic, uint64_t handle, uint32_t payload_len,
                                   bool retain) {
  MQ_UPDATE_LOCK;
  int64_t out = 0;
  check(mq_retain_message(idx_, topic.data(), (uint32_t)topic.size(), handle, payload_len,
                          retain ? 1 : 0, &out),
        "mq_retain_message");
  return out;
}

void TopicsIndex::RetainedDelete(const std::string& topic) {
  MQ_UPDATE_LOCK;
  check(mq_retained_delete(idx_, topic.data(), (uint32_t)topic.size()), "mq_retained_delete");
}

void TopicsIndex::RetainedAdd(const std::string& topic, uint64_t handle, uint32_t payload_len, bool retain) {
  MQ_UPDATE_LOCK;
  check(mq_retained_set(idx_, topic.data(), (uint32_t)topic.size(), handle, payload_len, retain ? 1 : 0),
        "mq_retained_set");
}

uint64_t TopicsIndex::RetainedLen() const { return mq_retained_len(idx_); }

size_t TopicsIndex::live_clients() const {
  std::shared_lock<WriterPreferringMutex> lk(tables_mu_);
  return clients_.live();
}

size_t TopicsIndex::live_filters() const {
  std::shared_lock<WriterPreferringMutex> lk(tables_mu_);
  return filters_.live();
}

std::vector<uint64_t> TopicsIndex::Messages(const std::string& filter) {
  const uint64_t offs[2] = {0, filter.size()};
  std::string bytes = filter;
  bytes.resize(bytes.size() + 16, '\0');  // readable padding (include/mqmatch.h)
  mq_msg_result* r = nullptr;
  check(mq_messages_batch(idx_, (const uint8_t*)bytes.data(), offs, 1, &r), "mq_messages_batch");
  std::vector<uint64_t> hs(r->handles + r->base[0], r->handles + r->base[0] + r->count[0]);
  mq_result_free(r);
  return hs;
}

SpanBatch::~SpanBatch() {
  mq_result_free(r_);
  ix_.epochs().end(stamp_);
}

std::string TopicView::client(uint32_t id) const { return b_->index().ClientName(id); }
std::string TopicView::filter(uint32_t id) const { return b_->index().FilterName(id); }

std::string TopicsIndex::ClientName(uint32_t id) const {
  std::shared_lock<WriterPreferringMutex> lk(tables_mu_);
  return clients_.str(id);
}

std::string TopicsIndex::FilterName(uint32_t id) const {
  std::shared_lock<WriterPreferringMutex> lk(tables_mu_);
  return filters_.str(id);
}

static PackedTopics pack(const std::vector<std::string>& topics) {
  PackedTopics p;
  size_t nb = 0;
  for (const std::string& t : topics) nb += t.size();
  p.bytes.reserve(nb + 16);
  p.offs.reserve(topics.size() + 1);
  for (const std::string& t : topics) p.add(t);
  p.finish();
  return p;
}

std::shared_ptr<const SpanBatch> TopicsIndex::SubscribersSpans(const PackedTopics& topics) {
  const uint64_t stamp = epochs_.begin();
  mq_span_result* r = nullptr;
  const int rc = mq_match_spans(idx_, (const uint8_t*)topics.bytes.data(), topics.offs.data(), topics.size(), &r);
  if (rc < 0) {
    epochs_.end(stamp);
    check(rc, "mq_match_spans");
  }
  // the result (and its pin of the host image) is owned from here on, whatever throws
  std::unique_ptr<mq_span_result, void (*)(void*)> own(r, mq_result_free);
  std::shared_ptr<const SpanBatch> batch;
  try {
    batch = std::make_shared<const SpanBatch>(*this, r, stamp);
  } catch (...) {
    epochs_.end(stamp);
    throw;
  }
  own.release();  // the batch frees it
  return batch;
}

std::vector<TopicView> TopicsIndex::SubscribersViews(const std::vector<std::string>& topics) {
  std::shared_ptr<const SpanBatch> batch = SubscribersSpans(pack(topics));
  std::vector<TopicView> out;
  out.reserve(topics.size());
  for (uint32_t t = 0; t < topics.size(); t++) out.emplace_back(batch, t);
  return out;
}

Subscribers TopicsIndex::Subscribers_(const std::string& topic) { return SubscribersBatch(std::vector<std::string>{topic})[0]; }

// One mq_match_spans call for the batch, with no host lock held; then each topic's Subscribers
// is rebuilt straight from its spans (the index's records, pinned by the result) with the
// topic's patches applied — no row copies (include/mqmatch.h, span format) — under a shared
// lock of the host tables. The batch's epoch keeps every id its rows name from being reused
// meanwhile; a subscription removed since the match (its stored entry gone) is rebuilt from the
// row itself.
std::vector<Subscribers> TopicsIndex::SubscribersBatch(const std::vector<std::string>& topics) {
  return SubscribersBatch(pack(topics));
}

std::vector<Subscribers> TopicsIndex::SubscribersBatch(const PackedTopics& topics) {
  struct Guard {
    Epochs& ep;
    uint64_t stamp;
    ~Guard() { ep.end(stamp); }
  } guard{epochs_, epochs_.begin()};
  mq_span_result* r = nullptr;
  check(mq_match_spans(idx_, (const uint8_t*)topics.bytes.data(), topics.offs.data(), topics.size(), &r),
        "mq_match_spans");
  // freed however this ends (an exception while building the maps must not leak the pin, or
  // every later update would wait for it); declared before the table lock, so released after it
  std::unique_ptr<mq_span_result, void (*)(void*)> own(r, mq_result_free);
  std::vector<Subscribers> out(topics.size());
  std::shared_lock<WriterPreferringMutex> lk(tables_mu_);
  auto stored = [&](uint32_t c, uint32_t f, const mq_client_row* row) {
    auto it = stored_.find({c, f});
    if (it != stored_.end()) return it->second;
    Subscription s;  // unsubscribed since the match
    s.Filter = filters_.str(f);
    if (row) {
      s.Identifier = row->identifier;
      s.Qos = row->meta & MQ_META_QOS_MASK;
    }
    return s;
  };
  std::unordered_map<uint32_t, uint32_t> patched;  // topic row -> meta
  for (size_t t = 0; t < out.size(); t++) {
    const mq_topic_spans& ts = r->topics[t];
    Subscribers& s = out[t];
    patched.clear();
    for (uint32_t k = 0; k < ts.n_patches; k++) {  // own or merge-set patches (mq_topic_patch)
      const mq_patch p = mq_topic_patch(r, (uint32_t)t, k);
      patched[p.row] = p.meta;
    }
    // records in gather order: a client's client row precedes its ident rows
    uint32_t rowi = 0;
    for (uint32_t k = 0; k < ts.n_spans; k++) {
      const mq_span& sp = r->spans[ts.span_base + k];
      for (uint32_t i = 0; i < sp.n_sub; i++, rowi++) {
        mq_client_row row = r->sub_pool[sp.sub_off + i];
        auto pit = patched.find(rowi);
        if (pit != patched.end()) row.meta = mq_patch_apply(pit->second, row.meta, row.identifier);
        const uint32_t kind = row.meta & MQ_ROW_KIND_MASK;
        if (kind == 0) {  // client row: merged Subscription
          Subscription sub = stored(row.client_id, row.filter_id, &row);
          sub.Qos = row.meta & MQ_META_QOS_MASK;
          sub.NoLocal = (row.meta & MQ_META_NOLOCAL) != 0;
          sub.HasIdentifiers = true;
          sub.Identifiers = {{sub.Filter, sub.Identifier}};
          s.Subscriptions[clients_.str(row.client_id)] = sub;
        } else if (kind == MQ_ROW_IDENT) {  // further Identifiers entry
          s.Subscriptions[clients_.str(row.client_id)].Identifiers[filters_.str(row.filter_id)] = row.identifier;
        }
      }
      if (!(r->flags & MQ_SPANS_PICKED))
        for (uint32_t i = 0; i < sp.n_shr; i++) {
          const mq_shared_row& row = r->shared_pool[sp.shr_off + i];
          s.Shared[filters_.str(row.filter_id)][clients_.str(row.client_id)] =
              stored(row.client_id, row.filter_id, nullptr);
        }
    }
    if (r->flags & MQ_SPANS_PICKED)
      for (uint32_t i = 0; i < ts.n_shared; i++) {
        const mq_shared_row& row = r->picked_rows[ts.picked_base + i];
        s.Shared[filters_.str(row.filter_id)][clients_.str(row.client_id)] =
            stored(row.client_id, row.filter_id, nullptr);
      }
    for (uint32_t i = 0; i < ts.n_inline; i++) {
      const mq_inline_row& row = r->inline_rows[ts.inline_base + i];
      auto it = inline_.find({row.identifier, row.filter_id});
      if (it != inline_.end()) {
        s.InlineSubscriptions[row.identifier] = it->second;
      } else {  // unsubscribed since the match
        InlineSubscription is;
        is.Sub.Filter = filters_.str(row.filter_id);
        is.Sub.Identifier = row.identifier;
        s.InlineSubscriptions[row.identifier] = is;
      }
    }
  }
  return out;
}

}  // namespace host
}  // namespace mq
