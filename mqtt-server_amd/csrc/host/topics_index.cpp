// C++ host mirror of the Go TopicsIndex over the C-ABI (topics_index.h).
#include "topics_index.h"

#include <cstring>

namespace mq {
namespace host {

static void check(int rc, const char* what) {
  if (rc < 0) throw EngineError(rc, std::string(what) + ": " + mq_last_error());
}

TopicsIndex::TopicsIndex(int device, bool select_shared) {
  mq_config cfg{device, select_shared ? MQ_CFG_SELECT_SHARED : 0u, 0, 0, 0, 0};
  check(mq_index_create(&cfg, &idx_), "mq_index_create");
}

TopicsIndex::~TopicsIndex() { mq_index_destroy(idx_); }

uint32_t TopicsIndex::cid(const std::string& c) {
  auto it = client_ids_.find(c);
  if (it != client_ids_.end()) return it->second;
  const uint32_t id = (uint32_t)clients_.size();
  clients_.push_back(c);
  client_ids_.emplace(c, id);
  return id;
}

uint32_t TopicsIndex::fid(const std::string& f) {
  auto it = filter_ids_.find(f);
  if (it != filter_ids_.end()) return it->second;
  const uint32_t id = (uint32_t)filters_.size();
  filters_.push_back(f);
  filter_ids_.emplace(f, id);
  return id;
}

bool TopicsIndex::Subscribe(const std::string& client, const Subscription& sub) {
  std::lock_guard<std::mutex> lk(mu_);
  const uint32_t c = cid(client), f = fid(sub.Filter);
  const uint8_t flags = (sub.NoLocal ? MQ_SUB_NOLOCAL : 0) | (sub.RetainAsPublished ? MQ_SUB_RAP : 0) |
                        (uint8_t)((sub.RetainHandling & 3) << MQ_SUB_RH_SHIFT);
  const int rc = mq_subscribe(idx_, sub.Filter.data(), (uint32_t)sub.Filter.size(), c, f, sub.Qos, flags,
                              sub.Identifier);
  check(rc, "mq_subscribe");
  Subscription stored = sub;
  stored.HasIdentifiers = false;
  stored.Identifiers.clear();
  stored_[{c, f}] = stored;
  return rc == 1;
}

bool TopicsIndex::Unsubscribe(const std::string& filter, const std::string& client) {
  std::lock_guard<std::mutex> lk(mu_);
  const int rc = mq_unsubscribe(idx_, filter.data(), (uint32_t)filter.size(), cid(client));
  check(rc, "mq_unsubscribe");
  return rc == 1;
}

bool TopicsIndex::InlineSubscribe(const InlineSubscription& sub) {
  std::lock_guard<std::mutex> lk(mu_);
  const uint32_t f = fid(sub.Sub.Filter);
  const int rc = mq_inline_subscribe(idx_, sub.Sub.Filter.data(), (uint32_t)sub.Sub.Filter.size(),
                                     sub.Sub.Identifier, f);
  check(rc, "mq_inline_subscribe");
  inline_[{sub.Sub.Identifier, f}] = sub;
  return rc == 1;
}

bool TopicsIndex::InlineUnsubscribe(int id, const std::string& filter) {
  std::lock_guard<std::mutex> lk(mu_);
  const int rc = mq_inline_unsubscribe(idx_, filter.data(), (uint32_t)filter.size(), id);
  check(rc, "mq_inline_unsubscribe");
  return rc == 1;
}

int64_t TopicsIndex::RetainMessage(const std::string& topic, uint64_t handle, uint32_t payload_len,
                                   bool retain) {
  int64_t out = 0;
  check(mq_retain_message(idx_, topic.data(), (uint32_t)topic.size(), handle, payload_len,
                          retain ? 1 : 0, &out),
        "mq_retain_message");
  return out;
}

void TopicsIndex::RetainedDelete(const std::string& topic) {
  check(mq_retained_delete(idx_, topic.data(), (uint32_t)topic.size()), "mq_retained_delete");
}

uint64_t TopicsIndex::RetainedLen() const { return mq_retained_len(idx_); }

std::vector<uint64_t> TopicsIndex::Messages(const std::string& filter) {
  const uint64_t offs[2] = {0, filter.size()};
  uint8_t pad[16] = {0};
  const uint8_t* bytes = filter.empty() ? pad : (const uint8_t*)filter.data();
  mq_msg_result* r = nullptr;
  check(mq_messages_batch(idx_, bytes, offs, 1, &r), "mq_messages_batch");
  std::vector<uint64_t> hs(r->handles + r->base[0], r->handles + r->base[0] + r->count[0]);
  mq_result_free(r);
  return hs;
}

Subscribers TopicsIndex::Subscribers_(const std::string& topic) { return SubscribersBatch({topic})[0]; }

// One mq_match_spans call for the batch; each topic's Subscribers is rebuilt straight from its
// spans (the index's records, pinned by the result) with the topic's patches applied — no row
// copies (include/mqmatch.h, span format).
std::vector<Subscribers> TopicsIndex::SubscribersBatch(const std::vector<std::string>& topics) {
  std::lock_guard<std::mutex> lk(mu_);
  std::string bytes;
  std::vector<uint64_t> offs(1, 0);
  for (const std::string& t : topics) {
    bytes += t;
    offs.push_back(bytes.size());
  }
  bytes.resize(bytes.size() + 16, '\0');  // readable padding (include/mqmatch.h)
  mq_span_result* r = nullptr;
  check(mq_match_spans(idx_, (const uint8_t*)bytes.data(), offs.data(), (uint32_t)topics.size(), &r),
        "mq_match_spans");
  std::vector<Subscribers> out(topics.size());
  std::unordered_map<uint32_t, uint32_t> patched;  // topic row -> meta
  for (size_t t = 0; t < topics.size(); t++) {
    const mq_topic_spans& ts = r->topics[t];
    Subscribers& s = out[t];
    patched.clear();
    for (uint32_t k = 0; k < ts.n_patches; k++) patched[r->patches[ts.patch_base + k].row] = r->patches[ts.patch_base + k].meta;
    // records in gather order: a client's client row precedes its ident rows
    uint32_t rowi = 0;
    for (uint32_t k = 0; k < ts.n_spans; k++) {
      const mq_span& sp = r->spans[ts.span_base + k];
      for (uint32_t i = 0; i < sp.n_sub; i++, rowi++) {
        mq_client_row row = r->sub_pool[sp.sub_off + i];
        auto pit = patched.find(rowi);
        if (pit != patched.end()) row.meta = pit->second;
        const uint32_t kind = row.meta & MQ_ROW_KIND_MASK;
        if (kind == 0) {  // client row: merged Subscription
          Subscription sub = stored_.at({row.client_id, row.filter_id});
          sub.Qos = row.meta & MQ_META_QOS_MASK;
          sub.NoLocal = (row.meta & MQ_META_NOLOCAL) != 0;
          sub.HasIdentifiers = true;
          sub.Identifiers = {{sub.Filter, sub.Identifier}};
          s.Subscriptions[clients_[row.client_id]] = sub;
        } else if (kind == MQ_ROW_IDENT) {  // further Identifiers entry
          s.Subscriptions[clients_[row.client_id]].Identifiers[filters_[row.filter_id]] = row.identifier;
        }
      }
      if (!(r->flags & MQ_SPANS_PICKED))
        for (uint32_t i = 0; i < sp.n_shr; i++) {
          const mq_shared_row& row = r->shared_pool[sp.shr_off + i];
          s.Shared[filters_[row.filter_id]][clients_[row.client_id]] = stored_.at({row.client_id, row.filter_id});
        }
    }
    if (r->flags & MQ_SPANS_PICKED)
      for (uint32_t i = 0; i < ts.n_shared; i++) {
        const mq_shared_row& row = r->picked_rows[ts.picked_base + i];
        s.Shared[filters_[row.filter_id]][clients_[row.client_id]] = stored_.at({row.client_id, row.filter_id});
      }
    for (uint32_t i = 0; i < ts.n_inline; i++) {
      const mq_inline_row& row = r->inline_rows[ts.inline_base + i];
      s.InlineSubscriptions[row.identifier] = inline_.at({row.identifier, row.filter_id});
    }
  }
  mq_result_free(r);
  return out;
}

}  // namespace host
}  // namespace mq
