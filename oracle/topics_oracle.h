// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// A CPU restatement of the reference Go `TopicsIndex` (xyzj/mqtt-server @ mochi-mqtt 2.7.9,
// /root/reference/topics.go:349-822 and packets/packets.go:168-274). It exists to check the
// MI355X engine (mqtt-server_amd/) and to time the CPU baseline in bench.py. Nothing in the
// product path may link, load or call it: only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg do.
//
// Parity pinning: the Go toolchain is absent (no `go`, no `gccgo`, no network),
// so the reference cannot be built or run here. The restatement is pinned by transcribing
// every known-answer test the reference holds for this path (topics_test.go:170-1067,
// server_test.go:1973-1999 with packets/tpackets.go:1848-1872) into tests/test_oracle_kat.py.
//
// The data structures deliberately mirror the Go ones (a particle per trie node holding
// hash maps of children / subscriptions / shared / inline subscriptions, recursive scans,
// per-call result maps and Subscription.Merge), so that the CPU baseline times the same
// algorithm the reference runs.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

namespace oracle {

// packets.Subscription (packets/packets.go:172-182). `identifiers` is the Go map; it is
// nil (has_identifiers=false) on every stored subscription (nothing in server.go sets it,
// server.go:1624-1640), and is created by the first Merge.
struct Subscription {
  std::string filter;
  int64_t identifier = 0;
  bool has_identifiers = false;
  std::map<std::string, int64_t> identifiers;
  uint8_t retain_handling = 0;
  uint8_t qos = 0;
  bool retain_as_published = false;
  bool no_local = false;

  // Subscription.Merge (packets/packets.go:254-274).
  Subscription merge(const Subscription& n) const;
};

// InlineSubscription (topics.go:306-309); the Handler func is not modelled.
struct InlineSubscription {
  Subscription sub;
};

// Subscribers (topics.go:312-317). Go maps are unordered; std::map gives a canonical order.
struct Subscribers {
  std::map<std::string, std::map<std::string, Subscription>> shared;
  std::map<std::string, Subscription> shared_selected;
  std::map<std::string, Subscription> subscriptions;
  std::map<int64_t, InlineSubscription> inline_subscriptions;
};

// Work counters for the roofline's algorithmic bytes:
// B = 8·L + 4 + 16·P + 16·S + 16·O per topic.
struct Counters {
  uint64_t levels = 0;   // L
  uint64_t lookups = 0;  // P: particles.get calls (topics.go:604,612,621)
  uint64_t scanned = 0;  // S: subscription records copied by GetAll at gathered particles
  uint64_t out_rows = 0; // O: client rows + non-base identifier rows + shared rows + inline rows
};

struct Particle;
using ParticleMap = std::unordered_map<std::string, std::unique_ptr<Particle>>;

// particle (topics.go:748-757).
struct Particle {
  std::string key;
  Particle* parent = nullptr;
  ParticleMap particles;
  std::unordered_map<std::string, Subscription> subscriptions;                        // keyed by client
  std::unordered_map<std::string, std::unordered_map<std::string, Subscription>> shared;  // group -> client
  std::unordered_map<int64_t, InlineSubscription> inline_subscriptions;               // keyed by identifier
  std::string retain_path;

  Particle* get(const std::string& k) const {
    auto it = particles.find(k);
    return it == particles.end() ? nullptr : it->second.get();
  }
  size_t shared_len() const {
    size_t n = 0;
    for (auto& g : shared) n += g.second.size();
    return n;
  }
};

// A retained packets.Packet as far as the index sees it (packets/packets.go:65-117): the
// host-side handle plus the two fields RetainMessage reads (topics.go:467).
struct RetainedPacket {
  uint64_t handle = 0;
  uint32_t payload_len = 0;
  bool retain = false;
};

// isolateParticle (topics.go:679-698).
std::string_view isolate_particle(std::string_view filter, int d, bool* has_next);
// strings.EqualFold against an ASCII target (Go unicode simple folding incl. U+017F, U+212A).
bool equal_fold_ascii(std::string_view s, std::string_view ascii_target);
// IsSharedFilter / IsValidFilter (topics.go:700-745).
bool is_shared_filter(std::string_view filter);
bool is_valid_filter(std::string_view filter, bool for_publish);
// auth.MatchTopic (hooks/auth/ledger.go:90-118): the ACL ledger's filter/topic test, with its
// captured '+' / '#' elements (spans into the topic). Not the TopicsIndex rules: a filter
// shorter than the topic matches it, and '#' needs at least one topic level at its position.
bool match_topic(std::string_view filter, std::string_view topic,
                 std::vector<std::pair<uint32_t, uint32_t>>* elements);

class TopicsIndex {
 public:
  TopicsIndex();

  bool inline_subscribe(const InlineSubscription& s);                // topics.go:368
  bool inline_unsubscribe(int64_t id, const std::string& filter);    // topics.go:382
  bool subscribe(const std::string& client, const Subscription& s);  // topics.go:401
  bool unsubscribe(const std::string& filter, const std::string& client);  // topics.go:423
  int64_t retain_message(const std::string& topic, const RetainedPacket& pk);  // topics.go:453
  std::vector<RetainedPacket> messages(const std::string& filter, Counters* c = nullptr) const;  // topics.go:525
  Subscribers subscribers(const std::string& topic, Counters* c = nullptr) const;  // topics.go:583

  // packets.Packets as TopicsIndex.Retained (topics.go:351): server.go:1726 deletes entries
  // directly (Q12); Len is consulted by scanMessages (topics.go:535).
  void retained_delete(const std::string& topic) { retained_.erase(topic); }
  void retained_add(const std::string& topic, const RetainedPacket& pk) { retained_[topic] = pk; }  // packets.go:79-83
  size_t retained_len() const { return retained_.size(); }
  bool retained_get(const std::string& topic, RetainedPacket* out) const;

  // white-box helpers used by the transcribed tests (topics_test.go:339-399)
  Particle* set(const std::string& topic, int d);
  Particle* seek(const std::string& filter, int d) const;
  void trim(Particle* n);
  Particle* root() const { return root_.get(); }
  size_t particle_count() const;

 private:
  void scan_subscribers(const std::string& topic, int d, const Particle* n, Subscribers& subs,
                        Counters* c) const;
  void gather_subscriptions(const std::string& topic, const Particle* p, Subscribers& subs,
                            Counters* c) const;
  void gather_shared(const Particle* p, Subscribers& subs, Counters* c) const;
  void gather_inline(const Particle* p, Subscribers& subs, Counters* c) const;
  void scan_messages(const std::string& filter, int d, const Particle* n,
                     std::vector<RetainedPacket>& pks, Counters* c) const;

  std::unique_ptr<Particle> root_;
  std::unordered_map<std::string, RetainedPacket> retained_;
};

// Subscribers.SelectShared with a deterministic pick (the Go pick is the first entry in
// random map order, topics.go:320-333) and MergeSharedSelected (topics.go:338-347).
void select_shared_first(Subscribers& s);
void merge_shared_selected(Subscribers& s);

}  // namespace oracle
