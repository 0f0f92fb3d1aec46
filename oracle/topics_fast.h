// CPU BASELINE — TEST / MEASUREMENT INFRASTRUCTURE ONLY (like the oracle it is built from).
//
// A second CPU restatement of TopicsIndex.Subscribers (/root/reference/topics.go:583-676,
// packets/packets.go:254-274), written for speed rather than for line-by-line fidelity, so that
// bench.py's cpu_baseline is a strong one. Same algorithm as the Go
// trie — a recursive scan over per-particle children maps keyed by segment strings, the three
// gathers with the '$' rule and Subscription.Merge — but:
//   - client and filter strings are interned to ids when the index is built (the "pre-hashed
//     keys"), so the per-topic result maps are flat per-thread tables indexed by client id with
//     epoch stamps instead of hash maps keyed by strings;
//   - subscriptions are flat per-particle arrays (no map copy per gather, GetAll);
//   - a topic is split into segments once (isolateParticle re-scans from the start per level).
// Its results are checked bit-exactly (digests) against the oracle in tests/test_oracle_kat.py.
// Built from a frozen oracle TopicsIndex; read-only and shared by every benchmark thread.
#pragma once

#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

#include "topics_oracle.h"

namespace oracle {

struct FastIndex;

// Snapshot of `idx` (client / filter ids from the maps; unknown strings get fresh ids).
FastIndex* fast_build(const TopicsIndex& idx, const std::unordered_map<std::string, uint32_t>& client_ids,
                      const std::unordered_map<std::string, uint32_t>& filter_ids);
void fast_free(FastIndex* f);

// Per-thread scratch of fast_subscribers (result tables sized by the index's client count).
struct FastScratch;
FastScratch* fast_scratch(const FastIndex& f);
void fast_scratch_free(FastScratch* s);

// Subscribers(topic) into the scratch; returns the number of result entries (client + shared +
// inline), and, when `digest` is set, the canonical digest of oracle_capi.cpp digest_subscribers
// and the four row counts.
uint64_t fast_subscribers(const FastIndex& f, FastScratch& s, const char* topic, uint32_t len,
                          uint64_t* digest, uint64_t counts[4]);

// Messages (topics.go:525-579), restated for speed the same way (bench_messages.py's
// cpu_baseline): the particle tree snapshotted into flat nodes (children maps keyed by segment
// plus a child list for the '+' / '#' enumerations), each node's retained handle looked up once
// at build time (the Retained map lookup scanMessages does per emitted particle), the filter
// split into segments once. Digest-checked against the oracle in tests/test_oracle_kat.py.
struct FastMsgIndex;
FastMsgIndex* fast_msg_build(const TopicsIndex& idx);
void fast_msg_free(FastMsgIndex* f);
// Messages(filter): the handles, appended to `out` (cleared first); returns their number.
uint64_t fast_messages(const FastMsgIndex& f, const char* filter, uint32_t len, std::vector<uint64_t>& out);

}  // namespace oracle
