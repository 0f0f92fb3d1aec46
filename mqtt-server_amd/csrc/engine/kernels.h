// Kernel-side structures and launch wrappers of the engine (kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "layout.h"

namespace mq {

constexpr uint32_t kLdsTab = 512;      // LDS merge-table slots per wavefront
constexpr uint32_t kScanBlock = 1024;  // topics per scan block (= chunk granule)
constexpr uint32_t kGatherCap = 64;    // per-topic gather slots written by the count pass
constexpr uint32_t kLdsTabMax = 384;   // table-bound records allowed in an LDS merge table
constexpr uint32_t kTList = 512;       // queued table-bound records per wave (flushed when full)
constexpr uint32_t kPairMax = 128;     // gathers covered by the pair analysis
constexpr uint32_t kHitMax = 128;      // (g, h) pair hits held per topic
constexpr uint32_t kBitWin = 2048;     // may-merge slots per table-bound bitmap window

// Device pointers of the resident index image.
struct DevIndex {
  const EdgeSlot* edges;
  uint64_t edge_mask;
  const NodeWalk* walk;
  const NodeLists* lists;
  const NodeMsg* msg;
  const SegInfo* seginfo;
  const uint8_t* segbytes;
  const SubRec* subs;
  const NodePair* npair;
  const PairEnt* pent;
  const uint32_t* plist;
  const ShrRec* shr;
  const InlRec* inl;
  const uint32_t* children;
  uint64_t retained_len;
  uint64_t empty_topic_handle;
  uint32_t empty_topic_live;
  uint32_t pad;
  uint32_t* err;  // [0] error bits (kErr*), [1] gather-slot overflow; checked by the host
};

constexpr uint32_t kErrWalkGuard = 1u;
constexpr uint32_t kErrTableFull = 2u;
constexpr uint64_t kWalkGuard = 1ull << 26;

// Exclusive offsets of a topic's outputs (scan of TopicCount).
struct TopicOff {
  uint64_t g, rows, shr, inl, tab;
};

// Same layout as mq_topic_result (include/mqmatch.h).
struct mq_topic_result_dev {
  uint64_t sub_base, shared_base, inline_base;
  uint32_t sub_cap, n_client, n_ident, n_shared, n_inline, reserved;
};

struct EmitArgs {
  DevIndex ix;
  uint32_t t0, t1;          // topic range of this chunk
  const TopicOff* off;      // per-topic offsets (n + 1)
  TopicOff base;            // off[t0]: the chunk's output buffers start here
  const uint32_t* gathers;
  uint32_t gather_stride;   // kGatherCap: per-topic slots of the count pass; 0: compact at off.g
  SubRec* rows;
  ShrRec* shr_rows;
  InlRec* inl_rows;
  uint32_t* tab;            // overflow pass: merge tables, key | row | meta planes of tab_cap
  uint64_t tab_cap;
  mq_topic_result_dev* res; // indexed t - t0
  // Fast pass (list == nullptr): merge tables in LDS. A topic whose table-bound records could
  // outgrow LDS appends {t, slots} to the overflow list and is left for the overflow pass
  // (list != nullptr), which claims `slots` of global table per topic.
  const uint32_t* list;     // overflow pass: pairs {topic, table slots}
  uint32_t n_list;
  uint32_t* ovf;            // [0] count, [1] total slots, [2] claim counter, [4..] pairs
  unsigned long long* wprof;  // diagnosis only (MQ_EMIT_PROF): per-phase wave cycles, kWp* slots
};

// k_emit wave-profile slots (EmitArgs::wprof).
enum : int {
  kWpWaves, kWpTotal, kWpSetup, kWpCopy, kWpMerge, kWpDrain, kWpTail, kWpMergeRecs,
  kWpTabRecs, kWpLookups, kWpProbes, kWpChunks, kWpCount = 16
};

void launch_walk(bool fill, const uint8_t* tb, const uint64_t* to, uint32_t n, const DevIndex& ix,
                 TopicCount* cnt, const TopicOff* off, uint32_t* gathers, hipStream_t s);
void launch_scan(const TopicCount* cnt, uint32_t n, TopicOff* bsum, TopicOff* bpre, TopicOff* off,
                 hipStream_t s);
void launch_emit(const EmitArgs& a, hipStream_t s);
void launch_msg(bool fill, const uint8_t* fb, const uint64_t* fo, uint32_t n, const DevIndex& ix,
                TopicCount* cnt, const TopicOff* off, uint64_t* handles, uint64_t* base,
                uint32_t* count, hipStream_t s);

}  // namespace mq
