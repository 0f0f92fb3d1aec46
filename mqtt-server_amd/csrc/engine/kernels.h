// Kernel-side structures and launch wrappers of the engine (kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "layout.h"

namespace mq {

constexpr uint32_t kMaxWaveBlocks = 1u << 22;  // grid cap of grid-stride wave-per-item kernels
                                                //   (a grid is limited to 2^32 threads)
constexpr uint32_t kScanBlock = 1024;  // topics per scan block (= chunk granule)
constexpr uint32_t kGatherCap = 64;    // per-topic gather slots written by the count pass
constexpr uint64_t kChunkRows = 0xF0000000ull;  // output rows per chunk (60 GiB of 16-B rows; u32 row indices)
constexpr uint32_t kChunkMin = 2;               // a large batch is cut into at least this many chunks
constexpr uint64_t kChunkRowsMin = 64ull << 20;  // ... unless they would hold fewer rows than this
constexpr uint32_t kChunkTail = 0;               // > 1: last chunk ~ kChunkRows / kChunkTail rows (measured: no gain)
constexpr uint32_t kSubBatchTopics = 1u << 22;  // topics per pipelined sub-batch (Device::match)
constexpr uint64_t kMsgSpecMB = 16384;  // Messages: speculative-count scratch budget (MiB)
constexpr uint32_t kMsgSpecCap = 32768;  // ... and at most this many handles per filter
constexpr uint32_t kMsgWavesPerEU = 6;   // k_msg register budget: 1 (none), 6 or 8 waves per SIMD
constexpr uint64_t kMsgWpeMinRetained = 4000000;  // ... used from this many retained topics on
constexpr uint32_t kCopyTile = 4096;   // rows one k_copy wavefront moves per tile
constexpr uint32_t kCopyBlocksPerCU = 8;   // persistent k_copy: 256-thread workgroups per CU
constexpr uint32_t kMergeBlocksPerCU = 0;  // persistent k_merge beside it (side stream)
constexpr uint32_t kMapSlots = 128;    // per-wave LDS map (gathered merge node -> gather index)
constexpr uint32_t kPairMax = 64;     // merge gathers covered by the pair analysis
constexpr uint32_t kHitMax = 128;      // hit lists staged per k_merge wave
constexpr uint32_t kPartBatch = 2;     // partner links loaded together per record
#ifdef MQ_DEV_BUILD
constexpr bool kDevBuild = true;       // make DEV=1: measurement variants and attribution bits
#else
constexpr bool kDevBuild = false;
#endif
// the set pass's fold (k_merge): per-wave LDS hash table of records (in the node map's place:
// kMapSlots keys and values), at most kFoldCap visits per chunk; a record's value: its meta
// (kSlotOwnMask bits) | what its visits found
constexpr uint32_t kFoldSlots = kMapSlots;
constexpr uint32_t kFoldCap = kFoldSlots * 3 / 4;
constexpr uint32_t kFoldNonBase = 1u << 13;  // a visit's partner comes before the record
constexpr uint32_t kFoldNoLocal = 1u << 14;  // a partner has NoLocal
constexpr uint32_t kFoldQos0 = 1u << 15;     // bit 15 + q: a partner has Qos q
// The set pass's fold of a merge gather too big for the hash fold (merge.hip fold_big): one word per
// visited record, (k + 1) << 5 | kBit*, kBigSlots of them in the map's LDS (keys and values) and
// the merge gathers' three kPairMax arrays, at most kBigFill visits per pass
constexpr uint32_t kBigSlots = 2 * kMapSlots + 3 * kPairMax;
constexpr uint32_t kBigFill = kBigSlots * 3 / 4;
constexpr uint32_t kBitNonBase = 1u, kBitNoLocal = 2u, kBitQos1 = 4u, kBitQos2 = 8u;
constexpr uint32_t kPatchRegions = 1024;  // span format: patch pool regions (one counter each)
// k_merge work counters (MQ_PROF_WORK), kWork per region: pair-table entries loaded, records
// resolved (pair slots read), partner links loaded, patches written
constexpr uint32_t kWork = 30;  // [24] .. [29] (k_set, maxima over the sets): cycles, records, pair-analysis
                                // cycles, resolution cycles, merge gathers, hit lists; [4..7]: set pass phase cycles (map, pair analysis, resolution, whole set);
                                // [8] topics the kernel resolved, [9] bytes of their maps' sources read;
                                // set pass fold: [10] visits folded, [11] visits of merge gathers too big
                                // to fold, [12] those gathers, [13] their may-merge records (n_merge),
                                // [14] records of the folded chunks' gathers, [15] folded chunks;
                                // [16..19] the big gathers by visits (<= 192, <= 384, <= 1024, more),
                                // [20..23] their visits
constexpr uint32_t kMergeWavesPerEU = 8;  // k_merge<spans> register budget: 1 (none), 6 or 8 waves per SIMD

// Device pointers of the resident index image.
struct DevIndex {
  const EdgeSlot* edges;
  uint64_t edge_mask;
  const NodeWalk* walk;
  const NodeLists* lists;
  const NodeInl* inls;  // per node: its inline subscriptions (read under NodeLists kFlagInline)
  const NodeMsg* msg;
  const SegInfo* seginfo;
  const uint8_t* segbytes;
  const SubRec* subs;
  const MergeRef* mref;
  const MergePart* mpart;
  const NodePair* npair;
  const PairEnt* pent;
  const PairSlot* plist;
  const ShrRec* shr;
  const InlRec* inl;
  const ChildRec* children;
  const XInfo* xinfo;  // sharded index only (else null): per node filter id + rank key
  const DeepTail* deep;       // sharded index with deep filters (else null): layout.h DeepTail
  const uint32_t* deep_codes;
  uint64_t deep_mask;         // the table's slots - 1
  uint64_t retained_len;
  uint64_t empty_topic_handle;
  uint32_t empty_topic_live;
  uint32_t pad;
  uint32_t* err;  // [0] error bits (kErr*), [1] gather-slot overflow; checked by the host
};

constexpr uint32_t kErrWalkGuard = 1u;
constexpr uint32_t kErrTableFull = 2u;
constexpr uint32_t kErrPickGuard = 4u;  // k_pick: hash partitions exhausted
constexpr uint32_t kErrDeepRank = 8u;   // sharded merge: a rank tie no DeepTail entry orders (a missing entry)
// one-sync batches (*unsafe bits): the batch must run again with host-sized buffers
constexpr uint32_t kUnsafeSpans = 1u;    // spans / GDesc records past their buffers
constexpr uint32_t kUnsafeDesc = 2u;     // k_merge: a slow-path topic without GDesc records
constexpr uint32_t kUnsafePatches = 4u;  // k_merge: a patch reservation past its region
constexpr uint64_t kWalkGuard = 1ull << 26;

// Exclusive offsets of a topic's outputs (scan of TopicCount).
struct TopicOff {
  uint64_t g, rows, shr, inl, merge;
};

// Same layout as mq_topic_result (include/mqmatch.h).
struct mq_topic_result_dev {
  uint64_t sub_base, shared_base, inline_base;
  uint32_t sub_cap, n_client, n_ident, n_shared, n_inline, reserved;
};

// One gather of a topic, flattened for the load-balanced copy (k_desc writes one per gather in
// compact gather order). Positions are relative to the output chunk and cumulative over its
// gathers: a topic's rows are the concatenation of its gathers' lists, so the position of a
// gather's first row is also its destination, and k_copy finds the gather of an output row by
// a cursor over these records.
struct GDesc {  // 32 B
  uint32_t r_pos;  // client-row stream: rows of the chunk before this gather
  uint32_t r_src;  // subs pool offset of the node's list
  uint32_t s_pos;  // shared rows
  uint32_t s_src;
  uint32_t i_pos;  // inline rows
  uint32_t i_src;
  uint32_t word;   // gather word (node | kGatherSubs | kGatherInline)
  uint32_t mdir;   // n_direct of the node | kDescMerge when its may-merge records are gathered
};
constexpr uint32_t kDescMerge = 1u << 31;
// Span format, sharded index: k_desc folds a merge gather's rank key (XInfo.rank) into the
// GDesc's i_pos (low) / i_src (high) words, which the span format does not otherwise use.

constexpr uint32_t kMaxShards = 16;  // sharded index: shards a batch's exchange can join

// One imported cross-shard list: per-topic offsets (.g) into its entries.
struct XSrc {  // another shard's export: topic t's entries xent[xoff[t], xoff[t + 1])
  const uint32_t* xoff;
  const XEnt* xent;
};
// The imported lists' per-topic offsets: exclusive scans of nf shards' per-topic counts (u32,
// n + 1 each, out[f]) in three launches whatever nf is. bsum / bpre: nf * (nb + 1) words, nb =
// ceil(n / kScanBlock).
struct XScanArgs {
  const uint32_t* in[kMaxShards - 1];
  uint32_t* out[kMaxShards - 1];     // null: the row's total only (bpre[row * (nb + 1) + nb])
  uint32_t stride[kMaxShards - 1];   // element i of row f at in[f][i * stride[f]] (0 or 1: packed)
};
void launch_xscan(const XScanArgs& a, uint32_t nf, uint64_t n, uint32_t* bsum, uint32_t* bpre, hipStream_t s);
// The walk-fused sharded begin's pack: topic t's exported entries from xents[t * g_stride, + xcount[t])
// to ents[xoff[t], ...) (u32 offsets, xoff[n] the total) unless the total passes cap (*unsafe |=
// kUnsafeXEnts); *total = the total; *gt = {the total, *gathers (the batch's gathers, a second
// row of the same batched scan), 0, 0, 0} for k_readback.
void launch_xpack32(uint32_t n, uint32_t g_stride, const uint32_t* xcount, const uint32_t* xoff, const XEnt* xents,
                    XEnt* ents, uint64_t cap, uint32_t* unsafe, unsigned long long* total, const uint32_t* gathers,
                    TopicOff* gt, hipStream_t s);

// Span-format records (include/mqmatch.h mq_span / mq_patch / mq_topic_spans).
struct SpanRec {  // one gathered particle: subs[sub_off, + n_sub), shr[shr_off, + n_shr)
  uint32_t sub_off, n_sub, shr_off, n_shr;
};
struct PatchRec {  // topic-relative record row -> replacement meta (merge base / ident / drop)
  uint32_t row, meta;
};
struct TopicSpansDev {  // == mq_topic_spans
  uint64_t span_base, patch_base, inline_base, picked_base;
  uint32_t n_spans, n_patches, n_inline, n_rows;
  uint32_t n_client, n_ident, n_shared, flags;  // flags: MQ_TOPIC_SET_PATCHES
};
static_assert(sizeof(TopicSpansDev) == 64, "mq_topic_spans layout");

// Per-chunk arguments of k_desc / k_copy / k_merge. In the span format (k_merge<true>) the
// whole batch is one chunk, GDesc row positions are topic-relative and k_merge emits patches.
struct EmitArgs {
  DevIndex ix;
  uint32_t t0, t1;          // topic range of this chunk
  const TopicOff* off;      // per-topic offsets (n + 1)
  TopicOff base;            // off[t0]: the chunk's output buffers start here
  GDesc* desc;              // indexed by absolute gather index
  const uint32_t* tiles;    // k_copy tile -> first gather: [client | shared | inline] tiles
  uint32_t n_tiles[3];      // tiles per stream
  uint32_t total[3];        // rows per stream in this chunk
  SubRec* rows;
  ShrRec* shr_rows;
  InlRec* inl_rows;
  mq_topic_result_dev* res; // indexed t - t0 (row format)
  // span format
  TopicSpansDev* sres;            // indexed t
  PatchRec* patches;              // patch pool: kPatchRegions regions of rcap patches; topic t
  unsigned long long* pcount;     //   reserves in region t % kPatchRegions with atomicAdd on
  uint64_t rcap;                  //   pcount[region] (may exceed rcap: the host grows the pool)
  unsigned long long* work;       // MQ_PROF_WORK: per region kWork counters (null: off)
  uint32_t* set_rec;              // MQ_PROF_WORK, set pass: records each representative resolved
  // sharded index: the other shards' exported cross-shard nodes of every topic (k_xlist), a
  // device table (a kernel-argument array indexed at run time would go through scratch)
  uint32_t n_xf;
  const struct XSrc* xsrc;
  // span format, walk without lists: per-topic counts from k_desc (rows, shared, merge; no inline
  // rows) in place of the offsets' differences
  const TopicCount* tc;
  // span format, merge-set dedup (rep == null: off). dd_phase 1: each set representative resolves
  // its merge gathers once into set-relative patches (row = x << kSetRowBits | k: record k of
  // its x-th merge gather's list) in the set pool, and its SetInfo; dd_phase 2: every deduped
  // topic copies its representative's patches, translating x to its own rows.
  const uint32_t* rep;
  const uint32_t* tslot;
  const uint32_t* mcount;  // merge gathers per topic, and the rows of their lists (k_desc, stride kPairMax)
  const uint32_t* mrow;
  const uint32_t* mlist;   // dedup: their particles and pair-block headers (k_desc, stride kPairMax):
  const uint2* mpair;      //   the map is built from these (topics with <= kPairMax merge gathers)
  uint32_t dd_phase;
  struct SetInfo* sets;
  PatchRec* spatches;
  unsigned long long* spcount;
  uint64_t srcap;
  uint32_t set_ref;                    // dd_phase 2: a deduped topic references its set's patches
                                       //   (device results) instead of copying them
  const uint32_t* rep_list;            // dd_phase 1: the set representatives (k_dedup_rep,
  const unsigned long long* n_reps;    //   DedupArgs layout) and their two counts, in device memory
  const uint32_t* wave_list;           // dd_phase 2 after k_finish: the topics that still need a
  const unsigned long long* n_wave;    //   wavefront (k_finish wrote the others' results)
  const uint64_t* mrank;               // sharded index: the merge gathers' rank keys (DescArgs)
  // one-sync batches: GDesc capacity (records); a topic whose slow path would read past it, or
  // whose patch reservation does not fit its region, sets *unsafe (bit 2 / bit 4) instead
  uint64_t desc_cap;
  uint32_t* unsafe;
  uint32_t g_stride;  // != 0: topic t's gathers at [t * g_stride, + tc[t].gathers) (DescArgs.g_stride)
  uint32_t exp;       // MQ_OPT_SET_EXP bits (set pass attribution; 0 in the product)
};
constexpr uint32_t kSetHeavy = 1024;  // a merge set with this many may-merge records goes first
constexpr uint32_t kSetRowBits = 26;  // set-relative patch rows: 6 bits of merge gather, 26 of slot
constexpr uint32_t kCodeSetRowBits = 23;  // == MQ_CODE_SET_ROW_BITS (host patch codes)
constexpr uint32_t kTopicSetPatches = 1;  // TopicSpansDev.flags: patches shared with a merge set
                                          //   (MQ_TOPIC_SET_PATCHES)
struct SetInfo {  // 24 B, per representative topic
  uint64_t base;   // its patches in the set pool
  uint32_t n, nonbase, ext, fit;
};

// Output chunk of a batch as k_desc sees it: where its rows start and where its k_copy tile
// table sits in the batch's tile array.
struct ChunkPlan {  // 32 B
  uint64_t rows, shr, inl;  // off[first topic of the chunk]
  uint32_t tile_off;        // its tiles: [client | shared | inline] from tiles + tile_off
  uint32_t n_tiles0, n_tiles1, pad;
};

// One k_desc launch over every topic of the batch.
struct DescArgs {
  DevIndex ix;
  uint32_t n;
  uint32_t gather_stride;
  const TopicOff* off;
  const uint32_t* gathers;
  const uint32_t* chunk_of_block;  // scan block -> chunk
  const ChunkPlan* plan;
  GDesc* desc;
  uint32_t* tiles;
  // span format: one SpanRec per gather, inline rows copied to inl_out at off[t].inl
  SpanRec* spans;
  InlRec* inl_out;
  TopicCount* tc_out;  // span format, walk without lists: per-topic rows / shared / merge counts
  // span format, merge-set dedup (null: off): per topic, the signature of its merge gathers'
  // particles (in gather order), their number, and the list itself (stride kPairMax)
  uint64_t* msig;
  uint32_t* mcount;
  uint32_t* mlist;
  uint32_t* mrow;  // the topic-relative row of each merge gather's first may-merge slot (stride kPairMax)
  uint2* mpair;    // its pair-block header (NodePair ent_off, ent_mask; stride kPairMax). With these
                   // lists k_merge maps a topic's merge gathers without GDesc records, which are
                   // then written only for a topic with more than kPairMax merge gathers
  uint64_t* mrank; // sharded index: each merge gather's DFS rank key (XInfo.rank; stride kPairMax)
  // sharded index, the export in k_desc (null: k_xlist exports): topic t's gathered cross-shard
  // nodes (gathered subscriptions at a node with a foreign partner, kFlagXNode) at its spans' own
  // positions (xents[g0, + xcount[t]): never more than its gathers), packed by k_xpack
  XEnt* xents;
  uint32_t* xcount;
  uint32_t* gw_out;  // sharded, walk-fused: every gather word at its span's position (k_xsig's GDesc
                     //   records for k_merge's linear paths are made from them)
  // MQ_OPT_WALK_EXP bit 0 (development builds, an attribution of the walk's level-0 probes):
  // topic t's root child (child, '+', '#') looked up before the walk by k_root_hint; bit 1 (round
  // 6) levels 0 and 1: root_hint[3t] the root child, [3t + 1] its literal child of segment 1,
  // [3t + 2] the root's '+' child's literal child of segment 1 (the two level-1 probes)
  const uint4* root_hint;
  uint32_t hint_levels;
  // one-sync batches (Device, MQ_OPT_ONE_SYNC): the capacities of spans / desc in records; a topic
  // that would write past them writes nothing and sets bit 1 of *unsafe (the batch is run again
  // with host-sized buffers). unsafe == null: sized by the host (no checks).
  uint64_t spans_cap, desc_cap;
  uint32_t* unsafe;
  // g_stride != 0 (the walk-fused desc of one-sync batches): topic t's spans and GDesc records sit
  // at [t * g_stride, + its gathers) instead of at off[t].g (no scan: off is unused), and
  // tc_out[t].gathers is its number of gathers. list != null: only the topics list[0, *n_list)
  // (the frontier walk's fallback topics), grid-stride.
  uint32_t g_stride;
  const uint32_t* list;
  const uint32_t* n_list;
  const TopicCount* g_count;  // list mode: the listed topics' gathers (their walk's counts)
  // k_dedup_insert folded in (dd_keys != null; DedupArgs' table): each topic with 1..kPairMax
  // merge gathers inserts its signature and gets its slot (dd_tslot; kNone: not deduped)
  unsigned long long* dd_keys;
  uint32_t* dd_vals;
  uint64_t dd_mask;
  uint32_t* dd_tslot;
};

// Merge-set dedup (span format): topics whose merge gathers are the same particles resolve to
// the same patches (up to row positions). k_dedup finds, per topic, a representative topic with
// the same merge gathers (exact: the lists are compared) — rep[t] == t for a topic that resolves
// itself. Table: 2^k slots of (u64 signature, u32 the topic that inserted it); n_sets counts the
// representatives.
struct DedupArgs {
  uint32_t n;
  const uint64_t* msig;
  const uint32_t* mcount;
  const uint32_t* mlist;
  unsigned long long* keys;  // table_mask + 1 signatures (0 = empty)
  uint32_t* vals;            // table_mask + 1 inserting topics (valid where keys != 0)
  uint64_t table_mask;
  uint32_t* tslot;           // per topic: its table slot (kNone: not deduped)
  uint32_t* rep;             // per topic: its representative
  unsigned long long* n_sets;  // [2]: representatives listed from the front (heavy) and the back;
                               //   [2]: the batch's gathers (sum of tc[t].gathers; tc != null)
  uint32_t* rep_list;          // those topics: heavy sets at [0, n_sets[0]), the others at
                               //   [n - n_sets[1], n) (heavy first: the set pass's tail is short)
  const TopicCount* tc;        // per-topic counts (k_desc; null: the offsets' differences): a set
  const struct TopicOff* off;  //   is heavy with >= heavy may-merge records
  uint32_t heavy;
  // sharded index (null / 0 otherwise): a merge set is also the same cross-shard entries of the
  // other shards (compared list by list); fcount[t]: their number (a topic whose local merge
  // gathers and foreign entries exceed k_merge's map is not deduped)
  const uint32_t* fcount;
  uint32_t n_xf;
  const struct XSrc* xsrc;
};
// insert = false: the signatures were inserted by the walk-fused desc (DescArgs.dd_keys)
void launch_dedup(const DedupArgs& a, hipStream_t s, bool insert = true);

// Sharded index, after the exchange (k_xsig): per topic, fold the imported cross-shard entries
// into the merge-set signature (msig) and count them (fcount); a topic whose map would overflow
// (local merge gathers + foreign entries >= kMapSlots) gets the GDesc records of k_merge's slow
// path (with rank keys), which k_desc_g16 wrote only for topics with > kPairMax merge gathers.
struct XSigArgs {
  DevIndex ix;
  uint32_t n;
  uint32_t n_xf;
  const struct XSrc* xsrc;
  uint64_t* msig;
  const uint32_t* mcount;
  uint32_t* fcount;
  const struct TopicOff* off;
  const uint32_t* gathers;
  uint32_t gather_stride;
  struct GDesc* desc;
  uint32_t g_stride;                // the walk-fused layout: topic t's gathers at t * g_stride, their
  const struct TopicCount* tc;      //   number tc[t].gathers (off unused)
  // non-null: k_dedup_insert's work too, on the finished signatures (DedupArgs keys / vals /
  // table_mask / tslot), so the dedup runs k_dedup_rep alone
  unsigned long long* dd_keys;
  uint32_t* dd_vals;
  uint64_t dd_mask;
  uint32_t* dd_tslot;
};
void launch_xsig(const XSigArgs& a, hipStream_t s);
// The merge set pass of an index that is not sharded (sets.hip): k_merge<spans, SET>'s results with
// only the set pass's code; a.rep_list / a.n_reps / a.sets / a.spatches as k_merge's dd_phase 1.
void launch_set(const EmitArgs& a, uint32_t blocks, hipStream_t s);

// Batched auth.MatchTopic (k_acl).
struct AclArgs {
  const uint8_t* filter_bytes;
  const uint64_t* filter_offs;
  const uint8_t* topic_bytes;
  const uint64_t* topic_offs;
  const uint32_t* pair_filter;
  const uint32_t* pair_topic;
  const uint64_t* elem_base;  // per pair: first (start, len) slot in elems
  uint64_t n_pairs;
  uint8_t* matched;
  uint32_t* n_elems;
  uint32_t* elems;
};
void launch_acl(const AclArgs& a, hipStream_t s);

// SelectShared on the device (k_pick): per topic, one member of every shared filter.
struct PickArgs {
  const mq_topic_result_dev* res;  // row format: n topic results (shared_base / n_shared read)
  const ShrRec* rows;              // the chunk's shared rows
  const TopicSpansDev* sres;       // span format: topics (span_base / n_spans / picked_base)
  const SpanRec* spans;            //   their spans, whose shared ranges index
  const ShrRec* pool;              //   the shared pool
  ShrRec* sel;                     // picked rows of topic t at [shared_base, + picked)
  uint32_t* n_out;                 // picked count of topic t at n_out[t * n_out_stride]
  uint32_t n_out_stride;
  uint32_t n;
  uint32_t* err;                   // kErrPickGuard
};
void launch_pick(const PickArgs& a, hipStream_t s);  // a.sres != null: span format

// lists = true: the count pass reads every gathered particle's lists and counts its rows, shared
// and inline members (the row format, and span batches with inline subscriptions or a device
// share pick); false: it counts gathers only and k_desc<true> counts the rest (DescArgs.tc_out).
// wpe: the count pass's register budget (8: eight waves per SIMD, with spills; else unconstrained).
// clamp (count pass): a topic's gather count is stored as at most kGatherCap (its slot), so the
// batch's offsets stay within n * kGatherCap; the overflow flag still says that one had more.
void launch_walk(bool fill, bool lists, uint32_t wpe, const uint8_t* tb, const uint64_t* to, uint32_t n,
                 const DevIndex& ix, TopicCount* cnt, const TopicOff* off, uint32_t* gathers, uint32_t* ovf,
                 hipStream_t s, bool clamp = false);
// The frontier walk (k_walkf, `group` lanes per topic: 4, 8 or 16), count pass: the same counts
// and gather slots as launch_walk(false, ...). Topics it cannot hold are listed in fb_list
// (*fb_count, zeroed by the caller) and walked by k_walk in fb_blocks persistent workgroups.
void launch_walk_front(uint32_t group, bool lists, uint32_t wpe, const uint8_t* tb, const uint64_t* to, uint32_t n,
                       const DevIndex& ix, TopicCount* cnt, uint32_t* gathers, uint32_t* ovf, uint32_t* fb_list,
                       uint32_t* fb_count, uint32_t fb_blocks, hipStream_t s, bool clamp = false);
// The frontier walk with k_desc fused into its epilogue (span format, dedup lists, no inline rows
// or share pick, one-sync batches): each topic's gathers go straight from LDS to its spans and
// merge lists at t * kGatherCap (da.g_stride); the fallback topics' k_walk and k_desc_g16 (list
// mode) follow. No scan: da.tc_out holds the per-topic counts.
void launch_walk_desc(uint32_t group, uint32_t wpe, const uint8_t* tb, const uint64_t* to, uint32_t n, const DevIndex& ix,
                      TopicCount* cnt, uint32_t* gathers, uint32_t* ovf, uint32_t* fb_list, uint32_t* fb_count,
                      uint32_t fb_blocks, const DescArgs& da, hipStream_t s);
void launch_scan(const TopicCount* cnt, uint32_t n, TopicOff* bsum, TopicOff* bpre, TopicOff* off,
                 hipStream_t s);
void launch_desc(const DescArgs& a, bool spans, hipStream_t s);
void launch_root_hint(const uint8_t* tb, const uint64_t* to, uint32_t n, const DevIndex& ix, uint4* out, uint32_t levels,
                      hipStream_t s);
void launch_copy(const EmitArgs& a, uint32_t max_blocks, hipStream_t s);
void launch_merge(const EmitArgs& a, bool spans, uint32_t wpe, uint32_t max_blocks, hipStream_t s);

// k_finish (span format, merge-set dedup, device results): thread per topic, after the set pass.
// A topic whose result needs no wavefront — no inline rows, and no may-merge records or a merge
// set (it references the set's patches) — gets its result record here; the others are listed
// for k_merge's topic pass.
struct FinishArgs {
  uint32_t n;
  const TopicOff* off;
  const TopicCount* tc;  // per-topic counts (k_desc), or null: the offsets' differences
  const uint32_t* tslot;
  const uint32_t* rep;
  const SetInfo* sets;
  TopicSpansDev* sres;
  uint32_t* wave_list;
  unsigned long long* n_wave;
  uint32_t g_stride;  // != 0: topic t's spans at t * g_stride (DescArgs.g_stride)
};
void launch_finish(const FinishArgs& a, hipStream_t s);
// Host span results: pack the merge rows of the topics with a merge set (tslot != kNone),
// mcount[t] of them from mrow[t * kPairMax]; base[t] their start, *total (zeroed) the count.
void launch_span_pack(uint32_t n, TopicSpansDev* sres, const SpanRec* src, SpanRec* dst, unsigned long long* total,
                      hipStream_t s);
void launch_mrow_pack(uint32_t n, const uint32_t* tslot, const uint32_t* mcount, const uint32_t* mrow,
                      uint32_t* base, uint32_t* rows, unsigned long long* total, hipStream_t s);
// Host span results: the sets' written patches packed (nbase[rep], *total zeroed) as PatchRecs
// (out) or patch codes (codes != null: MQ_SPANS_PATCH_CODES), and every topic's patch_base
// pointed into the packed arrays (its set's, or its own via the regions' roff).
void launch_set_pack(uint32_t n, const uint32_t* tslot, const uint32_t* rep, const SetInfo* sets,
                     const PatchRec* pool, uint64_t* nbase, PatchRec* out, uint32_t* codes, unsigned long long* total,
                     hipStream_t s);
void launch_host_rebase(uint32_t n, const uint32_t* rep, const uint64_t* nbase, const uint64_t* roff, uint64_t rcap,
                        TopicSpansDev* sres, hipStream_t s);
// k_msg count (fill = false) or fill pass. spec != null: the count pass also writes each filter's
// first spec_cap handles to spec[t * spec_cap ...] and flags (TopicCount.gathers) the filters the
// fill pass must still walk; the fill pass then walks only those.
void launch_msg(bool fill, const uint8_t* fb, const uint64_t* fo, uint32_t n, const DevIndex& ix,
                TopicCount* cnt, const TopicOff* off, uint64_t* handles, uint64_t* base,
                uint32_t* count, uint64_t* spec, uint32_t spec_cap, uint32_t wpe, hipStream_t s);
// Sharded index: the topics' gathered cross-shard nodes (kFlagXNode, subscriptions gathered).
// count = true: TopicCount.gathers = their number per topic; else written as XEnt at
// off[t].g with their number in counts[t] (the exported list, mq_xlist).
// The export written by k_desc (DescArgs.xents), packed: k_counts + scan of xcount give xoff; each
// topic's entries move from xents[off[t].g, ...) to ents[xoff[t].g, ...) unless the packed total
// passes cap (then *unsafe |= kUnsafeXEnts, nothing is written); total[0] = the packed total.
constexpr uint32_t kUnsafeXEnts = 16u;
void launch_xpack(uint32_t n, const TopicOff* off, uint32_t g_stride, const uint32_t* xcount, const TopicOff* xoff,
                  const TopicOff* xtot, const XEnt* xents, XEnt* ents, uint64_t cap, uint32_t* unsafe,
                  unsigned long long* total, hipStream_t s);
// cnt[t] = {xcount[t], tc[t].gathers, 0, 0, 0}: scanned, the export's offsets and (in .rows) the
// batch's gathers (the walk-fused layout has no scan of its own)
void launch_xcounts(const uint32_t* xcount, const TopicCount* tc, uint32_t n, TopicCount* cnt, hipStream_t s);
void launch_xlist(bool count, const DevIndex& ix, uint32_t n, const TopicOff* off, const uint32_t* gathers,
                  uint32_t gather_stride, TopicCount* cnt, const TopicOff* xoff, XEnt* ents, uint32_t* counts,
                  hipStream_t s);
// TopicCount.gathers = counts[t] (an imported list's counts, for launch_scan)
void launch_counts(const uint32_t* counts, uint32_t n, TopicCount* cnt, hipStream_t s);
// Pack the used prefix of every patch region (pcount[r] patches of region r) into `out` at
// roff[r] (span format, host results), or as patch codes into `codes` when it is not null.
void launch_patch_compact(const PatchRec* pool, uint64_t rcap, const unsigned long long* pcount,
                          const uint64_t* roff, PatchRec* out, uint32_t* codes, hipStream_t s);
void launch_msg_place(uint32_t n, const TopicCount* cnt, const TopicOff* off, const uint64_t* spec,
                      uint32_t spec_cap, uint64_t* handles, uint64_t* base, uint32_t* count, hipStream_t s);

// Incremental upload of the index image (Device::sync): dirty runs of the host mirrors, packed
// into one staging buffer (one H2D), copied into place on the device.
struct ScatterRun {
  uint64_t dst;    // device address
  uint64_t src;    // offset in the staging buffer (src % 16 == dst % 16)
  uint64_t bytes;  // <= kScatterRun
};
constexpr uint64_t kScatterRun = 64 << 10;
void launch_scatter(const ScatterRun* runs, uint32_t n, const uint8_t* stage, hipStream_t s);

// ---------------------------------------------------------------------------------------------
// Messages over the level-order retained image. The image holds the particles
// with a live retained message at or below them, level by level, each particle's image children
// consecutive and in its parent's order (the root's "$SYS" child last), so that
//   - the image children of a consecutive run [a, b) of one level are the consecutive run
//     [cl[a].x, cl[b - 1].y) of the next level;
//   - the live handles of a run are the consecutive run [lp[a], lp[b]) of h.
// A '+' level of a filter maps a run to a run, a final '+' or '#' emits whole runs of h; only a
// literal level below a wildcard fans out into lookups.
// The retained image's own edge table: (parent image position, segment key) -> child image
// position, for the image's particles only (a child with no live retained message at or below it
// has no entry). A literal lookup in the Messages walk is then one probe, where the index's edge
// table needs the probe, then the particle's image position and its check (two more random loads).
struct ImgEdge {  // 32 B, two per 64 B line; parent kImgEdgeEmpty: free
  uint32_t parent, child;
  uint64_t k0, k1, pad;
};
constexpr uint32_t kImgEdgeEmpty = 0xFFFFFFFFu;
struct KxSlot {  // the key index's table: key hash (0: free) -> entries [start, start + count)
  uint64_t h;
  uint32_t start, count;
};
// a literal level with at most this many rounds of particle probes (64 a round) probes them one by
// one without trying the key index (its table probe and two wave-wide searches come first)
constexpr uint32_t kKxMinRounds = 6;  // (r06/ac: 6 against 12, 10M 143.5-144.1 -> 146.2M, 100M 85.8 -> 87.9M filters/s)
MQ_HD uint64_t kx_hash(uint64_t k0, uint64_t k1) { return mix64(k0 ^ mix64(k1 + 0x9e3779b97f4a7c15ull)) | 1ull; }
// Key index build (Device::ensure_img): collect the image edges, sort them, fill the table.
void launch_kx_collect(const DevIndex& ix, const uint32_t* node, const uint32_t* pos, uint32_t n, uint32_t n_pos,
                       uint32_t* par, uint32_t* chd, uint64_t* k0, uint64_t* k1, uint64_t* h, uint32_t* perm,
                       unsigned long long* count, hipStream_t s);
// hipcub radix sorts (stable): temp == null returns the temp bytes needed
size_t kx_sort_u32(void* temp, size_t temp_bytes, const uint32_t* kin, uint32_t* kout, const uint32_t* vin,
                   uint32_t* vout, uint32_t n, hipStream_t s);
size_t kx_sort_u64(void* temp, size_t temp_bytes, const uint64_t* kin, uint64_t* kout, const uint32_t* vin,
                   uint32_t* vout, uint32_t n, hipStream_t s);
void launch_kx_gather32(const uint32_t* src, const uint32_t* perm, uint32_t* dst, uint32_t n, hipStream_t s);
void launch_kx_gather64(const uint64_t* src, const uint32_t* perm, uint64_t* dst, uint32_t n, hipStream_t s);
void launch_kx_count_keys(const uint64_t* h, uint32_t n, unsigned long long* keys, hipStream_t s);
void launch_kx_table(const uint64_t* h, uint32_t n, KxSlot* tab, uint64_t mask, uint32_t* err, hipStream_t s);
struct MsgImg {
  const uint32_t* node;  // image position -> particle
  const uint32_t* pos;   // particle -> image position (valid iff node[pos[p]] == p; n_pos entries)
  const uint2* cl;       // image position -> [x, y) image positions of its image children
  const uint32_t* lp;    // image position -> live particles before it in the image (n + 1)
  const uint64_t* h;     // live handles in image order
  const ImgEdge* edges;  // the image's edge table (null: look up through the index's, MQ_OPT_MSG_EDGES 0)
  uint64_t edge_mask;
  const uint32_t* gate;  // the fill passes run only while *gate != 0 (one-sync batches; null: always)
  uint32_t n, n_pos;
  // MQ_PROF_WORK (null: off): the count pass's clocks per filter (shader clocks >> 4, saturated)
  // and work counters: [0] fan-out lookups (particles probed level by level), [1] filters whose
  // frontier outgrew LDS (per-lane walk), [2] particles those walked per lane
  uint32_t* cyc;
  unsigned long long* work;
  // The image's key index (round 6; null: none): every image edge (parent position, key) ->
  // child position, sorted by (key hash, parent position) — kx_par / kx_chd / kx_k0 / kx_k1 — and a
  // table key hash -> its entries' range (kx_tab, kx_mask + 1 slots). A literal segment under runs
  // of particles is then one table probe and two binary searches per run (the children with that
  // key whose parent lies in the run), not one edge-table probe per particle of the runs.
  const struct KxSlot* kx_tab;
  uint64_t kx_mask;
  uint32_t kx_min_rounds;  // kKxMinRounds, or MQ_OPT_MSG_KEYIDX's value
  const uint32_t* kx_par;
  const uint32_t* kx_chd;
  const uint64_t* kx_k0;
  const uint64_t* kx_k1;
  // Runs at the boundary (mq_messages_runs_*, round 6): every run the walk finds is one MsgPiece
  // (== mq_msg_run) and nothing is copied; the fill passes also write each filter's first run and
  // run count (null: handles, as before)
  uint64_t* run_base;
  uint32_t* run_cnt;
};
// A run of h copied to the output: out[dst + k] = h[h0 + k], k < len. (Runs at the boundary: the
// result's mq_msg_run, include/mqmatch.h: first, count, at.)
struct MsgPiece {
  uint32_t h0, len;
  uint64_t dst;
};
// runs at the boundary for a batch the particle walk answered: filter t's handles as one run
void launch_msg_runs_of(uint32_t n, const uint64_t* base, const uint32_t* count, MsgPiece* runs, uint64_t* run_base,
                        uint32_t* run_cnt, hipStream_t s);
constexpr uint32_t kMsgPiece = 4096;    // handles per copy piece (a wavefront's work item)
constexpr uint32_t kMsgDirect = 8;      // runs this short are copied by the walk itself
constexpr uint32_t kMsgStack = 16;      // nested fan-outs a lane can hold (deeper: kErrMsgNest)
constexpr uint32_t kMsgFront = 256;     // k_msgq fan-out frontier: runs per level a wavefront holds in LDS
constexpr uint32_t kErrMsgNest = 16u;   // k_msgq: fan-out nesting beyond kMsgStack (walk k_msg)

// u32 exclusive scan: out[i] = in[0] + ... + in[i - 1], out[n] = total (out may be in).
// bsum / bpre: ceil(n / kScanBlock) + 1 entries each.
void launch_scan32(const uint32_t* in, uint64_t n, uint32_t* bsum, uint32_t* bpre, uint32_t* out,
                   hipStream_t s);
// Image build, one level: the image children of the level's positions [lo, lo + n).
// fill = false: cnt[p] = their number; fill = true (coff = scan of cnt): written from `next` on.
struct ImgLevelArgs {
  uint32_t* node;
  uint32_t* pos;
  uint2* cl;
  uint32_t* live;  // per image position: 1 if the particle's retained message is live
  uint32_t* cnt;
  const uint32_t* coff;
  uint32_t lo, n, next;
};
// the image's edge table (ImgEdge, mask + 1 slots, all free) from the index's edges between image
// particles (node / pos: the image, n positions, n_pos particle slots)
void launch_img_edges(const DevIndex& ix, const uint32_t* node, const uint32_t* pos, uint32_t n, uint32_t n_pos,
                      ImgEdge* edges, uint64_t mask, hipStream_t s);
void launch_img_root(uint32_t* node, uint32_t* pos, uint32_t* live, hipStream_t s);
void launch_img_level(bool fill, const DevIndex& ix, const ImgLevelArgs& a, hipStream_t s);
// h[lp[q]] = handle of node[q] for the live positions (lp: the scan of live)
void launch_img_compact(const DevIndex& ix, const uint32_t* node, const uint32_t* lp, uint32_t n,
                        uint64_t* h, hipStream_t s);
// A filter's output run as its walk found it (k_msgq run mode): handles h[h0, + len) go to the
// filter's output at dst; a long run's pieces start at the filter's piece slot pslot.
struct MsgRun {
  uint32_t h0, len, dst, pslot;
};
constexpr uint32_t kMsgRunCap = 256;  // runs recorded per filter (more: the filter is walked again)
// Messages passes (k_msgq):
//   kMsgCount  TopicCount.gathers = pieces, .rows = handles
//   kMsgFill   pieces at off[t].g, short runs copied directly, base / count written
//   kMsgRuns   as kMsgCount, and the filter's runs recorded (runs[t * run_cap ..], n_runs[t];
//              kNone: more than run_cap runs)
//   kMsgPlace  as kMsgFill, from the recorded runs without walking (a filter without them walks)
//   kMsgWideCount / kMsgWideFill  the work items a kMsgRuns pass exported (MsgWide): a wavefront
//              per item walks its particles lane by lane; the count records the item's runs (in
//              its wavefront's scratch) and adds its handles and pieces to its filter's counts (one
//              atomic each on cnt[t], after the count pass), which gives where they start; the fill
//              places the recorded runs from there (an item whose runs did not fit walks again)
enum MsgMode : int { kMsgCount = 0, kMsgFill = 1, kMsgRuns = 2, kMsgPlace = 3, kMsgWideCount = 4, kMsgWideFill = 5 };
// Wide filters (a literal segment under a fan-out of more than min_tot particles): the count
// pass (kMsgRuns) exports the fan-out's runs as work items of at most kMsgChunk particles and
// stops walking the filter (cnt[t].shared = 1 marks it; a kMsgFill walk of the filter stops at the
// same place), so one heavy filter spreads over the grid instead of holding one wavefront while
// the rest of the batch has long finished (10M retained: the heaviest filter took 1.8 ms of a
// 3.2 ms count pass).
struct MsgWork {  // filter t: particles [x, y) of a fan-out, to take the filter from byte s on
  uint32_t t, x, y, s;
  // the count's answers: where the item's handles and pieces start in its filter's output, and its
  // runs recorded in the scratch (run_off, n_runs; kNone: they did not fit, the fill walks again)
  uint32_t dst, pslot, run_off, n_runs;
};
struct MsgWide {
  MsgWork* items;
  uint32_t cap, min_tot;  // min_tot 0: no export
  uint32_t min_hits;      // ... a level through the key index: more than min_hits candidate entries
  uint32_t* n_items;      // items reserved (a reservation past cap fails: that filter walks alone)
  MsgRun* scratch;        // the counting wavefronts' recorded runs: wavefront w's at [w * per_wave, ...)
  uint32_t per_wave;
};
// a literal level through the key index exports more than this many candidate entries (its items
// look up entries, not particles; 10M retained: 512 -> 128, 83.4M -> 127.8M filters/s, r06/p)
constexpr uint32_t kMsgExportMinHits = 128;
#ifndef MQ_MSG_CHUNK
#define MQ_MSG_CHUNK 256
#endif
constexpr uint32_t kMsgChunk = MQ_MSG_CHUNK;  // particles per exported work item (or key-index entries)
constexpr uint32_t kMsgWorkEntries = 1u << 31;  // MsgWork.s: the item's [x, y) is a range of key-index entries
static_assert(kMsgChunk <= 256, "an entry item's hits must fit the fan-out frontier (kMsgFront)");
constexpr uint32_t kMsgWorkCap = 1u << 20;  // work items per batch (32 MB)
constexpr uint32_t kMsgWideRuns = 4096;     // recorded runs per wide-count wavefront (64 KB each)
constexpr uint32_t kMsgExportMin = 512;   // export a literal level under a fan-out of more particles (10M: 2048 -> 512, 2.75 -> 2.50 ms)
void launch_msgq(int mode, const uint8_t* fb, const uint64_t* fo, uint32_t n, const DevIndex& ix,
                 const MsgImg& img, TopicCount* cnt, const TopicOff* off, MsgPiece* pieces,
                 uint64_t* handles, uint64_t* base, uint32_t* count, MsgRun* runs, uint32_t run_cap,
                 uint32_t* n_runs, const MsgWide& w, uint32_t wide_blocks, hipStream_t s);
// One-sync span batches: every counter the batch's kernels accumulate into is zeroed by one
// launch at its start (small arrays by block 0, `big` grid-stride), and what the host reads at its
// end is gathered by one thread into the pinned FastBack record (no fill or copy commands on the
// stream: each cost a few microseconds of its own).
struct ResetArgs {
  void* p[8];
  uint32_t bytes[8];  // multiples of 4
  uint32_t n;
  unsigned long long* big;
  uint64_t big_words;
};
void launch_reset(const ResetArgs& a, hipStream_t s);
struct FastBackRec {  // == Device::FastBack
  TopicOff tot;
  uint32_t ovf, fallback, unsafe, err;
  unsigned long long n_sets[3];
  // host results: the topic pass's patches (all regions), the packed set patches and merge rows
  unsigned long long n_patches, set_total, mrow_total;
};
// k_readback: every count the host reads at a one-sync batch's end, written by a kernel straight
// into pinned host memory — no small device-to-host copies, which would queue on the DMA engine
// behind the previous pipelined batch's result copy and hold this batch's synchronisation.
struct ReadbackArgs {
  const TopicOff* tot;  // null: not read (the walk-fused desc has no scan)
  const uint32_t *ovf, *fallback, *unsafe, *err;
  const unsigned long long* n_sets;  // null: not read
  // host results (null: not read): the topic pass's per-region patch counts, whose exclusive
  // prefix (kPatchRegions + 1 entries) goes to roff in device memory; the packed totals
  const unsigned long long* pcount;
  uint64_t* roff;
  const unsigned long long *set_total, *mrow_total;
  FastBackRec* out;                  // device view of the pinned record
};
void launch_readback(const ReadbackArgs& a, hipStream_t s);
void launch_msg_copy(const MsgPiece* pieces, uint64_t n, const uint64_t* h, uint64_t* out, hipStream_t s);
// One-sync Messages batches: the output buffers are sized by earlier batches. k_msg_gate compares
// the batch's totals (the scan's last entry, on the device) with their capacities and opens the
// fill passes (gate[0] = 1) and the copy (*n_pieces = the piece count) only if they fit; the copy
// then runs a grid for up to cap_g pieces and reads its count from the device.
void launch_msg_gate(const TopicOff* tot, uint64_t cap_rows, uint64_t cap_g, uint32_t* gate, uint64_t* n_pieces,
                     hipStream_t s);
void launch_msg_copy_dev(const MsgPiece* pieces, const uint64_t* n_pieces, uint64_t cap_g, const uint64_t* h,
                         uint64_t* out, hipStream_t s);

}  // namespace mq
