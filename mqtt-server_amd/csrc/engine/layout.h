// Device-image layout shared by the host index builder (index.cpp) and the gfx950 kernels
// (kernels.hip). Every array here lives resident in HBM and is mirrored on the host, which
// applies updates and uploads only the dirty pages.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define MQ_HD __host__ __device__ __forceinline__
#else
#define MQ_HD inline
#endif

namespace mq {

constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kRoot = 0;

// ---- segment keys -------------------------------------------------------------------------
// A topic level ("segment") is keyed by 16 bytes. Segments of <= 15 bytes are stored inline
// (bytes little-endian, length in the top byte of k1): exact and collision-free. Longer
// segments carry two independent 64-bit hashes with 0xFF in the top byte of k1; a hit on
// such a key is verified byte-for-byte against the segment pool, so matching stays exact.
struct SegKey {
  uint64_t k0, k1;
};

constexpr uint32_t kInlineSegMax = 15;
constexpr uint64_t kLongMarker = 0xFFull << 56;

MQ_HD uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}

constexpr uint64_t kFnvOffset = 0xcbf29ce484222325ull, kFnvPrime = 0x100000001b3ull;
constexpr uint64_t kHashB0 = 0x84222325cbf29ce4ull, kGolden = 0x9e3779b97f4a7c15ull;

// Incremental form, so the device computes the key in the same pass that finds the '/'.
struct SegKeyBuilder {
  uint64_t k0 = 0, k1 = 0, a = kFnvOffset, b = kHashB0;
  uint32_t len = 0;
  MQ_HD void push(uint32_t c) {
    if (len < 8) k0 |= (uint64_t)c << (8 * len);
    else if (len < kInlineSegMax) k1 |= (uint64_t)c << (8 * (len - 8));
    a = (a ^ c) * kFnvPrime;
    b = (b + c + 1) * kGolden;
    b ^= b >> 29;
    len++;
  }
  MQ_HD SegKey finish() const {
    if (len <= kInlineSegMax) return SegKey{k0, k1 | ((uint64_t)len << 56)};
    return SegKey{mix64(a ^ ((uint64_t)len * kGolden)), (mix64(b + len) & ~kLongMarker) | kLongMarker};
  }
};

MQ_HD SegKey seg_key(const uint8_t* p, uint32_t len) {
  SegKeyBuilder kb;
  for (uint32_t i = 0; i < len; i++) kb.push(p[i]);
  return kb.finish();
}

MQ_HD bool seg_is_long(const SegKey& k) { return (k.k1 & kLongMarker) == kLongMarker; }

// The edge table's slot hash. 32-bit integer multiplies are quarter-rate on CDNA and the walk
// hashes one key per frontier particle and level, so the key's four words are folded with rotates
// and one multiply, then mixed by murmur3's 32-bit finalizer (three multiplies, against eleven
// for a 64-bit mix of the same key). Tables of 2^32 slots or more take their high bits from a
// second round (edge_hash); below that every probe uses edge_hash32 alone.
MQ_HD uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
MQ_HD uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}
MQ_HD uint32_t edge_hash32(uint32_t parent, const SegKey& k) {
  return fmix32((uint32_t)k.k0 ^ rotl32((uint32_t)(k.k0 >> 32), 11) ^ rotl32((uint32_t)k.k1, 21) ^
                rotl32((uint32_t)(k.k1 >> 32), 5) ^ parent * 0x9e3779b1u);
}
MQ_HD uint64_t edge_hash(uint32_t parent, const SegKey& k) {
  const uint32_t h = edge_hash32(parent, k);
  return (uint64_t)fmix32(h ^ 0x5bd1e995u) << 32 | h;
}
// edge_hash(parent, k) & mask, the high half only for tables of 2^32 slots or more
MQ_HD uint64_t edge_slot(uint32_t parent, const SegKey& k, uint64_t mask) {
  return (mask >> 32) ? edge_hash(parent, k) & mask : (uint64_t)(edge_hash32(parent, k) & (uint32_t)mask);
}

// ---- trie edges -----------------------------------------------------------------------------
// Global open-addressing table (linear probing, load <= 1/4 by default, MQ_OPT_EDGE_LOAD): (parent node, segment key) ->
// child node. Every child is here, '+' and '#' children included, so a literal topic
// segment "+"/"#" walks exactly like the reference's particles.get(key) (topics.go:604).
constexpr uint32_t kEdgeEmpty = 0xFFFFFFFFu;
constexpr uint32_t kEdgeTomb = 0xFFFFFFFEu;

// The slot also carries the child's own '+' and '#' children (a copy of its NodeWalk fields,
// Index::edge_walk_sync), so the walk learns them with the probe that finds the child instead
// of a dependent NodeWalk read.
struct EdgeSlot {  // 32 B
  uint64_t k0, k1;
  uint32_t parent;  // kEdgeEmpty / kEdgeTomb for free slots
  uint32_t child;
  uint32_t plus, hash;  // the child's plus_child / hash_child
};

// ---- nodes (particles, topics.go:748-757) -----------------------------------------------------
// Walk record, read by the match walk (16 B).
constexpr uint32_t kParentMask = 0x3FFFFFFFu;
constexpr uint32_t kFlagSeg0Wild = 1u << 30;  // path segment 0 starts with '+'/'#' (Q3 rule)
constexpr uint32_t kFlagXNode = 1u << 28;     // NodeLists.flags, sharded index: a subscription here
                                              // has a co-matchable filter on another shard
constexpr uint32_t kFlagPlusKey = 1u << 31;   // this node's key is "+"

struct NodeWalk {
  uint32_t plus_child;    // child keyed "+" or kNone
  uint32_t hash_child;    // child keyed "#" or kNone
  uint32_t parent_flags;  // parent id | kFlagSeg0Wild | kFlagPlusKey
  uint32_t seg;           // index into SegInfo for long keys (verification), else kNone
};

// Subscription lists of a node (32 B). Non-shared subscriptions sit in one slab:
// [sub_off, sub_off + n_direct) can never merge with another subscription of the same client
// for any topic; [sub_off + n_direct, + n_merge) may (the client has another filter that can
// co-match), and go through the per-topic merge table.
// The record also carries the node's pair-block header (NodePair.ent_off / ent_mask, kept equal by
// Index::set_pair_header), so the walk's epilogue reads one record per gathered particle instead
// of two. Inline subscriptions (rare) have their own array, NodeInl, read only under kFlagInline.
struct NodeLists {
  uint32_t sub_off, n_direct, n_merge;
  uint32_t shr_off, shr_cnt;
  uint32_t ent_off, ent_mask;  // pair block: PairEnt hash table (kNone mask: no may-merge slots)
  uint32_t flags;              // kFlagSeg0Wild | kFlagXNode | kFlagInline
};
constexpr NodeLists kEmptyLists{0, 0, 0, 0, 0, 0, 0xFFFFFFFFu, 0};
constexpr uint32_t kFlagInline = 1u << 27;  // NodeLists.flags: the node holds inline subscriptions
struct NodeInl {  // a node's inline subscriptions: inl[off, off + cnt)
  uint32_t off, cnt;
};

// Retained-message state and children of a node, for Messages (32 B).
constexpr uint32_t kRetainPath = 1u;  // particle.retainPath != "" (topics.go:755)
constexpr uint32_t kRetainLive = 2u;  // Retained map holds the path (Q12 decouples the two)
constexpr uint32_t kChildSys = 4u;    // key == "$SYS" under the root (topics.go:549)
constexpr uint32_t kRetainFlag = 8u;  // host only: the live packet's FixedHeader.Retain
struct NodeMsg {
  uint32_t child_off, child_cnt;  // children slab (ChildRec) for '+'/'#' enumeration
  uint32_t flags;                 // kRetainPath | kRetainLive | kChildSys
  uint32_t parent;                // parent node (the stackless Messages walk returns through it)
  uint64_t handle;                // retained packet handle when kRetainLive
  uint32_t below_live;            // live retained topics strictly below this particle: a '#'
                                  // frame's Messages count without walking the subtree
  uint32_t child_pos;             // position in the parent's children slab
};

// Entry of a node's children slab (24 B): the child and a copy of the NodeMsg fields a '+'/'#'
// enumeration needs, so that enumerating children reads the slab sequentially instead of one
// random NodeMsg per child (Index::child_rec_sync keeps the copy current).
struct ChildRec {
  uint32_t node;
  uint32_t child_off, child_cnt;  // the child's own children slab
  uint32_t flags;                 // kRetainPath | kRetainLive | kChildSys
  uint64_t handle;
};
static_assert(sizeof(ChildRec) == 24, "ChildRec layout");

// Sharded index: a node's filter id and DFS rank key, exported per batch for the
// node's cross-shard co-matches. rank = code(path) of SURVEY.md App. A.3, two bits per level
// (kappa + 1: literal 1, '+' 2, '#' 3) from the top, zero-padded, so a proper prefix sorts first;
// paths deeper than 32 levels keep their 32-level code and set `deep`.
struct XInfo {  // 16 B
  uint32_t fid;   // filter id of the node's non-shared subscriptions (kNone: none yet)
  uint32_t deep;  // 1: deeper than the rank key's 32 levels
  uint64_t rank;
};
constexpr uint32_t kForeign = 1u << 31;  // partner id of a filter held by another shard: kForeign | fid

// One exported cross-shard node of a topic (mq_xent).
struct XEnt {  // 16 B
  uint32_t fid;
  uint32_t deep;
  uint64_t rank;
};

// The DFS order beyond the rank key's 32 levels (sharded index): a deep filter's codes for its
// levels 33.. (kappa + 1 as in the rank key), 16 per word from the top, zero-padded, in
// Index::deep_codes[off, off + n). Words compare as the rank keys do, so two deep paths that tie
// in their keys are ordered by their first differing word (a proper prefix first). Entries sit
// in an open-addressed table keyed by filter id (Index::deep; fid kNone: a free slot), holding
// every deep filter the shard knows: its own nodes' and its foreign partners'.
constexpr uint32_t kDeepTomb = 0xFFFFFFFEu;  // a removed entry (sharded filter ids are < 2^31)
struct DeepTail {  // 16 B
  uint32_t fid;
  uint32_t off, n;
  uint32_t pad;
};

struct SegInfo {  // long segment bytes in the segment pool
  uint32_t off, len;
};

// ---- subscription records -------------------------------------------------------------------
// The record formats equal the output row formats (include/mqmatch.h) so that subscriptions
// that cannot merge are copied straight to the output.
struct SubRec {  // == mq_client_row
  uint32_t client;
  uint32_t filter_id;
  int32_t ident;
  uint32_t meta;  // qos | nolocal<<8 | rap<<9 | rh<<10 | row kind (output rows only)
};
// Partner links of may-merge subscriptions. A may-merge subscription (client c at node g)
// has partners: the other non-shared subscriptions of c whose filters can match one topic
// together with g's (Index::compatible). For a topic, the partners that are gathered decide
// the record alone: none -> a plain client row; all gathered later -> the merge base (client
// row with the partners' max Qos and OR'd NoLocal); one gathered earlier -> a non-base entry
// (an ident row when its identifier is > 0, else dropped). That is gatherSubscriptions +
// Subscription.Merge (topics.go:631-648, packets/packets.go:254-274) without a per-topic
// table. The links of one slot are MergePart records mpart[off, off + cnt); mref[pos] names
// them for the slot at subs pool position pos, PairSlot for the slots on pair lists.
struct MergeRef {  // 8 B, parallel to the subs pool
  uint32_t off, cnt;
};
struct MergePart {  // 8 B
  uint32_t node;  // the partner's node
  uint32_t meta;  // the partner's Qos | NoLocal (the bits Subscription.Merge takes from it)
};
// Pair blocks find a topic's merging records without touching the others. For a node g, the
// block maps each partner node h (a node holding a partner of one of g's may-merge
// subscriptions) to the list of g's may-merge slots whose client also subscribes at h, each
// named by its place k in g's subscription list (position sub_off + k: a slot keeps its k when
// the list's slab moves or a direct subscription is added, so updates patch single entries). A topic probes (g, h) only for pairs of nodes it gathers; the slots on
// the hit lists are exactly the records whose client has another match for the topic. Every
// other record is its client's only match and stays a plain client row.
struct NodePair {   // per node (16 B)
  uint32_t ent_off;   // PairEnt hash table (ent_mask + 1 entries, linear probing)
  uint32_t ent_mask;  // kNone: the node has no may-merge slots
  uint32_t list_off;  // the block's slot lists in the pair-list pool
  uint32_t n_lists;
};
struct PairEnt {  // 16 B
  uint32_t h;     // partner node; kNone = empty
  uint32_t off;   // absolute offset of the list in the pair-list pool
  uint32_t cnt;   // slots on the list
  uint32_t cap;   // host bookkeeping: the list's capacity | kPairBase (inside the node's base
                  // slab of lists, not released by itself); the kernels do not read it
};
constexpr uint32_t kPairBase = 0x80000000u;
struct PairSlot {  // 16 B: one slot on a pair list, with its partner links
  uint32_t k;       // the slot's place in g's subscription list (its row: the list's first + k)
  uint32_t mp_off;  // its MergePart records
  uint32_t mp_cnt;
  uint32_t meta;    // the slot's SubRec meta | kSlotIdentPos (its identifier is > 0): resolving
                    // the slot needs no load of the record itself; | the partner's bits (below)
};
constexpr uint32_t kSlotIdentPos = 0x1000u;  // the reserved meta bit (include/mqmatch.h)
// PairSlot.meta also carries the partner's Qos | NoLocal (MergePart.meta of the partner node h the
// list is for) at bits 16-18: meta | identpos | (qos | (nolocal ? 4 : 0)) << kSlotPartShift
constexpr uint32_t kSlotPartShift = 16;
constexpr uint32_t kSlotMetaMask = 0x0FFFu;  // the SubRec meta bits of PairSlot.meta
constexpr uint32_t kSlotOwnMask = 0x1FFFu;   //   and kSlotIdentPos
MQ_HD uint32_t slot_partner_bits(uint32_t partner_meta) {  // MergePart.meta -> PairSlot.meta bits
  return ((partner_meta & 3u) | ((partner_meta & 0x100u) ? 4u : 0u)) << kSlotPartShift;
}

MQ_HD uint32_t pair_hash(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

struct ShrRec {  // == mq_shared_row
  uint32_t filter_id;
  uint32_t client;
};
struct InlRec {  // == mq_inline_row
  int32_t ident;
  uint32_t filter_id;
};

constexpr uint32_t kMetaQos = 0x3u;
constexpr uint32_t kMetaNoLocal = 0x100u;
constexpr uint32_t kMetaRap = 0x200u;
constexpr uint32_t kMetaRhShift = 10;
constexpr uint32_t kRowIdent = 1u << 30;  // == MQ_ROW_IDENT
constexpr uint32_t kRowDrop = 1u << 31;   // == MQ_ROW_DROP

// Gather word written by the walk: node | kGatherSubs | kGatherInline.
constexpr uint32_t kGatherNode = 0x3FFFFFFFu;
constexpr uint32_t kGatherSubs = 1u << 30;    // gather non-shared subscriptions
constexpr uint32_t kGatherInline = 1u << 31;  // gather inline subscriptions

// Per-topic counts from the walk (count pass), exclusive-scanned into offsets.
// rows = non-shared records of the gathers (one output row each); merge = the may-merge ones.
struct TopicCount {
  uint32_t gathers, rows, shared, inlines, merge;
};

}  // namespace mq
