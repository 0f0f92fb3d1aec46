/*
 * mqmatch.h — C-ABI of the MI355X (gfx950) topic-matching engine that replaces the
 * reference's `TopicsIndex` hot path (/root/reference/topics.go:349-698).
 *
 * The Go broker reaches this through a thin cgo shim; every entry point
 * below names the reference interface it replaces. Conventions:
 *   - plain pointers and sizes only; strings are (ptr, len) and borrowed for the call only
 *     (cgo rule: nothing keeps Go memory);
 *   - return codes: >= 0 success, < 0 negative errno (MQ_E*); mq_last_error() describes the
 *     last failure on the calling thread;
 *   - client ids, filter ids and inline ids are u32 keys interned by the caller (the Go shim
 *     interns client-ID strings and full filter strings; handlers and packets.Packet values
 *     never cross the ABI, only ids and opaque retained-message handles do);
 *   - the handle is internally synchronised: updates are serialised (the analogue of
 *     root.Lock(), topics.go:402) and a batch runs on the snapshot sealed when it starts,
 *     which is at least as strong as the reference's lock-free readers (topics.go:583, Q11);
 *   - result buffers are owned by the library until mq_result_free().
 */
#ifndef MQMATCH_H
#define MQMATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MQ_ABI_VERSION 9

/* error codes (negative errno) */
#define MQ_EINVAL (-22)
#define MQ_ENOMEM (-12)
#define MQ_ENODEV (-19)
#define MQ_EIO (-5)
#define MQ_ERANGE (-34)
#define MQ_ESTALE (-116)

/* packets.Subscription flag bits (packets/packets.go:172-182) for mq_subscribe() */
#define MQ_SUB_NOLOCAL 0x1u         /* NoLocal */
#define MQ_SUB_RAP 0x2u             /* RetainAsPublished */
#define MQ_SUB_RH_SHIFT 2           /* RetainHandling, 2 bits */

/* mq_client_row.meta layout */
#define MQ_META_QOS_MASK 0x3u       /* merged Qos = max over the client's matches */
#define MQ_META_NOLOCAL 0x100u      /* merged NoLocal = OR over the client's matches */
#define MQ_META_RAP 0x200u          /* base RetainAsPublished */
#define MQ_META_RH_SHIFT 10         /* base RetainHandling, 2 bits */
/* bit 0x1000 is reserved (never set in output rows) */
/* Row kind of an output row (mq_topic_result): none = client row */
#define MQ_ROW_IDENT 0x40000000u    /* an Identifiers entry of an earlier client row's client */
#define MQ_ROW_DROP 0x80000000u     /* absorbed into an earlier client row (identifier 0) */
#define MQ_ROW_KIND_MASK 0xC0000000u

typedef struct mq_index mq_index;

/* mq_config.flags. MQ_CFG_SELECT_SHARED: SelectShared runs on the device (k_pick) and every
 * match result's shared rows hold only the picked member of each shared filter (its client
 * with the smallest id) — for brokers whose hooks do not implement OnSelectSubscribers
 * (server.go:1001-1006), where the Go pick is the first member in random map order
 * (topics.go:320-333). The shim then builds SharedSelected from these rows directly. */
#define MQ_CFG_SELECT_SHARED 1u

typedef struct mq_config {
  int32_t device;          /* HIP device ordinal; the device is first touched by mq_sync/match */
  uint32_t flags;          /* MQ_CFG_* */
  uint64_t expected_subs;  /* capacity hint (0 = default) */
  uint64_t expected_nodes; /* capacity hint (0 = default) */
  /* Sharded index: this handle holds shard shard_index of
   * shard_count (<= 16; 0 or 1: not sharded). Subscriptions are owned by a hash of the filter
   * (shared: of the group and path), inline subscriptions by identifier, retained messages by
   * topic. Every update must be issued to every shard's handle: each applies what it owns and
   * records the others' subscriptions of its clients as cross-shard merge partners. Return
   * values are the shard's part of the reference's: the owner answers Subscribe /
   * InlineSubscribe / RetainMessage (the others return 0; sum or OR them), Unsubscribe /
   * InlineUnsubscribe return whether the particle exists on this shard (OR them, Q10). Filter
   * ids must be < 2^31. A batch runs as mq_match_spans_begin on every shard, an exchange of the
   * exported lists, and mq_match_spans_end; the topic's Subscribers are the union of the
   * shards' results (disjoint: each shard emits its own subscriptions, merged exactly). */
  uint32_t shard_index;
  uint32_t shard_count;
} mq_config;

/* ---- lifecycle: NewTopicsIndex (topics.go:356-364) ---- */
int mq_index_create(const mq_config* cfg, mq_index** out);
void mq_index_destroy(mq_index* idx);
const char* mq_last_error(void);
uint32_t mq_abi_version(void);

/* ---- updates (serialised; visible to batches started after they return) ---- */

/* TopicsIndex.Subscribe(client, sub) (topics.go:401-419). `$SHARE/<group>/...` filters
 * (Unicode EqualFold on segment 0, Q9) are stored as shared subscriptions keyed by
 * (group, client). flags = MQ_SUB_*. Returns 1 if new, 0 if it replaced an existing one. */
int mq_subscribe(mq_index* idx, const char* filter, uint32_t flen, uint32_t client_id,
                 uint32_t filter_id, uint8_t qos, uint8_t flags, int32_t identifier);

/* TopicsIndex.Unsubscribe(filter, client) (topics.go:423-448). Returns 1 whenever the
 * filter's particle exists (Q10), else 0. */
int mq_unsubscribe(mq_index* idx, const char* filter, uint32_t flen, uint32_t client_id);

/* TopicsIndex.InlineSubscribe (topics.go:368-378): keyed by the inline identifier, no
 * $SHARE handling. Returns 1 if new. */
int mq_inline_subscribe(mq_index* idx, const char* filter, uint32_t flen, int32_t identifier,
                        uint32_t filter_id);

/* TopicsIndex.InlineUnsubscribe(id, filter) (topics.go:382-397). Returns 1 if the particle
 * exists (trims only when its inline set became empty). */
int mq_inline_unsubscribe(mq_index* idx, const char* filter, uint32_t flen, int32_t identifier);

/* TopicsIndex.RetainMessage(pk) (topics.go:453-476). `handle` is the caller's opaque id of
 * the packet; payload_len and retain are pk.Payload's length and pk.FixedHeader.Retain.
 * Returns 1 (stored), -1 (a retained packet with payload and Retain was cleared) or 0.
 * Written through *out; the int return is the status code. */
int mq_retain_message(mq_index* idx, const char* topic, uint32_t tlen, uint64_t handle,
                      uint32_t payload_len, uint8_t retain, int64_t* out);

/* TopicsIndex.Retained.Delete(topic) as called by the expiry sweep (server.go:1726): removes
 * the map entry only; the particle keeps its retain path (Q12). Returns 1 if it existed. */
int mq_retained_delete(mq_index* idx, const char* topic, uint32_t tlen);

/* TopicsIndex.Retained.Add(topic, pk) called outside RetainMessage (packets/packets.go:79-83; the
 * Go shim's Retained wrapper forwards it): the map entry (re)appears. Wildcard scans reach an
 * entry through a particle whose retain path is the topic (topics.go:555): such a particle's
 * entry becomes live with `handle` (Q12 re-add), and the "" entry is Q6's. Returns 1 then, 0 when
 * the topic has no particle with a retain path — only a literal filter's Retained.Get(filter)
 * sees such an entry (topics.go:539-544), and the caller's packet map answers that. payload_len
 * and retain: the packet's, for RetainMessage's -1 answer (topics.go:467). */
int mq_retained_set(mq_index* idx, const char* topic, uint32_t tlen, uint64_t handle, uint32_t payload_len,
                    uint8_t retain);

/* TopicsIndex.Retained.Len() (server.go:980) */
uint64_t mq_retained_len(const mq_index* idx);

/* Set up the calling thread's HIP runtime state for the index's device (a thread's first HIP calls
 * cost ~10 ms). Optional: every matching call does it before taking the index's lock; a caller
 * may do it ahead on the threads that will match. */
int mq_thread_warm(mq_index* idx);

/* Columnar bulk Subscribe for the restore path (server.go:1624-1640): n filters as
 * concatenated bytes + n+1 u64 offsets. out_new (nullable) receives Subscribe's results. An empty
 * index with no live host result is built in parallel; otherwise the entries are applied one by
 * one, as mq_subscribe would (never waiting for a live result). */
int mq_subscribe_bulk(mq_index* idx, const uint8_t* filter_bytes, const uint64_t* offsets,
                      const uint32_t* client_ids, const uint32_t* filter_ids, const uint8_t* qos,
                      const uint8_t* flags, const int32_t* identifiers, uint64_t n,
                      uint8_t* out_new);

/* Columnar Unsubscribe (topics.go:423-448) of n (filter, client) pairs, in order, under one
 * lock: out_existed[i] (nullable) = what mq_unsubscribe would return for pair i. */
int mq_unsubscribe_bulk(mq_index* idx, const uint8_t* filter_bytes, const uint64_t* offsets,
                        const uint32_t* client_ids, uint64_t n, uint8_t* out_existed);

/* Columnar bulk RetainMessage with payload (server.go:1688-1692). */
int mq_retain_bulk(mq_index* idx, const uint8_t* topic_bytes, const uint64_t* offsets,
                   const uint64_t* handles, uint64_t n);

/* ---- batched match: TopicsIndex.Subscribers (topics.go:583-628) ---- */

/* Client row: the merged packets.Subscription of one client (gatherSubscriptions +
 * Subscription.Merge, topics.go:631-648, packets/packets.go:254-274). filter_id/identifier/
 * RetainAsPublished/RetainHandling come from the base (first-gathered) subscription; qos is
 * the max and NoLocal the OR over all of the client's matching subscriptions. The Go
 * Identifiers map is {base filter: base identifier} plus the client's ident rows. */
typedef struct mq_client_row {
  uint32_t client_id;
  uint32_t filter_id;
  int32_t identifier;
  uint32_t meta; /* MQ_META_* */
} mq_client_row;

/* Identifiers-map entry other than the base one: a further matching filter of the client
 * with identifier > 0 (packets/packets.go:261-263). It is an mq_client_row whose meta has
 * MQ_ROW_IDENT set (its other meta bits are those of that subscription, not merged). */
typedef mq_client_row mq_ident_row;

/* Subscribers.Shared[filter][client] (topics.go:651-665): the stored subscription's own
 * filter and its client; the group members before the host's SelectShared pick. */
typedef struct mq_shared_row {
  uint32_t filter_id;
  uint32_t client_id;
} mq_shared_row;

/* Subscribers.InlineSubscriptions[id] (topics.go:668-676), last write already applied. */
typedef struct mq_inline_row {
  int32_t identifier;
  uint32_t filter_id;
} mq_inline_row;

/* Per-topic result descriptor. Every non-shared subscription the topic gathers leaves one
 * 16-byte row, in gather (DFS) order, in the region [sub_base, sub_base + sub_cap): a client
 * row (meta & MQ_ROW_KIND_MASK == 0) for the first-gathered subscription of each client, and
 * for a client's later matches an ident row (MQ_ROW_IDENT, identifier > 0) or a dropped row
 * (MQ_ROW_DROP). n_client / n_ident count the client / ident rows. Shared rows are
 * [shared_base, + n_shared), inline rows [inline_base, + n_inline). */
typedef struct mq_topic_result {
  uint64_t sub_base;
  uint64_t shared_base;
  uint64_t inline_base;
  uint32_t sub_cap;
  uint32_t n_client;
  uint32_t n_ident;
  uint32_t n_shared;
  uint32_t n_inline;
  uint32_t reserved;
} mq_topic_result;

typedef struct mq_match_result {
  uint32_t n_topics;
  uint32_t reserved;
  const mq_topic_result* topics; /* n_topics */
  const mq_client_row* sub_rows; /* client, ident and dropped rows (MQ_ROW_*) */
  const mq_shared_row* shared_rows;
  const mq_inline_row* inline_rows;
  uint64_t n_sub_rows, n_shared_rows, n_inline_rows;
} mq_match_result;

/* Match a batch of publish topics (n topics as concatenated bytes + n+1 u64 offsets, host
 * memory). Results are copied to library-owned host memory; free with mq_result_free. */
int mq_match_batch(mq_index* idx, const uint8_t* topic_bytes, const uint64_t* offsets, uint32_t n,
                   mq_match_result** out);

/* Device-resident variant (inputs already in HBM on the index's device, enqueued on
 * `hip_stream`, a hipStream_t or NULL). d_topic_bytes must be 16-byte aligned and readable up
 * to the next 16-byte boundary past its end (any hipMalloc / torch allocation is). `out` receives DEVICE pointers owned by the index and
 * valid until its next match call. Batches whose rows exceed the output budget are processed
 * in chunks; then only the last chunk's rows remain resident and out->topics covers that
 * chunk (out->n_topics); mq_match_chunks() reports the chunk count of the last call. */
int mq_match_device(mq_index* idx, const uint8_t* d_topic_bytes, const uint64_t* d_offsets,
                    uint32_t n, void* hip_stream, mq_match_result* out);
/* Device-resident results of every chunk: like mq_match_device, and for each output chunk, once
 * its kernels are queued, fn(user, chunk, first_topic, chunk_stream) is called on the calling
 * thread. The call returns once the batch (and the consumers' queued work) has completed, with
 * the batch's guard flags checked: a tripped guard fails this call with MQ_EIO. (mq_match_device
 * itself stays asynchronous: a guard tripped by its kernels fails the index's next call.) `chunk` holds device pointers (row offsets relative to the chunk) of topics
 * [first_topic, first_topic + chunk->n_topics); they stay valid for work the consumer enqueues
 * on `chunk_stream` before returning (e.g. a device-side fan-out or a D2H copy): the buffers are
 * reused only after that work. Replaces the reference's per-topic Subscribers() for GPU-side
 * consumers (topics.go:583). C consumers only: the Go shim uses mq_match_batch (no callbacks
 * into Go). */
typedef void (*mq_chunk_fn)(void* user, const mq_match_result* chunk, uint32_t first_topic, void* chunk_stream);
int mq_match_device_chunks(mq_index* idx, const uint8_t* d_topic_bytes, const uint64_t* d_offsets, uint32_t n,
                           void* hip_stream, mq_chunk_fn fn, void* user);
uint32_t mq_match_chunks(const mq_index* idx);

/* SelectShared on the device (topics.go:320-333) for device results (a chunk
 * handed to an mq_chunk_fn, or mq_match_device's output), enqueued on hip_stream: for every
 * topic t, one member (smallest client id) of each shared filter among its shared rows is
 * written to d_selected[topics[t].shared_base + k], k < d_n_selected[t]. d_selected holds
 * n_shared_rows rows, d_n_selected n_topics u32. The chunk is not modified. Replaces the
 * host's SelectShared when no OnSelectSubscribers hook picks (server.go:1001-1006). It takes
 * no handle lock, so an mq_chunk_fn may call it on its chunk; a match must have run first. */
int mq_select_shared_device(mq_index* idx, const mq_match_result* chunk, void* hip_stream,
                            mq_shared_row* d_selected, uint32_t* d_n_selected);

/* ---- span format: Subscribers without copying the gathered lists (ABI v5; v6: set patches) ----
 *
 * The row format above copies every gathered subscription of every topic into output rows; at
 * 10M subscriptions a topic gathers ~15k of them (the root '#', '+/...', 'x/#' lists, the same
 * for most topics), 245 KB per topic. The span format names them instead. A topic's result is
 *   - one mq_span per gathered particle, in gather (DFS) order: its non-shared records
 *     sub_pool[sub_off, + n_sub) (n_sub = 0 when the '$' rule drops them, Q3) and its shared
 *     members shared_pool[shr_off, + n_shr);
 *   - mq_patch records for the records whose row differs from the pool record: the merge base
 *     of a client with several matches (merged Qos / NoLocal), or a later match of the client
 *     (MQ_ROW_IDENT / MQ_ROW_DROP). `row` is the record's position in the concatenation of the
 *     topic's spans' sub ranges (0 .. n_rows-1); each row is patched at most once; patches are
 *     in no particular order;
 *   - the inline rows, last-write applied (as in the row format).
 * Expanding spans and applying patches gives exactly the row format's rows (mq_spans_expand).
 * Device results (mq_match_spans_device) may share patches between topics: topics whose gathered
 * particles with may-merge records are the same particles in the same order resolve to the same
 * patches up to where those particles' records sit in each topic's rows, so the batch resolves
 * each such merge set once. A topic with MQ_TOPIC_SET_PATCHES in its flags has its n_patches
 * patches at set_patches[patch_base, + n_patches), each naming its row as (x << 26 | k): record
 * k of the span of the topic's x-th particle with may-merge records, i.e. topic row
 * merge_rows[topic * 64 + x] + k (merge_rows: the row of that span's first record). Host results
 * (mq_match_spans, ABI v7) share them the same way, packed: the set patches in set_patches and
 * each such topic's merge rows at merge_rows[merge_row_base[topic]] (one per may-merge particle);
 * mq_topic_patch() below resolves either layout.
 * With MQ_CFG_SELECT_SHARED the picked shared members are materialised (picked_rows at
 * picked_base, n_shared of them) and flags has MQ_SPANS_PICKED. */
typedef struct mq_span {
  uint32_t sub_off, n_sub; /* records sub_pool[sub_off, + n_sub) */
  uint32_t shr_off, n_shr; /* members shared_pool[shr_off, + n_shr) */
} mq_span;

typedef struct mq_patch {
  uint32_t row;  /* topic-relative record row */
  uint32_t meta; /* replaces the pool record's meta (MQ_META_*, MQ_ROW_*) */
} mq_patch;

typedef struct mq_topic_spans {
  uint64_t span_base, patch_base, inline_base, picked_base;
  uint32_t n_spans, n_patches, n_inline;
  uint32_t n_rows;   /* gathered non-shared records (client + ident + dropped rows) */
  uint32_t n_client, n_ident;
  uint32_t n_shared; /* shared members (picked members with MQ_SPANS_PICKED) */
  uint32_t flags;    /* MQ_TOPIC_SET_PATCHES (device results only) */
} mq_topic_spans;

#define MQ_SPANS_PICKED 1u
#define MQ_SPANS_PATCH_CODES 2u /* host results (ABI v8): patches / set_patches hold 4-byte codes */
#define MQ_TOPIC_SET_PATCHES 1u
#define MQ_SET_ROW_BITS 26   /* set patch rows: x << MQ_SET_ROW_BITS | k */
#define MQ_MERGE_ROWS_STRIDE 64
/* Patch codes (host results with MQ_SPANS_PATCH_CODES; the arrays are then uint32_t): code =
 * row << 3 | op. op 1..6: the merge base of its client, Qos (op - 1) % 3, NoLocal (op - 1) / 3;
 * op 7: a later match of the client (MQ_ROW_IDENT when the record's identifier is > 0, else
 * MQ_ROW_DROP). The record's other meta bits are unchanged, so the code and the pool record give
 * the row's meta (mq_patch_apply). A set patch code's row is x << MQ_CODE_SET_ROW_BITS | k. Host
 * results use codes when every subscription list has fewer than 2^23 records. */
#define MQ_CODE_SET_ROW_BITS 23
#define MQ_PATCH_OP 0x20000000u /* mq_topic_patch's meta of a code: MQ_PATCH_OP | op */

typedef struct mq_span_result {
  uint32_t n_topics;
  uint32_t flags; /* MQ_SPANS_PICKED */
  const mq_topic_spans* topics;
  const mq_span* spans;
  const mq_patch* patches;
  const mq_inline_row* inline_rows;
  const mq_shared_row* picked_rows;
  const mq_client_row* sub_pool;    /* the index's subscription records */
  const mq_shared_row* shared_pool; /* the index's shared members */
  uint64_t n_spans;
  uint64_t n_patches; /* host result: patches, packed; device result: the patch pool's extent
                         (topic ranges lie in per-region parts of it, with unused gaps) */
  uint64_t n_inline_rows, n_picked_rows;
  uint64_t sub_pool_len, shared_pool_len;
  /* patches shared by topics with MQ_TOPIC_SET_PATCHES and the topics' merge rows; null / 0 when
     no topic shares. Device results: MQ_MERGE_ROWS_STRIDE merge rows per topic at topic * 64,
     merge_row_base null, set_patches the pool's extent (per-region parts with gaps). Host results
     (v7): set_patches packed, merge rows packed at merge_row_base[topic] (n_topics entries; 0 for
     a topic without MQ_TOPIC_SET_PATCHES) */
  const mq_patch* set_patches;
  const uint32_t* merge_rows;
  uint64_t n_set_patches;
  const uint32_t* merge_row_base;
  uint64_t n_merge_rows;
} mq_span_result;

/* Patch k (< n_patches) of topic t of a span result whose arrays the caller can read (a host
 * result, or a device result copied to the host): the topic's own patch, or its set patch with
 * the row translated through the topic's merge rows. Its meta is the row's new meta, or, for a
 * patch code, MQ_PATCH_OP | op: mq_patch_apply gives the row's meta in either case. */
static inline mq_patch mq_topic_patch(const mq_span_result* r, uint32_t t, uint32_t k) {
  const mq_topic_spans* ts = &r->topics[t];
  const int set = (ts->flags & MQ_TOPIC_SET_PATCHES) != 0;
  uint32_t xbits = MQ_SET_ROW_BITS;
  mq_patch p;
  if (r->flags & MQ_SPANS_PATCH_CODES) {
    const uint32_t* codes = (const uint32_t*)(set ? (const void*)r->set_patches : (const void*)r->patches);
    const uint32_t c = codes[ts->patch_base + k];
    p.row = c >> 3;
    p.meta = MQ_PATCH_OP | (c & 7u);
    xbits = MQ_CODE_SET_ROW_BITS;
  } else {
    p = set ? r->set_patches[ts->patch_base + k] : r->patches[ts->patch_base + k];
  }
  if (!set) return p;
  const uint32_t* mr = r->merge_rows + (r->merge_row_base ? (uint64_t)r->merge_row_base[t]
                                                           : (uint64_t)t * MQ_MERGE_ROWS_STRIDE);
  p.row = mr[p.row >> xbits] + (p.row & ((1u << xbits) - 1u));
  return p;
}

/* The meta of a patched row: a patch's meta (mq_topic_patch) applied to the pool record's. */
static inline uint32_t mq_patch_apply(uint32_t patch_meta, uint32_t meta, int32_t identifier) {
  if (!(patch_meta & MQ_PATCH_OP)) return patch_meta;
  const uint32_t op = patch_meta & 7u;
  if (op == 7u) return meta | (identifier > 0 ? MQ_ROW_IDENT : MQ_ROW_DROP);
  return (meta & ~(MQ_META_QOS_MASK | MQ_META_NOLOCAL)) | ((op - 1u) % 3u) | ((op - 1u) / 3u ? MQ_META_NOLOCAL : 0u);
}

/* Span-format Subscribers for a batch of host topics (as mq_match_batch). The result's arrays
 * are host copies; its pools point at the index's host image, and what they show a result stays
 * as it was at the match until mq_result_free: an update never waits for a result — the index
 * copies a subscription slab before it changes one a live result may see, and keeps what it
 * frees until no live result can see it (the reference's writers never wait for a reader's maps
 * either, topics.go:270-277, 401-419). Updates are preferred, as with Go's sync.RWMutex: while an
 * update waits (for the match in flight), new matches wait for it, so readers matching back to
 * back cannot starve updates. mq_subscribe_bulk does not wait for results either: while one is
 * live it takes the per-entry path (copy-on-write), so a pipelined caller holding a ticket or a
 * result may overlap a restore. */
int mq_match_spans(mq_index* idx, const uint8_t* topic_bytes, const uint64_t* offsets, uint32_t n,
                   mq_span_result** out);
/* The same, pipelined (ABI v8): mq_match_spans_submit runs the batch's kernels and returns with
 * the copy of its result into host memory still running on a copy stream, beside the next
 * submitted batch's kernels; mq_match_spans_wait waits for that copy and returns the result
 * (exactly mq_match_spans's), freeing the ticket. Every ticket must be waited for; results are
 * freed with mq_result_free. Batches k and k + 1 overlap: for consecutive batches the host-result
 * rate is bound by the larger of the kernels and the copies, not their sum. */
typedef struct mq_spans_ticket mq_spans_ticket;
int mq_match_spans_submit(mq_index* idx, const uint8_t* topic_bytes, const uint64_t* offsets, uint32_t n,
                          mq_spans_ticket** out);
int mq_match_spans_wait(mq_spans_ticket* ticket, mq_span_result** out);
/* Device-resident span format (inputs in HBM, enqueued on hip_stream, as mq_match_device). All
 * pointers in *out are DEVICE pointers owned by the index, valid until its next update or match
 * call. The whole batch is one result (no chunks); the call returns after the batch's kernels
 * have completed, with their guard flags checked (MQ_EIO when one tripped). A topic's spans are
 * spans[span_base, + n_spans): topics' ranges may have gaps between them (a batch run with one
 * host synchronisation places topic t's at t * 64), and n_spans of the result is the array's
 * extent. */
int mq_match_spans_device(mq_index* idx, const uint8_t* d_topic_bytes, const uint64_t* d_offsets,
                          uint32_t n, void* hip_stream, mq_span_result* out);
/* Materialise the rows of topics [first, first + count) of a HOST span result (mq_match_spans):
 * their sub rows (n_rows each, patches applied: exactly the row format's rows) and shared rows,
 * concatenated in topic order. Returns 0, or MQ_ERANGE when a capacity is too small; the
 * numbers of rows written go to *n_rows / *n_shared (nullable). Thread-safe for disjoint
 * outputs. */
int mq_spans_expand(const mq_span_result* r, uint32_t first, uint32_t count, mq_client_row* rows,
                    uint64_t rows_cap, mq_shared_row* shared, uint64_t shared_cap, uint64_t* n_rows,
                    uint64_t* n_shared);

/* ---- sharded batches (mq_config.shard_count > 1) ----
 * A topic's client merge (Subscription.Merge over the client's matches, in DFS order) can span
 * shards. mq_match_spans_begin walks the batch and exports, per topic, this shard's gathered
 * particles that hold a subscription whose client has a co-matchable filter on another shard:
 * the filter id and its DFS rank key (two bits per level, 32 levels).
 * The caller gathers every other shard's export (e.g. an all-gather over RCCL) and passes them
 * to mq_match_spans_end, which resolves this shard's records exactly against them. A cross-shard
 * tie beyond the key's 32 levels fails the batch loudly (MQ_EIO). */
typedef struct mq_xent {
  uint32_t filter_id;
  uint32_t deep; /* deeper than the rank key's 32 levels */
  uint64_t rank;
} mq_xent;

typedef struct mq_xlist {
  uint32_t n_topics;
  uint32_t shard;
  const uint32_t* counts; /* n_topics: entries per topic (DEVICE memory) */
  const mq_xent* ents;    /* the topics' entries in topic order (DEVICE memory) */
  uint64_t n_ents;
} mq_xlist;

/* Begin a span-format batch (inputs in HBM as mq_match_spans_device). *exported holds device
 * pointers owned by the index, valid until mq_match_spans_end; an index that is not sharded
 * exports nothing (n_ents = 0, null pointers). No update may run until the batch ends. */
int mq_match_spans_begin(mq_index* idx, const uint8_t* d_topic_bytes, const uint64_t* d_offsets, uint32_t n,
                         void* hip_stream, mq_xlist* exported);
/* End it with the other shards' exports (n_foreign <= 15 lists in device memory readable by
 * this index's device; 0 for an index that is not sharded): results as mq_match_spans_device. */
int mq_match_spans_end(mq_index* idx, const mq_xlist* foreign, uint32_t n_foreign, void* hip_stream,
                       mq_span_result* out);
/* The same with the results copied to host memory (as mq_match_spans). */
int mq_match_spans_end_host(mq_index* idx, const mq_xlist* foreign, uint32_t n_foreign, mq_span_result** out);

/* ---- batched reverse retained scan: TopicsIndex.Messages (topics.go:525-579) ---- */
typedef struct mq_msg_result {
  uint32_t n_filters;
  uint32_t reserved;
  const uint64_t* base;    /* n_filters: first handle of each filter */
  const uint32_t* count;   /* n_filters */
  const uint64_t* handles; /* retained-message handles (set per filter, order unspecified) */
  uint64_t n_handles;
} mq_msg_result;

int mq_messages_batch(mq_index* idx, const uint8_t* filter_bytes, const uint64_t* offsets,
                      uint32_t n, mq_msg_result** out);
int mq_messages_device(mq_index* idx, const uint8_t* d_filter_bytes, const uint64_t* d_offsets,
                       uint32_t n, void* hip_stream, mq_msg_result* out);

/* Messages as runs (round 6; SURVEY.md §7 step 8: `x/#` and `+` results kept as contiguous
 * intervals, expanded at the boundary). The walk over the level-order retained image finds each
 * filter's handles as runs of consecutive entries of one array — every particle's children are
 * one image range, so a final '+' is one run per run of parents and a final '#' one run per level
 * (topics.go:547-566) — and the result names those runs instead of copying the handles: filter i
 * has runs[run_base[i], + n_runs[i]), run r is handles[r.first, + r.count), and r.at is where the
 * run starts in the batch's expanded output (filter i's handles are [base[i], + count[i]) of it:
 * the same layout as mq_msg_result). `handles` is the retained image's handle array (level order),
 * or, for a batch that took the particle walk (the Q6 "" entry live, nesting beyond 16 fan-outs),
 * the batch's own handles with one run per filter. Handle order within a filter is unspecified, as
 * in mq_msg_result. */
typedef struct mq_msg_run {
  uint32_t first; /* index of the run's first handle in the result's handles */
  uint32_t count; /* handles in the run */
  uint64_t at;    /* where the run starts in the batch's expanded output */
} mq_msg_run;

typedef struct mq_msg_runs_result {
  uint32_t n_filters;
  uint32_t reserved;
  const uint64_t* run_base; /* n_filters: each filter's first run */
  const uint32_t* n_runs;   /* n_filters */
  const uint64_t* base;     /* n_filters: each filter's first handle in the expanded output */
  const uint32_t* count;    /* n_filters: each filter's handles */
  const mq_msg_run* runs;
  uint64_t n_runs_total;
  const uint64_t* handles;  /* the array the runs index */
  uint64_t n_handles;       /* its length */
  uint64_t n_expanded;      /* handles of the whole batch (sum of count) */
} mq_msg_runs_result;

/* Device result: every pointer is device memory owned by the index, valid until its next
 * Messages call (the image array until the retained set changes and a Messages call rebuilds it). */
int mq_messages_runs_device(mq_index* idx, const uint8_t* d_filter_bytes, const uint64_t* d_offsets,
                            uint32_t n, void* hip_stream, mq_msg_runs_result* out);
/* Host result (mq_result_free): the runs copied to host memory, `handles` a host copy of the image
 * shared by the results of one image version (copied once per version). */
int mq_messages_runs_batch(mq_index* idx, const uint8_t* filter_bytes, const uint64_t* offsets,
                           uint32_t n, mq_msg_runs_result** out);
/* Expand filters [first, first + count) of a host runs result into out (cap handles) in the
 * expanded layout: filter i's handles at out[base[i] - base[first], + count[i]) (a batch the
 * particle walk answered may leave gaps between filters); *n_out: the end of the last one. */
int mq_msg_runs_expand(const mq_msg_runs_result* r, uint32_t first, uint32_t count, uint64_t* out,
                       uint64_t cap, uint64_t* n_out);

/* Batched auth.MatchTopic (hooks/auth/ledger.go:90-118): the ACL ledger's
 * filter/topic test that the fan-out runs per recipient (server.go:1029 -> Ledger.ACLOk ->
 * RString.FilterMatches). Pairs index two string tables (filters, topics: bytes + u64 offsets)
 * so one publish topic can be tested against many ACL filters. Per pair: matched (0/1) and the
 * captured elements ('+' parts, the '#' remainder) as (start, len) spans into the pair's topic,
 * including those captured before a failed match, as the reference returns them. */
typedef struct mq_acl_result {
  uint64_t n_pairs;
  const uint8_t* matched;
  const uint32_t* n_elems;
  const uint64_t* elem_base;  /* pair p's spans: elems[2 * elem_base[p] .. + 2 * n_elems[p]) */
  const uint32_t* elems;
} mq_acl_result;
int mq_acl_match_batch(mq_index* idx, const uint8_t* filter_bytes, const uint64_t* filter_offs, uint32_t n_filters,
                       const uint8_t* topic_bytes, const uint64_t* topic_offs, uint32_t n_topics,
                       const uint32_t* pair_filter, const uint32_t* pair_topic, uint64_t n_pairs,
                       mq_acl_result** out);

void mq_result_free(void* result);

/* ---- device image, statistics and profiling ---- */

/* Push pending updates to the device image (incremental: only dirty pages are copied). */
int mq_sync(mq_index* idx, void* hip_stream);

typedef struct mq_stats {
  uint64_t nodes, edges, edge_capacity;
  uint64_t subs, subs_merge, shared, inlines;
  uint64_t retained, retained_live;
  uint64_t device_bytes, upload_bytes_total, syncs;
  uint64_t partners; /* partner links between may-merge subscriptions */
  uint64_t foreign;  /* sharded: other shards' subscriptions recorded as merge partners */
  uint32_t max_depth;
  uint32_t edge_load; /* the edge table's load bound at its current size: at most 1/edge_load of
                         its slots used (MQ_OPT_EDGE_LOAD, 2 from 2^30 slots on or beyond the
                         index's HBM budget for it) */
} mq_stats;
int mq_index_stats(const mq_index* idx, mq_stats* out);

/* Diagnostic, host only (no device work): brings the device-bound image up to date and checks
   its invariants — list bounds, partner links of may-merge subscriptions (symmetric, pointing at
   the partner's current slot). Returns 0, or MQ_EIO with the first violation in
   mq_last_error(). */
int mq_index_check(mq_index* idx);
/* Diagnostic, with device work: pushes pending updates, reads every device array back and
   compares it with the host mirror. Returns 0, or MQ_EIO with the first difference. */
int mq_device_check(mq_index* idx);

/* Engine options. The defaults are the product; these three trade memory for speed or size a
 * pool up front. Returns 0, or MQ_EINVAL for an unknown option or value. The measurement and
 * tuning knobs the benchmarks use (kernel variants, register budgets, synchronisation modes) are
 * in mqmatch_dev.h: development options, not part of the ABI's contract. */
#define MQ_OPT_CHUNK_ROWS 1       /* row format: output rows per chunk (default 0xF0000000) */
#define MQ_OPT_PATCH_CAP 6        /* span format: initial patch pool capacity (patches) */
#define MQ_OPT_EDGE_LOAD 13       /* edge table: at most 1/v of its slots used (2, 4, 8, 16 = default: sparser means
                                     shorter probe chains for the walk, more memory; a table of 2^30 slots or
                                     more keeps 1/2); applies from the next growth. Memory: 32 B per slot in
                                     HBM and again in the host mirror — 10M config-3 subscriptions (32.6M
                                     particles) take 537M slots, 17 GB, at 1/16 (4.3 GB at 1/4). A table that
                                     would outgrow an eighth of the device's memory (mq_index_create reads
                                     it) at 1/8 or 1/16 is kept at 1/4 instead (mq_stats.edge_load) */
int mq_set_option(mq_index* idx, uint32_t option, uint64_t value);

/* Kernel timing by HIP events recorded on the launch stream around each kernel. enable: 0 off,
 * MQ_PROF_TIMES kernel times, MQ_PROF_WORK also the span format's k_merge work counters
 * (pair-table loads, resolved records, partner links; entries "merge_*" with launches = count
 * and total_ms = 0), from which bench.py prices k_merge's algorithmic bytes. The counters cost
 * atomics: enable them for a measurement pass, not in a timed one. */
#define MQ_PROF_TIMES 1
#define MQ_PROF_WORK 2
#define MQ_PROF_WALK 4 /* times of the match walk's launches only (no events around the other kernels) */
typedef struct mq_kernel_time {
  char name[32];
  uint64_t launches;
  double total_ms;
} mq_kernel_time;
int mq_profile_enable(mq_index* idx, int enable);
int mq_profile_read(const mq_index* idx, mq_kernel_time* out, uint32_t cap); /* returns count */
int mq_profile_reset(mq_index* idx);

#ifdef __cplusplus
}
#endif

#endif /* MQMATCH_H */
