/*
 * mqmatch_dev.h — development and measurement options of the engine (mq_set_option, declared in
 * mqmatch.h). They select kernel variants and synchronisation modes for A/B measurements and
 * tuning sweeps (tools/tune_spans.py, tools/gpu/); the defaults are the product configuration
 * and a broker never sets them. No functions are declared here.
 */
#ifndef MQMATCH_DEV_H
#define MQMATCH_DEV_H

#define MQ_OPT_SUBBATCH_TOPICS 2  /* row format: topics per pipelined sub-batch */
#define MQ_OPT_MSG_SPEC_MB 3      /* Messages: speculative-count scratch budget (MiB; 0: two walks) */
#define MQ_OPT_MSG_WAVES 4        /* Messages: k_msg waves per SIMD (1, 6, 8; 0: by index size) */
#define MQ_OPT_SERIAL 5           /* 1: no side-stream overlap (isolated kernel timings) */
#define MQ_OPT_MERGE_WAVES 7      /* k_merge waves per SIMD the registers are budgeted for (1, 6, 7: set pass only, 8) */
#define MQ_OPT_MSG_IMAGE 8        /* Messages: 1 (default) runs over the level-order retained image;
                                     0 walks the particles (the path the Q6 state always takes) */
#define MQ_OPT_WALK_WAVES 9       /* thread-per-topic k_walk: waves per SIMD the registers are budgeted for (1, 8) */
#define MQ_OPT_WALK_LISTS 10      /* span format: 1 makes the walk count the lists (as the row format) */
#define MQ_OPT_MERGE_DEDUP 12     /* span format: 1 (default) resolves topics with the same merge gathers once
                                     (merge sets); 0: every topic resolves itself (a cross-check) */
#define MQ_OPT_SET_GRID 14        /* merge-set dedup: 1 (default): a wavefront per set; 0: persistent waves
                                     striding the set list */
#define MQ_OPT_WALK_GROUP 15      /* the match walk: 16 (default), 8 or 4 lanes per topic (level-synchronous
                                     frontier walk, k_walkf); 0: thread per topic (stackless DFS, k_walk) */
#define MQ_OPT_ONE_SYNC 16        /* span format, device results: 1 (default) runs a batch with one host
                                     synchronisation, at its end (buffers sized by earlier batches; a batch
                                     they cannot hold runs again, sized by the host); 0: the host reads the
                                     walk's totals and the patch counts between kernels */
#define MQ_OPT_SET_EXP 18         /* attribution experiments on the merge set pass (bits 0-3: results WRONG,
                                     timing only; accepted only by a library built with MQ_DEV_BUILD):
                                     bit 0 no partner links, bit 1 links loaded but not looked up, bit 2 no
                                     patch stores, bit 3 no binary search for a record's hit list; bit 4 (results
                                     exact) no early stop of a visit through a partner other than the record's first; bits 5 / 6 (exact)
                                     partner links loaded 3 / 4 per batch instead of 2 (bits 4-6 act on the
                                     link path: with bit 7); bit 7 (exact) records resolved through their
                                     partner links instead of the fold; bit 8 (exact) fold chunks of 16
                                     visits; bit 9 (exact) merge gathers too big for the hash fold resolved through
                                     their partner links instead of the record-keyed fold (round 5); bits 10 / 11
                                     (exact) that fold for merge gathers of up to two passes / any number of
                                     passes over their visits (default: one pass, kBigFill visits); bit 13
                                     (exact) k_merge's set pass instead of k_set (round 5); bit 14 (exact)
                                     k_set's record-keyed fold at k_merge's table size (kBigFill visits, not
                                     its own kSetBigFill); bit 15 (exact) k_set's hash fold at k_merge's
                                     128-slot table (kFoldCap visits per chunk, not its sized table of up to
                                     kSetFoldCap); bit 16 (exact) that table up to 3/4 full (default: 2/3); bit 17 (exact) up to 3/5 */
#define MQ_OPT_PATCH_CODES 20     /* host span results: 1 (default) 4-byte patch codes when the index allows them
                                     (MQ_SPANS_PATCH_CODES); 0: 8-byte mq_patch records */
#define MQ_OPT_MSG_EXPORT 19      /* Messages: 1 (default) hands a literal level under a fan-out of more than
                                     kMsgExportMin particles (through the key index: more than
                                     kMsgExportMinHits candidate entries) to work items any wavefront takes;
                                     > 1: that threshold for both; 0: the filter's wavefront walks it alone */
#define MQ_OPT_MSG_EDGES 21       /* Messages: 1 (default) looks a literal segment up in the retained image's own
                                     edge table (parent image position, segment) -> child image position, one
                                     probe; 0: the index's edge table, then the particle's image position */
#define MQ_OPT_MSG_EDGE_BUDGET 22  /* Messages: the image edge table's budget in MiB at 1/16 load (default 8192;
                                     4x that at 1/8, else 1/4): a small budget forces the sparser tables'
                                     fallbacks at a small index (their parity test) */
#define MQ_OPT_FAIL_NEXT 23       /* test hook, product-visible on purpose: the next v span batches fail as if a
                                     kernel guard had tripped (MQ_EIO), so that the error paths of the library a
                                     broker ships (pipelined tickets, the batching stages' retries) are tested on
                                     that library itself; it changes no result of a batch that is not failed, and
                                     a broker never sets it */
#define MQ_OPT_WALK_EXP 24        /* development builds: bit 0 looks every topic's level-0 child up in a kernel ahead
                                     of the frontier walk (k_root_hint), which then reads it instead of probing: the
                                     walk's saving bounds what staging the root's children in LDS could save;
                                     bit 1 (round 6): levels 0 and 1 (the frontier's level-1 probes too) */
#define MQ_OPT_MSG_KEYIDX 25      /* Messages: 1 (default) builds the retained image's key index with the image
                                     (edges sorted by key hash, then parent): a literal segment under runs whose
                                     particles take more than kKxMinRounds rounds of probes (64 a round) is one
                                     table probe and searches of the key's entries, when those take fewer
                                     dependent rounds; v >= 2: the same with v in place of kKxMinRounds; 0: one
                                     edge-table probe per particle of the runs */
#define MQ_OPT_MAX 25             /* the highest option number mq_set_option admits */
#define MQ_OPT_FUSE_DESC 17       /* one-sync span batches: 1 (default) runs k_desc in the frontier walk's
                                     epilogue (spans and merge lists at t * 64, no scan); 0: walk, scan, k_desc */

#endif
