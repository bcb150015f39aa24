/*
 * ruleset_hip.h — C ABI of libruleset_hip.so, the MI355X (gfx950) hot path of
 * ruleset-analysis: first-match classification of connection tuples against
 * ordered access-list rules, fused with the reducer's per-rule aggregation.
 *
 * The reference has no native FFI (it is Python-2 Hadoop streaming); each entry
 * point below replaces a region of the reference's Python loop, cited file:line.
 * Plain pointers and sizes only: "d_" pointers are device (HBM) pointers owned
 * by the caller, "h_" pointers are host pointers owned by the caller.  The
 * library owns only the compiled rule tables and the distinct-connection hash
 * table behind an rsa_ctx.  Every call returns an int status (RSA_OK or a
 * negative code) and rsa_last_error(ctx) describes the last failure.  Calls on
 * one ctx are serialised on the ctx's HIP stream (rsa_set_stream).
 */
#ifndef RULESET_HIP_H
#define RULESET_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RSA_OK 0
#define RSA_ERR_ARG (-1)      /* bad argument / shape                          */
#define RSA_ERR_HIP (-2)      /* HIP runtime error                              */
#define RSA_ERR_STATE (-3)    /* call out of order (e.g. no rules loaded)       */
#define RSA_ERR_CAPACITY (-4) /* distinct-connection table overflowed           */

/* Tuple flags (rsa_tuple.flags). */
#define RSA_F_VALID 0x01u /* line parsed and an ACL resolved: classify it     (mapper.py:124-156)  */
#define RSA_F_HIT 0x02u   /* line contains -6-302013 / -6-302015              (connlist-reducer.py:146) */
#define RSA_F_BUILT 0x04u /* reducer's BUILT regex matched                   (connlist-reducer.py:152-153) */
#define RSA_F_SWAP 0x08u  /* reducer key is (dst, src, sport) of the tuple, not (src, dst, dport) */

#define RSA_NO_RULE (-1)
#define RSA_NO_THRESHOLD 0xFFFFFFFFFFFFFFFFull

/* One packed connection tuple, 16 B (mapper.py:26-51 Connection + the fields the
 * reducer derives from the same line, connlist-reducer.py:152-165). */
typedef struct rsa_tuple {
  uint32_t src;    /* IPv4, host order                                     */
  uint32_t dst;    /* IPv4, host order                                     */
  uint16_t sport;  /* source port                                          */
  uint16_t dport;  /* destination port                                     */
  uint16_t list;   /* candidate list id = (host, acl, protocol)           */
  uint8_t flags;   /* RSA_F_*                                              */
  uint8_t pspell;  /* id of the protocol word as written (e.g. "TCP")      */
} rsa_tuple;

/* One compiled candidate-list entry, 32 B: an expanded permit rule reduced to
 * the integer predicate of FirewallRule.__contains__ (firewallrule.py:128-174).
 * Deny rules and rules whose protocol cannot match the list's protocol are
 * dropped at compile time (they can never be a connection's first match).
 *
 * A run entry (step != 0) stands for the rules gid, gid + stride, ...,
 * gid + span * stride that the preprocessors expanded from one port range
 * (preprosess_access_lists.py:58-89,256-276; preprosess_fortigate_acl.py:90-100,
 * 184-186), each holding ONE port of the range: a connection with port p in
 * [lo, lo + span] matches the rule gid + (p - lo) * stride of the run.  Lists
 * are in ascending first-gid order (the gid field). */
#define RSA_STEP_SPORT 0x80000000u /* run over the source port (else the destination port) */
typedef struct rsa_rule_entry {
  uint32_t src_lo, src_span;  /* (src - src_lo) <= src_span: IPy containment, */
  uint32_t dst_lo, dst_span;  /* net.ip <= x < net.ip + net.len()            */
  uint32_t port_lo;           /* sport_lo | dport_lo << 16                 */
  uint32_t port_span;         /* (sport_hi-sport_lo) | (dport_hi-dport_lo) << 16 */
  uint32_t gid;               /* global rule id = acl base + expanded ruleindex (first rule of a run) */
  uint32_t step;              /* 0, or run stride | RSA_STEP_SPORT if the run varies the source port */
} rsa_rule_entry;

/* Pruned perfect-hash tuple-space index (optional; compile.py build_index).
 * Per candidate list: entries [0, prefix) are scanned linearly; entries >= prefix
 * whose addresses are prefixes and whose ports are "any" or one value (and that
 * are not run entries) are grouped by (src mask, dst mask) (<= 64 groups per
 * record, ascending smallest entry index) and, inside a group, by port class
 * c = 0..3 with port mask {0, 0xFFFF0000 (dport), 0x0000FFFF (sport),
 * 0xFFFFFFFF}.  Each (group, class) owns a CHD (hash-and-displace) perfect-hash
 * table over the masked key (src & src_mask, dst & dst_mask, ports & port_mask),
 * ports = sport | dport << 16:
 *   H    = fmix32(ks ^ 0x9E3779B9) ^ fmix32(kd ^ 0x7F4A7C15) ^ fmix32(kp ^ 0x2545F491)
 *   d    = disp[disp_off + ((H >> 16) & disp_mask)]            (uint16 units of the image)
 *   x    = (H + d * ((H >> 16) | 1)) & 0xFFFF,  slot = (x * n_slots) >> 16,
 *          n_slots <= 65536 (24-bit multiplier operands)
 *   word = image[slot_off + slot] = (H & 0xFFFF) << 16 | record-local entry index,
 *          0xFFFFFFFF = empty (image word 0 is always empty: absent classes
 *          point there with n_slots = 1)
 * holding the smallest entry index with that key.  Pruning: per non-zero src
 * (dst) mask of a record, a CHD table over H = fmix32((src & mask) ^ 0x9E3779B9)
 * (dst: ^ 0x7F4A7C15) whose slot value indexes a uint64 bitmap of the groups
 * holding a rule on that prefix (bitmap 0 is empty: an empty slot, 0, and a
 * tag mismatch both read it); groups with mask 0 are in src_any (dst_any).
 * A tuple probes only the groups in (src bitmap & dst bitmap).  All other
 * entries are residual (a first-gid-ascending list scanned linearly).
 *
 * Lists longer than 0xF000 entries are chains of records, one per chunk of
 * 0xF000 entries (records n_lists .. n_records-1 are the continuation chunks):
 * a lane moves to record `next` only while its best gid exceeds `next_min`.
 * The answer is identical to the linear scan: the minimum matching gid (the
 * device verifies the hashed candidate against the full entry).
 *
 * Everything lives in ONE uint32 image: word 0 = 0xFFFFFFFF, word 1 =
 * RSA_PHT_MAGIC, word 2 = n_lists, word 3 = list_off (word offset of n_records
 * rsa_pht_list records), word 4 = n_records, word 5 = flags (bit 1: every
 * pruning table has 16-bit slots), words 6..7 = 0; records sit at 4-word
 * aligned offsets, bitmaps at even offsets (low word first). */
#define RSA_PHT_MAGIC 0x34415352u
#define RSA_PHT_NONE 0xFFFFFFFFu

/* The partial-key bucket index (word 1 = RSA_BKT_MAGIC; ruleset-analysis_amd/
 * bucketindex.py): the same header and list records (rsa_pht_list), where
 * group_off / n_groups are the record's rsa_bkt_table descriptors (ascending
 * min_gid) and mask_off / n_masks / bm_off / n_bitmaps are unused.  A table
 * keys its entries on (src & src_mask, dst & dst_mask, ports & port_mask);
 * its n_buckets buckets are two uint32 slots each at bucket_off (even),
 * slot = tag11 << 21 | len5 << 16 | first16 (len 0: empty), the bucket's rows
 * being residual rows entry_base + first .. + len - 1 (first-gid ascending).
 * For key hash h = fmix32(ks ^ kd * 0x9E3779B1 ^ kp * 0x85EBCA77 ^ 0x2545F491) the
 * candidate buckets are ((h & 0xFFFF) * n_buckets) >> 16 and ((h >> 16) *
 * n_buckets) >> 16, the tag ((h >> 16) ^ h) & 0x7FF.  Row filter words (one
 * per bucket row at filter_off + first + i) are slen6 << 26 | dlen6 << 20 |
 * pm2 << 18 | fp18: the low 18 bits of the same hash (seed 0x6A09E667) over
 * the row's exact bits (src, dst under their prefix masks; sport if pm2 bit 0,
 * dport if bit 1).  Exact: no deferred lines. */
#define RSA_BKT_MAGIC 0x35415352u
typedef struct rsa_bkt_table {   /* 32 B */
  uint32_t src_mask, dst_mask, port_mask;
  uint32_t bucket_off;           /* image word offset of the bucket slots (even)   */
  uint32_t n_buckets;            /* 1 .. 65536                                     */
  uint32_t filter_off;           /* image word offset of the row filters (one per bucket row) */
  uint32_t min_gid;              /* smallest first gid of the table's entries      */
  uint32_t entry_base;           /* residual row of the table's first bucket row   */
} rsa_bkt_table;

typedef struct rsa_pht_table {
  uint32_t slot_off;   /* first slot word in the image                           */
  uint32_t disp_off;   /* first displacement, in uint16 units of the image       */
  uint32_t n_slots;    /* table size (slots), >= 1                               */
  uint32_t disp_mask;  /* displacement buckets - 1 (power of two)                */
} rsa_pht_table;

typedef struct rsa_pht_group {   /* 80 B */
  uint32_t src_mask, dst_mask;
  uint32_t min_idx;          /* smallest record-local entry index in the group    */
  uint32_t class_mask;       /* bit c: port class c has a real table (else it points at word 0) */
  rsa_pht_table table[4];    /* port classes any, dport, sport, sport+dport       */
} rsa_pht_group;

#define RSA_PHT_NARROW 0x80000000u   /* rsa_pht_mask.slot: 16-bit slots */
typedef struct rsa_pht_mask {    /* 16 B: one pruning table (src tables first: rsa_pht_list.n_src_masks) */
  uint32_t mask;             /* address mask (non-zero)                           */
  uint32_t slot;             /* slot_off | RSA_PHT_NARROW: uint16 slots (H & 0xFF) << 8 | value,
                                slot_off in uint16 units, values 1..255; else uint32
                                slots (H & 0xFFFF) << 16 | value; 0 = empty (value 0) */
  uint32_t disp_off;         /* first displacement, uint16 units                  */
  uint32_t size;             /* n_slots | disp_mask << 17; slot value = bitmap index */
} rsa_pht_mask;

typedef struct rsa_pht_list {    /* 80 B: one list (or one chained chunk of a list) */
  uint32_t group_off, n_groups;  /* rsa_pht_group records (image word offset)     */
  uint32_t mask_off, n_masks;    /* rsa_pht_mask records                          */
  uint32_t resid_beg, resid_end; /* this record's residual entries               */
  uint32_t prefix;               /* entries scanned linearly before the index (first record only) */
  uint32_t bm_off;               /* uint64 bitmaps (image word offset, even)     */
  uint32_t src_any_lo, src_any_hi, dst_any_lo, dst_any_hi;
  uint32_t entry_beg, entry_len; /* this record's entries in rsa_load_rules' entries */
  uint32_t n_bitmaps;
  uint32_t after_min;            /* smallest gid of the list's entries >= prefix (RSA_PHT_NONE: none) */
  uint32_t next;                 /* continuation record, or RSA_PHT_NONE           */
  uint32_t next_min;             /* smallest gid of the continuation chunk          */
  uint32_t n_src_masks;          /* mask records [0, n_src_masks) are src tables, the rest dst */
  uint32_t reserved;
} rsa_pht_list;

/* Options (rsa_set_option). */
#define RSA_OPT_AUTO_FILTER 1 /* split a large first batch to derive the exact per-rule insert filter (default 1) */
#define RSA_OPT_USE_INDEX 2   /* classify with the loaded index (1) or the linear lists (0)                  */
#define RSA_OPT_FILTER_SLICE 5 /* auto filter: first 1/N (>= 1M lines) of a large batch builds the bound (default 256)       */
#define RSA_OPT_FILTER_STEPS 7 /* auto filter: bound refinements, each after RSA_OPT_FILTER_GROWTH x the previous lines (default 3) */
#define RSA_OPT_FILTER_GROWTH 24 /* auto filter: lines of each bound refinement's slice over the previous ones (default 4) */
#define RSA_OPT_CLASSIFY_PAIR 28 /* the global-memory bucket index (lists too large for LDS) classifies two lines per lane (1, default) or one (0) */
#define RSA_OPT_COUNTER_WORDS16 26 /* 16-bit gid|hit words between classification and counting when every gid fits 15 bits and the LDS histogram holds the rules (1, default) */
#define RSA_OPT_ROUTE_ROWS 29 /* TESTING: rsa_merge starts every routed export in a buffer of this many rows (0, default: the rows the last merge needed) -- forces the re-export path */
#define RSA_OPT_FORCE_DEFER 8  /* TESTING: every index candidate goes to the exact deferred-line path        */
#define RSA_OPT_PROFILE_SKIP 3 /* PROFILING ONLY, results invalid: bit0 skips counters, bit1 skips the table, bit2 skips table updates */
#define RSA_OPT_PRECHECK 9     /* pre-check monotone slot fields with a plain load before their atomics (default 1)       */
#define RSA_OPT_WAVE_CAP_SCATTER 11 /* TESTING: cap scatter by wave grouping (the path for > 16384 capped rules) */
#define RSA_OPT_GROUP_TASKS 12 /* index lookup: candidate groups dealt out over the wave (1, default) or per-lane loops (0) */
#define RSA_OPT_PROFILE_CLASSIFY 13 /* PROFILING ONLY, results invalid: bit0 no index lookup, bit1 pruning only (bucket index: probes only), bit2 no verification (bucket: no serial fallback) */
#define RSA_OPT_STATS 10       /* PROFILING: count table work into the rsa_stats counters (default 0)                 */
#define RSA_OPT_HOT_SPLIT 14   /* pre-combine regions holding > max(RSA_OPT_HOT_MIN, 4 x mean) records on all CUs (default 1) */
#define RSA_OPT_HOT_MIN 15     /* hot-region minimum in records (default 65536; below it TESTING: any region above it is hot) */
#define RSA_OPT_PARSE_STAGED 16 /* TESTING: the text parse stages each workgroup's lines in LDS (1) instead of register-window
                                   16-byte HBM reads (0, default; text that is not 16-byte aligned is always staged) */
#define RSA_OPT_REGION_IMPORT 17 /* rsa_import: records sorted by table region, merged per region in LDS (1, default) or device atomics per record (0) */
#define RSA_OPT_OWNER_WORLD 19   /* multi-GPU merge (0 = off): the ctx's table also holds the merged entries of the rules it owns (gid % world == rank); rsa_export leaves those at home, rsa_emit returns only those */
#define RSA_OPT_OWNER_RANK 20    /* this ctx's rank for RSA_OPT_OWNER_WORLD */
#define RSA_OPT_MIN_REGIONS_LOG2 21 /* table regions: at least 2^v of them (one k_reduce workgroup each) while a region keeps >= 1024 slots (default 10); takes effect at rsa_reset */
#define RSA_OPT_REGION_RECORDS 22 /* table regions: at least the previous job's pass-1 record count / v of them (rounded up to a power of two, at most 4096; 0 = off; default 49152): more k_reduce workgroups for record-heavy jobs; takes effect at rsa_reset */
#define RSA_OPT_REDUCE_BIG 23 /* pass-1 merges of jobs with more than 1024 table regions through a 4096-entry LDS table (1, default) instead of 3072 (0); takes effect per pass-1 launch */
#define RSA_OPT_COUNT_SORT 18    /* rule sets past the LDS counters (> 13312 rules): per-rule line/hit counters by a counting sort of the lines by rule block and LDS histograms (1, default) or one device atomic per line (0) */

/* One distinct (rule, connection) aggregate, 40 B (connlist-reducer.py:162-176). */
typedef struct rsa_conn_record {
  uint64_t min_order; /* smallest order key (first occurrence in sort order) */
  uint32_t gid;
  uint32_t for_ip;    /* reducer key FROMIP                                   */
  uint32_t to_ip;     /* reducer key TOIP                                     */
  uint16_t to_port;   /* reducer key TOPORT                                   */
  uint8_t pspell;     /* reducer key PROTO (spelling id)                      */
  uint8_t pad;
  uint32_t count;     /* conns[conn]                                          */
  uint32_t first;     /* connFirst[conn] as an order-isomorphic timestamp code */
  uint32_t last;      /* connLast[conn]                                       */
  uint32_t pad2;
} rsa_conn_record;

typedef struct rsa_ctx rsa_ctx;

/* Context: one per device.  Replaces the per-process setup of mapper.py:79-117
 * and connlist-reducer.py:32-49 (the rule DB lives in HBM instead). */
int rsa_ctx_create(int device, rsa_ctx **out);
int rsa_ctx_destroy(rsa_ctx *ctx);
const char *rsa_last_error(const rsa_ctx *ctx);
int rsa_set_stream(rsa_ctx *ctx, void *hip_stream);
int rsa_set_option(rsa_ctx *ctx, int option, int64_t value);
int rsa_version(void);

/* Upload compiled candidate lists (host arrays).  list_offsets has n_lists+1
 * entries; entries[list_offsets[l] .. list_offsets[l+1]) is list l in ascending
 * gid order.  Replaces mapper.py:159-166 (candidate list per line).  n_rules is
 * the number of global rule ids (counter length). */
int rsa_load_rules(rsa_ctx *ctx, const rsa_rule_entry *h_entries, uint32_t n_entries,
                   const uint32_t *h_list_offsets, uint32_t n_lists, uint32_t n_rules);

/* Upload a pruned perfect-hash tuple-space index image over the lists of
 * rsa_load_rules (same list ids) and its residual entries.  Enables
 * RSA_OPT_USE_INDEX.  Every record, offset, table and slot value is validated
 * against the image and the loaded lists, so no kernel can read out of bounds. */
int rsa_load_index(rsa_ctx *ctx, const uint32_t *h_image, uint32_t image_words, const rsa_rule_entry *h_resid,
                   uint32_t n_resid);

/* Bind caller-owned device counters, each n_rules long (n_rules from
 * rsa_load_rules, or rsa_set_rule_count when no rules are loaded):
 *   d_matches  uint64  mapper-emitted lines per rule (blocks exist iff > 0)
 *   d_hits     uint64  "Total number of hits" (connlist-reducer.py:146-148)
 *   d_distinct uint32  distinct connections inserted per rule
 *   d_thresh   uint64  cap threshold P per rule, RSA_NO_THRESHOLD if uncapped */
int rsa_bind_counters(rsa_ctx *ctx, uint64_t *d_matches, uint64_t *d_hits, uint32_t *d_distinct,
                      uint64_t *d_thresh);
int rsa_set_rule_count(rsa_ctx *ctx, uint32_t n_rules);

/* (Re)initialise the distinct-connection table with room for `capacity`
 * distinct (rule, connection) pairs, zero the bound counters and set the
 * per-rule cap (config.py:15 MAX_NUMBER_OF_CONNECTIONS_PER_RULE).  `capacity`
 * is an upper bound: it is clamped to the largest table (4096 regions of 65536
 * slots at 2/3 load, ~179M entries); more distinct entries than the table holds
 * fail the job with RSA_ERR_CAPACITY. */
int rsa_reset(rsa_ctx *ctx, uint64_t capacity, uint32_t cap);

/* Pass 1 — classify + aggregate a batch resident in HBM (mapper.py:123-189 fused
 * with connlist-reducer.py:62-176).  d_ts: uint32 order-isomorphic timestamp
 * codes; d_order: uint64 unique order keys isomorphic to the reducer's input
 * order (LC_ALL=C sort of the line within its key).  d_gid_out (nullable)
 * receives the first-match gid or RSA_NO_RULE per tuple. */
int rsa_classify(rsa_ctx *ctx, const rsa_tuple *d_tuples, const uint32_t *d_ts, const uint64_t *d_order,
                 uint64_t n, int32_t *d_gid_out);

/* Classification only: first-match gid per tuple, no aggregation (the mapper
 * drop-in, mapper.py:159-189).  Needs rsa_load_rules; no counters/table. */
int rsa_classify_only(rsa_ctx *ctx, const rsa_tuple *d_tuples, uint64_t n, int32_t *d_gid_out);

/* Pass 1 with the rule already known per tuple (the reducer drop-in: the key
 * comes from the mapper's output line, connlist-reducer.py:63-75). */
int rsa_aggregate_gids(rsa_ctx *ctx, const rsa_tuple *d_tuples, const uint32_t *d_ts, const uint64_t *d_order,
                       const int32_t *d_gid, uint64_t n);

/* Device time (ms, HIP events on the ctx stream) of the pass-1 kernel launches
 * of the last rsa_classify / rsa_aggregate_gids call (waits for them). */
int rsa_last_pass1_ms(rsa_ctx *ctx, float *h_ms);
/* The same time split into classification (k_classify + k_tail) and
 * aggregation (k_aggregate) launches. */
int rsa_last_pass1_times(rsa_ctx *ctx, float *h_classify_ms, float *h_aggregate_ms);
/* Number of classification launches (filter slices) of the last pass-1 call. */
int rsa_last_pass1_launches(rsa_ctx *ctx, uint32_t *h_n);

/* Resolve the cap (connlist-reducer.py:151): for every rule with
 * distinct >= cap, P = the order key of the line that inserted the cap-th
 * distinct connection, written to d_thresh.  *h_n_capped receives the number
 * of capped rules (0 means no recount pass is needed).  h_n_capped may be
 * NULL: no host round trip; the count stays on the device and the next
 * rsa_recount of the cached batch skips its work there when it is 0.  Only a
 * NULL resolution arms that skip (a caller that reads the count may rewrite
 * d_thresh before its recount, as the multi-GPU merge does with the global
 * thresholds, so its recount never skips on the local count); the skip is
 * consumed by that recount and disarmed by any other resolution or reset. */
int rsa_resolve_cap(rsa_ctx *ctx, uint32_t *h_n_capped);

/* Pass 2 — recount occurrences with order <= P for capped rules, per batch.
 * d_gid may be the d_gid_out of pass 1, or NULL to re-classify. */
int rsa_recount(rsa_ctx *ctx, const rsa_tuple *d_tuples, const uint32_t *d_ts, const uint64_t *d_order,
                const int32_t *d_gid, uint64_t n);

/* Emit the final connection tables (connlist-reducer.py:108-126 data) into
 * d_out (caller device buffer of `max_records`), unordered.  *h_n receives the
 * number of records; RSA_ERR_CAPACITY if it exceeds max_records. */
int rsa_emit(rsa_ctx *ctx, rsa_conn_record *d_out, uint64_t max_records, uint64_t *h_n);

/* Multi-GPU merge (replaces the Hadoop shuffle, runAnalysis.sh:42-56).
 * rsa_export: every table entry with its pass-1 (which=0) or pass-2 (which=1)
 * aggregates, or (which=2) the pass-1 aggregates of only the entries that can
 * still reach the report after rsa_resolve_cap on this shard's table: rules
 * without a threshold, and entries with min_order <= the shard's P (which is
 * >= the global P, so nothing that can matter is dropped); rsa_import: merge
 * such records into this ctx's table (which=0: insert-or-combine; which=1:
 * combine into the pass-2 fields of existing keys). */
int rsa_table_size(rsa_ctx *ctx, uint64_t *h_n);
int rsa_export(rsa_ctx *ctx, int which, rsa_conn_record *d_out, uint64_t max_records, uint64_t *h_n);
/* The same export routed to the owners (the keyed shuffle of
 * runAnalysis.sh:12,42-56: rules partitioned gid % world, the reducer
 * partitioning): the records of owner r form segment r of d_out (segments in
 * owner order, each unordered inside), d_counts[r] (DEVICE, world uint64)
 * receives its size.  No host round trip: the caller exchanges the device
 * counts and reads send and receive sizes together.  Requires
 * RSA_OPT_OWNER_WORLD == world (1..256); this rank's own segment is empty.
 * Records past max_records are dropped while d_counts keep the true sizes
 * (the caller compares their sum with its capacity). */
int rsa_export_routed(rsa_ctx *ctx, int which, uint32_t world, rsa_conn_record *d_out, uint64_t max_records,
                      uint64_t *d_counts);
int rsa_import(rsa_ctx *ctx, int which, const rsa_conn_record *d_in, uint64_t n);

/* The whole multi-GPU merge behind one call (the reference's
 * keyed shuffle into NUM_REDUCERS reducers and `hadoop dfs -getmerge`,
 * runAnalysis.sh:12,42-56, README.md:35-38).  Every rank has run pass 1 over
 * its own shard on its own ctx (rsa_reset, rsa_classify / rsa_aggregate_gids);
 * rank r owns the rules with gid % world == r.  rsa_merge then runs, on every
 * rank together:
 *   1. SUM all_reduce of the line and hit counters;
 *   2. this shard's cap resolution, and the routed export (rsa_export_routed,
 *      which=2) of the entries other ranks own that can still reach the
 *      report; an all_to_allv of the per-owner counts (with an overflow flag)
 *      and ONE host read of send and receive sizes, then an all_to_allv of the
 *      40-B rows; the owners import them (which=0) and resolve their caps;
 *   3. MAX all_reduce of the owners' thresholds (-1 = none) with the import
 *      overflow need: every rank holds every rule's P in d_thresh;
 *   4. if any rule is capped: the pass-2 recount over h_batches, a routed
 *      export (which=1), the exchange, the owners' import (which=1);
 *   5. rsa_emit of the owned rules' final rows into a ctx buffer, and a SUM
 *      all_reduce of the owned distinct counts (d_distinct) with every rank's
 *      row count;
 *   6. flags & RSA_MERGE_GATHER: the owners' rows to rank 0 (rsa_gather).
 * Afterwards d_matches/d_hits/d_thresh/d_distinct hold the merged counters on
 * every rank.  A distinct-connection table overflow on any rank (pass 1 or the
 * import) returns RSA_ERR_CAPACITY on EVERY rank, with h_info->needed = the
 * entries the fullest table must hold (0 if unknown): rerun the job with
 * rsa_reset at that capacity.  At world 1 no collective runs (the merge is the
 * single-GPU job: resolve, recount if capped, emit) unless flags has
 * RSA_MERGE_ALWAYS_EXCHANGE: then every step runs over the transport anyway
 * (self exchanges; a one-GPU check of a transport, results unchanged).
 *
 * The collectives go through a transport: rsa_merge_rccl binds an RCCL
 * communicator (the path over xGMI); any other collective library (MPI, a
 * host-side TCP group) fills rsa_transport itself.  host_buffers != 0: the
 * callbacks receive pinned HOST buffers (the library stages device data
 * through them) -- a CPU-only collective; else device pointers on `stream`
 * (the ctx stream).  Callbacks return 0 on success. */
typedef struct rsa_transport {
  void *self;
  int32_t world, rank;
  int32_t host_buffers;
  /* in place over n int64: op 0 = sum, 1 = max */
  int (*all_reduce_i64)(void *self, int64_t *buf, uint64_t n, int op, void *stream);
  /* rows to every rank: h_send_bytes[r] bytes, the r-th consecutive segment of
   * send, go to rank r; the h_recv_bytes[r] bytes from rank r land at recv +
   * sum(h_recv_bytes[0..r)).  h_*_bytes are host arrays of world entries. */
  int (*all_to_allv)(void *self, const void *send, const uint64_t *h_send_bytes, void *recv,
                     const uint64_t *h_recv_bytes, void *stream);
} rsa_transport;

typedef struct rsa_shard_batch {   /* one pass-1 batch of this rank's shard (for the pass-2 recount) */
  const rsa_tuple *d_tuples;
  const uint32_t *d_ts;
  const uint64_t *d_order;
  const int32_t *d_gid;            /* pass 1's d_gid_out, or NULL to re-classify */
  uint64_t n;
} rsa_shard_batch;

#define RSA_MERGE_GATHER 1
#define RSA_MERGE_ALWAYS_EXCHANGE 2

typedef struct rsa_merge_info {
  const rsa_conn_record *d_rows;   /* after the gather: on rank 0 every owner's rows in rank order (NULL
                                      elsewhere); else this rank's own rules' rows.  A ctx buffer, valid
                                      until the ctx's next merge or destroy (rsa_merge_rows copies it) */
  uint64_t n_rows;
  uint64_t owner_rows;             /* this rank's own rules' final rows */
  uint64_t gather_rows;            /* rows the gather moves to rank 0 from the other ranks */
  uint64_t route1_sent, route1_self, route1_recv;   /* pass-1 exchange rows (self: kept at home) */
  uint64_t route2_sent, route2_self, route2_recv;   /* pass-2 exchange rows */
  uint64_t allreduce_bytes;        /* payload of the counter, threshold and size all_reduces */
  uint64_t needed;                 /* RSA_ERR_CAPACITY: entries the fullest table must hold (0: unknown) */
  uint32_t reexports;              /* exports repeated because the route buffer was too small */
  uint32_t pass2;                  /* 1 if some rule was capped (the recount ran) */
} rsa_merge_info;

int rsa_merge(rsa_ctx *ctx, const rsa_transport *t, const rsa_shard_batch *h_batches, uint32_t n_batches,
              int flags, rsa_merge_info *h_info);
/* The owners' rows of the last rsa_merge to rank 0 (every rank calls it; the
 * sizes are known from the merge, no extra collective): h_info->d_rows /
 * n_rows become rank 0's gathered rows (NULL / 0 elsewhere). */
int rsa_gather(rsa_ctx *ctx, const rsa_transport *t, rsa_merge_info *h_info);
/* Copy rows of the last merge into d_out (device, max_records rows): which 0 =
 * this rank's own rules' rows, 1 = the last gather's rows (rank 0).  *h_n
 * receives the count; RSA_ERR_CAPACITY if it exceeds max_records. */
int rsa_merge_rows(rsa_ctx *ctx, int which, rsa_conn_record *d_out, uint64_t max_records, uint64_t *h_n);

/* RCCL (over xGMI) as the transport.  The library resolves RCCL at run time
 * (the librccl already loaded in the process, else librccl.so.1).  Rank 0
 * makes a unique id, the caller broadcasts its 128 bytes by any means, every
 * rank creates its communicator on the ctx's device; one communicator serves
 * any number of merges. */
int rsa_rccl_unique_id(uint8_t h_id[128]);
int rsa_rccl_comm_create(rsa_ctx *ctx, int32_t world, int32_t rank, const uint8_t h_id[128], void **comm);
int rsa_rccl_comm_destroy(void *comm);
int rsa_merge_rccl(rsa_ctx *ctx, void *comm, const rsa_shard_batch *h_batches, uint32_t n_batches, int flags,
                   rsa_merge_info *h_info);
int rsa_gather_rccl(rsa_ctx *ctx, void *comm, rsa_merge_info *h_info);

/* Profiling counters (collected while RSA_OPT_STATS is on): h_out[0] lines
 * combined into the table, [1] probes beyond a line's home slot, [2] probes that
 * took the atomic (claim) path, [3] slot-field atomics issued.  reset != 0
 * zeroes them after the read. */
int rsa_stats(rsa_ctx *ctx, uint64_t *h_out4, int reset);

/* Shadowed-rule analysis (preprosess_access_lists.py:508-521): for every rule i
 * of one access list, the smallest j < i whose rule CONTAINS rule i
 * (FirewallRule.__contains__, firewallrule.py:128-174: equal action, protocol
 * 'ip' or equal, src and dst networks contained, ports "no port" or equal), or
 * -1.  Rules are given in list order; one port per side (the preprocessors'
 * expansion, SURVEY.md trap 3).  Host buffers in and out. */
typedef struct rsa_shadow_rule {
  uint32_t src_lo, src_span;  /* IPv4 network [lo, lo + span] (IPv6: interval code)  */
  uint32_t dst_lo, dst_span;
  int32_t sport, dport;       /* one port, -1 = NO_PORT, <= -2 a list (rsa_shadowed_ports) */
  uint16_t proto;             /* protocol id, 0 = 'ip'                              */
  uint8_t action;             /* 1 permit, 0 deny                                   */
  uint8_t v4;                 /* address family code: 1 both IPv4; 3/4/5 = 2 + (src IPv6) + 2 x (dst IPv6),
                                 the IPv6 sides as containment-preserving interval codes; only rules of
                                 one code compare; 0 never contains / is contained */
  uint32_t reserved;
} rsa_shadow_rule;
int rsa_shadowed(rsa_ctx *ctx, const rsa_shadow_rule *h_rules, uint32_t n, int32_t *h_cover);
/* The same for rules whose port sides may be lists: a side <= -2 names the list
 * h_ports[-side - 2] = count, followed by its ports (firewallrule.py:162-171:
 * every port of the other rule's list must be in this rule's list). */
int rsa_shadowed_ports(rsa_ctx *ctx, const rsa_shadow_rule *h_rules, uint32_t n, const int32_t *h_ports,
                       uint32_t n_ports, int32_t *h_cover);

/* ---- Text parse: one firewall's log text resident in
 * HBM -> the packed inputs of rsa_classify.  Replaces the per-line Python of
 * mapper.py:123-166 (get_builtconn, Connection, ACL of the ingress interface,
 * candidate list) and connlist-reducer.py:146-165 (hit test, BUILT regex, key,
 * timestamp).  Lines end at '\n' (the terminator belongs to its line; a final
 * line may lack it).  The device parses the canonical grammar of the ASA
 * "Built {inbound,outbound} {TCP,UDP}" message and of the reducer's BUILT
 * regex (Python `re` backtracking order restated: lazy `.*?`, greedy `.*`,
 * leftmost search); a line outside it (non-canonical address/port text, an
 * unknown protocol spelling, a timestamp outside the code range, an interface
 * whose lookup raises) is marked RSA_LINE_HOST and the host parser decides it. */
#define RSA_LINE_IGNORE 0   /* no Built message: the mapper skips the line (mapper.py:124-126)   */
#define RSA_LINE_NOACL 1    /* ingress interface without ACL (mapper.py:145-150)                 */
#define RSA_LINE_MISSING 2  /* ACL missing from the DB (mapper.py:151-156); disp >> 8 = interface */
#define RSA_LINE_CLASSIFY 3 /* tuple valid: classify it                                         */
#define RSA_LINE_HOST 4     /* outside the device grammar: the host parser decides              */
#define RSA_LIST_HOST 0xFFFFu /* rsa_parse_ifc list id: the host decides (list lookup raises)    */
#define RSA_IFC_NAME_MAX 47

/* One interface of the firewall (db.firewalls[host]), 64 B. */
typedef struct rsa_parse_ifc {
  char name[48];               /* name bytes (len <= RSA_IFC_NAME_MAX)                        */
  uint32_t len;
  uint32_t kind;               /* RSA_LINE_CLASSIFY, RSA_LINE_MISSING or RSA_LINE_HOST       */
  uint16_t list_tcp, list_udp; /* candidate list ids (kind CLASSIFY), or RSA_LIST_HOST         */
  uint32_t reserved;
} rsa_parse_ifc;

/* One protocol spelling of the reducer key (connlist-reducer.py:155), 16 B;
 * its index in the table is the rsa_tuple.pspell id. */
typedef struct rsa_parse_spell {
  char word[15];
  uint8_t len;
} rsa_parse_spell;

/* Timestamp codes written by rsa_parse_text, order-isomorphic to the reducer's
 * 'YYYY-MM-DD HH:MM:SS' strings (connlist-reducer.py:163-165) for years
 * 2000..2127: ((((Y - 2000) * 12 + M - 1) * 32 + D) * 86400 + h * 3600 + m * 60 + s. */
#define RSA_TS_YEAR0 2000

/* Number of lines of text[0, n_bytes). */
int rsa_text_count_lines(rsa_ctx *ctx, const uint8_t *d_text, uint64_t n_bytes, uint64_t *h_n_lines);
/* Line start offsets: d_off[0 .. n_lines] (d_off[n_lines] = n_bytes). */
int rsa_text_line_offsets(rsa_ctx *ctx, const uint8_t *d_text, uint64_t n_bytes, uint64_t *d_off, uint64_t n_lines);
/* Both in one pass over the text: *h_n_lines = number of lines; when it is
 * <= max_lines, d_off[0 .. n_lines] as rsa_text_line_offsets writes them,
 * else RSA_ERR_CAPACITY (d_off unspecified; retry with room for *h_n_lines + 1
 * offsets). */
int rsa_text_split(rsa_ctx *ctx, const uint8_t *d_text, uint64_t n_bytes, uint64_t *d_off, uint64_t max_lines,
                   uint64_t *h_n_lines);
/* Parse every line: d_tuples (zero unless CLASSIFY), d_ts (codes, 0 unless
 * hit+BUILT), d_disp (RSA_LINE_* | interface index << 8).  h_ifcs / h_spells are
 * host tables (n_ifcs <= 4096, n_spells <= 64). */
int rsa_parse_text(rsa_ctx *ctx, const uint8_t *d_text, const uint64_t *d_off, uint64_t n_lines,
                   const rsa_parse_ifc *h_ifcs, uint32_t n_ifcs, const rsa_parse_spell *h_spells, uint32_t n_spells,
                   rsa_tuple *d_tuples, uint32_t *d_ts, uint32_t *d_disp);
/* Order keys: d_order[i] = base + rank of line i (without its '\n') in unsigned
 * byte order, ties by line index — the order LC_ALL=C sort gives the reducer
 * within one key (runAnalysis.sh:42-56).  Device string sort: 7-byte chunks,
 * groups refined by radix sorts until every line is settled. */
int rsa_order_keys(rsa_ctx *ctx, const uint8_t *d_text, const uint64_t *d_off, uint64_t n_lines, uint64_t base,
                   uint64_t *d_order);
/* Order keys within groups: d_order[i] = base + rank of (d_group[i], line i's
 * bytes), for the lines with d_group[i] >= 0 (the others get distinct ranks
 * after them).  The reducer compares order keys of ONE rule's lines only (its
 * cap point and first-seen order, connlist-reducer.py:151,167-176), so with the
 * line's rule as its group the keys are exact, and lines of different rules
 * are never compared: most groups are settled by the timestamp prefix. */
int rsa_order_keys_grouped(rsa_ctx *ctx, const uint8_t *d_text, const uint64_t *d_off, uint64_t n_lines,
                           const int32_t *d_group, uint64_t base, uint64_t *d_order);

/* ---- Reducer drop-in parse: the sorted mapper stream ("host;acl;idx\t<log line>"
 * per line) resident in HBM -> the per-line inputs of rsa_aggregate_gids.
 * Replaces the per-line Python of connlist-reducer.py:62-79,146-165: strip,
 * split('\t', 1), the hit test and the BUILT regex on the value, key and
 * timestamp.  Per line: d_disp = RSA_RED_KEYED (d_tuples: src = FROMIP, dst =
 * TOIP, dport = TOPORT, pspell, flags RSA_F_HIT / RSA_F_BUILT; d_ts the code
 * when hit+BUILT), RSA_RED_NOISE (no tab after strip: the reducer's "Unable to
 * unpack" line), or RSA_LINE_HOST (outside the device grammar: non-canonical
 * address/port text, an unknown protocol spelling, a timestamp outside the code
 * range); | RSA_RED_SAME_KEY when the line's key bytes equal the previous
 * line's (both keyed).  Key validity (split(';'), int(), DB lookup) is decided
 * by the host once per run of equal keys. */
#define RSA_RED_KEYED 0
#define RSA_RED_NOISE 1
#define RSA_RED_SAME_KEY 0x100u
int rsa_parse_reduce(rsa_ctx *ctx, const uint8_t *d_text, const uint64_t *d_off, uint64_t n_lines,
                     const rsa_parse_spell *h_spells, uint32_t n_spells, rsa_tuple *d_tuples, uint32_t *d_ts,
                     uint32_t *d_disp);

/* Synchronise the ctx stream (tests, host hand-off). */
int rsa_sync(rsa_ctx *ctx);

#ifdef __cplusplus
}
#endif

#endif /* RULESET_HIP_H */
