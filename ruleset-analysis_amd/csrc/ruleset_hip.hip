// ruleset_hip.hip — MI355X (gfx950, CDNA4) hot path of ruleset-analysis.
//
// What the reference does per log line (Python 2, one process per Hadoop split):
//   mapper.py:159-189           build the candidate rule list, scan it with
//                               FirewallRule.__contains__ (firewallrule.py:128-174),
//                               emit the FIRST matching expanded rule index;
//   connlist-reducer.py:62-176  per rule: count lines, count "hits"
//                               (-6-302013/-6-302015), keep a distinct-connection
//                               dict capped at MAX_NUMBER_OF_CONNECTIONS_PER_RULE
//                               (config.py:15), in sorted-line order.
//
// What this library does instead (integer work; HBM/atomic/VALU bound; no MFMA):
//   classify  one lane per tuple, waves "waterfall" over the distinct candidate
//             lists present (list id broadcast by readlane, so rule data is
//             wave-uniform: scalar loads).  Per list: a linear scan of the first
//             `prefix` entries with wave-level early exit (short first matches
//             never go further), then a perfect-hash tuple-space index staged in
//             LDS: per rule shape (src mask, dst mask, port mask) one CHD
//             (hash-and-displace) table maps the masked key to the smallest list
//             index with that key; the lane keeps the minimum candidate, verifies
//             it against the full entry (the 16-bit tag may collide) and scans the
//             few residual entries.  A failed verification defers the line to an
//             exact linear scan.  The answer is the minimum matching gid = the
//             reference's first match.
//   pass 1    per-line gid|hit words (then an LDS-privatised histogram gives the
//             per-rule line/hit counters) and an open-addressing (rule,
//             connection) table in HBM keyed by device atomics; new entries are
//             appended to a compact used-slot list.
//   filter    after the first slice of a large batch, each rule that already has
//             >= cap connections gets an exact upper bound F of its threshold;
//             later lines with order > F cannot change any output and skip the
//             table.
//   cap       P = cap-th smallest first-seen order of a rule (two LSD radix
//             sorts of the capped entries), the reducer's frozen-dict point.
//   pass 2    recount (count/first/last) of occurrences with order <= P for the
//             capped rules only.
//   emit      compact the used slots to rsa_conn_record rows.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ruleset_hip.h"
#include "rsa_internal.h"

namespace {

constexpr unsigned long long kEmpty = 0xFFFFFFFFFFFFFFFFull;
constexpr unsigned long long kBusy = 0xFFFFFFFFFFFFFFFEull;
constexpr uint32_t kNoGid = 0xFFFFFFFFu;
constexpr int kBlock = 256;

// One distinct (rule, connection) aggregate in HBM, 64 B.
// min_order, first and last share one 16-B group so that a single vector load
// can pre-check all three monotone fields.
struct alignas(64) Slot {
  unsigned long long kA;         // for_ip << 32 | to_ip
  unsigned long long kB;         // gid << 32 | pspell << 16 | to_port ; kEmpty / kBusy
  unsigned long long min_order;  // first occurrence (reducer input order)
  unsigned int first, last;      // pass-1 timestamp range
  unsigned int count;            // pass-1 occurrences
  unsigned int count2, first2, last2;   // pass-2 aggregates (order <= P only)
  unsigned int pad[4];           // pad[0]: the entry's used-list index (region path)
};
static_assert(sizeof(Slot) == 64, "slot layout");
static_assert(offsetof(Slot, first) % 8 == 0 && offsetof(Slot, last) == offsetof(Slot, first) + 4,
              "first/last form one 8-B word");
static_assert(sizeof(rsa_tuple) == 16, "tuple layout");
static_assert(sizeof(rsa_rule_entry) == 32, "rule layout");
static_assert(sizeof(rsa_pht_group) == 80, "group layout");
static_assert(sizeof(rsa_pht_mask) == 16, "mask layout");
static_assert(sizeof(rsa_pht_list) == 80, "list record layout");
static_assert(sizeof(rsa_conn_record) == 40, "record layout");

// Rule data is read through the constant address space so that wave-uniform
// loads become scalar (s_load) loads through the scalar cache.
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(4))) const v4u const_v4u;
typedef __attribute__((address_space(4))) const uint32_t const_u32;

struct Rules {
  const const_v4u* e;           // linear entries, 2 x v4u each (gid-ascending per list)
  const v4u* eg;                // the same entries for per-lane (divergent) loads
  const const_u32* off;         // n_lists + 1
  uint32_t n_lists;
  uint32_t n_rules;
  // pruned perfect-hash tuple-space index (optional): one uint32 image
  // (include/ruleset_hip.h) holding list, group and mask records, bitmaps and
  // the CHD tables; read per lane (LDS copy or global)
  const const_v4u* resid;       // residual entries (gid-ascending per list)
  const uint32_t* img;          // the image (global copy)
  uint32_t img_words;
  uint32_t list_off;            // word offset of the list records
  int indexed;
  int force_defer;              // testing: every index candidate takes the exact deferred path
  int group_tasks;              // RSA_OPT_GROUP_TASKS: candidate groups dealt out over the wave (index_lookup_wave)
  int prof;                     // RSA_OPT_PROFILE_CLASSIFY (results invalid): 1 no lookup, 2 pruning only, 4 no verification
  int bkt;                      // the image is the partial-key bucket index (RSA_BKT_MAGIC): bucket_lookup
  int bkt_filters;              // ... with LDS row filters (image word 5 bit 0)
  const v4u* residg;            // residual + bucket entries for per-lane (divergent) loads
};

struct Agg {
  unsigned long long* matches;
  unsigned long long* hits;
  unsigned long long* packed;        // per rule, rules beyond the LDS histogram: hits << 32 | lines of one launch
  unsigned int* distinct;
  const unsigned long long* thresh;
  const unsigned long long* filter;  // per rule: lines with order > filter cannot matter
  Slot* slots;
  unsigned long long mask;           // capacity - 1 (power of two)
  unsigned long long* used;          // used-slot list: gid << 32 | slot
  unsigned long long* used_n;
  unsigned long long* ukey;          // per used-list index: the entry's current min_order (kept by k_reduce<1>;
                                     // the slot's pad[0] holds its used-list index)
  unsigned int* flags;               // [0] overflow, [1] bad gid/list/state
  uint32_t cap;
  uint32_t skip;                     // profiling only (RSA_OPT_PROFILE_SKIP): 1 counters, 2 table, 4 table updates
  uint32_t precheck;                 // RSA_OPT_PRECHECK: plain-load pre-check of the monotone slot fields
  unsigned long long* stats;         // RSA_OPT_STATS: [0] table lines, [1] extra probes, [2] atomic-path probes, [3] atomics
  uint32_t* occ;                     // occupancy bitmap of the slots (one bit per slot)
  uint32_t rs_bits;                  // region = 2^rs_bits slots (linear probing wraps inside a region)
  uint32_t np_bits;                  // 2^np_bits regions; a key's region = top np_bits of its slot hash
  uint32_t tent2;                    // pass 1's last slice: records of rules under a filter bound also go
                                     // into the pass-2 fields (exact when the final threshold equals the bound)
};

__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

__device__ __forceinline__ unsigned long long slot_hash(unsigned long long kA, unsigned long long kB) {
  return mix64(kA ^ (kB * 0x9e3779b97f4a7c15ull));
}

// counter[key] += 1 for every lane with `ok`: the lanes sharing the key of the
// first such lane are counted with one atomic (a rule that dominates the wave),
// every other lane adds its own (device atomics on distinct addresses proceed
// in parallel; a full waterfall would serialise up to 64 rounds on waves whose
// keys are all different, the common case for fresh table entries).
// Wave-uniform control flow.
template <typename T>
__device__ __forceinline__ void wave_count_hot(bool ok, uint32_t key, T* counter) {
  const unsigned long long pending = __ballot(ok);
  if (!pending) return;
  const int leader = __builtin_ctzll(pending);
  const uint32_t k = __builtin_amdgcn_readlane(key, leader);
  const unsigned long long peers = __ballot(ok && key == k);
  if ((int)__lane_id() == leader) atomicAdd(&counter[k], (T)__popcll(peers));
  if (ok && key != k) atomicAdd(&counter[key], (T)1);
}

// Home slot of a key hash: region = top np_bits, offset = low rs_bits.
__device__ __forceinline__ unsigned long long slot_home(const Agg& A, unsigned long long hh) {
  const unsigned long long r = A.np_bits ? (hh >> (64 - A.np_bits)) : 0ull;
  return (r << A.rs_bits) | (hh & ((1ull << A.rs_bits) - 1ull));
}

__device__ __forceinline__ unsigned long long slot_next(const Agg& A, unsigned long long s) {
  const unsigned long long m = (1ull << A.rs_bits) - 1ull;
  return (s & ~m) | ((s + 1ull) & m);
}

// Reducer key of a tuple (connlist-reducer.py:162: PROTO;FROMIP;TOIP;TOPORT).
__device__ __forceinline__ void conn_key(uint4 t, uint32_t gid, unsigned long long& kA, unsigned long long& kB) {
  const uint32_t flags = (t.w >> 16) & 0xFFu;
  const uint32_t pspell = t.w >> 24;
  const bool swap = flags & RSA_F_SWAP;
  const uint32_t for_ip = swap ? t.y : t.x;
  const uint32_t to_ip = swap ? t.x : t.y;
  const uint32_t to_port = swap ? (t.z & 0xFFFFu) : (t.z >> 16);
  kA = ((unsigned long long)for_ip << 32) | to_ip;
  kB = ((unsigned long long)gid << 32) | ((unsigned long long)pspell << 16) | to_port;
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// NB: bit-cast a *value*: hipcc (ROCm 7.2) miscompiles __builtin_bit_cast applied
// directly to an ext-vector element lvalue such as b.y (it reads element 0).
__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }

// The integer form of FirewallRule.__contains__ for a compiled entry
// (firewallrule.py:154-171; action/protocol are settled at compile time):
// IPy containment as unsigned range tests, both port ranges at once with packed
// 16-bit arithmetic ((p - lo) <= span per half  <=>  min(d, span) == d).
__device__ __forceinline__ bool entry_match(v4u a, v4u b, uint32_t src, uint32_t dst, uint32_t ports) {
  const uint32_t lo = b.x, span = b.y;
  const u16x2 d = as_u16x2(ports) - as_u16x2(lo);
  const u16x2 m = __builtin_elementwise_min(d, as_u16x2(span));
  return ((src - a.x) <= a.y) & ((dst - a.z) <= a.w) & (as_u32(m) == as_u32(d));
}

// gid a matching entry assigns to the connection: the entry's gid, or for a
// run entry (step != 0) the rule of the run holding the connection's port,
// gid + (p - lo) * stride (include/ruleset_hip.h rsa_rule_entry).
__device__ __forceinline__ uint32_t entry_gid(v4u b, uint32_t ports) {
  const uint32_t st = b.w;
  const bool on_sport = st & RSA_STEP_SPORT;
  const uint32_t p = on_sport ? (ports & 0xFFFFu) : (ports >> 16);
  const uint32_t lo = on_sport ? (b.x & 0xFFFFu) : (b.x >> 16);
  return b.z + (p - lo) * (st & ~RSA_STEP_SPORT);
}

// Linear first-match scan of entries [beg, end) for the `mine` lanes.  Entries
// are in ascending first-gid order and an entry never yields a gid below its
// own, so the wave stops once no searching lane's best exceeds the first gid
// of the entries still ahead.
__device__ __forceinline__ uint32_t scan_list(const const_v4u* E, uint32_t beg, uint32_t end, bool mine, uint32_t best,
                                              uint32_t src, uint32_t dst, uint32_t ports) {
  uint32_t e = beg;
  const const_v4u* p = E + 2 * (size_t)beg;
  for (; e + 4 <= end; e += 4, p += 8) {
    const v4u a0 = p[0], b0 = p[1], a1 = p[2], b1 = p[3], a2 = p[4], b2 = p[5], a3 = p[6], b3 = p[7];
    const uint32_t c0 = entry_match(a0, b0, src, dst, ports) ? entry_gid(b0, ports) : kNoGid;
    const uint32_t c1 = entry_match(a1, b1, src, dst, ports) ? entry_gid(b1, ports) : kNoGid;
    const uint32_t c2 = entry_match(a2, b2, src, dst, ports) ? entry_gid(b2, ports) : kNoGid;
    const uint32_t c3 = entry_match(a3, b3, src, dst, ports) ? entry_gid(b3, ports) : kNoGid;
    if (mine) best = min(best, min(min(c0, c1), min(c2, c3)));
    if (__ballot(mine && best > b3.z) == 0) return best;
  }
  for (; e < end; ++e, p += 2) {
    const v4u a = p[0], b = p[1];
    if (mine && entry_match(a, b, src, dst, ports)) best = min(best, entry_gid(b, ports));
  }
  return best;
}

constexpr uint32_t kDefer = 0xFFFFFFFEu;   // the index candidate failed verification: exact scan later
constexpr uint32_t kNoCand = 0xFFFFu;
constexpr int kImgSmallMax = 19456;   // LDS image words that still allow two 1024-thread workgroups per CU (2 x 76 KiB)

// murmur3 finaliser; must equal compile.py fmix32.
__device__ __forceinline__ uint32_t fmix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}
constexpr uint32_t kSaltS = 0x9E3779B9u, kSaltD = 0x7F4A7C15u, kSaltP = 0x2545F491u;

// Index image reads: the LDS copy through address-space-3 pointers (ds_read),
// the global copy through plain pointers.
typedef __attribute__((address_space(3))) const uint32_t lds_u32;
typedef __attribute__((address_space(3))) const uint16_t lds_u16;
typedef __attribute__((address_space(3))) const v4u lds_v4u;
__device__ __forceinline__ v4u rd4(const lds_u32* img, uint32_t w) { return *reinterpret_cast<const lds_v4u*>(img + w); }
__device__ __forceinline__ v4u rd4(const uint32_t* img, uint32_t w) { return *reinterpret_cast<const v4u*>(img + w); }
__device__ __forceinline__ uint32_t rd16(const lds_u32* img, uint32_t h) { return reinterpret_cast<const lds_u16*>(img)[h]; }
typedef unsigned int v2u __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) const v2u lds_v2u;
// two consecutive words at an even word offset: one ds_read_b64 (64 banks,
// half the LDS cycles of the ds_read2_b32 pair)
__device__ __forceinline__ v2u rd2(const lds_u32* img, uint32_t w) { return *reinterpret_cast<const lds_v2u*>(img + w); }
__device__ __forceinline__ v2u rd2(const uint32_t* img, uint32_t w) { return *reinterpret_cast<const v2u*>(img + w); }
__device__ __forceinline__ uint32_t rd16(const uint32_t* img, uint32_t h) { return reinterpret_cast<const uint16_t*>(img)[h]; }

// CHD slot (compile.py pht_slot): x = (H + d * ((H >> 16) | 1)) mod 2^16,
// slot = (x * n_slots) >> 16.  All operands fit the 24-bit multiplier
// (n_slots <= 2^16), so both products are full-rate v_mad/v_mul_u32_u24
// (the 32-bit v_mul_lo/hi and v_mad_u64 they replace issue at quarter rate).
// NB: HIP's __umul24 returns a SIGNED int: a product >= 2^31 (x * n_slots with
// n_slots > 2^15) must be shifted as unsigned, or the slot index goes negative.
__device__ __forceinline__ uint32_t umul24(uint32_t a, uint32_t b) { return (uint32_t)__umul24(a, b); }
__device__ __forceinline__ uint32_t pht_slot(uint32_t H, uint32_t d, uint32_t n_slots) {
  const uint32_t x = (umul24(d, (H >> 16) | 1u) + H) & 0xFFFFu;
  return umul24(x, n_slots) >> 16;
}

// One CHD probe (compile.py _probe): H -> the slot's 16-bit value, or kNoCand.
// b = {slot_off, disp_off (uint16 units), n_slots, disp_mask}.
template <typename P32>
__device__ __forceinline__ uint32_t pht_probe(P32 img, uint32_t H, v4u b) {
  const uint32_t d = rd16(img, b.y + ((H >> 16) & b.w));
  const uint32_t w = img[b.x + pht_slot(H, d, b.z)];
  return ((w >> 16) == (H & 0xFFFFu)) ? (w & 0xFFFFu) : kNoCand;
}

// PROFILING BUILD ONLY (make variant DEFS=-DRSA_PHASE_PROF=1): per-wave wall
// cycles (s_memtime) of the classifier's phases, summed over all waves into
// g_phase and read by rsa_phase_prof.  The markers wait for outstanding LDS
// and scalar loads (lgkmcnt), so the timed kernel is slower than the real one
// and the split is indicative only.
#ifdef RSA_PHASE_PROF
struct PhaseAcc {
  unsigned long long last, acc[8];
};
// [0..7] classifier phases, [8] its wave iterations; [9..11] k_reduce<1>
// workgroup cycles in setup, record inserts and flushes, [12] its workgroups;
// [13..16] inside them: waiting for the record loads, LDS inserts, the flush
// up to the claims, the flush's scan and slot writes; [17..24] the same for
// k_reduce<2> (the recount)
constexpr int kPhaseWords = 25;
__device__ unsigned long long g_phase[kPhaseWords];
#define RSA_PH_PARAM , PhaseAcc& ph
#define RSA_PH_ARG , ph
#define PH(k)                                                      \
  do {                                                             \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();    \
    ph.acc[k] += t_ - ph.last;                                     \
    ph.last = t_;                                                  \
  } while (0)
#else
#define RSA_PH_PARAM
#define RSA_PH_ARG
#define PH(k) \
  do {        \
  } while (0)
#endif

constexpr int kAttempts = 4;   // compile.py PHT_ATTEMPTS
constexpr uint32_t kListWords = 20, kGroupWords = 20, kMaskWords = 4;

// Pruning stage of the index lookup for ONE lane (compile.py pht_lookup): each
// src/dst mask table maps the masked address to a bitmap of the groups holding
// a rule on that prefix; the candidate groups are those in both the src and
// the dst bitmap.  A pruning slot holds tag << 8 | value (16-bit slots, tag =
// H & 0xFF) or tag << 16 | value (32-bit, tag = H & 0xFFFF); value indexes
// the record's uint64 bitmaps, where bitmap 0 is empty: an empty slot (0) or
// a tag mismatch reads bitmap 0, so every probe ORs a bitmap in, branch-free.
// The src tables come first (n_src_masks), then the dst tables: each side is
// its own loop with its address and salt fixed, kU masks per iteration phase
// by phase (all reads of a phase in flight before the first is waited for; a
// short last batch repeats its last mask: OR is idempotent).  kNarrow: every
// table of the image has 16-bit slots (image word 5 bit 1, wave-uniform), so
// the slot width is not decided per table.
template <bool kNarrow, int kPruneU, typename P32>
__device__ __forceinline__ unsigned long long prune_side(P32 img, uint32_t moff, uint32_t k0, uint32_t k1, uint32_t key,
                                                         uint32_t salt, uint32_t bm_off) {
  unsigned long long acc = 0ull;
  for (uint32_t k = k0; k < k1; k += kPruneU) {
    v4u m[kPruneU];
    uint32_t H[kPruneU], w[kPruneU];
#pragma unroll
    for (int u = 0; u < kPruneU; ++u) m[u] = rd4(img, moff + kMaskWords * min(k + u, k1 - 1));
#pragma unroll
    for (int u = 0; u < kPruneU; ++u) {
      H[u] = fmix32((key & m[u].x) ^ salt);
      w[u] = rd16(img, m[u].z + ((H[u] >> 16) & (m[u].w >> 17)));   // displacement
    }
#pragma unroll
    for (int u = 0; u < kPruneU; ++u) {
      const uint32_t hidx = (m[u].y & 0x7FFFFFFFu) + pht_slot(H[u], w[u], m[u].w & 0x1FFFFu);
      if (kNarrow) {
        w[u] = rd16(img, hidx);
      } else {
        const uint32_t narrow = m[u].y >> 31;
        const uint32_t w32 = img[hidx >> narrow];
        w[u] = narrow ? (w32 >> ((hidx & 1u) << 4)) & 0xFFFFu : w32;
      }
    }
#pragma unroll
    for (int u = 0; u < kPruneU; ++u) {
      uint32_t v;
      if (kNarrow) {
        v = (w[u] >> 8) == (H[u] & 0xFFu) ? (w[u] & 0xFFu) : 0u;
      } else {
        const uint32_t sh = (m[u].y >> 31) ? 8u : 16u, fm = (1u << sh) - 1u;
        v = (w[u] >> sh) == (H[u] & fm) ? (w[u] & fm) : 0u;
      }
      const v2u bb = rd2(img, bm_off + 2 * v);   // bm_off is even (compile.py: alloc align=2)
      acc |= ((unsigned long long)bb.y << 32) | bb.x;
    }
  }
  return acc;
}

#ifndef RSA_PRUNE_U
#define RSA_PRUNE_U 4   // pruning masks per batch (all their LDS reads in flight together)
#endif
// lw: the lane's list record {group_off, n_groups, mask_off, n_masks}, {…,
// bm_off}, {src_any, dst_any}, n_src_masks at word 18.
template <bool kNarrow, typename P32>
__device__ __forceinline__ unsigned long long index_candidates(P32 img, uint32_t lw, uint32_t src, uint32_t dst) {
  const v4u h0 = rd4(img, lw);
  const v4u h2 = rd4(img, lw + 8);
  unsigned long long S = ((unsigned long long)h2.y << 32) | h2.x;
  unsigned long long D = ((unsigned long long)h2.w << 32) | h2.z;
  const uint32_t bm_off = img[lw + 7];
  const uint32_t nm = h0.w, ns = img[lw + 18];   // the first ns records are the src tables
  if (kNarrow) {
    S |= prune_side<true, RSA_PRUNE_U>(img, h0.z, 0u, ns, src, kSaltS, bm_off);
    D |= prune_side<true, RSA_PRUNE_U>(img, h0.z, ns, nm, dst, kSaltD, bm_off);
  } else {   // (rare: a list with more than 255 distinct group bitmaps) one mask at a time
    S |= prune_side<false, 1>(img, h0.z, 0u, ns, src, kSaltS, bm_off);
    D |= prune_side<false, 1>(img, h0.z, ns, nm, dst, kSaltD, bm_off);
  }
  return S & D;
}

// A candidate group's record: header and the four port-class tables.
struct GroupRec {
  v4u a;        // {src_mask, dst_mask, min_idx, class_mask}
  v4u t[4];     // the port-class tables
};

template <typename P32>
__device__ __forceinline__ GroupRec group_rec(P32 img, uint32_t gw) {
  GroupRec r;
  r.a = rd4(img, gw);
#pragma unroll
  for (int c = 0; c < 4; ++c) r.t[c] = rd4(img, gw + 4 + 4 * c);
  return r;
}

// Port-class hash components of a tuple (compile.py PORT_CLASSES: any, dport,
// sport, both).
struct PortHash {
  uint32_t p1, p2, p3;
};
__device__ __forceinline__ PortHash port_hash(uint32_t ports) {
  return {fmix32((ports & 0xFFFF0000u) ^ kSaltP), fmix32((ports & 0x0000FFFFu) ^ kSaltP), fmix32(ports ^ kSaltP)};
}

// The four port-class probes of a candidate group for one tuple: the smallest
// list index >= floor among the group's tables, or kNoCand.
template <typename P32>
__device__ __forceinline__ uint32_t group_probe(P32 img, const GroupRec& g, uint32_t src, uint32_t dst,
                                                const PortHash& hp, uint32_t floor) {
  const uint32_t hsd = fmix32((src & g.a.x) ^ kSaltS) ^ fmix32((dst & g.a.y) ^ kSaltD);
  uint32_t c0 = pht_probe(img, hsd ^ fmix32(0u ^ kSaltP), g.t[0]);
  uint32_t c1 = pht_probe(img, hsd ^ hp.p1, g.t[1]);
  uint32_t c2 = pht_probe(img, hsd ^ hp.p2, g.t[2]);
  uint32_t c3 = pht_probe(img, hsd ^ hp.p3, g.t[3]);
  c0 = c0 >= floor ? c0 : kNoCand;
  c1 = c1 >= floor ? c1 : kNoCand;
  c2 = c2 >= floor ? c2 : kNoCand;
  c3 = c3 >= floor ? c3 : kNoCand;
  return min(min(c0, c1), min(c2, c3));
}

// Verification of candidate bi against its entry (16-bit tags collide) and,
// for ONE lane, the retries above a failed candidate: the candidate groups in
// ascending min index, until a group's min index cannot beat the best
// candidate.  Returns gid, kNoGid or kDefer.
template <typename P32>
__device__ __forceinline__ uint32_t index_verify(const Rules& R, P32 img, uint32_t lw, unsigned long long cand0,
                                                 uint32_t bi, uint32_t src, uint32_t dst, uint32_t ports) {
  const uint32_t group_off = img[lw];
  for (int attempt = 0;; ++attempt) {
    if (bi == kNoCand) return kNoGid;
    if (R.force_defer) return kDefer;
    const uint32_t ebeg = img[lw + 12];
    const v4u ea = R.eg[2 * (size_t)(ebeg + bi)], eb = R.eg[2 * (size_t)(ebeg + bi) + 1];
    if (entry_match(ea, eb, src, dst, ports)) return entry_gid(eb, ports);
    if (attempt + 1 >= kAttempts) return kDefer;
    const uint32_t floor = bi + 1;   // a tag collision: every true candidate lies above bi
    bi = kNoCand;
    const PortHash hp = port_hash(ports);
    unsigned long long cand = cand0;
    while (cand) {
      const uint32_t g = (uint32_t)__builtin_ctzll(cand);
      cand &= cand - 1;
      const GroupRec G = group_rec(img, group_off + kGroupWords * g);
      if (G.a.z >= bi) break;   // groups ascend in min index: no later group can do better
      bi = min(bi, group_probe(img, G, src, dst, hp, floor));
    }
  }
}

// Index lookup for ONE lane, all in the lane's own control flow (the
// RSA_OPT_GROUP_TASKS=0 form): pruning, the candidate groups in ascending
// min index with early exit, verification.
template <bool kNarrow, typename P32>
__device__ __forceinline__ uint32_t index_lookup(const Rules& R, P32 img, uint32_t lw, uint32_t src, uint32_t dst,
                                                 uint32_t ports) {
  if (R.prof & 1) return kNoGid;
  const unsigned long long cand0 = index_candidates<kNarrow>(img, lw, src, dst);
  if (!cand0 || (R.prof & 2)) return kNoGid;
  const uint32_t group_off = img[lw];
  const PortHash hp = port_hash(ports);
  uint32_t bi = kNoCand;
  unsigned long long cand = cand0;
  while (cand) {
    const uint32_t g = (uint32_t)__builtin_ctzll(cand);
    cand &= cand - 1;
    const GroupRec G = group_rec(img, group_off + kGroupWords * g);   // all five reads before the test
    if (G.a.z >= bi) break;
    bi = min(bi, group_probe(img, G, src, dst, hp, 0u));
  }
  if (R.prof & 4) return bi == kNoCand ? kNoGid : bi;
  return index_verify(R, img, lw, cand0, bi, src, dst, ports);
}

typedef __attribute__((address_space(3))) uint32_t lds_w32;

// Order LDS traffic of one wave between lanes: the compiler may not move LDS
// accesses across this point (the LDS executes one wave's instructions in
// order).
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Index lookup for the lanes with `ix` (WAVE-UNIFORM call, all lanes).  The
// pruning stage runs per lane; every lane then probes its own first candidate
// group (the one of smallest min index), and the remaining candidate (lane,
// group) pairs of the whole wave are dealt out as tasks, 64 per round, so a
// lane with many candidate groups no longer holds the wave for the others
// (per-lane loops ran max-over-lanes iterations: ~4.3 at 10k rules against a
// mean of 1.6; the remainder is ~0.7 tasks per lane, one round).  All
// candidate groups are probed (no early exit), so the per-lane minimum equals
// the serial loop's first attempt.  scr: this wave's 64 LDS words (the task
// list {group word << 6 | owner lane}, then per-owner minima via ds_min).
// Returns gid, kNoGid or kDefer for the ix lanes.
template <bool kNarrow, typename P32>
__device__ __forceinline__ uint32_t index_lookup_wave(const Rules& R, P32 img, uint32_t lw, bool ix, uint32_t src,
                                                      uint32_t dst, uint32_t ports, lds_w32* scr RSA_PH_PARAM) {
  if (R.prof & 1) return kNoGid;
  const unsigned long long cand0 = ix ? index_candidates<kNarrow>(img, lw, src, dst) : 0ull;
  PH(2);
  if (__ballot(cand0 != 0ull) == 0ull || (R.prof & 2)) return kNoGid;
  const uint32_t lane = __lane_id();
  const uint32_t group_off = ix ? img[lw] : 0u;
  const PortHash hp = port_hash(ports);
  // round 0: the lane's own first group
  uint32_t bi = kNoCand;
  if (cand0) {
    const uint32_t g = (uint32_t)__builtin_ctzll(cand0);
    bi = group_probe(img, group_rec(img, group_off + kGroupWords * g), src, dst, hp, 0u);
  }
  PH(3);
  unsigned long long rem = cand0 & (cand0 - 1ull);   // this lane's groups not yet probed
  if (__ballot(rem != 0ull) != 0ull) {
    // exclusive prefix of the remaining counts over the wave, by bit planes
    const uint32_t cnt = (uint32_t)__popcll(rem);
    uint32_t excl = 0;
    for (uint32_t b = 0; b < 6; ++b) {
      const unsigned long long plane = __ballot((cnt >> b) & 1u);
      if (__ballot(cnt >> b) == 0ull) break;
      excl += (uint32_t)__popcll(plane & ((1ull << lane) - 1ull)) << b;
    }
    const uint32_t total = __builtin_amdgcn_readlane(excl + cnt, 63);
    uint32_t pos = excl;   // wave task index of the lane's next group
    for (uint32_t base = 0; base < total; base += 64) {
      while (rem && pos < base + 64) {   // deal this round's tasks
        const uint32_t g = (uint32_t)__builtin_ctzll(rem);
        rem &= rem - 1ull;
        scr[pos - base] = ((group_off + kGroupWords * g) << 6) | lane;
        ++pos;
      }
      wave_lds_fence();
      const bool has = base + lane < total;
      const uint32_t task = has ? scr[lane] : lane;
      wave_lds_fence();
      scr[lane] = kNoCand;
      const uint32_t j = task & 63u;
      const uint32_t s_o = __shfl(src, j), d_o = __shfl(dst, j);
      const PortHash hp_o = {(uint32_t)__shfl(hp.p1, j), (uint32_t)__shfl(hp.p2, j), (uint32_t)__shfl(hp.p3, j)};
      wave_lds_fence();
      if (has) {
        const uint32_t c = group_probe(img, group_rec(img, task >> 6), s_o, d_o, hp_o, 0u);
        if (c != kNoCand) __atomic_fetch_min(&scr[j], c, __ATOMIC_RELAXED);
      }
      wave_lds_fence();
      bi = min(bi, scr[lane]);
      wave_lds_fence();
    }
  }
  PH(4);
  if (!ix || cand0 == 0ull) return kNoGid;
  if (R.prof & 4) return bi == kNoCand ? kNoGid : bi;
  const uint32_t v = index_verify(R, img, lw, cand0, bi, src, dst, ports);
  PH(5);
  return v;
}

// ---- partial-key bucket index (RSA_BKT_MAGIC, bucketindex.py) ---------------------
// Per list record a few tables, each keyed on (src & sm, dst & dm, ports & pm)
// of a template every one of its entries is exact on; a table is a bucketised
// cuckoo hash (2 candidate buckets of 2 slots) whose slot locates the
// bucket of entries with that key (rows entry_base
// + first .. + len of the residual array, first-gid ascending; the slot is
// tag11 << 21 | len5 << 16 | first16).  A lane probes
// every table (both buckets: independent LDS reads), checks the entries of the
// slots whose tag matches with the full predicate; every entry containing the
// connection is in a probed bucket, so the minimum is the linear scan's.
constexpr uint32_t kBktTableWords = 8;
constexpr uint32_t kBktTagMask = 0x7FFu, kBktLenMask = 0x1Fu;   // slot = tag11 << 21 | len5 << 16 | first16
constexpr uint32_t kBktMulD = 0x9E3779B1u, kBktMulP = 0x85EBCA77u;
constexpr uint32_t kBktSeedKey = 0x2545F491u, kBktSeedRow = 0x6A09E667u, kBktFpMask = 0x3FFFFu;   // bucketindex.py

// Row filter (bucketindex.py row_filters): f = slen6 << 26 | dlen6 << 20 |
// pm2 << 18 | fp18 over the row's own exact bits; a row that contains the
// connection always passes.
__device__ __forceinline__ uint32_t len_mask(uint32_t l) { return l ? 0xFFFFFFFFu << (32u - l) : 0u; }
__device__ __forceinline__ bool row_passes(uint32_t f, uint32_t src, uint32_t dst, uint32_t ports) {
  const uint32_t pm = ((f >> 18) & 1u ? 0x0000FFFFu : 0u) | ((f >> 19) & 1u ? 0xFFFF0000u : 0u);
  const uint32_t h = fmix32((src & len_mask(f >> 26)) ^ ((dst & len_mask((f >> 20) & 63u)) * kBktMulD) ^
                            ((ports & pm) * kBktMulP) ^ kBktSeedRow);
  return ((h ^ f) & kBktFpMask) == 0u;
}

// must equal bucketindex.py bkt_hash / bkt_buckets
__device__ __forceinline__ uint32_t bkt_hash(uint32_t ks, uint32_t kd, uint32_t kp, uint32_t seed) {
  return fmix32(ks ^ (kd * kBktMulD) ^ (kp * kBktMulP) ^ seed);
}

// Entries [beg, end) of one bucket (first-gid ascending) for ONE lane: the
// lane stops at the first entry whose first gid cannot beat its best.
__device__ __forceinline__ uint32_t scan_bucket(const v4u* __restrict__ E, uint32_t beg, uint32_t end, uint32_t best,
                                                uint32_t src, uint32_t dst, uint32_t ports) {
  for (uint32_t e = beg; e < end; ++e) {
    const v4u a = E[2 * (size_t)e], b = E[2 * (size_t)e + 1];
    if (b.z >= best) break;
    if (entry_match(a, b, src, dst, ports)) best = min(best, entry_gid(b, ports));
  }
  return best;
}

// One table (descriptor a = {src_mask, dst_mask, port_mask, bucket_off}, b =
// {n_buckets, filter_off, min_gid, entry_base}): hash, both candidate
// buckets, every row of the slots whose tag matches (no row filters).
template <typename P32>
__device__ __forceinline__ uint32_t bkt_table(const Rules& R, P32 img, v4u a, v4u b, uint32_t src, uint32_t dst,
                                              uint32_t ports, uint32_t best) {
  const uint32_t h = bkt_hash(src & a.x, dst & a.y, ports & a.z, kBktSeedKey);
  const uint32_t b1 = umul24(h & 0xFFFFu, b.x) >> 16;   // n_buckets <= 2^16: 24-bit operands
  const uint32_t b2 = umul24(h >> 16, b.x) >> 16;
  const uint32_t tag = ((h >> 16) ^ h) & kBktTagMask;
  const v2u s1 = rd2(img, a.w + 2 * b1), s2 = rd2(img, a.w + 2 * b2);
  const uint32_t sl[4] = {s1.x, s1.y, s2.x, s2.y};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t w = sl[q];
    const uint32_t len = (w >> 16) & kBktLenMask;
    if (len && (w >> 21) == tag && !(q >= 2 && b2 == b1)) {
      const uint32_t beg = b.w + (w & 0xFFFFu);
      best = scan_bucket(R.residg, beg, beg + len, best, src, dst, ports);
    }
  }
  return best;
}

// The tables of one list record for ONE lane, one after the other (ascending
// min gid: stop once the best beats a table's smallest gid).  The general
// form: every slot whose tag matches, in every table.
template <typename P32>
__device__ __forceinline__ uint32_t bucket_lookup_serial(const Rules& R, P32 img, uint32_t lw, uint32_t src,
                                                         uint32_t dst, uint32_t ports, uint32_t best) {
  const uint32_t toff = img[lw], nt = img[lw + 1];
  for (uint32_t j = 0; j < nt; ++j) {
    const uint32_t tw = toff + kBktTableWords * j;
    const v4u a = rd4(img, tw), b = rd4(img, tw + 4);
    if (best <= b.z) break;
    best = bkt_table(R, img, a, b, src, dst, ports, best);
  }
  return best;
}

constexpr int kBktMaxTables = 8;   // bucketindex.py MAX_TABLES


// Phased form: (A) every table's probe -- LDS reads only, all independent --
// keeping the tag-matching slots of the (at most four) tables with one;
// without row filters (B') their buckets two at a time, both first rows
// loaded together; with row filters (B) per hit bucket the first row whose
// LDS filter the connection passes (LDS only); (C) the (at most two) candidate rows loaded together and checked in
// full; a candidate that fails (an 18-bit filter collision, or a side the
// filter cannot check: port ranges, runs) continues its bucket's scan.  A
// lane with more hit tables or candidates, or two tag-matching slots in one
// table (an 11-bit tag collision), takes the serial form.  Typically one
// global load per matched line, none for an unmatched one.
// Image reads of the global (HBM) image are L2 round trips on the lane's
// dependent chain, so that variant reads what it needs of a record or table
// descriptor together, up front (kGlb); the LDS image re-reads words where
// they are used (registers are its limit: 64 VGPRs at 8 waves per SIMD).
// The first hit table's min_gid / entry_base are kept from the descriptor read
// of its probe (cfg4 0.912 -> 0.905 ms per k_classify launch,
// profiles/r05/ab_summary.txt r05n).
template <typename P32>
constexpr bool kGlobalImg = false;
template <>
constexpr bool kGlobalImg<const uint32_t*> = true;

// toff / nt: the record's table descriptors and their count (words 0 and 1 of
// the list record at lw).
template <typename P32>
__device__ __forceinline__ uint32_t bucket_lookup(const Rules& R, P32 img, uint32_t lw, uint32_t toff, uint32_t nt,
                                                  uint32_t src, uint32_t dst, uint32_t ports, uint32_t best) {
  constexpr bool kGlb = kGlobalImg<P32>;
  uint32_t h0 = 0u, h1 = 0u, h2 = 0u, h3 = 0u;   // hit slot words, in table order
  uint32_t tj = 0u;                              // their tables, 4 bits each (hit k at bits 4k)
  uint32_t nh = 0u;
  // (global image) the first hit table's min_gid / entry_base, kept from the
  // descriptor read of the probe (no second dependent read in (B') for the
  // common single hit)
  uint32_t g0 = 0u, e0 = 0u;
  bool slow = false;
#pragma unroll
  for (int j = 0; j < kBktMaxTables; ++j) {
    if ((uint32_t)j < nt) {
      const uint32_t tw = toff + kBktTableWords * j;
      const v4u a = rd4(img, tw);
      v4u d = {0u, 0u, 0u, 0u};   // n_buckets, filter_off, min_gid, entry_base
      if (kGlb)
        d = rd4(img, tw + 4);
      else
        d.x = img[tw + 4];
      const uint32_t nb = d.x;
      const uint32_t h = bkt_hash(src & a.x, dst & a.y, ports & a.z, kBktSeedKey);
      const uint32_t b1 = umul24(h & 0xFFFFu, nb) >> 16;
      const uint32_t b2 = umul24(h >> 16, nb) >> 16;
      const uint32_t tag = ((h >> 16) ^ h) & kBktTagMask;
      const v2u s1 = rd2(img, a.w + 2 * b1), s2 = rd2(img, a.w + 2 * b2);
      const uint32_t sl[4] = {s1.x, s1.y, s2.x, s2.y};
      uint32_t f = 0u;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t w = sl[q];
        const bool m = ((w >> 16) & kBktLenMask) != 0u && (w >> 21) == tag && !(q >= 2 && b2 == b1);
        slow |= m && f != 0u;
        f = (m && f == 0u) ? w : f;
      }
      if (f) {
        h0 = nh == 0u ? f : h0;
        h1 = nh == 1u ? f : h1;
        h2 = nh == 2u ? f : h2;
        h3 = nh == 3u ? f : h3;
        if (kGlb) {
          g0 = nh == 0u ? d.z : g0;
          e0 = nh == 0u ? d.w : e0;
        }
        tj |= (uint32_t)j << (4 * (nh & 7u));
        ++nh;
      }
    }
  }
  if (R.prof & 2) return best ^ (nh & 0x80000000u);             // PROFILING: probes only (results invalid)
  if ((slow || nh > 4u) && !(R.prof & 4)) return bucket_lookup_serial(R, img, lw, src, dst, ports, best);
  if (nh > 4u) nh = 4u;                                          // (only under R.prof & 4)
  if (!R.bkt_filters) {
    // (B') no row filters: the hit buckets two at a time, both first rows in flight
    for (uint32_t p = 0; p < nh; p += 2) {
      const uint32_t wa = p ? h2 : h0, wb = p ? h3 : h1;
      const uint32_t ja = (tj >> (4 * p)) & 0xFu;
      const bool two = p + 1 < nh;
      const uint32_t jb = two ? (tj >> (4 * p + 4)) & 0xFu : ja;
      v2u ma, mb;   // min_gid, entry_base
      if (kGlb && p == 0) {
        ma = v2u{g0, e0};
        mb = two ? rd2(img, toff + kBktTableWords * jb + 6) : ma;
      } else {
        ma = rd2(img, toff + kBktTableWords * ja + 6);
        mb = rd2(img, toff + kBktTableWords * jb + 6);
      }
      const uint32_t ea = ma.y + (wa & 0xFFFFu), eb = mb.y + ((two ? wb : wa) & 0xFFFFu);
      const v4u aa = R.residg[2 * (size_t)ea], ca = R.residg[2 * (size_t)ea + 1];
      const v4u ab = R.residg[2 * (size_t)eb], cb = R.residg[2 * (size_t)eb + 1];
      if (best > ma.x) {
        if (ca.z < best && entry_match(aa, ca, src, dst, ports)) best = min(best, entry_gid(ca, ports));
        const uint32_t la = (wa >> 16) & kBktLenMask;
        if (la > 1u) best = scan_bucket(R.residg, ea + 1, ea + la, best, src, dst, ports);
      }
      if (two && best > mb.x) {
        if (cb.z < best && entry_match(ab, cb, src, dst, ports)) best = min(best, entry_gid(cb, ports));
        const uint32_t lb = (wb >> 16) & kBktLenMask;
        if (lb > 1u) best = scan_bucket(R.residg, eb + 1, eb + lb, best, src, dst, ports);
      }
    }
    return best;
  }
  // (B) candidate rows: absolute residual row and the rows left in its bucket
  uint32_t r0 = 0u, n0 = 0u, r1 = 0u, n1 = 0u, nc = 0u;
  for (uint32_t k = 0; k < nh; ++k) {
    const uint32_t w = k == 0u ? h0 : k == 1u ? h1 : k == 2u ? h2 : h3;
    const uint32_t j = (tj >> (4 * k)) & 0xFu;
    const v4u d = rd4(img, toff + kBktTableWords * j + 4);     // n_buckets, filter_off, min_gid, entry_base
    if (best <= d.z) break;                                    // tables ascend in min gid
    const uint32_t first = w & 0xFFFFu, end = first + ((w >> 16) & kBktLenMask);
    for (uint32_t r = first; r < end; ++r) {
      if (row_passes(img[d.y + r], src, dst, ports)) {
        r1 = nc == 1u ? d.w + r : r1;
        n1 = nc == 1u ? end - r - 1u : n1;
        r0 = nc == 0u ? d.w + r : r0;
        n0 = nc == 0u ? end - r - 1u : n0;
        ++nc;
        break;
      }
    }
  }
  if (nc > 2u) return bucket_lookup_serial(R, img, lw, src, dst, ports, best);
  if (nc == 0u) return best;
  // (C) the candidates' rows, both loads in flight
  const uint32_t rb = nc > 1u ? r1 : r0;
  const v4u a0 = R.residg[2 * (size_t)r0], c0 = R.residg[2 * (size_t)r0 + 1];
  const v4u a1 = R.residg[2 * (size_t)rb], c1 = R.residg[2 * (size_t)rb + 1];
  if (c0.z < best) {
    if (entry_match(a0, c0, src, dst, ports)) {
      best = min(best, entry_gid(c0, ports));
    } else if (n0) {
      best = scan_bucket(R.residg, r0 + 1u, r0 + 1u + n0, best, src, dst, ports);
    }
  }
  if (nc > 1u && c1.z < best) {
    if (entry_match(a1, c1, src, dst, ports)) {
      best = min(best, entry_gid(c1, ports));
    } else if (n1) {
      best = scan_bucket(R.residg, r1 + 1u, r1 + 1u + n1, best, src, dst, ports);
    }
  }
  return best;
}

// First-match classification of one wave of tuples.  Linear scans (the whole
// list without the index; the prefix and the residual entries with it) run as
// a waterfall over the distinct lists present in the wave (list id broadcast
// by readlane, so entries are wave-uniform scalar loads); the index lookup
// runs per lane.  kExact: ignore the index (the deferred-line path).
// kMode: 0 = pht index, per-lane group loops; 1 = pht index, candidate groups
// dealt out over the wave (RSA_OPT_GROUP_TASKS); 2 = bucket index.
template <bool kExact, int kMode, bool kNarrow, typename P32>
__device__ __forceinline__ uint32_t classify_wave(uint4 t, bool active, const Rules& R, P32 img, unsigned int* flags,
                                                  lds_w32* scr RSA_PH_PARAM) {
  const uint32_t list = t.w & 0xFFFFu;
  if (active && list >= R.n_lists) {
    atomicOr(&flags[1], 1u);
    active = false;
  }
  uint32_t best = kNoGid;
  if (kExact || !R.indexed) {
    unsigned long long pending = __ballot(active);
    while (pending) {
      const int leader = __builtin_ctzll(pending);
      const uint32_t L = __builtin_amdgcn_readlane(list, leader);
      const bool mine = active && list == L;
      pending &= ~__ballot(mine);
      const uint32_t b = scan_list(R.e, R.off[L], R.off[L + 1], mine, kNoGid, t.x, t.y, t.z);
      if (mine) best = b;
    }
    return active ? best : kNoGid;
  }
  // list record fields (include/ruleset_hip.h rsa_pht_list) are read from the
  // image where they are used: lw = the lane's current record.  (Reading the
  // global image's record words once, up front, costs the emission's
  // order/timestamp prefetch its registers: cfg4 0.905 -> 0.968-1.105 ms per
  // launch, profiles/r05/ab_summary.txt r05n.)
  uint32_t lw = R.list_off + kListWords * (active ? list : 0u);
  // 1. prefix scans
  const uint32_t pre_n = active ? img[lw + 6] : 0u;
  PH(0);
  unsigned long long pending = __ballot(active && pre_n != 0);
  while (pending) {
    const int leader = __builtin_ctzll(pending);
    const uint32_t L = __builtin_amdgcn_readlane(list, leader);
    const bool mine = active && list == L;
    pending &= ~__ballot(mine);
    const uint32_t beg = R.off[L];
    const uint32_t pre = __builtin_amdgcn_readlane(pre_n, leader);
    const uint32_t b = scan_list(R.e, beg, beg + pre, mine, kNoGid, t.x, t.y, t.z);
    if (mine) best = b;
  }
  // 2. per record of the lane's chain: the index (per lane), then the residual
  // scan (waterfall over the records present); the next chunk only while the
  // lane's best exceeds its smallest gid
  bool go = active && best > img[lw + 15];
  bool deferred = false;
  PH(1);
  while (__ballot(go)) {
    const bool ix = go && img[lw + 1] != 0;
    uint32_t c = kNoGid;
    if (kMode == 2) {
      // partial-key bucket index: exact, never deferred
      if (ix && !(R.prof & 1)) {
        if (R.force_defer) {
          c = kDefer;
        } else {
          c = bucket_lookup(R, img, lw, img[lw], img[lw + 1], t.x, t.y, t.z, best);
        }
      }
    } else if (kMode == 1) {
      c = index_lookup_wave<kNarrow>(R, img, lw, ix, t.x, t.y, t.z, scr RSA_PH_ARG);
    } else if (ix) {
      c = index_lookup<kNarrow>(R, img, lw, t.x, t.y, t.z);
    }
    if (ix) {
      if (c == kDefer) {
        deferred = true;
        go = false;
      } else {
        best = min(best, c);
      }
    }
    const uint32_t rb = go ? img[lw + 4] : 0u, re = go ? img[lw + 5] : 0u;
    const bool want = go && rb < re;
    pending = __ballot(want);
    while (pending) {
      const int leader = __builtin_ctzll(pending);
      const uint32_t Q = __builtin_amdgcn_readlane(lw, leader);
      const bool mine = want && lw == Q;
      pending &= ~__ballot(mine);
      const uint32_t b = scan_list(R.resid, __builtin_amdgcn_readlane(rb, leader), __builtin_amdgcn_readlane(re, leader),
                                   mine, best, t.x, t.y, t.z);
      if (mine) best = b;
    }
    if (go) {
      const uint32_t next = img[lw + 16];
      go = next != RSA_PHT_NONE && best > img[lw + 17];
      if (go) lw = R.list_off + kListWords * next;
    }
    PH(6);
  }
  if (deferred) return kDefer;
  return active ? best : kNoGid;
}

// Insert-or-combine (kA, kB) into the open-addressing table.  A slot is claimed
// EMPTY->BUSY by a device atomic (executed at the memory side, beyond the
// per-XCD L2s), its kA published, then kB published, both by atomics.  A
// published key never changes during a job, so each probe first reads the
// slot's head {kA, kB} and {min_order, first, last} with plain 16-B loads: the
// line they come from (possibly a stale per-XCD copy) is a snapshot of memory,
// and kA was final in memory before kB was, so a published kB in the snapshot
// comes with its final kA.  A match or another published key is therefore
// decided without atomics; only a slot that looks EMPTY or BUSY takes the
// atomic path (CAS; a lane that sees BUSY re-reads the slot).  The three
// monotone fields are then updated only where the snapshot does not already
// rule the update out (min_order/first only decrease, last only increases, so
// any value the snapshot holds bounds the current one).  Returns the slot index
// (or kEmpty on overflow); *fresh is set when this call created the entry.
struct SlotHead {
  v4u k;   // kA lo, kA hi, kB lo, kB hi
  v4u m;   // min_order lo, min_order hi, first, last
};

__device__ __forceinline__ SlotHead load_head(const Slot* c) {
  SlotHead r;
  r.k = *reinterpret_cast<const volatile v4u*>(&c->kA);
  r.m = *reinterpret_cast<const volatile v4u*>(&c->min_order);
  return r;
}

// Combine one occurrence into an existing entry s whose head snapshot is hd;
// returns the number of atomics issued.
__device__ __forceinline__ uint32_t slot_update(const Agg& A, Slot* s, const SlotHead& hd, unsigned int cnt,
                                                unsigned int first, unsigned int last, unsigned long long order) {
  if (A.skip & 4u) return 0;   // profiling only
  atomicAdd(&s->count, cnt);
  const unsigned long long mo = ((unsigned long long)hd.m.y << 32) | hd.m.x;
  const bool all = !A.precheck;
  const bool u0 = all || order < mo, u1 = all || first < hd.m.z, u2 = all || last > hd.m.w;
  if (u0) atomicMin(&s->min_order, order);
  if (u1) atomicMin(&s->first, first);
  if (u2) atomicMax(&s->last, last);
  return 1u + u0 + u1 + u2;
}

// Agent-scope (write-through) stores of a claimed slot's key half kA and its
// aggregates; the caller waits for them before publishing kB.
__device__ __forceinline__ void slot_init(Slot* c, unsigned long long kA, unsigned int cnt, unsigned int first,
                                          unsigned int last, unsigned long long order) {
  __hip_atomic_store(&c->kA, kA, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&c->min_order, order, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(&c->first), ((unsigned long long)last << 32) | first,
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&c->count, cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ unsigned long long table_combine_at(const Agg& A, unsigned long long kA,
                                                               unsigned long long kB, unsigned int cnt,
                                                               unsigned int first, unsigned int last,
                                                               unsigned long long order, bool* fresh,
                                                               unsigned long long h, SlotHead hd,
                                                               uint32_t* st = nullptr) {
  unsigned long long probes = 0, atomic_probes = 0;
  unsigned long long found = kEmpty;
  while (true) {
    Slot* c = &A.slots[h];
    const unsigned long long pa = ((unsigned long long)hd.k.y << 32) | hd.k.x;
    const unsigned long long pb = ((unsigned long long)hd.k.w << 32) | hd.k.z;
    if (pb != kEmpty && pb != kBusy) {
      if (pb == kB && pa == kA) {
        found = h;
        break;
      }
    } else {
      ++atomic_probes;
      const unsigned long long cur = atomicCAS(&c->kB, kEmpty, kBusy);
      if (cur == kEmpty) {
        // The slot is ours and invisible until kB is published: write kA and the
        // aggregates with agent-scope (write-through) stores, wait for them to
        // complete, then publish kB.  Finders only update the fields after they
        // have seen kB, so their atomics act on these values.
        slot_init(c, kA, cnt, first, last, order);
        atomicOr(&A.occ[h >> 5], 1u << (h & 31));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        atomicExch(&c->kB, kB);
        *fresh = true;
        if (st) {
          st[0] += 1;
          st[1] += (uint32_t)probes;
          st[2] += (uint32_t)atomic_probes;
          st[3] += 2;
        }
        return h;
      }
      if (cur == kBusy) {
        hd = load_head(c);
        continue;
      }
      if (cur == kB && atomicOr(&c->kA, 0ull) == kA) {
        found = h;
        break;
      }
    }
    h = slot_next(A, h);
    if (++probes >= (1ull << A.rs_bits)) break;
    hd = load_head(&A.slots[h]);
  }
  if (found == kEmpty) {
    atomicOr(&A.flags[0], 1u);
    return kEmpty;
  }
  const uint32_t n_at = slot_update(A, &A.slots[found], hd, cnt, first, last, order);
  if (st) {
    st[0] += 1;
    st[1] += (uint32_t)probes;
    st[2] += (uint32_t)atomic_probes;
    st[3] += n_at + (uint32_t)atomic_probes;
  }
  return found;
}

__device__ __forceinline__ unsigned long long table_combine(const Agg& A, unsigned long long kA,
                                                            unsigned long long kB, unsigned int cnt,
                                                            unsigned int first, unsigned int last,
                                                            unsigned long long order, bool* fresh) {
  const unsigned long long h = slot_home(A, slot_hash(kA, kB));
  return table_combine_at(A, kA, kB, cnt, first, last, order, fresh, h, load_head(&A.slots[h]));
}

// Find an existing key (after pass 1 completed: plain loads are coherent across
// the kernel boundary).  A slot is live only if its occupancy bit is set: the
// slots are not cleared between jobs (rsa_reset clears the bitmap), so an
// unoccupied slot may hold a key of an earlier job.
__device__ __forceinline__ Slot* table_find(const Agg& A, unsigned long long kA, unsigned long long kB) {
  unsigned long long h = slot_home(A, slot_hash(kA, kB));
  for (unsigned long long probes = 0; probes < (1ull << A.rs_bits); ++probes) {
    Slot* c = &A.slots[h];
    if (!((A.occ[h >> 5] >> (h & 31)) & 1u)) return nullptr;
    const unsigned long long cb = c->kB;
    if (cb == kEmpty) return nullptr;
    if (cb == kB && c->kA == kA) return c;
    h = slot_next(A, h);
  }
  return nullptr;
}

struct alignas(32) Rec {
  unsigned long long kA, kB, order;
  uint32_t ts, region;
};
static_assert(sizeof(Rec) == 32, "record layout");

__device__ __forceinline__ uint32_t key_region(const Agg& A, unsigned long long hh) {
  return A.np_bits ? (uint32_t)(hh >> (64 - A.np_bits)) : 0u;
}

// Workgroup exclusive scan of one uint32 per thread (blockDim.x <= 1024);
// returns the thread's offset and writes the total to *total.  sh: >= 16 words.
__device__ __forceinline__ uint32_t block_exscan(uint32_t v, uint32_t* sh, uint32_t* total) {
  const unsigned lane = __lane_id(), w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  uint32_t x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if ((int)lane >= o) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  uint32_t before = 0, all = 0;
  for (unsigned q = 0; q < nw; ++q) {
    const uint32_t t = sh[q];
    if (q < w) before += t;
    all += t;
  }
  __syncthreads();
  *total = all;
  return before + x - v;
}

// ---- two lines per lane: the global bucket image (BASELINE config 4) ------
// The global-image classifier is latency bound (VALU busy 0.16): a lane's
// chain -- list record, table descriptors, bucket slots, bucket rows, the
// rule's filter bound -- is a series of dependent L2/HBM round trips, and
// occupancy is already at 8 waves per SIMD.  k_classify_pair gives each lane
// two lines and runs their chains side by side: the probes of both lines'
// tables are issued together (addresses selected, not branched, so the loads
// share one basic block), then both lines' first bucket rows, then both
// filter bounds before either line's stores.  Same answers as classify_wave
// (the minimum gid over the same candidate rows; the early exits only skip
// rows whose first gid cannot beat the lane's best).

// The prefix scan of classify_wave for the lanes with `active` (waterfall over
// the lists present).
__device__ __forceinline__ void prefix_scan_wave(const Rules& R, uint32_t list, bool active, uint32_t pre_n, uint4 t,
                                                 uint32_t& best) {
  unsigned long long pending = __ballot(active && pre_n != 0);
  while (pending) {
    const int leader = __builtin_ctzll(pending);
    const uint32_t L = __builtin_amdgcn_readlane(list, leader);
    const bool mine = active && list == L;
    pending &= ~__ballot(mine);
    const uint32_t beg = R.off[L];
    const uint32_t pre = __builtin_amdgcn_readlane(pre_n, leader);
    const uint32_t b = scan_list(R.e, beg, beg + pre, mine, kNoGid, t.x, t.y, t.z);
    if (mine) best = b;
  }
}

// The residual scan of record lw for the lanes with `go` (waterfall over the
// records present).
template <typename P32>
__device__ __forceinline__ void resid_scan_wave(const Rules& R, P32 img, bool go, uint32_t lw, uint4 t, uint32_t& best) {
  const uint32_t rb = go ? img[lw + 4] : 0u, re = go ? img[lw + 5] : 0u;
  const bool want = go && rb < re;
  unsigned long long pending = __ballot(want);
  while (pending) {
    const int leader = __builtin_ctzll(pending);
    const uint32_t Q = __builtin_amdgcn_readlane(lw, leader);
    const bool mine = want && lw == Q;
    pending &= ~__ballot(mine);
    const uint32_t b = scan_list(R.resid, __builtin_amdgcn_readlane(rb, leader), __builtin_amdgcn_readlane(re, leader),
                                 mine, best, t.x, t.y, t.z);
    if (mine) best = b;
  }
}

// One lane's tag-matching bucket slots (bucket_lookup's phase A state).
struct BktHits {
  uint32_t h0, h1, h2, h3;   // hit slot words, in table order
  uint32_t tj;               // their tables, 4 bits each
  uint32_t nh;
  uint32_t g0, e0;           // the first hit table's min_gid / entry_base
  uint32_t slow;             // two matching slots in one table: the serial form
};

// Table j of the record whose descriptors start at toff, for a lane with
// `on`; a lane without (no table j, or no lookup) reads the image header
// instead (word 0.., one bucket at word 0) and records nothing, so every lane
// issues the same loads.
__device__ __forceinline__ void bkt_probe_j(const uint32_t* img, uint32_t toff, bool on, uint32_t j, uint32_t src,
                                            uint32_t dst, uint32_t ports, BktHits& H) {
  const uint32_t tw = on ? toff + kBktTableWords * j : 0u;
  const v4u a = rd4(img, tw);
  const v4u d = rd4(img, tw + 4);   // n_buckets, filter_off, min_gid, entry_base
  const uint32_t nb = on ? d.x : 1u;
  const uint32_t h = bkt_hash(src & a.x, dst & a.y, ports & a.z, kBktSeedKey);
  const uint32_t b1 = umul24(h & 0xFFFFu, nb) >> 16;
  const uint32_t b2 = umul24(h >> 16, nb) >> 16;
  const uint32_t tag = ((h >> 16) ^ h) & kBktTagMask;
  const uint32_t bo = on ? a.w : 0u;
  const v2u s1 = rd2(img, bo + 2 * b1), s2 = rd2(img, bo + 2 * b2);
  const uint32_t sl[4] = {s1.x, s1.y, s2.x, s2.y};
  uint32_t f = 0u, slow = 0u;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t w = sl[q];
    const bool m = on && ((w >> 16) & kBktLenMask) != 0u && (w >> 21) == tag && !(q >= 2 && b2 == b1);
    slow |= (m && f != 0u) ? 1u : 0u;
    f = (m && f == 0u) ? w : f;
  }
  H.slow |= slow;
  if (f) {
    H.h0 = H.nh == 0u ? f : H.h0;
    H.h1 = H.nh == 1u ? f : H.h1;
    H.h2 = H.nh == 2u ? f : H.h2;
    H.h3 = H.nh == 3u ? f : H.h3;
    H.g0 = H.nh == 0u ? d.z : H.g0;
    H.e0 = H.nh == 0u ? d.w : H.e0;
    H.tj |= j << (4 * (H.nh & 7u));
    ++H.nh;
  }
}

// Hit k's bucket rows for one lane (bucket_lookup's (B') for one hit): the
// first row loaded by the caller (ra, rc), the rest of the bucket scanned.
__device__ __forceinline__ uint32_t bkt_rows(const Rules& R, v2u ge, uint32_t w, v4u ra, v4u rc, uint32_t src,
                                             uint32_t dst, uint32_t ports, uint32_t best) {
  if (best > ge.x) {
    if (rc.z < best && entry_match(ra, rc, src, dst, ports)) best = min(best, entry_gid(rc, ports));
    const uint32_t len = (w >> 16) & kBktLenMask;
    const uint32_t e = ge.y + (w & 0xFFFFu);
    if (len > 1u) best = scan_bucket(R.residg, e + 1, e + len, best, src, dst, ports);
  }
  return best;
}

__device__ __forceinline__ uint32_t hit_word(const BktHits& H, uint32_t k) {
  return k == 0u ? H.h0 : k == 1u ? H.h1 : k == 2u ? H.h2 : H.h3;
}

// Both lines' bucket lookups (no row filters; the global image).  ia / ib:
// the lanes whose line looks the record up; returns their new bests.
__device__ __forceinline__ void bucket_lookup_pair(const Rules& R, const uint32_t* img, uint32_t lwa, bool ia, uint4 ta,
                                                   uint32_t& besta, uint32_t lwb, bool ib, uint4 tb, uint32_t& bestb) {
  const uint32_t toffa = img[lwa], nta = ia ? img[lwa + 1] : 0u;
  const uint32_t toffb = img[lwb], ntb = ib ? img[lwb + 1] : 0u;
  BktHits A = {}, B = {};
#pragma unroll
  for (uint32_t j = 0; j < (uint32_t)kBktMaxTables; ++j) {
    const bool pa = j < nta, pb = j < ntb;
    if (!__ballot(pa || pb)) break;   // wave-uniform: no lane has a table j
    bkt_probe_j(img, toffa, pa, j, ta.x, ta.y, ta.z, A);
    bkt_probe_j(img, toffb, pb, j, tb.x, tb.y, tb.z, B);
  }
  // (rare) two matching slots in one table, or more than four hit tables
  const bool sa = ia && (A.slow || A.nh > 4u), sb = ib && (B.slow || B.nh > 4u);
  if (sa) besta = bucket_lookup_serial(R, img, lwa, ta.x, ta.y, ta.z, besta);
  if (sb) bestb = bucket_lookup_serial(R, img, lwb, tb.x, tb.y, tb.z, bestb);
  const uint32_t na = (ia && !sa) ? A.nh : 0u, nb = (ib && !sb) ? B.nh : 0u;
  for (uint32_t k = 0; __ballot(k < na || k < nb); ++k) {
    const bool oa = k < na, ob = k < nb;
    const uint32_t wa = hit_word(A, k), wb = hit_word(B, k);
    v2u ga = {A.g0, A.e0}, gb = {B.g0, B.e0};
    if (k > 0u) {   // (a second hit table: its min_gid / entry_base)
      ga = oa ? rd2(img, toffa + kBktTableWords * ((A.tj >> (4 * k)) & 0xFu) + 6) : ga;
      gb = ob ? rd2(img, toffb + kBktTableWords * ((B.tj >> (4 * k)) & 0xFu) + 6) : gb;
    }
    // both first rows in flight together (a lane without a hit reads row 0)
    const uint32_t ea = oa ? ga.y + (wa & 0xFFFFu) : 0u, eb = ob ? gb.y + (wb & 0xFFFFu) : 0u;
    const v4u aa = R.residg[2 * (size_t)ea], ca = R.residg[2 * (size_t)ea + 1];
    const v4u ab = R.residg[2 * (size_t)eb], cb = R.residg[2 * (size_t)eb + 1];
    if (oa) besta = bkt_rows(R, ga, wa, aa, ca, ta.x, ta.y, ta.z, besta);
    if (ob) bestb = bkt_rows(R, gb, wb, ab, cb, tb.x, tb.y, tb.z, bestb);
  }
}

// classify_wave<false, 2, false> for two lines per lane (global bucket image,
// no row filters).
__device__ __forceinline__ void classify_pair_bkt(uint4 ta, bool aa, uint4 tb, bool ab, const Rules& R,
                                                  const uint32_t* img, unsigned int* flags, uint32_t& ga,
                                                  uint32_t& gb) {
  const uint32_t la = ta.w & 0xFFFFu, lb = tb.w & 0xFFFFu;
  if (aa && la >= R.n_lists) {
    atomicOr(&flags[1], 1u);
    aa = false;
  }
  if (ab && lb >= R.n_lists) {
    atomicOr(&flags[1], 1u);
    ab = false;
  }
  uint32_t besta = kNoGid, bestb = kNoGid;
  uint32_t lwa = R.list_off + kListWords * (aa ? la : 0u), lwb = R.list_off + kListWords * (ab ? lb : 0u);
  const uint32_t prea = aa ? img[lwa + 6] : 0u, preb = ab ? img[lwb + 6] : 0u;
  const uint32_t mina = img[lwa + 15], minb = img[lwb + 15];
  prefix_scan_wave(R, la, aa, prea, ta, besta);
  prefix_scan_wave(R, lb, ab, preb, tb, bestb);
  bool goa = aa && besta > mina, gob = ab && bestb > minb;
  bool defa = false, defb = false;
  while (__ballot(goa || gob)) {
    const bool ixa = goa && img[lwa + 1] != 0, ixb = gob && img[lwb + 1] != 0;
    if (!(R.prof & 1)) {
      if (R.force_defer) {
        defa = defa || ixa;
        defb = defb || ixb;
      } else {
        bucket_lookup_pair(R, img, lwa, ixa, ta, besta, lwb, ixb, tb, bestb);
      }
    }
    if (ixa && defa) goa = false;
    if (ixb && defb) gob = false;
    resid_scan_wave(R, img, goa, lwa, ta, besta);
    resid_scan_wave(R, img, gob, lwb, tb, bestb);
    if (goa) {
      const uint32_t next = img[lwa + 16];
      goa = next != RSA_PHT_NONE && besta > img[lwa + 17];
      if (goa) lwa = R.list_off + kListWords * next;
    }
    if (gob) {
      const uint32_t next = img[lwb + 16];
      gob = next != RSA_PHT_NONE && bestb > img[lwb + 17];
      if (gob) lwb = R.list_off + kListWords * next;
    }
  }
  ga = defa ? kDefer : (aa ? besta : kNoGid);
  gb = defb ? kDefer : (ab ? bestb : kNoGid);
}

// Where pass 1 puts its per-line results (k_classify / k_tail with kEmit),
// without appends to shared cursors (no atomics or workgroup barriers in the
// classifier): the line's gid|hit word for the per-rule counters (k_count);
// for every hit + BUILT line below its rule's filter bound a 32-B record and
// its table region (connlist-reducer.py:146-176), compacted per 64-line
// window (a wave's lines): window w holds its wcnt[w] records in slots
// [64 w, 64 w + wcnt[w]) of the line-indexed record arrays.
constexpr uint32_t kWin = 64;
struct Emit {
  uint32_t* gh;                         // gid | hit << 31, 0xFFFFFFFF: no rule
  uint16_t* gh16;                       // instead of gh when the rules fit 15 bits: gid | hit << 15, 0xFFFF
  const uint32_t* ts;
  const unsigned long long* ord;
  Rec* recs;                            // window-compacted records
  uint16_t* regs;                       // their regions
  uint32_t* wcnt;                       // records per 64-line window
};

// k_classify's emission arguments, passed FIRST (kernarg offset 0) and read
// from the kernarg segment where they are used (classify_emit_args): held in
// SGPRs across the lookup they spilled to VGPR lanes (55 SGPRs, ~25 v_readlane
// restores per emission); re-read they cost two scalar loads per iteration.
struct EmitPack {
  unsigned long long gh, gh16, ts, ord, recs, regs, wcnt, filter;   // device addresses (global memory)
  uint32_t cap, skip, np_bits, pad;
};

template <typename T>
__device__ __forceinline__ T* global_ptr(unsigned long long a) {
  // an integer -> global (address space 1) pointer -> generic pointer: the
  // address space stays known, so accesses through it are global_*, not flat_*
  typedef __attribute__((address_space(1))) T gT;
  return (T*)(gT*)a;
}


// The emission's Agg fields and Emit pointers, loaded from the kernarg segment
// at this point of the loop (the empty asm makes the pointer opaque per
// iteration, so the loads are not hoisted into long-lived SGPRs).
__device__ __forceinline__ void classify_emit_args(const EmitPack& ep_arg, Agg& A, Emit& E) {
  typedef __attribute__((address_space(4))) const EmitPack cEmitPack;
  cEmitPack* ep = (cEmitPack*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(ep));
  EmitPack p;   // field by field (an address-space-qualified aggregate does not copy-construct)
  p.gh = ep->gh;
  p.gh16 = ep->gh16;
  p.ts = ep->ts;
  p.ord = ep->ord;
  p.recs = ep->recs;
  p.regs = ep->regs;
  p.wcnt = ep->wcnt;
  p.filter = ep->filter;
  p.cap = ep->cap;
  p.skip = ep->skip;
  p.np_bits = ep->np_bits;
  E.gh = global_ptr<uint32_t>(p.gh);
  E.gh16 = p.gh16 ? global_ptr<uint16_t>(p.gh16) : nullptr;
  E.ts = global_ptr<const uint32_t>(p.ts);
  E.ord = global_ptr<const unsigned long long>(p.ord);
  E.recs = global_ptr<Rec>(p.recs);
  E.regs = global_ptr<uint16_t>(p.regs);
  E.wcnt = global_ptr<uint32_t>(p.wcnt);
  A.filter = global_ptr<const unsigned long long>(p.filter);
  A.cap = p.cap;
  A.skip = p.skip;
  A.np_bits = p.np_bits;
}

// The record of one line, or false (need).  kPre: the line's order and
// timestamp were loaded ahead (o_pre, ts_pre; kPf 2).
// kPreF: the rule's filter bound was loaded ahead too (f_pre; k_classify_pair
// loads both lines' bounds before either line's stores)
template <bool kPre = false, bool kPreF = false>
__device__ __forceinline__ bool make_rec(uint32_t i, uint4 t, uint32_t gid, const Agg& A, const Emit& E, Rec& r,
                                         unsigned long long o_pre = 0, uint32_t ts_pre = 0,
                                         unsigned long long f_pre = 0) {
  const uint32_t flags = (t.w >> 16) & 0xFFu;
  bool need = gid != kNoGid && (flags & RSA_F_HIT) && (flags & RSA_F_BUILT) && A.cap > 0 && !(A.skip & 2u);
  if (!need) return false;
  // the three loads in flight together (one memory round trip, not two)
  const unsigned long long o = kPre ? o_pre : E.ord[i];
  const uint32_t ts = kPre ? ts_pre : __builtin_nontemporal_load(&E.ts[i]);
  const unsigned long long f = kPreF ? f_pre : A.filter[gid];
  r.ts = ts;
  if (o > f) return false;   // exact skip: capped with threshold <= filter < order
  conn_key(t, gid, r.kA, r.kB);
  r.order = o;
  r.region = key_region(A, slot_hash(r.kA, r.kB));
  return true;
}

// Emission for one wave of classified lines (wave-uniform call; lanes with
// !in do nothing).  i = the lane's line, lines of a wave are i - lane .. + 63.
template <bool kPre = false, bool kPreF = false>
__device__ __forceinline__ void emit_wave(uint32_t i, uint32_t n, bool in, uint4 t, uint32_t gid, const Agg& A,
                                          const Emit& E, unsigned long long o_pre = 0, uint32_t ts_pre = 0,
                                          unsigned long long f_pre = 0) {
  const uint32_t flags = (t.w >> 16) & 0xFFu;
  const bool matched = in && gid != kNoGid;
  const bool hit = matched && (flags & RSA_F_HIT);
  if (in) {
    if (E.gh16)
      E.gh16[i] = (uint16_t)(matched ? (gid | (hit ? 0x8000u : 0u)) : 0xFFFFu);
    else
      E.gh[i] = matched ? (gid | (hit ? 0x80000000u : 0u)) : 0xFFFFFFFFu;
  }
  Rec r;
  const bool need = in && make_rec<kPre, kPreF>(i, t, gid, A, E, r, o_pre, ts_pre, f_pre);
  const unsigned long long mask = __ballot(need);
  const uint32_t lane = __lane_id();
  const uint32_t w0 = i - lane;   // the window's first line (waves cover aligned 64-line windows)
  if (need) {
    const uint32_t slot = w0 + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
    E.recs[slot] = r;
    E.regs[slot] = (uint16_t)r.region;
  }
  if (lane == 0 && w0 < n) E.wcnt[w0 / kWin] = (uint32_t)__popcll(mask);
}

// Emission of one deferred line (k_tail): appended to its window's records.
__device__ __forceinline__ void emit_one(uint32_t i, uint4 t, uint32_t gid, const Agg& A, const Emit& E) {
  const uint32_t flags = (t.w >> 16) & 0xFFu;
  const bool matched = gid != kNoGid;
  const bool hit = matched && (flags & RSA_F_HIT);
  if (E.gh16)
    E.gh16[i] = (uint16_t)(matched ? (gid | (hit ? 0x8000u : 0u)) : 0xFFFFu);
  else
    E.gh[i] = matched ? (gid | (hit ? 0x80000000u : 0u)) : 0xFFFFFFFFu;
  Rec r;
  if (!make_rec(i, t, gid, A, E, r)) return;
  const uint32_t w = i / kWin;
  const uint32_t slot = w * kWin + atomicAdd(&E.wcnt[w], 1u);   // < 64: a window has 64 lines
  E.recs[slot] = r;
  E.regs[slot] = (uint16_t)r.region;
}

// Pass 1a — first-match classification (mapper.py:159-189): gid or RSA_NO_RULE
// per tuple into gout (nullable), index image staged in LDS when kImg > 0;
// with kEmit the line's counter word and table record (emit_wave).  Lines
// whose index candidate failed verification kAttempts times go to `tail`
// (k_tail scans and emits them exactly).
template <int kImg, bool kEmit, int kMode, bool kNarrow>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(kImg > kImgSmallMax ? 4 : 8, 8))) void k_classify(
    EmitPack EP, const uint4* __restrict__ T, unsigned long long n, int32_t* __restrict__ gout, Rules R,
    unsigned int* flags, uint32_t* tail, unsigned long long* tail_n) {
  Agg A = {};
  Emit E = {};
  __shared__ __attribute__((aligned(16))) uint32_t lds_img[kImg > 0 ? kImg : 4];
  __shared__ uint32_t lds_task[kMode == 1 ? 1024 : 64];   // 64 words per wave (index_lookup_wave)
  lds_w32* scr = (lds_w32*)lds_task + (kMode == 1 ? (threadIdx.x & ~63u) : 0u);
  if (kImg > 0 && R.indexed) {
    const uint4* src = reinterpret_cast<const uint4*>(R.img);
    uint4* dst = reinterpret_cast<uint4*>(lds_img);
    for (uint32_t w = threadIdx.x; w < (R.img_words + 3) / 4; w += blockDim.x) dst[w] = src[w];
  }
  __syncthreads();
  // 32-bit line indices: batches are < 2^31 lines (run_pass1, rsa_classify_only)
  const uint32_t n32 = (uint32_t)n;
  const uint32_t stride = gridDim.x * blockDim.x;
#ifdef RSA_PHASE_PROF
  PhaseAcc ph = {};
  unsigned long long waves_seen = 0;
#endif
  // Prefetch (kPf): 1 = the next iteration's tuple, 2 = also
  // its order and timestamp (the emission loads), loaded before this
  // iteration's stores, so waiting for them does not wait for the stores
  // (vmcnt counts stores too).  Default: 2 for the global-image variants and
  // the bucket index (52-53 VGPRs, room at 8 waves/SIMD), 0 for the LDS-image
  // pht variants (at the 64-VGPR budget prefetching spills: 0.77 -> 1.03 /
  // 1.17 ms per cfg3 launch, profiles/r04ai_*).
  constexpr int kPf = (kImg == 0 || kMode == 2) ? 2 : 0;
  const uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x;
  uint4 t_next = make_uint4(0u, 0u, 0u, 0u);
  unsigned long long o_next = 0ull;
  uint32_t ts_next = 0u;
  if (kPf >= 1 && i0 < n32) t_next = T[i0];
  if (kPf >= 2 && kEmit && i0 < n32) {
    classify_emit_args(EP, A, E);
    o_next = E.ord[i0];
    ts_next = __builtin_nontemporal_load(&E.ts[i0]);
  }
  for (uint32_t base = blockIdx.x * blockDim.x; base < n32; base += stride) {
#ifdef RSA_PHASE_PROF
    ph.last = __builtin_amdgcn_s_memtime();
    ++waves_seen;
#endif
    const uint32_t i = base + threadIdx.x;
    const bool in = i < n32;
    uint4 t;
    unsigned long long o_cur = 0ull;
    uint32_t ts_cur = 0u;
    if (kPf >= 1) {
      t = t_next;
      t_next = i + stride < n32 ? T[i + stride] : make_uint4(0u, 0u, 0u, 0u);
      if (kPf >= 2 && kEmit) {
        classify_emit_args(EP, A, E);
        o_cur = o_next;
        ts_cur = ts_next;
        o_next = i + stride < n32 ? E.ord[i + stride] : 0ull;
        ts_next = i + stride < n32 ? __builtin_nontemporal_load(&E.ts[i + stride]) : 0u;
      }
    } else {
      t = in ? T[i] : make_uint4(0u, 0u, 0u, 0u);
    }
    const bool valid = in && (((t.w >> 16) & 0xFFu) & RSA_F_VALID);
    uint32_t gid;
    if (kImg > 0) {
      gid = classify_wave<false, kMode, kNarrow>(t, valid, R, (const lds_u32*)lds_img, flags, scr RSA_PH_ARG);
    } else {
      gid = classify_wave<false, kMode, kNarrow>(t, valid, R, R.img, flags, scr RSA_PH_ARG);
    }
    const bool defer = gid == kDefer;
    const unsigned long long dm = __ballot(defer);
    if (dm) {   // rare: one device atomic per wave (no workgroup barrier in the loop)
      const int leader = __builtin_ctzll(dm);
      unsigned long long pos = 0;
      if ((int)__lane_id() == leader) pos = atomicAdd(tail_n, (unsigned long long)__popcll(dm));
      pos = ((unsigned long long)__builtin_amdgcn_readlane((uint32_t)(pos >> 32), leader) << 32) |
            __builtin_amdgcn_readlane((uint32_t)pos, leader);
      if (defer) tail[pos + __popcll(dm & ((1ull << __lane_id()) - 1ull))] = (uint32_t)i;
    }
    if (gout && in && !defer) gout[i] = (int32_t)gid;
    if (kEmit) {
      classify_emit_args(EP, A, E);
      emit_wave<kPf >= 2>(i, n32, in && !defer, t, gid, A, E, o_cur, ts_cur);
    }
    PH(7);
  }
#ifdef RSA_PHASE_PROF
  if (__lane_id() == 0) {
    for (int k = 0; k < 8; ++k) atomicAdd(&g_phase[k], ph.acc[k]);
    atomicAdd(&g_phase[8], waves_seen);
  }
#endif
}

// Pass 1a for the global bucket image, two lines per lane (lines i and i +
// stride of each iteration; see classify_pair_bkt).  The tuples of the next
// iteration and the emission's order / timestamp loads are issued ahead, as
// in k_classify's global variants.
// (256-thread workgroups: no LDS and no barriers, so a CU holds as many as
// its registers allow -- six at the 80-VGPR cap, 24 waves)
#ifndef RSA_PAIR_WAVES
#define RSA_PAIR_WAVES 6   // minimum waves per SIMD (register cap: 80 VGPRs)
#endif
constexpr int kPairThreads = 256;
template <bool kEmit>
__global__ __launch_bounds__(kPairThreads) __attribute__((amdgpu_waves_per_eu(RSA_PAIR_WAVES, 8))) void k_classify_pair(
    EmitPack EP, const uint4* __restrict__ T, unsigned long long n, int32_t* __restrict__ gout, Rules R,
    unsigned int* flags, uint32_t* tail, unsigned long long* tail_n) {
  Agg A = {};
  Emit E = {};
  const uint32_t n32 = (uint32_t)n;
  const uint32_t stride = gridDim.x * blockDim.x;
  const uint32_t* img = R.img;
  for (uint32_t base = blockIdx.x * blockDim.x; base < n32; base += 2 * stride) {
    const uint32_t i0 = base + threadIdx.x, i1 = i0 + stride;
    const bool in0 = i0 < n32, in1 = i1 < n32;
    const uint4 t0 = in0 ? T[i0] : make_uint4(0u, 0u, 0u, 0u);
    const uint4 t1 = in1 ? T[i1] : make_uint4(0u, 0u, 0u, 0u);
    unsigned long long o0 = 0ull, o1 = 0ull;
    uint32_t s0 = 0u, s1 = 0u;
    if (kEmit) {
      classify_emit_args(EP, A, E);
      if (in0) {
        o0 = E.ord[i0];
        s0 = __builtin_nontemporal_load(&E.ts[i0]);
      }
      if (in1) {
        o1 = E.ord[i1];
        s1 = __builtin_nontemporal_load(&E.ts[i1]);
      }
    }
    const bool v0 = in0 && (((t0.w >> 16) & 0xFFu) & RSA_F_VALID);
    const bool v1 = in1 && (((t1.w >> 16) & 0xFFu) & RSA_F_VALID);
    uint32_t g0, g1;
    classify_pair_bkt(t0, v0, t1, v1, R, img, flags, g0, g1);
    const bool d0 = g0 == kDefer, d1 = g1 == kDefer;
    const unsigned long long dm0 = __ballot(d0), dm1 = __ballot(d1);
    if (dm0 | dm1) {   // (testing only: R.force_defer) one device atomic per wave
      const int leader = __builtin_ctzll(dm0 | dm1);
      unsigned long long pos = 0;
      if ((int)__lane_id() == leader)
        pos = atomicAdd(tail_n, (unsigned long long)(__popcll(dm0) + __popcll(dm1)));
      pos = ((unsigned long long)__builtin_amdgcn_readlane((uint32_t)(pos >> 32), leader) << 32) |
            __builtin_amdgcn_readlane((uint32_t)pos, leader);
      const unsigned long long below = (1ull << __lane_id()) - 1ull;
      if (d0) tail[pos + __popcll(dm0 & below)] = i0;
      if (d1) tail[pos + __popcll(dm0) + __popcll(dm1 & below)] = i1;
    }
    if (gout && in0 && !d0) gout[i0] = (int32_t)g0;
    if (gout && in1 && !d1) gout[i1] = (int32_t)g1;
    if (kEmit) {
      classify_emit_args(EP, A, E);
      // both rules' filter bounds before either line's stores (for the lines
      // make_rec takes: a rule, hit and BUILT, the table on)
      const bool tab = A.cap > 0 && !(A.skip & 2u);
      const uint32_t hb = RSA_F_HIT | RSA_F_BUILT;
      const bool r0 = tab && in0 && !d0 && g0 != kNoGid && (((t0.w >> 16) & hb) == hb);
      const bool r1 = tab && in1 && !d1 && g1 != kNoGid && (((t1.w >> 16) & hb) == hb);
#ifndef RSA_ABL_NOFILTER
#define RSA_ABL_NOFILTER 0   // PROFILING builds only (results invalid): no filter-bound loads
#endif
      const unsigned long long f0 = RSA_ABL_NOFILTER ? ~0ull : (r0 ? A.filter[g0] : 0ull);
      const unsigned long long f1 = RSA_ABL_NOFILTER ? ~0ull : (r1 ? A.filter[g1] : 0ull);
      emit_wave<true, true>(i0, n32, in0 && !d0, t0, g0, A, E, o0, s0, f0);
      emit_wave<true, true>(i1, n32, in1 && !d1, t1, g1, A, E, o1, s1, f1);
    }
  }
}

// Pass 1a, deferred lines: exact linear scan of their whole list (+ emission).
template <bool kEmit>
__global__ __launch_bounds__(kBlock) void k_tail(const uint4* __restrict__ T, int32_t* __restrict__ gout, Rules R,
                                                 unsigned int* flags, const uint32_t* __restrict__ tail,
                                                 const unsigned long long* tail_n, Agg A, Emit E) {
  const unsigned long long n = *tail_n;
  const unsigned long long stride = (unsigned long long)gridDim.x * kBlock;
  for (unsigned long long base = (unsigned long long)blockIdx.x * kBlock; base < n; base += stride) {
    const unsigned long long j = base + threadIdx.x;
    const bool in = j < n;
    const unsigned long long i = in ? tail[j] : 0u;
    const uint4 t = in ? T[i] : make_uint4(0u, 0u, 0u, 0u);
    const bool valid = in && (((t.w >> 16) & 0xFFu) & RSA_F_VALID);
#ifdef RSA_PHASE_PROF
    PhaseAcc ph = {};   // (the exact tail is not profiled)
#endif
    const uint32_t gid = classify_wave<true, 0, false>(t, valid, R, R.img, flags, nullptr RSA_PH_ARG);
    if (gout && in) gout[i] = (int32_t)gid;
    if (kEmit && in) emit_one((uint32_t)i, t, gid, A, E);
  }
}

// packed[key] += m | h << 32 for every lane with `m` (h implies m): one
// 64-bit device atomic per line (the lanes sharing the key of the wave's
// first one combined into one), where a per-key waterfall over the wave
// serialises up to 64 rounds on waves whose rules all differ -- the common
// case with millions of rules (BASELINE config 4).  Wave-uniform control flow.
__device__ __forceinline__ void wave_count_packed(bool m, bool h, uint32_t key, unsigned long long* packed) {
  const unsigned long long pending = __ballot(m);
  if (!pending) return;
  const unsigned long long hm = __ballot(h);
  const int leader = __builtin_ctzll(pending);
  const uint32_t k = __builtin_amdgcn_readlane(key, leader);
  const unsigned long long peers = __ballot(m && key == k);
  if ((int)__lane_id() == leader)
    atomicAdd(&packed[k], (unsigned long long)__popcll(peers) | ((unsigned long long)__popcll(peers & hm) << 32));
  if (m && key != k) atomicAdd(&packed[key], 1ull | ((unsigned long long)(h ? 1u : 0u) << 32));
}

// matches/hits += the packed counts of one launch (< 2^31 lines, so neither
// half overflows), packed cleared for the next launch.
__global__ __launch_bounds__(kBlock) void k_count_flush(unsigned long long* __restrict__ packed, uint32_t n_rules,
                                                       unsigned long long* __restrict__ matches,
                                                       unsigned long long* __restrict__ hits) {
  const uint32_t stride = gridDim.x * kBlock;
  for (uint32_t r = blockIdx.x * kBlock + threadIdx.x; r < n_rules; r += stride) {
    const unsigned long long v = packed[r];
    if (!v) continue;
    packed[r] = 0;
    matches[r] += v & 0xFFFFFFFFull;
    if (v >> 32) hits[r] += v >> 32;
  }
}

// Per-rule line / hit counters from the gid|hit words of pass 1a
// (connlist-reducer.py:146-148 and the mapper's per-rule output lines):
// LDS-privatised when the rules fit (kLds), else wave-aggregated atomics.
template <int kLds>
__global__ __launch_bounds__(1024) void k_count(const uint32_t* __restrict__ gh, unsigned long long n, uint32_t n_rules,
                                                Agg A) {
  __shared__ uint32_t cnt[kLds > 0 ? 2 * kLds : 1];
  if (kLds > 0) {
    for (uint32_t r = threadIdx.x; r < 2u * kLds; r += blockDim.x) cnt[r] = 0;
    __syncthreads();
  }
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x * 4;
  for (unsigned long long base = (unsigned long long)blockIdx.x * blockDim.x * 4; base < n; base += stride) {
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const unsigned long long i = base + (unsigned long long)k * blockDim.x + threadIdx.x;
      w[k] = i < n ? gh[i] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool m = w[k] != 0xFFFFFFFFu;
      const uint32_t g = w[k] & 0x7FFFFFFFu;
      const bool h = m && (w[k] >> 31);
      if (kLds > 0) {
        if (m) atomicAdd(&cnt[g], 1u);
        if (h) atomicAdd(&cnt[kLds + g], 1u);
      } else {
        wave_count_packed(m, h, g, A.packed);
      }
    }
  }
  if (kLds > 0) {
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < n_rules; r += blockDim.x) {
      const uint32_t m = cnt[r], hh = cnt[kLds + r];
      if (m) atomicAdd(&A.matches[r], (unsigned long long)m);
      if (hh) atomicAdd(&A.hits[r], (unsigned long long)hh);
    }
  }
}

// The same LDS histogram over 16-bit words (gid | hit << 15, 0xFFFF = no rule;
// rule sets that fit 15 bits): eight words per 16-B load, half the bytes.
template <int kLds>
__global__ __launch_bounds__(1024) void k_count16(const uint16_t* __restrict__ gh, unsigned long long n,
                                                  uint32_t n_rules, Agg A) {
  __shared__ uint32_t cnt[2 * kLds];
  for (uint32_t r = threadIdx.x; r < 2u * kLds; r += blockDim.x) cnt[r] = 0;
  __syncthreads();
  const unsigned long long n8 = n / 8;   // whole 16-B groups (gh is 16-B aligned: the batch's word 0)
  const uint4* g4 = reinterpret_cast<const uint4*>(gh);
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long q = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; q < n8 + 1; q += stride) {
    uint32_t w[4];
    if (q < n8) {
      const uint4 v = g4[q];
      w[0] = v.x;
      w[1] = v.y;
      w[2] = v.z;
      w[3] = v.w;
    } else {   // the tail words (< 8)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const unsigned long long i = q * 8 + 2 * k;
        const uint32_t lo = i < n ? gh[i] : 0xFFFFu, hi = i + 1 < n ? gh[i + 1] : 0xFFFFu;
        w[k] = lo | (hi << 16);
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t x = (w[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
      if (x != 0xFFFFu) {
        const uint32_t g = x & 0x7FFFu;
        atomicAdd(&cnt[g], 1u);
        if (x >> 15) atomicAdd(&cnt[kLds + g], 1u);
      }
    }
  }
  __syncthreads();
  for (uint32_t r = threadIdx.x; r < n_rules; r += blockDim.x) {
    const uint32_t m = cnt[r], hh = cnt[kLds + r];
    if (m) atomicAdd(&A.matches[r], (unsigned long long)m);
    if (hh) atomicAdd(&A.hits[r], (unsigned long long)hh);
  }
}

// ---- Per-rule counters past the LDS histogram (rule sets > kCnt, BASELINE
// config 4's 3.45M rules): one device atomic per line (k_count<0>) runs at
// ~13 G lines/s against memory-side atomics, so the gid|hit words are instead
// counting-sorted by rule block (kCntBlock consecutive rules) and every block
// counted in LDS:
//   k_cnt_hist / exclusive scan / k_cnt_scatter   words grouped by block
//   k_seg_starts / k_cnt_plan                      block segments cut into tasks
//                                                  of <= kCntChunk words
//   k_cnt_reduce                                   one LDS histogram per task,
//                                                  added to matches/hits (plain
//                                                  read-modify-write when the task
//                                                  is its block's only one)
// 16 B of streaming traffic per line instead of one scattered atomic.
constexpr int kMaxRegions = 4096;   // table regions (and count blocks) per partition
constexpr uint32_t kCntBits = 13, kCntBlock = 1u << kCntBits;
constexpr uint32_t kCntChunk = 1u << 18;

struct CntTask {
  unsigned long long beg, end;
  uint32_t block, single;
};

// lanes whose key equals the first active lane's: that lane adds their count
// (one LDS atomic instead of up to 64 on one address); returns whether this
// lane's own add is still due
__device__ __forceinline__ bool wave_peer_add(bool act, uint32_t key, uint32_t* cnt, uint32_t add_hits,
                                              bool h, uint32_t* hcnt) {
  const unsigned long long pending = __ballot(act);
  if (!pending) return false;
  const int leader = __builtin_ctzll(pending);
  const uint32_t k = __builtin_amdgcn_readlane(key, leader);
  const unsigned long long peers = __ballot(act && key == k);
  const unsigned long long hm = add_hits ? __ballot(act && h) : 0ull;
  if ((int)__lane_id() == leader) {
    atomicAdd(&cnt[k], (uint32_t)__popcll(peers));
    const uint32_t hh = (uint32_t)__popcll(peers & hm);
    if (hh) atomicAdd(&hcnt[k], hh);
  }
  return act && key != k;
}

__global__ __launch_bounds__(1024) void k_cnt_hist(const uint32_t* __restrict__ gh, unsigned long long n,
                                                   uint32_t n_blocks, uint32_t n_tiles, uint32_t tile_len,
                                                   uint32_t* __restrict__ hist) {
  __shared__ uint32_t hc[kMaxRegions];
  const uint32_t tile = blockIdx.x;
  for (uint32_t b = threadIdx.x; b < n_blocks; b += blockDim.x) hc[b] = 0;
  __syncthreads();
  const unsigned long long beg = (unsigned long long)tile * tile_len;
  const unsigned long long end = beg + tile_len < n ? beg + tile_len : n;
  for (unsigned long long base = beg; base < end; base += 4ull * blockDim.x) {   // block-uniform trip count
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const unsigned long long i = base + (unsigned long long)k * blockDim.x + threadIdx.x;
      w[k] = i < end ? gh[i] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool act = w[k] != 0xFFFFFFFFu;
      const uint32_t b = (w[k] & 0x7FFFFFFFu) >> kCntBits;
      if (wave_peer_add(act, b, hc, 0, false, nullptr)) atomicAdd(&hc[b], 1u);
    }
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < n_blocks; b += blockDim.x) hist[(size_t)b * n_tiles + tile] = hc[b];
}

__global__ __launch_bounds__(1024) void k_cnt_scatter(const uint32_t* __restrict__ gh, unsigned long long n,
                                                      uint32_t n_blocks, uint32_t n_tiles, uint32_t tile_len,
                                                      const uint32_t* __restrict__ offs, uint32_t* __restrict__ out) {
  __shared__ uint32_t cur[kMaxRegions];
  const uint32_t tile = blockIdx.x;
  for (uint32_t b = threadIdx.x; b < n_blocks; b += blockDim.x) cur[b] = offs[(size_t)b * n_tiles + tile];
  __syncthreads();
  const unsigned long long beg = (unsigned long long)tile * tile_len;
  const unsigned long long end = beg + tile_len < n ? beg + tile_len : n;
  const uint32_t lane = __lane_id();
  for (unsigned long long base = beg; base < end; base += 4ull * blockDim.x) {
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const unsigned long long i = base + (unsigned long long)k * blockDim.x + threadIdx.x;
      w[k] = i < end ? gh[i] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool act = w[k] != 0xFFFFFFFFu;
      const uint32_t b = (w[k] & 0x7FFFFFFFu) >> kCntBits;
      // the first active lane's block: one cursor bump for all its peers
      const unsigned long long pending = __ballot(act);
      if (!pending) continue;
      const int leader = __builtin_ctzll(pending);
      const uint32_t bl = __builtin_amdgcn_readlane(b, leader);
      const unsigned long long peers = __ballot(act && b == bl);
      uint32_t at = 0;
      if ((int)lane == leader) at = atomicAdd(&cur[bl], (uint32_t)__popcll(peers));
      at = __builtin_amdgcn_readlane(at, leader);
      if (act && b == bl) {
        out[at + (uint32_t)__popcll(peers & ((1ull << lane) - 1ull))] = w[k];
      } else if (act) {
        out[atomicAdd(&cur[b], 1u)] = w[k];
      }
    }
  }
}

// One workgroup: block segments [starts[b], starts[b+1]) cut into tasks of at
// most `chunk` words; ctl[0] = the task count.
__global__ __launch_bounds__(1024) void k_cnt_plan(const unsigned long long* __restrict__ starts, uint32_t n_blocks,
                                                   uint32_t chunk, CntTask* __restrict__ tasks, uint32_t max_tasks,
                                                   uint32_t* __restrict__ ctl) {
  __shared__ uint32_t sh[18];
  uint32_t carry = 0;
  for (uint32_t b0 = 0; b0 < n_blocks; b0 += blockDim.x) {
    const uint32_t b = b0 + threadIdx.x;
    const unsigned long long s = b < n_blocks ? starts[b] : 0, e = b < n_blocks ? starts[b + 1] : 0;
    const uint32_t k = (uint32_t)((e - s + chunk - 1) / chunk);
    uint32_t total;
    const uint32_t off = carry + block_exscan(k, sh, &total);
    for (uint32_t q = 0; q < k && off + q < max_tasks; ++q) {
      CntTask t;
      t.beg = s + (unsigned long long)q * chunk;
      t.end = t.beg + chunk < e ? t.beg + chunk : e;
      t.block = b;
      t.single = k == 1;
      tasks[off + q] = t;
    }
    carry += total;
  }
  if (threadIdx.x == 0) ctl[0] = carry < max_tasks ? carry : max_tasks;
}

__global__ __launch_bounds__(1024) void k_cnt_reduce(const uint32_t* __restrict__ words,
                                                     const CntTask* __restrict__ tasks, const uint32_t* __restrict__ ctl,
                                                     uint32_t n_rules, unsigned long long* __restrict__ matches,
                                                     unsigned long long* __restrict__ hits) {
  __shared__ uint32_t cm[kCntBlock], ch[kCntBlock];
  if (blockIdx.x >= ctl[0]) return;   // workgroup-uniform
  const CntTask t = tasks[blockIdx.x];
  for (uint32_t r = threadIdx.x; r < kCntBlock; r += blockDim.x) cm[r] = ch[r] = 0;
  __syncthreads();
  for (unsigned long long base = t.beg; base < t.end; base += 4ull * blockDim.x) {
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const unsigned long long i = base + (unsigned long long)k * blockDim.x + threadIdx.x;
      w[k] = i < t.end ? words[i] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool act = w[k] != 0xFFFFFFFFu;
      const uint32_t r = w[k] & (kCntBlock - 1u);
      const bool h = act && (w[k] >> 31);
      if (wave_peer_add(act, r, cm, 1, h, ch)) {
        atomicAdd(&cm[r], 1u);
        if (h) atomicAdd(&ch[r], 1u);
      }
    }
  }
  __syncthreads();
  const uint32_t r0 = t.block << kCntBits;
  for (uint32_t r = threadIdx.x; r < kCntBlock && r0 + r < n_rules; r += blockDim.x) {
    const uint32_t m = cm[r], h = ch[r];
    if (!m) continue;
    if (t.single) {
      matches[r0 + r] += m;
      if (h) hits[r0 + r] += h;
    } else {
      atomicAdd(&matches[r0 + r], (unsigned long long)m);
      if (h) atomicAdd(&hits[r0 + r], (unsigned long long)h);
    }
  }
}

// ---- Pass 1b — the reducer's aggregation of classified lines
// (connlist-reducer.py:62-79,146-176), as an on-chip shuffle.
//
// The distinct-connection table is split into regions of 2^rs_bits slots; a
// key's region is the top np_bits of its slot hash and its home slot lies in
// that region (linear probing wraps inside it).  Table writes are scattered
// memory transactions (the chip sustains ~20 G/s of them against ~125 G/s of
// 64-B streaming lines), so instead of one read-modify-write per line:
//   k_aggregate   per-rule line/hit counters (LDS histogram) and, for each hit
//                 line the BUILT regex matched that can still change an output
//                 (order <= filter[gid]), a 32-B record appended in line order;
//   k_part_hist / exclusive scan / k_part_scatter
//                 a stable-free counting sort of the records by region;
//   k_reduce      one workgroup per region: records aggregated in an LDS hash
//                 table (count, first, last, min_order per key), then merged
//                 into the region's slots with plain loads and stores — the
//                 workgroup owns its region for the whole kernel, new slots are
//                 claimed in an LDS copy of the region's occupancy bitmap.
// Records per key shrink to one merge per LDS round.

constexpr int kAggU = 4;
// Pass 1b with the rule already known per line (rsa_aggregate_gids, the
// reducer drop-in): per-rule counters (LDS histogram when the rules fit) and
// the window-compacted records of emit_wave.
template <int kLds>
__global__ __launch_bounds__(1024) void k_aggregate(const uint4* __restrict__ T, const uint32_t* __restrict__ TS,
                                                    const unsigned long long* __restrict__ ORD,
                                                    const int32_t* __restrict__ G, unsigned long long n,
                                                    uint32_t n_rules, Agg A, Rec* __restrict__ recs,
                                                    uint16_t* __restrict__ regs, uint32_t* __restrict__ wcnt) {
  __shared__ uint32_t cnt[kLds > 0 ? 2 * kLds : 1];   // matches, hits
  const bool counters = !(A.skip & 1u);
  if (kLds > 0) {
    for (uint32_t r = threadIdx.x; r < 2u * kLds; r += blockDim.x) cnt[r] = 0;
    __syncthreads();
  }
  const bool table = A.cap > 0 && !(A.skip & 2u);
  const unsigned long long span = (unsigned long long)blockDim.x * kAggU;
  for (unsigned long long base = (unsigned long long)blockIdx.x * span; base < n;
       base += (unsigned long long)gridDim.x * span) {
#pragma unroll
    for (int k = 0; k < kAggU; ++k) {
      const unsigned long long i = base + (unsigned long long)k * blockDim.x + threadIdx.x;
      const bool in = i < n;
      uint32_t gid = in ? (uint32_t)G[i] : kNoGid;
      const uint4 t = in ? T[i] : make_uint4(0u, 0u, 0u, 0u);
      const uint32_t flags = (t.w >> 16) & 0xFFu;
      if (gid != kNoGid && gid >= n_rules) {
        atomicOr(&A.flags[1], 2u);
        gid = kNoGid;
      }
      const bool matched = gid != kNoGid;
      const bool hit = matched && (flags & RSA_F_HIT);
      if (counters) {
        if (kLds > 0) {
          if (matched) atomicAdd(&cnt[gid], 1u);
          if (hit) atomicAdd(&cnt[kLds + gid], 1u);
        } else {
          wave_count_packed(matched, hit, gid, A.packed);
        }
      }
      bool need = table && hit && (flags & RSA_F_BUILT);
      unsigned long long o = 0;
      if (need) {
        o = ORD[i];
        need = o <= A.filter[gid];
      }
      need = need && in;
      const unsigned long long mask = __ballot(need);
      const uint32_t lane = __lane_id();
      const unsigned long long w0 = i - lane;   // the wave's 64-line window
      if (need) {
        Rec r;
        conn_key(t, gid, r.kA, r.kB);
        r.order = o;
        r.ts = TS[i];
        r.region = key_region(A, slot_hash(r.kA, r.kB));
        const unsigned long long slot = w0 + __popcll(mask & ((1ull << lane) - 1ull));
        recs[slot] = r;
        regs[slot] = (uint16_t)r.region;
      }
      if (lane == 0 && w0 < n) wcnt[w0 / kWin] = (uint32_t)__popcll(mask);
    }
  }
  if (kLds > 0) {
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < n_rules; r += blockDim.x) {
      const uint32_t m = cnt[r], hh = cnt[kLds + r];
      if (m) atomicAdd(&A.matches[r], (unsigned long long)m);
      if (hh) atomicAdd(&A.hits[r], (unsigned long long)hh);
    }
  }
}

// Counting sort of the records by region.  The records are window-compacted
// (window w's wcnt[w] records in slots 64 w ..), tiles are `tile` lines (a
// power of two multiple of 64, chosen per launch as the largest that still
// gives >= kPartTilesWant workgroups, capped at kPartTileMax so the scatter's
// runs per region stay ~10 records); the histogram matrix is region-major (hist[region * n_tiles +
// tile]) so that its exclusive scan gives every (region, tile) run its output
// offset.
constexpr uint32_t kPartTileMin = 8192, kPartTileMax = 262144;
[[maybe_unused]] constexpr uint32_t kPartTilesWant = 384;   // (RSA_PART_TILES_CU=0: the power-of-two tiles)
#ifndef RSA_PART_TILES_CU
#define RSA_PART_TILES_CU 1   // region sort tiles: RSA_PART_TPC per CU (else the power-of-two tiles for >= 384 workgroups)
#endif
#ifndef RSA_PART_TPC
#define RSA_PART_TPC 2        // tiles per CU (the scatter holds two 1024-thread workgroups per CU)
#endif

// Both partition kernels walk their tile as groups of kPartW windows per wave:
// the group's window counts are wave-uniform (scalar) loads, and the live
// records of the group are dealt to the lanes densely (record q of the group ->
// window k = #{prefix <= q}, slot q - prefix[k]), so a wave does ~one pass per
// 64 records instead of one per 64 window slots (windows are ~1/3 full).
// Tiles are multiples of 8192 lines, so a tile's first window is a multiple of
// kPartW.
constexpr int kPartW = 4;

struct WinGroup {
  uint32_t p1, p2, p3, tot;
};

__device__ __forceinline__ WinGroup win_group(const uint32_t* __restrict__ wcnt, unsigned long long w0,
                                              unsigned long long wend) {
  uint32_t c[kPartW];
#pragma unroll
  for (int k = 0; k < kPartW; ++k) c[k] = w0 + k < wend ? wcnt[w0 + k] : 0u;
  WinGroup g;
  g.p1 = c[0];
  g.p2 = g.p1 + c[1];
  g.p3 = g.p2 + c[2];
  g.tot = g.p3 + c[3];
  return g;
}

// line-slot index of record q (< g.tot) of the window group starting at w0
__device__ __forceinline__ unsigned long long win_slot(const WinGroup& g, unsigned long long w0, uint32_t q) {
  const uint32_t k = (uint32_t)(q >= g.p1) + (uint32_t)(q >= g.p2) + (uint32_t)(q >= g.p3);
  const uint32_t pre = k == 0 ? 0u : k == 1 ? g.p1 : k == 2 ? g.p2 : g.p3;
  return (w0 + k) * kWin + (q - pre);
}

__global__ __launch_bounds__(1024) void k_part_hist(const uint16_t* __restrict__ regs, const uint32_t* __restrict__ wcnt,
                                                    unsigned long long n, uint32_t n_regions, uint32_t n_tiles,
                                                    uint32_t tile_len, uint32_t* __restrict__ hist) {
  __shared__ uint32_t hcount[kMaxRegions];
  const uint32_t tile = blockIdx.x;
  for (uint32_t r = threadIdx.x; r < n_regions; r += blockDim.x) hcount[r] = 0;
  __syncthreads();
  const unsigned long long beg = (unsigned long long)tile * tile_len;
  const unsigned long long end = beg + tile_len < n ? beg + tile_len : n;
  const unsigned long long wend = (end + kWin - 1) / kWin;
  const uint32_t lane = __lane_id(), nwv = blockDim.x >> 6;
  for (unsigned long long w0 = beg / kWin + (threadIdx.x >> 6) * kPartW; w0 < wend; w0 += (unsigned long long)nwv * kPartW) {
    const WinGroup g = win_group(wcnt, w0, wend);
    for (uint32_t q = lane; q < g.tot; q += 2 * kWin) {   // two records per lane in flight
      const bool two = q + kWin < g.tot;
      const uint32_t r0 = regs[win_slot(g, w0, q)];
      const uint32_t r1 = two ? regs[win_slot(g, w0, q + kWin)] : 0u;
      atomicAdd(&hcount[r0], 1u);
      if (two) atomicAdd(&hcount[r1], 1u);
    }
  }
  __syncthreads();
  for (uint32_t r = threadIdx.x; r < n_regions; r += blockDim.x) hist[(size_t)r * n_tiles + tile] = hcount[r];
}



// A window group's counts with one 16-B load (wcnt is padded by kPartW words
// and w0 is a multiple of kPartW): no per-window branches.
__device__ __forceinline__ WinGroup win_group4(const uint32_t* __restrict__ wcnt, unsigned long long w0,
                                               unsigned long long wend) {
  const uint4 c = *reinterpret_cast<const uint4*>(wcnt + w0);
  WinGroup g;
  g.p1 = w0 < wend ? c.x : 0u;
  g.p2 = g.p1 + (w0 + 1 < wend ? c.y : 0u);
  g.p3 = g.p2 + (w0 + 2 < wend ? c.z : 0u);
  g.tot = g.p3 + (w0 + 3 < wend ? c.w : 0u);
  return g;
}

__global__ __launch_bounds__(1024) void k_part_scatter(const Rec* __restrict__ recs, const uint16_t* __restrict__ regs,
                                                       const uint32_t* __restrict__ wcnt, unsigned long long n,
                                                       uint32_t n_regions, uint32_t n_tiles, uint32_t tile_len,
                                                       const uint32_t* __restrict__ offs, Rec* __restrict__ out,
                                                       Rec* __restrict__ junk) {
  __shared__ uint32_t cur[kMaxRegions];
  const uint32_t tile = blockIdx.x;
  for (uint32_t r = threadIdx.x; r < n_regions; r += blockDim.x) cur[r] = offs[(size_t)r * n_tiles + tile];
  __syncthreads();
  const unsigned long long beg = (unsigned long long)tile * tile_len;
  const unsigned long long end = beg + tile_len < n ? beg + tile_len : n;
  const unsigned long long wend = (end + kWin - 1) / kWin;
  const uint32_t lane = __lane_id(), nwv = blockDim.x >> 6;
  const unsigned long long wstep = (unsigned long long)nwv * kPartW;
  unsigned long long w0 = beg / kWin + (threadIdx.x >> 6) * kPartW;
  // software pipeline over the wave's trips (a trip = two records per lane of
  // one window group; a group holds <= 256 records, so <= 2 trips): the
  // window counts are read a group ahead and the records a trip ahead, both
  // before the current trip's scattered stores, so the waits for those loads
  // do not include the stores' completion (vmcnt counts stores too, in issue
  // order).  For that every load and store is unconditional: invalid lanes
  // read the group's first slot and write a junk record of their own lane.
  // The records travel as plain 16-B vectors (region = the record's last
  // word: the 2-B region array is not read here).
  const uint4* R4 = reinterpret_cast<const uint4*>(recs);
  uint4* O4 = reinterpret_cast<uint4*>(out);
  uint4* J4 = reinterpret_cast<uint4*>(junk) + 2 * lane;
  const WinGroup zero = {0, 0, 0, 0};
  const unsigned long long wlast = beg / kWin;   // an in-range group start for clamped loads
  WinGroup g = w0 < wend ? win_group4(wcnt, w0, wend) : zero;
  uint4 c1 = *reinterpret_cast<const uint4*>(wcnt + (w0 + wstep < wend ? w0 + wstep : wlast));
  uint32_t qb = 0;
  const unsigned long long wl = w0 < wend ? w0 : wlast;
  bool v0 = lane < g.tot, v1 = lane + kWin < g.tot;
  unsigned long long j0 = v0 ? win_slot(g, wl, lane) : wl * kWin;
  unsigned long long j1 = v1 ? win_slot(g, wl, lane + kWin) : wl * kWin;
  uint4 a0 = R4[2 * j0], b0 = R4[2 * j0 + 1], a1 = R4[2 * j1], b1 = R4[2 * j1 + 1];
  while (w0 < wend) {
    const bool adv = qb + 2 * kWin >= g.tot;   // wave-uniform: the next trip is the next window group's first
    const unsigned long long nw0 = adv ? w0 + wstep : w0;
    WinGroup ng = g;
    if (adv) {
      const unsigned long long w1 = w0 + wstep;
      ng.p1 = w1 < wend ? c1.x : 0u;
      ng.p2 = ng.p1 + (w1 + 1 < wend ? c1.y : 0u);
      ng.p3 = ng.p2 + (w1 + 2 < wend ? c1.z : 0u);
      ng.tot = ng.p3 + (w1 + 3 < wend ? c1.w : 0u);
    }
    const uint32_t nqb = adv ? 0u : qb + 2 * kWin;
    // the counts of the group after nw0 (used next iteration)
    const uint4 c2 = *reinterpret_cast<const uint4*>(wcnt + (nw0 + wstep < wend ? nw0 + wstep : wlast));
    const unsigned long long nwl = nw0 < wend ? nw0 : wlast;
    const bool nv0 = nqb + lane < ng.tot, nv1 = nqb + lane + kWin < ng.tot;
    const unsigned long long nj0 = nv0 ? win_slot(ng, nwl, nqb + lane) : nwl * kWin;
    const unsigned long long nj1 = nv1 ? win_slot(ng, nwl, nqb + lane + kWin) : nwl * kWin;
    const uint4 na0 = R4[2 * nj0], nb0 = R4[2 * nj0 + 1], na1 = R4[2 * nj1], nb1 = R4[2 * nj1 + 1];
    const uint32_t p0 = v0 ? atomicAdd(&cur[b0.w], 1u) : 0u;
    const uint32_t p1 = v1 ? atomicAdd(&cur[b1.w], 1u) : 0u;
    uint4* d0 = v0 ? O4 + 2 * (size_t)p0 : J4;
    uint4* d1 = v1 ? O4 + 2 * (size_t)p1 : J4;
    d0[0] = a0;
    d0[1] = b0;
    d1[0] = a1;
    d1[1] = b1;
    a0 = na0;
    b0 = nb0;
    a1 = na1;
    b1 = nb1;
    v0 = nv0;
    v1 = nv1;
    w0 = nw0;
    g = ng;
    c1 = c2;
    qb = nqb;
  }
}

// Exclusive scan of n uint32 (three launches: per-block scan + block sums,
// scan of the block sums in one workgroup, add).  kScanBlock elements per block.
constexpr int kScanBlock = 4096;

__global__ __launch_bounds__(1024) void k_scan_blocks(uint32_t* __restrict__ a, unsigned long long n,
                                                      uint32_t* __restrict__ sums) {
  __shared__ uint32_t sh[18];
  const unsigned long long beg = (unsigned long long)blockIdx.x * kScanBlock + threadIdx.x * 4;
  uint32_t v[4], c = 0;
  for (int k = 0; k < 4; ++k) {
    v[k] = beg + k < n ? a[beg + k] : 0u;
    c += v[k];
  }
  uint32_t total;
  uint32_t run = block_exscan(c, sh, &total);
  for (int k = 0; k < 4; ++k) {
    if (beg + k < n) a[beg + k] = run;
    run += v[k];
  }
  if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

// (sums[nb] receives the grand total)
__global__ __launch_bounds__(1024) void k_scan_sums(uint32_t* __restrict__ sums, uint32_t nb) {
  __shared__ uint32_t sh[18];
  uint32_t carry = 0;
  for (uint32_t b0 = 0; b0 < nb; b0 += blockDim.x) {
    const uint32_t j = b0 + threadIdx.x;
    const uint32_t v = j < nb ? sums[j] : 0u;
    uint32_t total;
    const uint32_t ex = block_exscan(v, sh, &total);
    if (j < nb) sums[j] = carry + ex;
    carry += total;
  }
  if (threadIdx.x == 0) sums[nb] = carry;
}

__global__ __launch_bounds__(1024) void k_scan_add(uint32_t* __restrict__ a, unsigned long long n,
                                                   const uint32_t* __restrict__ sums) {
  const unsigned long long beg = (unsigned long long)blockIdx.x * kScanBlock + threadIdx.x * 4;
  const uint32_t add = sums[blockIdx.x];
  for (int k = 0; k < 4; ++k)
    if (beg + k < n) a[beg + k] += add;
}

// One workgroup per region: LDS aggregation of the region's records in rounds
// (a round takes at most as many records as the LDS table has free entries
// below 3/4 load, so it can never overflow; the table is flushed once fewer than
// 512 free entries remain below that load, and at the end), each flush merging every LDS entry into the
// region's slots.  Only this workgroup touches the region during the kernel:
// existing keys are found through the region's occupancy bitmap (slots
// occupied before this flush hold published keys; a slot claimed during this
// flush belongs to a DIFFERENT key, since the keys of one flush are distinct)
// and updated with plain loads and stores; a new key claims a free slot with
// an LDS atomic on the bitmap copy and writes the whole slot.
// LDS hash entries (a multiple of the 1024-thread block): 3072 (108 KiB) for
// pass 1, 2048 for the sparser pass-2 recount — one workgroup per CU either way.
#ifndef RSA_RED1
#define RSA_RED1 3072
#endif
template <int kPass>
constexpr int kRedE = kPass == 1 ? RSA_RED1 : 2048;
#ifndef RSA_REGION_MAX_BITS
#define RSA_REGION_MAX_BITS 16
#endif
constexpr int kRegionMaxBits = RSA_REGION_MAX_BITS;   // region <= 2^16 slots (bitmap copy 8 KiB)

// kPass 1: the pass-1 reduction above.  kPass 2: the cap recount
// (connlist-reducer.py:151-176 after the dict froze) from the records pass 1
// kept: records of capped rules with order <= P are aggregated the same way
// into the pass-2 fields of their (existing) slots; nothing is inserted.  A
// region's records may lie in several segments (one per pass-1 launch):
// starts[s * (n_regions + 1) + r] .. starts[s * (n_regions + 1) + r + 1].
constexpr int kMaxSegs = 16;
#ifndef RSA_HOT_TRIES
#define RSA_HOT_TRIES 1   // lds_agg_insert_lane: wave-combining tries for keys shared by >= kHotMin lanes
                          // (r05o: 2 -> 1 cfg5 9.63 -> 9.45 ms/step, cfg3 within noise; 0: cfg5 10.28)
#endif
constexpr int kHotTries = RSA_HOT_TRIES, kHotMin = 8;
// k_reduce / k_hot_combine flush the LDS table at 3/4 of its entries (5/8
// and 7/8 measured slower: profiles/r06/ab_kreduce.txt)
template <int kE>
constexpr uint32_t kRedRoom = (uint32_t)(3 * kE) / 4u;
__device__ __forceinline__ unsigned long long readlane64(unsigned long long v, int l) {
  return ((unsigned long long)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l) << 32) |
         __builtin_amdgcn_readlane((uint32_t)v, l);
}
// One (possibly pre-combined) record per lane into a workgroup's LDS
// aggregation table (open addressing; the caller keeps it below 3/4 load):
// count summed, first/last min/max, first-seen order min (kMinOrder).  Hot
// keys: a rule with one distinct connection puts all its records into one
// region, so lanes sharing the key of one of the wave's first live lanes are
// combined with wave reductions and enter the table as ONE insert (LDS atomics
// on one address serialise over the lanes).  Wave-uniform call.
// Returns true for the lane that created a new table entry (the caller counts
// them into `used` with one LDS atomic per wave: a per-lane add on that one
// word serialises over the wave's new keys).
template <int kE, bool kMinOrder>
__device__ __forceinline__ bool lds_agg_insert_lane(unsigned long long (&e_kA)[kE], unsigned long long (&e_kB)[kE],
                                                    unsigned long long (&e_mo)[kE], uint32_t (&e_first)[kE],
                                                    uint32_t (&e_last)[kE], uint32_t (&e_cnt)[kE], bool have,
                                                    unsigned long long kA, unsigned long long kB, unsigned long long mo,
                                                    uint32_t first, uint32_t last, uint32_t cnt) {
  unsigned long long pending = __ballot(have);
  for (int att = 0; att < kHotTries && pending; ++att) {
    const int l0 = __builtin_ctzll(pending);
    const unsigned long long kA0 = readlane64(kA, l0), kB0 = readlane64(kB, l0);
    const bool dom = have && kA == kA0 && kB == kB0;
    const unsigned long long dm = __ballot(dom);
    pending &= ~dm;
    if (__popcll(dm) >= kHotMin) {
      uint32_t f = dom ? first : 0xFFFFFFFFu, l = dom ? last : 0u, c = dom ? cnt : 0u;
      unsigned long long o = dom ? mo : ~0ull;
#pragma unroll
      for (int sh = 32; sh; sh >>= 1) {
        f = min(f, (uint32_t)__shfl_xor((int)f, sh));
        l = max(l, (uint32_t)__shfl_xor((int)l, sh));
        c += (uint32_t)__shfl_xor((int)c, sh);
        const unsigned long long oo = __shfl_xor(o, sh);
        o = oo < o ? oo : o;
      }
      if (dom) {
        if ((int)__lane_id() == l0) {
          cnt = c;
          first = f;
          last = l;
          mo = o;
        } else {
          have = false;
        }
      }
    }
  }
  if (!have) return false;
  const uint32_t h = (uint32_t)mix64(kA ^ (kB * 0x9e3779b97f4a7c15ull));
  uint32_t e = (kE & (kE - 1)) == 0 ? (h & (kE - 1)) : __umulhi(h, (uint32_t)kE);
  while (true) {
    // kB and kA read with both loads in flight (one LDS round trip): the LDS
    // executes a wave's operations in issue order (volatile keeps that order),
    // and a creator stores kA before it publishes kB, so a kA read issued
    // after a kB read that sees the published key sees its final kA
    // (profiles/r06/ab_kreduce.txt: aggregation 3.29 -> 3.26 ms/step at cfg3)
    const unsigned long long cur = *reinterpret_cast<volatile unsigned long long*>(&e_kB[e]);
    const unsigned long long curA = *reinterpret_cast<volatile unsigned long long*>(&e_kA[e]);
    if (cur == kEmpty) {
      if (atomicCAS(&e_kB[e], kEmpty, kBusy) == kEmpty) {
        e_kA[e] = kA;
        e_mo[e] = mo;
        e_first[e] = first;
        e_last[e] = last;
        e_cnt[e] = cnt;
        __hip_atomic_store(&e_kB[e], kB, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        return true;
      }
      continue;
    }
    if (cur == kBusy) continue;
    if (cur == kB && curA == kA) {
      atomicAdd(&e_cnt[e], cnt);
      atomicMin(&e_first[e], first);
      atomicMax(&e_last[e], last);
      if (kMinOrder) atomicMin(&e_mo[e], mo);
      return false;
    }
    e = e + 1 == (uint32_t)kE ? 0u : e + 1;
  }
}

template <int kE, bool kMinOrder>
__device__ __forceinline__ void lds_agg_insert(unsigned long long (&e_kA)[kE], unsigned long long (&e_kB)[kE],
                                               unsigned long long (&e_mo)[kE], uint32_t (&e_first)[kE],
                                               uint32_t (&e_last)[kE], uint32_t (&e_cnt)[kE], uint32_t& used,
                                               bool have, unsigned long long kA, unsigned long long kB,
                                               unsigned long long mo, uint32_t first, uint32_t last, uint32_t cnt) {
  const bool fresh = lds_agg_insert_lane<kE, kMinOrder>(e_kA, e_kB, e_mo, e_first, e_last, e_cnt, have, kA, kB, mo,
                                                        first, last, cnt);
  const unsigned long long fm = __ballot(fresh);
  if (fm && (int)__lane_id() == __builtin_ctzll(fm)) atomicAdd(&used, (uint32_t)__popcll(fm));
}

// A hot region's pre-combined records (k_hot_combine): one per key and
// combining workgroup flush, 40 B.
struct HRec {
  unsigned long long kA, kB, mo;
  uint32_t first, last, cnt, pad;
};
static_assert(sizeof(HRec) == 40, "hot record layout");

#ifndef RSA_COUNT_PER_CU
#define RSA_COUNT_PER_CU 1   // k_count workgroups per CU (one is resident: 104 KiB LDS); fewer workgroups, fewer histogram-flush atomics
#endif
#ifndef RSA_RED2_WPE
#define RSA_RED2_WPE 8   // pass 2: 64 VGPRs, two 1024-thread workgroups per CU (73 KiB LDS each)
#endif
#ifndef RSA_RED1_WPE
#define RSA_RED1_WPE 4   // pass 1: one 1024-thread workgroup per CU (3072 LDS entries, 127 KiB)
#endif
template <int kPass, int kE = kRedE<kPass>, int kBits = kRegionMaxBits>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(kPass == 2 ? RSA_RED2_WPE : RSA_RED1_WPE, 8))) void k_reduce(const Rec* __restrict__ recs,
                                                 const unsigned long long* __restrict__ starts, uint32_t n_segs,
                                                 Agg A, const unsigned long long* __restrict__ hot_base,
                                                 const uint32_t* __restrict__ hot_fill, const HRec* __restrict__ hot,
                                                 const unsigned int* __restrict__ skip_zero) {
  __shared__ unsigned long long e_kA[kE], e_kB[kE], e_mo[kE];
  __shared__ uint32_t e_first[kE], e_last[kE], e_cnt[kE];
  __shared__ uint32_t occ[1u << (kBits - 5)];     // occupied before this flush
  __shared__ uint32_t claim[1u << (kBits - 5)];   // claimed during this flush
  __shared__ uint32_t used;
  __shared__ uint32_t sh[18];
  __shared__ unsigned long long sh_base;
  // skip_zero: the device-side count of capped rules (a recount after a cap
  // resolution whose count the host did not read): none, nothing to recount
  if (skip_zero && *skip_zero == 0) return;   // workgroup-uniform
#ifdef RSA_PHASE_PROF
  const unsigned long long rp_t0 = __builtin_amdgcn_s_memtime();
#endif
  const uint32_t region = blockIdx.x;
  const uint32_t n_regions = 1u << A.np_bits;
  // a hot region's records were pre-combined by k_hot_combine: read those
  const bool is_hot = hot_base && hot_base[region] != kEmpty;   // workgroup-uniform
  unsigned long long total_recs = 0;
  if (is_hot) {
    total_recs = hot_fill[region];
    n_segs = 1;
  } else {
    for (uint32_t sg = 0; sg < n_segs; ++sg)
      total_recs += starts[(size_t)sg * (n_regions + 1) + region + 1] - starts[(size_t)sg * (n_regions + 1) + region];
  }
  if (total_recs == 0) return;   // workgroup-uniform
  const uint32_t rs = 1u << A.rs_bits, words = (rs + 31) / 32;
  const unsigned long long rbase = (unsigned long long)region << A.rs_bits;
  uint32_t* gocc = A.occ + (rbase >> 5);
  for (uint32_t w = threadIdx.x; w < words; w += blockDim.x) {
    occ[w] = gocc[w];
    claim[w] = 0;
  }
  for (uint32_t e = threadIdx.x; e < kE; e += blockDim.x) e_kB[e] = kEmpty;
  if (threadIdx.x == 0) used = 0;
  __syncthreads();
#ifdef RSA_PHASE_PROF
  // PROFILING BUILD ONLY: wave 0's wall cycles per phase (the phases end at
  // workgroup barriers, so one wave's clock is the workgroup's)
  unsigned long long rp_t = __builtin_amdgcn_s_memtime(), rp_acc[3] = {0ull, 0ull, 0ull};
  unsigned long long rq_t = rp_t, rq_acc[4] = {0ull, 0ull, 0ull, 0ull};
  rp_acc[0] = rp_t - rp_t0;
#define RP(k)                                                     \
  do {                                                            \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();   \
    rp_acc[k] += t_ - rp_t;                                       \
    rp_t = t_;                                                    \
    rq_t = t_;                                                    \
  } while (0)
// sub-phases (the loads are waited for right after they are issued)
#define RQ(k)                                                     \
  do {                                                            \
    if ((k) == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();   \
    rq_acc[k] += t_ - rq_t;                                       \
    rq_t = t_;                                                    \
  } while (0)
#else
#define RP(k) \
  do {        \
  } while (0)
#define RQ(k) \
  do {        \
  } while (0)
#endif
  uint32_t sg = 0;
  unsigned long long pos = is_hot ? hot_base[region] : starts[region];
  unsigned long long end = is_hot ? pos + total_recs : starts[region + 1];
  while (true) {
    while (pos >= end && sg + 1 < n_segs) {   // workgroup-uniform: next segment
      ++sg;
      pos = starts[(size_t)sg * (n_regions + 1) + region];
      end = starts[(size_t)sg * (n_regions + 1) + region + 1];
    }
    const bool last_round = pos >= end;
    if (!last_round) {
      const uint32_t room = kRedRoom<kE> - used;
      const unsigned long long take = end - pos < room ? end - pos : room;
      __syncthreads();   // every thread has read `used` before any insert changes it
      for (unsigned long long jb = 0; jb < take; jb += blockDim.x) {   // workgroup-uniform trip count
        const unsigned long long j = jb + threadIdx.x;
        bool have = j < take;
        unsigned long long kA = 0, kB = 0, mo = 0;
        uint32_t first = 0, last = 0, cnt = 1;
        if (is_hot) {
          if (have) {
            const HRec hr = hot[pos + j];
            kA = hr.kA;
            kB = hr.kB;
            mo = hr.mo;
            first = hr.first;
            last = hr.last;
            cnt = hr.cnt;
          }
        } else {
          if (have) {
            const Rec r = recs[pos + j];
            kA = r.kA;
            kB = r.kB;
            mo = r.order;
            first = last = r.ts;
          }
        }
        RQ(0);
        if (kPass == 2 && !is_hot && have) {   // (hot records of pass 2 were filtered when combined)
          const unsigned long long P = A.thresh[kB >> 32];
          if (P == RSA_NO_THRESHOLD || mo > P) have = false;
        }
        lds_agg_insert<kE, kPass == 1>(e_kA, e_kB, e_mo, e_first, e_last, e_cnt, used, have, kA, kB, mo,
                                                 first, last, cnt);
        RQ(1);
      }
      pos += take;
      __syncthreads();
      bool more = pos < end;
      for (uint32_t q = sg + 1; q < n_segs && !more; ++q)
        more = starts[(size_t)q * (n_regions + 1) + region + 1] > starts[(size_t)q * (n_regions + 1) + region];
      RP(1);
      if (used + 512u <= kRedRoom<kE> && more) continue;   // workgroup-uniform: room for 512 more
    }
    if (used > 0) {   // workgroup-uniform (read after a barrier)
      // flush: merge every LDS entry into the region; new slots are appended to
      // the used list with ONE device atomic per flush (a per-wave append on
      // the single cursor word would serialise ~30 atomics per workgroup on it)
      constexpr int kPer = kE / 1024;
      unsigned long long new_slot[kPer];   // statically indexed (a counter index would spill it)
      bool is_new[kPer];
      // the home slots of this thread's entries first, every load in flight
      // at once (the table is ~3% full, so nearly every key is settled at its
      // home slot: an update there needs no further round trip).  Slots
      // occupied before this flush are written only by the workgroup's one
      // entry of their key, so the prefetched words stay current.
      uint32_t home[kPer];
      bool at_home[kPer];
      v4u pk[kPer], pm[kPer], pc[kPer];
#pragma unroll
      for (int q = 0; q < kPer; ++q) {
        const uint32_t e = threadIdx.x + q * blockDim.x;
        const unsigned long long kB = e_kB[e];
        home[q] = kB != kEmpty ? (uint32_t)slot_hash(e_kA[e], kB) & (rs - 1) : 0u;
        at_home[q] = kB != kEmpty && ((occ[home[q] >> 5] >> (home[q] & 31)) & 1u);
        if (at_home[q]) {
          const Slot* sl = &A.slots[rbase + home[q]];
          pk[q] = *reinterpret_cast<const v4u*>(&sl->kA);
          if (kPass == 1) pm[q] = *reinterpret_cast<const v4u*>(&sl->min_order);
          pc[q] = *reinterpret_cast<const v4u*>(&sl->count);
        }
      }
#pragma unroll
      for (int q = 0; q < kPer; ++q) {
        const uint32_t e = threadIdx.x + q * blockDim.x;
        const unsigned long long kB = e_kB[e];
        bool fresh = false;
        unsigned long long slot = kEmpty;
        const uint32_t gid = (uint32_t)(kB >> 32);
        const unsigned long long kA = e_kA[e];
        if (at_home[q] && (((unsigned long long)pk[q].w << 32) | pk[q].z) == kB &&
            (((unsigned long long)pk[q].y << 32) | pk[q].x) == kA) {
          Slot* sl = &A.slots[rbase + home[q]];
          v4u c = pc[q];
          if (kPass == 1) {
            const v4u m = pm[q];
            const unsigned long long mo = ((unsigned long long)m.y << 32) | m.x;
            const unsigned long long nmo = e_mo[e] < mo ? e_mo[e] : mo;
            v4u nm;
            nm.x = (uint32_t)nmo;
            nm.y = (uint32_t)(nmo >> 32);
            nm.z = min(m.z, e_first[e]);
            nm.w = max(m.w, e_last[e]);
            *reinterpret_cast<v4u*>(&sl->min_order) = nm;
            if (nmo < mo) A.ukey[sl->pad[0]] = nmo;   // the cap resolution's copy of the key
            c.x += e_cnt[e];
            if (A.tent2 && A.filter[gid] != RSA_NO_THRESHOLD) {
              c.y += e_cnt[e];
              c.z = min(c.z, e_first[e]);
              c.w = max(c.w, e_last[e]);
            }
          } else {
            c.y += e_cnt[e];
            c.z = min(c.z, e_first[e]);
            c.w = max(c.w, e_last[e]);
          }
          *reinterpret_cast<v4u*>(&sl->count) = c;
          e_kB[e] = kEmpty;
        } else if (kB != kEmpty) {
          uint32_t loc = home[q];
          for (uint32_t probes = 0; probes < rs; ++probes, loc = (loc + 1) & (rs - 1)) {
            const uint32_t bit = 1u << (loc & 31);
            if (occ[loc >> 5] & bit) {
              Slot* sl = &A.slots[rbase + loc];
              const v4u k = *reinterpret_cast<const v4u*>(&sl->kA);
              if ((((unsigned long long)k.w << 32) | k.z) != kB || (((unsigned long long)k.y << 32) | k.x) != kA)
                continue;
              if (kPass == 1) {
                const v4u m = *reinterpret_cast<const v4u*>(&sl->min_order);
                const unsigned long long mo = ((unsigned long long)m.y << 32) | m.x;
                const unsigned long long nmo = e_mo[e] < mo ? e_mo[e] : mo;
                v4u nm;
                nm.x = (uint32_t)nmo;
                nm.y = (uint32_t)(nmo >> 32);
                nm.z = min(m.z, e_first[e]);
                nm.w = max(m.w, e_last[e]);
                *reinterpret_cast<v4u*>(&sl->min_order) = nm;
                if (nmo < mo) A.ukey[sl->pad[0]] = nmo;
                sl->count += e_cnt[e];
                if (A.tent2 && A.filter[gid] != RSA_NO_THRESHOLD) {
                  sl->count2 += e_cnt[e];
                  sl->first2 = min(sl->first2, e_first[e]);
                  sl->last2 = max(sl->last2, e_last[e]);
                }
              } else {
                sl->count2 += e_cnt[e];
                sl->first2 = min(sl->first2, e_first[e]);
                sl->last2 = max(sl->last2, e_last[e]);
              }
              slot = rbase + loc;
              break;
            }
            if (kPass == 2) break;   // every pass-2 key was inserted in pass 1
            if (atomicOr(&claim[loc >> 5], bit) & bit) continue;   // claimed in this flush by another key
            // the slot is written below, once its used-list index is known
            // (no other key of this flush reads a claimed slot)
            slot = rbase + loc;
            fresh = true;
            break;
          }
          if (slot == kEmpty) atomicOr(&A.flags[kPass == 1 ? 0 : 1], kPass == 1 ? 1u : 4u);
          if (!fresh) e_kB[e] = kEmpty;
        }
        if (kPass == 1) {
          wave_count_hot(fresh, gid, A.distinct);
          is_new[q] = fresh;
          new_slot[q] = ((unsigned long long)gid << 32) | (uint32_t)slot;
        }
      }
      RQ(2);
      if (kPass == 1) {
        uint32_t total, n_new = 0;
#pragma unroll
        for (int q = 0; q < kPer; ++q) n_new += is_new[q] ? 1u : 0u;
        const uint32_t off = block_exscan(n_new, sh, &total);
        if (threadIdx.x == 0 && total) sh_base = atomicAdd(A.used_n, (unsigned long long)total);
        __syncthreads();
        uint32_t k = 0;
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
          if (!is_new[q]) continue;
          const uint32_t e = threadIdx.x + q * blockDim.x;
          const unsigned long long ui = sh_base + off + k++;
          // the whole 64-B slot as four 16-B stores (Slot layout)
          const unsigned long long kA = e_kA[e], kB = e_kB[e], mo = e_mo[e];
          const uint32_t fi = e_first[e], la = e_last[e], cn = e_cnt[e];
          const bool t2 = A.tent2 && A.filter[(uint32_t)(kB >> 32)] != RSA_NO_THRESHOLD;
          v4u* sw = reinterpret_cast<v4u*>(&A.slots[(uint32_t)new_slot[q]]);
          sw[0] = v4u{(uint32_t)kA, (uint32_t)(kA >> 32), (uint32_t)kB, (uint32_t)(kB >> 32)};
          sw[1] = v4u{(uint32_t)mo, (uint32_t)(mo >> 32), fi, la};
          sw[2] = v4u{cn, t2 ? cn : 0u, t2 ? fi : 0xFFFFFFFFu, t2 ? la : 0u};
          sw[3] = v4u{(uint32_t)ui, 0u, 0u, 0u};
          A.used[ui] = new_slot[q];
          A.ukey[ui] = e_mo[e];
          e_kB[e] = kEmpty;
        }
      }
      __syncthreads();
      for (uint32_t w = threadIdx.x; w < words; w += blockDim.x) {
        occ[w] |= claim[w];
        claim[w] = 0;
      }
      if (threadIdx.x == 0) used = 0;
      __syncthreads();
      RQ(3);
      RP(2);
    }
    if (last_round) break;
  }
  if (kPass == 1)
    for (uint32_t w = threadIdx.x; w < words; w += blockDim.x) gocc[w] = occ[w];
#ifdef RSA_PHASE_PROF
  if (threadIdx.x == 0) {
    constexpr int b = kPass == 1 ? 9 : 17;
    for (int k = 0; k < 3; ++k) atomicAdd(&g_phase[b + k], rp_acc[k]);
    atomicAdd(&g_phase[b + 3], 1ull);
    for (int k = 0; k < 4; ++k) atomicAdd(&g_phase[b + 4 + k], rq_acc[k]);
  }
#endif
#undef RP
#undef RQ
}

// ---- hot regions (skewed traffic: a few connections on most lines, BASELINE
// config 5's Zipf population).  Every record of one key lands in one region,
// and one k_reduce workgroup per region would read a hot region's millions
// of records alone.  k_hot_plan marks the regions holding more than
// max(kHotMinRecs, kHotFactor x the mean) records of the segments and deals
// their ranges out as slices; k_hot_combine (all CUs) aggregates each slice
// in an LDS table and appends one HRec per key and flush to the region's
// contiguous area of the hot buffer; k_reduce then merges that instead.  Pass
// 2 does the same over its filtered records (capped rules, order <= P), so the
// combined counts stay exact for the recount.
constexpr uint32_t kHotSlice = 65536, kHotMinRecs = 65536, kHotFactor = 4;
struct HotTask {
  unsigned long long beg, end;
  uint32_t region, pad;
};
// ctl[0] tasks planned, ctl[1] task cursor; *hot_total: hot buffer records reserved
__global__ void k_hot_plan(const unsigned long long* __restrict__ starts, uint32_t n_segs, uint32_t n_regions,
                           HotTask* __restrict__ tasks, uint32_t max_tasks, uint32_t* __restrict__ ctl,
                           unsigned long long* __restrict__ hot_total, unsigned long long* __restrict__ hot_base,
                           uint32_t* __restrict__ hot_fill, unsigned long long min_recs, uint32_t factor,
                           const unsigned int* __restrict__ skip_zero) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_regions) return;
  if (skip_zero && *skip_zero == 0) {   // (see k_reduce)
    hot_fill[r] = 0;
    hot_base[r] = kEmpty;
    return;
  }
  unsigned long long all = 0, mine = 0;
  for (uint32_t sg = 0; sg < n_segs; ++sg) {
    const unsigned long long* st = starts + (size_t)sg * (n_regions + 1);
    all += st[n_regions] - st[0];
    mine += st[r + 1] - st[r];
  }
  const unsigned long long thr = max(min_recs, factor * (all / n_regions));
  hot_fill[r] = 0;
  if (mine <= thr) {
    hot_base[r] = kEmpty;
    return;
  }
  uint32_t nt = 0;
  for (uint32_t sg = 0; sg < n_segs; ++sg) {
    const unsigned long long* st = starts + (size_t)sg * (n_regions + 1);
    nt += (uint32_t)((st[r + 1] - st[r] + kHotSlice - 1) / kHotSlice);
  }
  const uint32_t t0 = atomicAdd(&ctl[0], nt);
  if (t0 + nt > max_tasks) {   // (cannot happen: max_tasks bounds every plan) leave the region to k_reduce
    hot_base[r] = kEmpty;
    return;
  }
  hot_base[r] = atomicAdd(hot_total, mine);
  uint32_t t = t0;
  for (uint32_t sg = 0; sg < n_segs; ++sg) {
    const unsigned long long* st = starts + (size_t)sg * (n_regions + 1);
    for (unsigned long long b = st[r]; b < st[r + 1]; b += kHotSlice)
      tasks[t++] = HotTask{b, min(b + kHotSlice, st[r + 1]), r, sg};
  }
}

// Persistent grid: every workgroup takes slices until none is left (the
// count planned is read on the device); per slice an LDS table, flushed when
// it could overflow and at the slice end, one device atomic per flush.
template <int kPass>
__global__ __launch_bounds__(1024) void k_hot_combine(const Rec* __restrict__ recs, const HotTask* __restrict__ tasks,
                                                      uint32_t* __restrict__ ctl, Agg A,
                                                      const unsigned long long* __restrict__ hot_base,
                                                      uint32_t* __restrict__ hot_fill, HRec* __restrict__ hot) {
  constexpr int kE = RSA_RED1;
  __shared__ unsigned long long e_kA[kE], e_kB[kE], e_mo[kE];
  __shared__ uint32_t e_first[kE], e_last[kE], e_cnt[kE];
  __shared__ uint32_t used, task;
  __shared__ uint32_t sh[18];
  __shared__ unsigned long long sh_base;
  for (uint32_t e = threadIdx.x; e < (uint32_t)kE; e += blockDim.x) e_kB[e] = kEmpty;
  if (threadIdx.x == 0) used = 0;
  const uint32_t n_tasks = ctl[0];
  while (true) {
    __syncthreads();
    if (threadIdx.x == 0) task = atomicAdd(&ctl[1], 1u);
    __syncthreads();
    const uint32_t t = task;
    if (t >= n_tasks) break;   // workgroup-uniform: every workgroup drains here
    const HotTask T = tasks[t];
    unsigned long long pos = T.beg;
    while (pos < T.end || used > 0) {   // workgroup-uniform (read after a barrier)
      if (pos < T.end) {
        const uint32_t room = kRedRoom<kE> - used;
        const unsigned long long take = T.end - pos < room ? T.end - pos : room;
        __syncthreads();   // every thread has read `used` before any insert changes it
        for (unsigned long long jb = 0; jb < take; jb += blockDim.x) {
          const unsigned long long j = jb + threadIdx.x;
          bool have = j < take;
          Rec r;
          if (have) r = recs[pos + j];
          if (kPass == 2 && have) {
            const unsigned long long P = A.thresh[r.kB >> 32];
            if (P == RSA_NO_THRESHOLD || r.order > P) have = false;
          }
          lds_agg_insert<kE, kPass == 1>(e_kA, e_kB, e_mo, e_first, e_last, e_cnt, used, have, r.kA, r.kB, r.order,
                                         r.ts, r.ts, 1u);
        }
        pos += take;
        __syncthreads();
        if (pos < T.end && used + 1024u <= kRedRoom<kE>) continue;   // room for more of this slice
      }
      // flush: the table's entries to the region's hot area
      constexpr int kPer = kE / 1024;
      uint32_t n_mine = 0;
#pragma unroll
      for (int q = 0; q < kPer; ++q) n_mine += e_kB[threadIdx.x + q * 1024] != kEmpty ? 1u : 0u;
      uint32_t total;
      const uint32_t off = block_exscan(n_mine, sh, &total);
      if (threadIdx.x == 0) sh_base = total ? hot_base[T.region] + atomicAdd(&hot_fill[T.region], total) : 0ull;
      __syncthreads();
      unsigned long long at = sh_base + off;
#pragma unroll
      for (int q = 0; q < kPer; ++q) {
        const uint32_t e = threadIdx.x + q * 1024;
        if (e_kB[e] == kEmpty) continue;
        HRec h;
        h.kA = e_kA[e];
        h.kB = e_kB[e];
        h.mo = e_mo[e];
        h.first = e_first[e];
        h.last = e_last[e];
        h.cnt = e_cnt[e];
        h.pad = 0;
        hot[at++] = h;
        e_kB[e] = kEmpty;
      }
      __syncthreads();
      if (threadIdx.x == 0) used = 0;
      __syncthreads();
    }
  }
}

// Segment starts of one pass-1 launch: starts[r] = base + offs[r * n_tiles],
// starts[n_regions] = base + the record total (written by k_scan_sums).
// (hot_ctl / hot_total / ncap / cursor, nullable: the counters the hot-region
// plan and the next cap resolution accumulate into, zeroed here instead of
// by four memset launches per pass-1 launch; every earlier reader of them
// precedes this kernel in stream order)
__global__ void k_seg_starts(const uint32_t* __restrict__ offs, uint32_t n_tiles, uint32_t n_regions,
                             unsigned long long base, const uint32_t* __restrict__ total, unsigned long long* starts,
                             uint32_t* hot_ctl, unsigned long long* hot_total, unsigned int* ncap,
                             unsigned long long* cursor, unsigned long long* job_recs) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < n_regions) starts[r] = base + offs[(size_t)r * n_tiles];
  if (r == n_regions) {
    starts[r] = base + *total;
    if (job_recs) *job_recs += *total;   // the job's pass-1 records (region policy of the next rsa_reset)
  }
  if (r == 0) {
    if (hot_ctl) hot_ctl[0] = hot_ctl[1] = hot_ctl[2] = hot_ctl[3] = 0u;
    if (hot_total) *hot_total = 0ull;
    if (ncap) *ncap = 0u;
    if (cursor) *cursor = 0ull;
  }
}

// Pass 2: lines with order <= P of capped rules recount count/first/last into
// the pass-2 fields (gids from pass 1 or from a classify-only run).
__global__ __launch_bounds__(kBlock) void k_pass2(const uint4* __restrict__ T, const uint32_t* __restrict__ TS,
                                                  const unsigned long long* __restrict__ ORD, unsigned long long n,
                                                  const int32_t* __restrict__ gin, uint32_t n_rules, Agg A) {
  const unsigned long long stride = (unsigned long long)gridDim.x * kBlock;
  for (unsigned long long base = (unsigned long long)blockIdx.x * kBlock; base < n; base += stride) {
    const unsigned long long i = base + threadIdx.x;
    if (i >= n) continue;
    const uint32_t gid = (uint32_t)gin[i];
    if (gid >= n_rules) continue;
    const uint4 t = T[i];
    const uint32_t flags = (t.w >> 16) & 0xFFu;
    if ((flags & (RSA_F_HIT | RSA_F_BUILT)) != (RSA_F_HIT | RSA_F_BUILT)) continue;
    const unsigned long long P = A.thresh[gid];
    if (P == RSA_NO_THRESHOLD) continue;
    const unsigned long long o = ORD[i];
    if (o > P) continue;
    unsigned long long kA, kB;
    conn_key(t, gid, kA, kB);
    Slot* s = table_find(A, kA, kB);
    if (!s) {
      atomicOr(&A.flags[1], 4u);
      continue;
    }
    const uint32_t ts = TS[i];
    atomicAdd(&s->count2, 1u);
    atomicMin(&s->first2, ts);
    atomicMax(&s->last2, ts);
  }
}

__device__ __forceinline__ void slot_clear(Slot* S, unsigned long long i) {
  Slot s;
  s.kA = 0;
  s.kB = kEmpty;
  s.min_order = kEmpty;
  s.first = 0xFFFFFFFFu;
  s.last = 0;
  s.count = 0;
  s.count2 = 0;
  s.first2 = 0xFFFFFFFFu;
  s.last2 = 0;
  s.pad[0] = s.pad[1] = s.pad[2] = s.pad[3] = 0;
  S[i] = s;
}

__global__ void k_table_init(Slot* S, unsigned long long cap) {
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += stride)
    slot_clear(S, i);
}

// [0]: some rule under a filter bound got a threshold other than the bound;
// [1]: some rule without a bound is capped now.
__global__ void k_tent_check(const unsigned long long* filter, const unsigned long long* thresh, uint32_t n_rules,
                             uint32_t* out) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_rules) return;
  const unsigned long long f = filter[g], t = thresh[g];
  const bool moved = f != RSA_NO_THRESHOLD && t != f, now = f == RSA_NO_THRESHOLD && t != RSA_NO_THRESHOLD;
  if (moved) atomicAdd(&out[0], 1u);   // counts (RSA_DEBUG prints them)
  if (now) atomicAdd(&out[1], 1u);
}

// The pass-2 fields of every used slot back to empty (the last slice's
// tentative counts are replayed by a full recount).
__global__ void k_pass2_clear(Slot* S, const unsigned long long* used, const unsigned long long* n_p,
                              unsigned long long cap) {
  unsigned long long n = *n_p;
  if (n > cap) n = cap;
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    Slot* s = &S[(uint32_t)used[i]];
    s->count2 = 0;
    s->first2 = 0xFFFFFFFFu;
    s->last2 = 0;
  }
}

// Reset only the slots the last job used.
__global__ void k_table_clear(Slot* S, const unsigned long long* used, const unsigned long long* n_p,
                              unsigned long long cap) {
  unsigned long long n = *n_p;
  if (n > cap) n = cap;
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    slot_clear(S, (uint32_t)used[i]);
}

// ---- cap resolution (exact): P = cap-th smallest min_order among a rule's entries.
// Every rule with >= cap entries gets a contiguous segment (allocated by an
// atomic cursor, so no scan is needed); the entries' min_order keys are
// scattered into it and one workgroup per rule radix-selects the cap-th
// smallest key, 8 bits at a time from the top (keys are unique order keys).
//
// prev[g] is an earlier selection of this job (the last filter slice, or "none"):
// an upper bound of the rule's P now, since a rule's entries only gain members
// and their min_orders only decrease.  The cap entries at or below it then
// still are, so the cap-th smallest key now is among the keys <= prev[g]: only
// those are scattered (prev may alias out).
__global__ void k_cap_mark(const unsigned int* distinct, uint32_t n_rules, uint32_t cap,
                           const unsigned long long* prev, uint32_t* cidx, uint32_t* capped_gid,
                           uint32_t* capped_start, uint32_t* capped_fill, unsigned long long* capped_prev,
                           unsigned int* n_capped, unsigned long long* total, unsigned long long* out) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_rules) return;
  const unsigned long long pv = prev[g];
  out[g] = RSA_NO_THRESHOLD;
  if (cap > 0 && distinct[g] >= cap) {
    const unsigned int c = atomicAdd(n_capped, 1u);
    cidx[g] = c;
    capped_gid[c] = g;
    capped_prev[c] = pv;
    capped_start[c] = (uint32_t)atomicAdd(total, (unsigned long long)distinct[g]);
    capped_fill[c] = 0;
  } else {
    cidx[g] = 0xFFFFFFFFu;
  }
}

// Scatter the capped rules' min_order keys into their segments when the
// capped rules do not fit the LDS counters below.  Lanes of one wave that share
// a rule take their positions from one atomic (hot rules would otherwise
// serialise thousands of atomics on one counter).
__device__ __forceinline__ void cap_scatter_waves(const Slot* S, const unsigned long long* used,
                                                  unsigned long long n_used, const uint32_t* cidx,
                                                  const uint32_t* capped_start, uint32_t* capped_fill,
                                                  const unsigned long long* ukey, const unsigned long long* cprev,
                                                  unsigned long long* keys, unsigned long long max_keys,
                                                  unsigned int* flags) {
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long base = (unsigned long long)blockIdx.x * blockDim.x; base < n_used; base += stride) {
    const unsigned long long i = base + threadIdx.x;
    uint32_t c = 0xFFFFFFFFu;
    unsigned long long key = 0;
    if (i < n_used) {
      const unsigned long long u = used[i];
      c = cidx[u >> 32];   // only the capped rules' entries are read
      if (c != 0xFFFFFFFFu) {
        key = ukey ? ukey[i] : S[(uint32_t)u].min_order;
        if (key > cprev[c]) c = 0xFFFFFFFFu;
      }
    }
    const bool ok = c != 0xFFFFFFFFu;
    // lanes that share a rule are grouped first (ballots only, no memory
    // waits), then every group leader reserves its group's positions with ONE
    // returning atomic, all leaders' atomics in flight together
    const unsigned lane = __lane_id();
    unsigned long long pending = __ballot(ok);
    uint32_t my_leader = lane, my_rank = 0, my_cnt = 0;
    while (pending) {
      const int leader = __builtin_ctzll(pending);
      const uint32_t k = __builtin_amdgcn_readlane(c, leader);
      const unsigned long long peers = __ballot(ok && c == k);
      pending &= ~peers;
      if (ok && c == k) {
        my_leader = (uint32_t)leader;
        my_rank = __popcll(peers & ((1ull << lane) - 1ull));
        my_cnt = __popcll(peers);
      }
    }
    uint32_t b = 0;
    if (ok && lane == my_leader) b = atomicAdd(&capped_fill[c], my_cnt);
    b = __shfl(b, (int)my_leader);
    const unsigned long long pos = ok ? (unsigned long long)capped_start[c] + b + my_rank : 0ull;
    if (ok) {
      if (pos < max_keys) keys[pos] = key;
      else atomicOr(&flags[1], 16u);
    }
  }
}

// The scatter when the capped rules fit an LDS counter array (n_capped <=
// kCapLds; else the wave grouping above): each workgroup takes a contiguous
// chunk of the used list, ranks its entries per rule with LDS atomics, reserves
// every rule's run with one global atomic per (workgroup, rule), then writes the
// keys.  Constant work per entry, where the wave grouping loops once per
// distinct rule in the wave.
constexpr int kCapLds = 16384;
constexpr int kCapPer = 16;                 // entries per thread (1024 threads: a chunk of 16384)
__global__ __launch_bounds__(1024) void k_cap_scatter_lds(const Slot* S, const unsigned long long* used,
                                                          const unsigned long long* n_used_p,
                                                          const unsigned int* n_capped_p, uint32_t lds_max,
                                                          const uint32_t* cidx, const uint32_t* capped_start,
                                                          uint32_t* capped_fill, const unsigned long long* ukey,
                                                          const unsigned long long* cprev, unsigned long long* keys,
                                                          unsigned long long max_keys, unsigned int* flags) {
  __shared__ uint32_t cnt[kCapLds];
  // counts are read on the device (no host round trip): a persistent grid
  // walks the chunks of the used list
  const uint32_t n_capped = *n_capped_p;
  if (n_capped == 0) return;   // workgroup-uniform
  const unsigned long long n_used = *n_used_p < max_keys ? *n_used_p : max_keys;   // (overflow: flagged elsewhere)
  if (n_capped > lds_max) {
    cap_scatter_waves(S, used, n_used, cidx, capped_start, capped_fill, ukey, cprev, keys, max_keys, flags);
    return;
  }
  const unsigned long long chunk = 1024ull * kCapPer;
  for (unsigned long long base = (unsigned long long)blockIdx.x * chunk; base < n_used; base += gridDim.x * chunk) {
  for (uint32_t r = threadIdx.x; r < n_capped; r += blockDim.x) cnt[r] = 0;
  __syncthreads();
  uint32_t cc[kCapPer], rank[kCapPer];
  unsigned long long key[kCapPer];
#pragma unroll
  for (int k = 0; k < kCapPer; ++k) {
    const unsigned long long i = base + (unsigned long long)k * blockDim.x + threadIdx.x;
    cc[k] = 0xFFFFFFFFu;
    key[k] = 0;
    if (i < n_used) {
      const unsigned long long u = used[i];
      cc[k] = cidx[u >> 32];
      if (cc[k] != 0xFFFFFFFFu) {
        key[k] = ukey ? ukey[i] : S[(uint32_t)u].min_order;
        if (key[k] > cprev[cc[k]]) cc[k] = 0xFFFFFFFFu;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < kCapPer; ++k) rank[k] = cc[k] != 0xFFFFFFFFu ? atomicAdd(&cnt[cc[k]], 1u) : 0u;
  __syncthreads();
  // every rule's run reserved with one returning device atomic per (workgroup,
  // rule); a thread's atomics are all issued before any result is used, so
  // they overlap instead of paying one round trip each
  {
    constexpr int kRes = kCapLds / 1024;
    uint32_t res[kRes];
#pragma unroll
    for (int q = 0; q < kRes; ++q) {
      const uint32_t r = threadIdx.x + (uint32_t)q * 1024u;
      const uint32_t m = r < n_capped ? cnt[r] : 0u;
      res[q] = m ? atomicAdd(&capped_fill[r], m) : 0u;
    }
#pragma unroll
    for (int q = 0; q < kRes; ++q) {
      const uint32_t r = threadIdx.x + (uint32_t)q * 1024u;
      if (r < n_capped) cnt[r] = res[q];
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kCapPer; ++k) {
    if (cc[k] == 0xFFFFFFFFu) continue;
    const unsigned long long pos = (unsigned long long)capped_start[cc[k]] + cnt[cc[k]] + rank[k];
    if (pos < max_keys) keys[pos] = key[k];
    else atomicOr(&flags[1], 16u);
  }
  __syncthreads();   // cnt is reset for the next chunk
  }
}

// One workgroup per capped rule: the cap-th smallest key of its segment.  A
// min/max pass bounds the keys; radix select then runs on (key - min) in 8-bit
// digits from the highest set bit of (max - min) down, so the digits of keys
// that share their top bits (time-ordered order keys) still spread over the
// bins.  Per-wave LDS histograms keep bin contention inside a wave.
// 256 threads per rule: segments are ~cap..2 cap keys, so a pass is a few
// keys per thread and the passes are barrier-bound; four times the rules in
// flight at once (eight workgroups per CU) instead of wider workgroups
constexpr int kSelThreads = 256;
constexpr int kSelR = 16;   // register-resident keys per thread
__global__ __launch_bounds__(kSelThreads) void k_cap_select(const unsigned long long* keys,
                                                            const uint32_t* capped_start, const uint32_t* capped_fill,
                                                            const uint32_t* capped_gid, uint32_t cap,
                                                            const unsigned int* n_capped_p, unsigned long long* out) {
  constexpr int kWaves = kSelThreads / 64;
  __shared__ uint32_t hist[kWaves][256];
  __shared__ unsigned long long red_min[kWaves], red_max[kWaves];
  __shared__ unsigned long long sh_prefix;
  __shared__ uint32_t sh_k;
  // a persistent grid over the capped rules (their number is read on the device)
  const uint32_t n_capped = *n_capped_p;
  for (uint32_t c = blockIdx.x; c < n_capped; c += gridDim.x) {
  const unsigned long long* seg = keys + capped_start[c];
  const uint32_t n = capped_fill[c];
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // min / max; the segment's first kSelR x kSelThreads keys stay in
  // registers for the digit passes (segments are ~cap..a few x cap keys), the
  // rest is read again per pass
  unsigned long long mn = ~0ull, mx = 0;
  unsigned long long kv[kSelR];
#pragma unroll
  for (int r = 0; r < kSelR; ++r) {
    const uint32_t j = threadIdx.x + (uint32_t)r * kSelThreads;
    kv[r] = j < n ? seg[j] : 0ull;
  }
#pragma unroll
  for (int r = 0; r < kSelR; ++r) {
    if (threadIdx.x + (uint32_t)r * kSelThreads < n) {
      mn = kv[r] < mn ? kv[r] : mn;
      mx = kv[r] > mx ? kv[r] : mx;
    }
  }
  for (uint32_t j = threadIdx.x + kSelR * kSelThreads; j < n; j += kSelThreads) {
    const unsigned long long k = seg[j];
    mn = k < mn ? k : mn;
    mx = k > mx ? k : mx;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long a = __shfl_xor(mn, o), b = __shfl_xor(mx, o);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  if (lane == 0) {
    red_min[w] = mn;
    red_max[w] = mx;
  }
  if (threadIdx.x == 0) {
    sh_prefix = 0;
    sh_k = cap;
  }
  __syncthreads();
  mn = red_min[0];
  mx = red_max[0];
  for (int q = 1; q < kWaves; ++q) {
    mn = red_min[q] < mn ? red_min[q] : mn;
    mx = red_max[q] > mx ? red_max[q] : mx;
  }
  const unsigned long long range = mx - mn;
  const int top = range ? 63 - __builtin_clzll(range) : 0;     // highest set bit of the range
  int shift = top >= 8 ? top - 7 : 0;
  unsigned long long hi_mask = 0;                                // bits above the current digit, fixed so far
  // exactly cap keys (the common case after a filter slice: the cap entries
  // at or below the earlier selection, nothing new below it): the largest;
  // cap 1: the smallest (workgroup-uniform: n, cap)
  if (n == cap || cap == 1) {
    if (threadIdx.x == 0) out[capped_gid[c]] = n == cap ? mx : mn;
    __syncthreads();
    continue;
  }
  while (true) {
    for (int q = threadIdx.x; q < kWaves * 256; q += kSelThreads) (&hist[0][0])[q] = 0;
    __syncthreads();
    const unsigned long long prefix = sh_prefix;
#pragma unroll
    for (int r = 0; r < kSelR; ++r) {
      const unsigned long long v = kv[r] - mn;
      if (threadIdx.x + (uint32_t)r * kSelThreads < n && (v & hi_mask) == prefix)
        atomicAdd(&hist[w][(v >> shift) & 255u], 1u);
    }
    for (uint32_t j = threadIdx.x + kSelR * kSelThreads; j < n; j += kSelThreads) {
      const unsigned long long v = seg[j] - mn;
      if ((v & hi_mask) == prefix) atomicAdd(&hist[w][(v >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      uint32_t hv[4], sum = 0;
      for (int q = 0; q < 4; ++q) {
        uint32_t t = 0;
        for (int ww = 0; ww < kWaves; ++ww) t += hist[ww][4 * lane + q];
        hv[q] = t;
        sum += t;
      }
      uint32_t incl = sum;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t v = __shfl_up(incl, o);
        if ((int)lane >= o) incl += v;
      }
      const uint32_t excl = incl - sum;
      const uint32_t k = sh_k;
      if (k > excl && k <= incl) {
        uint32_t acc = excl, d = 4 * lane;
        for (int q = 0; q < 4; ++q) {
          if (k <= acc + hv[q]) {
            d = 4 * lane + q;
            break;
          }
          acc += hv[q];
        }
        sh_k = k - acc;
        sh_prefix = prefix | ((unsigned long long)d << shift);
      }
    }
    hi_mask |= 0xFFull << shift;
    __syncthreads();
    if (shift == 0) break;
    // the last digit may overlap bits already fixed: they are equal in every
    // key still counted, so the selection stays exact
    shift = shift >= 8 ? shift - 8 : 0;
  }
  if (threadIdx.x == 0) out[capped_gid[c]] = sh_prefix + mn;
  __syncthreads();   // the shared state is rewritten for the next rule
  }
}

__device__ __forceinline__ rsa_conn_record make_record(const Slot& s, int which) {
  rsa_conn_record r;
  r.min_order = s.min_order;
  r.gid = (uint32_t)(s.kB >> 32);
  r.for_ip = (uint32_t)(s.kA >> 32);
  r.to_ip = (uint32_t)s.kA;
  r.to_port = (uint16_t)(s.kB & 0xFFFFu);
  r.pspell = (uint8_t)((s.kB >> 16) & 0xFFu);
  r.pad = 0;
  r.count = which ? s.count2 : s.count;
  r.first = which ? s.first2 : s.first;
  r.last = which ? s.last2 : s.last;
  r.pad2 = 0;
  return r;
}

// mode 0: final report rows; mode 1: export pass-1 aggregates; mode 2: export pass-2;
// mode 3: export the pass-1 aggregates of the entries that can still matter
// under this table's own thresholds (rsa_resolve_cap): no threshold, or
// min_order <= P (a shard's P bounds the global one from above).
// With owner_world > 0 (the multi-GPU merge, RSA_OPT_OWNER_WORLD) the table
// is this rank's shard table AND the merged table of the rules it owns (gid %
// owner_world == owner_rank): exports (modes 1-3) leave the owned entries at
// home, the final rows (mode 0) are the owned entries only.
// Each thread takes kEmitU entries per iteration; one device atomic per
// workgroup iteration reserves the output rows (a per-wave append on the one
// cursor word serialises there).
constexpr int kEmitU = 4;

// The emission decision for used-list entry i (k_emit and the routed export):
// which = -1 (not emitted), 0 (pass-1 aggregates) or 1 (pass-2); the slot is
// gathered into *sl only for emitted entries.
__device__ __forceinline__ int emit_select(const Slot* S, const unsigned long long* used,
                                           const unsigned long long* thresh, int mode, uint32_t owner_world,
                                           uint32_t owner_rank, const unsigned long long* ukey, unsigned long long i,
                                           Slot* sl) {
  const unsigned long long u = used[i];
  const uint32_t gid = (uint32_t)(u >> 32);
  // decided from the used list (rule id) and the key copy before the 64 B
  // slot is gathered: entries of capped rules past the threshold and entries
  // of other owners are never read
  if (owner_world && (gid % owner_world == owner_rank) != (mode == 0)) return -1;
  if (ukey && (mode == 0 || mode == 3)) {
    const unsigned long long P = thresh[gid];
    if (P != RSA_NO_THRESHOLD && ukey[i] > P) return -1;
  }
  *sl = S[(uint32_t)u];
  if (mode == 0) {
    const unsigned long long P = thresh[sl->kB >> 32];
    if (P == RSA_NO_THRESHOLD) return 0;
    return sl->min_order <= P ? 1 : -1;
  }
  if (mode == 1) return 0;
  if (mode == 3) {
    const unsigned long long P = thresh[sl->kB >> 32];
    return (P == RSA_NO_THRESHOLD || sl->min_order <= P) ? 0 : -1;
  }
  return sl->count2 != 0 ? 1 : -1;
}

__global__ __launch_bounds__(1024) void k_emit(const Slot* S, const unsigned long long* used,
                                               const unsigned long long* n_used_p, unsigned long long slot_cap,
                                               const unsigned long long* thresh, int mode, rsa_conn_record* out,
                                               unsigned long long max_out, unsigned long long* cursor,
                                               uint32_t owner_world, uint32_t owner_rank,
                                               const unsigned long long* ukey) {
  __shared__ uint32_t sh[18];
  __shared__ unsigned long long sh_base;
  // the used-slot count is read on the device (persistent grid): no host
  // round trip before the launch
  const unsigned long long n_used = *n_used_p < slot_cap ? *n_used_p : slot_cap;
  const unsigned long long span = (unsigned long long)blockDim.x * kEmitU;
  for (unsigned long long base = (unsigned long long)blockIdx.x * span; base < n_used;
       base += (unsigned long long)gridDim.x * span) {
    int which[kEmitU];
    Slot sl[kEmitU];
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < kEmitU; ++k) {
      const unsigned long long i = base + (unsigned long long)k * blockDim.x + threadIdx.x;
      which[k] = i < n_used ? emit_select(S, used, thresh, mode, owner_world, owner_rank, ukey, i, &sl[k]) : -1;
      c += which[k] >= 0 ? 1u : 0u;
    }
    uint32_t total;
    const uint32_t off = block_exscan(c, sh, &total);
    if (threadIdx.x == 0) sh_base = total ? atomicAdd(cursor, (unsigned long long)total) : 0ull;
    __syncthreads();
    unsigned long long pos = sh_base + off;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kEmitU; ++k) {
      if (which[k] < 0) continue;
      if (pos < max_out) out[pos] = make_record(sl[k], which[k]);
      ++pos;
    }
  }
}

// ---- Routed export (multi-GPU merge, the keyed shuffle of runAnalysis.sh:44):
// the exported records grouped by owner rank gid % world, segment r at the sum
// of the counts of the owners before it.  Pass 1 (kRoute = false) counts per
// owner into counts[world] (device); pass 2 computes the segment bases from
// those counts (each workgroup, world <= kRouteMax) and writes every record at
// base[owner] + a per-(workgroup, owner) range reserved with one device atomic.
// The two passes take the same decisions (the table does not change between
// them).  Records past max_out are dropped; counts hold the true sizes.
constexpr int kRouteMax = 256;
template <bool kRoute>
__global__ __launch_bounds__(1024) void k_emit_route(const Slot* S, const unsigned long long* used,
                                                     const unsigned long long* n_used_p, unsigned long long slot_cap,
                                                     const unsigned long long* thresh, int mode, uint32_t world,
                                                     uint32_t owner_rank, const unsigned long long* ukey,
                                                     unsigned long long* counts, unsigned long long* cursors,
                                                     rsa_conn_record* out, unsigned long long max_out) {
  __shared__ uint32_t cnt[kRouteMax];             // per owner: this group's records (of this iteration, kRoute)
  __shared__ unsigned long long seg[kRouteMax];   // kRoute: segment base of each owner
  __shared__ unsigned long long at[kRouteMax];    // kRoute: this iteration's first row of each owner
  const unsigned long long n_used = *n_used_p < slot_cap ? *n_used_p : slot_cap;
  const unsigned long long span = (unsigned long long)blockDim.x * kEmitU;
  for (uint32_t o = threadIdx.x; o < world; o += blockDim.x) {
    cnt[o] = 0;
    if (kRoute) {
      unsigned long long b = 0;
      for (uint32_t q = 0; q < o; ++q) b += counts[q];
      seg[o] = b;
    }
  }
  __syncthreads();
  for (unsigned long long base = (unsigned long long)blockIdx.x * span; base < n_used;
       base += (unsigned long long)gridDim.x * span) {
    int which[kEmitU];
    Slot sl[kEmitU];
    uint32_t rank[kEmitU];
#pragma unroll
    for (int k = 0; k < kEmitU; ++k) {
      const unsigned long long i = base + (unsigned long long)k * blockDim.x + threadIdx.x;
      which[k] = i < n_used ? emit_select(S, used, thresh, mode, world, owner_rank, ukey, i, &sl[k]) : -1;
      rank[k] = which[k] >= 0 ? atomicAdd(&cnt[(uint32_t)(sl[k].kB >> 32) % world], 1u) : 0u;
    }
    if (!kRoute) continue;
    __syncthreads();
    for (uint32_t o = threadIdx.x; o < world; o += blockDim.x) {
      const uint32_t c = cnt[o];
      at[o] = seg[o] + (c ? atomicAdd(&cursors[o], (unsigned long long)c) : 0ull);
      cnt[o] = 0;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kEmitU; ++k) {
      if (which[k] < 0) continue;
      const unsigned long long pos = at[(uint32_t)(sl[k].kB >> 32) % world] + rank[k];
      if (pos < max_out) out[pos] = make_record(sl[k], which[k]);
    }
  }
  if (!kRoute) {
    __syncthreads();
    for (uint32_t o = threadIdx.x; o < world; o += blockDim.x)
      if (cnt[o]) atomicAdd(&counts[o], (unsigned long long)cnt[o]);
  }
}

// ---- Owner import (multi-GPU merge): received rsa_conn_records are merged
// into this ctx's table the way pass 1 merges its records -- counting-sorted
// by table region into HRecs (k_imp_hist, a scan, k_imp_scatter), then one
// k_reduce workgroup per region (LDS aggregation, plain loads and stores on the
// region's own slots) -- instead of device atomics per record on the slots.
constexpr uint32_t kImpChunk = 16384;   // records per workgroup chunk (16 per thread)

__device__ __forceinline__ void imp_key(const rsa_conn_record& r, unsigned long long& kA, unsigned long long& kB) {
  kA = ((unsigned long long)r.for_ip << 32) | r.to_ip;
  kB = ((unsigned long long)r.gid << 32) | ((unsigned long long)r.pspell << 16) | r.to_port;
}

__global__ __launch_bounds__(1024) void k_imp_hist(const rsa_conn_record* __restrict__ in, unsigned long long n, Agg A,
                                                   uint32_t n_regions, uint32_t* __restrict__ counts) {
  __shared__ uint32_t h[kMaxRegions];
  for (uint32_t r = threadIdx.x; r < n_regions; r += blockDim.x) h[r] = 0;
  __syncthreads();
  for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (unsigned long long)gridDim.x * blockDim.x) {
    unsigned long long kA, kB;
    imp_key(in[i], kA, kB);
    atomicAdd(&h[key_region(A, slot_hash(kA, kB))], 1u);
  }
  __syncthreads();
  for (uint32_t r = threadIdx.x; r < n_regions; r += blockDim.x)
    if (h[r]) atomicAdd(&counts[r], h[r]);
}

// base: exclusive scan of the region counts; cursor: zeroed.  One device
// atomic per (chunk, region) reserves the chunk's run of each region.
__global__ __launch_bounds__(1024) void k_imp_scatter(const rsa_conn_record* __restrict__ in, unsigned long long n,
                                                      Agg A, uint32_t n_regions, const uint32_t* __restrict__ base,
                                                      uint32_t* __restrict__ cursor, HRec* __restrict__ out) {
  __shared__ uint32_t cnt[kMaxRegions], at[kMaxRegions];
  for (unsigned long long c0 = (unsigned long long)blockIdx.x * kImpChunk; c0 < n;
       c0 += (unsigned long long)gridDim.x * kImpChunk) {
    const unsigned long long c1 = c0 + kImpChunk < n ? c0 + kImpChunk : n;
    for (uint32_t r = threadIdx.x; r < n_regions; r += blockDim.x) cnt[r] = 0;
    __syncthreads();
    for (unsigned long long i = c0 + threadIdx.x; i < c1; i += blockDim.x) {
      unsigned long long kA, kB;
      imp_key(in[i], kA, kB);
      atomicAdd(&cnt[key_region(A, slot_hash(kA, kB))], 1u);
    }
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < n_regions; r += blockDim.x) {
      at[r] = cnt[r] ? base[r] + atomicAdd(&cursor[r], cnt[r]) : 0u;
      cnt[r] = 0;
    }
    __syncthreads();
    for (unsigned long long i = c0 + threadIdx.x; i < c1; i += blockDim.x) {
      const rsa_conn_record r = in[i];
      unsigned long long kA, kB;
      imp_key(r, kA, kB);
      const uint32_t g = key_region(A, slot_hash(kA, kB));
      HRec h;
      h.kA = kA;
      h.kB = kB;
      h.mo = r.min_order;
      h.first = r.first;
      h.last = r.last;
      h.cnt = r.count;
      h.pad = 0;
      out[at[g] + atomicAdd(&cnt[g], 1u)] = h;
    }
    __syncthreads();
  }
}

// every region reads its HRecs: hot_base = base, hot_fill = counts
__global__ void k_imp_desc(const uint32_t* __restrict__ base, const uint32_t* __restrict__ counts, uint32_t n_regions,
                           unsigned long long* __restrict__ hot_base, uint32_t* __restrict__ hot_fill) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_regions) return;
  hot_base[r] = base[r];
  hot_fill[r] = counts[r];
}

// New slots are appended to the used list with one device atomic per 1024
// records (workgroup scan), not one per wave: every import record of a fresh
// owner table is new, and per-wave appends serialise on the one cursor word.
__global__ __launch_bounds__(1024) void k_import(const rsa_conn_record* __restrict__ in, unsigned long long n,
                                                 int which, Agg A) {
  __shared__ uint32_t sh[18];
  __shared__ unsigned long long sh_base;
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long base = (unsigned long long)blockIdx.x * blockDim.x; base < n; base += stride) {
    const unsigned long long i = base + threadIdx.x;
    bool fresh = false;
    unsigned long long slot = kEmpty;
    uint32_t gid = kNoGid;
    if (i < n) {
      const rsa_conn_record r = in[i];
      gid = r.gid;
      const unsigned long long kA = ((unsigned long long)r.for_ip << 32) | r.to_ip;
      const unsigned long long kB = ((unsigned long long)r.gid << 32) | ((unsigned long long)r.pspell << 16) | r.to_port;
      if (which == 0) {
        slot = table_combine(A, kA, kB, r.count, r.first, r.last, r.min_order, &fresh);
      } else {
        Slot* s = table_find(A, kA, kB);
        if (!s) {
          atomicOr(&A.flags[1], 8u);
        } else {
          atomicAdd(&s->count2, r.count);
          atomicMin(&s->first2, r.first);
          atomicMax(&s->last2, r.last);
        }
      }
    }
    wave_count_hot(fresh, gid, A.distinct);
    uint32_t total;
    const uint32_t off = block_exscan(fresh ? 1u : 0u, sh, &total);   // workgroup-uniform trip count
    if (threadIdx.x == 0) sh_base = total ? atomicAdd(A.used_n, (unsigned long long)total) : 0ull;
    __syncthreads();
    if (fresh) A.used[sh_base + off] = ((unsigned long long)gid << 32) | (uint32_t)slot;
    __syncthreads();
  }
}

// ---- Shadowed-rule analysis (preprosess_access_lists.py:508-521): cover[i] =
// the smallest j < i with rule j containing rule i (firewallrule.py:128-174),
// or -1.  One thread per rule i; candidate rules j are staged in LDS tiles of
// kShadowTile, ascending; a workgroup stops once every thread has its cover
// or the tiles pass its largest i.
constexpr int kShadowTile = 1024;
static_assert(sizeof(rsa_shadow_rule) == 32, "shadow rule layout");

// One port side of FirewallRule.__contains__ (firewallrule.py:162-171): self
// "any" ([NO_PORT]) contains every list, else every port of the other list
// must be in self's list.  A side is one port (>= 0), -1 (any) or a list
// (<= -2: ports[-v - 2] = count, the ports after it; rsa_shadowed_ports).
__device__ __forceinline__ bool side_contains(int32_t a, int32_t b, const int32_t* __restrict__ ports) {
  if (a == -1) return true;
  if (a >= 0 && b >= -1) return b == a;
  const int32_t* al = a <= -2 ? ports + (-a - 2) : nullptr;
  const int32_t* bl = b <= -2 ? ports + (-b - 2) : nullptr;
  const int32_t na = al ? al[0] : 1, nb = bl ? bl[0] : 1;
  for (int32_t x = 0; x < nb; ++x) {
    const int32_t q = bl ? bl[1 + x] : b;
    bool in = false;
    for (int32_t y = 0; y < na && !in; ++y) in = (al ? al[1 + y] : a) == q;
    if (!in) return false;
  }
  return true;
}

__device__ __forceinline__ bool rule_contains(const rsa_shadow_rule& a, const rsa_shadow_rule& b,
                                              const int32_t* __restrict__ ports) {
  if (a.action != b.action) return false;                         // :146
  if (a.proto != 0 && a.proto != b.proto) return false;           // :150
  // family codes (1 both IPv4, 3..5 IPv6 sides in order-isomorphic
  // interval codes): IPy never contains an address of another version
  if (!a.v4 || a.v4 != b.v4) return false;
  const unsigned long long as = a.src_lo, bs = b.src_lo, ad = a.dst_lo, bd = b.dst_lo;
  if (bs < as || bs + b.src_span > as + a.src_span) return false;   // :154 other.src in self.src
  if (bd < ad || bd + b.dst_span > ad + a.dst_span) return false;   // :158
  if (a.sport != b.sport || a.sport < -1 || b.sport < -1)         // :162-165
    if (!side_contains(a.sport, b.sport, ports)) return false;
  if (a.dport != b.dport || a.dport < -1 || b.dport < -1)         // :168-171
    if (!side_contains(a.dport, b.dport, ports)) return false;
  return true;
}

__global__ __launch_bounds__(1024) void k_shadow(const rsa_shadow_rule* __restrict__ rules, uint32_t n,
                                                 const int32_t* __restrict__ ports, int32_t* __restrict__ cover) {
  __shared__ rsa_shadow_rule tile[kShadowTile];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = i < n;
  rsa_shadow_rule me = {};
  if (in) me = rules[i];
  int32_t found = -1;
  const uint32_t last = min(n, (blockIdx.x + 1) * blockDim.x) - 1;   // largest i of the workgroup
  for (uint32_t t0 = 0; t0 < last; t0 += kShadowTile) {
    if (__syncthreads_and(!in || found >= 0)) break;   // workgroup-uniform
    for (uint32_t q = threadIdx.x; q < kShadowTile; q += blockDim.x)
      if (t0 + q < n) tile[q] = rules[t0 + q];
    __syncthreads();
    if (in && found < 0) {
      const uint32_t lim = min((uint32_t)kShadowTile, i > t0 ? i - t0 : 0u);
      for (uint32_t q = 0; q < lim; ++q) {
        if (rule_contains(tile[q], me, ports)) {
          found = (int32_t)(t0 + q);
          break;
        }
      }
    }
    __syncthreads();
  }
  if (in) cover[i] = found;
}

}  // namespace

struct rsa_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int cu_count = 256;
  std::string err;
  // rules
  rsa_rule_entry* d_entries = nullptr;
  uint32_t n_entries = 0;
  uint32_t* d_off = nullptr;
  std::vector<uint32_t> h_off;        // host copy of the list offsets (validation)
  uint32_t n_lists = 0;
  uint32_t n_rules = 0;
  bool rules_loaded = false;
  // perfect-hash tuple-space index
  uint32_t* d_img = nullptr;
  uint32_t list_off = 0;
  uint32_t img_words = 0;
  rsa_rule_entry* d_resid = nullptr;
  bool index_loaded = false;
  bool indexed = false;
  bool bkt_index = false;               // the loaded image is the bucket index (RSA_BKT_MAGIC)
  bool bkt_filters = false;             // ... with row filters
  bool prune_narrow = false;            // pht index: all pruning tables narrow (image word 5 bit 1)
  bool force_defer = false;
  bool group_tasks = true;     // RSA_OPT_GROUP_TASKS
  uint32_t prof_classify = 0;  // RSA_OPT_PROFILE_CLASSIFY
  bool wave_cap_scatter = false;       // testing: cap scatter by wave grouping (the > kCapLds path)
  // caller-owned counters
  unsigned long long* d_matches = nullptr;
  unsigned long long* d_hits = nullptr;
  unsigned int* d_distinct = nullptr;
  unsigned long long* d_thresh = nullptr;
  void* merge_state = nullptr;   // merge.hip (rsa_merge's buffers)
  uint64_t route_rows = 0;       // RSA_OPT_ROUTE_ROWS (testing)
  // library-owned table
  Slot* d_slots = nullptr;
  unsigned long long slot_cap = 0;    // power of two in use
  unsigned long long slot_alloc = 0;  // allocated (and initialised) slots
  unsigned long long* d_used = nullptr;
  unsigned long long* d_ukey = nullptr;   // per used-list index: the entry's min_order (k_reduce<1> keeps it)
  bool ukey_ok = true;                    // every entry of this job came through k_reduce<1> (no CAS import)
  unsigned long long* d_used_n = nullptr;
  unsigned long long used_last = 0;   // used slots at the last host read (upper bound for clearing)
  bool table_dirty = false;           // used list may be non-empty
  bool slots_init = false;            // every slot of the allocation holds an empty key (the atomic import needs it)
  uint32_t cap = 1000;
  bool table_ready = false;
  unsigned long long* d_filter = nullptr;
  uint32_t filter_len = 0;
  unsigned long long* d_packed = nullptr;   // k_count / k_aggregate packed counters (rules > kCnt)
  // hot-region split (k_hot_plan / k_hot_combine)
  uint32_t min_regions_log2 = 10;           // RSA_OPT_MIN_REGIONS_LOG2: >= 1024 k_reduce workgroups (4 per CU)
  uint32_t region_records = 49152;           // RSA_OPT_REGION_RECORDS: regions >= previous job's records / this
  bool reduce_big = true;                    // RSA_OPT_REDUCE_BIG: 4096-entry k_reduce<1> above 1024 regions
  unsigned long long* d_job_recs = nullptr;  // pass-1 records of the current job (k_seg_starts accumulates)
  bool job_recs_valid = false;               // d_job_recs holds a finished job's count
  unsigned long long h_job_recs = 0;         // d_job_recs as read by the last emission (no extra sync)
  bool h_job_recs_valid = false;
  bool tent2_on = false;                    // the current pass-1 launch is the last slice after the filter steps
  uint32_t late_seg = 0xFFFFFFFFu;          // its record segment (pass-2 fields of filtered rules hold its records)
  uint32_t tent_skip = 0;                   // jobs left without the tentative pass-2 fields (set when they missed)
  bool classify_pair = true;            // RSA_OPT_CLASSIFY_PAIR: the global bucket image classifies two lines per lane
  uint32_t* d_chk = nullptr;                // [0] a filtered rule's threshold moved, [1] a rule capped only now
  bool parse_staged = false;                // RSA_OPT_PARSE_STAGED (textparse.hip): LDS-staged lines, not register windows
  bool region_import = true;                // RSA_OPT_REGION_IMPORT: rsa_import by region sort + k_reduce
  bool slots_clean = true;                  // no slot holds a key of an earlier job (k_import's CAS claims need it)
  bool hot_split = true;                    // RSA_OPT_HOT_SPLIT
  bool hot_ctl_zeroed = false;              // d_hot_ctl / d_hot_total zeroed by the last k_seg_starts
  bool cap_ctl_zeroed = false;              // d_flags[2] / d_cursor zeroed by the last k_seg_starts
  bool ncap_on_device = false;              // d_flags[2] = capped rules of the last rsa_resolve_cap(ctx, NULL):
                                            //   the next rsa_recount may skip on the device when it is 0
  unsigned long long hot_min = kHotMinRecs; // RSA_OPT_HOT_MIN: a hot region holds more than max(hot_min,
  uint32_t hot_factor = kHotFactor;         //   hot_factor x the mean region) records
  void* d_hot = nullptr;                    // HRec[hot_alloc]
  size_t hot_alloc = 0;
  void* d_hot_tasks = nullptr;              // HotTask[tasks_alloc]
  size_t tasks_alloc = 0;
  unsigned long long* d_hot_base = nullptr; // [kMaxRegions]
  uint32_t* d_hot_fill = nullptr;           // [kMaxRegions]
  uint32_t* d_hot_ctl = nullptr;            // [4]: tasks planned, task cursor
  unsigned long long* d_hot_total = nullptr;
  // per-rule counters by rule block (k_cnt_*), rule sets > kCnt
  bool count_sort = true;                   // RSA_OPT_COUNT_SORT
  uint32_t owner_world = 0, owner_rank = 0; // RSA_OPT_OWNER_WORLD / _RANK (k_emit)
  uint32_t* d_cnt_words = nullptr;          // gid|hit words grouped by rule block
  unsigned long long cnt_words_alloc = 0;
  unsigned long long* d_cnt_starts = nullptr;
  unsigned long long cnt_starts_alloc = 0;
  CntTask* d_cnt_tasks = nullptr;
  unsigned long long cnt_tasks_alloc = 0;
  uint32_t* d_cnt_ctl = nullptr;
  unsigned long long cnt_ctl_alloc = 0;
  bool auto_tighten = true;
  bool tightened = false;
  uint32_t profile_skip = 0;
  bool precheck = true;
  bool stats_on = false;
  unsigned long long* d_stats = nullptr;   // 4 counters (RSA_OPT_STATS)
  uint32_t filter_slice = 256;
  // auto filter: bound refinements (each after filter_growth x the previous
  // lines): 1M / 4M / 16M.  1M then 16M lines measured cfg3 7.91 -> 7.80 and
  // cfg5 9.55 -> 9.30 but cfg2 5.65 -> 6.84 ms/step (profiles/r05j_*, r05k_*);
  // the bound of the long last slice must come from ~16M lines (from 9M:
  // 14.8 ms/step at cfg3; from 36M: 9.5)
  uint32_t filter_steps = 3;
  uint32_t filter_growth = 4;         // RSA_OPT_FILTER_GROWTH
  uint32_t* d_tail = nullptr;         // deferred line indices
  unsigned long long* d_tail_n = nullptr;
  unsigned long long tail_alloc = 0;
  int32_t* d_gscratch = nullptr;      // gids of a recount whose caller keeps none
  uint32_t* d_gh = nullptr;           // pass-1 gid | hit << 31 per line (k_count input)
  unsigned long long gh_alloc = 0;
  // on-chip shuffle of pass 1b: records, their region-sorted copy, histograms
  void* d_recs = nullptr;
  void* d_recs2 = nullptr;
  void* d_junk = nullptr;               // 64 records: the sink of k_part_scatter's invalid lanes
  unsigned long long* d_route_cur = nullptr;   // rsa_export_routed: per-owner cursors
  unsigned long long recs_alloc = 0;
  unsigned long long recs2_alloc = 0;
  uint16_t* d_regs = nullptr;          // region of each record (the histogram pass reads only these)
  unsigned long long regs_alloc = 0;
  uint32_t* d_wcnt = nullptr;          // records per 64-line window
  unsigned long long wcnt_alloc = 0;
  unsigned long long* d_nrecs = nullptr;
  uint32_t* d_hist = nullptr;
  unsigned long long hist_alloc = 0;
  uint32_t* d_scan_sums = nullptr;
  unsigned long long scan_sums_alloc = 0;
  uint32_t* d_occ = nullptr;          // slot occupancy bitmap
  unsigned long long occ_alloc = 0;   // words
  uint32_t rs_bits = 10, np_bits = 0;
  // pass-1 records kept for the recount: one batch per job, one segment per launch
  unsigned long long* d_starts = nullptr;   // kMaxSegs x (regions + 1)
  unsigned long long seg_base = 0;
  uint32_t n_segs = 0;
  bool rec_cache = false;
  const void* cache_T = nullptr;
  unsigned long long cache_n = 0;
  uint32_t pass1_calls = 0;
  unsigned long long gscratch_alloc = 0;
  unsigned int* d_flags = nullptr;       // 4 words
  unsigned long long* d_cursor = nullptr;
  // cap-resolution scratch
  uint32_t* d_cidx = nullptr;
  uint32_t* d_capped_gid = nullptr;
  uint32_t* d_capped_cnt = nullptr;
  uint32_t* d_capped_start = nullptr;
  unsigned long long* d_capped_prev = nullptr;   // per capped rule: the earlier selection bounding it
  uint32_t cidx_len = 0;
  unsigned long long* d_keys = nullptr;   // capped rules' min_order keys, one segment per rule
  unsigned long long sort_alloc = 0;
  // pass-1 kernel timing (HIP events on the ctx stream)
  hipEvent_t ev[48] = {};             // per pass-1 launch: start, classified, aggregated
  bool gh16 = true;                   // RSA_OPT_COUNTER_WORDS16: 16-bit gid|hit words when the rules fit
  int ev_used = 0;
  bool debug = false;                 // RSA_DEBUG=1 in the environment: per-launch counts on stderr
};

namespace {

int fail(rsa_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return code;
}

#define HIPCHK(ctx, expr)                                                                          \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess) return fail((ctx), RSA_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

Rules rules_of(const rsa_ctx* c) {
  Rules r;
  r.e = (const const_v4u*)(c->d_entries);
  r.eg = reinterpret_cast<const v4u*>(c->d_entries);
  r.off = (const const_u32*)(c->d_off);
  r.n_lists = c->n_lists;
  r.n_rules = c->n_rules;
  r.list_off = c->list_off;
  r.resid = (const const_v4u*)(c->d_resid);
  r.img = c->d_img;
  r.img_words = c->img_words;
  r.indexed = c->indexed ? 1 : 0;
  r.force_defer = c->force_defer ? 1 : 0;
  r.group_tasks = c->group_tasks ? 1 : 0;
  r.prof = (int)c->prof_classify;
  r.bkt = c->bkt_index ? 1 : 0;
  r.bkt_filters = c->bkt_filters ? 1 : 0;
  r.residg = reinterpret_cast<const v4u*>(c->d_resid);
  return r;
}

Agg agg_of(const rsa_ctx* c) {
  Agg a;
  a.matches = c->d_matches;
  a.hits = c->d_hits;
  a.distinct = c->d_distinct;
  a.thresh = c->d_thresh;
  a.filter = c->d_filter;
  a.packed = c->d_packed;
  a.slots = c->d_slots;
  a.mask = c->slot_cap ? c->slot_cap - 1 : 0;
  a.used = c->d_used;
  a.ukey = c->d_ukey;
  a.used_n = c->d_used_n;
  a.flags = c->d_flags;
  a.cap = c->cap;
  a.skip = c->profile_skip;
  a.precheck = c->precheck ? 1u : 0u;
  a.stats = c->stats_on ? c->d_stats : nullptr;
  a.occ = c->d_occ;
  a.rs_bits = c->rs_bits;
  a.np_bits = c->np_bits;
  a.tent2 = c->tent2_on ? 1u : 0u;
  return a;
}

unsigned grid_for_threads(const rsa_ctx* c, unsigned long long n, unsigned threads, unsigned per_cu) {
  unsigned long long g = (n + threads - 1) / threads;
  const unsigned long long lim = (unsigned long long)c->cu_count * per_cu;
  if (g > lim) g = lim;
  if (g == 0) g = 1;
  return (unsigned)g;
}

unsigned grid_for(const rsa_ctx* c, unsigned long long n, unsigned per_cu) {
  unsigned long long g = (n + kBlock - 1) / kBlock;
  const unsigned long long lim = (unsigned long long)c->cu_count * per_cu;
  if (g > lim) g = lim;
  if (g == 0) g = 1;
  return (unsigned)g;
}

// The sticky error flags (d_flags[0..1]) of a host copy f of d_flags[0..3].
int flags_status(rsa_ctx* c, const unsigned int* f) {
  if (f[0]) return fail(c, RSA_ERR_CAPACITY, "distinct-connection table overflow (capacity %llu)", c->slot_cap);
  if (f[1] & 1u) return fail(c, RSA_ERR_ARG, "tuple references a candidate list id >= n_lists (%u)", c->n_lists);
  if (f[1] & 2u) return fail(c, RSA_ERR_ARG, "rule id >= n_rules (%u)", c->n_rules);
  if (f[1] & 4u) return fail(c, RSA_ERR_STATE, "pass 2 found an occurrence with no pass-1 entry");
  if (f[1] & 8u) return fail(c, RSA_ERR_STATE, "pass-2 import of a key absent from the table");
  if (f[1] & 16u) return fail(c, RSA_ERR_STATE, "cap selection: more entries than the table reported");
  return RSA_OK;
}

int need_agg(rsa_ctx* c) {
  if (!c->d_matches || !c->d_hits || !c->d_distinct || !c->d_thresh)
    return fail(c, RSA_ERR_STATE, "counters not bound (rsa_bind_counters)");
  if (!c->table_ready) return fail(c, RSA_ERR_STATE, "table not initialised (rsa_reset)");
  return RSA_OK;
}

int used_count(rsa_ctx* c, unsigned long long* n) {
  HIPCHK(c, hipMemcpyAsync(n, c->d_used_n, sizeof *n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (*n > c->slot_cap) *n = c->slot_cap;
  c->used_last = *n;
  return RSA_OK;
}

template <typename T>
int upload(rsa_ctx* c, T** dst, const T* src, size_t n) {
  hipFree(*dst);
  *dst = nullptr;
  HIPCHK(c, hipMalloc(dst, (n ? n : 1) * sizeof(T)));
  if (n) HIPCHK(c, hipMemcpy(*dst, src, n * sizeof(T), hipMemcpyHostToDevice));
  return RSA_OK;
}

// Exact selection of P for every rule with >= cap distinct entries in the
// current table, written to out[] (RSA_NO_THRESHOLD for the others).  On the
// final table this is the reducer's cap threshold; on a partial table it is an
// upper bound of it (the filter): first-seen orders only decrease and the set
// of connections only grows as more lines are aggregated.
int cap_select(rsa_ctx* c, unsigned long long* out, uint32_t* h_n_capped) {
  // h_n_capped == nullptr: no host round trip (the filter steps of pass 1);
  // the counts the kernels need (capped rules, used slots) are read on the
  // device, the key buffer holds every slot, and the sticky error flags are
  // checked by the final selection and the emission
  if (h_n_capped) *h_n_capped = 0;
  const uint32_t nr = c->n_rules;
  if (nr == 0) return RSA_OK;
  if (c->cidx_len < nr) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    hipFree(c->d_cidx);
    hipFree(c->d_capped_gid);
    hipFree(c->d_capped_cnt);
    hipFree(c->d_capped_start);
    hipFree(c->d_capped_prev);
    c->d_cidx = c->d_capped_gid = c->d_capped_cnt = c->d_capped_start = nullptr;
    c->d_capped_prev = nullptr;
    c->cidx_len = 0;
    HIPCHK(c, hipMalloc(&c->d_cidx, (size_t)nr * sizeof(uint32_t)));
    HIPCHK(c, hipMalloc(&c->d_capped_gid, (size_t)nr * sizeof(uint32_t)));
    HIPCHK(c, hipMalloc(&c->d_capped_cnt, (size_t)nr * sizeof(uint32_t)));
    HIPCHK(c, hipMalloc(&c->d_capped_start, (size_t)nr * sizeof(uint32_t)));
    HIPCHK(c, hipMalloc(&c->d_capped_prev, (size_t)nr * sizeof(unsigned long long)));
    c->cidx_len = nr;
  }
  if (c->sort_alloc < c->slot_cap) {   // a key per slot at most: sized once per table size
    HIPCHK(c, hipStreamSynchronize(c->stream));
    hipFree(c->d_keys);
    c->d_keys = nullptr;
    c->sort_alloc = 0;
    HIPCHK(c, hipMalloc(&c->d_keys, c->slot_cap * sizeof(unsigned long long)));
    c->sort_alloc = c->slot_cap;
  }
  unsigned int* d_ncap = c->d_flags + 2;
  if (!c->cap_ctl_zeroed) {   // (a pass-1 launch zeroes them in k_seg_starts)
    HIPCHK(c, hipMemsetAsync(d_ncap, 0, sizeof(unsigned int), c->stream));
    HIPCHK(c, hipMemsetAsync(c->d_cursor, 0, sizeof(unsigned long long), c->stream));
  }
  c->cap_ctl_zeroed = false;
  c->ncap_on_device = false;
  // the keys: read from the used-list-ordered copy k_reduce<1> keeps
  // (16 B per used entry, coalesced) unless an entry was claimed by the CAS
  // import; only keys at or below the rule's earlier selection (the job's last
  // filter slice) are scattered and selected over
  const unsigned long long* ukey = c->ukey_ok ? c->d_ukey : nullptr;
  const unsigned long long* prev = c->d_filter;
  k_cap_mark<<<(nr + kBlock - 1) / kBlock, kBlock, 0, c->stream>>>(c->d_distinct, nr, c->cap, prev, c->d_cidx,
                                                                   c->d_capped_gid, c->d_capped_start,
                                                                   c->d_capped_cnt, c->d_capped_prev, d_ncap,
                                                                   c->d_cursor, out);
  HIPCHK(c, hipGetLastError());
  // the scatter picks its variant from the device-side count of capped rules
  // (LDS counters for <= kCapLds rules)
  const uint32_t lds_max = c->wave_cap_scatter ? 0u : (uint32_t)kCapLds;
  k_cap_scatter_lds<<<c->cu_count * 2, 1024, 0, c->stream>>>(c->d_slots, c->d_used, c->d_used_n, d_ncap, lds_max,
                                                             c->d_cidx, c->d_capped_start, c->d_capped_cnt, ukey,
                                                             c->d_capped_prev, c->d_keys, c->sort_alloc, c->d_flags);
  HIPCHK(c, hipGetLastError());
  const unsigned sel_grid = nr < (uint32_t)c->cu_count * 8 ? nr : (unsigned)c->cu_count * 8;
  k_cap_select<<<sel_grid, kSelThreads, 0, c->stream>>>(c->d_keys, c->d_capped_start, c->d_capped_cnt, c->d_capped_gid,
                                                        c->cap, d_ncap, out);
  HIPCHK(c, hipGetLastError());
  if (c->debug) {
    // the selection's volume: capped rules, their entries, the keys scattered
    unsigned int f[4];
    unsigned long long tot = 0, used_n = 0;
    HIPCHK(c, hipMemcpyAsync(f, c->d_flags, sizeof f, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(&tot, c->d_cursor, sizeof tot, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(&used_n, c->d_used_n, sizeof used_n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::vector<uint32_t> fill(f[2]);
    if (f[2]) {
      HIPCHK(c, hipMemcpy(fill.data(), c->d_capped_cnt, f[2] * sizeof(uint32_t), hipMemcpyDeviceToHost));
    }
    unsigned long long sc = 0;
    for (uint32_t v : fill) sc += v;
    fprintf(stderr, "[rsa] cap select: %u capped rules, %llu of %llu used entries theirs, %llu keys scattered\n", f[2],
            tot, used_n, sc);
  }
  if (h_n_capped) {
    // one round trip: the capped-rule count (d_flags[2]) with the sticky
    // error flags, which also cover every launch before this selection
    unsigned int f[4];
    HIPCHK(c, hipMemcpyAsync(f, c->d_flags, sizeof f, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    *h_n_capped = f[2];
    if (c->debug) fprintf(stderr, "[rsa] cap select: %u capped rules\n", f[2]);
    return flags_status(c, f);
  }
  return RSA_OK;
}

// Deferred-line region of `tail_alloc` entries and its counter.
int ensure_tail(rsa_ctx* c, unsigned long long n) {
  if (!c->d_tail_n) HIPCHK(c, hipMalloc(&c->d_tail_n, sizeof(unsigned long long)));
  if (n <= c->tail_alloc) return RSA_OK;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  hipFree(c->d_tail);
  c->d_tail = nullptr;
  c->tail_alloc = 0;
  HIPCHK(c, hipMalloc(&c->d_tail, n * sizeof(uint32_t)));
  c->tail_alloc = n;
  return RSA_OK;
}

template <typename T>
int ensure_buf(rsa_ctx* c, T** p, unsigned long long* have, unsigned long long n) {
  if (n <= *have) return RSA_OK;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  hipFree(*p);
  *p = nullptr;
  *have = 0;
  HIPCHK(c, hipMalloc(p, n * sizeof(T)));
  *have = n;
  return RSA_OK;
}

constexpr int kMaxEvents = 48;

int ensure_events(rsa_ctx* c) {
  for (int k = 0; k < kMaxEvents; ++k)
    if (!c->ev[k]) HIPCHK(c, hipEventCreate(&c->ev[k]));
  return RSA_OK;
}

// LDS image capacities (32-bit words) of k_classify.
constexpr int kImgSmall = kImgSmallMax;   // 76 KiB: two 1024-thread workgroups per CU (32 waves)
constexpr int kImgLarge = 38912;   // 152 KiB: one workgroup per CU

template <bool kEmit, int kMode, bool kNarrow>
void launch_classify_img(rsa_ctx* c, const uint4* t, uint64_t m, int32_t* go, const Rules& r, const Agg& ag,
                         const Emit& e) {
  EmitPack ep = {};
  ep.gh = reinterpret_cast<unsigned long long>(e.gh);
  ep.gh16 = reinterpret_cast<unsigned long long>(e.gh16);
  ep.ts = reinterpret_cast<unsigned long long>(e.ts);
  ep.ord = reinterpret_cast<unsigned long long>(e.ord);
  ep.recs = reinterpret_cast<unsigned long long>(e.recs);
  ep.regs = reinterpret_cast<unsigned long long>(e.regs);
  ep.wcnt = reinterpret_cast<unsigned long long>(e.wcnt);
  ep.filter = reinterpret_cast<unsigned long long>(ag.filter);
  ep.cap = ag.cap;
  ep.skip = ag.skip;
  ep.np_bits = ag.np_bits;
  if (kMode == 2 && c->classify_pair && c->indexed && !c->bkt_filters &&
      !(c->img_words <= (uint32_t)kImgLarge)) {
    // the global bucket image: two lines per lane
    const unsigned long long lanes = (m + 1) / 2;
    k_classify_pair<kEmit><<<grid_for_threads(c, lanes, kPairThreads, 4 * RSA_PAIR_WAVES / (kPairThreads / 64)),
                             kPairThreads, 0, c->stream>>>(ep, t, m, go, r, c->d_flags, c->d_tail, c->d_tail_n);
  } else if (c->indexed && c->img_words <= (uint32_t)kImgSmall) {
    k_classify<kImgSmall, kEmit, kMode, kNarrow><<<grid_for_threads(c, m, 1024, 2), 1024, 0, c->stream>>>(
        ep, t, m, go, r, c->d_flags, c->d_tail, c->d_tail_n);
  } else if (c->indexed && c->img_words <= (uint32_t)kImgLarge) {
    k_classify<kImgLarge, kEmit, kMode, kNarrow><<<grid_for_threads(c, m, 1024, 1), 1024, 0, c->stream>>>(
        ep, t, m, go, r, c->d_flags, c->d_tail, c->d_tail_n);
  } else {
    k_classify<0, kEmit, kMode, kNarrow><<<grid_for_threads(c, m, 1024, 2), 1024, 0, c->stream>>>(
        ep, t, m, go, r, c->d_flags, c->d_tail, c->d_tail_n);
  }
}

// Classification (+ exact tail) of lines [0, m) of T (already offset) into go
// (nullable); with `e` also the pass-1 emission (counter words, records).
template <bool kEmit>
int launch_classify_t(rsa_ctx* c, const uint4* t, uint64_t m, int32_t* go, const Emit& e) {
  const Rules r = rules_of(c);
  const Agg ag = agg_of(c);
  // the pruning tables' slot width is a kernel variant: every table narrow
  // (the common case) or each table deciding its own
  if (c->bkt_index) {
    launch_classify_img<kEmit, 2, false>(c, t, m, go, r, ag, e);
  } else if (c->group_tasks && c->prune_narrow) {
    launch_classify_img<kEmit, 1, true>(c, t, m, go, r, ag, e);
  } else if (c->group_tasks) {
    launch_classify_img<kEmit, 1, false>(c, t, m, go, r, ag, e);
  } else if (c->prune_narrow) {
    launch_classify_img<kEmit, 0, true>(c, t, m, go, r, ag, e);
  } else {
    launch_classify_img<kEmit, 0, false>(c, t, m, go, r, ag, e);
  }
  HIPCHK(c, hipGetLastError());
  // deferred lines (their number is read on the device: no host sync)
  k_tail<kEmit><<<c->cu_count * 4, kBlock, 0, c->stream>>>(t, go, r, c->d_flags, c->d_tail, c->d_tail_n, ag, e);
  HIPCHK(c, hipGetLastError());
  return RSA_OK;
}

int launch_classify(rsa_ctx* c, const uint4* t, uint64_t m, int32_t* go, const Emit* e) {
  int rc = ensure_tail(c, m);
  if (rc) return rc;
  HIPCHK(c, hipMemsetAsync(c->d_tail_n, 0, sizeof(unsigned long long), c->stream));
  if (e) return launch_classify_t<true>(c, t, m, go, *e);
  Emit none = {};
  return launch_classify_t<false>(c, t, m, go, none);
}

// LDS-privatised counter capacity (rules): 2 x 4 B per rule (lines, hits),
// 104 KiB, so one 1024-thread workgroup is resident per CU; the grid is sized
// for two per CU (launch_aggregate), i.e. two rounds of workgroups.
constexpr int kCnt = 13312;

// Exclusive scan of n uint32 in place (device); returns the device address of
// the grand total.
int exclusive_scan(rsa_ctx* c, uint32_t* d, unsigned long long n, uint32_t** total) {
  const unsigned long long nb = n ? (n + kScanBlock - 1) / kScanBlock : 1;
  int rc = ensure_buf(c, &c->d_scan_sums, &c->scan_sums_alloc, nb + 1);
  if (rc) return rc;
  *total = c->d_scan_sums + nb;
  if (n == 0) {
    HIPCHK(c, hipMemsetAsync(*total, 0, sizeof(uint32_t), c->stream));
    return RSA_OK;
  }
  k_scan_blocks<<<(unsigned)nb, 1024, 0, c->stream>>>(d, n, c->d_scan_sums);
  k_scan_sums<<<1, 1024, 0, c->stream>>>(c->d_scan_sums, (uint32_t)nb);
  k_scan_add<<<(unsigned)nb, 1024, 0, c->stream>>>(d, n, c->d_scan_sums);
  HIPCHK(c, hipGetLastError());
  return RSA_OK;
}

int ensure_hot_ctl(rsa_ctx* c) {
  if (!c->d_hot_base) {
    HIPCHK(c, hipMalloc(&c->d_hot_base, kMaxRegions * sizeof(unsigned long long)));
    HIPCHK(c, hipMalloc(&c->d_hot_fill, kMaxRegions * sizeof(uint32_t)));
    HIPCHK(c, hipMalloc(&c->d_hot_ctl, 4 * sizeof(uint32_t)));
    HIPCHK(c, hipMalloc(&c->d_hot_total, sizeof(unsigned long long)));
  }
  return RSA_OK;
}

// The hot-region split for the records of segments [seg0, seg0 + n_segs) of
// d_starts (at most `records` records): plan, combine; returns the hot
// descriptors for k_reduce in *base / *fill / *hot (nullptr: split off).
template <int kPass>
int hot_split(rsa_ctx* c, uint32_t seg0, uint32_t n_segs, unsigned long long records,
              const unsigned long long** base, const uint32_t** fill, const HRec** hot,
              const unsigned int* skip_zero = nullptr) {
  *base = nullptr;
  *fill = nullptr;
  *hot = nullptr;
  const bool zeroed = c->hot_ctl_zeroed;
  c->hot_ctl_zeroed = false;
  if (!c->hot_split || records == 0) return RSA_OK;
  const uint32_t n_regions = 1u << c->np_bits;
  int rc0 = ensure_hot_ctl(c);
  if (rc0) return rc0;
  const size_t max_tasks = records / kHotSlice + (size_t)n_segs * n_regions + 1;
  if (max_tasks > c->tasks_alloc || records > c->hot_alloc) HIPCHK(c, hipStreamSynchronize(c->stream));
  if (max_tasks > c->tasks_alloc) {
    hipFree(c->d_hot_tasks);
    c->d_hot_tasks = nullptr;
    c->tasks_alloc = 0;
    HIPCHK(c, hipMalloc(&c->d_hot_tasks, max_tasks * sizeof(HotTask)));
    c->tasks_alloc = max_tasks;
  }
  if (records > c->hot_alloc) {
    hipFree(c->d_hot);
    c->d_hot = nullptr;
    c->hot_alloc = 0;
    HIPCHK(c, hipMalloc(&c->d_hot, records * sizeof(HRec)));
    c->hot_alloc = records;
  }
  if (!zeroed) {   // (pass 1 zeroes them in k_seg_starts)
    HIPCHK(c, hipMemsetAsync(c->d_hot_ctl, 0, 4 * sizeof(uint32_t), c->stream));
    HIPCHK(c, hipMemsetAsync(c->d_hot_total, 0, sizeof(unsigned long long), c->stream));
  }
  HotTask* tasks = static_cast<HotTask*>(c->d_hot_tasks);
  k_hot_plan<<<(n_regions + 255) / 256, 256, 0, c->stream>>>(c->d_starts + (size_t)seg0 * (n_regions + 1), n_segs,
                                                             n_regions, tasks, (uint32_t)max_tasks, c->d_hot_ctl,
                                                             c->d_hot_total, c->d_hot_base, c->d_hot_fill, c->hot_min,
                                                             c->hot_factor, skip_zero);
  k_hot_combine<kPass><<<c->cu_count, 1024, 0, c->stream>>>(reinterpret_cast<const Rec*>(c->d_recs2), tasks,
                                                             c->d_hot_ctl, agg_of(c), c->d_hot_base, c->d_hot_fill,
                                                             static_cast<HRec*>(c->d_hot));
  HIPCHK(c, hipGetLastError());
  *base = c->d_hot_base;
  *fill = c->d_hot_fill;
  *hot = static_cast<const HRec*>(c->d_hot);
  return RSA_OK;
}

// Window-compacted record buffers of a pass-1 launch over m lines.
int prepare_records(rsa_ctx* c, uint64_t m) {
  const uint64_t mw = (m + kWin - 1) / kWin * kWin;
  int rc = ensure_buf(c, reinterpret_cast<Rec**>(&c->d_recs), &c->recs_alloc, mw);
  if (!rc) rc = ensure_buf(c, &c->d_regs, &c->regs_alloc, mw);
  if (!rc) rc = ensure_buf(c, &c->d_wcnt, &c->wcnt_alloc, mw / kWin + kPartW);   // (padded: win_group4)
  return rc;
}

// Tile length (lines) of the tiled counting sorts (the region sort of the
// records, the rule-block sort of the counter words) over m lines: the tiles
// are dealt to the CUs evenly -- RSA_PART_TPC workgroups per CU, in multiples
// of kPartTileMin lines, at most kPartTileMax (power-of-two tiles for >= 384
// workgroups left a third of the CUs with one scatter workgroup more than the
// rest: -0.2 to -0.3 ms/step, profiles/r06/ab_part_tiles_per_cu.txt)
uint32_t part_tile_len(const rsa_ctx* c, uint64_t m) {
#if RSA_PART_TILES_CU
  const unsigned long long want = (unsigned long long)c->cu_count * RSA_PART_TPC;
  const unsigned long long tl = ((m + want - 1) / want + kPartTileMin - 1) / kPartTileMin * kPartTileMin;
  return (uint32_t)(tl < kPartTileMin ? kPartTileMin : tl > kPartTileMax ? kPartTileMax : tl);
#else
  uint32_t tile_len = kPartTileMin;
  while (tile_len < kPartTileMax && (unsigned long long)tile_len * 2 * kPartTilesWant <= m) tile_len <<= 1;
  return tile_len;
#endif
}

// Per-rule counters of m gid|hit words by rule block (rule sets > kCnt, at
// most kMaxRegions blocks): see k_cnt_hist.
int count_by_block(rsa_ctx* c, const uint32_t* gh, uint64_t m) {
  const uint32_t n_blocks = (c->n_rules + kCntBlock - 1) >> kCntBits;
  const uint32_t tile_len = part_tile_len(c, m);
  const uint32_t n_tiles = (uint32_t)((m + tile_len - 1) / tile_len);
  const unsigned long long hl = (unsigned long long)n_blocks * n_tiles;
  const unsigned long long max_tasks = m / kCntChunk + n_blocks + 1;
  int rc = ensure_buf(c, &c->d_hist, &c->hist_alloc, hl);
  if (!rc) rc = ensure_buf(c, &c->d_cnt_words, &c->cnt_words_alloc, m);
  if (!rc) rc = ensure_buf(c, &c->d_cnt_starts, &c->cnt_starts_alloc, n_blocks + 1);
  if (!rc) rc = ensure_buf(c, &c->d_cnt_tasks, &c->cnt_tasks_alloc, max_tasks);
  if (!rc) rc = ensure_buf(c, &c->d_cnt_ctl, &c->cnt_ctl_alloc, 4);
  if (rc) return rc;
  k_cnt_hist<<<n_tiles, 1024, 0, c->stream>>>(gh, m, n_blocks, n_tiles, tile_len, c->d_hist);
  HIPCHK(c, hipGetLastError());
  uint32_t* total = nullptr;
  rc = exclusive_scan(c, c->d_hist, hl, &total);
  if (rc) return rc;
  k_cnt_scatter<<<n_tiles, 1024, 0, c->stream>>>(gh, m, n_blocks, n_tiles, tile_len, c->d_hist, c->d_cnt_words);
  k_seg_starts<<<(n_blocks + 1 + 255) / 256, 256, 0, c->stream>>>(c->d_hist, n_tiles, n_blocks, 0, total,
                                                                  c->d_cnt_starts, nullptr, nullptr, nullptr, nullptr,
                                                                  nullptr);
  k_cnt_plan<<<1, 1024, 0, c->stream>>>(c->d_cnt_starts, n_blocks, kCntChunk, c->d_cnt_tasks, (uint32_t)max_tasks,
                                        c->d_cnt_ctl);
  k_cnt_reduce<<<(unsigned)max_tasks, 1024, 0, c->stream>>>(c->d_cnt_words, c->d_cnt_tasks, c->d_cnt_ctl, c->n_rules,
                                                            c->d_matches, c->d_hits);
  HIPCHK(c, hipGetLastError());
  return RSA_OK;
}

// Pass 1b over lines [a, a + m) of the batch: the per-rule counters (k_count
// over the gid|hit words `gh` of a classifying pass 1a, or k_aggregate over
// given gids, which also writes the line-indexed records), then the counting
// sort of the records by table region into d_recs2[a ..] (records <= lines,
// so no record count is needed on the host) and the per-region LDS reduction
// and merge (k_reduce).
// With gh, the counters cover the words [gh_count, gh_count + m_count) (the
// auto-tightening slices count once, all of the batch's lines with the last).
int launch_aggregate(rsa_ctx* c, const uint4* t, const uint32_t* ts, const unsigned long long* o, const int32_t* g,
                     const uint32_t* gh, uint64_t a, uint64_t m, const uint32_t* gh_count, uint64_t m_count,
                     const uint16_t* gh16_count = nullptr) {
  const Agg ag = agg_of(c);
  int rc = RSA_OK;
  if (gh || gh16_count) {
    if (!(ag.skip & 1u) && m_count) {
      const uint64_t units = (m_count + 3) / 4;
      if (gh16_count) {
        // 16-bit words (rules <= kCnt)
        if (reinterpret_cast<uintptr_t>(gh16_count) & 15u) return fail(c, RSA_ERR_STATE, "misaligned counter words");
        k_count16<kCnt><<<grid_for_threads(c, (m_count + 7) / 8 + 1, 1024, RSA_COUNT_PER_CU), 1024, 0, c->stream>>>(
            gh16_count, m_count, c->n_rules, ag);
      } else if (c->n_rules <= (uint32_t)kCnt) {
        k_count<kCnt><<<grid_for_threads(c, units, 1024, RSA_COUNT_PER_CU), 1024, 0, c->stream>>>(gh_count, m_count,
                                                                                                  c->n_rules, ag);
      } else if (c->count_sort && ((c->n_rules + kCntBlock - 1) >> kCntBits) <= (uint32_t)kMaxRegions) {
        const int rc2 = count_by_block(c, gh_count, m_count);
        if (rc2) return rc2;
      } else {
        k_count<0><<<grid_for_threads(c, units, 1024, 8), 1024, 0, c->stream>>>(gh_count, m_count, c->n_rules, ag);
        k_count_flush<<<grid_for(c, c->n_rules, 8), kBlock, 0, c->stream>>>(c->d_packed, c->n_rules, c->d_matches,
                                                                            c->d_hits);
      }
    }
  } else {
    rc = prepare_records(c, m);
    if (rc) return rc;
    const uint64_t units = (m + kAggU - 1) / kAggU;
    Rec* recs = reinterpret_cast<Rec*>(c->d_recs);
    if (c->n_rules <= (uint32_t)kCnt) {
      k_aggregate<kCnt><<<grid_for_threads(c, units, 1024, 2), 1024, 0, c->stream>>>(t, ts, o, g, m, c->n_rules, ag,
                                                                                     recs, c->d_regs, c->d_wcnt);
    } else {
      k_aggregate<0><<<grid_for_threads(c, units, 1024, 2), 1024, 0, c->stream>>>(t, ts, o, g, m, c->n_rules, ag,
                                                                                  recs, c->d_regs, c->d_wcnt);
      if (!(ag.skip & 1u))
        k_count_flush<<<grid_for(c, c->n_rules, 8), kBlock, 0, c->stream>>>(c->d_packed, c->n_rules, c->d_matches,
                                                                            c->d_hits);
    }
  }
  HIPCHK(c, hipGetLastError());
  if (ag.cap == 0 || (ag.skip & 2u)) return RSA_OK;   // no table this job
  const Rec* recs = reinterpret_cast<const Rec*>(c->d_recs);
  // region-sorted records: at the launch's line offset while this job's
  // records are kept for the recount (rsa_recount), else from 0
  if (c->rec_cache && (c->n_segs >= (uint32_t)kMaxSegs || a + m > c->recs2_alloc)) c->rec_cache = false;
  const unsigned long long seg_base = c->rec_cache ? a : 0;
  if (!c->rec_cache) {
    c->n_segs = 0;
    rc = ensure_buf(c, reinterpret_cast<Rec**>(&c->d_recs2), &c->recs2_alloc, m);
    if (rc) return rc;
  }
  Rec* sorted = reinterpret_cast<Rec*>(c->d_recs2) + seg_base;
  const uint32_t n_regions = 1u << c->np_bits;
  const uint32_t tile_len = part_tile_len(c, m);
  const uint32_t n_tiles = (uint32_t)((m + tile_len - 1) / tile_len);
  const unsigned long long hl = (unsigned long long)n_regions * n_tiles;
  rc = ensure_buf(c, &c->d_hist, &c->hist_alloc, hl);
  if (rc) return rc;
  k_part_hist<<<n_tiles, 1024, 0, c->stream>>>(c->d_regs, c->d_wcnt, m, n_regions, n_tiles, tile_len, c->d_hist);
  HIPCHK(c, hipGetLastError());
  uint32_t* total = nullptr;
  rc = exclusive_scan(c, c->d_hist, hl, &total);
  if (rc) return rc;
  k_part_scatter<<<n_tiles, 1024, 0, c->stream>>>(recs, c->d_regs, c->d_wcnt, m, n_regions, n_tiles, tile_len, c->d_hist,
                                                  sorted, static_cast<Rec*>(c->d_junk));
  HIPCHK(c, hipGetLastError());
  unsigned long long* st = c->d_starts + (size_t)c->n_segs * (n_regions + 1);
  rc = ensure_hot_ctl(c);
  if (rc) return rc;
  k_seg_starts<<<(n_regions + 1 + 255) / 256, 256, 0, c->stream>>>(c->d_hist, n_tiles, n_regions, seg_base, total, st,
                                                                   c->d_hot_ctl, c->d_hot_total, c->d_flags + 2,
                                                                   c->d_cursor, c->d_job_recs);
  if (c->d_job_recs) c->job_recs_valid = true;
  c->hot_ctl_zeroed = true;
  c->cap_ctl_zeroed = true;
  const unsigned long long* hb = nullptr;
  const uint32_t* hf = nullptr;
  const HRec* hr = nullptr;
  rc = hot_split<1>(c, c->n_segs, 1, m, &hb, &hf, &hr);
  if (rc) return rc;
  // record-heavy jobs (the region policy chose more than 1024 regions) merge
  // through a 4096-entry LDS table (regions of at most 2^15 slots, so both
  // bitmaps fit: 156 KiB): cfg5 9.84 -> 9.61 ms/step, while cfg3's 1024
  // regions keep 3072 entries (4096 there: 8.03 -> 8.17; profiles/r04ao_*)
  if (c->np_bits > 10 && c->rs_bits <= 15 && c->reduce_big) {
    k_reduce<1, 4096, 15><<<n_regions, 1024, 0, c->stream>>>(reinterpret_cast<const Rec*>(c->d_recs2), st, 1, ag, hb,
                                                             hf, hr, nullptr);
  } else {
    k_reduce<1><<<n_regions, 1024, 0, c->stream>>>(reinterpret_cast<const Rec*>(c->d_recs2), st, 1, ag, hb, hf, hr,
                                                   nullptr);
  }
  HIPCHK(c, hipGetLastError());
  if (c->rec_cache) ++c->n_segs;
  if (c->debug) {
    uint32_t nr = 0;
    HIPCHK(c, hipMemcpyAsync(&nr, total, sizeof nr, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    fprintf(stderr, "[rsa] pass-1 launch: %llu lines -> %u records\n", (unsigned long long)m, nr);
  }
  return RSA_OK;
}

// Pass 1 over one batch: classification into gids (gout, or the ctx scratch),
// then aggregation of the classified lines; with given gids (reducer drop-in)
// aggregation only.  With auto-tightening, a large first batch is split: the
// first 1/filter_slice builds the table, the filter is computed, and the rest
// of the batch skips the table for lines that cannot change any output; with
// filter_steps > 1 the filter is refined again after 4x, 16x, ... that many
// lines.
int run_pass1(rsa_ctx* c, int classify, const rsa_tuple* T, const uint32_t* TS, const uint64_t* ORD, const int32_t* G,
              int32_t* gout, uint64_t n) {
  int rc = ensure_events(c);
  if (rc) return rc;
  c->ev_used = 0;
  if (n > 0x7FFFFFFFull) return fail(c, RSA_ERR_ARG, "batch larger than 2^31 tuples: split it");
  // the records of a job's only batch are kept for its recount
  if (c->pass1_calls++ == 0) {
    rc = ensure_buf(c, reinterpret_cast<Rec**>(&c->d_recs2), &c->recs2_alloc, n);
    if (rc) return rc;
    c->rec_cache = true;
    c->cache_T = T;
    c->cache_n = n;
    c->n_segs = 0;
  } else {
    c->rec_cache = false;
  }
  uint32_t* gh = nullptr;
  // 16-bit counter words when every gid fits 15 bits and the LDS histogram
  // takes the rules (half the bytes written by k_classify and read by the count)
  const bool narrow = classify && c->gh16 && c->n_rules <= (uint32_t)kCnt && c->n_rules < 0x7FFFu;
  if (classify) {
    rc = ensure_buf(c, &c->d_gh, &c->gh_alloc, n);
    if (rc) return rc;
    gh = c->d_gh;
  }
  // count_from: the first line whose gid|hit word the launch counts (the
  // tightening slices leave theirs to the last one: the per-rule counters do
  // not feed the filter bounds, and each counting launch ends in a flush of
  // every rule's counter from every workgroup)
  auto launch = [&](uint64_t a, uint64_t m, uint64_t count_from) -> int {
    if (m == 0) return RSA_OK;
    if (c->ev_used + 3 > kMaxEvents) return fail(c, RSA_ERR_STATE, "too many pass-1 launches in one call");
    const uint4* t = reinterpret_cast<const uint4*>(T) + a;
    const unsigned long long* o = reinterpret_cast<const unsigned long long*>(ORD) + a;
    HIPCHK(c, hipEventRecord(c->ev[c->ev_used], c->stream));
    if (classify) {
      int rc2 = prepare_records(c, m);
      if (rc2) return rc2;
      Emit e;
      e.gh = narrow ? nullptr : gh + a;
      e.gh16 = narrow ? reinterpret_cast<uint16_t*>(gh) + a : nullptr;
      e.ts = TS + a;
      e.ord = o;
      e.recs = reinterpret_cast<Rec*>(c->d_recs);
      e.regs = c->d_regs;
      e.wcnt = c->d_wcnt;
      rc2 = launch_classify(c, t, m, gout ? gout + a : nullptr, &e);
      if (rc2) return rc2;
    }
    HIPCHK(c, hipEventRecord(c->ev[c->ev_used + 1], c->stream));
    const int rc2 = launch_aggregate(c, t, TS + a, o, G ? G + a : nullptr, classify && !narrow ? gh + a : nullptr, a,
                                     m, classify && !narrow ? gh + count_from : nullptr, a + m - count_from,
                                     classify && narrow ? reinterpret_cast<uint16_t*>(gh) + count_from : nullptr);
    if (rc2) return rc2;
    HIPCHK(c, hipEventRecord(c->ev[c->ev_used + 2], c->stream));
    c->ev_used += 3;
    return RSA_OK;
  };
  c->table_dirty = true;
  const uint64_t kMinSplit = 1ull << 22;
  if (c->auto_tighten && !c->tightened && c->cap > 0 && n >= kMinSplit) {
    uint64_t done = 0;
    uint64_t next = n / c->filter_slice;
    if (next < (1ull << 20)) next = n < (1ull << 21) ? n / 2 : (1ull << 20);
    for (uint32_t step = 0; step < c->filter_steps && next < n; ++step) {
      rc = launch(done, next - done, next);
      if (rc) return rc;
      rc = cap_select(c, c->d_filter, nullptr);   // on the device: no host round trip
      if (rc) return rc;
      done = next;
      next = next * c->filter_growth;
    }
    c->tightened = true;
    // the last slice runs under the final filter bounds: its records of
    // bounded rules also go into the pass-2 fields, so the recount only has
    // to replay the earlier slices when the thresholds equal the bounds
    // (learned per context: after a job whose thresholds moved below the
    // bounds, so that the tentative fields had to be cleared and replayed,
    // the next kTentBackoff jobs do not fill them)
    bool tent = c->rec_cache && c->n_segs + 1 < (uint32_t)kMaxSegs && n - done + done <= c->recs2_alloc;
    if (tent && c->tent_skip) {
      --c->tent_skip;
      tent = false;
    }
    if (tent) {
      c->late_seg = c->n_segs;
      c->tent2_on = true;
    }
    rc = launch(done, n - done, 0);
    c->tent2_on = false;
    if (tent && (rc || !c->rec_cache || c->n_segs != c->late_seg + 1)) c->late_seg = 0xFFFFFFFFu - 1;   // (a reset is due)
    return rc;
  }
  return launch(0, n, 0);
}

int emit_mode(rsa_ctx* c, int mode, rsa_conn_record* out, uint64_t max_out, uint64_t* h_n) {
  if (!c || !h_n) return RSA_ERR_ARG;
  int rc = need_agg(c);
  if (rc) return rc;
  if (max_out && !out) return fail(c, RSA_ERR_ARG, "null output buffer");
  HIPCHK(c, hipMemsetAsync(c->d_cursor, 0, sizeof(unsigned long long), c->stream));
  c->cap_ctl_zeroed = false;   // d_cursor is advanced below: the next cap_select zeroes it itself
  // persistent grid (two 1024-thread workgroups per CU) over the device-side
  // used count; one round trip for the emitted count and the error flags
  k_emit<<<c->cu_count * 2, 1024, 0, c->stream>>>(c->d_slots, c->d_used, c->d_used_n, c->slot_cap, c->d_thresh, mode,
                                                  out, max_out, c->d_cursor, c->owner_world, c->owner_rank,
                                                  c->ukey_ok ? c->d_ukey : nullptr);
  HIPCHK(c, hipGetLastError());
  unsigned long long n = 0;
  unsigned int f[4];
  HIPCHK(c, hipMemcpyAsync(&n, c->d_cursor, sizeof n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(f, c->d_flags, sizeof f, hipMemcpyDeviceToHost, c->stream));
  // the job's pass-1 record count rides along (the next rsa_reset sizes its
  // regions from it without a round trip of its own)
  const bool read_recs = c->job_recs_valid && c->d_job_recs;
  if (read_recs)
    HIPCHK(c, hipMemcpyAsync(&c->h_job_recs, c->d_job_recs, sizeof c->h_job_recs, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->h_job_recs_valid = read_recs;
  rc = flags_status(c, f);
  if (rc) return rc;
  *h_n = n;
  if (n > max_out) return fail(c, RSA_ERR_CAPACITY, "%llu records do not fit in %llu", n, (unsigned long long)max_out);
  return RSA_OK;
}

}  // namespace

extern "C" {

int rsa_version(void) { return 2; }

int rsa_ctx_create(int device, rsa_ctx** out) {
  if (!out) return RSA_ERR_ARG;
  *out = nullptr;
  if (hipSetDevice(device) != hipSuccess) return RSA_ERR_HIP;
  rsa_ctx* c = new rsa_ctx();
  c->device = device;
  const char* dbg = getenv("RSA_DEBUG");
  c->debug = dbg && dbg[0] == '1';
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    c->cu_count = prop.multiProcessorCount;
  if (hipMalloc(&c->d_flags, 4 * sizeof(unsigned int)) != hipSuccess ||
      hipMalloc(&c->d_cursor, sizeof(unsigned long long)) != hipSuccess ||
      hipMalloc(&c->d_junk, 64 * sizeof(Rec)) != hipSuccess ||
      hipMalloc(&c->d_used_n, sizeof(unsigned long long)) != hipSuccess ||
      hipMemset(c->d_flags, 0, 4 * sizeof(unsigned int)) != hipSuccess ||
      hipMemset(c->d_used_n, 0, sizeof(unsigned long long)) != hipSuccess) {
    rsa_ctx_destroy(c);
    return RSA_ERR_HIP;
  }
  *out = c;
  return RSA_OK;
}

int rsa_ctx_destroy(rsa_ctx* c) {
  if (!c) return RSA_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  void* bufs[] = {c->d_tail, c->d_tail_n, c->d_gscratch, c->d_gh, c->d_stats, c->d_recs, c->d_recs2, c->d_junk, c->d_route_cur, c->d_regs, c->d_wcnt, c->d_nrecs, c->d_starts, c->d_hist,
                  c->d_scan_sums, c->d_occ, c->d_entries, c->d_off,
                  c->d_img, c->d_resid,
                  c->d_slots, c->d_used, c->d_ukey, c->d_used_n, c->d_filter, c->d_packed, c->d_hot, c->d_hot_tasks, c->d_hot_base,
                  c->d_hot_fill, c->d_hot_ctl, c->d_hot_total, c->d_cnt_words, c->d_cnt_starts,
                  c->d_cnt_tasks, c->d_cnt_ctl, c->d_flags, c->d_cursor, c->d_job_recs, c->d_cidx,
                  c->d_capped_gid, c->d_capped_cnt, c->d_capped_start, c->d_capped_prev, c->d_keys, c->d_chk};
  for (void* b : bufs) (void)hipFree(b);
  if (c->merge_state) rsa_internal_merge_free(c->merge_state);
  for (int k = 0; k < kMaxEvents; ++k)
    if (c->ev[k]) (void)hipEventDestroy(c->ev[k]);
  delete c;
  return RSA_OK;
}

const char* rsa_last_error(const rsa_ctx* c) { return c ? c->err.c_str() : "null ctx"; }

int rsa_set_stream(rsa_ctx* c, void* s) {
  if (!c) return RSA_ERR_ARG;
  c->stream = reinterpret_cast<hipStream_t>(s);
  return RSA_OK;
}

int rsa_set_option(rsa_ctx* c, int option, int64_t value) {
  if (!c) return RSA_ERR_ARG;
  switch (option) {
    case RSA_OPT_AUTO_FILTER:
      c->auto_tighten = value != 0;
      return RSA_OK;
    case RSA_OPT_FILTER_SLICE:
      if (value < 2 || value > 65536) return fail(c, RSA_ERR_ARG, "filter slice must be in [2, 65536]");
      c->filter_slice = (uint32_t)value;
      return RSA_OK;
    case RSA_OPT_FORCE_DEFER:
      c->force_defer = value != 0;
      return RSA_OK;
    case RSA_OPT_PROFILE_CLASSIFY:
      c->prof_classify = (uint32_t)value;
      return RSA_OK;
    case RSA_OPT_GROUP_TASKS:
      c->group_tasks = value != 0;
      return RSA_OK;
    case RSA_OPT_WAVE_CAP_SCATTER:
      c->wave_cap_scatter = value != 0;
      return RSA_OK;
    case RSA_OPT_FILTER_STEPS:
      if (value < 1 || value > 8) return fail(c, RSA_ERR_ARG, "filter steps must be in [1, 8]");
      c->filter_steps = (uint32_t)value;
      return RSA_OK;
    case RSA_OPT_FILTER_GROWTH:
      if (value < 2 || value > 64) return fail(c, RSA_ERR_ARG, "filter growth must be in [2, 64]");
      c->filter_growth = (uint32_t)value;
      return RSA_OK;
    case RSA_OPT_PROFILE_SKIP:
      c->profile_skip = (uint32_t)value;
      return RSA_OK;
    case RSA_OPT_PRECHECK:
      c->precheck = value != 0;
      return RSA_OK;
    case RSA_OPT_PARSE_STAGED:
      c->parse_staged = value != 0;
      return RSA_OK;
    case RSA_OPT_MIN_REGIONS_LOG2:
      if (value < 0 || value > 12) return fail(c, RSA_ERR_ARG, "RSA_OPT_MIN_REGIONS_LOG2 must be 0..12");
      c->min_regions_log2 = (uint32_t)value;
      return RSA_OK;
    case RSA_OPT_REDUCE_BIG:
      c->reduce_big = value != 0;
      return RSA_OK;
    case RSA_OPT_COUNTER_WORDS16:
      c->gh16 = value != 0;
      return RSA_OK;
    case RSA_OPT_CLASSIFY_PAIR:
      c->classify_pair = value != 0;
      return RSA_OK;
    case RSA_OPT_ROUTE_ROWS:
      if (value < 0) return fail(c, RSA_ERR_ARG, "RSA_OPT_ROUTE_ROWS must be >= 0");
      c->route_rows = (uint64_t)value;
      return RSA_OK;
    case RSA_OPT_REGION_RECORDS:
      if (value < 0 || value > 0xFFFFFFFFll) return fail(c, RSA_ERR_ARG, "RSA_OPT_REGION_RECORDS must be 0..2^32-1");
      c->region_records = (uint32_t)value;
      return RSA_OK;
    case RSA_OPT_REGION_IMPORT:
      c->region_import = value != 0;
      return RSA_OK;
    case RSA_OPT_COUNT_SORT:
      c->count_sort = value != 0;
      return RSA_OK;
    case RSA_OPT_OWNER_WORLD:
      if (value < 0) return fail(c, RSA_ERR_ARG, "owner world must be >= 0");
      c->owner_world = (uint32_t)value;
      return RSA_OK;
    case RSA_OPT_OWNER_RANK:
      if (value < 0) return fail(c, RSA_ERR_ARG, "owner rank must be >= 0");
      c->owner_rank = (uint32_t)value;
      return RSA_OK;
    case RSA_OPT_HOT_SPLIT:
      c->hot_split = value != 0;
      return RSA_OK;
    case RSA_OPT_HOT_MIN:
      if (value < 1) return fail(c, RSA_ERR_ARG, "hot-region minimum must be >= 1 record");
      c->hot_min = (unsigned long long)value;
      c->hot_factor = value < (int64_t)kHotMinRecs ? 0u : kHotFactor;   // testing: any region above the minimum
      return RSA_OK;
    case RSA_OPT_STATS:
      if (value && !c->d_stats) {
        HIPCHK(c, hipMalloc(&c->d_stats, 4 * sizeof(unsigned long long)));
        HIPCHK(c, hipMemset(c->d_stats, 0, 4 * sizeof(unsigned long long)));
      }
      c->stats_on = value != 0;
      return RSA_OK;
    case RSA_OPT_USE_INDEX:
      if (value && !c->index_loaded) return fail(c, RSA_ERR_STATE, "no index loaded");
      c->indexed = value != 0;
      return RSA_OK;
    default:
      return fail(c, RSA_ERR_ARG, "unknown option %d", option);
  }
}

hipStream_t rsa_internal_stream(rsa_ctx* c) { return c->stream; }
int rsa_internal_fail(rsa_ctx* c, int code, const char* msg) { return fail(c, code, "%s", msg); }
int rsa_internal_parse_staged(rsa_ctx* c) { return c->parse_staged ? 1 : 0; }
int rsa_internal_device(rsa_ctx* c) { return c->device; }
void rsa_internal_counters(rsa_ctx* c, unsigned long long** m, unsigned long long** h, unsigned int** d,
                           unsigned long long** t, uint32_t* n_rules) {
  *m = c->d_matches;
  *h = c->d_hits;
  *d = c->d_distinct;
  *t = c->d_thresh;
  *n_rules = c->n_rules;
}
void** rsa_internal_merge_slot(rsa_ctx* c) { return &c->merge_state; }
uint64_t rsa_internal_route_rows(rsa_ctx* c) { return c->route_rows; }

int rsa_sync(rsa_ctx* c) {
  if (!c) return RSA_ERR_ARG;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return RSA_OK;
}

int rsa_load_rules(rsa_ctx* c, const rsa_rule_entry* h_entries, uint32_t n_entries, const uint32_t* h_off,
                   uint32_t n_lists, uint32_t n_rules) {
  if (!c || !h_off || (n_entries && !h_entries)) return fail(c, RSA_ERR_ARG, "null argument");
  if (n_lists > 65536) return fail(c, RSA_ERR_ARG, "n_lists %u > 65536 (tuple list id is 16-bit)", n_lists);
  if (n_rules >= 0x7FFFFFFFu) return fail(c, RSA_ERR_ARG, "n_rules too large");
  if (h_off[0] != 0 || h_off[n_lists] != n_entries) return fail(c, RSA_ERR_ARG, "list offsets do not span entries");
  for (uint32_t l = 0; l < n_lists; ++l) {
    if (h_off[l + 1] < h_off[l]) return fail(c, RSA_ERR_ARG, "list offsets not monotone at %u", l);
    for (uint32_t e = h_off[l]; e < h_off[l + 1]; ++e) {
      if (h_entries[e].gid >= n_rules) return fail(c, RSA_ERR_ARG, "entry %u gid %u >= n_rules", e, h_entries[e].gid);
      const uint32_t st = h_entries[e].step;
      if (st) {   // a run: its last rule must exist too
        const uint32_t span = (st & RSA_STEP_SPORT) ? (h_entries[e].port_span & 0xFFFFu) : (h_entries[e].port_span >> 16);
        if ((uint64_t)h_entries[e].gid + (uint64_t)span * (st & ~RSA_STEP_SPORT) >= n_rules)
          return fail(c, RSA_ERR_ARG, "entry %u: run reaches past n_rules", e);
      }
      if (e > h_off[l] && h_entries[e].gid < h_entries[e - 1].gid)
        return fail(c, RSA_ERR_ARG, "list %u not in ascending gid order at entry %u", l, e);
    }
  }
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  int rc = upload(c, &c->d_entries, h_entries, n_entries);
  if (rc) return rc;
  rc = upload(c, &c->d_off, h_off, (size_t)n_lists + 1);
  if (rc) return rc;
  c->h_off.assign(h_off, h_off + n_lists + 1);
  c->n_entries = n_entries;
  c->n_lists = n_lists;
  c->n_rules = n_rules;
  c->rules_loaded = true;
  c->indexed = false;  // an index must be (re)loaded for these lists
  c->index_loaded = false;
  return RSA_OK;
}

namespace {

// A 16-bit-slot pruning table inside the image whose slot values are all <
// `limit` (the record's bitmap count; an empty slot is 0, bitmap 0).
bool table16_ok(const uint32_t* img, uint32_t words, const rsa_pht_table& t, uint32_t limit) {
  if (t.n_slots == 0 || t.n_slots > 0x10000u || (uint64_t)t.slot_off + t.n_slots > 2ull * words || (t.disp_mask & (t.disp_mask + 1)) != 0 ||
      (uint64_t)t.disp_off + t.disp_mask + 1 > 2ull * words || limit == 0 || limit > 0x100u)
    return false;
  const uint16_t* h = reinterpret_cast<const uint16_t*>(img);
  for (uint32_t q = 0; q < t.n_slots; ++q)
    if ((h[t.slot_off + q] & 0xFFu) >= limit) return false;
  return true;
}

// A CHD table inside the image whose slot values are all < `limit`; `empty`:
// the empty slot word (0xFFFFFFFF in the group tables, 0 in the pruning
// tables, whose value 0 is a valid index: bitmap 0).
bool table_ok(const uint32_t* img, uint32_t words, const rsa_pht_table& t, uint32_t limit,
              uint32_t empty = 0xFFFFFFFFu) {
  if (t.n_slots == 0 || t.n_slots > 0x10000u || (uint64_t)t.slot_off + t.n_slots > words || (t.disp_mask & (t.disp_mask + 1)) != 0 ||
      (uint64_t)t.disp_off + t.disp_mask + 1 > 2ull * words || limit == 0)
    return false;
  for (uint32_t q = 0; q < t.n_slots; ++q) {
    const uint32_t w = img[t.slot_off + q];
    if (w != empty && (w & 0xFFFFu) >= limit) return false;
  }
  return true;
}

}  // namespace

int rsa_load_index(rsa_ctx* c, const uint32_t* img, uint32_t words, const rsa_rule_entry* h_resid, uint32_t n_resid) {
  if (!c || !img || (n_resid && !h_resid)) return fail(c, RSA_ERR_ARG, "null argument");
  if (!c->rules_loaded) return fail(c, RSA_ERR_STATE, "load the candidate lists first");
  if (words < 8 || img[0] != 0xFFFFFFFFu || (img[1] != RSA_PHT_MAGIC && img[1] != RSA_BKT_MAGIC))
    return fail(c, RSA_ERR_ARG, "not an index image (word 0 must be empty, word 1 RSA_PHT_MAGIC or RSA_BKT_MAGIC)");
  const bool bkt = img[1] == RSA_BKT_MAGIC;
  if (words > (1u << 26)) return fail(c, RSA_ERR_ARG, "index image larger than 2^26 words");   // task words: gw << 6
  const uint32_t nl = c->n_lists;
  if (img[2] != nl) return fail(c, RSA_ERR_ARG, "image has %u lists, %u are loaded", img[2], nl);
  const uint32_t lo = img[3], nrec = img[4];
  const uint32_t lw = sizeof(rsa_pht_list) / 4, gw = sizeof(rsa_pht_group) / 4, mw = sizeof(rsa_pht_mask) / 4;
  if (nrec < nl || lo % 4 || (uint64_t)lo + (uint64_t)lw * nrec > words)
    return fail(c, RSA_ERR_ARG, "list records outside the image");
  // validate everything the kernels index with, so no launch can read out of
  // bounds and every chain terminates: a list's records cover its entries in
  // order, continuation records have larger ids than their predecessor
  std::vector<uint8_t> claimed(nrec, 0);
  for (uint32_t l = 0; l < nl; ++l) {
    uint32_t r = l, at = c->h_off[l];
    while (true) {
      if (claimed[r]) return fail(c, RSA_ERR_ARG, "record %u claimed twice", r);
      claimed[r] = 1;
      rsa_pht_list h;
      memcpy(&h, img + lo + (size_t)lw * r, sizeof h);
      if (h.entry_beg != at || (uint64_t)h.entry_beg + h.entry_len > c->h_off[l + 1])
        return fail(c, RSA_ERR_ARG, "list %u record %u: entry range differs from the loaded list", l, r);
      const uint32_t len = h.entry_len;
      if (h.resid_beg > h.resid_end || h.resid_end > n_resid)
        return fail(c, RSA_ERR_ARG, "list %u record %u: residual range out of bounds", l, r);
      if (h.prefix > len || (r != l && h.prefix != 0))
        return fail(c, RSA_ERR_ARG, "list %u record %u: bad prefix %u", l, r, h.prefix);
      for (uint32_t e = h.resid_beg; e < h.resid_end; ++e) {
        if (h_resid[e].gid >= c->n_rules) return fail(c, RSA_ERR_ARG, "residual entry %u gid out of range", e);
        if (e > h.resid_beg && h_resid[e].gid < h_resid[e - 1].gid)
          return fail(c, RSA_ERR_ARG, "list %u: residual not gid-ascending", l);
      }
      if (bkt && h.n_groups != 0) {
        // bucket index: table descriptors, bucket arrays and every slot's rows
        const uint32_t tw = sizeof(rsa_bkt_table) / 4;
        if (h.n_groups > (uint32_t)kBktMaxTables || h.group_off % 4 ||
            (uint64_t)h.group_off + (uint64_t)tw * h.n_groups > words)
          return fail(c, RSA_ERR_ARG, "list %u record %u: table descriptors outside the image", l, r);
        uint32_t prev_min = 0;
        for (uint32_t g = 0; g < h.n_groups; ++g) {
          rsa_bkt_table T;
          memcpy(&T, img + h.group_off + (size_t)tw * g, sizeof T);
          if (T.n_buckets == 0 || T.n_buckets > 0x10000u || T.bucket_off % 2 ||
              (uint64_t)T.bucket_off + 2ull * T.n_buckets > words)
            return fail(c, RSA_ERR_ARG, "list %u table %u: buckets outside the image", l, g);
          if (T.min_gid < prev_min) return fail(c, RSA_ERR_ARG, "list %u: tables not in ascending min gid", l);
          prev_min = T.min_gid;
          for (uint32_t s = 0; s < 2 * T.n_buckets; ++s) {
            const uint32_t w = img[T.bucket_off + s], len = (w >> 16) & 0x1Fu;
            if (!len) continue;
            const uint64_t beg = (uint64_t)T.entry_base + (w & 0xFFFFu);
            if (beg + len > n_resid) return fail(c, RSA_ERR_ARG, "list %u table %u: bucket rows out of bounds", l, g);
            if ((img[5] & 1u) && (uint64_t)T.filter_off + (w & 0xFFFFu) + len > words)
              return fail(c, RSA_ERR_ARG, "list %u table %u: row filters outside the image", l, g);
            for (uint64_t e = beg; e < beg + len; ++e)
              if (h_resid[e].gid >= c->n_rules || (e > beg && h_resid[e].gid < h_resid[e - 1].gid))
                return fail(c, RSA_ERR_ARG, "list %u table %u: bucket rows not gid-ascending or out of range", l, g);
          }
        }
      } else if (h.n_groups != 0) {
        if (h.n_groups > 64) return fail(c, RSA_ERR_ARG, "list %u: more than 64 groups", l);
        if (len > 0xFFFEu) return fail(c, RSA_ERR_ARG, "list %u record %u: indexed chunk too long", l, r);
        if (h.group_off % 4 || (uint64_t)h.group_off + (uint64_t)gw * h.n_groups > words || h.mask_off % 4 ||
            (uint64_t)h.mask_off + (uint64_t)mw * h.n_masks > words || h.bm_off % 2 ||
            (uint64_t)h.bm_off + 2ull * h.n_bitmaps > words)
          return fail(c, RSA_ERR_ARG, "list %u: records outside the image", l);
        for (uint32_t g = 0; g < h.n_groups; ++g) {
          rsa_pht_group G;
          memcpy(&G, img + h.group_off + (size_t)gw * g, sizeof G);
          if (G.class_mask > 0xFu) return fail(c, RSA_ERR_ARG, "list %u group %u: class_mask beyond 4 classes", l, g);
          for (int k = 0; k < 4; ++k) {
            if (!table_ok(img, words, G.table[k], len))
              return fail(c, RSA_ERR_ARG, "list %u group %u class %d: table outside the image or index out of list", l,
                          g, k);
            // a class outside the mask is skipped by whole waves: it must be the empty table
            if (!(G.class_mask >> k & 1u) && (G.table[k].slot_off != 0 || G.table[k].n_slots != 1))
              return fail(c, RSA_ERR_ARG, "list %u group %u class %d: not in class_mask but not the empty table", l,
                          g, k);
          }
        }
        if (h.n_src_masks > h.n_masks) return fail(c, RSA_ERR_ARG, "list %u: more src tables than tables", l);
        for (uint32_t m = 0; m < h.n_masks; ++m) {
          rsa_pht_mask M;
          memcpy(&M, img + h.mask_off + (size_t)mw * m, sizeof M);
          const rsa_pht_table T = {M.slot & ~RSA_PHT_NARROW, M.disp_off, M.size & 0x1FFFFu, M.size >> 17};
          if (!(M.slot & RSA_PHT_NARROW) && (img[5] & 2u))
            return fail(c, RSA_ERR_ARG, "list %u mask %u: 32-bit slots in an image flagged all-narrow", l, m);
          if ((M.slot & RSA_PHT_NARROW) ? !table16_ok(img, words, T, h.n_bitmaps)
                                        : !table_ok(img, words, T, h.n_bitmaps, 0u))
            return fail(c, RSA_ERR_ARG, "list %u mask %u: table outside the image or bitmap out of range", l, m);
        }
      }
      at = h.entry_beg + h.entry_len;
      if (h.next == RSA_PHT_NONE) break;
      if (h.next <= r || h.next < nl || h.next >= nrec)
        return fail(c, RSA_ERR_ARG, "list %u record %u: bad continuation record %u", l, r, h.next);
      r = h.next;
    }
    if (at != c->h_off[l + 1]) return fail(c, RSA_ERR_ARG, "list %u: records do not cover its entries", l);
  }
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  // padded to whole 16-B vectors (the LDS staging copies uint4s)
  std::vector<uint32_t> padded(img, img + words);
  padded.resize((words + 3) / 4 * 4, 0u);
  int rc = upload(c, &c->d_img, padded.data(), padded.size());
  if (!rc) rc = upload(c, &c->d_resid, h_resid, n_resid);
  if (rc) return rc;
  c->img_words = words;
  c->list_off = lo;
  c->index_loaded = true;
  c->bkt_index = bkt;
  c->bkt_filters = bkt && (img[5] & 1u);
  c->prune_narrow = !bkt && (img[5] & 2u);
  c->indexed = true;
  return RSA_OK;
}

int rsa_set_rule_count(rsa_ctx* c, uint32_t n_rules) {
  if (!c) return RSA_ERR_ARG;
  if (c->rules_loaded && n_rules != c->n_rules) return fail(c, RSA_ERR_ARG, "rule count differs from loaded rules");
  c->n_rules = n_rules;
  return RSA_OK;
}

int rsa_bind_counters(rsa_ctx* c, uint64_t* m, uint64_t* h, uint32_t* d, uint64_t* t) {
  if (!c || !m || !h || !d || !t) return fail(c, RSA_ERR_ARG, "null counter pointer");
  c->d_matches = reinterpret_cast<unsigned long long*>(m);
  c->d_hits = reinterpret_cast<unsigned long long*>(h);
  c->d_distinct = reinterpret_cast<unsigned int*>(d);
  c->d_thresh = reinterpret_cast<unsigned long long*>(t);
  return RSA_OK;
}

int rsa_reset(rsa_ctx* c, uint64_t capacity, uint32_t cap) {
  if (!c) return RSA_ERR_ARG;
  if (!c->d_matches) return fail(c, RSA_ERR_STATE, "counters not bound (rsa_bind_counters)");
  // the table is at most kMaxRegions regions of 2^kRegionMaxBits slots
  const unsigned long long max_slots = (unsigned long long)kMaxRegions << kRegionMaxBits;
  // A caller's capacity is an upper bound (callers pass the number of hit
  // lines, the case where every line is a new connection): clamp it to the
  // largest table; a real overflow still fails the job (RSA_ERR_CAPACITY).
  const unsigned long long max_cap = (max_slots - 64) / 3 * 2;
  if (capacity > max_cap) capacity = max_cap;
  HIPCHK(c, hipSetDevice(c->device));
  unsigned long long want = 1024;
  const unsigned long long need = capacity + capacity / 2 + 64;
  while (want < need) want <<= 1;
  if (c->occ_alloc < want / 32) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    hipFree(c->d_occ);
    c->d_occ = nullptr;
    c->occ_alloc = 0;
    HIPCHK(c, hipMalloc(&c->d_occ, want / 32 * sizeof(uint32_t)));
    c->occ_alloc = want / 32;
  }
  HIPCHK(c, hipMemsetAsync(c->d_occ, 0, want / 32 * sizeof(uint32_t), c->stream));
  if (!c->d_starts)
    HIPCHK(c, hipMalloc(&c->d_starts, (size_t)kMaxSegs * (kMaxRegions + 1) * sizeof(unsigned long long)));
  c->pass1_calls = 0;
  c->rec_cache = false;
  c->n_segs = 0;
  c->seg_base = 0;
  {
    uint32_t bits = 0;
    while ((1ull << bits) < want) ++bits;
    // regions of at most 2^16 slots, and at least 2^min_regions_log2 of them
    // (one k_reduce workgroup each: 1024 = four per CU, so a CU's workgroups
    // overlap their flushes; cfg2 7.43 -> 6.37 ms/step against 256) while
    // they keep >= 1024 slots
    // and, when the previous job of this ctx classified many records, at least
    // records / region_records of them (k_reduce<1> time grows with a region's
    // records; cfg4/cfg5 at ~87M records: 11.04 -> 10.63 / 10.46 -> 9.68 ms per
    // step at 4096 regions, while cfg3's 41M keep 1024: profiles/r04ak_*)
    uint32_t want_np = c->min_regions_log2;
    if (c->region_records && c->job_recs_valid) {
      // the count as the job's emission read it, else one read here
      unsigned long long prev = c->h_job_recs;
      if (!c->h_job_recs_valid) {
        HIPCHK(c, hipMemcpyAsync(&prev, c->d_job_recs, sizeof prev, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
      }
      uint32_t lg = 0;
      while (lg < 12u && (1ull << lg) * c->region_records < prev) ++lg;
      if (lg > want_np) want_np = lg;
    }
    uint32_t rs = bits < (uint32_t)kRegionMaxBits ? bits : (uint32_t)kRegionMaxBits;
    while (rs > 10 && bits - rs < want_np) --rs;
    c->rs_bits = rs;
    c->np_bits = bits - rs;
  }
  if (!c->d_job_recs) HIPCHK(c, hipMalloc(&c->d_job_recs, sizeof(unsigned long long)));
  HIPCHK(c, hipMemsetAsync(c->d_job_recs, 0, sizeof(unsigned long long), c->stream));
  c->job_recs_valid = false;
  c->h_job_recs_valid = false;
  c->ncap_on_device = false;
  if (want > c->slot_alloc) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    hipFree(c->d_slots);
    hipFree(c->d_used);
    hipFree(c->d_ukey);
    c->d_slots = nullptr;
    c->d_used = nullptr;
    c->d_ukey = nullptr;
    c->slot_alloc = 0;
    HIPCHK(c, hipMalloc(&c->d_slots, want * sizeof(Slot)));
    HIPCHK(c, hipMalloc(&c->d_used, want * sizeof(unsigned long long)));
    HIPCHK(c, hipMalloc(&c->d_ukey, want * sizeof(unsigned long long)));
    // A fresh allocation is written only where the per-record atomic import
    // needs empty keys: every other path finds occupancy in the job's bitmap
    // and writes a whole slot when it claims one, so never-claimed slots are
    // never read (a cold job at cfg3's bound: 7 GB of slots, 5.9 ms of
    // k_table_init saved)
    if (!c->region_import) {
      k_table_init<<<grid_for(c, want, 8), kBlock, 0, c->stream>>>(c->d_slots, want);
      HIPCHK(c, hipGetLastError());
    }
    c->slots_init = !c->region_import;
    c->slot_alloc = want;
    c->table_dirty = false;
  } else if (!c->region_import && !c->slots_init) {
    // (the atomic import chosen after jobs that left claimed slots behind
    // without clearing them: every slot once)
    k_table_init<<<grid_for(c, c->slot_alloc, 8), kBlock, 0, c->stream>>>(c->d_slots, c->slot_alloc);
    HIPCHK(c, hipGetLastError());
    c->slots_init = true;
    c->table_dirty = false;
  } else if (c->table_dirty && !c->region_import) {
    // the per-record atomic import (RSA_OPT_REGION_IMPORT=0) claims slots by
    // CAS on an empty key: clear exactly the slots the previous job used
    // (they may lie anywhere in the allocation; their number is read on the
    // device).  Every other path decides occupancy by the bitmap cleared
    // below and writes a whole slot when it claims one, so the slots keep
    // the previous job's contents (no 64 B write per used slot per job).
    k_table_clear<<<c->cu_count * 8, kBlock, 0, c->stream>>>(c->d_slots, c->d_used, c->d_used_n, c->slot_alloc);
    HIPCHK(c, hipGetLastError());
    c->table_dirty = false;
  }
  if (c->region_import) c->slots_init = false;   // this job's claims stay behind uncleared
  c->slots_clean = !c->table_dirty && c->slots_init;
  c->ukey_ok = true;
  c->slot_cap = want;
  c->cap = cap;
  HIPCHK(c, hipMemsetAsync(c->d_used_n, 0, sizeof(unsigned long long), c->stream));
  const size_t nr = c->n_rules;
  if (nr) {
    HIPCHK(c, hipMemsetAsync(c->d_matches, 0, nr * sizeof(unsigned long long), c->stream));
    HIPCHK(c, hipMemsetAsync(c->d_hits, 0, nr * sizeof(unsigned long long), c->stream));
    HIPCHK(c, hipMemsetAsync(c->d_distinct, 0, nr * sizeof(unsigned int), c->stream));
    HIPCHK(c, hipMemsetAsync(c->d_thresh, 0xFF, nr * sizeof(unsigned long long), c->stream));
  }
  if (c->filter_len < (nr ? nr : 1) || !c->d_filter) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    hipFree(c->d_filter);
    c->d_filter = nullptr;
    c->filter_len = 0;
    hipFree(c->d_packed);
    c->d_packed = nullptr;
    HIPCHK(c, hipMalloc(&c->d_filter, (nr ? nr : 1) * sizeof(unsigned long long)));
    HIPCHK(c, hipMalloc(&c->d_packed, (nr ? nr : 1) * sizeof(unsigned long long)));
    c->filter_len = nr ? (uint32_t)nr : 1;
  }
  HIPCHK(c, hipMemsetAsync(c->d_filter, 0xFF, (nr ? nr : 1) * sizeof(unsigned long long), c->stream));
  HIPCHK(c, hipMemsetAsync(c->d_packed, 0, (nr ? nr : 1) * sizeof(unsigned long long), c->stream));
  c->tightened = false;
  c->late_seg = 0xFFFFFFFFu;
  c->tent2_on = false;
  HIPCHK(c, hipMemsetAsync(c->d_flags, 0, 4 * sizeof(unsigned int), c->stream));
  c->table_ready = true;
  return RSA_OK;
}

int rsa_classify(rsa_ctx* c, const rsa_tuple* T, const uint32_t* TS, const uint64_t* ORD, uint64_t n, int32_t* gout) {
  if (!c) return RSA_ERR_ARG;
  if (!c->rules_loaded) return fail(c, RSA_ERR_STATE, "no rules loaded");
  int rc = need_agg(c);
  if (rc) return rc;
  if (n == 0) return RSA_OK;
  if (!T || !TS || !ORD) return fail(c, RSA_ERR_ARG, "null tuple/ts/order pointer");
  return run_pass1(c, 1, T, TS, ORD, nullptr, gout, n);
}

int rsa_classify_only(rsa_ctx* c, const rsa_tuple* T, uint64_t n, int32_t* gout) {
  if (!c) return RSA_ERR_ARG;
  if (!c->rules_loaded) return fail(c, RSA_ERR_STATE, "no rules loaded");
  if (n == 0) return RSA_OK;
  if (!T || !gout) return fail(c, RSA_ERR_ARG, "null tuple/gid pointer");
  if (!c->d_flags) return fail(c, RSA_ERR_STATE, "ctx not initialised");
  if (n > 0x7FFFFFFFull) return fail(c, RSA_ERR_ARG, "batch larger than 2^31 tuples");
  return launch_classify(c, reinterpret_cast<const uint4*>(T), n, gout, nullptr);
}

int rsa_aggregate_gids(rsa_ctx* c, const rsa_tuple* T, const uint32_t* TS, const uint64_t* ORD, const int32_t* G,
                       uint64_t n) {
  if (!c) return RSA_ERR_ARG;
  int rc = need_agg(c);
  if (rc) return rc;
  if (n == 0) return RSA_OK;
  if (!T || !TS || !ORD || !G) return fail(c, RSA_ERR_ARG, "null tuple/ts/order/gid pointer");
  return run_pass1(c, 0, T, TS, ORD, G, nullptr, n);
}

int rsa_last_pass1_times(rsa_ctx* c, float* h_classify_ms, float* h_aggregate_ms) {
  if (!c || !h_classify_ms || !h_aggregate_ms) return RSA_ERR_ARG;
  float tc = 0.f, ta = 0.f;
  for (int k = 0; k + 3 <= c->ev_used; k += 3) {
    HIPCHK(c, hipEventSynchronize(c->ev[k + 2]));
    float a = 0.f, b = 0.f;
    HIPCHK(c, hipEventElapsedTime(&a, c->ev[k], c->ev[k + 1]));
    HIPCHK(c, hipEventElapsedTime(&b, c->ev[k + 1], c->ev[k + 2]));
    tc += a;
    ta += b;
  }
  *h_classify_ms = tc;
  *h_aggregate_ms = ta;
  return RSA_OK;
}

int rsa_last_pass1_launches(rsa_ctx* c, uint32_t* h_n) {
  if (!c || !h_n) return RSA_ERR_ARG;
  *h_n = (uint32_t)(c->ev_used / 3);
  return RSA_OK;
}

int rsa_last_pass1_ms(rsa_ctx* c, float* h_ms) {
  if (!h_ms) return RSA_ERR_ARG;
  float a = 0.f, b = 0.f;
  const int rc = rsa_last_pass1_times(c, &a, &b);
  if (rc) return rc;
  *h_ms = a + b;
  return RSA_OK;
}

int rsa_resolve_cap(rsa_ctx* c, uint32_t* h_n_capped) {
  if (!c) return RSA_ERR_ARG;
  int rc = need_agg(c);
  if (rc) return rc;
  rc = cap_select(c, c->d_thresh, h_n_capped);
  // with no host count the recount reads it on the device (and returns at
  // once when it is 0); a caller that read the count decides itself, and may
  // rewrite the thresholds before the recount (the multi-GPU merge installs
  // the global ones), so its recount never skips on the local count
  c->ncap_on_device = rc == RSA_OK && h_n_capped == nullptr;
  return rc;
}

constexpr uint32_t kTentBackoff = 8;

int rsa_recount(rsa_ctx* c, const rsa_tuple* T, const uint32_t* TS, const uint64_t* ORD, const int32_t* G,
                uint64_t n) {
  if (!c) return RSA_ERR_ARG;
  int rc = need_agg(c);
  if (rc) return rc;
  if (n == 0) return RSA_OK;
  if (!T || !TS || !ORD) return fail(c, RSA_ERR_ARG, "null tuple/ts/order pointer");
  // pass 1's last slice put its records of bounded rules into the pass-2
  // fields (Agg::tent2): exact when every bounded rule's threshold equals its
  // bound and no rule was capped only at the end; then the recount replays the
  // earlier slices only.  Otherwise those fields are cleared and everything
  // is replayed.
  uint32_t n_segs = c->n_segs;
  const bool tent = c->late_seg != 0xFFFFFFFFu;
  bool clear = tent;
  const bool cached = c->rec_cache && c->cache_T == (const void*)T && c->cache_n == n && c->n_segs > 0;
  if (tent && cached && c->late_seg + 1 == c->n_segs && c->n_rules) {
    if (!c->d_chk) HIPCHK(c, hipMalloc(&c->d_chk, 2 * sizeof(uint32_t)));
    HIPCHK(c, hipMemsetAsync(c->d_chk, 0, 2 * sizeof(uint32_t), c->stream));
    k_tent_check<<<(c->n_rules + kBlock - 1) / kBlock, kBlock, 0, c->stream>>>(
        c->d_filter, c->d_thresh, c->n_rules, c->d_chk);
    uint32_t h[2] = {1u, 1u};
    HIPCHK(c, hipMemcpyAsync(h, c->d_chk, sizeof h, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->debug) fprintf(stderr, "[rsa] recount: %u bounded rules moved below their bound, %u capped only now\n", h[0], h[1]);
    if (!h[0] && !h[1]) {
      clear = false;
      n_segs = c->late_seg;   // the last slice is already counted
    }
    c->tent_skip = clear ? kTentBackoff : 0u;
  }
  if (clear) {
    k_pass2_clear<<<c->cu_count * 8, kBlock, 0, c->stream>>>(c->d_slots, c->d_used, c->d_used_n, c->slot_alloc);
    HIPCHK(c, hipGetLastError());
  }
  c->late_seg = 0xFFFFFFFFu;   // (a second recount replays everything)
  if (cached) {
    // every occurrence with order <= P of a capped rule produced a pass-1
    // record (P <= the filter bound in force when its line was aggregated)
    if (n_segs == 0) return RSA_OK;
    const unsigned long long* hb = nullptr;
    const uint32_t* hf = nullptr;
    const HRec* hr = nullptr;
    const unsigned int* skip = c->ncap_on_device ? c->d_flags + 2 : nullptr;
    c->ncap_on_device = false;
    int rc2 = hot_split<2>(c, 0, n_segs, n, &hb, &hf, &hr, skip);
    if (rc2) return rc2;
    // (a resolution whose count the host did not read leaves it at d_flags[2]:
    // the kernels skip their work on the device when no rule is capped)
    k_reduce<2><<<1u << c->np_bits, 1024, 0, c->stream>>>(reinterpret_cast<const Rec*>(c->d_recs2), c->d_starts,
                                                         n_segs, agg_of(c), hb, hf, hr, skip);
    HIPCHK(c, hipGetLastError());
    return RSA_OK;
  }
  if (!G) {
    // re-classify into scratch gids
    if (!c->rules_loaded) return fail(c, RSA_ERR_STATE, "no rules loaded (recount without gids re-classifies)");
    rc = ensure_buf(c, &c->d_gscratch, &c->gscratch_alloc, n);
    if (!rc) rc = rsa_classify_only(c, T, n, c->d_gscratch);
    if (rc) return rc;
    G = c->d_gscratch;
  }
  k_pass2<<<grid_for(c, n, 16), kBlock, 0, c->stream>>>(reinterpret_cast<const uint4*>(T), TS,
                                                        reinterpret_cast<const unsigned long long*>(ORD), n, G,
                                                        c->n_rules, agg_of(c));
  HIPCHK(c, hipGetLastError());
  return RSA_OK;
}

int rsa_emit(rsa_ctx* c, rsa_conn_record* out, uint64_t max_out, uint64_t* h_n) {
  return emit_mode(c, 0, out, max_out, h_n);
}

int rsa_export(rsa_ctx* c, int which, rsa_conn_record* out, uint64_t max_out, uint64_t* h_n) {
  if (which < 0 || which > 2) return fail(c, RSA_ERR_ARG, "which must be 0, 1 or 2");
  return emit_mode(c, which == 2 ? 3 : which ? 2 : 1, out, max_out, h_n);
}

int rsa_export_routed(rsa_ctx* c, int which, uint32_t world, rsa_conn_record* out, uint64_t max_out,
                      uint64_t* d_counts) {
  if (!c) return RSA_ERR_ARG;
  if (which < 0 || which > 2) return fail(c, RSA_ERR_ARG, "which must be 0, 1 or 2");
  if (world == 0 || world > (uint32_t)kRouteMax) return fail(c, RSA_ERR_ARG, "world must be 1..%d", kRouteMax);
  if (!d_counts) return fail(c, RSA_ERR_ARG, "null counts pointer");
  if (max_out && !out) return fail(c, RSA_ERR_ARG, "null output buffer");
  int rc = need_agg(c);
  if (rc) return rc;
  if (c->owner_world != world) return fail(c, RSA_ERR_STATE, "RSA_OPT_OWNER_WORLD must equal world");
  const int mode = which == 2 ? 3 : which ? 2 : 1;
  unsigned long long* counts = reinterpret_cast<unsigned long long*>(d_counts);
  // counts[world] (caller's) and the route cursors[world] (ctx scratch)
  if (!c->d_route_cur) HIPCHK(c, hipMalloc(&c->d_route_cur, kRouteMax * sizeof(unsigned long long)));
  HIPCHK(c, hipMemsetAsync(counts, 0, world * sizeof(unsigned long long), c->stream));
  HIPCHK(c, hipMemsetAsync(c->d_route_cur, 0, world * sizeof(unsigned long long), c->stream));
  const unsigned long long* uk = c->ukey_ok ? c->d_ukey : nullptr;
  k_emit_route<false><<<c->cu_count * 2, 1024, 0, c->stream>>>(c->d_slots, c->d_used, c->d_used_n, c->slot_cap,
                                                              c->d_thresh, mode, world, c->owner_rank, uk, counts,
                                                              c->d_route_cur, out, max_out);
  k_emit_route<true><<<c->cu_count * 2, 1024, 0, c->stream>>>(c->d_slots, c->d_used, c->d_used_n, c->slot_cap,
                                                             c->d_thresh, mode, world, c->owner_rank, uk, counts,
                                                             c->d_route_cur, out, max_out);
  HIPCHK(c, hipGetLastError());
  c->cap_ctl_zeroed = false;
  return RSA_OK;
}

int rsa_import(rsa_ctx* c, int which, const rsa_conn_record* in, uint64_t n) {
  if (!c) return RSA_ERR_ARG;
  if (which != 0 && which != 1) return fail(c, RSA_ERR_ARG, "which must be 0 or 1");
  int rc = need_agg(c);
  if (rc) return rc;
  if (n == 0) return RSA_OK;
  if (!in) return fail(c, RSA_ERR_ARG, "null input records");
  c->table_dirty = true;
  if (!c->region_import) {
    if (which == 0 && !c->slots_clean)
      return fail(c, RSA_ERR_STATE, "RSA_OPT_REGION_IMPORT=0 imports need the table cleared: set it before rsa_reset");
    if (which == 0) c->ukey_ok = false;   // CAS claims do not know their used-list index: cap resolution reads slots
    k_import<<<grid_for_threads(c, n, 1024, 4), 1024, 0, c->stream>>>(in, n, which, agg_of(c));
    HIPCHK(c, hipGetLastError());
    return RSA_OK;
  }
  if (n > 0xFFFFFFFFull) return fail(c, RSA_ERR_ARG, "more than 2^32 records in one import");
  const uint32_t n_regions = 1u << c->np_bits;
  if (!c->d_hot_base) {
    HIPCHK(c, hipMalloc(&c->d_hot_base, kMaxRegions * sizeof(unsigned long long)));
    HIPCHK(c, hipMalloc(&c->d_hot_fill, kMaxRegions * sizeof(uint32_t)));
    HIPCHK(c, hipMalloc(&c->d_hot_ctl, 4 * sizeof(uint32_t)));
    HIPCHK(c, hipMalloc(&c->d_hot_total, sizeof(unsigned long long)));
  }
  if (n > c->hot_alloc) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    hipFree(c->d_hot);
    c->d_hot = nullptr;
    c->hot_alloc = 0;
    HIPCHK(c, hipMalloc(&c->d_hot, n * sizeof(HRec)));
    c->hot_alloc = n;
  }
  // counts [0, n_regions], scanned in place (k_scan_sums writes the total at
  // [n_regions]); cursors behind them
  int rc2 = ensure_buf(c, &c->d_scan_sums, &c->scan_sums_alloc, 2ull * (kMaxRegions + 1));
  if (rc2) return rc2;
  uint32_t* counts = c->d_scan_sums;
  uint32_t* cursor = c->d_scan_sums + kMaxRegions + 1;
  HIPCHK(c, hipMemsetAsync(counts, 0, 2ull * (kMaxRegions + 1) * sizeof(uint32_t), c->stream));
  const Agg ag = agg_of(c);
  k_imp_hist<<<grid_for_threads(c, n, 1024, 2), 1024, 0, c->stream>>>(in, n, ag, n_regions, counts);
  k_scan_sums<<<1, 1024, 0, c->stream>>>(counts, n_regions);
  k_imp_scatter<<<grid_for_threads(c, (n + kImpChunk - 1) / kImpChunk * 1024, 1024, 2), 1024, 0, c->stream>>>(
      in, n, ag, n_regions, counts, cursor, static_cast<HRec*>(c->d_hot));
  k_imp_desc<<<(n_regions + 255) / 256, 256, 0, c->stream>>>(counts, cursor, n_regions, c->d_hot_base, c->d_hot_fill);
  if (which == 0)
    k_reduce<1><<<n_regions, 1024, 0, c->stream>>>(nullptr, c->d_starts, 0, ag, c->d_hot_base, c->d_hot_fill,
                                                   static_cast<const HRec*>(c->d_hot), nullptr);
  else
    k_reduce<2><<<n_regions, 1024, 0, c->stream>>>(nullptr, c->d_starts, 0, ag, c->d_hot_base, c->d_hot_fill,
                                                   static_cast<const HRec*>(c->d_hot), nullptr);
  HIPCHK(c, hipGetLastError());
  return RSA_OK;
}

int rsa_shadowed(rsa_ctx* c, const rsa_shadow_rule* h_rules, uint32_t n, int32_t* h_cover) {
  return rsa_shadowed_ports(c, h_rules, n, nullptr, 0, h_cover);
}

int rsa_shadowed_ports(rsa_ctx* c, const rsa_shadow_rule* h_rules, uint32_t n, const int32_t* h_ports,
                       uint32_t n_ports, int32_t* h_cover) {
  if (!c || (n && (!h_rules || !h_cover)) || (n_ports && !h_ports)) return fail(c, RSA_ERR_ARG, "null argument");
  if (n == 0) return RSA_OK;
  // every list a rule names lies inside the port array (the kernel trusts them)
  for (uint32_t k = 0; k < n; ++k) {
    for (int32_t v : {h_rules[k].sport, h_rules[k].dport}) {
      if (v >= -1) continue;
      const uint64_t at = (uint64_t)(-(int64_t)v - 2);
      if (at >= n_ports || h_ports[at] < 1 || at + 1 + (uint64_t)h_ports[at] > n_ports)
        return fail(c, RSA_ERR_ARG, "rule %u: port list outside the port array", k);
    }
  }
  HIPCHK(c, hipSetDevice(c->device));
  rsa_shadow_rule* d_rules = nullptr;
  int32_t* d_cover = nullptr;
  int32_t* d_ports = nullptr;
  HIPCHK(c, hipMalloc(&d_rules, (size_t)n * sizeof(rsa_shadow_rule)));
  if (hipMalloc(&d_cover, (size_t)n * sizeof(int32_t)) != hipSuccess ||
      hipMalloc(&d_ports, (size_t)(n_ports ? n_ports : 1) * sizeof(int32_t)) != hipSuccess) {
    hipFree(d_rules);
    hipFree(d_cover);
    return fail(c, RSA_ERR_HIP, "hipMalloc of the shadow buffers failed");
  }
  int rc = RSA_OK;
  hipError_t e = hipMemcpyAsync(d_rules, h_rules, (size_t)n * sizeof(rsa_shadow_rule), hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess && n_ports)
    e = hipMemcpyAsync(d_ports, h_ports, (size_t)n_ports * sizeof(int32_t), hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) {
    k_shadow<<<(n + 1023) / 1024, 1024, 0, c->stream>>>(d_rules, n, d_ports, d_cover);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(h_cover, d_cover, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) rc = fail(c, RSA_ERR_HIP, "rsa_shadowed: %s", hipGetErrorString(e));
  hipFree(d_rules);
  hipFree(d_cover);
  hipFree(d_ports);
  return rc;
}

#ifdef RSA_PHASE_PROF
// PROFILING BUILD ONLY: the classifier's phase cycles (see PhaseAcc): out[0..7]
// summed wave cycles per phase, out[8] wave iterations; out[9..16] k_reduce<1>'s
// (g_phase).
int rsa_phase_prof(rsa_ctx* c, uint64_t* h_out, int reset) {
  if (!c || !h_out) return RSA_ERR_ARG;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpyFromSymbol(h_out, HIP_SYMBOL(g_phase), kPhaseWords * sizeof(uint64_t)));
  if (reset) {
    const uint64_t z[kPhaseWords] = {};
    HIPCHK(c, hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof z));
  }
  return RSA_OK;
}
#endif

int rsa_stats(rsa_ctx* c, uint64_t* h_out, int reset) {
  if (!c || !h_out) return RSA_ERR_ARG;
  if (!c->d_stats) {
    for (int k = 0; k < 4; ++k) h_out[k] = 0;
    return RSA_OK;
  }
  HIPCHK(c, hipMemcpyAsync(h_out, c->d_stats, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (reset) HIPCHK(c, hipMemsetAsync(c->d_stats, 0, 4 * sizeof(uint64_t), c->stream));
  return RSA_OK;
}

int rsa_table_size(rsa_ctx* c, uint64_t* h_n) {
  if (!c || !h_n) return RSA_ERR_ARG;
  int rc = need_agg(c);
  if (rc) return rc;
  unsigned long long n = 0;
  rc = used_count(c, &n);
  if (rc) return rc;
  *h_n = n;
  return RSA_OK;
}

}  // extern "C"
