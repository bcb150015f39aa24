// ruleset_hip.hip — MI355X (gfx950, CDNA4) hot path of ruleset-analysis.
//
// What the reference does per log line (Python 2, one process per Hadoop split):
//   mapper.py:159-189        build the candidate rule list, scan it with
//                            FirewallRule.__contains__ (firewallrule.py:128-174),
//                            emit the FIRST matching expanded rule index;
//   connlist-reducer.py:62-176  per rule: count lines, count "hits"
//                            (-6-302013/-6-302015), keep a distinct-connection
//                            dict capped at MAX_NUMBER_OF_CONNECTIONS_PER_RULE
//                            (config.py:15) in sorted-line order.
//
// What this library does instead (integer work, HBM/VALU bound, no MFMA):
//   pass 1  one lane per tuple; a wave "waterfalls" over the distinct candidate
//           lists present in it, so rule entries are wave-uniform and come in
//           through the scalar cache; the first match is the minimum matching
//           gid (lists are gid-sorted); per-rule counters and a distinct
//           (rule, connection) hash table are updated with device atomics.
//   cap     per capped rule, the order key of the line that inserted the
//           cap-th distinct connection, by an 8-pass radix select over the
//           table's per-entry minimum order keys.
//   pass 2  recount (count/first/last) of occurrences with order <= P for the
//           capped rules only — the exact restatement of the frozen dict.
//   emit    compact the table to rsa_conn_record rows.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/ruleset_hip.h"

namespace {

constexpr unsigned long long kEmpty = 0xFFFFFFFFFFFFFFFFull;
constexpr unsigned long long kBusy = 0xFFFFFFFFFFFFFFFEull;
constexpr uint32_t kNoGid = 0xFFFFFFFFu;
constexpr int kBlock = 256;

// One distinct (rule, connection) aggregate in HBM, 64 B (one half L2 line).
struct alignas(64) Slot {
  unsigned long long kA;         // for_ip << 32 | to_ip
  unsigned long long kB;         // gid << 32 | pspell << 16 | to_port ; kEmpty / kBusy
  unsigned long long min_order;  // first occurrence (reducer input order)
  unsigned int count, first, last;      // pass-1 aggregates (all occurrences)
  unsigned int count2, first2, last2;   // pass-2 aggregates (order <= P only)
  unsigned int pad[4];
};
static_assert(sizeof(Slot) == 64, "slot layout");
static_assert(sizeof(rsa_tuple) == 16, "tuple layout");
static_assert(sizeof(rsa_rule_entry) == 32, "rule layout");
static_assert(sizeof(rsa_conn_record) == 40, "record layout");

// Rule entries are read through the constant address space so that wave-uniform
// loads become scalar (s_load) loads through the scalar cache.
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(4))) const v4u const_uint4;
typedef __attribute__((address_space(4))) const uint32_t const_u32;

struct Rules {
  const const_uint4* e;   // 2 x uint4 per entry
  const const_u32* off;
  uint32_t n_lists;
  uint32_t n_rules;
};

struct Agg {
  unsigned long long* matches;
  unsigned long long* hits;
  unsigned int* distinct;
  const unsigned long long* thresh;
  const unsigned long long* filter;  // per rule: lines with order > filter cannot matter (cap)
  Slot* slots;
  unsigned long long mask;  // capacity - 1 (power of two)
  unsigned int* flags;      // [0] overflow, [1] bad gid/list
  uint32_t cap;
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

// counter[key] += 1 for every lane with `ok`, one device atomic per distinct key
// in the wave (lanes sharing a rule are counted first: hot rules would otherwise
// serialise thousands of atomics on one address).  Wave-uniform control flow.
template <typename T>
__device__ __forceinline__ void wave_count_by_key(bool ok, uint32_t key, T* counter) {
  unsigned long long pending = __ballot(ok);
  while (pending) {
    const int leader = __builtin_ctzll(pending);
    const uint32_t k = __builtin_amdgcn_readlane(key, leader);
    const unsigned long long peers = __ballot(ok && key == k);
    pending &= ~peers;
    if ((int)__lane_id() == leader) atomicAdd(&counter[k], (T)__popcll(peers));
  }
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

// First-match classification of one wave of tuples.  Entry loads are wave-uniform
// (list id broadcast by readlane), so they are scalar loads through the K$.
__device__ __forceinline__ uint32_t classify_wave(uint4 t, bool active, const Rules& R, unsigned int* flags) {
  uint32_t list = t.w & 0xFFFFu;
  if (active && list >= R.n_lists) {
    atomicOr(&flags[1], 1u);
    active = false;
  }
  uint32_t best = kNoGid;
  unsigned long long pending = __ballot(active);
  const uint32_t src = t.x, dst = t.y;
  const uint32_t sp = t.z & 0xFFFFu, dp = t.z >> 16;
  while (pending) {
    const int leader = __builtin_ctzll(pending);
    const uint32_t L = __builtin_amdgcn_readlane(list, leader);
    const bool mine = active && list == L;
    pending &= ~__ballot(mine);
    const uint32_t beg = R.off[L];
    const uint32_t end = R.off[L + 1];
    uint32_t e = beg;
    for (; e + 4 <= end; e += 4) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const v4u a = R.e[2 * (e + j)];
        const v4u b = R.e[2 * (e + j) + 1];
        const bool m = ((src - a.x) <= a.y) & ((dst - a.z) <= a.w) &
                       ((sp - (b.x & 0xFFFFu)) <= (b.y & 0xFFFFu)) & ((dp - (b.x >> 16)) <= (b.y >> 16));
        best = min(best, (m & mine) ? b.z : kNoGid);
      }
      if (__ballot(mine && best == kNoGid) == 0) break;
    }
    if (e + 4 > end) {
      for (; e < end; ++e) {
        const v4u a = R.e[2 * e];
        const v4u b = R.e[2 * e + 1];
        const bool m = ((src - a.x) <= a.y) & ((dst - a.z) <= a.w) &
                       ((sp - (b.x & 0xFFFFu)) <= (b.y & 0xFFFFu)) & ((dp - (b.x >> 16)) <= (b.y >> 16));
        best = min(best, (m & mine) ? b.z : kNoGid);
      }
    }
  }
  return active ? best : kNoGid;
}

// Insert-or-combine (kA, kB) into the open-addressing table.  All key reads are
// device atomics (executed beyond the per-XCD L2s, so every XCD sees one value).
// A slot is claimed EMPTY->BUSY, its kA published, then kB published; a lane
// that reads BUSY retries the same slot on its next iteration.  Every key word
// is only ever accessed by device atomics, which execute beyond the per-XCD
// L2s, so no XCD can observe a stale copy.
__device__ __forceinline__ bool table_combine(const Agg& A, unsigned long long kA, unsigned long long kB,
                                              unsigned int cnt, unsigned int first, unsigned int last,
                                              unsigned long long order) {
  bool fresh = false;
  unsigned long long h = slot_hash(kA, kB) & A.mask;
  unsigned long long probes = 0;
  Slot* s = nullptr;
  while (true) {
    Slot* c = &A.slots[h];
    const unsigned long long cur = atomicCAS(&c->kB, kEmpty, kBusy);
    if (cur == kEmpty) {
      // kA is published by a device atomic; waiting for its completion before the
      // kB exchange orders the two at the memory side (no cache write-back fence).
      atomicExch(&c->kA, kA);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      atomicExch(&c->kB, kB);
      fresh = true;
      s = c;
      break;
    }
    if (cur == kBusy) continue;
    if (cur == kB) {
      if (atomicOr(&c->kA, 0ull) == kA) {
        s = c;
        break;
      }
    }
    h = (h + 1) & A.mask;
    if (++probes > A.mask) break;
  }
  if (!s) {
    atomicOr(&A.flags[0], 1u);
    return false;
  }
  atomicAdd(&s->count, cnt);
  atomicMin(&s->first, first);
  atomicMax(&s->last, last);
  atomicMin(&s->min_order, order);
  return fresh;
}

// Find an existing key (after pass 1 completed: plain loads are coherent across
// the kernel boundary).
__device__ __forceinline__ Slot* table_find(const Agg& A, unsigned long long kA, unsigned long long kB) {
  unsigned long long h = slot_hash(kA, kB) & A.mask;
  for (unsigned long long probes = 0; probes <= A.mask; ++probes) {
    Slot* c = &A.slots[h];
    const unsigned long long cb = c->kB;
    if (cb == kEmpty) return nullptr;
    if (cb == kB && c->kA == kA) return c;
    h = (h + 1) & A.mask;
  }
  return nullptr;
}

// Pass-1 modes: classify + aggregate (mapper fused with reducer), aggregate with
// the gid given per tuple (reducer drop-in), classify only (mapper drop-in).
enum { kClassifyAgg = 0, kGivenAgg = 1, kClassifyOnly = 2 };

template <int kMode>
__global__ __launch_bounds__(kBlock) void k_pass1(const uint4* __restrict__ T, const uint32_t* __restrict__ TS,
                                                  const unsigned long long* __restrict__ ORD, unsigned long long n,
                                                  const int32_t* __restrict__ gin, int32_t* __restrict__ gout,
                                                  Rules R, Agg A) {
  const unsigned long long stride = (unsigned long long)gridDim.x * kBlock;
  for (unsigned long long base = (unsigned long long)blockIdx.x * kBlock; base < n; base += stride) {
    const unsigned long long i = base + threadIdx.x;
    const bool in = i < n;
    const uint4 t = in ? T[i] : make_uint4(0u, 0u, 0u, 0u);
    const uint32_t flags = (t.w >> 16) & 0xFFu;
    uint32_t gid;
    if (kMode == kGivenAgg) {
      gid = in ? (uint32_t)gin[i] : kNoGid;
    } else {
      gid = classify_wave(t, in && (flags & RSA_F_VALID), R, A.flags);
    }
    if (kMode != kGivenAgg && gout && in) gout[i] = (int32_t)gid;
    if (kMode == kClassifyOnly) continue;
    if (gid != kNoGid && gid >= R.n_rules) atomicOr(&A.flags[1], 2u);
    const bool matched = gid < R.n_rules;
    const bool hit = matched && (flags & RSA_F_HIT);
    wave_count_by_key(matched, gid, A.matches);
    wave_count_by_key(hit, gid, A.hits);
    bool fresh = false;
    if (hit && (flags & RSA_F_BUILT) && A.cap > 0) {
      const unsigned long long o = ORD[i];
      // exact skip: the rule is already capped with threshold <= filter < o
      if (o <= A.filter[gid]) {
        unsigned long long kA, kB;
        conn_key(t, gid, kA, kB);
        const uint32_t ts = TS[i];
        fresh = table_combine(A, kA, kB, 1u, ts, ts, o);
      }
    }
    wave_count_by_key(fresh, gid, A.distinct);
  }
}

template <bool kGiven>
__global__ __launch_bounds__(kBlock) void k_pass2(const uint4* __restrict__ T, const uint32_t* __restrict__ TS,
                                                  const unsigned long long* __restrict__ ORD, unsigned long long n,
                                                  const int32_t* __restrict__ gin, Rules R, Agg A) {
  const unsigned long long stride = (unsigned long long)gridDim.x * kBlock;
  for (unsigned long long base = (unsigned long long)blockIdx.x * kBlock; base < n; base += stride) {
    const unsigned long long i = base + threadIdx.x;
    const bool in = i < n;
    const uint4 t = in ? T[i] : make_uint4(0u, 0u, 0u, 0u);
    const uint32_t flags = (t.w >> 16) & 0xFFu;
    uint32_t gid;
    if (kGiven) {
      gid = in ? (uint32_t)gin[i] : kNoGid;
    } else {
      gid = classify_wave(t, in && (flags & RSA_F_VALID), R, A.flags);
    }
    if (gid == kNoGid || gid >= R.n_rules) continue;
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

__global__ void k_table_init(Slot* S, unsigned long long cap) {
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += stride) {
    Slot s;
    s.kA = 0;
    s.kB = kEmpty;
    s.min_order = kEmpty;
    s.count = 0;
    s.first = 0xFFFFFFFFu;
    s.last = 0;
    s.count2 = 0;
    s.first2 = 0xFFFFFFFFu;
    s.last2 = 0;
    s.pad[0] = s.pad[1] = s.pad[2] = s.pad[3] = 0;
    S[i] = s;
  }
}

// Wave-aggregated append to a global cursor: one atomic per wave.  Must be
// called by every lane of the wave (wave-uniform control flow).
__device__ __forceinline__ unsigned long long wave_append(bool ok, unsigned long long* cursor) {
  const unsigned long long mask = __ballot(ok);
  if (mask == 0) return 0;
  const unsigned lane = __lane_id();
  const int leader = __builtin_ctzll(mask);
  unsigned long long base = 0;
  if ((int)lane == leader) base = atomicAdd(cursor, (unsigned long long)__popcll(mask));
  base = __shfl(base, leader);
  return base + __popcll(mask & ((1ull << lane) - 1ull));
}

// ---- cap resolution (exact): P = cap-th smallest min_order among a rule's entries.
// Capped entries are compacted to (min_order, capped index) pairs, sorted by
// min_order then stably by capped index (two LSD radix sorts), so each capped
// rule's entries form one ascending segment and P is the segment's cap-th element.
__global__ void k_cap_mark(const unsigned int* distinct, uint32_t n_rules, uint32_t cap, uint32_t* cidx,
                           uint32_t* capped_gid, uint32_t* capped_cnt, unsigned int* n_capped,
                           unsigned long long* thresh) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_rules) return;
  thresh[g] = RSA_NO_THRESHOLD;
  if (cap > 0 && distinct[g] >= cap) {
    const unsigned int c = atomicAdd(n_capped, 1u);
    cidx[g] = c;
    capped_gid[c] = g;
    capped_cnt[c] = distinct[g];
  } else {
    cidx[g] = 0xFFFFFFFFu;
  }
}

__global__ __launch_bounds__(kBlock) void k_cap_collect(const Slot* S, unsigned long long cap_slots,
                                                        const uint32_t* cidx, unsigned long long* keys,
                                                        uint32_t* vals, unsigned long long* cursor) {
  const unsigned long long stride = (unsigned long long)gridDim.x * kBlock;
  for (unsigned long long base = (unsigned long long)blockIdx.x * kBlock; base < cap_slots; base += stride) {
    const unsigned long long i = base + threadIdx.x;
    uint32_t c = 0xFFFFFFFFu;
    unsigned long long o = 0;
    if (i < cap_slots) {
      const unsigned long long kB = S[i].kB;
      if (kB < kBusy) {
        c = cidx[kB >> 32];
        o = S[i].min_order;
      }
    }
    const bool ok = c != 0xFFFFFFFFu;
    const unsigned long long pos = wave_append(ok, cursor);
    if (ok) {
      keys[pos] = o;
      vals[pos] = c;
    }
  }
}

__global__ void k_cap_pick(const unsigned long long* sorted_orders, const uint32_t* start, const uint32_t* capped_gid,
                           uint32_t n_capped, uint32_t cap, unsigned long long* thresh) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < n_capped) thresh[capped_gid[c]] = sorted_orders[(size_t)start[c] + cap - 1];
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

// mode 0: final report rows; mode 1: export pass-1 aggregates; mode 2: export pass-2.
__global__ __launch_bounds__(kBlock) void k_emit(const Slot* S, unsigned long long cap_slots,
                                                 const unsigned long long* thresh, int mode, rsa_conn_record* out,
                                                 unsigned long long max_out, unsigned long long* cursor) {
  const unsigned long long stride = (unsigned long long)gridDim.x * kBlock;
  for (unsigned long long base = (unsigned long long)blockIdx.x * kBlock; base < cap_slots; base += stride) {
    const unsigned long long i = base + threadIdx.x;
    int which = -1;
    Slot s;
    if (i < cap_slots) {
      s = S[i];
      if (s.kB < kBusy) {
        if (mode == 0) {
          const unsigned long long P = thresh[s.kB >> 32];
          if (P == RSA_NO_THRESHOLD) which = 0;
          else if (s.min_order <= P) which = 1;
        } else if (mode == 1) {
          which = 0;
        } else if (s.count2 != 0) {
          which = 1;
        }
      }
    }
    const unsigned long long k = wave_append(which >= 0, cursor);
    if (which >= 0 && k < max_out) out[k] = make_record(s, which);
  }
}

__global__ void k_import(const rsa_conn_record* __restrict__ in, unsigned long long n, int which, Agg A) {
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const rsa_conn_record r = in[i];
    const unsigned long long kA = ((unsigned long long)r.for_ip << 32) | r.to_ip;
    const unsigned long long kB = ((unsigned long long)r.gid << 32) | ((unsigned long long)r.pspell << 16) | r.to_port;
    if (which == 0) {
      const bool fresh = table_combine(A, kA, kB, r.count, r.first, r.last, r.min_order);
      if (fresh) atomicAdd(&A.distinct[r.gid], 1u);
    } else {
      Slot* s = table_find(A, kA, kB);
      if (!s) {
        atomicOr(&A.flags[1], 8u);
        continue;
      }
      atomicAdd(&s->count2, r.count);
      atomicMin(&s->first2, r.first);
      atomicMax(&s->last2, r.last);
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_count_used(const Slot* S, unsigned long long cap_slots,
                                                       unsigned long long* cursor) {
  const unsigned long long stride = (unsigned long long)gridDim.x * kBlock;
  for (unsigned long long base = (unsigned long long)blockIdx.x * kBlock; base < cap_slots; base += stride) {
    const unsigned long long i = base + threadIdx.x;
    const bool used = i < cap_slots && S[i].kB < kBusy;
    wave_append(used, cursor);
  }
}

}  // namespace

struct rsa_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  rsa_rule_entry* d_entries = nullptr;
  uint32_t n_entries = 0;
  uint32_t* d_off = nullptr;
  uint32_t n_lists = 0;
  uint32_t n_rules = 0;
  bool rules_loaded = false;
  unsigned long long* d_matches = nullptr;
  unsigned long long* d_hits = nullptr;
  unsigned int* d_distinct = nullptr;
  unsigned long long* d_thresh = nullptr;
  unsigned long long* d_filter = nullptr;  // library-owned, n_rules
  uint32_t filter_len = 0;
  bool auto_tighten = true;
  bool tightened = false;
  Slot* d_slots = nullptr;
  unsigned long long slot_cap = 0;    // power of two
  unsigned long long slot_alloc = 0;  // allocated slots
  uint32_t cap = 1000;
  bool table_ready = false;
  unsigned int* d_flags = nullptr;       // 4 words
  unsigned long long* d_cursor = nullptr;
  // cap-resolution scratch
  uint32_t* d_cidx = nullptr;
  uint32_t cidx_len = 0;
  uint32_t* d_capped_gid = nullptr;
  uint32_t* d_capped_cnt = nullptr;
  uint32_t* d_capped_start = nullptr;
  uint32_t capped_alloc = 0;
  // sort scratch (capped entries)
  unsigned long long* d_keys[2] = {nullptr, nullptr};
  uint32_t* d_vals[2] = {nullptr, nullptr};
  unsigned long long sort_alloc = 0;
  void* d_temp = nullptr;
  size_t temp_alloc = 0;
  int cu_count = 256;
  std::string err;
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

#define HIPCHK(ctx, expr)                                                                   \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) return fail((ctx), RSA_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

Rules rules_of(const rsa_ctx* c) {
  Rules r;
  r.e = (const const_uint4*)(c->d_entries);
  r.off = (const const_u32*)(c->d_off);
  r.n_lists = c->n_lists;
  r.n_rules = c->n_rules;
  return r;
}

Agg agg_of(const rsa_ctx* c) {
  Agg a;
  a.matches = c->d_matches;
  a.hits = c->d_hits;
  a.distinct = c->d_distinct;
  a.thresh = c->d_thresh;
  a.filter = c->d_filter;
  a.slots = c->d_slots;
  a.mask = c->slot_cap ? c->slot_cap - 1 : 0;
  a.flags = c->d_flags;
  a.cap = c->cap;
  return a;
}

unsigned grid_for(const rsa_ctx* c, unsigned long long n, unsigned per_cu) {
  unsigned long long g = (n + kBlock - 1) / kBlock;
  const unsigned long long lim = (unsigned long long)c->cu_count * per_cu;
  if (g > lim) g = lim;
  if (g == 0) g = 1;
  return (unsigned)g;
}

int check_flags(rsa_ctx* c) {
  unsigned int f[4];
  HIPCHK(c, hipMemcpyAsync(f, c->d_flags, sizeof f, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (f[0]) return fail(c, RSA_ERR_CAPACITY, "distinct-connection table overflow (capacity %llu)", c->slot_cap);
  if (f[1] & 1u) return fail(c, RSA_ERR_ARG, "tuple references a candidate list id >= n_lists (%u)", c->n_lists);
  if (f[1] & 2u) return fail(c, RSA_ERR_ARG, "rule id >= n_rules (%u)", c->n_rules);
  if (f[1] & 4u) return fail(c, RSA_ERR_STATE, "pass 2 found an occurrence with no pass-1 entry");
  if (f[1] & 8u) return fail(c, RSA_ERR_STATE, "pass-2 import of a key absent from the table");
  return RSA_OK;
}

int need_agg(rsa_ctx* c) {
  if (!c->d_matches || !c->d_hits || !c->d_distinct || !c->d_thresh)
    return fail(c, RSA_ERR_STATE, "counters not bound (rsa_bind_counters)");
  if (!c->table_ready) return fail(c, RSA_ERR_STATE, "table not initialised (rsa_reset)");
  return RSA_OK;
}

}  // namespace

static int run_pass1(rsa_ctx* c, int mode, const rsa_tuple* T, const uint32_t* TS, const uint64_t* ORD,
                     const int32_t* G, int32_t* gout, uint64_t n);

extern "C" {

int rsa_version(void) { return 1; }

int rsa_ctx_create(int device, rsa_ctx** out) {
  if (!out) return RSA_ERR_ARG;
  *out = nullptr;
  rsa_ctx* c = new rsa_ctx();
  c->device = device;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    delete c;
    return RSA_ERR_HIP;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    c->cu_count = prop.multiProcessorCount;
  if (hipMalloc(&c->d_flags, 4 * sizeof(unsigned int)) != hipSuccess ||
      hipMalloc(&c->d_cursor, sizeof(unsigned long long)) != hipSuccess) {
    delete c;
    return RSA_ERR_HIP;
  }
  hipMemset(c->d_flags, 0, 4 * sizeof(unsigned int));
  *out = c;
  return RSA_OK;
}

int rsa_ctx_destroy(rsa_ctx* c) {
  if (!c) return RSA_OK;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  hipFree(c->d_entries);
  hipFree(c->d_off);
  hipFree(c->d_slots);
  hipFree(c->d_flags);
  hipFree(c->d_cursor);
  hipFree(c->d_cidx);
  hipFree(c->d_capped_gid);
  hipFree(c->d_capped_cnt);
  hipFree(c->d_capped_start);
  hipFree(c->d_filter);
  hipFree(c->d_keys[0]);
  hipFree(c->d_keys[1]);
  hipFree(c->d_vals[0]);
  hipFree(c->d_vals[1]);
  hipFree(c->d_temp);
  delete c;
  return RSA_OK;
}

const char* rsa_last_error(const rsa_ctx* c) { return c ? c->err.c_str() : "null ctx"; }

int rsa_set_stream(rsa_ctx* c, void* s) {
  if (!c) return RSA_ERR_ARG;
  c->stream = reinterpret_cast<hipStream_t>(s);
  return RSA_OK;
}

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
      if (e > h_off[l] && h_entries[e].gid < h_entries[e - 1].gid)
        return fail(c, RSA_ERR_ARG, "list %u not in ascending gid order at entry %u", l, e);
    }
  }
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  hipFree(c->d_entries);
  hipFree(c->d_off);
  c->d_entries = nullptr;
  c->d_off = nullptr;
  const size_t eb = (size_t)(n_entries ? n_entries : 1) * sizeof(rsa_rule_entry);
  HIPCHK(c, hipMalloc(&c->d_entries, eb));
  HIPCHK(c, hipMalloc(&c->d_off, (size_t)(n_lists + 1) * sizeof(uint32_t)));
  if (n_entries) HIPCHK(c, hipMemcpy(c->d_entries, h_entries, (size_t)n_entries * sizeof(rsa_rule_entry), hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->d_off, h_off, (size_t)(n_lists + 1) * sizeof(uint32_t), hipMemcpyHostToDevice));
  c->n_entries = n_entries;
  c->n_lists = n_lists;
  c->n_rules = n_rules;
  c->rules_loaded = true;
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
  HIPCHK(c, hipSetDevice(c->device));
  unsigned long long want = 1024;
  const unsigned long long need = capacity + capacity / 2 + 64;
  while (want < need) want <<= 1;
  if (want > c->slot_alloc) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    hipFree(c->d_slots);
    c->d_slots = nullptr;
    c->slot_alloc = 0;
    HIPCHK(c, hipMalloc(&c->d_slots, want * sizeof(Slot)));
    c->slot_alloc = want;
  }
  c->slot_cap = want;
  c->cap = cap;
  k_table_init<<<grid_for(c, want, 8), kBlock, 0, c->stream>>>(c->d_slots, want);
  HIPCHK(c, hipGetLastError());
  const size_t nr = c->n_rules;
  if (nr) {
    HIPCHK(c, hipMemsetAsync(c->d_matches, 0, nr * sizeof(unsigned long long), c->stream));
    HIPCHK(c, hipMemsetAsync(c->d_hits, 0, nr * sizeof(unsigned long long), c->stream));
    HIPCHK(c, hipMemsetAsync(c->d_distinct, 0, nr * sizeof(unsigned int), c->stream));
    HIPCHK(c, hipMemsetAsync(c->d_thresh, 0xFF, nr * sizeof(unsigned long long), c->stream));
  }
  if (c->filter_len < nr || !c->d_filter) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    hipFree(c->d_filter);
    c->d_filter = nullptr;
    c->filter_len = 0;
    HIPCHK(c, hipMalloc(&c->d_filter, (nr ? nr : 1) * sizeof(unsigned long long)));
    c->filter_len = nr ? (uint32_t)nr : 1;
  }
  HIPCHK(c, hipMemsetAsync(c->d_filter, 0xFF, (nr ? nr : 1) * sizeof(unsigned long long), c->stream));
  c->tightened = false;
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
  return run_pass1(c, kClassifyAgg, T, TS, ORD, nullptr, gout, n);
}

int rsa_classify_only(rsa_ctx* c, const rsa_tuple* T, uint64_t n, int32_t* gout) {
  if (!c) return RSA_ERR_ARG;
  if (!c->rules_loaded) return fail(c, RSA_ERR_STATE, "no rules loaded");
  if (n == 0) return RSA_OK;
  if (!T || !gout) return fail(c, RSA_ERR_ARG, "null tuple/gid pointer");
  Agg a = agg_of(c);
  k_pass1<kClassifyOnly><<<grid_for(c, n, 16), kBlock, 0, c->stream>>>(reinterpret_cast<const uint4*>(T), nullptr,
                                                                      nullptr, n, nullptr, gout, rules_of(c), a);
  HIPCHK(c, hipGetLastError());
  return RSA_OK;
}

int rsa_aggregate_gids(rsa_ctx* c, const rsa_tuple* T, const uint32_t* TS, const uint64_t* ORD, const int32_t* G,
                       uint64_t n) {
  if (!c) return RSA_ERR_ARG;
  int rc = need_agg(c);
  if (rc) return rc;
  if (n == 0) return RSA_OK;
  if (!T || !TS || !ORD || !G) return fail(c, RSA_ERR_ARG, "null tuple/ts/order/gid pointer");
  return run_pass1(c, kGivenAgg, T, TS, ORD, G, nullptr, n);
}

static int ensure_temp(rsa_ctx* c, size_t bytes) {
  if (bytes <= c->temp_alloc) return RSA_OK;
  hipFree(c->d_temp);
  c->d_temp = nullptr;
  c->temp_alloc = 0;
  HIPCHK(c, hipMalloc(&c->d_temp, bytes));
  c->temp_alloc = bytes;
  return RSA_OK;
}

// Exact selection of P for every rule with >= cap distinct entries in the
// current table, written to out[] (RSA_NO_THRESHOLD for the others).  On the
// final table this is the reducer's cap threshold; on a partial table it is an
// upper bound of it (the filter), because first-seen orders only decrease and
// the set of connections only grows as more lines are aggregated.
static int cap_select(rsa_ctx* c, unsigned long long* out, uint32_t* h_n_capped) {
  int rc = check_flags(c);
  if (rc) return rc;
  const uint32_t nr = c->n_rules;
  *h_n_capped = 0;
  if (nr == 0) return RSA_OK;
  if (c->cidx_len < nr) {
    hipFree(c->d_cidx);
    hipFree(c->d_capped_gid);
    hipFree(c->d_capped_cnt);
    hipFree(c->d_capped_start);
    c->d_cidx = c->d_capped_gid = c->d_capped_cnt = c->d_capped_start = nullptr;
    c->cidx_len = 0;
    HIPCHK(c, hipMalloc(&c->d_cidx, (size_t)nr * sizeof(uint32_t)));
    HIPCHK(c, hipMalloc(&c->d_capped_gid, (size_t)nr * sizeof(uint32_t)));
    HIPCHK(c, hipMalloc(&c->d_capped_cnt, (size_t)nr * sizeof(uint32_t)));
    HIPCHK(c, hipMalloc(&c->d_capped_start, (size_t)nr * sizeof(uint32_t)));
    c->cidx_len = nr;
  }
  unsigned int* d_ncap = c->d_flags + 2;
  HIPCHK(c, hipMemsetAsync(d_ncap, 0, sizeof(unsigned int), c->stream));
  HIPCHK(c, hipMemsetAsync(c->d_cursor, 0, sizeof(unsigned long long), c->stream));
  k_cap_mark<<<(nr + kBlock - 1) / kBlock, kBlock, 0, c->stream>>>(c->d_distinct, nr, c->cap, c->d_cidx,
                                                                   c->d_capped_gid, c->d_capped_cnt, d_ncap, out);
  HIPCHK(c, hipGetLastError());
  unsigned int ncap = 0;
  HIPCHK(c, hipMemcpyAsync(&ncap, d_ncap, sizeof ncap, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  *h_n_capped = ncap;
  if (ncap == 0) return RSA_OK;
  // upper bound on capped entries: every used slot
  unsigned long long bound = c->slot_cap;
  if (c->sort_alloc < bound) {
    for (int k = 0; k < 2; ++k) {
      hipFree(c->d_keys[k]);
      hipFree(c->d_vals[k]);
      c->d_keys[k] = nullptr;
      c->d_vals[k] = nullptr;
    }
    c->sort_alloc = 0;
    for (int k = 0; k < 2; ++k) {
      HIPCHK(c, hipMalloc(&c->d_keys[k], bound * sizeof(unsigned long long)));
      HIPCHK(c, hipMalloc(&c->d_vals[k], bound * sizeof(uint32_t)));
    }
    c->sort_alloc = bound;
  }
  k_cap_collect<<<grid_for(c, c->slot_cap, 8), kBlock, 0, c->stream>>>(c->d_slots, c->slot_cap, c->d_cidx,
                                                                       c->d_keys[0], c->d_vals[0], c->d_cursor);
  HIPCHK(c, hipGetLastError());
  unsigned long long m = 0;
  HIPCHK(c, hipMemcpyAsync(&m, c->d_cursor, sizeof m, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (m > 0xFFFFFFFFull) return fail(c, RSA_ERR_CAPACITY, "more than 2^32 capped entries");
  int cbits = 1;
  while (cbits < 32 && (1ull << cbits) < ncap) ++cbits;
  // sort by min_order, then stably by capped index; exclusive scan of segment sizes
  hipcub::DoubleBuffer<unsigned long long> keys(c->d_keys[0], c->d_keys[1]);
  hipcub::DoubleBuffer<uint32_t> vals(c->d_vals[0], c->d_vals[1]);
  size_t t1 = 0, t2 = 0, t3 = 0;
  HIPCHK(c, hipcub::DeviceRadixSort::SortPairs(nullptr, t1, keys, vals, (int)m, 0, 64, c->stream));
  HIPCHK(c, hipcub::DeviceRadixSort::SortPairs(nullptr, t2, vals, keys, (int)m, 0, cbits, c->stream));
  HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(nullptr, t3, c->d_capped_cnt, c->d_capped_start, (int)ncap, c->stream));
  size_t tb = t1 > t2 ? t1 : t2;
  if (t3 > tb) tb = t3;
  rc = ensure_temp(c, tb);
  if (rc) return rc;
  HIPCHK(c, hipcub::DeviceRadixSort::SortPairs(c->d_temp, tb, keys, vals, (int)m, 0, 64, c->stream));
  HIPCHK(c, hipcub::DeviceRadixSort::SortPairs(c->d_temp, tb, vals, keys, (int)m, 0, cbits, c->stream));
  HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(c->d_temp, tb, c->d_capped_cnt, c->d_capped_start, (int)ncap,
                                             c->stream));
  k_cap_pick<<<(ncap + kBlock - 1) / kBlock, kBlock, 0, c->stream>>>(keys.Current(), c->d_capped_start,
                                                                     c->d_capped_gid, ncap, c->cap, out);
  HIPCHK(c, hipGetLastError());
  return RSA_OK;
}

int rsa_resolve_cap(rsa_ctx* c, uint32_t* h_n_capped) {
  if (!c || !h_n_capped) return RSA_ERR_ARG;
  int rc = need_agg(c);
  if (rc) return rc;
  return cap_select(c, c->d_thresh, h_n_capped);
}

// Pass 1 over one batch.  With auto-tightening, a large first batch is split:
// the first 1/16 builds the table, then the filter (an exact upper bound of each
// capped rule's threshold) is computed, and the rest of the batch skips the
// table for lines that cannot change any output.
static int run_pass1(rsa_ctx* c, int mode, const rsa_tuple* T, const uint32_t* TS, const uint64_t* ORD,
                     const int32_t* G, int32_t* gout, uint64_t n) {
  auto launch = [&](uint64_t a, uint64_t m) -> int {
    const uint4* t = reinterpret_cast<const uint4*>(T) + a;
    const unsigned long long* o = reinterpret_cast<const unsigned long long*>(ORD) + a;
    if (mode == kClassifyAgg) {
      k_pass1<kClassifyAgg><<<grid_for(c, m, 16), kBlock, 0, c->stream>>>(t, TS + a, o, m, nullptr,
                                                                          gout ? gout + a : nullptr, rules_of(c),
                                                                          agg_of(c));
    } else {
      k_pass1<kGivenAgg><<<grid_for(c, m, 16), kBlock, 0, c->stream>>>(t, TS + a, o, m, G + a, nullptr,
                                                                       rules_of(c), agg_of(c));
    }
    HIPCHK(c, hipGetLastError());
    return RSA_OK;
  };
  const uint64_t kMinSplit = 1ull << 22;
  if (c->auto_tighten && !c->tightened && c->cap > 0 && n >= kMinSplit) {
    const uint64_t first = n / 16;
    int rc = launch(0, first);
    if (rc) return rc;
    uint32_t ncap = 0;
    rc = cap_select(c, c->d_filter, &ncap);
    if (rc) return rc;
    c->tightened = true;
    return launch(first, n - first);
  }
  return launch(0, n);
}

int rsa_recount(rsa_ctx* c, const rsa_tuple* T, const uint32_t* TS, const uint64_t* ORD, const int32_t* G,
                uint64_t n) {
  if (!c) return RSA_ERR_ARG;
  int rc = need_agg(c);
  if (rc) return rc;
  if (n == 0) return RSA_OK;
  if (!T || !TS || !ORD) return fail(c, RSA_ERR_ARG, "null tuple/ts/order pointer");
  if (G) {
    k_pass2<true><<<grid_for(c, n, 16), kBlock, 0, c->stream>>>(
        reinterpret_cast<const uint4*>(T), TS, reinterpret_cast<const unsigned long long*>(ORD), n, G, rules_of(c),
        agg_of(c));
  } else {
    if (!c->rules_loaded) return fail(c, RSA_ERR_STATE, "no rules loaded (recount without gids re-classifies)");
    k_pass2<false><<<grid_for(c, n, 16), kBlock, 0, c->stream>>>(
        reinterpret_cast<const uint4*>(T), TS, reinterpret_cast<const unsigned long long*>(ORD), n, nullptr,
        rules_of(c), agg_of(c));
  }
  HIPCHK(c, hipGetLastError());
  return RSA_OK;
}

static int emit_mode(rsa_ctx* c, int mode, rsa_conn_record* out, uint64_t max_out, uint64_t* h_n) {
  if (!c || !h_n) return RSA_ERR_ARG;
  int rc = need_agg(c);
  if (rc) return rc;
  if (max_out && !out) return fail(c, RSA_ERR_ARG, "null output buffer");
  HIPCHK(c, hipMemsetAsync(c->d_cursor, 0, sizeof(unsigned long long), c->stream));
  k_emit<<<grid_for(c, c->slot_cap, 8), kBlock, 0, c->stream>>>(c->d_slots, c->slot_cap, c->d_thresh, mode, out,
                                                                 max_out, c->d_cursor);
  HIPCHK(c, hipGetLastError());
  unsigned long long n = 0;
  HIPCHK(c, hipMemcpyAsync(&n, c->d_cursor, sizeof n, hipMemcpyDeviceToHost, c->stream));
  rc = check_flags(c);  // synchronises
  if (rc) return rc;
  *h_n = n;
  if (n > max_out) return fail(c, RSA_ERR_CAPACITY, "%llu records do not fit in %llu", n, (unsigned long long)max_out);
  return RSA_OK;
}

int rsa_emit(rsa_ctx* c, rsa_conn_record* out, uint64_t max_out, uint64_t* h_n) {
  return emit_mode(c, 0, out, max_out, h_n);
}

int rsa_export(rsa_ctx* c, int which, rsa_conn_record* out, uint64_t max_out, uint64_t* h_n) {
  if (which != 0 && which != 1) return fail(c, RSA_ERR_ARG, "which must be 0 or 1");
  return emit_mode(c, which ? 2 : 1, out, max_out, h_n);
}

int rsa_import(rsa_ctx* c, int which, const rsa_conn_record* in, uint64_t n) {
  if (!c) return RSA_ERR_ARG;
  if (which != 0 && which != 1) return fail(c, RSA_ERR_ARG, "which must be 0 or 1");
  int rc = need_agg(c);
  if (rc) return rc;
  if (n == 0) return RSA_OK;
  if (!in) return fail(c, RSA_ERR_ARG, "null input records");
  k_import<<<grid_for(c, n, 16), kBlock, 0, c->stream>>>(in, n, which, agg_of(c));
  HIPCHK(c, hipGetLastError());
  return RSA_OK;
}

int rsa_table_size(rsa_ctx* c, uint64_t* h_n) {
  if (!c || !h_n) return RSA_ERR_ARG;
  int rc = need_agg(c);
  if (rc) return rc;
  HIPCHK(c, hipMemsetAsync(c->d_cursor, 0, sizeof(unsigned long long), c->stream));
  k_count_used<<<grid_for(c, c->slot_cap, 8), kBlock, 0, c->stream>>>(c->d_slots, c->slot_cap, c->d_cursor);
  HIPCHK(c, hipGetLastError());
  unsigned long long n = 0;
  HIPCHK(c, hipMemcpyAsync(&n, c->d_cursor, sizeof n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  *h_n = n;
  return RSA_OK;
}

}  // extern "C"
