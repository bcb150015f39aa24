// The multi-GPU merge behind one C-ABI call (rsa_merge / rsa_merge_rccl /
// rsa_gather): the replacement of the reference's keyed shuffle into
// NUM_REDUCERS reducers and of `hadoop dfs -getmerge` (runAnalysis.sh:12,42-56,
// README.md:35-38; connlist-reducer.py:146-176 is what each owner's table then
// holds).  The protocol (include/ruleset_hip.h, rsa_merge) is the one
// ruleset_analysis_amd/dist.py models for the CPU tests: owner = gid % world,
// counters SUM, routed pass-1 export + all_to_allv, owner import + cap
// resolution, thresholds MAX, pass-2 recount + exchange, owners emit, sizes
// SUM, gather to rank 0.
//
// Everything between the collectives stays on the device; each exchange reads
// its send and receive sizes on the host once (the all_to_allv needs them), as
// do the threshold phase (capped-any + overflow need) and the size phase.
// The transport is a pair of callbacks (rsa_transport); RCCL is resolved at
// run time (dlopen/dlsym) so the library loads and runs single-GPU without it.

#include <dlfcn.h>
#include <rccl/rccl.h>   // types and enum values only: the functions come from dlsym

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

#include "rsa_internal.h"

namespace {

constexpr uint64_t kRec = sizeof(rsa_conn_record);   // 40 B rows on the wire
constexpr int kWorldMax = 256;                       // rsa_export_routed's limit
constexpr int64_t kNoThresh = -1;                    // 0xFFFF_FFFF_FFFF_FFFF as int64

int mfail(rsa_ctx* c, int code, const char* fmt, ...) {
  char buf[400];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  return rsa_internal_fail(c, code, buf);
}

#define MHIP(ctx, expr)                                                                              \
  do {                                                                                               \
    hipError_t e_ = (expr);                                                                          \
    if (e_ != hipSuccess) return mfail((ctx), RSA_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

// ---- device helpers (all tiny: vectors of n_rules or world entries) --------

// send[2r] = counts[r], send[2r+1] = flag: the per-owner counts with this
// rank's overflow flag riding along
__global__ void k_pack_counts(const unsigned long long* __restrict__ counts, uint32_t world, long long flag,
                              long long* __restrict__ send) {
  const uint32_t r = threadIdx.x;
  if (r < world) {
    send[2 * r] = (long long)counts[r];
    send[2 * r + 1] = flag;
  }
}

// out[i] = thresh[i] for the owned rules (gid % world == rank), -1 for the
// others; out[n] = need (the import overflow need, MAX-reduced with the rest)
__global__ void k_owned_thresh(const unsigned long long* __restrict__ thresh, uint32_t n, uint32_t world,
                               uint32_t rank, long long need, long long* __restrict__ out) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += gridDim.x * blockDim.x)
    out[i] = i == n ? need : (i % world == rank ? (long long)thresh[i] : kNoThresh);
}

// the merged thresholds back into d_thresh; any[0] = 1 if some rule is capped
__global__ void k_thresh_back(const long long* __restrict__ in, uint32_t n, unsigned long long* __restrict__ thresh,
                              unsigned int* __restrict__ any) {
  bool capped = false;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    thresh[i] = (unsigned long long)in[i];
    capped |= in[i] != kNoThresh;
  }
  if (capped) any[0] = 1u;   // a plain store of the same value from any lane
}

// out[i] = distinct[i] of the owned rules, 0 else; out[n + r] = 0 except this
// rank's row count at out[n + rank]
__global__ void k_owned_distinct(const unsigned int* __restrict__ distinct, uint32_t n, uint32_t world, uint32_t rank,
                                 long long rows, long long* __restrict__ out) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n + world; i += gridDim.x * blockDim.x)
    out[i] = i < n ? (i % world == rank ? (long long)distinct[i] : 0) : (i - n == rank ? rows : 0);
}

__global__ void k_distinct_back(const long long* __restrict__ in, uint32_t n, unsigned int* __restrict__ distinct) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    distinct[i] = (unsigned int)in[i];
}

uint32_t grid_of(uint64_t n) { return (uint32_t)std::min<uint64_t>((n + 255) / 256 + 1, 1024); }

// ---- per-ctx state -----------------------------------------------------------

struct DevBuf {
  void* p = nullptr;
  uint64_t bytes = 0;
};

struct State {
  DevBuf route, recv, emit, gather, vec, counts, csend, crecv, any;
  void* host = nullptr;           // pinned staging (small vectors, and host-buffer transports)
  uint64_t host_bytes = 0;
  uint64_t route_rows = 0;        // the rows the next routed export starts with (the last merge's need)
  uint64_t cur_rows = 0;          // the rows the current export may write
  uint64_t emit_rows = 0;
  // the last merge's owner rows and every rank's row count (for rsa_gather)
  bool have_part = false, forced = false;
  uint64_t part_rows = 0, gathered_rows = 0;
  bool have_gather = false;
  std::vector<uint64_t> sizes;
  int32_t part_world = 0, part_rank = 0;
};

State& state(rsa_ctx* c) {
  void** slot = rsa_internal_merge_slot(c);
  if (!*slot) *slot = new State();
  return *static_cast<State*>(*slot);
}

int grow(rsa_ctx* c, DevBuf& b, uint64_t bytes) {
  if (b.bytes >= bytes) return RSA_OK;
  MHIP(c, hipStreamSynchronize(rsa_internal_stream(c)));
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
  const uint64_t want = std::max<uint64_t>(bytes + bytes / 8, 256);
  MHIP(c, hipMalloc(&b.p, want));
  b.bytes = want;
  return RSA_OK;
}

int grow_host(rsa_ctx* c, State& S, uint64_t bytes) {
  if (S.host_bytes >= bytes) return RSA_OK;
  MHIP(c, hipStreamSynchronize(rsa_internal_stream(c)));
  if (S.host) (void)hipHostFree(S.host);
  S.host = nullptr;
  S.host_bytes = 0;
  const uint64_t want = std::max<uint64_t>(bytes + bytes / 8, 4096);
  MHIP(c, hipHostMalloc(&S.host, want, hipHostMallocDefault));
  S.host_bytes = want;
  return RSA_OK;
}

// ---- the transport, with host staging when the callbacks want host buffers --

struct Xport {
  rsa_ctx* c;
  const rsa_transport* t;
  State& S;
  hipStream_t s;
  uint64_t* allreduce_bytes;

  int all_reduce(long long* d, uint64_t n, int op) {
    *allreduce_bytes += 8 * n;
    if (!t->host_buffers) {
      if (t->all_reduce_i64(t->self, reinterpret_cast<int64_t*>(d), n, op, s))
        return mfail(c, RSA_ERR_HIP, "transport all_reduce failed (rank %d)", t->rank);
      return RSA_OK;
    }
    int rc = grow_host(c, S, 8 * n);
    if (rc) return rc;
    MHIP(c, hipMemcpyAsync(S.host, d, 8 * n, hipMemcpyDeviceToHost, s));
    MHIP(c, hipStreamSynchronize(s));
    if (t->all_reduce_i64(t->self, static_cast<int64_t*>(S.host), n, op, s))
      return mfail(c, RSA_ERR_HIP, "transport all_reduce failed (rank %d)", t->rank);
    MHIP(c, hipMemcpyAsync(d, S.host, 8 * n, hipMemcpyHostToDevice, s));
    return RSA_OK;
  }

  int all_to_allv(const void* d_send, const uint64_t* sb, void* d_recv, const uint64_t* rb) {
    const int w = t->world;
    if (!t->host_buffers) {
      if (t->all_to_allv(t->self, d_send, sb, d_recv, rb, s))
        return mfail(c, RSA_ERR_HIP, "transport all_to_allv failed (rank %d)", t->rank);
      return RSA_OK;
    }
    uint64_t st = 0, rt = 0;
    for (int r = 0; r < w; ++r) st += sb[r], rt += rb[r];
    // one pinned block: [send | recv]
    int rc = grow_host(c, S, st + rt + 64);
    if (rc) return rc;
    uint8_t* hs = static_cast<uint8_t*>(S.host);
    uint8_t* hr = hs + ((st + 63) & ~63ull);
    if (st) MHIP(c, hipMemcpyAsync(hs, d_send, st, hipMemcpyDeviceToHost, s));
    MHIP(c, hipStreamSynchronize(s));
    if (t->all_to_allv(t->self, hs, sb, hr, rb, s))
      return mfail(c, RSA_ERR_HIP, "transport all_to_allv failed (rank %d)", t->rank);
    if (rt) MHIP(c, hipMemcpyAsync(d_recv, hr, rt, hipMemcpyHostToDevice, s));
    MHIP(c, hipStreamSynchronize(s));   // the pinned block is reused by the next call
    return RSA_OK;
  }
};

struct OwnerGuard {   // RSA_OPT_OWNER_WORLD/RANK back to 0 however the merge ends
  rsa_ctx* c;
  ~OwnerGuard() {
    rsa_set_option(c, RSA_OPT_OWNER_WORLD, 0);
    rsa_set_option(c, RSA_OPT_OWNER_RANK, 0);
  }
};

// The routed export of `which` (0/1/2) into S.route, with its per-owner device
// counts in S.counts; a too-small buffer is handled by the caller (route).
int export_routed(rsa_ctx* c, State& S, int which, uint32_t world, uint64_t rows) {
  rows = std::max<uint64_t>(rows, 1);
  int rc = grow(c, S.route, rows * kRec);
  if (rc) return rc;
  S.cur_rows = rows;
  rc = grow(c, S.counts, world * 8);
  if (rc) return rc;
  return rsa_export_routed(c, which, world, static_cast<rsa_conn_record*>(S.route.p), rows,
                           static_cast<uint64_t*>(S.counts.p));
}

// the rows a routed export starts with: RSA_OPT_ROUTE_ROWS, else what the
// last exports needed (first merge: the table size)
int start_rows(rsa_ctx* c, State& S, uint64_t* rows) {
  const uint64_t opt = rsa_internal_route_rows(c);
  if (opt) {
    *rows = opt;
    return RSA_OK;
  }
  if (!S.route_rows) {
    uint64_t ts = 0;
    int rc = rsa_table_size(c, &ts);
    if (rc) return rc;
    S.route_rows = std::max<uint64_t>(ts, 1);
  }
  *rows = S.route_rows;
  return RSA_OK;
}

// One exchange of the routed export in S.route/S.counts: counts (+ flag)
// all_to_allv, one host read of the sizes, rows all_to_allv into S.recv.
// Returns RSA_OK with *n_recv rows received, or RSA_ERR_CAPACITY on every rank
// when any rank's flag is set.
int route(Xport& X, int which, uint32_t world, uint32_t rank, long long flag, uint64_t* n_recv, uint64_t* sent,
          uint64_t* self, uint64_t* recv_other, uint32_t* reexports) {
  rsa_ctx* c = X.c;
  State& S = X.S;
  int rc = grow(c, S.csend, 16 * world);
  if (!rc) rc = grow(c, S.crecv, 16 * world);
  if (rc) return rc;
  k_pack_counts<<<1, kWorldMax, 0, X.s>>>(static_cast<const unsigned long long*>(S.counts.p), world, flag,
                                          static_cast<long long*>(S.csend.p));
  MHIP(c, hipGetLastError());
  std::vector<uint64_t> b16(world, 16);
  rc = X.all_to_allv(S.csend.p, b16.data(), S.crecv.p, b16.data());
  if (rc) return rc;
  rc = grow_host(c, S, 24 * world);
  if (rc) return rc;
  int64_t* h = static_cast<int64_t*>(S.host);   // [counts world | recv 2*world]
  MHIP(c, hipMemcpyAsync(h, S.counts.p, 8 * world, hipMemcpyDeviceToHost, X.s));
  MHIP(c, hipMemcpyAsync(h + world, S.crecv.p, 16 * world, hipMemcpyDeviceToHost, X.s));
  MHIP(c, hipStreamSynchronize(X.s));
  std::vector<uint64_t> sb(world), rb(world);
  bool any_flag = false;
  uint64_t total = 0, rtot = 0;
  for (uint32_t r = 0; r < world; ++r) {
    any_flag |= h[world + 2 * r + 1] != 0;
    sb[r] = (uint64_t)h[r];
    rb[r] = (uint64_t)h[world + 2 * r];
    total += sb[r];
    rtot += rb[r];
  }
  if (any_flag) return mfail(c, RSA_ERR_CAPACITY, "distinct-connection table overflow on at least one rank");
  if (total > S.cur_rows) {   // the export dropped rows past its buffer: again at the exact size
    rc = export_routed(c, S, which, world, total);
    if (rc) return rc;
    ++*reexports;
  }
  S.route_rows = std::max(S.route_rows, total);
  *sent = total - sb[rank];
  *self = sb[rank];
  *recv_other = rtot - rb[rank];
  for (uint32_t r = 0; r < world; ++r) sb[r] *= kRec, rb[r] *= kRec;
  rc = grow(c, S.recv, std::max<uint64_t>(rtot, 1) * kRec);
  if (rc) return rc;
  rc = X.all_to_allv(S.route.p, sb.data(), S.recv.p, rb.data());
  if (rc) return rc;
  *n_recv = rtot;
  return RSA_OK;
}

// rsa_emit into S.emit, grown to the table size when it does not fit.
int emit_final(rsa_ctx* c, State& S, uint64_t* rows) {
  if (!S.emit_rows) {
    uint64_t n = 0;
    int rc = rsa_table_size(c, &n);
    if (rc) return rc;
    S.emit_rows = std::max<uint64_t>(n, 1);
  }
  for (int attempt = 0; attempt < 2; ++attempt) {
    int rc = grow(c, S.emit, S.emit_rows * kRec);
    if (rc) return rc;
    S.emit_rows = S.emit.bytes / kRec;
    uint64_t n = 0;
    rc = rsa_emit(c, static_cast<rsa_conn_record*>(S.emit.p), S.emit_rows, &n);
    if (rc == RSA_OK) {
      *rows = n;
      return RSA_OK;
    }
    if (rc != RSA_ERR_CAPACITY || attempt) return rc;
    uint64_t ts = 0;
    rc = rsa_table_size(c, &ts);
    if (rc) return rc;
    S.emit_rows = std::max(n, ts);
  }
  return mfail(c, RSA_ERR_STATE, "emit did not fit");
}

int check_transport(rsa_ctx* c, const rsa_transport* t) {
  if (!t) return mfail(c, RSA_ERR_ARG, "null transport");
  if (t->world < 1 || t->world > kWorldMax || t->rank < 0 || t->rank >= t->world)
    return mfail(c, RSA_ERR_ARG, "transport world %d / rank %d out of range (world 1..%d)", t->world, t->rank,
                 kWorldMax);
  return RSA_OK;
}

int gather_rows(rsa_ctx* c, const rsa_transport* t, rsa_merge_info* info) {
  State& S = state(c);
  if (!S.have_part) return mfail(c, RSA_ERR_STATE, "no merge to gather (rsa_merge first)");
  if (S.part_world != t->world || S.part_rank != t->rank)
    return mfail(c, RSA_ERR_ARG, "the transport's world/rank differ from the merge's");
  const uint32_t world = (uint32_t)t->world, rank = (uint32_t)t->rank;
  S.have_gather = false;
  if (world == 1 && !S.forced) {
    info->d_rows = static_cast<const rsa_conn_record*>(S.emit.p);
    info->n_rows = S.gathered_rows = S.part_rows;
    S.have_gather = true;
    return RSA_OK;
  }
  uint64_t total = 0;
  for (uint64_t v : S.sizes) total += v;
  std::vector<uint64_t> sb(world, 0), rb(world, 0);
  sb[0] = S.part_rows * kRec;
  if (rank == 0)
    for (uint32_t r = 0; r < world; ++r) rb[r] = S.sizes[r] * kRec;
  int rc = grow(c, S.gather, (rank == 0 ? std::max<uint64_t>(total, 1) : 1) * kRec);
  if (rc) return rc;
  uint64_t dummy = 0;
  Xport X{c, t, S, rsa_internal_stream(c), &dummy};
  rc = X.all_to_allv(S.emit.p, sb.data(), S.gather.p, rb.data());
  if (rc) return rc;
  info->d_rows = rank == 0 ? static_cast<const rsa_conn_record*>(S.gather.p) : nullptr;
  info->n_rows = S.gathered_rows = rank == 0 ? total : 0;
  S.have_gather = true;
  return RSA_OK;
}

}  // namespace

extern "C" {

void rsa_internal_merge_free(void* p) {
  State* S = static_cast<State*>(p);
  for (DevBuf* b : {&S->route, &S->recv, &S->emit, &S->gather, &S->vec, &S->counts, &S->csend, &S->crecv, &S->any})
    if (b->p) (void)hipFree(b->p);
  if (S->host) (void)hipHostFree(S->host);
  delete S;
}

int rsa_merge(rsa_ctx* c, const rsa_transport* t, const rsa_shard_batch* h_batches, uint32_t n_batches, int flags,
              rsa_merge_info* info) {
  if (!c || !info) return RSA_ERR_ARG;
  int rc = check_transport(c, t);
  if (rc) return rc;
  if (n_batches && !h_batches) return mfail(c, RSA_ERR_ARG, "null batches");
  memset(info, 0, sizeof *info);
  unsigned long long *d_m, *d_h, *d_t;
  unsigned int* d_d;
  uint32_t n;
  rsa_internal_counters(c, &d_m, &d_h, &d_d, &d_t, &n);
  if (!d_m) return mfail(c, RSA_ERR_STATE, "counters not bound (rsa_bind_counters)");
  MHIP(c, hipSetDevice(rsa_internal_device(c)));
  State& S = state(c);
  S.have_part = S.have_gather = false;
  if (flags & ~(RSA_MERGE_GATHER | RSA_MERGE_ALWAYS_EXCHANGE)) return mfail(c, RSA_ERR_ARG, "unknown merge flags %d", flags);
  const uint32_t world = (uint32_t)t->world, rank = (uint32_t)t->rank;
  const bool multi = world > 1 || (flags & RSA_MERGE_ALWAYS_EXCHANGE);
  if (multi && (!t->all_reduce_i64 || !t->all_to_allv)) return mfail(c, RSA_ERR_ARG, "transport callbacks missing");
  hipStream_t s = rsa_internal_stream(c);
  Xport X{c, t, S, s, &info->allreduce_bytes};
  const uint64_t nv = (uint64_t)n + world + 2;   // the longest vector: distinct + sizes
  if ((rc = grow(c, S.vec, 8 * std::max<uint64_t>(2ull * n, nv)))) return rc;
  if ((rc = grow(c, S.any, 8))) return rc;
  long long* vec = static_cast<long long*>(S.vec.p);

  // 1. line and hit counters: one SUM all_reduce
  if (multi) {
    MHIP(c, hipMemcpyAsync(vec, d_m, 8ull * n, hipMemcpyDeviceToDevice, s));
    MHIP(c, hipMemcpyAsync(vec + n, d_h, 8ull * n, hipMemcpyDeviceToDevice, s));
    if ((rc = X.all_reduce(vec, 2ull * n, 0))) return rc;
    MHIP(c, hipMemcpyAsync(d_m, vec, 8ull * n, hipMemcpyDeviceToDevice, s));
    MHIP(c, hipMemcpyAsync(d_h, vec + n, 8ull * n, hipMemcpyDeviceToDevice, s));
  }
  if ((rc = rsa_set_option(c, RSA_OPT_OWNER_WORLD, world))) return rc;
  OwnerGuard guard{c};
  if ((rc = rsa_set_option(c, RSA_OPT_OWNER_RANK, rank))) return rc;

  // 2. this shard's cap resolution and the routed export of what others own
  long long failed = 0;
  uint32_t n_capped = 0;
  rc = rsa_resolve_cap(c, &n_capped);
  if (rc == RSA_OK && multi) {
    uint64_t rows = 0;
    if ((rc = start_rows(c, S, &rows))) return rc;
    rc = export_routed(c, S, 2, world, rows);
  }
  if (rc == RSA_ERR_CAPACITY) {
    failed = 1;
    if (multi) {
      if ((rc = grow(c, S.counts, world * 8))) return rc;
      MHIP(c, hipMemsetAsync(S.counts.p, 0, world * 8, s));
    }
  } else if (rc) {
    return rc;
  }
  bool capped_any = n_capped > 0;
  if (multi) {
    uint64_t n_recv = 0;
    rc = route(X, 2, world, rank, failed, &n_recv, &info->route1_sent, &info->route1_self, &info->route1_recv,
               &info->reexports);
    if (rc) return rc;
    long long need = 0;
    if (n_recv) {
      // the received entries join the owned ones: the owned rules' thresholds
      // are resolved again over the merged entries
      rc = rsa_import(c, 0, static_cast<const rsa_conn_record*>(S.recv.p), n_recv);
      if (rc == RSA_OK) rc = rsa_resolve_cap(c, &n_capped);
      if (rc == RSA_ERR_CAPACITY) {
        uint64_t ts = 0;
        (void)rsa_table_size(c, &ts);
        need = (long long)std::max<uint64_t>(ts + n_recv, 1);   // the shard's entries and every received one
      } else if (rc) {
        return rc;
      }
    }
    // 3. the owners' thresholds (MAX; the others say "none" = -1) with the need
    k_owned_thresh<<<grid_of(n + 1), 256, 0, s>>>(d_t, n, world, rank, need, vec);
    MHIP(c, hipGetLastError());
    if ((rc = X.all_reduce(vec, (uint64_t)n + 1, 1))) return rc;
    MHIP(c, hipMemsetAsync(S.any.p, 0, 8, s));
    k_thresh_back<<<grid_of(n), 256, 0, s>>>(vec, n, d_t, static_cast<unsigned int*>(S.any.p));
    MHIP(c, hipGetLastError());
    int64_t* h = static_cast<int64_t*>(S.host);
    MHIP(c, hipMemcpyAsync(h, vec + n, 8, hipMemcpyDeviceToHost, s));
    MHIP(c, hipMemcpyAsync(h + 1, S.any.p, 8, hipMemcpyDeviceToHost, s));
    MHIP(c, hipStreamSynchronize(s));
    if (h[0]) {
      info->needed = (uint64_t)h[0];
      return mfail(c, RSA_ERR_CAPACITY, "distinct-connection table overflow on at least one rank (merge import)");
    }
    capped_any = (h[1] & 0xFFFFFFFFll) != 0;
  } else if (failed) {
    return mfail(c, RSA_ERR_CAPACITY, "distinct-connection table overflow");
  }

  // 4. the pass-2 recount of the capped rules and its exchange
  if (capped_any) {
    info->pass2 = 1;
    for (uint32_t b = 0; b < n_batches; ++b) {
      const rsa_shard_batch& B = h_batches[b];
      if ((rc = rsa_recount(c, B.d_tuples, B.d_ts, B.d_order, B.d_gid, B.n))) return rc;
    }
    if (multi) {
      uint64_t rows = 0;
      if ((rc = start_rows(c, S, &rows))) return rc;
      if ((rc = export_routed(c, S, 1, world, rows))) return rc;
      uint64_t n_recv = 0;
      rc = route(X, 1, world, rank, 0, &n_recv, &info->route2_sent, &info->route2_self, &info->route2_recv,
                 &info->reexports);
      if (rc) return rc;
      if (n_recv && (rc = rsa_import(c, 1, static_cast<const rsa_conn_record*>(S.recv.p), n_recv))) return rc;
    }
  }

  // 5. the owners' final rows, the owned distinct counts and every rank's size
  uint64_t rows = 0;
  if ((rc = emit_final(c, S, &rows))) return rc;
  S.sizes.assign(world, 0);
  S.sizes[rank] = rows;
  if (multi) {
    k_owned_distinct<<<grid_of((uint64_t)n + world), 256, 0, s>>>(d_d, n, world, rank, (long long)rows, vec);
    MHIP(c, hipGetLastError());
    if ((rc = X.all_reduce(vec, (uint64_t)n + world, 0))) return rc;
    k_distinct_back<<<grid_of(n), 256, 0, s>>>(vec, n, d_d);
    MHIP(c, hipGetLastError());
    if ((rc = grow_host(c, S, 8ull * world))) return rc;
    int64_t* h = static_cast<int64_t*>(S.host);
    MHIP(c, hipMemcpyAsync(h, vec + n, 8ull * world, hipMemcpyDeviceToHost, s));
    MHIP(c, hipStreamSynchronize(s));
    for (uint32_t r = 0; r < world; ++r) S.sizes[r] = (uint64_t)h[r];
  }
  S.have_part = true;
  S.part_rows = rows;
  S.part_world = (int32_t)world;
  S.part_rank = (int32_t)rank;
  S.forced = multi && world == 1;
  info->owner_rows = rows;
  for (uint32_t r = 1; r < world; ++r) info->gather_rows += S.sizes[r];
  info->d_rows = static_cast<const rsa_conn_record*>(S.emit.p);
  info->n_rows = rows;
  if (flags & RSA_MERGE_GATHER) return gather_rows(c, t, info);
  return RSA_OK;
}

int rsa_merge_rows(rsa_ctx* c, int which, rsa_conn_record* d_out, uint64_t max_records, uint64_t* h_n) {
  if (!c || !h_n) return RSA_ERR_ARG;
  if (which != 0 && which != 1) return mfail(c, RSA_ERR_ARG, "which must be 0 or 1");
  State& S = state(c);
  if (which == 0 ? !S.have_part : !S.have_gather)
    return mfail(c, RSA_ERR_STATE, which == 0 ? "no merge (rsa_merge first)" : "no gather (rsa_gather first)");
  const uint64_t n = which == 0 ? S.part_rows : S.gathered_rows;
  *h_n = n;
  if (n > max_records) return mfail(c, RSA_ERR_CAPACITY, "%llu rows do not fit in %llu", (unsigned long long)n,
                                    (unsigned long long)max_records);
  if (!n) return RSA_OK;
  if (!d_out) return mfail(c, RSA_ERR_ARG, "null output buffer");
  MHIP(c, hipSetDevice(rsa_internal_device(c)));
  const void* src = which == 0 || (S.part_world == 1 && !S.forced) ? S.emit.p : S.gather.p;
  MHIP(c, hipMemcpyAsync(d_out, src, n * kRec, hipMemcpyDeviceToDevice, rsa_internal_stream(c)));
  return RSA_OK;
}

int rsa_gather(rsa_ctx* c, const rsa_transport* t, rsa_merge_info* info) {
  if (!c || !info) return RSA_ERR_ARG;
  int rc = check_transport(c, t);
  if (rc) return rc;
  MHIP(c, hipSetDevice(rsa_internal_device(c)));
  return gather_rows(c, t, info);
}

}  // extern "C"

// ---- RCCL -------------------------------------------------------------------

namespace {

struct Rccl {
  bool ok = false;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclCommCount) count = nullptr;
  decltype(&ncclCommUserRank) user_rank = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};

// The process's RCCL: the one already loaded (e.g. by the framework that owns
// the process group), else librccl.so.1 from the library path.
const Rccl& rccl() {
  static Rccl R;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen(nullptr, RTLD_NOW);
    if (!h || !dlsym(h, "ncclCommInitRank")) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h || !dlsym(h, "ncclCommInitRank")) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
#define RSYM(field, name) R.field = reinterpret_cast<decltype(R.field)>(dlsym(h, name))
    RSYM(get_unique_id, "ncclGetUniqueId");
    RSYM(init_rank, "ncclCommInitRank");
    RSYM(destroy, "ncclCommDestroy");
    RSYM(count, "ncclCommCount");
    RSYM(user_rank, "ncclCommUserRank");
    RSYM(all_reduce, "ncclAllReduce");
    RSYM(send, "ncclSend");
    RSYM(recv, "ncclRecv");
    RSYM(group_start, "ncclGroupStart");
    RSYM(group_end, "ncclGroupEnd");
    RSYM(error_string, "ncclGetErrorString");
#undef RSYM
    R.ok = R.get_unique_id && R.init_rank && R.destroy && R.count && R.user_rank && R.all_reduce && R.send &&
           R.recv && R.group_start && R.group_end && R.error_string;
  });
  return R;
}

int rccl_all_reduce(void* self, int64_t* buf, uint64_t n, int op, void* stream) {
  const Rccl& R = rccl();
  return R.all_reduce(buf, buf, n, ncclInt64, op ? ncclMax : ncclSum, static_cast<ncclComm_t>(self),
                      static_cast<hipStream_t>(stream)) != ncclSuccess;
}

// grouped point-to-point: one send and one receive per peer with bytes to move
// (self included: RCCL copies it); peers with nothing to move are skipped
int rccl_all_to_allv(void* self, const void* send, const uint64_t* sb, void* recv, const uint64_t* rb, void* stream) {
  const Rccl& R = rccl();
  ncclComm_t comm = static_cast<ncclComm_t>(self);
  hipStream_t s = static_cast<hipStream_t>(stream);
  int world = 0;
  if (R.count(comm, &world) != ncclSuccess) return 1;
  if (R.group_start() != ncclSuccess) return 1;
  uint64_t so = 0, ro = 0;
  int bad = 0;
  for (int r = 0; r < world; ++r) {
    if (sb[r]) bad |= R.send(static_cast<const uint8_t*>(send) + so, sb[r], ncclUint8, r, comm, s) != ncclSuccess;
    if (rb[r]) bad |= R.recv(static_cast<uint8_t*>(recv) + ro, rb[r], ncclUint8, r, comm, s) != ncclSuccess;
    so += sb[r];
    ro += rb[r];
  }
  bad |= R.group_end() != ncclSuccess;
  return bad;
}

int rccl_transport(rsa_ctx* c, void* comm, rsa_transport* t) {
  const Rccl& R = rccl();
  if (!R.ok) return mfail(c, RSA_ERR_STATE, "RCCL not found (librccl.so.1)");
  if (!comm) return mfail(c, RSA_ERR_ARG, "null communicator");
  int world = 0, rank = 0;
  if (R.count(static_cast<ncclComm_t>(comm), &world) != ncclSuccess ||
      R.user_rank(static_cast<ncclComm_t>(comm), &rank) != ncclSuccess)
    return mfail(c, RSA_ERR_ARG, "not an RCCL communicator");
  *t = rsa_transport{comm, world, rank, 0, rccl_all_reduce, rccl_all_to_allv};
  return RSA_OK;
}

}  // namespace

extern "C" {

int rsa_rccl_unique_id(uint8_t h_id[128]) {
  const Rccl& R = rccl();
  if (!h_id) return RSA_ERR_ARG;
  if (!R.ok) return RSA_ERR_STATE;
  ncclUniqueId id;
  if (R.get_unique_id(&id) != ncclSuccess) return RSA_ERR_HIP;
  static_assert(sizeof id == 128, "unique id size");
  memcpy(h_id, &id, sizeof id);
  return RSA_OK;
}

int rsa_rccl_comm_create(rsa_ctx* c, int32_t world, int32_t rank, const uint8_t h_id[128], void** comm) {
  if (!c || !h_id || !comm) return RSA_ERR_ARG;
  const Rccl& R = rccl();
  if (!R.ok) return mfail(c, RSA_ERR_STATE, "RCCL not found (librccl.so.1)");
  if (world < 1 || rank < 0 || rank >= world) return mfail(c, RSA_ERR_ARG, "world %d / rank %d", world, rank);
  MHIP(c, hipSetDevice(rsa_internal_device(c)));
  ncclUniqueId id;
  memcpy(&id, h_id, sizeof id);
  ncclComm_t cm = nullptr;
  const ncclResult_t r = R.init_rank(&cm, world, id, rank);
  if (r != ncclSuccess) return mfail(c, RSA_ERR_HIP, "ncclCommInitRank: %s", R.error_string(r));
  *comm = cm;
  return RSA_OK;
}

int rsa_rccl_comm_destroy(void* comm) {
  const Rccl& R = rccl();
  if (!comm) return RSA_OK;
  if (!R.ok) return RSA_ERR_STATE;
  return R.destroy(static_cast<ncclComm_t>(comm)) == ncclSuccess ? RSA_OK : RSA_ERR_HIP;
}

int rsa_merge_rccl(rsa_ctx* c, void* comm, const rsa_shard_batch* h_batches, uint32_t n_batches, int flags,
                   rsa_merge_info* h_info) {
  if (!c) return RSA_ERR_ARG;
  rsa_transport t;
  int rc = rccl_transport(c, comm, &t);
  if (rc) return rc;
  return rsa_merge(c, &t, h_batches, n_batches, flags, h_info);
}

int rsa_gather_rccl(rsa_ctx* c, void* comm, rsa_merge_info* h_info) {
  if (!c) return RSA_ERR_ARG;
  rsa_transport t;
  int rc = rccl_transport(c, comm, &t);
  if (rc) return rc;
  return rsa_gather(c, &t, h_info);
}

}  // extern "C"
