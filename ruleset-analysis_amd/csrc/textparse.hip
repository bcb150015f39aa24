// textparse.hip — device parse of firewall log text for MI355X (gfx950):
// SURVEY.md §8f row 1, the step before the hot path.  Text of one firewall
// sits in HBM; the kernels here produce what rsa_classify consumes.
//
//   k_nl_count / k_nl_offsets line split: '\n' bytes counted per 64-KiB block
//                             (16-B loads, exact zero-byte test); the line
//                             starts in one pass (decoupled look-back over the
//                             block counts, bytes held in registers);
//   k_parse                   one lane per line: the mapper's message parse
//                             (get_builtconn, mapper.py:124-142 — restated by
//                             logparse._GB), the ACL of the
//                             ingress interface and its candidate list
//                             (mapper.py:145-166), and the reducer's facts for
//                             the same line (connlist-reducer.py:146-165): hit
//                             test, BUILT regex with Python `re`'s backtracking
//                             order, key (SWAP or not), timestamp code;
//   order keys                the rank of each line's bytes (LC_ALL=C sort of
//                             the mapper stream, runAnalysis.sh:42-56): 7-byte
//                             big-endian chunks + a length field, groups of
//                             equal prefixes refined by stable LSD radix sorts
//                             (k_rs_*, hand-written) over the key bits that
//                             vary; classes of <= 64 lines ranked directly
//                             by string comparison (k_finish_small).
//
// Anything outside the canonical grammar is marked RSA_LINE_HOST: the host
// parser (logparse._parse_one) decides those lines, so every error the
// reference raises is raised by the same code and message.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <string>


#include "../../include/ruleset_hip.h"
#include "rsa_internal.h"
#include "textparse_line.h"

namespace {

#define TPCHK(c, expr)                                                            \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess) {                                                       \
      const std::string m_ = std::string(#expr ": ") + hipGetErrorString(e_);     \
      return rsa_internal_fail((c), RSA_ERR_HIP, m_.c_str());                     \
    }                                                                             \
  } while (0)

// ---------------------------------------------------------------------------
// Line split
constexpr uint32_t kSplitThreads = 1024, kSplitPer = 64;
constexpr uint64_t kSplitBlock = (uint64_t)kSplitThreads * kSplitPer;   // 64 KiB per workgroup

// high bit of every byte of w that equals '\n' (exact: no borrow between bytes)
__device__ __forceinline__ uint32_t nl_bits(uint32_t w) {
  const uint32_t x = w ^ 0x0A0A0A0Au;
  const uint32_t t = (x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
  return ~(t | x | 0x7F7F7F7Fu);
}

// '\n' count of this thread's 64 bytes [a, a + 64) clipped to n
__device__ __forceinline__ uint32_t seg_count(const uint8_t* __restrict__ text, uint64_t a, uint64_t n, bool aligned) {
  uint32_t cnt = 0;
  if (aligned && a + kSplitPer <= n) {
    const uint4* q = reinterpret_cast<const uint4*>(text + a);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint4 v = q[k];
      cnt += __popc(nl_bits(v.x)) + __popc(nl_bits(v.y)) + __popc(nl_bits(v.z)) + __popc(nl_bits(v.w));
    }
  } else {
    for (uint64_t i = a; i < a + kSplitPer && i < n; ++i) cnt += text[i] == '\n';
  }
  return cnt;
}

// exclusive scan over the 1024 threads of a block; *total = block sum
__device__ uint32_t block_exscan(uint32_t v, uint32_t* sh, uint32_t* total) {
  const uint32_t lane = __lane_id(), wave = threadIdx.x / 64;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) sh[wave] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (uint32_t w = 0; w < blockDim.x / 64; ++w) {
      const uint32_t t = sh[w];
      sh[w] = acc;
      acc += t;
    }
    sh[16] = acc;
  }
  __syncthreads();
  *total = sh[16];
  return sh[wave] + x - v;
}

__global__ __launch_bounds__(kSplitThreads) void k_nl_count(const uint8_t* __restrict__ text, uint64_t n, int aligned,
                                                             uint32_t* __restrict__ counts) {
  __shared__ uint32_t sh[17];
  const uint64_t a = (uint64_t)blockIdx.x * kSplitBlock + (uint64_t)threadIdx.x * kSplitPer;
  uint32_t total;
  block_exscan(seg_count(text, a, n, aligned != 0), sh, &total);
  if (threadIdx.x == 0) counts[blockIdx.x] = total;
}

// Line starts in one pass (decoupled look-back): workgroups take the 64-KiB
// blocks in launch order (an atomic ticket, so a block only ever waits on
// blocks already running), count their '\n's with their bytes held in
// registers, publish the count, add the predecessors' counts walking back to
// the first published inclusive prefix, publish their own inclusive prefix,
// and write the line starts from the registers: the text is read once.
constexpr unsigned long long kLbAgg = 1ull << 62, kLbIncl = 1ull << 63, kLbVal = kLbAgg - 1;
constexpr uint32_t kLbSpinMax = 1u << 26;   // a wait this long is a bug: flagged, never a hang
__global__ __launch_bounds__(kSplitThreads) void k_nl_offsets(const uint8_t* __restrict__ text, uint64_t n, int aligned,
                                                               uint64_t* __restrict__ off, uint64_t n_lines,
                                                               unsigned long long* __restrict__ state,
                                                               unsigned int* __restrict__ ticket) {
  __shared__ uint32_t sh[17];
  __shared__ uint32_t sh_b;
  __shared__ unsigned long long sh_prefix;
  if (threadIdx.x == 0) sh_b = atomicAdd(&ticket[0], 1u);
  __syncthreads();
  const uint32_t b = sh_b;
  const uint64_t a = (uint64_t)b * kSplitBlock + (uint64_t)threadIdx.x * kSplitPer;
  const bool vec = aligned && a + kSplitPer <= n;
  uint32_t w[16];
  uint32_t mine = 0;
  if (vec) {
    const uint4* q = reinterpret_cast<const uint4*>(text + a);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint4 v = q[k];
      w[4 * k] = v.x;
      w[4 * k + 1] = v.y;
      w[4 * k + 2] = v.z;
      w[4 * k + 3] = v.w;
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) mine += __popc(nl_bits(w[k]));
  } else {
    for (uint64_t i = a; i < a + kSplitPer && i < n; ++i) mine += text[i] == '\n';
  }
  uint32_t total;
  const uint32_t excl = block_exscan(mine, sh, &total);
  if (threadIdx.x < 64) {
    // wave 0 looks back 64 blocks at a time: the nearest published inclusive
    // prefix among them and the aggregates after it; an unpublished block
    // after the last inclusive one means another look
    unsigned long long run = 0;
    const uint32_t lane = threadIdx.x;
    if (b == 0) {
      if (lane == 0) __hip_atomic_store(&state[0], kLbIncl | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0) __hip_atomic_store(&state[b], kLbAgg | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int64_t top = (int64_t)b - 1;   // the window is blocks (top - 63, top]
      uint32_t spins = 0;
      while (true) {
        const int64_t p = top - (int64_t)lane;
        const unsigned long long v =
            p >= 0 ? __hip_atomic_load(&state[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kLbIncl;
        // lanes in order of distance: the first inclusive one ends the walk
        const unsigned long long incl = __ballot((v & kLbIncl) != 0);
        const int stop = incl ? __builtin_ctzll(incl) : 64;   // lanes [0, stop) must be aggregates
        const unsigned long long ready = __ballot((v & (kLbIncl | kLbAgg)) != 0);
        const unsigned long long need = stop >= 64 ? ~0ull : ((2ull << stop) - 1ull);
        if ((ready & need) != need) {   // someone in the window not published yet: look again
          if (++spins > kLbSpinMax) {
            if (lane == 0) atomicOr(&ticket[1], 1u);
            break;
          }
          continue;
        }
        unsigned long long x = ((int)lane <= stop && p >= 0) ? (v & kLbVal) : 0ull;
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
        run += x;
        if (stop < 64) break;
        top -= 64;
      }
      if (lane == 0)
        __hip_atomic_store(&state[b], kLbIncl | (run + total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) sh_prefix = run;
  }
  __syncthreads();
  uint64_t k = sh_prefix + excl;
  if (!mine) return;
  if (vec) {
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      uint32_t bits = nl_bits(w[e]);
      while (bits) {
        const uint32_t byte = (uint32_t)__builtin_ctz(bits) >> 3;
        bits &= bits - 1;
        if (k + 1 <= n_lines) off[k + 1] = a + 4 * e + byte + 1;
        ++k;
      }
    }
    return;
  }
  for (uint64_t i = a; i < a + kSplitPer && i < n; ++i)
    if (text[i] == '\n') {
      if (k + 1 <= n_lines) off[k + 1] = i + 1;
      ++k;
    }
}

__global__ void k_set_u64(uint64_t* p, uint64_t v) { *p = v; }

// k_parse: a workgroup stages the text of its kParseWG lines in LDS with
// coalesced 4-byte loads, then every lane parses its line from LDS through
// the word-cached accessor (one LDS read per 4 bytes scanned).  A workgroup
// whose lines do not fit parses straight from HBM with byte loads.
// 28 KB of staged text + the scan's slots and tables: four workgroups per CU
// (a workgroup whose lines average more than 224 B defers them to the slow pass)
constexpr uint32_t kParseWG = 128, kStageBytes = 28672;
#ifndef RSA_TPL_PROF
#define RSA_TPL_PROF 0   // PROFILING builds only (results invalid): 1 template scan without tpl_finish, 2 no scan either
#endif

// A line the template pass defers (rsa_text::kLineDefer): its index is
// appended to the slow list (one device atomic per wave).
__device__ __forceinline__ void defer_append(bool defer, uint64_t i, uint32_t* __restrict__ slow_idx,
                                             unsigned int* __restrict__ slow_n) {
  const unsigned long long b = __ballot(defer);
  if (!b) return;
  const int leader = __builtin_ctzll(b);
  const uint32_t lane = __lane_id();
  uint32_t at = 0;
  if ((int)lane == leader) at = atomicAdd(slow_n, (unsigned int)__popcll(b));
  at = __builtin_amdgcn_readlane(at, leader);
  if (defer) slow_idx[at + (uint32_t)__popcll(b & ((1ull << lane) - 1ull))] = (uint32_t)i;
}

// kReduce: the reducer drop-in's lines (rsa_text::reduce_line, plus the
// same-key flag against the previous line of the batch).  The workgroup's
// lines are staged in LDS; the mapper form runs here only for text that is not
// 16-byte aligned (k_parse_win is the default).  Both parse the template form
// only (kDefer): other classified lines go to the slow list for k_parse_slow.
template <bool kReduce>
__global__ __launch_bounds__(kParseWG) void k_parse(const uint8_t* __restrict__ text, const uint64_t* __restrict__ off,
                                                    uint64_t n_lines, const rsa_parse_ifc* __restrict__ ifcs,
                                                    uint32_t n_ifcs, const rsa_parse_spell* __restrict__ spells,
                                                    uint32_t n_spells, rsa_tuple* __restrict__ tuples,
                                                    uint32_t* __restrict__ ts_out, uint32_t* __restrict__ disp,
                                                    uint32_t* __restrict__ slow_idx, unsigned int* __restrict__ slow_n) {
  __shared__ uint32_t sm[kStageBytes / 4 + 8];   // (+8: tpl_finish's 16-B field reads past a line)
  // the template scan (rsa_text::tpl) over the staged lines
  constexpr bool kScan = !kReduce;
  __shared__ uint32_t tprog[kScan ? rsa_text::tpl::kProgLen : 1];
  __shared__ uint8_t tcls[kScan ? 256 : 1];
  __shared__ uint32_t tslot[kScan ? kParseWG * rsa_text::tpl::kSlotWords : 1];
  if (kScan) {
    constexpr rsa_text::tpl::ClsTable kCls = rsa_text::tpl::cls_table();
    for (uint32_t k = threadIdx.x; k < rsa_text::tpl::kProgLen; k += blockDim.x) tprog[k] = rsa_text::tpl::kProg[k];
    for (uint32_t k = threadIdx.x; k < 256; k += blockDim.x) tcls[k] = kCls.t[k];
  }
  const uint64_t l0 = (uint64_t)blockIdx.x * kParseWG;
  const uint64_t l1 = l0 + kParseWG < n_lines ? l0 + kParseWG : n_lines;
  const uint64_t n_bytes = off[n_lines];
  const uint64_t base = off[l0] & ~3ull, span = off[l1] - base;
  const bool staged = span <= kStageBytes;   // workgroup-uniform
  if (staged) {
    const uint32_t nw = (uint32_t)((span + 3) / 4);
    const uint32_t* src = reinterpret_cast<const uint32_t*>(text + base);
    for (uint32_t w = threadIdx.x; w < nw; w += blockDim.x) {
      const uint64_t at = base + 4ull * w;
      uint32_t x;
      if (at + 4 <= n_bytes) {
        x = src[w];
      } else {
        x = 0;
        for (uint32_t k = 0; k < 4; ++k)
          if (at + k < n_bytes) x |= (uint32_t)text[at + k] << (8 * k);
      }
      sm[w] = x;
    }
  }
  __syncthreads();
  const uint64_t i = l0 + threadIdx.x;
  if (i >= l1) return;
  const uint64_t a = off[i], b = off[i + 1];
  uint64_t len = b - a;
  if (len && text[b - 1] == '\n') --len;
  rsa_tuple tup = {0u, 0u, 0, 0, 0, 0, 0};
  uint32_t ts = 0, d = rsa_text::kLineDefer;
  if (len < 0xFFFFFFFFull) {
    if (kReduce) {
      // the previous line: staged unless it is the workgroup's first line's predecessor
      const uint64_t pa = i ? off[i - 1] : 0;
      uint64_t plen = a - pa;
      if (plen && text[a - 1] == '\n') --plen;
      const bool pin = i > 0 && plen < 0xFFFFFFFFull;
      if (staged) {
        const rsa_text::WordLn s{sm, (uint32_t)(a - base), (uint32_t)len};
        rsa_text::reduce_line<true>(s, spells, n_spells, tup, ts, d);
        if (pin && d != RSA_RED_NOISE && d != rsa_text::kLineDefer) {
          bool same;
          if (i > l0) {
            const rsa_text::WordLn q{sm, (uint32_t)(pa - base), (uint32_t)plen};
            same = rsa_text::same_key(s, q);
          } else {
            const rsa_text::GWordLn q{reinterpret_cast<const uint32_t*>(text), text, pa, n_bytes, (uint32_t)plen, ~0ull,
                                      0u};
            same = rsa_text::same_key(s, q);
          }
          if (same) d |= RSA_RED_SAME_KEY;
        }
      } else {
        d = rsa_text::kLineDefer;   // lines too long to stage: the slow pass reads them from HBM
      }
    } else if (staged) {
      const rsa_text::WordLn s{sm, (uint32_t)(a - base), (uint32_t)len};
      uint32_t* slot = tslot + threadIdx.x * rsa_text::tpl::kSlotWords;
      if (RSA_TPL_PROF == 2) {
        d = RSA_LINE_NOACL + (s[len > 1 ? 1 : 0] == 0xFFu);
      } else if (RSA_TPL_PROF == 1) {
        d = RSA_LINE_NOACL + !rsa_text::tpl::scan(s, tprog, tcls, slot);
      } else if (!(rsa_text::tpl::scan(s, tprog, tcls, slot) &&
                   rsa_text::tpl_finish(s, slot, ifcs, n_ifcs, spells, n_spells, tup, ts, d))) {
        tup = rsa_tuple{0u, 0u, 0, 0, 0, 0, 0};
        ts = 0;
        d = rsa_text::kLineDefer;
      }
    } else {
      d = rsa_text::kLineDefer;
    }
  }
  defer_append(d == rsa_text::kLineDefer, i, slow_idx, slow_n);
  tuples[i] = tup;
  ts_out[i] = ts;
  disp[i] = d;
}

// k_parse_win: the template pass without staging.  Every lane reads its own
// line straight from HBM through a register window: two aligned 16-B chunks,
// funnel-shifted once per 16 bytes so that the line's next 16 bytes sit at
// fixed register positions (the shift is the line's start modulo 16, the
// same every round), the chunk after them loaded one round ahead.  LDS holds
// only the program, the class table and the slots (~10 KB per workgroup,
// where staging the text took 38 KB and held a CU to eight waves), so
// occupancy is set by registers.  tpl_finish reads its few fields through
// 4-byte loads (the line is in L2 by then).  The text must be 16-B aligned
// (the host checks).
__device__ __forceinline__ uint4 text_chunk(const uint4* __restrict__ t16, const uint8_t* __restrict__ text,
                                            uint64_t ci, uint64_t n_full, uint64_t n_bytes) {
  if (ci < n_full) return t16[ci];
  uint32_t w[4] = {0u, 0u, 0u, 0u};   // the buffer's last, partial chunk (or past the end: zeros)
  for (uint32_t k = 0; k < 16; ++k)
    if (16 * ci + k < n_bytes) w[k >> 2] |= (uint32_t)text[16 * ci + k] << (8 * (k & 3));
  return uint4{w[0], w[1], w[2], w[3]};
}

__global__ __launch_bounds__(kParseWG) void k_parse_win(const uint8_t* __restrict__ text,
                                                       const uint64_t* __restrict__ off, uint64_t n_lines,
                                                       const rsa_parse_ifc* __restrict__ ifcs, uint32_t n_ifcs,
                                                       const rsa_parse_spell* __restrict__ spells, uint32_t n_spells,
                                                       rsa_tuple* __restrict__ tuples, uint32_t* __restrict__ ts_out,
                                                       uint32_t* __restrict__ disp, uint32_t* __restrict__ slow_idx,
                                                       unsigned int* __restrict__ slow_n) {
  using namespace rsa_text::tpl;
  __shared__ uint32_t tprog[kProgLen];
  __shared__ uint8_t tcls[256];
  __shared__ uint32_t tslot[kParseWG * kSlotWords];
  {
    constexpr ClsTable kCls = cls_table();
    for (uint32_t k = threadIdx.x; k < kProgLen; k += blockDim.x) tprog[k] = kProg[k];
    for (uint32_t k = threadIdx.x; k < 256; k += blockDim.x) tcls[k] = kCls.t[k];
  }
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * kParseWG + threadIdx.x;
  const bool have = i < n_lines;
  const uint64_t n_bytes = off[n_lines];
  uint64_t a = 0, len = 0;
  if (have) {
    a = off[i];
    const uint64_t b = off[i + 1];
    len = b - a;
    if (len && text[b - 1] == '\n') --len;
  }
  const bool scannable = have && len < 0xFFFFu;
  const uint32_t n = scannable ? (uint32_t)len : 0u;
  uint32_t nmax = n;   // the wave's longest line: the trip count of every lane
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t y = (uint32_t)__shfl_xor((int)nmax, o);
    nmax = y > nmax ? y : nmax;
  }
  uint32_t* slot = tslot + threadIdx.x * kSlotWords;
  const uint4* t16 = reinterpret_cast<const uint4*>(text);
  const uint64_t n_full = n_bytes >> 4;
  uint64_t ci = a >> 4;
  const uint32_t q = (uint32_t)(a >> 2) & 3u, r = ((uint32_t)a & 3u) * 8u;
  uint4 w0 = text_chunk(t16, text, ci, n_full, n_bytes), w1 = text_chunk(t16, text, ci + 1, n_full, n_bytes);
  State st = start(tprog);
  for (uint32_t base = 0; base < nmax; base += 16) {
    const uint4 w2 = text_chunk(t16, text, ci + 2, n_full, n_bytes);   // the next round's second chunk
    const uint32_t W[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
    uint32_t X[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) X[j] = q == 0 ? W[j] : q == 1 ? W[j + 1] : q == 2 ? W[j + 2] : W[j + 3];
    uint32_t B[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) B[k] = __builtin_amdgcn_alignbit(X[k + 1], X[k], r);
    if (RSA_TPL_PROF == 2) {
      st.ok ^= B[0] ^ B[1] ^ B[2] ^ B[3];   // (the loads only)
    } else {
#pragma unroll
      for (uint32_t k = 0; k < 16; ++k) {
        const uint32_t idx = base + k;
        step(st, idx, (B[k >> 2] >> (8 * (k & 3))) & 0xFFu, lt01(idx, n), tprog, tcls, slot);
      }
    }
    w0 = w1;
    w1 = w2;
    ++ci;
  }
  if (!have) return;
  rsa_tuple tup = {0u, 0u, 0, 0, 0, 0, 0};
  uint32_t ts = 0, d = rsa_text::kLineDefer;
  if (RSA_TPL_PROF) {
    d = RSA_LINE_NOACL + (st.ok == 7u);
  } else if (scannable && st.ok && tprog[st.seg] == kEndSeg) {
    const uint64_t nw = n_bytes >> 2;
    uint32_t tail = 0;
    for (uint32_t k = 0; k < (uint32_t)(n_bytes & 3u); ++k) tail |= (uint32_t)text[4 * nw + k] << (8 * k);
    const rsa_text::GWordU s{reinterpret_cast<const uint32_t*>(text), a, nw, tail, (uint32_t)len};
    if (!rsa_text::tpl_finish(s, slot, ifcs, n_ifcs, spells, n_spells, tup, ts, d)) {
      tup = rsa_tuple{0u, 0u, 0, 0, 0, 0, 0};
      ts = 0;
      d = rsa_text::kLineDefer;
    }
  }
  defer_append(d == rsa_text::kLineDefer, i, slow_idx, slow_n);
  tuples[i] = tup;
  ts_out[i] = ts;
  disp[i] = d;
}

// The deferred lines, densely packed: the general parse (the regexes'
// backtracking restated), reading from HBM.  Persistent grid over the
// device-side count.
// k_parse_slow's lanes each walk their lines through dependent 4-byte loads,
// so more resident waves hide more of that latency: at 6 waves per SIMD (80
// VGPRs) and 3072 workgroups the parse step of a 30M-line job takes 10.41-10.52
// ms against 10.84 at the compiler's 102 VGPRs (4 waves, 2048 workgroups); 8
// waves (64 VGPRs) gains nothing (tools/ab_text.sh, profiles/r05/ab_summary.txt r05s)
#ifndef RSA_SLOW_WAVES
#define RSA_SLOW_WAVES 6   // minimum waves per SIMD for k_parse_slow (register cap; 0 = compiler's choice)
#endif
#ifndef RSA_SLOW_GRID
#define RSA_SLOW_GRID 3072
#endif
#if RSA_SLOW_WAVES
#define RSA_SLOW_ATTR __attribute__((amdgpu_waves_per_eu(RSA_SLOW_WAVES, 8)))
#else
#define RSA_SLOW_ATTR
#endif
constexpr uint32_t kSlowGrid = RSA_SLOW_GRID;
template <bool kReduce>
__global__ __launch_bounds__(kParseWG) RSA_SLOW_ATTR void k_parse_slow(const uint8_t* __restrict__ text,
                                                         const uint64_t* __restrict__ off, uint64_t n_lines,
                                                         const rsa_parse_ifc* __restrict__ ifcs, uint32_t n_ifcs,
                                                         const rsa_parse_spell* __restrict__ spells, uint32_t n_spells,
                                                         const uint32_t* __restrict__ slow_idx,
                                                         const unsigned int* __restrict__ slow_n,
                                                         rsa_tuple* __restrict__ tuples, uint32_t* __restrict__ ts_out,
                                                         uint32_t* __restrict__ disp) {
  const uint32_t ns = *slow_n;
  const uint64_t n_bytes = off[n_lines];
  const uint32_t* w32 = reinterpret_cast<const uint32_t*>(text);
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < ns; j += gridDim.x * blockDim.x) {
    const uint64_t i = slow_idx[j];
    const uint64_t a = off[i], b = off[i + 1];
    uint64_t len = b - a;
    if (len && text[b - 1] == '\n') --len;
    rsa_tuple tup = {0u, 0u, 0, 0, 0, 0, 0};
    uint32_t ts = 0, d = RSA_LINE_HOST;
    const rsa_text::GWordLn s{w32, text, a, n_bytes, (uint32_t)len, ~0ull, 0u};
    if (len >= 0xFFFFFFFFull) {
      // (a line of 4 GiB: the host parser's)
    } else if (kReduce) {
      rsa_text::reduce_line(s, spells, n_spells, tup, ts, d);
      if (i > 0 && d != RSA_RED_NOISE) {
        const uint64_t pa = off[i - 1];
        uint64_t plen = a - pa;
        if (plen && text[a - 1] == '\n') --plen;
        const rsa_text::GWordLn q{w32, text, pa, n_bytes, (uint32_t)plen, ~0ull, 0u};
        if (rsa_text::same_key(s, q)) d |= RSA_RED_SAME_KEY;
      }
    } else {
      rsa_text::parse_line(s, ifcs, n_ifcs, spells, n_spells, tup, ts, d);
    }
    tuples[i] = tup;
    ts_out[i] = ts;
    disp[i] = d;
  }
}

// ---------------------------------------------------------------------------
// Order keys.  Round r key of a line: bytes [7r, 7r + 7) big-endian (0 past the
// end) << 8 | min(bytes left, 8): equal keys <=> equal 7-byte windows with the
// same "ended here" status, and key order is byte order (a prefix sorts
// first).  A line is settled once its group (equal keys so far) is a singleton
// or its bytes ended in this window (then the whole group is equal strings,
// already in line-index order: the sorts are stable).
__device__ __forceinline__ uint64_t chunk_key(const uint8_t* __restrict__ text, uint64_t n_bytes, uint64_t a,
                                              uint32_t len, uint64_t pos) {
  const uint32_t rem = len > pos ? (uint32_t)(len - pos) : 0u;
  if (!rem) return 0;
  const uint64_t p = a + pos;
  uint64_t k;
  if (p + 12 <= n_bytes) {   // three aligned words hold bytes p .. p + 6 (text is 4-byte aligned)
    const uint32_t* t32 = reinterpret_cast<const uint32_t*>(text);
    const uint64_t q = p >> 2;
    const uint32_t sh = (uint32_t)(p & 3) * 8;
    const uint64_t lo = (uint64_t)t32[q] | ((uint64_t)t32[q + 1] << 32);
    const uint64_t x = sh ? (lo >> sh) | ((uint64_t)t32[q + 2] << (64 - sh)) : lo;   // bytes p .. p + 7, little endian
    k = __builtin_bswap64(x) & ~0xFFull;                                               // b0 .. b6 big endian, << 8
    if (rem < 7) k &= ~0ull << (64 - 8 * rem);
  } else {
    k = 0;
    for (uint32_t j = 0; j < 7; ++j) k = k << 8 | (j < rem ? text[p + j] : 0u);
    k <<= 8;
  }
  return k | (rem < 8 ? rem : 8u);
}

// 8 bytes of a line from byte p of the text, big-endian, zero past `rem`
// (rem >= 1 bytes of the line remain at p); text is 4-byte aligned.
__device__ __forceinline__ uint64_t line_chunk8(const uint8_t* __restrict__ text, uint64_t n_bytes, uint64_t p,
                                                uint32_t rem) {
  uint64_t k;
  if (p + 12 <= n_bytes) {
    const uint32_t* t32 = reinterpret_cast<const uint32_t*>(text);
    const uint64_t q = p >> 2;
    const uint32_t sh = (uint32_t)(p & 3) * 8;
    const uint64_t lo = (uint64_t)t32[q] | ((uint64_t)t32[q + 1] << 32);
    const uint64_t x = sh ? (lo >> sh) | ((uint64_t)t32[q + 2] << (64 - sh)) : lo;
    k = __builtin_bswap64(x);
  } else {
    k = 0;
    for (uint32_t j = 0; j < 8; ++j) k = k << 8 | (p + j < n_bytes ? text[p + j] : 0u);
  }
  if (rem < 8) k &= ~0ull << (64 - 8 * rem);
  return k;
}

// round 0: every line's length without '\n' (kept for the later rounds) and its first key
// A line that is not the last and does not end in '\n' (or is 4 GiB long):
// its length cannot be taken from the next line's start (nl_bad, one atomic
// per wave; k_compact then reads lens[] instead).
__device__ __forceinline__ void note_nl(bool bad, uint32_t* __restrict__ nl_bad) {
  const unsigned long long b = __ballot(bad);
  if (b && (int)__lane_id() == __builtin_ctzll(b)) atomicOr(nl_bad, 1u);
}

__global__ void k_keys0(const uint8_t* __restrict__ text, const uint64_t* __restrict__ off, uint32_t n,
                        uint64_t n_bytes, uint32_t* __restrict__ lens, uint64_t* __restrict__ keys,
                        uint32_t* __restrict__ ids, uint32_t* __restrict__ nl_bad) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t a = 0, b = 0, len = 0;
  bool nl = true;
  if (j < n) {
    a = off[j];
    b = off[j + 1];
    len = b - a;
    nl = len && text[b - 1] == '\n';
    if (nl) --len;
  }
  note_nl(j + 1 < n && (!nl || len >= 0xFFFFFFFFull), nl_bad);
  if (j >= n) return;
  const uint32_t l32 = len < 0xFFFFFFFFull ? (uint32_t)len : 0xFFFFFFFFu;
  lens[j] = l32;
  keys[j] = chunk_key(text, n_bytes, a, l32, 0u);
  ids[j] = j;
}

// Grouped order keys, round -1: per line its length, its group as a 32-bit
// sort key (a negative group -- a line no rank is asked for -- sorts last as
// 0xFFFFFFFF) and its id.
__global__ void k_grp0(const int32_t* __restrict__ group, const uint8_t* __restrict__ text,
                       const uint64_t* __restrict__ off, uint32_t n, uint32_t none, uint32_t* __restrict__ lens,
                       uint32_t* __restrict__ keys, uint32_t* __restrict__ ids, uint32_t* __restrict__ nl_bad) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t a = 0, b = 0, len = 0;
  bool nl = true;
  if (j < n) {
    a = off[j];
    b = off[j + 1];
    len = b - a;
    nl = len && text[b - 1] == '\n';
    if (nl) --len;
  }
  note_nl(j + 1 < n && (!nl || len >= 0xFFFFFFFFull), nl_bad);
  if (j >= n) return;
  lens[j] = len < 0xFFFFFFFFull ? (uint32_t)len : 0xFFFFFFFFu;
  const int32_t g = group[j];
  keys[j] = g < 0 ? none : (uint32_t)g;
  ids[j] = j;
}

// Reductions to a few device words: a persistent grid (kRedGrid workgroups)
// reduces in registers, waves and LDS, then one atomic per workgroup -- one
// atomic per wave on the same word serialises ~n/64 atomics at one L2 address.
constexpr uint32_t kRedGrid = 1024, kRedThreads = 256;

// the largest group (atomicMax into *mx, zeroed by the caller)
__global__ __launch_bounds__(kRedThreads) void k_grp_max(const int32_t* __restrict__ group, uint32_t n,
                                                         uint32_t* __restrict__ mx) {
  __shared__ int32_t sh[kRedThreads / 64];
  int32_t g = 0;
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
    const int32_t y = group[j];
    g = y > g ? y : g;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const int32_t y = __shfl_xor(g, o);
    g = y > g ? y : g;
  }
  if (__lane_id() == 0) sh[threadIdx.x >> 6] = g;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t w = 1; w < blockDim.x / 64; ++w) g = sh[w] > g ? sh[w] : g;
    if (g > 0) atomicMax(mx, (uint32_t)g);
  }
}

// after the sort by group: group starts (+1, max-scanned by the caller)
__global__ void k_grp_bounds(const uint32_t* __restrict__ keys, uint32_t m, uint32_t* __restrict__ bstart) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  bstart[j] = (j == 0 || keys[j] != keys[j - 1]) ? j + 1 : 0u;
}

// a line alone in its group, or without a group, is settled at its position
__global__ void k_grp_settle(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ ids,
                             const uint32_t* __restrict__ first, uint32_t m, uint32_t none, uint64_t base,
                             uint64_t* __restrict__ order, uint32_t* __restrict__ keep) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const bool last_in_group = j + 1 == m || keys[j + 1] != keys[j];
  const bool settled = keys[j] == none || (first[j] == j + 1 && last_in_group);
  if (settled) order[ids[j]] = base + j;
  keep[j] = settled ? 0u : 1u;
}

struct Act {               // an unsettled line: its text offset, id, the position its class starts at, length
  uint64_t off;            // (offset and length travel with the element: the rounds read them in order
  uint32_t id, gs, len;    //  instead of gathering them by line id)
};
static_assert(sizeof(Act) == 24, "Act layout");

// the window of a class: its depth (bytes all its lines share, cdep) plus the
// further common prefix k_lcp found (cmin), both indexed by the class start
// (preH / preL: the line's 16 bytes from the class depth, big-endian, as k_lcp
// read them: a window inside them needs no text read -- text reads by line
// are one HBM transaction each, the staged bytes are coalesced)
__global__ void k_keys(const uint8_t* __restrict__ text, uint64_t n_bytes, const Act* __restrict__ act, uint32_t m,
                       const uint32_t* __restrict__ cdep, const uint32_t* __restrict__ cmin,
                       const uint64_t* __restrict__ preH, const uint64_t* __restrict__ preL,
                       uint64_t* __restrict__ keys, uint64_t* __restrict__ vals) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const Act x = act[j];
  const uint32_t e = cmin[x.gs], len = x.len;
  const uint64_t pos = (uint64_t)cdep[x.gs] + e;
  uint64_t key;
  if (e <= 9u) {
    const uint32_t rem = len > pos ? (uint32_t)(len - pos) : 0u;
    const uint64_t H = preH[j], L = preL[j];
    // bytes e .. e + 6 at the top (shifts stay below 64)
    const uint64_t w = e == 0 ? H : e < 8 ? (H << (8u * e)) | (L >> (64u - 8u * e)) : L << (8u * (e - 8u));
    uint64_t k = w & ~0xFFull;
    if (rem && rem < 7) k &= ~0ull << (64u - 8u * rem);
    key = rem ? (k | (rem < 8 ? rem : 8u)) : 0ull;
  } else {
    key = chunk_key(text, n_bytes, x.off, len, pos);
  }
  keys[j] = key;
  vals[j] = (uint64_t)x.gs << 32 | x.id;
}

// Common-prefix skip: every line of a class is compared with the class's
// first line from the class depth on; the class minimum of those lengths
// (segmented over the wave, one atomicMin per class and wave into cmin[gs],
// set to ~0 by k_cls_first) is where the class's lines first differ, so the
// next window starts there -- the bytes all of them share (a syslog header,
// "Built inbound TCP connection ...") cost one pass instead of a round per 7
// bytes.  Capped at kLcpMax bytes per pass (the window then starts there).
constexpr uint32_t kLcpMax = 4096;
// (the line's first 16 bytes from the depth go to preH / preL for k_keys)
__global__ void k_lcp(const uint8_t* __restrict__ text, uint64_t n_bytes, const Act* __restrict__ act,
                      const uint32_t* __restrict__ first1, uint32_t m, const uint32_t* __restrict__ cdep,
                      uint32_t* __restrict__ cmin, uint64_t* __restrict__ preH, uint64_t* __restrict__ preL) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t e = 0xFFFFFFFFu, gs = 0xFFFFFFFFu;
  if (j < m) {
    const Act x = act[j];
    gs = x.gs;
    const Act ya = act[first1[j] - 1];   // the class's first line
    const uint32_t y = ya.id;
    const uint32_t d = cdep[gs], la = x.len, lb = ya.len;
    const uint32_t ra = la > d ? la - d : 0u, rb = lb > d ? lb - d : 0u;
    const uint32_t lim = (ra < rb ? ra : rb) < kLcpMax ? (ra < rb ? ra : rb) : kLcpMax;
    const uint64_t pa = x.off + d;
    const uint64_t H = ra ? line_chunk8(text, n_bytes, pa, ra) : 0ull;
    const uint64_t L = ra > 8 ? line_chunk8(text, n_bytes, pa + 8, ra - 8) : 0ull;
    preH[j] = H;
    preL[j] = L;
    e = lim;
    if (y != x.id) {
      const uint64_t pb = ya.off + d;
      for (uint32_t p = 0; p < lim; p += 8) {
        const uint64_t ka = p == 0 ? H : p == 8 ? L : line_chunk8(text, n_bytes, pa + p, la - d - p),
                       kb = line_chunk8(text, n_bytes, pb + p, lb - d - p);
        if (ka != kb) {
          const uint32_t q = p + (uint32_t)__builtin_clzll(ka ^ kb) / 8u;
          e = q < lim ? q : lim;
          break;
        }
      }
    }
  }
  // segmented min over the wave (a class's elements are contiguous)
  const uint32_t lane = __lane_id();
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t ye = (uint32_t)__shfl_down((int)e, o), yg = (uint32_t)__shfl_down((int)gs, o);
    if (lane + o < 64 && yg == gs && ye < e) e = ye;
  }
  const uint32_t pg = (uint32_t)__shfl_up((int)gs, 1);
  if (j < m && (lane == 0 || pg != gs)) atomicMin(&cmin[gs], e);
}

// a window that split nothing (only after a capped k_lcp): the classes move on by 7 bytes
__global__ void k_dep_adv(const Act* __restrict__ act, uint32_t m, const uint32_t* __restrict__ cdep,
                          const uint32_t* __restrict__ cmin, uint32_t* __restrict__ cnext) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const uint32_t g = act[j].gs;
  cnext[g] = cdep[g] + cmin[g] + 7u;   // (every element writes its class's one value)
}

// 1 if this round can change anything: a group whose keys differ, or a line
// that ends in this window (else the round is skipped: no sort, no settle)
// live[1..2]: the OR over all keys of (key ^ keys[0]) -- the bits that vary
// this round; the sort then runs over those bits only.  live[3]: some class
// has a key below its predecessor's -- else every class is already in key
// order (time-ordered logs: the header windows) and the round needs no sort
// (persistent grid of kRedGrid x kRedThreads; one atomic per word and workgroup)
__global__ __launch_bounds__(kRedThreads) void k_round_live(const uint64_t* __restrict__ keys,
                                                            const Act* __restrict__ act, uint32_t m,
                                                            uint32_t* __restrict__ live) {
  __shared__ uint32_t sh[kRedThreads / 64][4];
  uint32_t v[4] = {0u, 0u, 0u, 0u};
  const uint64_t k0 = keys[0];
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m; j += gridDim.x * blockDim.x) {
    const uint64_t k = keys[j];
    const bool ended = (k & 0xFFu) < 8u;
    const bool same = j > 0 && act[j].gs == act[j - 1].gs;
    const uint64_t kp = same ? keys[j - 1] : k;
    v[0] |= (ended || kp != k) ? 1u : 0u;
    v[3] |= k < kp ? 1u : 0u;
    const uint64_t d = k ^ k0;
    v[1] |= (uint32_t)d;
    v[2] |= (uint32_t)(d >> 32);
  }
  for (int o = 32; o > 0; o >>= 1)
    for (int q = 0; q < 4; ++q) v[q] |= (uint32_t)__shfl_xor((int)v[q], o);
  if (__lane_id() == 0)
    for (int q = 0; q < 4; ++q) sh[threadIdx.x >> 6][q] = v[q];
  __syncthreads();
  if (threadIdx.x < 4) {
    uint32_t x = 0;
    for (uint32_t w = 0; w < blockDim.x / 64; ++w) x |= sh[w][threadIdx.x];
    if (x) atomicOr(&live[threadIdx.x], x);
  }
}

// a round already in (class, key) order: the values split into gs / ids in place
__global__ void k_split_vals(const uint64_t* __restrict__ vals, uint32_t m, uint32_t* __restrict__ gs,
                             uint32_t* __restrict__ ids) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const uint64_t v = vals[j];
  gs[j] = (uint32_t)(v >> 32);
  ids[j] = (uint32_t)v;
}

__global__ void k_gs_iota(const uint64_t* __restrict__ vals, uint32_t m, uint32_t* __restrict__ gs,
                          uint32_t* __restrict__ idx) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  gs[j] = (uint32_t)(vals[j] >> 32);
  idx[j] = j;
}

__global__ void k_gather(const uint64_t* __restrict__ keys, const uint64_t* __restrict__ vals,
                         const uint32_t* __restrict__ perm, uint32_t m, uint64_t* __restrict__ keys_out,
                         uint32_t* __restrict__ gs, uint32_t* __restrict__ ids) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const uint32_t q = perm[j];
  keys_out[j] = keys[q];
  const uint64_t v = vals[q];
  gs[j] = (uint32_t)(v >> 32);
  ids[j] = (uint32_t)v;
}

// first index of each gs run (max-scan input): j at a run start, else 0
__global__ void k_run_first(const uint32_t* __restrict__ gs, uint32_t m, uint32_t* __restrict__ out) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  out[j] = (j == 0 || gs[j] != gs[j - 1]) ? j : 0u;
}

// After the sort of round r: element j sits at position pos = gs + (j - first);
// pos_start = pos at a new-group boundary, else 0 (max-scanned by the caller).
__global__ void k_bounds(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ gs,
                         const uint32_t* __restrict__ first, uint32_t m, uint32_t* __restrict__ pos,
                         uint32_t* __restrict__ bstart) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const uint32_t g = gs ? gs[j] : 0u;
  const uint32_t p = gs ? g + (j - first[j]) : j;
  pos[j] = p;
  const bool b = j == 0 || keys[j] != keys[j - 1] || (gs && gs[j] != gs[j - 1]);
  bstart[j] = b ? p + 1 : 0u;   // +1: position 0 is a valid group start
}

// settle or keep each element; kept ones get a flag for the compaction scan
__global__ void k_settle(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ gs,
                         const uint32_t* __restrict__ ids, const uint32_t* __restrict__ pos,
                         const uint32_t* __restrict__ ngs1, uint32_t m, uint64_t base, uint64_t* __restrict__ order,
                         uint32_t* __restrict__ keep) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const bool last_in_group =
      j + 1 == m || keys[j + 1] != keys[j] || (gs && gs[j + 1] != gs[j]);
  const bool first_in_group = ngs1[j] == pos[j] + 1;
  const bool ended = (keys[j] & 0xFFu) < 8u;
  const bool settled = ended || (first_in_group && last_in_group);
  if (settled) order[ids[j]] = base + pos[j];
  keep[j] = settled ? 0u : 1u;
}

// the kept elements into act; their new classes' depth into cnext[new start]:
// the old class's window end (cdep + cmin of the old start gs_old, 0 when
// gs_old is null) + adv (7: the window matched; 0: the group stage)
// (in: the elements in this order, whose offset and length are taken; null:
// gathered by line id from off / lens -- after a sort)
// (gathered by id: when every line but the last ends in '\n' -- *nl_bad == 0
// -- the length comes from the next line's start, the same 64-B line as the
// offset as a rule, so one random read instead of two)
__global__ void k_compact(const uint32_t* __restrict__ ids, const uint32_t* __restrict__ ngs1,
                          const uint32_t* __restrict__ keep, const uint32_t* __restrict__ slot, uint32_t m,
                          Act* __restrict__ out, const uint32_t* __restrict__ gs_old, const uint32_t* __restrict__ cdep,
                          const uint32_t* __restrict__ cmin, uint32_t* __restrict__ cnext, uint32_t adv,
                          const Act* __restrict__ in, const uint64_t* __restrict__ off,
                          const uint32_t* __restrict__ lens, uint32_t n_lines, const uint32_t* __restrict__ nl_bad) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m || !keep[j]) return;
  const uint32_t g = ngs1[j] - 1, id = ids[j];
  uint64_t o;
  uint32_t l;
  if (in) {
    const Act x = in[j];
    o = x.off;
    l = x.len;
  } else if (!*nl_bad && id + 1 < n_lines) {
    o = off[id];
    l = (uint32_t)(off[id + 1] - o - 1);
  } else {
    o = off[id];
    l = lens[id];
  }
  out[slot[j]] = Act{o, id, g, l};
  cnext[g] = (gs_old ? cdep[gs_old[j]] + cmin[gs_old[j]] : 0u) + adv;   // (the same value from every member)
}

// ---- small-class finish: a class (lines equal in their first `depth` bytes,
// contiguous in act) of at most kSmallClass lines is ranked directly: each
// lane counts the members that sort before its line (bytes from `depth` on,
// a prefix first, equal strings by line index), so its position is the class
// start + that count -- no further rounds of sorts for it.  After the first
// live window nearly every class is small (lines of one rule that share a
// second), so the global rounds stop early.
constexpr uint32_t kSmallClass = 64;

// per element of act: 1 + index of its class's first element at class starts, else 0
// (cmin non-null: the class's k_lcp minimum is reset to ~0 at its first element)
__global__ void k_cls_first(const Act* __restrict__ act, uint32_t m, uint32_t* __restrict__ out,
                            uint32_t* __restrict__ cmin) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const bool f = j == 0 || act[j].gs != act[j - 1].gs;
  out[j] = f ? j + 1 : 0u;
  if (f && cmin) cmin[act[j].gs] = 0xFFFFFFFFu;
}

// (after the max-scan of k_cls_first): the class size, stored at its first element
__global__ void k_cls_size(const Act* __restrict__ act, const uint32_t* __restrict__ first1, uint32_t m,
                           uint32_t* __restrict__ size) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  if (j + 1 == m || act[j + 1].gs != act[j].gs) size[first1[j] - 1] = j + 2 - first1[j];
}

// rank every element of a small class; keep[j] = 1 for the elements of large
// classes.  keys[j]: the element's window key at its class's window start
// (k_keys).  A member's rank is the number of members with a smaller key plus
// the members with an equal key and a smaller id -- exact when the equal keys
// are equal strings (the window holds their ends).  Members whose equal window
// goes on (a tie group) are not compared further here: the group becomes a
// class of its own, starting at its position in the class, one window deeper
// (its members written to tie[] at their rank, tkeep[] = 1, its depth to
// tdep[start]); it joins the current round behind the large classes, where the
// common-prefix pass skips the bytes its lines share.
// The members' keys and ids are staged in LDS: a workgroup's elements
// [b0, b0 + 256) have their small classes inside [b0 - 64, b0 + 320).
constexpr uint32_t kFinThreads = 256, kFinSpan = kFinThreads + 2 * kSmallClass;
__global__ __launch_bounds__(kFinThreads) void k_finish_small(
    const Act* __restrict__ act, const uint64_t* __restrict__ keys, const uint32_t* __restrict__ first1,
    const uint32_t* __restrict__ size, uint32_t m, const uint32_t* __restrict__ cdep,
    const uint32_t* __restrict__ cmin, uint64_t base, uint64_t* __restrict__ order, uint32_t* __restrict__ keep,
    Act* __restrict__ tie, uint32_t* __restrict__ tkeep, uint32_t* __restrict__ tdep) {
  __shared__ uint64_t skey[kFinSpan];
  __shared__ uint32_t sid[kFinSpan];
  const int64_t lo = (int64_t)blockIdx.x * kFinThreads - (int64_t)kSmallClass;
  for (uint32_t q = threadIdx.x; q < kFinSpan; q += blockDim.x) {
    const int64_t k = lo + (int64_t)q;
    if (k >= 0 && k < (int64_t)m) {
      skey[q] = keys[k];
      sid[q] = act[k].id;
    }
  }
  __syncthreads();
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const uint32_t cs = first1[j] - 1, cn = size[cs];
  if (cn > kSmallClass) {
    keep[j] = 1u;
    tkeep[j] = 0u;
    return;
  }
  keep[j] = 0u;
  const Act x = act[j];
  const uint64_t kx = keys[j];
  uint32_t lt = 0, eq_before = 0, eq = 0;
  for (uint32_t k = cs; k < cs + cn; ++k) {
    if (k == j) continue;
    const uint32_t q = (uint32_t)((int64_t)k - lo);   // inside the staged span
    const uint64_t ky = skey[q];
    lt += ky < kx ? 1u : 0u;
    if (ky == kx) {
      ++eq;
      eq_before += sid[q] < x.id ? 1u : 0u;
    }
  }
  const uint32_t slot = cs + lt + eq_before;   // the member's rank, as an index into the class's range
  if (eq == 0 || (kx & 0xFFu) != 8u) {         // unique, or equal strings
    order[x.id] = base + x.gs + lt + eq_before;
    tkeep[slot] = 0u;
  } else {                                     // a tie group past the window: its own class
    const uint32_t g = x.gs + lt;
    tie[slot] = Act{x.off, x.id, g, x.len};
    tkeep[slot] = 1u;
    tdep[g] = cdep[x.gs] + cmin[x.gs] + 7u;    // (the same value from every member)
  }
}

// the tie groups' depth into cdep (after the finisher: their starts are no
// other live class's start)
__global__ void k_tie_dep(const Act* __restrict__ act, uint32_t m, const uint32_t* __restrict__ tdep,
                          uint32_t* __restrict__ cdep) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const uint32_t g = act[j].gs;
  cdep[g] = tdep[g];
}

// compaction of the kept elements (slot: exclusive scan of keep)
__global__ void k_compact_act(const Act* __restrict__ in, const uint32_t* __restrict__ keep,
                              const uint32_t* __restrict__ slot, uint32_t m, Act* __restrict__ out,
                              const uint64_t* __restrict__ kin, const uint64_t* __restrict__ vin,
                              uint64_t* __restrict__ kout, uint64_t* __restrict__ vout) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m || !keep[j]) return;
  const uint32_t q = slot[j];
  out[q] = in[j];
  if (kin) {
    kout[q] = kin[j];
    vout[q] = vin[j];
  }
}

inline uint32_t blocks(uint64_t n, uint32_t t) { return (uint32_t)((n + t - 1) / t); }

// ---- scans and the LSD radix sort of the order keys (hand-written) ----------
// Scans: kScanTile elements per workgroup (1024 threads x 4), the tile sums
// scanned by one workgroup, then added back.  Max-scans are inclusive (group
// starts), plus-scans inclusive or exclusive.
constexpr uint32_t kScanThreads = 1024, kScanPer = 4, kScanTile = kScanThreads * kScanPer;

struct OpPlus {
  template <typename T>
  __device__ static T f(T a, T b) { return a + b; }
  template <typename T>
  __device__ static T id() { return 0; }
};
struct OpMax {
  template <typename T>
  __device__ static T f(T a, T b) { return a > b ? a : b; }
  template <typename T>
  __device__ static T id() { return 0; }
};

// workgroup scan of one value per thread (Op commutative: + or max): this
// thread's exclusive and inclusive values and the workgroup total
template <typename Op, typename T>
__device__ __forceinline__ void wg_scan(T v, T* sh, T& excl, T& incl, T& total) {
  const uint32_t lane = __lane_id(), w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  T x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const T y = __shfl_up(x, o);
    if ((int)lane >= o) x = Op::f(x, y);
  }
  T xe = __shfl_up(x, 1);
  if (lane == 0) xe = Op::template id<T>();
  if (lane == 63) sh[w] = x;
  __syncthreads();
  T before = Op::template id<T>(), all = Op::template id<T>();
  for (uint32_t q = 0; q < nw; ++q) {
    const T t = sh[q];
    if (q < w) before = Op::f(before, t);
    all = Op::f(all, t);
  }
  __syncthreads();
  incl = Op::f(before, x);
  excl = Op::f(before, xe);
  total = all;
}

// pass 1: per tile, the scan inside the tile (out) and the tile's total
template <typename Op, bool kIncl, typename Tin, typename Tout>
__global__ __launch_bounds__(kScanThreads) void k_scan_tiles(const Tin* __restrict__ in, Tout* __restrict__ out,
                                                             uint64_t n, Tout* __restrict__ sums) {
  __shared__ Tout sh[16];
  const uint64_t beg = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanPer;
  // 32-bit elements of a full, 16-B aligned group: one 16-B load and store
  // per thread (coalesced), else element by element
  constexpr bool kVec = sizeof(Tin) == 4 && sizeof(Tout) == 4 && kScanPer == 4;
  const bool vec = kVec && beg + kScanPer <= n && ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15u) == 0;
  Tout v[kScanPer];
  Tout c = Op::template id<Tout>();
  if (vec) {
    const uint4 q = *reinterpret_cast<const uint4*>(in + beg);
    v[0] = (Tout)q.x;
    v[1] = (Tout)q.y;
    v[2] = (Tout)q.z;
    v[3] = (Tout)q.w;
  } else {
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; ++k) v[k] = beg + k < n ? (Tout)in[beg + k] : Op::template id<Tout>();
  }
#pragma unroll
  for (uint32_t k = 0; k < kScanPer; ++k) c = Op::f(c, v[k]);
  Tout ex, inc, total;
  wg_scan<Op>(c, sh, ex, inc, total);
  Tout run = ex;
  Tout o[kScanPer];
#pragma unroll
  for (uint32_t k = 0; k < kScanPer; ++k) {
    const Tout nx = Op::f(run, v[k]);
    o[k] = kIncl ? nx : run;
    run = nx;
  }
  if (vec) {
    *reinterpret_cast<uint4*>(out + beg) = uint4{(uint32_t)o[0], (uint32_t)o[1], (uint32_t)o[2], (uint32_t)o[3]};
  } else {
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; ++k)
      if (beg + k < n) out[beg + k] = o[k];
  }
  if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

// pass 2: one workgroup scans the tile totals in place (exclusive), the
// grand total into sums[nb]
template <typename Op, typename T>
__global__ __launch_bounds__(kScanThreads) void k_scan_tile_sums(T* __restrict__ sums, uint32_t nb) {
  __shared__ T sh[16];
  T carry = Op::template id<T>();
  for (uint32_t b0 = 0; b0 < nb; b0 += blockDim.x) {
    const uint32_t j = b0 + threadIdx.x;
    const T v = j < nb ? sums[j] : Op::template id<T>();
    T ex, inc, total;
    wg_scan<Op>(v, sh, ex, inc, total);
    if (j < nb) sums[j] = Op::f(carry, ex);
    carry = Op::f(carry, total);
  }
  if (threadIdx.x == 0) sums[nb] = carry;
}

// pass 3: add each tile's exclusive prefix
template <typename Op, typename Tout>
__global__ __launch_bounds__(kScanThreads) void k_scan_tiles_add(Tout* __restrict__ out, uint64_t n,
                                                                 const Tout* __restrict__ sums) {
  const uint64_t beg = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanPer;
  const Tout add = sums[blockIdx.x];
  constexpr bool kVec = sizeof(Tout) == 4 && kScanPer == 4;
  if (kVec && beg + kScanPer <= n && (reinterpret_cast<uintptr_t>(out) & 15u) == 0) {
    uint4 q = *reinterpret_cast<const uint4*>(out + beg);
    q.x = (uint32_t)Op::f(add, (Tout)q.x);
    q.y = (uint32_t)Op::f(add, (Tout)q.y);
    q.z = (uint32_t)Op::f(add, (Tout)q.z);
    q.w = (uint32_t)Op::f(add, (Tout)q.w);
    *reinterpret_cast<uint4*>(out + beg) = q;
    return;
  }
#pragma unroll
  for (uint32_t k = 0; k < kScanPer; ++k)
    if (beg + k < n) out[beg + k] = Op::f(add, out[beg + k]);
}

// sum of n uint32 into *total (uint64, zeroed by the caller): one device atomic per workgroup
__global__ __launch_bounds__(kScanThreads) void k_sum_u32(const uint32_t* __restrict__ in, uint64_t n,
                                                          unsigned long long* __restrict__ total) {
  __shared__ unsigned long long sh[16];
  const uint64_t beg = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanPer;
  unsigned long long c = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanPer; ++k) c += beg + k < n ? in[beg + k] : 0u;
  unsigned long long ex, inc, all;
  wg_scan<OpPlus>(c, sh, ex, inc, all);
  if (threadIdx.x == 0 && all) atomicAdd(total, all);
}

// LSD radix sort of (key, value) pairs, 8-bit digits: per pass a digit
// histogram per tile of kRsTile elements (bin-major, so its exclusive scan is
// every (digit, tile) run's output offset), then a stable scatter: a tile is
// walked row by row (one element per thread), each lane ranked among the
// earlier lanes of its wave with the same digit (eight ballots), the waves'
// digit counts turned into output bases in LDS.  Only the bits [b0, b1) the
// caller asks for are sorted (bits outside them must be equal in every key,
// or be allowed to order ties).
constexpr uint32_t kRsThreads = 1024, kRsRows = 8, kRsTile = kRsThreads * kRsRows;

__device__ __forceinline__ unsigned long long match_digit(uint32_t d, bool valid) {
  unsigned long long peers = __ballot(valid);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const unsigned long long bb = __ballot(valid && ((d >> b) & 1u));
    peers &= ((d >> b) & 1u) ? bb : ~bb;
  }
  return valid ? peers : 0ull;
}

template <typename K>
__global__ __launch_bounds__(kRsThreads) void k_rs_hist(const K* __restrict__ keys, uint32_t n, uint32_t shift,
                                                        uint32_t n_tiles, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  if (threadIdx.x < 256) h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kRsTile;
  const uint32_t lane = __lane_id();
  for (uint32_t r = 0; r < kRsRows; ++r) {
    const uint64_t i = base + (uint64_t)r * kRsThreads + threadIdx.x;
    const bool valid = i < n;
    const uint32_t d = valid ? (uint32_t)(keys[i] >> shift) & 255u : 0u;
    const unsigned long long peers = match_digit(d, valid);   // one LDS atomic per distinct digit of the wave
    if (valid && __popcll(peers & ((1ull << lane) - 1ull)) == 0) atomicAdd(&h[d], (uint32_t)__popcll(peers));
  }
  __syncthreads();
  if (threadIdx.x < 256) hist[(size_t)threadIdx.x * n_tiles + blockIdx.x] = h[threadIdx.x];
}

template <typename K, typename V>
__global__ __launch_bounds__(kRsThreads) void k_rs_scatter(const K* __restrict__ kin, const V* __restrict__ vin,
                                                           K* __restrict__ kout, V* __restrict__ vout, uint32_t n,
                                                           uint32_t shift, uint32_t n_tiles,
                                                           const uint32_t* __restrict__ offs) {
  __shared__ uint32_t run[256];                       // next output position per digit
  __shared__ uint32_t wc[kRsThreads / 64][256];       // the row's per-wave digit counts, then their output bases
  const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
  if (threadIdx.x < 256) run[threadIdx.x] = offs[(size_t)threadIdx.x * n_tiles + blockIdx.x];
  const uint64_t base = (uint64_t)blockIdx.x * kRsTile;
  for (uint32_t r = 0; r < kRsRows; ++r) {
    for (uint32_t q = threadIdx.x; q < (kRsThreads / 64) * 256; q += kRsThreads) (&wc[0][0])[q] = 0;
    __syncthreads();
    const uint64_t i = base + (uint64_t)r * kRsThreads + threadIdx.x;
    const bool valid = i < n;
    const K k = valid ? kin[i] : K(0);
    const V v = valid ? vin[i] : V(0);
    const uint32_t d = (uint32_t)(k >> shift) & 255u;
    const unsigned long long peers = match_digit(d, valid);
    const uint32_t rank = __popcll(peers & ((1ull << lane) - 1ull));
    if (valid && rank == 0) wc[w][d] = __popcll(peers);
    __syncthreads();
    if (threadIdx.x < 256) {
      uint32_t x = run[threadIdx.x];
      for (uint32_t q = 0; q < kRsThreads / 64; ++q) {
        const uint32_t cnt = wc[q][threadIdx.x];
        wc[q][threadIdx.x] = x;
        x += cnt;
      }
      run[threadIdx.x] = x;
    }
    __syncthreads();
    if (valid) {
      const uint32_t pos = wc[w][d] + rank;
      kout[pos] = k;
      vout[pos] = v;
    }
    __syncthreads();   // wc is cleared for the next row
  }
}


// host: scan of n elements (three passes: tile scans, a scan of the tile
// sums, the sums added back).  sums: scan_sums_len(n) words
template <typename Op, bool kIncl, typename Tin, typename Tout>
void scan(hipStream_t st, const Tin* in, Tout* out, uint64_t n, Tout* sums) {
  if (!n) return;
  const uint32_t nb = (uint32_t)((n + kScanTile - 1) / kScanTile);
  hipLaunchKernelGGL((k_scan_tiles<Op, kIncl, Tin, Tout>), dim3(nb), dim3(kScanThreads), 0, st, in, out, n, sums);
  hipLaunchKernelGGL((k_scan_tile_sums<Op, Tout>), dim3(1), dim3(kScanThreads), 0, st, sums, nb);
  hipLaunchKernelGGL((k_scan_tiles_add<Op, Tout>), dim3(nb), dim3(kScanThreads), 0, st, out, n, sums);
}

inline size_t scan_sums_len(uint64_t n) { return 2 * ((size_t)((n + kScanTile - 1) / kScanTile) + 2); }

// scratch of radix_pairs for n elements: hist (256 per tile) and its scan sums
inline size_t rs_hist_len(uint64_t n) { return (size_t)256 * ((n + kRsTile - 1) / kRsTile); }

// host: stable sort of (kA, vA) by key bits [b0, b1) into (kB, vB); (kT, vT)
// is ping-pong space, hist / sums scratch (rs_hist_len, scan_sums_len of it)
template <typename K, typename V>
void radix_pairs(hipStream_t st, const K* kA, K* kB, const V* vA, V* vB, uint32_t n, uint32_t b0, uint32_t b1,
                 K* kT, V* vT, uint32_t* hist, uint32_t* sums) {
  if (!n) return;
  const uint32_t passes = b1 > b0 ? (b1 - b0 + 7) / 8 : 0u;
  if (!passes) {
    (void)hipMemcpyAsync(kB, kA, (size_t)n * sizeof(K), hipMemcpyDeviceToDevice, st);
    (void)hipMemcpyAsync(vB, vA, (size_t)n * sizeof(V), hipMemcpyDeviceToDevice, st);
    return;
  }
  const uint32_t n_tiles = (n + kRsTile - 1) / kRsTile;
  const K* ks = kA;
  const V* vs = vA;
  for (uint32_t p = 0; p < passes; ++p) {
    const bool to_b = ((passes - 1 - p) & 1u) == 0u;   // the last pass writes (kB, vB)
    K* kd = to_b ? kB : kT;
    V* vd = to_b ? vB : vT;
    const uint32_t shift = b0 + 8 * p;
    hipLaunchKernelGGL((k_rs_hist<K>), dim3(n_tiles), dim3(kRsThreads), 0, st, ks, n, shift, n_tiles, hist);
    scan<OpPlus, false, uint32_t, uint32_t>(st, hist, hist, (uint64_t)256 * n_tiles, sums);
    hipLaunchKernelGGL((k_rs_scatter<K, V>), dim3(n_tiles), dim3(kRsThreads), 0, st, ks, vs, kd, vd, n, shift, n_tiles,
                       hist);
    ks = kd;
    vs = vd;
  }
}



struct Scratch {           // one hipMallocAsync'd arena, freed on the stream at the end
  rsa_ctx* c;
  hipStream_t st;
  void* base = nullptr;
  ~Scratch() {
    if (base) (void)hipFreeAsync(base, st);
  }
};

}  // namespace

extern "C" {

int rsa_text_count_lines(rsa_ctx* c, const uint8_t* d_text, uint64_t n, uint64_t* h_n_lines) {
  if (!c || !h_n_lines || (n && !d_text)) return RSA_ERR_ARG;
  *h_n_lines = 0;
  if (!n) return RSA_OK;
  hipStream_t st = rsa_internal_stream(c);
  const uint64_t nb = (n + kSplitBlock - 1) / kSplitBlock;
  if (nb > 0xFFFFFFFFull) return rsa_internal_fail(c, RSA_ERR_ARG, "text too large");
  const int aligned = (reinterpret_cast<uintptr_t>(d_text) & 15u) == 0;
  Scratch S{c, st};
  const size_t need = nb * 4 + 16 + 256;
  TPCHK(c, hipMallocAsync(&S.base, need, st));
  uint32_t* counts = static_cast<uint32_t*>(S.base);
  unsigned long long* total =
      reinterpret_cast<unsigned long long*>(static_cast<char*>(S.base) + ((nb * 4 + 15) / 16) * 16);
  TPCHK(c, hipMemsetAsync(total, 0, 8, st));
  hipLaunchKernelGGL(k_nl_count, dim3((uint32_t)nb), dim3(kSplitThreads), 0, st, d_text, n, aligned, counts);
  hipLaunchKernelGGL(k_sum_u32, dim3((uint32_t)((nb + kScanTile - 1) / kScanTile)), dim3(kScanThreads), 0, st,
                     counts, nb, total);
  TPCHK(c, hipGetLastError());
  uint64_t h_total = 0;
  uint8_t last = 0;
  TPCHK(c, hipMemcpyAsync(&h_total, total, 8, hipMemcpyDeviceToHost, st));
  TPCHK(c, hipMemcpyAsync(&last, d_text + n - 1, 1, hipMemcpyDeviceToHost, st));
  TPCHK(c, hipStreamSynchronize(st));
  *h_n_lines = h_total + (last != '\n' ? 1 : 0);
  return RSA_OK;
}

}  // extern "C"

namespace {
// One pass over the text: line starts d_off[1 ..] for lines < max_lines + 1
// (k_nl_offsets) and the line count (the last block's inclusive prefix, + 1
// when the text does not end in '\n').  d_off[0] = 0; the caller sets
// d_off[n_lines].
int split_pass(rsa_ctx* c, const uint8_t* d_text, uint64_t n, uint64_t* d_off, uint64_t max_lines,
               uint64_t* h_count) {
  hipStream_t st = rsa_internal_stream(c);
  *h_count = 0;
  hipLaunchKernelGGL(k_set_u64, dim3(1), dim3(1), 0, st, d_off, (uint64_t)0);
  if (!n) return RSA_OK;
  const uint64_t nb = (n + kSplitBlock - 1) / kSplitBlock;
  if (nb > 0xFFFFFFFFull) return rsa_internal_fail(c, RSA_ERR_ARG, "text too large");
  const int aligned = (reinterpret_cast<uintptr_t>(d_text) & 15u) == 0;
  Scratch S{c, st};
  TPCHK(c, hipMallocAsync(&S.base, nb * 8 + 64, st));
  unsigned long long* state = static_cast<unsigned long long*>(S.base);   // per block: look-back word
  unsigned int* ticket = reinterpret_cast<unsigned int*>(state + nb);     // [0] ticket, [1] error flag
  TPCHK(c, hipMemsetAsync(S.base, 0, nb * 8 + 64, st));
  hipLaunchKernelGGL(k_nl_offsets, dim3((uint32_t)nb), dim3(kSplitThreads), 0, st, d_text, n, aligned, d_off, max_lines,
                     state, ticket);
  TPCHK(c, hipGetLastError());
  unsigned int err = 0;
  unsigned long long last_state = 0;
  uint8_t last = 0;
  TPCHK(c, hipMemcpyAsync(&err, ticket + 1, 4, hipMemcpyDeviceToHost, st));
  TPCHK(c, hipMemcpyAsync(&last_state, state + nb - 1, 8, hipMemcpyDeviceToHost, st));
  TPCHK(c, hipMemcpyAsync(&last, d_text + n - 1, 1, hipMemcpyDeviceToHost, st));
  TPCHK(c, hipStreamSynchronize(st));
  if (err || !(last_state & kLbIncl)) return rsa_internal_fail(c, RSA_ERR_HIP, "text split: look-back did not resolve");
  *h_count = (last_state & kLbVal) + (last != '\n' ? 1u : 0u);
  return RSA_OK;
}
}  // namespace

extern "C" {

int rsa_text_line_offsets(rsa_ctx* c, const uint8_t* d_text, uint64_t n, uint64_t* d_off, uint64_t n_lines) {
  if (!c || !d_off || (n && !d_text)) return RSA_ERR_ARG;
  uint64_t count = 0;
  const int rc = split_pass(c, d_text, n, d_off, n_lines, &count);
  if (rc) return rc;
  hipLaunchKernelGGL(k_set_u64, dim3(1), dim3(1), 0, rsa_internal_stream(c), d_off + n_lines, n);
  TPCHK(c, hipGetLastError());
  return RSA_OK;
}

int rsa_text_split(rsa_ctx* c, const uint8_t* d_text, uint64_t n, uint64_t* d_off, uint64_t max_lines,
                   uint64_t* h_n_lines) {
  if (!c || !d_off || !h_n_lines || (n && !d_text)) return RSA_ERR_ARG;
  uint64_t count = 0;
  const int rc = split_pass(c, d_text, n, d_off, max_lines, &count);
  *h_n_lines = count;
  if (rc) return rc;
  if (count > max_lines)
    return rsa_internal_fail(c, RSA_ERR_CAPACITY, "rsa_text_split: more lines than max_lines (*h_n_lines holds the count)");
  hipLaunchKernelGGL(k_set_u64, dim3(1), dim3(1), 0, rsa_internal_stream(c), d_off + count, n);
  TPCHK(c, hipGetLastError());
  return RSA_OK;
}

int rsa_parse_text(rsa_ctx* c, const uint8_t* d_text, const uint64_t* d_off, uint64_t n_lines,
                   const rsa_parse_ifc* h_ifcs, uint32_t n_ifcs, const rsa_parse_spell* h_spells, uint32_t n_spells,
                   rsa_tuple* d_tuples, uint32_t* d_ts, uint32_t* d_disp) {
  if (!c || (n_lines && (!d_text || !d_off || !d_tuples || !d_ts || !d_disp))) return RSA_ERR_ARG;
  if (n_ifcs > 4096 || n_spells > 64 || (n_ifcs && !h_ifcs) || (n_spells && !h_spells))
    return rsa_internal_fail(c, RSA_ERR_ARG, "rsa_parse_text: bad interface/spelling table");
  for (uint32_t k = 0; k < n_ifcs; ++k)
    if (h_ifcs[k].len > RSA_IFC_NAME_MAX || h_ifcs[k].len == 0)
      return rsa_internal_fail(c, RSA_ERR_ARG, "rsa_parse_text: interface name length out of range");
  for (uint32_t k = 0; k < n_spells; ++k)
    if (h_spells[k].len > 15) return rsa_internal_fail(c, RSA_ERR_ARG, "rsa_parse_text: spelling too long");
  if (!n_lines) return RSA_OK;
  hipStream_t st = rsa_internal_stream(c);
  Scratch S{c, st};
  const size_t ib = (size_t)n_ifcs * sizeof(rsa_parse_ifc), sb = (size_t)n_spells * sizeof(rsa_parse_spell);
  TPCHK(c, hipMallocAsync(&S.base, ib + sb + 64, st));
  rsa_parse_ifc* d_ifcs = static_cast<rsa_parse_ifc*>(S.base);
  rsa_parse_spell* d_spells = reinterpret_cast<rsa_parse_spell*>(static_cast<char*>(S.base) + ib);
  if (ib) TPCHK(c, hipMemcpyAsync(d_ifcs, h_ifcs, ib, hipMemcpyHostToDevice, st));
  if (sb) TPCHK(c, hipMemcpyAsync(d_spells, h_spells, sb, hipMemcpyHostToDevice, st));
  TPCHK(c, hipStreamSynchronize(st));   // the host tables may go away after return
  if (reinterpret_cast<uintptr_t>(d_text) & 3u)
    return rsa_internal_fail(c, RSA_ERR_ARG, "rsa_parse_text: d_text must be 4-byte aligned");
  const uint64_t nb = (n_lines + kParseWG - 1) / kParseWG;
  if (nb > 0x7FFFFFFFull || n_lines > 0xFFFFFFFFull) return rsa_internal_fail(c, RSA_ERR_ARG, "too many lines");
  Scratch L{c, st};   // slow list: count, then the deferred line indices
  TPCHK(c, hipMallocAsync(&L.base, 16 + n_lines * 4, st));
  unsigned int* slow_n = static_cast<unsigned int*>(L.base);
  uint32_t* slow_idx = reinterpret_cast<uint32_t*>(static_cast<char*>(L.base) + 16);
  TPCHK(c, hipMemsetAsync(slow_n, 0, 4, st));
  // register-window reads need 16-byte aligned text; otherwise the lines are
  // staged in LDS (RSA_OPT_PARSE_STAGED forces that form, for its tests)
  if (!rsa_internal_parse_staged(c) && !(reinterpret_cast<uintptr_t>(d_text) & 15u))
    hipLaunchKernelGGL(k_parse_win, dim3((uint32_t)nb), dim3(kParseWG), 0, st, d_text, d_off, n_lines, d_ifcs, n_ifcs,
                       d_spells, n_spells, d_tuples, d_ts, d_disp, slow_idx, slow_n);
  else
    hipLaunchKernelGGL((k_parse<false>), dim3((uint32_t)nb), dim3(kParseWG), 0, st, d_text, d_off, n_lines, d_ifcs,
                       n_ifcs, d_spells, n_spells, d_tuples, d_ts, d_disp, slow_idx, slow_n);
  hipLaunchKernelGGL((k_parse_slow<false>), dim3((uint32_t)(nb < kSlowGrid ? nb : kSlowGrid)), dim3(kParseWG), 0, st,
                     d_text, d_off, n_lines, d_ifcs, n_ifcs, d_spells, n_spells, slow_idx, slow_n, d_tuples, d_ts,
                     d_disp);
  TPCHK(c, hipGetLastError());
  return RSA_OK;   // (the arenas are freed in stream order)
}

int rsa_parse_reduce(rsa_ctx* c, const uint8_t* d_text, const uint64_t* d_off, uint64_t n_lines,
                     const rsa_parse_spell* h_spells, uint32_t n_spells, rsa_tuple* d_tuples, uint32_t* d_ts,
                     uint32_t* d_disp) {
  if (!c || (n_lines && (!d_text || !d_off || !d_tuples || !d_ts || !d_disp))) return RSA_ERR_ARG;
  if (n_spells > 64 || (n_spells && !h_spells))
    return rsa_internal_fail(c, RSA_ERR_ARG, "rsa_parse_reduce: bad spelling table");
  for (uint32_t k = 0; k < n_spells; ++k)
    if (h_spells[k].len > 15) return rsa_internal_fail(c, RSA_ERR_ARG, "rsa_parse_reduce: spelling too long");
  if (!n_lines) return RSA_OK;
  if (reinterpret_cast<uintptr_t>(d_text) & 3u)
    return rsa_internal_fail(c, RSA_ERR_ARG, "rsa_parse_reduce: d_text must be 4-byte aligned");
  const uint64_t nb = (n_lines + kParseWG - 1) / kParseWG;
  if (nb > 0x7FFFFFFFull) return rsa_internal_fail(c, RSA_ERR_ARG, "too many lines");
  hipStream_t st = rsa_internal_stream(c);
  Scratch S{c, st};
  const size_t sb = (size_t)n_spells * sizeof(rsa_parse_spell);
  TPCHK(c, hipMallocAsync(&S.base, sb + 64, st));
  rsa_parse_spell* d_spells = static_cast<rsa_parse_spell*>(S.base);
  if (sb) TPCHK(c, hipMemcpyAsync(d_spells, h_spells, sb, hipMemcpyHostToDevice, st));
  TPCHK(c, hipStreamSynchronize(st));   // the host table may go away after return
  if (n_lines > 0xFFFFFFFFull) return rsa_internal_fail(c, RSA_ERR_ARG, "too many lines");
  Scratch L{c, st};   // slow list: count, then the deferred line indices
  TPCHK(c, hipMallocAsync(&L.base, 16 + n_lines * 4, st));
  unsigned int* slow_n = static_cast<unsigned int*>(L.base);
  uint32_t* slow_idx = reinterpret_cast<uint32_t*>(static_cast<char*>(L.base) + 16);
  TPCHK(c, hipMemsetAsync(slow_n, 0, 4, st));
  hipLaunchKernelGGL((k_parse<true>), dim3((uint32_t)nb), dim3(kParseWG), 0, st, d_text, d_off, n_lines, nullptr, 0u,
                     d_spells, n_spells, d_tuples, d_ts, d_disp, slow_idx, slow_n);
  hipLaunchKernelGGL((k_parse_slow<true>), dim3((uint32_t)(nb < kSlowGrid ? nb : kSlowGrid)), dim3(kParseWG), 0, st,
                     d_text, d_off, n_lines, nullptr, 0u, d_spells, n_spells, slow_idx, slow_n, d_tuples, d_ts, d_disp);
  TPCHK(c, hipGetLastError());
  return RSA_OK;   // (the arenas are freed in stream order)
}

int rsa_order_keys(rsa_ctx* c, const uint8_t* d_text, const uint64_t* d_off, uint64_t n_lines, uint64_t base,
                   uint64_t* d_order) {
  return rsa_order_keys_grouped(c, d_text, d_off, n_lines, nullptr, base, d_order);
}

int rsa_order_keys_grouped(rsa_ctx* c, const uint8_t* d_text, const uint64_t* d_off, uint64_t n_lines,
                           const int32_t* d_group, uint64_t base, uint64_t* d_order) {
  if (!c || (n_lines && (!d_text || !d_off || !d_order))) return RSA_ERR_ARG;
  if (n_lines >= 0x7FFFFFFFull) return rsa_internal_fail(c, RSA_ERR_ARG, "rsa_order_keys: too many lines");
  if (reinterpret_cast<uintptr_t>(d_text) & 3u)
    return rsa_internal_fail(c, RSA_ERR_ARG, "rsa_order_keys: d_text must be 4-byte aligned");
  if (!n_lines) return RSA_OK;
  hipStream_t st = rsa_internal_stream(c);
  const uint32_t n = (uint32_t)n_lines;
  unsigned gbits = 1;   // bits of a position (< n)
  while (gbits < 32 && (1ull << gbits) < (uint64_t)n) ++gbits;
  const size_t N = ((size_t)n + 63) / 64 * 64;
  const size_t H = rs_hist_len(N), SL = scan_sums_len(H > N ? H : N);
  // keysA/keysB/keysT u64, valsA/valsB/valsT u64, gs/ids/first/pos/bstart/keep/slot/lens u32,
  // act/act3 Act (and a spare), class depths cdep/cnext/cmin u32, radix histogram + scan sums, flag words
  const size_t bytes = N * (8 * 6 + 4 * 8 + sizeof(Act) * 3 + 4 * 5) + (H + SL) * 4 + 512;
  Scratch S{c, st};
  TPCHK(c, hipMallocAsync(&S.base, bytes, st));
  char* p = static_cast<char*>(S.base);
  uint64_t* keysA = reinterpret_cast<uint64_t*>(p); p += N * 8;
  uint64_t* keysB = reinterpret_cast<uint64_t*>(p); p += N * 8;
  uint64_t* keysT = reinterpret_cast<uint64_t*>(p); p += N * 8;
  uint64_t* valsA = reinterpret_cast<uint64_t*>(p); p += N * 8;
  uint64_t* valsB = reinterpret_cast<uint64_t*>(p); p += N * 8;
  uint64_t* valsT = reinterpret_cast<uint64_t*>(p); p += N * 8;
  uint32_t* gs = reinterpret_cast<uint32_t*>(p); p += N * 4;
  uint32_t* ids = reinterpret_cast<uint32_t*>(p); p += N * 4;
  uint32_t* first = reinterpret_cast<uint32_t*>(p); p += N * 4;
  uint32_t* pos = reinterpret_cast<uint32_t*>(p); p += N * 4;
  uint32_t* bstart = reinterpret_cast<uint32_t*>(p); p += N * 4;
  uint32_t* keep = reinterpret_cast<uint32_t*>(p); p += N * 4;
  uint32_t* slot = reinterpret_cast<uint32_t*>(p); p += N * 4;
  uint32_t* lens = reinterpret_cast<uint32_t*>(p); p += N * 4;
  Act* act = reinterpret_cast<Act*>(p); p += N * sizeof(Act);
  Act* act3 = reinterpret_cast<Act*>(p); p += N * sizeof(Act);
  Act* tie = reinterpret_cast<Act*>(p); p += N * sizeof(Act);       // finisher tie groups, by rank
  uint32_t* tkeep = reinterpret_cast<uint32_t*>(p); p += N * 4;   // ... their flags
  uint32_t* tdep = reinterpret_cast<uint32_t*>(p); p += N * 4;    // ... their depth, by class start
  uint32_t* cdep = reinterpret_cast<uint32_t*>(p); p += N * 4;    // per class start: bytes its lines share
  uint32_t* cnext = reinterpret_cast<uint32_t*>(p); p += N * 4;   // ... of the classes the next round forms
  uint32_t* cmin = reinterpret_cast<uint32_t*>(p); p += N * 4;    // per class start: k_lcp's further common bytes
  uint32_t* hist = reinterpret_cast<uint32_t*>(p); p += H * 4;
  uint32_t* sums = reinterpret_cast<uint32_t*>(p); p += SL * 4;
  uint32_t* flags = reinterpret_cast<uint32_t*>((reinterpret_cast<uintptr_t>(p) + 63) & ~(uintptr_t)63);
  uint32_t* idsA = reinterpret_cast<uint32_t*>(valsA);   // the first sort's values are u32 line ids
  uint32_t* idsB = reinterpret_cast<uint32_t*>(valsB);
  uint32_t* idsT = reinterpret_cast<uint32_t*>(valsT);
  // exclusive plus-scan of m flags (u32) into out; the count of set flags is out[m-1] + in[m-1]
  auto exscan = [&](const uint32_t* in, uint32_t* out, uint32_t m) {
    scan<OpPlus, false, uint32_t, uint32_t>(st, in, out, m, sums);
  };
  auto maxscan = [&](const uint32_t* in, uint32_t* out, uint32_t m) {
    scan<OpMax, true, uint32_t, uint32_t>(st, in, out, m, sums);
  };

  uint32_t* nl_bad = flags + 8;   // (set by k_grp0 / k_keys0: see note_nl)
  TPCHK(c, hipMemsetAsync(nl_bad, 0, 4, st));
  uint64_t n_bytes = 0;
  TPCHK(c, hipMemcpyAsync(&n_bytes, d_off + n, 8, hipMemcpyDeviceToHost, st));
  TPCHK(c, hipStreamSynchronize(st));
  uint32_t adv0 = 7;   // the depth of the classes the first stage leaves
  if (d_group) {
    // grouped: ranks of (group, line bytes); the groups come first (one sort
    // over the bits a group key has), so only lines of one group are ever
    // compared (the reducer compares order keys of one rule's lines only), and
    // a group of one line is settled at once.  Then the byte rounds from round 0.
    TPCHK(c, hipMemsetAsync(flags, 0, 4, st));
    hipLaunchKernelGGL(k_grp_max, dim3(blocks(n, kRedThreads) < kRedGrid ? blocks(n, kRedThreads) : kRedGrid),
                       dim3(kRedThreads), 0, st, d_group, n, flags);
    uint32_t gmax = 0;
    TPCHK(c, hipMemcpyAsync(&gmax, flags, 4, hipMemcpyDeviceToHost, st));
    TPCHK(c, hipStreamSynchronize(st));
    // group keys 0 .. gmax, a line without a group (-1) gmax + 1: last
    unsigned kbits = 1;
    while (kbits < 32 && (1ull << kbits) <= (uint64_t)gmax + 1) ++kbits;
    uint32_t* gkA = reinterpret_cast<uint32_t*>(keysA);
    uint32_t* gkB = reinterpret_cast<uint32_t*>(keysB);
    uint32_t* gkT = reinterpret_cast<uint32_t*>(keysT);
    hipLaunchKernelGGL(k_grp0, dim3(blocks(n, 256)), dim3(256), 0, st, d_group, d_text, d_off, n, gmax + 1, lens,
                       gkA, idsA, nl_bad);
    radix_pairs<uint32_t, uint32_t>(st, gkA, gkB, idsA, idsB, n, 0, kbits, gkT, idsT, hist, sums);
    hipLaunchKernelGGL(k_grp_bounds, dim3(blocks(n, 256)), dim3(256), 0, st, gkB, n, bstart);
    maxscan(bstart, first, n);
    hipLaunchKernelGGL(k_grp_settle, dim3(blocks(n, 256)), dim3(256), 0, st, gkB, idsB, first, n, gmax + 1, base,
                       d_order, keep);
    adv0 = 0;
  } else {
    // round 0: all lines
    hipLaunchKernelGGL(k_keys0, dim3(blocks(n, 256)), dim3(256), 0, st, d_text, d_off, n, n_bytes, lens, keysA, idsA,
                       nl_bad);
    radix_pairs<uint64_t, uint32_t>(st, keysA, keysB, idsA, idsB, n, 0, 64, keysT, idsT, hist, sums);
    hipLaunchKernelGGL(k_bounds, dim3(blocks(n, 256)), dim3(256), 0, st, keysB, (const uint32_t*)nullptr,
                       (const uint32_t*)nullptr, n, pos, bstart);
    maxscan(bstart, first, n);
    hipLaunchKernelGGL(k_settle, dim3(blocks(n, 256)), dim3(256), 0, st, keysB, (const uint32_t*)nullptr, idsB, pos,
                       first, n, base, d_order, keep);
  }
  exscan(keep, slot, n);
  hipLaunchKernelGGL(k_compact, dim3(blocks(n, 256)), dim3(256), 0, st, idsB, first, keep, slot, n, act,
                     (const uint32_t*)nullptr, (const uint32_t*)nullptr, (const uint32_t*)nullptr, cdep, adv0,
                     (const Act*)nullptr, d_off, (const uint32_t*)lens, n, (const uint32_t*)nl_bad);
  uint32_t m = 0, lastk = 0;
  TPCHK(c, hipMemcpyAsync(&m, slot + n - 1, 4, hipMemcpyDeviceToHost, st));
  TPCHK(c, hipMemcpyAsync(&lastk, keep + n - 1, 4, hipMemcpyDeviceToHost, st));
  TPCHK(c, hipStreamSynchronize(st));
  m += lastk;
  uint32_t* live = flags;   // [0] the round splits something, [1..2] the key bits that vary
  while (m > 0) {
    // the bytes every line of a class shares past its depth are skipped: the
    // window starts at the class's first differing byte (k_lcp); the window
    // keys; then the classes of at most kSmallClass lines are ranked here
    // (k_finish_small) and the others go on to the sort of their windows
    hipLaunchKernelGGL(k_cls_first, dim3(blocks(m, 256)), dim3(256), 0, st, act, m, bstart, cmin);
    maxscan(bstart, first, m);
    hipLaunchKernelGGL(k_lcp, dim3(blocks(m, 256)), dim3(256), 0, st, d_text, n_bytes, act, first, m, cdep, cmin,
                       keysT, valsT);
    hipLaunchKernelGGL(k_keys, dim3(blocks(m, 256)), dim3(256), 0, st, d_text, n_bytes, act, m, cdep, cmin,
                       (const uint64_t*)keysT, (const uint64_t*)valsT, keysB, valsB);
    hipLaunchKernelGGL(k_cls_size, dim3(blocks(m, 256)), dim3(256), 0, st, act, first, m, pos);
    hipLaunchKernelGGL(k_finish_small, dim3(blocks(m, kFinThreads)), dim3(kFinThreads), 0, st, act, keysB, first, pos,
                       m, cdep, cmin, base, d_order, keep, tie, tkeep, tdep);
    exscan(keep, slot, m);
    hipLaunchKernelGGL(k_compact_act, dim3(blocks(m, 256)), dim3(256), 0, st, act, keep, slot, m, act3, keysB, valsB,
                       keysA, valsA);
    exscan(tkeep, bstart, m);
    uint32_t nt = 0;
    {
      uint32_t nm = 0, lastt = 0;
      TPCHK(c, hipMemcpyAsync(&nm, slot + m - 1, 4, hipMemcpyDeviceToHost, st));
      TPCHK(c, hipMemcpyAsync(&lastk, keep + m - 1, 4, hipMemcpyDeviceToHost, st));
      TPCHK(c, hipMemcpyAsync(&nt, bstart + m - 1, 4, hipMemcpyDeviceToHost, st));
      TPCHK(c, hipMemcpyAsync(&lastt, tkeep + m - 1, 4, hipMemcpyDeviceToHost, st));
      TPCHK(c, hipStreamSynchronize(st));
      const uint32_t nb = nm + lastk;
      nt += lastt;
      // the tie groups behind the large classes (each group contiguous)
      if (nt) {
        hipLaunchKernelGGL(k_compact_act, dim3(blocks(m, 256)), dim3(256), 0, st, tie, tkeep, bstart, m, act3 + nb,
                           (const uint64_t*)nullptr, (const uint64_t*)nullptr, (uint64_t*)nullptr, (uint64_t*)nullptr);
        hipLaunchKernelGGL(k_tie_dep, dim3(blocks(nt, 256)), dim3(256), 0, st, act3 + nb, nt, tdep, cdep);
        // their windows: the common-prefix pass and keys over the tie groups alone
        hipLaunchKernelGGL(k_cls_first, dim3(blocks(nt, 256)), dim3(256), 0, st, act3 + nb, nt, bstart, cmin);
        maxscan(bstart, first, nt);
        hipLaunchKernelGGL(k_lcp, dim3(blocks(nt, 256)), dim3(256), 0, st, d_text, n_bytes, act3 + nb, first, nt, cdep,
                           cmin, keysT, valsT);
        hipLaunchKernelGGL(k_keys, dim3(blocks(nt, 256)), dim3(256), 0, st, d_text, n_bytes, act3 + nb, nt, cdep, cmin,
                           (const uint64_t*)keysT, (const uint64_t*)valsT, keysA + nb, valsA + nb);
      }
      m = nb + nt;
      Act* sw = act;
      act = act3;
      act3 = sw;
    }
    if (m == 0) break;
    // a window that splits nothing (only after a k_lcp capped at kLcpMax):
    // no sort; the sort of a live window runs over the key bits that vary only
    TPCHK(c, hipMemsetAsync(live, 0, 16, st));
    hipLaunchKernelGGL(k_round_live, dim3(blocks(m, kRedThreads) < kRedGrid ? blocks(m, kRedThreads) : kRedGrid),
                       dim3(kRedThreads), 0, st, keysA, act, m, live);
    uint32_t h_live[4] = {0, 0, 0, 0};
    TPCHK(c, hipMemcpyAsync(h_live, live, 16, hipMemcpyDeviceToHost, st));
    TPCHK(c, hipStreamSynchronize(st));
    if (!h_live[0]) {
      hipLaunchKernelGGL(k_dep_adv, dim3(blocks(m, 256)), dim3(256), 0, st, act, m, cdep, cmin, cnext);
      uint32_t* sw = cdep;
      cdep = cnext;
      cnext = sw;
      continue;
    }
    const bool sorted = h_live[3] != 0;
    if (!sorted) {
      // every class already in key order: no sort
      hipLaunchKernelGGL(k_split_vals, dim3(blocks(m, 256)), dim3(256), 0, st, valsA, m, gs, ids);
    } else {
      const uint64_t vary = (uint64_t)h_live[2] << 32 | h_live[1];
      const unsigned b0 = vary ? (unsigned)__builtin_ctzll(vary) : 0u;
      const unsigned b1 = vary ? 64u - (unsigned)__builtin_clzll(vary) : 0u;
      // stable LSD: by the chunk key, then by the group start
      radix_pairs<uint64_t, uint64_t>(st, keysA, keysB, valsA, valsB, m, b0, b1, keysT, valsT, hist, sums);
      hipLaunchKernelGGL(k_gs_iota, dim3(blocks(m, 256)), dim3(256), 0, st, valsB, m, gs, ids);
      // by group start (only the bits a position can have), carrying the index
      radix_pairs<uint32_t, uint32_t>(st, gs, first, ids, pos, m, 0, gbits, reinterpret_cast<uint32_t*>(keysT), idsT,
                                      hist, sums);
      hipLaunchKernelGGL(k_gather, dim3(blocks(m, 256)), dim3(256), 0, st, keysB, valsB, pos, m, keysA, gs, ids);
    }
    // now keysA / gs / ids are in (group start, chunk key) order
    hipLaunchKernelGGL(k_run_first, dim3(blocks(m, 256)), dim3(256), 0, st, gs, m, bstart);
    maxscan(bstart, first, m);
    hipLaunchKernelGGL(k_bounds, dim3(blocks(m, 256)), dim3(256), 0, st, keysA, gs, first, m, pos, bstart);
    maxscan(bstart, slot, m);
    hipLaunchKernelGGL(k_settle, dim3(blocks(m, 256)), dim3(256), 0, st, keysA, gs, ids, pos, slot, m, base, d_order,
                       keep);
    // slot (new group start + 1) is still needed by k_compact: scan the keep flags into `first`
    exscan(keep, first, m);
    // (unsorted: element j is act[j], its offset and length read in order;
    // sorted: gathered by line id)
    hipLaunchKernelGGL(k_compact, dim3(blocks(m, 256)), dim3(256), 0, st, ids, slot, keep, first, m, act3,
                       (const uint32_t*)gs, (const uint32_t*)cdep, (const uint32_t*)cmin, cnext, 7u,
                       sorted ? (const Act*)nullptr : (const Act*)act, d_off, (const uint32_t*)lens, n,
                       (const uint32_t*)nl_bad);
    {
      Act* swa = act;
      act = act3;
      act3 = swa;
    }
    uint32_t* sw = cdep;
    cdep = cnext;
    cnext = sw;
    uint32_t nm = 0;
    TPCHK(c, hipMemcpyAsync(&nm, first + m - 1, 4, hipMemcpyDeviceToHost, st));
    TPCHK(c, hipMemcpyAsync(&lastk, keep + m - 1, 4, hipMemcpyDeviceToHost, st));
    TPCHK(c, hipStreamSynchronize(st));
    m = nm + lastk;
  }
  TPCHK(c, hipGetLastError());
  return RSA_OK;
}

}  // extern "C"
