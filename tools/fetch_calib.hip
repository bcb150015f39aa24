// FETCH_SIZE calibration for the access shapes of the pass-1 kernels
// (MI355X_MICROARCH.md §HBM: FETCH_SIZE reads half the bytes of wide coalesced
// streaming reads; other widths are uncalibrated).  Each kernel reads a known
// number of bytes from a 2 GiB buffer (past the 256 MiB Infinity Cache):
//   k_stream16  16 B per lane, coalesced (k_classify's tuple loads)
//   k_seq32     32 B per lane, consecutive records (k_reduce's record reads)
//   k_rand32    32 B per lane at random record positions (k_part_scatter's gathers)
//   k_rand64    64 B per lane at random slot positions (k_reduce / k_emit slot reads)
// Run: rocprofv3 --pmc FETCH_SIZE -- tools/_build/fetch_calib; tools/fetch_calib.py
// turns the per-kernel FETCH_SIZE into bytes-per-known-byte factors.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
      return 1;                                                        \
    }                                                                  \
  } while (0)

__global__ void k_stream16(const uint4* __restrict__ a, uint64_t n16, unsigned long long* sink) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) atomicAdd(sink, 1ull);
}

__global__ void k_seq32(const uint4* __restrict__ a, uint64_t n32, unsigned long long* sink) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n32; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = a[2 * i], w = a[2 * i + 1];
    acc ^= v.x ^ v.y ^ w.z ^ w.w;
  }
  if (acc == 0x12345678u) atomicAdd(sink, 1ull);
}

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  return x;
}

// `count` reads of `words` uint4 at random positions (units of `words` uint4)
template <int kWords>
__global__ void k_rand(const uint4* __restrict__ a, uint64_t units, uint64_t count, unsigned long long* sink) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t u = mix(i * 0x9e3779b97f4a7c15ull) % units;
#pragma unroll
    for (int k = 0; k < kWords; ++k) {
      const uint4 v = a[u * kWords + k];
      acc ^= v.x ^ v.w;
    }
  }
  if (acc == 0x12345678u) atomicAdd(sink, 1ull);
}

int main() {
  const uint64_t bytes = 2ull << 30;
  uint4* a = nullptr;
  unsigned long long* sink = nullptr;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&sink, 8));
  CK(hipMemset(a, 1, bytes));
  const int grid = 256 * 8, block = 256;
  const uint64_t n16 = bytes / 16, n32 = bytes / 32, count = 32ull << 20;   // 32 Mi random reads
  k_stream16<<<grid, block>>>(a, n16, sink);
  k_seq32<<<grid, block>>>(a, n32, sink);
  k_rand<2><<<grid, block>>>(a, bytes / 32, count, sink);
  k_rand<4><<<grid, block>>>(a, bytes / 64, count, sink);
  CK(hipDeviceSynchronize());
  printf("{\"stream16_bytes\": %llu, \"seq32_bytes\": %llu, \"rand32_bytes\": %llu, \"rand64_bytes\": %llu}\n",
         (unsigned long long)bytes, (unsigned long long)bytes, (unsigned long long)(count * 32),
         (unsigned long long)(count * 64));
  CK(hipFree(a));
  CK(hipFree(sink));
  return 0;
}
