// Internal helpers shared by the libmirec.so translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include "../../include/mirec.h"

namespace mirec {

void set_error(const char* fmt, ...);

inline int hip_status(hipError_t e, const char* what) {
  if (e == hipSuccess) return 0;
  set_error("%s: %s", what, hipGetErrorString(e));
  return -(1000 + (int)e);
}

// Launch-time check: every kernel launch goes through this so a bad
// configuration is reported instead of silently dropped.
inline int launch_status(const char* what) {
  return hip_status(hipGetLastError(), what);
}

constexpr int kWave = 64;

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
  return x;
}

__device__ __forceinline__ int wave_sum_i(int x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
  return x;
}

// Block-wide exclusive scan of one int per thread (blockDim.x <= 1024,
// multiple of 64). `lds` needs blockDim.x/64 + 1 ints. Returns the exclusive
// prefix; *total gets the block sum. Contains __syncthreads(). Every lane reads
// the wave totals in one burst of LDS loads (no serial pass by one thread between
// two more barriers).
__device__ __forceinline__ int block_exclusive_scan(int x, int* lds, int* total) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  // inclusive scan within the wave
  int v = x;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    int y = __shfl_up(v, off, 64);
    if (lane >= off) v += y;
  }
  if (lane == 63) lds[wid] = v;
  __syncthreads();
  int pre = 0, tot = 0;
  for (int w = 0; w < nw; ++w) {
    const int t = lds[w];
    pre += w < wid ? t : 0;
    tot += t;
  }
  __syncthreads();                      // lds is reused by the next scan
  *total = tot;
  return pre + v - x;
}

// Binary search for `key` in sorted cols[lo, hi).
__device__ __forceinline__ bool sorted_contains(const int32_t* __restrict__ cols, int64_t lo,
                                                int64_t hi, int32_t key) {
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    int32_t c = cols[mid];
    if (c == key) return true;
    if (c < key) lo = mid + 1; else hi = mid;
  }
  return false;
}

}  // namespace mirec
