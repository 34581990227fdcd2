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

// Inclusive scan over the 64 lanes of a wave (every lane active): Hillis-Steele inside
// each 16-lane row with DPP row shifts (a lane whose source falls outside its row keeps
// 0), then the row totals (lanes 15, 31, 47) carried across rows with readlane. Four
// DPP adds and three readlanes — no LDS round trip (a __shfl_up is a ds_bpermute).
__device__ __forceinline__ int wave_inclusive_scan(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);   // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);   // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);   // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);   // row_shr:8
  const int r0 = __builtin_amdgcn_readlane(v, 15);
  const int r1 = __builtin_amdgcn_readlane(v, 31);
  const int r2 = __builtin_amdgcn_readlane(v, 47);
  const int row = (int)(threadIdx.x & 63) >> 4;
  return v + (row > 0 ? r0 : 0) + (row > 1 ? r1 : 0) + (row > 2 ? r2 : 0);
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
  const int v = wave_inclusive_scan(x);
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
