// Look-ahead lists of the deferred Adam (adam.hip): for consecutive batches b,
// b+1 of a chunk, out_b = uniq(b+1) \ uniq(b) in ascending order — the rows the
// next forward pass reads that step b's Adam does not touch. One workgroup per
// batch (any multiple of 64 lanes); uniq(b) is staged in LDS when it fits,
// membership by binary search. Shared by segsort.hip's launches and the K35 chunk
// preparation (step.hip).
#pragma once
#include "common.h"

namespace mirec {

constexpr int kDiffLds = 8192;

__device__ __forceinline__ void uniq_ahead_diff_batch(
    const int32_t* __restrict__ uniq, const int32_t* __restrict__ n_uniq, int64_t stride,
    int64_t n_batches, int32_t* __restrict__ out, int32_t* __restrict__ n_out, int64_t b,
    int32_t* a_lds, int* scan_lds) {
  if (b + 1 >= n_batches) {                 // last batch of the chunk: nothing ahead
    if (threadIdx.x == 0) n_out[b] = 0;
    return;
  }
  const int32_t* __restrict__ A = uniq + b * stride;
  const int32_t* __restrict__ Bv = uniq + (b + 1) * stride;
  const int na = n_uniq[b], nb = n_uniq[b + 1];
  const bool lds = na <= kDiffLds;
  if (lds)
    for (int i = threadIdx.x; i < na; i += blockDim.x) a_lds[i] = A[i];
  __syncthreads();
  const int32_t* S = lds ? a_lds : A;
  int32_t* __restrict__ o = out + b * stride;
  int base = 0;
  for (int c0 = 0; c0 < nb; c0 += blockDim.x) {
    const int i = c0 + threadIdx.x;
    int f = 0;
    int32_t x = 0;
    if (i < nb) {
      x = Bv[i];
      int lo = 0, hi = na;
      while (lo < hi) { const int mid = (lo + hi) >> 1; if (S[mid] < x) lo = mid + 1; else hi = mid; }
      f = (lo < na && S[lo] == x) ? 0 : 1;
    }
    int tot;
    const int ex = block_exclusive_scan(f, scan_lds, &tot);
    if (f) o[base + ex] = x;
    base += tot;
  }
  if (threadIdx.x == 0) n_out[b] = base;
}

}  // namespace mirec
