// K2 — deterministic grouping of gradient contributions by table row.
//
// torch's nn.Embedding(sparse=False) backward (bpr.py:40-41) zero-fills a dense
// [n_rows, d] gradient and index_adds every looked-up row into it.  Here the
// contributions are grouped instead: a stable LSD radix sort of (row id,
// contribution index) gives, per distinct row, the ordered list of its
// contributions, which K5 (adam.hip) or the dense scatter below sums in that
// fixed order — bitwise reproducible, no float atomics.
//
// The sort runs in ONE workgroup (1024 lanes): n is a training batch's
// contribution count (C2: 512 user keys, 2,560 item keys), far too small to
// fill the chip, and the sort depends only on ids, so the trainer runs it
// ahead of the model step on a side stream.  Up to kLdsMax keys the whole
// sort lives in LDS (1-bit stable splits, one block scan per bit); larger n
// uses the same algorithm over global ping-pong buffers.
#include "common.h"

namespace mirec {

constexpr int kSortThreads = 1024;
constexpr int kLdsMax = 8192;
constexpr int kIpt = kLdsMax / kSortThreads;  // items per thread in the LDS path

__device__ __forceinline__ int nbits_for(int64_t key_space) {
  int b = 0;
  while (b < 31 && ((int64_t)1 << b) < key_space) ++b;
  return b;
}

// uniq/seg from sorted keys held in `skey` (LDS or global), blocked arrangement
template <typename KeyPtr>
__device__ void emit_segments(KeyPtr skey, int n, int32_t* __restrict__ uniq,
                              int32_t* __restrict__ seg, int32_t* __restrict__ n_uniq,
                              int* scan_lds) {
  int base_u = 0;
  for (int c0 = 0; c0 < n; c0 += kSortThreads) {
    const int i = c0 + threadIdx.x;
    int f = 0;
    int32_t kv = 0;
    if (i < n) {
      kv = skey[i];
      f = (i == 0 || skey[i - 1] != kv) ? 1 : 0;
    }
    int tot;
    const int ex = block_exclusive_scan(f, scan_lds, &tot);
    if (f) {
      uniq[base_u + ex] = kv;
      seg[base_u + ex] = i;
    }
    base_u += tot;
  }
  if (threadIdx.x == 0) {
    seg[base_u] = n;
    n_uniq[0] = base_u;
  }
}

// One workgroup per batch: batch b sorts keys[b*batch_n, min((b+1)*batch_n, n_total))
// and writes perm/uniq at b*batch_n, seg at b*(batch_n+1), n_uniq[b].
__global__ __launch_bounds__(kSortThreads) void segsort_lds_kernel(
    const int64_t* __restrict__ keys_all, int64_t n_total, int batch_n, int nbits,
    int32_t* __restrict__ perm_all, int32_t* __restrict__ uniq_all,
    int32_t* __restrict__ seg_all, int32_t* __restrict__ n_uniq_all) {
  __shared__ int32_t kA[kLdsMax], vA[kLdsMax], kB[kLdsMax], vB[kLdsMax];
  __shared__ int scan_lds[kSortThreads / 64 + 1];
  const int64_t b = blockIdx.x;
  const int n = (int)min((int64_t)batch_n, n_total - b * batch_n);
  const int64_t* __restrict__ keys = keys_all + b * batch_n;
  int32_t* __restrict__ perm = perm_all + b * batch_n;
  int32_t* __restrict__ uniq = uniq_all + b * batch_n;
  int32_t* __restrict__ seg = seg_all + b * (batch_n + 1);
  int32_t* __restrict__ n_uniq = n_uniq_all + b;
  for (int i = threadIdx.x; i < n; i += kSortThreads) {
    kA[i] = (int32_t)keys[i];
    vA[i] = i;
  }
  __syncthreads();
  int32_t *ks = kA, *vs = vA, *kd = kB, *vd = vB;
  const int ipt = (n + kSortThreads - 1) / kSortThreads;
  const int lo = threadIdx.x * ipt;
  const int hi = min(n, lo + ipt);
  for (int bit = 0; bit < nbits; ++bit) {
    int z = 0;
    for (int i = lo; i < hi; ++i) z += ((ks[i] >> bit) & 1) ? 0 : 1;
    int Z;
    const int ez = block_exclusive_scan(z, scan_lds, &Z);
    int zb = ez;  // zeros before element i
    for (int i = lo; i < hi; ++i) {
      const int32_t kv = ks[i];
      const int one = (kv >> bit) & 1;
      const int dst = one ? (Z + (i - zb)) : zb;
      kd[dst] = kv;
      vd[dst] = vs[i];
      zb += 1 - one;
    }
    __syncthreads();
    int32_t* t;
    t = ks; ks = kd; kd = t;
    t = vs; vs = vd; vd = t;
  }
  for (int i = threadIdx.x; i < n; i += kSortThreads) perm[i] = vs[i];
  emit_segments(ks, n, uniq, seg, n_uniq, scan_lds);
}

// Same algorithm, global ping-pong buffers, processed in chunks of
// kSortThreads*kIpt with running offsets (any n up to INT32_MAX).
__global__ __launch_bounds__(kSortThreads) void segsort_global_kernel(
    const int64_t* __restrict__ keys_all, int64_t n_total, int batch_n, int nbits,
    int32_t* __restrict__ perm_all, int32_t* __restrict__ uniq_all,
    int32_t* __restrict__ seg_all, int32_t* __restrict__ n_uniq_all, int32_t* __restrict__ ws) {
  __shared__ int scan_lds[kSortThreads / 64 + 1];
  const int64_t b = blockIdx.x;
  const int n = (int)min((int64_t)batch_n, n_total - b * batch_n);
  const int64_t* __restrict__ keys = keys_all + b * batch_n;
  int32_t* __restrict__ perm = perm_all + b * batch_n;
  int32_t* __restrict__ uniq = uniq_all + b * batch_n;
  int32_t* __restrict__ seg = seg_all + b * (batch_n + 1);
  int32_t* __restrict__ n_uniq = n_uniq_all + b;
  int32_t* kA = ws + b * 4 * (int64_t)batch_n;
  int32_t* vA = kA + batch_n;
  int32_t* kB = vA + batch_n;
  int32_t* vB = kB + batch_n;
  for (int i = threadIdx.x; i < n; i += kSortThreads) {
    kA[i] = (int32_t)keys[i];
    vA[i] = i;
  }
  __syncthreads();
  int32_t *ks = kA, *vs = vA, *kd = kB, *vd = vB;
  constexpr int CH = kSortThreads * kIpt;
  for (int bit = 0; bit < nbits; ++bit) {
    // total zeros
    int zloc = 0;
    for (int i = threadIdx.x; i < n; i += kSortThreads) zloc += ((ks[i] >> bit) & 1) ? 0 : 1;
    int Z;
    (void)block_exclusive_scan(zloc, scan_lds, &Z);
    int zrun = 0;  // zeros in earlier chunks
    for (int c0 = 0; c0 < n; c0 += CH) {
      const int lo = c0 + threadIdx.x * kIpt;
      const int hi = min(n, lo + kIpt);
      int z = 0;
      for (int i = lo; i < hi; ++i) z += ((ks[i] >> bit) & 1) ? 0 : 1;
      int zc;
      const int ez = block_exclusive_scan(z, scan_lds, &zc);
      int zb = zrun + ez;
      for (int i = lo; i < hi; ++i) {
        const int32_t kv = ks[i];
        const int one = (kv >> bit) & 1;
        const int dst = one ? (Z + (i - zb)) : zb;
        kd[dst] = kv;
        vd[dst] = vs[i];
        zb += 1 - one;
      }
      zrun += zc;
    }
    __threadfence_block();
    __syncthreads();
    int32_t* t;
    t = ks; ks = kd; kd = t;
    t = vs; vs = vd; vd = t;
  }
  for (int i = threadIdx.x; i < n; i += kSortThreads) perm[i] = vs[i];
  __syncthreads();
  emit_segments(ks, n, uniq, seg, n_uniq, scan_lds);
}

// Dense scatter of grouped sums (autograd-compatible path): one wave per
// distinct row, lanes over the row's columns, contributions in fixed order.
__global__ __launch_bounds__(256) void segment_scatter_add_kernel(
    const float* __restrict__ rows, int d, const int32_t* __restrict__ perm,
    const int32_t* __restrict__ uniq, const int32_t* __restrict__ seg,
    const int32_t* __restrict__ n_uniq_dev, float* __restrict__ dense, int64_t n_rows) {
  const int nu = n_uniq_dev[0];
  const int lane = threadIdx.x & 63;
  for (int u = blockIdx.x * 4 + (threadIdx.x >> 6); u < nu; u += gridDim.x * 4) {
    const int64_t row = uniq[u];
    if (row < 0 || row >= n_rows) continue;
    const int s0 = seg[u], s1 = seg[u + 1];
    for (int c = lane; c < d; c += 64) {
      float acc = 0.f;
      for (int i = s0; i < s1; ++i) acc += rows[(int64_t)perm[i] * d + c];
      dense[row * d + c] += acc;
    }
  }
}

}  // namespace mirec

using namespace mirec;

extern "C" size_t mirec_segment_sort_workspace_size(int64_t n, int64_t key_space) {
  (void)key_space;
  if (n <= kLdsMax) return 256;
  return (size_t)4 * (size_t)n * sizeof(int32_t) + 256;
}

extern "C" int mirec_segment_sort_batched(const int64_t* keys, int64_t n, int64_t batch_n,
                                          int64_t key_space, int32_t* perm, int32_t* uniq,
                                          int32_t* seg, int32_t* n_uniq_dev, void* ws,
                                          size_t ws_bytes, void* stream) {
  if (n < 0 || key_space <= 0 || key_space > INT32_MAX || n > INT32_MAX || batch_n < 0 ||
      !seg || !n_uniq_dev || (n > 0 && (!keys || !perm || !uniq || batch_n == 0))) {
    set_error("mirec_segment_sort: bad arguments");
    return -1;
  }
  hipStream_t st = (hipStream_t)stream;
  int nb = 0;
  while (nb < 31 && ((int64_t)1 << nb) < key_space) ++nb;
  if (n == 0) {  // one empty batch: seg[0] = 0, n_uniq = 0
    hipLaunchKernelGGL(segsort_lds_kernel, dim3(1), dim3(kSortThreads), 0, st, keys, (int64_t)0,
                       1, nb, perm, uniq, seg, n_uniq_dev);
    return launch_status("mirec_segment_sort");
  }
  const int64_t n_batches = (n + batch_n - 1) / batch_n;
  if (batch_n <= kLdsMax) {
    hipLaunchKernelGGL(segsort_lds_kernel, dim3((unsigned)n_batches), dim3(kSortThreads), 0, st,
                       keys, n, (int)batch_n, nb, perm, uniq, seg, n_uniq_dev);
  } else {
    const size_t need = (size_t)4 * (size_t)(n_batches * batch_n) * sizeof(int32_t);
    if (!ws || ws_bytes < need) {
      set_error("mirec_segment_sort: workspace %zu < %zu", ws_bytes, need);
      return -1;
    }
    hipLaunchKernelGGL(segsort_global_kernel, dim3((unsigned)n_batches), dim3(kSortThreads), 0,
                       st, keys, n, (int)batch_n, nb, perm, uniq, seg, n_uniq_dev,
                       (int32_t*)ws);
  }
  return launch_status("mirec_segment_sort");
}

extern "C" int mirec_segment_sort(const int64_t* keys, int64_t n, int64_t key_space,
                                  int32_t* perm, int32_t* uniq, int32_t* seg,
                                  int32_t* n_uniq_dev, void* ws, size_t ws_bytes, void* stream) {
  return mirec_segment_sort_batched(keys, n, n > 0 ? n : 1, key_space, perm, uniq, seg,
                                    n_uniq_dev, ws, ws_bytes, stream);
}

extern "C" int mirec_segment_scatter_add_f32(const float* rows, int32_t d, const int32_t* perm,
                                             const int32_t* uniq, const int32_t* seg,
                                             const int32_t* n_uniq_dev, int64_t n_max_uniq,
                                             float* dense, int64_t n_rows, void* stream) {
  if (n_max_uniq == 0) return 0;
  if (!rows || !perm || !uniq || !seg || !n_uniq_dev || !dense || d <= 0 || n_max_uniq < 0) {
    set_error("mirec_segment_scatter_add_f32: bad arguments");
    return -1;
  }
  int64_t g = (n_max_uniq + 3) / 4;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(segment_scatter_add_kernel, dim3((unsigned)g), dim3(256), 0,
                     (hipStream_t)stream, rows, d, perm, uniq, seg, n_uniq_dev, dense, n_rows);
  return launch_status("mirec_segment_scatter_add_f32");
}

// ---------------------------------------------------------------------------
// Look-ahead lists of the deferred Adam (adam.hip): for consecutive batches b,
// b+1 of a chunk, out_b = uniq(b+1) \ uniq(b) in ascending order — the rows the
// next forward pass reads that step b's Adam does not touch. One workgroup per
// batch; uniq(b) is staged in LDS when it fits, membership by binary search.
namespace mirec {

constexpr int kDiffLds = 8192;

__global__ __launch_bounds__(kSortThreads) void uniq_ahead_diff_kernel(
    const int32_t* __restrict__ uniq, const int32_t* __restrict__ n_uniq, int64_t stride,
    int64_t n_batches, int32_t* __restrict__ out, int32_t* __restrict__ n_out) {
  __shared__ int32_t a_lds[kDiffLds];
  __shared__ int scan_lds[kSortThreads / 64 + 1];
  const int64_t b = blockIdx.x;
  if (b + 1 >= n_batches) {                 // last batch of the chunk: nothing ahead
    if (threadIdx.x == 0) n_out[b] = 0;
    return;
  }
  const int32_t* __restrict__ A = uniq + b * stride;
  const int32_t* __restrict__ Bv = uniq + (b + 1) * stride;
  const int na = n_uniq[b], nb = n_uniq[b + 1];
  const bool lds = na <= kDiffLds;
  if (lds)
    for (int i = threadIdx.x; i < na; i += kSortThreads) a_lds[i] = A[i];
  __syncthreads();
  const int32_t* S = lds ? a_lds : A;
  int32_t* __restrict__ o = out + b * stride;
  int base = 0;
  for (int c0 = 0; c0 < nb; c0 += kSortThreads) {
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

extern "C" int mirec_uniq_ahead_diff(const int32_t* uniq, const int32_t* n_uniq, int64_t stride,
                                     int64_t n_batches, int32_t* out, int32_t* n_out,
                                     void* stream) {
  if (!uniq || !n_uniq || !out || !n_out || stride <= 0 || n_batches < 0) {
    mirec::set_error("mirec_uniq_ahead_diff: bad arguments");
    return -1;
  }
  if (n_batches == 0) return 0;
  hipLaunchKernelGGL(mirec::uniq_ahead_diff_kernel, dim3((unsigned)n_batches),
                     dim3(mirec::kSortThreads), 0, (hipStream_t)stream, uniq, n_uniq, stride,
                     n_batches, out, n_out);
  return mirec::launch_status("mirec_uniq_ahead_diff");
}
