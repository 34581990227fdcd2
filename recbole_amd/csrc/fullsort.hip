// K6 — full-sort evaluator: user x all-items scores on FP32 MFMA, fused with
// the pad/history mask, a per-user top-K and the positive test, so the
// [users x items] score matrix never exists in HBM.
//
// Restates, for one batch of users:
//   BPR.full_sort_predict          scores = U[u] @ E_I^T       (bpr.py:91-96)
//   Trainer._full_sort_batch_eval  [:,0] = -inf; [history] = -inf;
//                                  positives swapped into columns [0,pos_len)
//                                                              (trainer.py:328-353)
//   TopKEvaluator.collect          flip(-1) + topk(max(topk))  (evaluators.py:53-76)
//   _calculate_metrics             pos_idx = topk_idx >= I - pos_len (:134)
// The swap + flip only relabel columns so that "index >= I - pos_len" means
// "is a positive": per item the (score, is_positive) pair is unchanged, so the
// result is the K best unmasked items and, per rank, whether it is a positive.
// Ties are broken by (score desc, item id asc); torch.topk leaves tie order
// unspecified, so tied scores are the one place results may legitimately differ.
//
// Tiling (gfx950, wave64): a workgroup = 4 waves = 128 users. Each wave keeps
// its 32 users' embedding in registers as the MFMA B operand
// (v_mfma_f32_32x32x2_f32: lane l holds B[k][j = l&31]) and sweeps all items in
// tiles of 32 staged once per workgroup in LDS (rows padded to D+2 floats so the
// ds_read_b64 A-fragment reads are conflict-free). The 32x32 accumulator puts one
// USER per lane column and 16 ITEMS per lane, so each lane keeps a private
// register top-K for its user over its half of the items (no cross-lane traffic in
// the sweep); the two halves merge at the end. The k order inside the dot product
// is permuted (k = 4*(s>>1) + 2h + (s&1)) so both operands load as float2; the
// MFMA result is an exact-f32 fma chain in that order.
#include "common.h"

namespace mirec {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kFsThreads = 256;

// Sorted insert into a best-first register list, branch-free (v_cndmask only;
// bitwise |/& on the predicates so clang emits no exec-mask branches).
// Scan form: strict '>' — each lane visits its items in increasing id order,
// so an equal score arriving later (higher id) correctly ranks after.
template <int KC>
__device__ __forceinline__ void topk_insert(float (&ts)[KC], int (&ti)[KC], float v, int id) {
#pragma unroll
  for (int t = KC - 1; t > 0; --t) {
    const bool up = v > ts[t - 1];
    const bool here = v > ts[t];
    const float ns = up ? ts[t - 1] : (here ? v : ts[t]);
    const int ni = up ? ti[t - 1] : (here ? id : ti[t]);
    ts[t] = ns;
    ti[t] = ni;
  }
  const bool h0 = v > ts[0];
  ts[0] = h0 ? v : ts[0];
  ti[0] = h0 ? id : ti[0];
}

// Merge form: full order (score desc, id asc) for combining two lanes' lists.
template <int KC>
__device__ __forceinline__ void topk_merge_insert(float (&ts)[KC], int (&ti)[KC], float v,
                                                  int id) {
#pragma unroll
  for (int t = KC - 1; t > 0; --t) {
    const bool up = (v > ts[t - 1]) | ((v == ts[t - 1]) & (id < ti[t - 1]));
    const bool here = (v > ts[t]) | ((v == ts[t]) & (id < ti[t]));
    const float ns = up ? ts[t - 1] : (here ? v : ts[t]);
    const int ni = up ? ti[t - 1] : (here ? id : ti[t]);
    ts[t] = ns;
    ti[t] = ni;
  }
  const bool h0 = (v > ts[0]) | ((v == ts[0]) & (id < ti[0]));
  ts[0] = h0 ? v : ts[0];
  ti[0] = h0 ? id : ti[0];
}

// Stage items [base, base+32) of EI into LDS rows of LDR floats (zero past I).
template <int D>
__device__ __forceinline__ void stage_tile(const float* __restrict__ EI, int64_t I, int64_t base,
                                           float* __restrict__ tile) {
  constexpr int LDR = D + 2;
  constexpr int V4 = D / 4;
  const float4* __restrict__ E4 = reinterpret_cast<const float4*>(EI);
#pragma unroll
  for (int f = threadIdx.x; f < 32 * V4; f += kFsThreads) {
    const int row = f / V4;
    const int c4 = f - row * V4;
    const int64_t item = base + row;
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
    if (item < I) x = E4[item * V4 + c4];
    float2* dst = reinterpret_cast<float2*>(tile + row * LDR + 4 * c4);
    dst[0] = make_float2(x.x, x.y);
    dst[1] = make_float2(x.z, x.w);
  }
}

// lane (j = l&31, h = l>>5) holds user row q's elements in the permuted k order
template <int D>
__device__ __forceinline__ void load_user_operand(const float* __restrict__ Uq, int64_t q, bool qv,
                                                  int h, float (&ub)[D / 2]) {
#pragma unroll
  for (int s2 = 0; s2 < D / 4; ++s2) {
    float2 x = make_float2(0.f, 0.f);
    if (qv) x = *reinterpret_cast<const float2*>(Uq + q * D + 4 * s2 + 2 * h);
    ub[2 * s2] = x.x;
    ub[2 * s2 + 1] = x.y;
  }
}

// NT = 32-item sub-tiles per staged tile: NT = 2 (64 items) for D <= 128 — two
// independent MFMA accumulators per wave (the chains interleave) and one workgroup
// barrier per 64 items instead of per 32: at D = 128 a 32-item tile is only 64 MFMAs
// per wave between barriers.
template <int D> struct FsSub { static constexpr int n = D <= 128 ? 2 : 1; };

template <int D, int KC>
// Two waves per SIMD (<= 256 VGPRs, no spills for D <= 128): the second wave's
// VALU top-K work overlaps the first one's MFMAs — measured 1.43x over one wave
// per SIMD at C2 (21.6 -> 15.0 ms). D = 256 keeps one (its user operand alone
// takes 128 VGPRs).
#ifndef MIREC_FS_WAVES_PER_EU
#define MIREC_FS_WAVES_PER_EU(D) ((D) <= 128 ? 2 : 1)
#endif
__global__ __launch_bounds__(kFsThreads, MIREC_FS_WAVES_PER_EU(D)) void fullsort_topk_kernel(
    const float* __restrict__ Uq, int64_t nq, const float* __restrict__ EI, int64_t I,
    const int64_t* __restrict__ hist_ptr, const int32_t* __restrict__ hist_cols,
    const int64_t* __restrict__ pos_ptr, const int32_t* __restrict__ pos_cols, int K,
    float* __restrict__ top_scores, int32_t* __restrict__ top_ids,
    uint8_t* __restrict__ pos_flags, int64_t span) {
  constexpr int LDR = D + 2;
  constexpr int V4 = D / 4;
  constexpr int NT = FsSub<D>::n;                                 // 32-item sub-tiles per tile
  constexpr int TI = 32 * NT;                                     // items per tile
  constexpr int NPF = (TI * V4 + kFsThreads - 1) / kFsThreads;    // float4 per thread per tile
  // item split (gridDim.y > 1): this workgroup sweeps items [ilo, ihi) and writes its
  // partial lists (merged by fullsort_merge_kernel); span is a multiple of TI
  const bool split = gridDim.y > 1;
  const int64_t ilo = (int64_t)blockIdx.y * span;
  const int64_t ihi = min(I, ilo + span);
  __shared__ __attribute__((aligned(16))) float tile[2][TI * LDR];
  __shared__ uint32_t hmask[2][NT][128];   // history bits of the WG's 128 users over one tile
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int j = lane & 31;
  const int h = lane >> 5;
  const int64_t q = ((int64_t)blockIdx.x * 4 + w) * 32 + j;
  const bool qv = q < nq;

  float ub[D / 2];
  load_user_operand<D>(Uq, q, qv, h, ub);

  float ts[KC];
  int ti[KC];
#pragma unroll
  for (int t = 0; t < KC; ++t) { ts[t] = -INFINITY; ti[t] = -1; }
  float thr = -INFINITY;

  // History cursor, one per user, owned by thread u < 128 of the workgroup:
  // `hnext` is the user's next history item >= the current tile; a tile's mask
  // only loads when it actually consumes an entry (~deg/ntile per tile).
  const int64_t qu = (int64_t)blockIdx.x * 128 + threadIdx.x;
  int64_t hcur = 0, hend = 0;
  int64_t hnext = INT64_MAX;
  if (threadIdx.x < 128 && qu < nq && hist_ptr) {
    hcur = hist_ptr[qu];
    hend = hist_ptr[qu + 1];
    if (ilo > 0) {                          // sorted: lower_bound of the split's first item
      int64_t a = hcur, b = hend;
      while (a < b) {
        const int64_t mid = (a + b) >> 1;
        if (hist_cols[mid] < ilo) a = mid + 1; else b = mid;
      }
      hcur = a;
    }
    if (hcur < hend) hnext = hist_cols[hcur];
  }
  auto build_mask = [&](int64_t base, uint32_t (*dst)[128]) {
    if (threadIdx.x < 128) {
#pragma unroll
      for (int sub = 0; sub < NT; ++sub) {
        const int64_t b0 = base + 32 * sub;
        uint32_t msk = 0;
        while (hnext < b0 + 32) {
          msk |= 1u << (uint32_t)(hnext - b0);
          ++hcur;
          hnext = hcur < hend ? (int64_t)hist_cols[hcur] : INT64_MAX;
        }
        dst[sub][threadIdx.x] = msk;
      }
    }
  };

  const float4* __restrict__ E4 = reinterpret_cast<const float4*>(EI);
  // the next tile in flight in PH = NT parts (one sub-tile's worth of registers at a
  // time: part p stored to LDS when sub-tile p + 1 starts, the next part issued)
  constexpr int PH = NT;
  constexpr int NPP = (NPF + PH - 1) / PH;
  float4 pf[NPP];
  auto load_tile = [&](int64_t base, int part = 0) {
#pragma unroll
    for (int kk = 0; kk < NPP; ++kk) {
      const int k = part * NPP + kk;
      const int f = threadIdx.x + k * kFsThreads;
      const int row = f / V4;
      const int c4 = f - row * V4;
      const int64_t item = base + row;
      pf[kk] = (k < NPF && f < TI * V4 && item < I) ? E4[item * V4 + c4]
                                                     : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_tile = [&](float* dst, int part = 0) {
#pragma unroll
    for (int kk = 0; kk < NPP; ++kk) {
      const int k = part * NPP + kk;
      const int f = threadIdx.x + k * kFsThreads;
      if (k < NPF && f < TI * V4) {
        const int row = f / V4;
        const int c4 = f - row * V4;
        float2* p = reinterpret_cast<float2*>(dst + row * LDR + 4 * c4);
        p[0] = make_float2(pf[kk].x, pf[kk].y);
        p[1] = make_float2(pf[kk].z, pf[kk].w);
      }
    }
  };

  const int64_t ntile = (ihi - ilo + TI - 1) / TI;
#pragma unroll
  for (int part = 0; part < PH; ++part) {
    load_tile(ilo, part);
    store_tile(tile[0], part);
  }
  build_mask(ilo, hmask[0]);
  __syncthreads();
  int cur = 0;
  const int ul = w * 32 + j;   // this lane's user within the workgroup
  for (int64_t t = 0; t < ntile; ++t) {
    const int64_t base = ilo + t * TI;
    const bool more = t + 1 < ntile;
    if (more) load_tile(base + TI, 0);       // global loads in flight under the MFMAs
    // the sub-tiles one after the other (one accumulator: the registers of the
    // 32-item form), one workgroup barrier per tile
#pragma unroll 1
    for (int sub = 0; sub < NT; ++sub) {
      if (sub > 0 && more) {                   // a part of the next tile to LDS, the next part
        store_tile(tile[cur ^ 1], sub - 1);    // in flight
        load_tile(base + TI, sub);
      }
      floatx16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      const float* arow = tile[cur] + (32 * sub + j) * LDR + 2 * h;
#pragma unroll
      for (int s2 = 0; s2 < D / 4; ++s2) {
        const float2 a = *reinterpret_cast<const float2*>(arow + 4 * s2);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, ub[2 * s2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, ub[2 * s2 + 1], acc, 0, 0, 0);
      }
      // Rows of this lane that can enter its list: valid item, not pad, not history.
      // C[item row][user col]: rows (r&3) + 8*(r>>2) + 4h
      const int64_t sb = base + 32 * sub;
      const uint32_t hm = hmask[cur][sub][ul];
      uint32_t ok = 0;
      float best = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        const int64_t item = sb + row;
        const bool valid = qv & (item < ihi) & (item != 0) & !((hm >> row) & 1u);
        ok |= (valid ? 1u : 0u) << r;
        best = fmaxf(best, valid ? acc[r] : -INFINITY);
      }
      // The two lanes of a user scan disjoint item halves; an item below the
      // partner's K-th best already has K better items, so it can never reach the
      // final (merged) top-K: filter with the stronger of the two thresholds.
      thr = fmaxf(thr, __shfl_xor(thr, 32, 64));
#ifdef MIREC_FS_NO_TOPK   // profiling variant (tools/build_variant.sh): MFMA + mask only
      thr = fmaxf(thr, best);
      if (false) {
#else
      if (__any(best > thr)) {             // wave-uniform: rare once the lists fill up
#endif
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
          const float sc = acc[r];
          if (((ok >> r) & 1u) && sc > thr) {
            topk_insert<KC>(ts, ti, sc, (int)(sb + row));
            thr = fmaxf(thr, ts[KC - 1]);
          }
        }
      }
    }
    if (more) {
      build_mask(base + TI, hmask[cur ^ 1]);
      store_tile(tile[cur ^ 1], PH - 1);
    }
    __syncthreads();
    cur ^= 1;
  }

#ifdef MIREC_FS_NO_TOPK
  ts[0] = thr;   // keep the scores live in the profiling variant
#endif
  // merge the two item halves of each user: lane j takes lane j+32's list
#pragma unroll
  for (int t = 0; t < KC; ++t) {
    const float os = __shfl(ts[t], j + 32, 64);
    const int oi = __shfl(ti[t], j + 32, 64);
    if (h == 0) topk_merge_insert<KC>(ts, ti, os, oi);
  }
  if (h == 0 && qv && split) {             // partial lists of this item range
#pragma unroll
    for (int t = 0; t < KC; ++t) {
      if (t < K) {
        const int64_t o = ((int64_t)blockIdx.y * nq + q) * K + t;
        top_scores[o] = ts[t];
        top_ids[o] = ti[t];
      }
    }
  }
  if (h == 0 && qv && !split) {
    const int64_t p0 = pos_ptr ? pos_ptr[q] : 0;
    const int64_t p1 = pos_ptr ? pos_ptr[q + 1] : 0;
#pragma unroll
    for (int t = 0; t < KC; ++t) {
      if (t < K) {
        const int64_t o = q * K + t;
        if (top_scores) top_scores[o] = ts[t];
        if (top_ids) top_ids[o] = ti[t];
        if (pos_flags)
          pos_flags[o] = (ti[t] >= 0 && sorted_contains(pos_cols, p0, p1, ti[t])) ? 1 : 0;
      }
    }
  }
}

// Merge of the item-split partial lists: per user, the K best of the S lists by
// (score desc, id asc) — the same total order as one sweep, so the same top-K.
template <int KC>
__global__ __launch_bounds__(256) void fullsort_merge_kernel(
    int64_t nq, int S, int K, const float* __restrict__ ps, const int32_t* __restrict__ pi,
    const int64_t* __restrict__ pos_ptr, const int32_t* __restrict__ pos_cols,
    float* __restrict__ top_scores, int32_t* __restrict__ top_ids,
    uint8_t* __restrict__ pos_flags) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nq) return;
  float ts[KC];
  int ti[KC];
#pragma unroll
  for (int t = 0; t < KC; ++t) { ts[t] = -INFINITY; ti[t] = -1; }
  for (int s = 0; s < S; ++s)
    for (int t = 0; t < K; ++t) {
      const int64_t o = ((int64_t)s * nq + q) * K + t;
      topk_merge_insert<KC>(ts, ti, ps[o], pi[o]);
    }
  const int64_t p0 = pos_ptr ? pos_ptr[q] : 0;
  const int64_t p1 = pos_ptr ? pos_ptr[q + 1] : 0;
#pragma unroll
  for (int t = 0; t < KC; ++t) {
    if (t < K) {
      const int64_t o = q * K + t;
      if (top_scores) top_scores[o] = ts[t];
      if (top_ids) top_ids[o] = ti[t];
      if (pos_flags) pos_flags[o] = (ti[t] >= 0 && sorted_contains(pos_cols, p0, p1, ti[t])) ? 1 : 0;
    }
  }
}

// Plain score matrix S[q, i] (compat path for full_sort_predict): A = users in
// registers, B = item tile from LDS, so the accumulator has the ITEM on the lane
// and each store instruction writes 128 contiguous bytes of a score row.
template <int D>
__global__ __launch_bounds__(kFsThreads) void score_matrix_kernel(const float* __restrict__ Uq,
                                                                  int64_t nq,
                                                                  const float* __restrict__ EI,
                                                                  int64_t I, float* __restrict__ S) {
  constexpr int LDR = D + 2;
  __shared__ __attribute__((aligned(16))) float tile[32 * LDR];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int j = lane & 31;
  const int h = lane >> 5;
  const int64_t qb = ((int64_t)blockIdx.x * 4 + w) * 32;
  const int64_t q = qb + j;
  float ub[D / 2];
  load_user_operand<D>(Uq, q, q < nq, h, ub);
  const int64_t ntile = (I + 31) / 32;
  for (int64_t t = 0; t < ntile; ++t) {
    const int64_t base = t * 32;
    __syncthreads();
    stage_tile<D>(EI, I, base, tile);
    __syncthreads();
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const float* brow = tile + j * LDR + 2 * h;
#pragma unroll
    for (int s2 = 0; s2 < D / 4; ++s2) {
      const float2 b = *reinterpret_cast<const float2*>(brow + 4 * s2);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ub[2 * s2], b.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ub[2 * s2 + 1], b.y, acc, 0, 0, 0);
    }
    const int64_t item = base + j;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t uq = qb + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (uq < nq && item < I) S[uq * I + item] = acc[r];
    }
  }
}

}  // namespace mirec

using namespace mirec;

extern "C" int mirec_fullsort_topk_f32(const float* Uq, int64_t nq, const float* EI, int64_t I,
                                       int32_t d, const int64_t* hist_ptr,
                                       const int32_t* hist_cols, const int64_t* pos_ptr,
                                       const int32_t* pos_cols, int32_t K, float* top_scores,
                                       int32_t* top_ids, uint8_t* pos_flags, void* stream) {
  if (nq == 0) return 0;
  if (!Uq || !EI || nq < 0 || I <= 0 || K < 1 || (hist_ptr && !hist_cols) ||
      (pos_ptr && !pos_cols) || (pos_flags && !pos_ptr)) {
    set_error("mirec_fullsort_topk_f32: bad arguments");
    return -1;
  }
  if (I > INT32_MAX) {
    set_error("mirec_fullsort_topk_f32: item count exceeds int32");
    return -1;
  }
  const dim3 grd((unsigned)((nq + 127) / 128));
  hipStream_t st = (hipStream_t)stream;
#define MIREC_FS(DD, KK)                                                                      \
  hipLaunchKernelGGL((fullsort_topk_kernel<DD, KK>), grd, dim3(kFsThreads), 0, st, Uq, nq, EI, \
                     I, hist_ptr, hist_cols, pos_ptr, pos_cols, K, top_scores, top_ids,        \
                     pos_flags, (int64_t)((I + 63) / 64 * 64))
#define MIREC_FS_D(DD)                                 \
  case DD:                                             \
    if (K <= 10) MIREC_FS(DD, 10);                     \
    else if (K <= 20) MIREC_FS(DD, 20);                \
    else if (K <= 50) MIREC_FS(DD, 50);                \
    else { set_error("mirec_fullsort_topk_f32: K=%d > 50", K); return -1; } \
    break;
  switch (d) {
    MIREC_FS_D(32)
    MIREC_FS_D(64)
    MIREC_FS_D(128)
    MIREC_FS_D(256)
    default:
      set_error("mirec_fullsort_topk_f32: embedding_size %d not in {32,64,128,256}", d);
      return -1;
  }
#undef MIREC_FS_D
#undef MIREC_FS
  return launch_status("mirec_fullsort_topk_f32");
}

extern "C" size_t mirec_fullsort_topk_split_workspace_size(int64_t nq, int32_t K,
                                                          int32_t n_split) {
  if (nq <= 0 || K <= 0 || n_split <= 0) return 256;
  return (size_t)n_split * (size_t)nq * (size_t)K * (sizeof(float) + sizeof(int32_t)) + 256;
}

extern "C" int mirec_fullsort_topk_split_f32(const float* Uq, int64_t nq, const float* EI,
                                             int64_t I, int32_t d, const int64_t* hist_ptr,
                                             const int32_t* hist_cols, const int64_t* pos_ptr,
                                             const int32_t* pos_cols, int32_t K, int32_t n_split,
                                             void* ws, size_t ws_bytes, float* top_scores,
                                             int32_t* top_ids, uint8_t* pos_flags, void* stream) {
  if (nq == 0) return 0;
  if (!Uq || !EI || nq < 0 || I <= 0 || K < 1 || K > 50 || n_split < 1 || n_split > 64 ||
      (hist_ptr && !hist_cols) || (pos_ptr && !pos_cols) || (pos_flags && !pos_ptr)) {
    set_error("mirec_fullsort_topk_split_f32: bad arguments");
    return -1;
  }
  if (I > INT32_MAX) {
    set_error("mirec_fullsort_topk_split_f32: item count exceeds int32");
    return -1;
  }
  const size_t need = mirec_fullsort_topk_split_workspace_size(nq, K, n_split);
  if (!ws || ws_bytes < need) {
    set_error("mirec_fullsort_topk_split_f32: workspace %zu < %zu", ws_bytes, need);
    return -1;
  }
  float* ps = (float*)ws;
  int32_t* pi = (int32_t*)(ps + (size_t)n_split * nq * K);
  const int64_t tiles = (I + 63) / 64;               // 64: a multiple of every kernel's tile
  const int64_t span = (tiles + n_split - 1) / n_split * 64;
  const int S = (int)((I + span - 1) / span);
  const dim3 grd((unsigned)((nq + 127) / 128), (unsigned)S);
  hipStream_t st = (hipStream_t)stream;
#define MIREC_FSS(DD, KK)                                                                     \
  hipLaunchKernelGGL((fullsort_topk_kernel<DD, KK>), grd, dim3(kFsThreads), 0, st, Uq, nq, EI, \
                     I, hist_ptr, hist_cols, nullptr, nullptr, K, ps, pi, nullptr, span);      \
  hipLaunchKernelGGL((fullsort_merge_kernel<KK>), dim3((unsigned)((nq + 255) / 256)), dim3(256), \
                     0, st, nq, S, K, ps, pi, pos_ptr, pos_cols, top_scores, top_ids, pos_flags)
#define MIREC_FSS_D(DD)                                \
  case DD:                                             \
    if (K <= 10) { MIREC_FSS(DD, 10); }                \
    else if (K <= 20) { MIREC_FSS(DD, 20); }           \
    else { MIREC_FSS(DD, 50); }                        \
    break;
  switch (d) {
    MIREC_FSS_D(32)
    MIREC_FSS_D(64)
    MIREC_FSS_D(128)
    MIREC_FSS_D(256)
    default:
      set_error("mirec_fullsort_topk_split_f32: embedding_size %d not in {32,64,128,256}", d);
      return -1;
  }
#undef MIREC_FSS_D
#undef MIREC_FSS
  return launch_status("mirec_fullsort_topk_split_f32");
}

extern "C" int mirec_score_matrix_f32(const float* Uq, int64_t nq, const float* EI, int64_t I,
                                      int32_t d, float* S, void* stream) {
  if (nq == 0) return 0;
  if (!Uq || !EI || !S || nq < 0 || I <= 0) {
    set_error("mirec_score_matrix_f32: bad arguments");
    return -1;
  }
  const dim3 grd((unsigned)((nq + 127) / 128));
  hipStream_t st = (hipStream_t)stream;
  switch (d) {
    case 32: hipLaunchKernelGGL(score_matrix_kernel<32>, grd, dim3(kFsThreads), 0, st, Uq, nq, EI, I, S); break;
    case 64: hipLaunchKernelGGL(score_matrix_kernel<64>, grd, dim3(kFsThreads), 0, st, Uq, nq, EI, I, S); break;
    case 128: hipLaunchKernelGGL(score_matrix_kernel<128>, grd, dim3(kFsThreads), 0, st, Uq, nq, EI, I, S); break;
    case 256: hipLaunchKernelGGL(score_matrix_kernel<256>, grd, dim3(kFsThreads), 0, st, Uq, nq, EI, I, S); break;
    default:
      set_error("mirec_score_matrix_f32: embedding_size %d not in {32,64,128,256}", d);
      return -1;
  }
  return launch_status("mirec_score_matrix_f32");
}
