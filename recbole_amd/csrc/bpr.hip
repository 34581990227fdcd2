// K3 — fused BPR forward + backward, D/4 lanes per positive.
//
// Restates BPR.calculate_loss (recbole/model/general_recommender/bpr.py:74-83)
// and BPRLoss (recbole/model/loss.py:43-49) plus the autograd backward torch
// runs for them, on the pairwise layout of GeneralNegSampleDataLoader
// (general_dataloader.py:235-241, Interaction.repeat interaction.py:189-217):
// row r = j*B + k carries (user[k], pos[k], neg[r]).  All `times` rows of one
// positive share u_k and p_k, so a wave loads them ONCE and streams only the
// negatives: (2 + times) rows per positive instead of 3*times.
//
// Backward follows torch's op order: mean -> neg -> log -> add -> sigmoid:
//   g = -(1/R) / (gamma + s);  dx = g * (1 - s) * s;  d pos = dx, d neg = -dx
//   du = dx*p - dx*n, dp = dx*u, dn = -dx*u   (summed over the rows of a key
//   by the segment reduction, K2/K5).
#include "bpr_math.h"

namespace mirec {

template <int D>
struct RowVec {
  static constexpr int E = D >= 64 ? D / 64 : 1;   // floats per lane
  static constexpr int ACT = D >= 64 ? 64 : D;     // active lanes
  float x[E];
};

template <int D>
__device__ __forceinline__ void load_row(const float* __restrict__ base, int lane, RowVec<D>& r) {
  constexpr int E = RowVec<D>::E;
  const float* p = base + lane * E;
  if constexpr (E == 4) {
    float4 v = *reinterpret_cast<const float4*>(p);
    r.x[0] = v.x; r.x[1] = v.y; r.x[2] = v.z; r.x[3] = v.w;
  } else if constexpr (E == 2) {
    float2 v = *reinterpret_cast<const float2*>(p);
    r.x[0] = v.x; r.x[1] = v.y;
  } else {
    r.x[0] = p[0];
  }
}

template <int D>
__device__ __forceinline__ void store_row(float* __restrict__ base, int lane, const float* x) {
  constexpr int E = RowVec<D>::E;
  float* p = base + lane * E;
  if constexpr (E == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(x[0], x[1], x[2], x[3]);
  } else if constexpr (E == 2) {
    *reinterpret_cast<float2*>(p) = make_float2(x[0], x[1]);
  } else {
    p[0] = x[0];
  }
}

// D/4 lanes per positive (one float4 of every row per lane: 16-B loads, a 512-B
// row of D = 128 is one half-wave access), 64/(D/4) positives per wave. The
// negatives are gathered NB at a time with all their loads issued before the
// first reduction, so a positive costs ~2 dependent memory round trips instead
// of one per negative.
// AT_IDS: the gradient row of every slot is written at its row id (gU + id*D for the
// user, gI + id*D for the items) instead of at its slot — the row-sharded step, whose
// ids are positions in the received message buffer and whose gradient rows go back in
// the same positions (csrc/shard.hip): K3 and the backward gather in one launch.
// Register budget: 6 waves per SIMD for rows of d <= 128 (80 VGPRs; the compiler keeps
// 88 B per lane in scratch, which costs less than the waves it buys: the past-LLC gather
// at B = 65,536 reads + writes 4.94 TB/s against 4.57 at 4 waves, tools/gather_probe.py).
#ifndef MIREC_K3_WAVES
#define MIREC_K3_WAVES 6
#endif
template <int D> struct K3Waves { static constexpr int n = D <= 128 ? MIREC_K3_WAVES : 1; };
// Gradient-row stores are non-temporal: each row is written once and read by a later
// launch, so it should not displace the gathered rows in the caches (4.35 -> 4.57 TB/s).
#ifndef MIREC_K3_TEMPORAL
#define MIREC_K3_NT 1
#endif
__device__ __forceinline__ void grad_store(float* p, const float4& x) {
#if defined(MIREC_K3_NT)
  typedef float f4v __attribute__((ext_vector_type(4)));
  f4v v = {x.x, x.y, x.z, x.w};
  __builtin_nontemporal_store(v, reinterpret_cast<f4v*>(p));
#else
  *reinterpret_cast<float4*>(p) = x;
#endif
}

template <int D, bool AT_IDS = false>
__global__ __launch_bounds__(256, K3Waves<D>::n) void bpr_fwd_bwd_kernel(
    const float* __restrict__ EU, int64_t nU, const float* __restrict__ EI, int64_t nI,
    const int64_t* __restrict__ user, const int64_t* __restrict__ pos,
    const int64_t* __restrict__ neg, int64_t B, int times, float gamma, float grad_scale,
    float* __restrict__ loss_k, float* __restrict__ pos_score, float* __restrict__ neg_score,
    float* __restrict__ gU, float* __restrict__ gI, float* __restrict__ coef) {
  constexpr int LPR = D / 4;
  constexpr int GPW = 64 / LPR;
  constexpr int NB = 4;
  const int lane = threadIdx.x & 63;
  const int g = lane / LPR;
  const int l = lane - g * LPR;
  const int64_t k = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * GPW + g;
  if (k >= B) return;  // whole lane group exits together (shuffles stay in the group)

  // row ids clamped as int32 (tables hold < 2^31 rows; the host checks): half the
  // registers of int64 ids, which buys the occupancy the gather needs
  const int64_t u64 = user[k], p64 = pos[k];
  const int uid = (int)(u64 < 0 ? 0 : (u64 >= nU ? nU - 1 : u64));
  const int pid = (int)(p64 < 0 ? 0 : (p64 >= nI ? nI - 1 : p64));
  const float4 u = reinterpret_cast<const float4*>(EU + (int64_t)uid * D)[l];
  const float4 p = reinterpret_cast<const float4*>(EI + (int64_t)pid * D)[l];
  int nid[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    const int64_t id = q < times ? neg[(int64_t)q * B + k] : 0;
    nid[q] = (int)(id < 0 ? 0 : (id >= nI ? nI - 1 : id));
  }
  int wid[NB];                        // AT_IDS: this group's negative ids (the next load early)
#pragma unroll
  for (int q = 0; q < NB; ++q) wid[q] = nid[q];
  // the first group's negative rows in flight with u and p: all the rows of a positive
  // with T <= NB in one dependent level after the ids
  float4 nf[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q)
    nf[q] = q < times ? reinterpret_cast<const float4*>(EI + (int64_t)nid[q] * D)[l]
                      : make_float4(0.f, 0.f, 0.f, 0.f);
  const float sp = group_sum<LPR>(dot4(u, p));
  float4 gu = make_float4(0.f, 0.f, 0.f, 0.f), gp = gu;
  float lsum = 0.f;
  const float ng = -grad_scale;
  for (int j0 = 0; j0 < times; j0 += NB) {
    float4 n[NB];
#pragma unroll
    for (int q = 0; q < NB; ++q)
      n[q] = j0 == 0 ? nf[q]
                     : (j0 + q < times ? reinterpret_cast<const float4*>(EI + (int64_t)nid[q] * D)[l]
                                       : make_float4(0.f, 0.f, 0.f, 0.f));
    // ids of the next group in flight under this group's arithmetic
#pragma unroll
    for (int q = 0; q < NB; ++q) wid[q] = nid[q];
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const int j = j0 + NB + q;
      const int64_t id = j < times ? neg[(int64_t)j * B + k] : 0;
      nid[q] = (int)(id < 0 ? 0 : (id >= nI ? nI - 1 : id));
    }
    float sn[NB];
#pragma unroll
    for (int q = 0; q < NB; ++q) sn[q] = group_sum<LPR>(dot4(u, n[q]));
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const int j = j0 + q;
      if (j < times) {
        const BprCoef cf = bpr_coef(sp, sn[q], gamma, ng);
        lsum += cf.nll;
        const float dx = cf.dx;
        float4 gn;
        pair_contrib(gu, gp, gn, dx, u, p, n[q]);
        const int64_t r = (int64_t)j * B + k;
        if (gI) grad_store(gI + (AT_IDS ? (int64_t)wid[q] : B + r) * D + 4 * l, gn);
        if (l == 0) {
          if (neg_score) neg_score[r] = sn[q];
          if (coef) coef[r] = dx;
        }
      }
    }
  }
  if (gU) grad_store(gU + (AT_IDS ? (int64_t)uid : k) * D + 4 * l, gu);
  if (gI) grad_store(gI + (AT_IDS ? (int64_t)pid : k) * D + 4 * l, gp);
  if (l == 0) {
    if (loss_k) loss_k[k] = lsum;
    if (pos_score) pos_score[k] = sp;
  }
}

// Data-parallel rebuild of K3's gradient rows for a GLOBAL batch from the
// exchanged coefficients: same lane layout, same row loads, same pair_contrib
// sequence (negatives in order), so the rows are bit-identical to K3's on one
// GPU. Coefficient of row (j, k): coef[(k / Bl) * stride + j * Bl + k % Bl] (the
// per-rank blocks of the exchange buffer; Bl = positives per rank).
template <int D>
__global__ __launch_bounds__(256) void bpr_contrib_kernel(
    const float* __restrict__ EU, int64_t nU, const float* __restrict__ EI, int64_t nI,
    const int64_t* __restrict__ user, const int64_t* __restrict__ pos,
    const int64_t* __restrict__ neg, int64_t B, int times, const float* __restrict__ coef,
    int64_t Bl, int64_t stride, float* __restrict__ gU, float* __restrict__ gI) {
  constexpr int LPR = D / 4;
  constexpr int GPW = 64 / LPR;
  constexpr int NB = 4;
  const int lane = threadIdx.x & 63;
  const int g = lane / LPR;
  const int l = lane - g * LPR;
  const int64_t k = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * GPW + g;
  if (k >= B) return;
  int64_t uid = user[k], pid = pos[k];
  uid = uid < 0 ? 0 : (uid >= nU ? nU - 1 : uid);
  pid = pid < 0 ? 0 : (pid >= nI ? nI - 1 : pid);
  const float4 u = reinterpret_cast<const float4*>(EU + uid * D)[l];
  const float4 p = reinterpret_cast<const float4*>(EI + pid * D)[l];
  const float* __restrict__ ck = coef + (k / Bl) * stride + (k % Bl);
  float4 gu = make_float4(0.f, 0.f, 0.f, 0.f), gp = gu;
  for (int j0 = 0; j0 < times; j0 += NB) {
    float4 n[NB];
    float dx[NB];
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const int j = j0 + q;
      int64_t id = j < times ? neg[(int64_t)j * B + k] : 0;
      id = id < 0 ? 0 : (id >= nI ? nI - 1 : id);
      n[q] = j < times ? reinterpret_cast<const float4*>(EI + id * D)[l]
                       : make_float4(0.f, 0.f, 0.f, 0.f);
      dx[q] = j < times ? ck[(int64_t)j * Bl] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const int j = j0 + q;
      if (j < times) {
        float4 gn;
        pair_contrib(gu, gp, gn, dx[q], u, p, n[q]);
        reinterpret_cast<float4*>(gI + (B + (int64_t)j * B + k) * D)[l] = gn;
      }
    }
  }
  reinterpret_cast<float4*>(gU + k * D)[l] = gu;
  reinterpret_cast<float4*>(gI + k * D)[l] = gp;
}

// score[r] = <EU[u[r]], EI[i[r]]> — BPR.predict (bpr.py:85-89) and the
// sampled-evaluation scorer; one wave per row.
template <int D>
__global__ __launch_bounds__(256) void dot_rows_kernel(const float* __restrict__ EU, int64_t nU,
                                                       const float* __restrict__ EI, int64_t nI,
                                                       const int64_t* __restrict__ u,
                                                       const int64_t* __restrict__ it, int64_t n,
                                                       float* __restrict__ out) {
  constexpr int E = RowVec<D>::E;
  constexpr int ACT = RowVec<D>::ACT;
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= n) return;
  int64_t a = u[r], b = it[r];
  a = a < 0 ? 0 : (a >= nU ? nU - 1 : a);
  b = b < 0 ? 0 : (b >= nI ? nI - 1 : b);
  float part = 0.f;
  if (lane < ACT) {
    RowVec<D> x, y;
    load_row<D>(EU + a * D, lane, x);
    load_row<D>(EI + b * D, lane, y);
#pragma unroll
    for (int e = 0; e < E; ++e) part += x.x[e] * y.x[e];
  }
  const float s = wave_sum(part);
  if (lane == 0) out[r] = s;
}

}  // namespace mirec

using namespace mirec;

extern "C" int mirec_dot_rows_f32(const float* EU, int64_t nU, const float* EI, int64_t nI,
                                  int32_t d, const int64_t* u, const int64_t* i, int64_t n,
                                  float* out, void* stream) {
  if (n == 0) return 0;
  if (!EU || !EI || !u || !i || !out || n < 0) {
    set_error("mirec_dot_rows_f32: bad arguments");
    return -1;
  }
  const dim3 grd((unsigned)((n + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
  switch (d) {
    case 32: hipLaunchKernelGGL(dot_rows_kernel<32>, grd, dim3(256), 0, st, EU, nU, EI, nI, u, i, n, out); break;
    case 64: hipLaunchKernelGGL(dot_rows_kernel<64>, grd, dim3(256), 0, st, EU, nU, EI, nI, u, i, n, out); break;
    case 128: hipLaunchKernelGGL(dot_rows_kernel<128>, grd, dim3(256), 0, st, EU, nU, EI, nI, u, i, n, out); break;
    case 256: hipLaunchKernelGGL(dot_rows_kernel<256>, grd, dim3(256), 0, st, EU, nU, EI, nI, u, i, n, out); break;
    default:
      set_error("mirec_dot_rows_f32: embedding_size %d not in {32,64,128,256}", d);
      return -1;
  }
  return launch_status("mirec_dot_rows_f32");
}

namespace {

int launch_bpr(const float* EU, int64_t nU, const float* EI, int64_t nI, int32_t d,
               const int64_t* user, const int64_t* pos, const int64_t* neg, int64_t B,
               int32_t times, float gamma, float grad_scale, float* loss_k, float* pos_score,
               float* neg_score, float* gU, float* gI, float* coef, void* stream,
               const char* what, bool at_ids = false) {
  if (B == 0) return 0;
  if (!EU || !EI || !user || !pos || (times > 0 && !neg) || B < 0 || times < 0 || nU <= 0 ||
      nI <= 0 || nU > INT32_MAX || nI > INT32_MAX) {
    set_error("%s: bad arguments", what);
    return -1;
  }
  const dim3 blk(256);
  hipStream_t st = (hipStream_t)stream;
#define MIREC_BPR_CASE(DD)                                                                    \
  case DD:                                                                                    \
    hipLaunchKernelGGL((at_ids ? bpr_fwd_bwd_kernel<DD, true>                         \
                                 : bpr_fwd_bwd_kernel<DD, false>),                        \
                       dim3((unsigned)((B + 4 * (256 / DD) - 1) / (4 * (256 / DD)))), blk, 0, \
                       st, EU, nU, EI, nI, user, pos,                                         \
                       neg, B, times, gamma, grad_scale, loss_k, pos_score, neg_score, gU, gI, \
                       coef);                                                                 \
    break;
  switch (d) {
    MIREC_BPR_CASE(32)
    MIREC_BPR_CASE(64)
    MIREC_BPR_CASE(128)
    MIREC_BPR_CASE(256)
    default:
      set_error("%s: embedding_size %d not in {32,64,128,256}", what, d);
      return -1;
  }
#undef MIREC_BPR_CASE
  return launch_status(what);
}

}  // namespace

extern "C" int mirec_bpr_fwd_bwd_f32(const float* EU, int64_t nU, const float* EI, int64_t nI,
                                     int32_t d, const int64_t* user, const int64_t* pos,
                                     const int64_t* neg, int64_t B, int32_t times, float gamma,
                                     float grad_scale, float* loss_k, float* pos_score,
                                     float* neg_score, float* gU, float* gI, void* stream) {
  return launch_bpr(EU, nU, EI, nI, d, user, pos, neg, B, times, gamma, grad_scale, loss_k,
                    pos_score, neg_score, gU, gI, nullptr, stream, "mirec_bpr_fwd_bwd_f32");
}

// K3 with every gradient row written at its row id (the row-sharded step: ids are message
// positions, gradient rows return in the same positions) — grad may be the same buffer
// for both tables; the ids of one batch must be distinct slots (they are: one message
// position per slot).
extern "C" int mirec_bpr_fwd_bwd_at_ids_f32(const float* E, int64_t nE, int32_t d,
                                           const int64_t* user, const int64_t* pos,
                                           const int64_t* neg, int64_t B, int32_t times,
                                           float gamma, float grad_scale, float* loss_k,
                                           float* grad, void* stream) {
  if (B > 0 && !grad) {
    set_error("mirec_bpr_fwd_bwd_at_ids_f32: grad is required");
    return -1;
  }
  return launch_bpr(E, nE, E, nE, d, user, pos, neg, B, times, gamma, grad_scale, loss_k,
                    nullptr, nullptr, grad, grad, nullptr, stream,
                    "mirec_bpr_fwd_bwd_at_ids_f32", true);
}

extern "C" int mirec_bpr_fwd_coef_f32(const float* EU, int64_t nU, const float* EI, int64_t nI,
                                      int32_t d, const int64_t* user, const int64_t* pos,
                                      const int64_t* neg, int64_t B, int32_t times, float gamma,
                                      float grad_scale, float* loss_k, float* coef,
                                      void* stream) {
  if (B > 0 && times > 0 && !coef) {
    set_error("mirec_bpr_fwd_coef_f32: coef is required");
    return -1;
  }
  return launch_bpr(EU, nU, EI, nI, d, user, pos, neg, B, times, gamma, grad_scale, loss_k,
                    nullptr, nullptr, nullptr, nullptr, coef, stream, "mirec_bpr_fwd_coef_f32");
}

extern "C" int mirec_bpr_contrib_f32(const float* EU, int64_t nU, const float* EI, int64_t nI,
                                     int32_t d, const int64_t* user, const int64_t* pos,
                                     const int64_t* neg, int64_t B, int32_t times,
                                     const float* coef, int64_t coef_block,
                                     int64_t coef_stride, float* gU, float* gI, void* stream) {
  if (B == 0) return 0;
  if (!EU || !EI || !user || !pos || (times > 0 && (!neg || !coef)) || !gU || !gI || B < 0 ||
      times < 0 || nU <= 0 || nI <= 0 || coef_block <= 0 || coef_stride < times * coef_block) {
    set_error("mirec_bpr_contrib_f32: bad arguments");
    return -1;
  }
  hipStream_t st = (hipStream_t)stream;
  const dim3 blk(256);
#define MIREC_CONTRIB_CASE(DD)                                                                \
  case DD:                                                                                    \
    hipLaunchKernelGGL(bpr_contrib_kernel<DD>,                                                \
                       dim3((unsigned)((B + 4 * (256 / DD) - 1) / (4 * (256 / DD)))), blk, 0, \
                       st, EU, nU, EI, nI, user, pos, neg, B, times, coef, coef_block,        \
                       coef_stride, gU, gI);                                                  \
    break;
  switch (d) {
    MIREC_CONTRIB_CASE(32)
    MIREC_CONTRIB_CASE(64)
    MIREC_CONTRIB_CASE(128)
    MIREC_CONTRIB_CASE(256)
    default:
      set_error("mirec_bpr_contrib_f32: embedding_size %d not in {32,64,128,256}", d);
      return -1;
  }
#undef MIREC_CONTRIB_CASE
  return launch_status("mirec_bpr_contrib_f32");
}
