// K7 — graph propagation for LightGCN: CSR SpMM over the normalised
// user-item adjacency with a fused epilogue, plus the small EmbLoss helpers.
//
// Restates (recbole/model/general_recommender/lightgcn.py):
//   forward()               E_{l+1} = A_hat @ E_l  (torch.sparse.mm, :118-124),
//                           mean over the stacked layers (:125-126)
//   its autograd backward   dE_l = A_hat^T dE_{l+1} + dMean/(L+1);  A_hat is
//                           symmetric (same pattern both ways, value
//                           d_i^-1/2 d_j^-1/2), so the forward CSR serves both
//   EmbLoss                 ||X||_F / B of the gathered ego rows (loss.py:79-84)
//
// One launch computes, for every row r of the CSR,
//   y   = sum_{j in row r} val[j] * X[col[j]]          (j ascending)
//   y  += add_scale * ADD[r]                          (optional; backward Horner step)
//   Y[r] = y                                          (optional)
//   ACC_OUT[r] = (ACC_IN[r] + y) * acc_scale           (optional; running layer sum / mean)
// Every operand is a "split rows" reference (lo, hi, split): row r lives at
// lo + r*d for r < split, else hi + (r-split)*d. That lets the user and item
// tables (two nn.Parameters) act as the one [U+I, d] ego matrix without the
// torch.cat copy the reference makes (:107-113), and lets the backward write the
// two weight gradients directly.
//
// Work decomposition (load balance under Zipf degrees): the host plan cuts every
// row into near-equal units of about `piece` nonzeros, at most 1024 per row (a
// hub item of a Zipf graph has millions of edges). A unit is handled by a group of
// D/4 lanes (one float4 of the row per lane; 64/(D/4) rows per wave). Rows of
// one unit apply the epilogue directly; the units of a longer row write their
// partial sums to `partial` and a second kernel adds them in unit order and
// applies the epilogue — deterministic, no float atomics. The inner loop loads
// (col, val) pairs cooperatively, one per lane of the group, broadcasts them
// with ds_bpermute, and keeps 4 row loads in flight per lane.
#include "common.h"

namespace mirec {

struct RowsRef {
  float* lo;
  float* hi;
  int64_t split;
  __device__ __forceinline__ float* row(int64_t r, int d) const {
    return r < split ? lo + r * d : hi + (r - split) * d;
  }
};

struct Epilogue {
  RowsRef add;
  float add_scale;
  RowsRef y;
  RowsRef acc_in;
  RowsRef acc_out;
  float acc_scale;
};

__device__ __forceinline__ float4 f4_fma(float s, float4 x, float4 a) {
  a.x = fmaf(s, x.x, a.x);
  a.y = fmaf(s, x.y, a.y);
  a.z = fmaf(s, x.z, a.z);
  a.w = fmaf(s, x.w, a.w);
  return a;
}

template <int D>
__device__ __forceinline__ void apply_epilogue(const Epilogue& ep, int64_t r, int l, float4 y) {
  if (ep.add.lo) {
    const float4 a = reinterpret_cast<const float4*>(ep.add.row(r, D))[l];
    y.x += ep.add_scale * a.x;
    y.y += ep.add_scale * a.y;
    y.z += ep.add_scale * a.z;
    y.w += ep.add_scale * a.w;
  }
  if (ep.y.lo) reinterpret_cast<float4*>(ep.y.row(r, D))[l] = y;
  if (ep.acc_out.lo) {
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ep.acc_in.lo) a = reinterpret_cast<const float4*>(ep.acc_in.row(r, D))[l];
    a.x = (a.x + y.x) * ep.acc_scale;
    a.y = (a.y + y.y) * ep.acc_scale;
    a.z = (a.z + y.z) * ep.acc_scale;
    a.w = (a.w + y.w) * ep.acc_scale;
    reinterpret_cast<float4*>(ep.acc_out.row(r, D))[l] = a;
  }
}

template <int D>
__global__ __launch_bounds__(256) void spmm_units_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ cols,
    const float* __restrict__ vals, const int32_t* __restrict__ unit_row,
    const int64_t* __restrict__ unit_beg, const int32_t* __restrict__ unit_slot,
    int64_t n_units, int32_t piece, RowsRef x, Epilogue ep, float* __restrict__ partial) {
  constexpr int LPR = D / 4;          // lanes per row
  constexpr int GPW = 64 / LPR;       // rows (units) per wave
  const int lane = threadIdx.x & 63;
  const int g = lane / LPR;
  const int l = lane - g * LPR;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t n_waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t ub = wave * GPW; ub < n_units; ub += n_waves * GPW) {
    const int64_t u = ub + g;
    int64_t b = 0, e = 0, r = 0;
    int32_t slot = -1;
    if (u < n_units) {
      r = unit_row[u];
      b = unit_beg[u];
      e = unit_beg[u + 1];   // units tile each row in order: the next one starts here
      slot = unit_slot[u];
    }
    const int len = (int)(e - b);
    (void)piece;
    int maxlen = len;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) maxlen = max(maxlen, __shfl_xor(maxlen, off, 64));
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int o = 0; o < maxlen; o += LPR) {
      int c = 0;
      float v = 0.f;
      if (o + l < len) {
        c = cols[b + o + l];
        v = vals[b + o + l];
      }
      const int cnt = min(LPR, maxlen - o);   // wave-uniform
      int t = 0;
      for (; t + 4 <= cnt; t += 4) {
        int ct[4];
        float vt[4];
        float4 xv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          ct[q] = __shfl(c, g * LPR + t + q, 64);
          vt[q] = __shfl(v, g * LPR + t + q, 64);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
          xv[q] = (o + t + q < len)
                      ? reinterpret_cast<const float4*>(x.row(ct[q], D))[l]
                      : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (o + t + q < len) acc = f4_fma(vt[q], xv[q], acc);
      }
      for (; t < cnt; ++t) {
        const int ct = __shfl(c, g * LPR + t, 64);
        const float vt = __shfl(v, g * LPR + t, 64);
        if (o + t < len) acc = f4_fma(vt, reinterpret_cast<const float4*>(x.row(ct, D))[l], acc);
      }
    }
    if (u < n_units) {
      if (slot >= 0)
        reinterpret_cast<float4*>(partial + (int64_t)slot * D)[l] = acc;
      else
        apply_epilogue<D>(ep, r, l, acc);
    }
  }
}

template <int D>
__global__ __launch_bounds__(256) void spmm_fixup_kernel(const int32_t* __restrict__ fix_row,
                                                         const int32_t* __restrict__ fix_ptr,
                                                         int64_t n_fix,
                                                         const float* __restrict__ partial,
                                                         Epilogue ep) {
  constexpr int LPR = D / 4;
  constexpr int GPW = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const int g = lane / LPR;
  const int l = lane - g * LPR;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t n_waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t f = wave * GPW + g; f < n_fix; f += n_waves * GPW) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int32_t s = fix_ptr[f]; s < fix_ptr[f + 1]; ++s) {
      const float4 p = reinterpret_cast<const float4*>(partial + (int64_t)s * D)[l];
      acc.x += p.x;
      acc.y += p.y;
      acc.z += p.z;
      acc.w += p.w;
    }
    apply_epilogue<D>(ep, fix_row[f], l, acc);
  }
}

// sq[i] = sum_k table[idx[i], k]^2 (one wave per row, fixed lane order).
__global__ __launch_bounds__(256) void gather_sqnorm_kernel(const float* __restrict__ table,
                                                            int64_t n_rows, int d,
                                                            const int64_t* __restrict__ idx,
                                                            int64_t n, float* __restrict__ sq) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t n_waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = wave; i < n; i += n_waves) {
    int64_t r = idx[i];
    r = r < 0 ? 0 : (r >= n_rows ? n_rows - 1 : r);
    const float* row = table + r * d;
    float s = 0.f;
    for (int k = lane; k < d; k += 64) s = fmaf(row[k], row[k], s);
    s = wave_sum(s);
    if (lane == 0) sq[i] = s;
  }
}

// out[i, :] = scale[0] * table[idx[i], :]
__global__ __launch_bounds__(256) void gather_scale_kernel(const float* __restrict__ table,
                                                           int64_t n_rows, int d,
                                                           const int64_t* __restrict__ idx,
                                                           int64_t n,
                                                           const float* __restrict__ scale,
                                                           float* __restrict__ out) {
  const float s = scale[0];
  const int64_t total = n * d;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / d;
    const int64_t k = e - i * d;
    int64_t r = idx[i];
    r = r < 0 ? 0 : (r >= n_rows ? n_rows - 1 : r);
    out[e] = s * table[r * d + k];
  }
}

static RowsRef to_ref(const mirec_rows_ref& a) { return RowsRef{a.lo, a.hi ? a.hi : a.lo, a.split}; }

static unsigned grid_for(int64_t waves_needed) {
  int64_t blocks = (waves_needed + 3) / 4;   // 4 waves per 256-thread block
  if (blocks > 256 * 32) blocks = 256 * 32;
  if (blocks < 1) blocks = 1;
  return (unsigned)blocks;
}

}  // namespace mirec

using namespace mirec;

extern "C" int mirec_spmm_csr_f32(const int64_t* row_ptr, const int32_t* cols, const float* vals,
                                  int64_t n_rows, int32_t d, const int32_t* unit_row,
                                  const int64_t* unit_beg, const int32_t* unit_slot,
                                  int64_t n_units, int32_t piece, const int32_t* fix_row,
                                  const int32_t* fix_ptr, int64_t n_fix, float* partial,
                                  const mirec_rows_ref* x, const mirec_spmm_epilogue* ep,
                                  void* stream) {
  if (!row_ptr || !x || !ep || !x->lo || n_rows < 0 || n_units < n_rows || piece < 1 ||
      (n_fix > 0 && (!fix_row || !fix_ptr || !partial)) || (n_units > 0 && (!unit_row || !unit_beg || !unit_slot))) {
    set_error("mirec_spmm_csr_f32: bad arguments");
    return -1;
  }
  if (!ep->y.lo && !ep->acc_out.lo) {
    set_error("mirec_spmm_csr_f32: epilogue writes nothing (y and acc_out both NULL)");
    return -1;
  }
  if (n_units == 0) return 0;
  Epilogue e{to_ref(ep->add), ep->add_scale, to_ref(ep->y), to_ref(ep->acc_in),
             to_ref(ep->acc_out), ep->acc_scale};
  const RowsRef xr = to_ref(*x);
  hipStream_t st = (hipStream_t)stream;
#define MIREC_SPMM(DD)                                                                        \
  case DD: {                                                                                  \
    constexpr int GPW = 64 / (DD / 4);                                                        \
    hipLaunchKernelGGL(spmm_units_kernel<DD>, dim3(grid_for((n_units + GPW - 1) / GPW)),      \
                       dim3(256), 0, st, row_ptr, cols, vals, unit_row, unit_beg, unit_slot,  \
                       n_units, piece, xr, e, partial);                                        \
    if (n_fix > 0)                                                                             \
      hipLaunchKernelGGL(spmm_fixup_kernel<DD>, dim3(grid_for((n_fix + GPW - 1) / GPW)),      \
                         dim3(256), 0, st, fix_row, fix_ptr, n_fix, partial, e);               \
  } break;
  switch (d) {
    MIREC_SPMM(32)
    MIREC_SPMM(64)
    MIREC_SPMM(128)
    MIREC_SPMM(256)
    default:
      set_error("mirec_spmm_csr_f32: embedding_size %d not in {32,64,128,256}", d);
      return -1;
  }
#undef MIREC_SPMM
  return launch_status("mirec_spmm_csr_f32");
}

extern "C" int mirec_gather_sqnorm_f32(const float* table, int64_t n_rows, int32_t d,
                                       const int64_t* idx, int64_t n, float* sq, void* stream) {
  if (n == 0) return 0;
  if (!table || !idx || !sq || n < 0 || n_rows <= 0 || d <= 0) {
    set_error("mirec_gather_sqnorm_f32: bad arguments");
    return -1;
  }
  hipLaunchKernelGGL(gather_sqnorm_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                     table, n_rows, d, idx, n, sq);
  return launch_status("mirec_gather_sqnorm_f32");
}

extern "C" int mirec_gather_scale_rows_f32(const float* table, int64_t n_rows, int32_t d,
                                           const int64_t* idx, int64_t n, const float* scale_dev,
                                           float* out, void* stream) {
  if (n == 0) return 0;
  if (!table || !idx || !scale_dev || !out || n < 0 || n_rows <= 0 || d <= 0) {
    set_error("mirec_gather_scale_rows_f32: bad arguments");
    return -1;
  }
  int64_t blocks = (n * d + 255) / 256;
  if (blocks > 256 * 16) blocks = 256 * 16;
  hipLaunchKernelGGL(gather_scale_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     (hipStream_t)stream, table, n_rows, d, idx, n, scale_dev, out);
  return launch_status("mirec_gather_scale_rows_f32");
}
