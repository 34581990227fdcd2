// K8 — context-aware field embedding + factorization machine + BCE, fused.
//
// Restates, for one batch of samples (recbole/model/...):
//   ContextRecommender.embed_input_fields / concat_embed_input_fields
//     (abstract_recommender.py:286-412): token fields through one offset table
//     (FMEmbedding, layers.py:121-144), token_seq fields as masked means
//     sum(mask*e) / (cnt + 1e-8) (:231-272), float fields as E_f[j] * x_j
//     (:199-214); concatenated [token | token_seq | float] along the field axis;
//   FMFirstOrderLinear.forward (layers.py:1029-1062): sum of the first-order
//     weights (float: w_j*x_j, token: w[id], token_seq: sum of masked w) + bias;
//   BaseFactorizationMachine(reduce_sum=True) (layers.py:147-171):
//     0.5 * sum_k ((sum_f e_fk)^2 - sum_f e_fk^2);
//   DeepFM.forward's y_fm = first_order + fm (deepfm.py:58-70);
//   sigmoid + nn.BCELoss (mean) and their autograd backward.
// The MLP of DeepFM stays a chain of library GEMMs (torch.nn.Linear on
// hipBLASLt); this kernel produces its input (the concatenated field rows) and
// consumes its input gradient.
//
// Layout: one group of LPS = pow2 >= d lanes per sample (lane k owns column k of
// every field row; 64/LPS samples per wave). Field rows of d = 16 floats are one
// 64-B segment per gather. Backward writes per-contribution gradient rows
// (field-major) for the K2 grouping / scatter or the compact Adam — no dense
// gradient of the (up to 33 M-row) table is formed here.
#include "common.h"

namespace mirec {

constexpr int kCtxThreads = 256;

template <int LPS>
__device__ __forceinline__ float group_sum(float x) {
#pragma unroll
  for (int off = LPS / 2; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
  return x;
}

__device__ __forceinline__ int64_t clamp_row(int64_t r, int64_t n) {
  return r < 0 ? 0 : (r >= n ? n - 1 : r);
}

// Forward, two launches. (1) gather: one block row per field (blockIdx.y = f, so the
// field descriptor is block-uniform), LPS lanes per sample: the field's row (token),
// masked mean (token_seq) or scaled row (float) -> concat[b, f, :], its first-order
// term -> fo[b, f], the token row id -> keys. Every (sample, field) pair is independent:
// B * F groups in flight instead of B. (2) reduce, LPS lanes per sample: the FM sums
// S = sum_f e, Q = sum_f e^2 and the first-order sums by kind, all in field order (the
// one-kernel order), y_fm; S is kept for the backward.
template <int LPS>
__global__ __launch_bounds__(kCtxThreads) void ctx_fm_gather_kernel(
    const mirec_ctx_field* __restrict__ fields, int n_fields, int64_t B, int d,
    float* __restrict__ concat, float* __restrict__ fo) {
  constexpr int SPW = 64 / LPS;
  const int lane = threadIdx.x & 63;
  const int k = lane % LPS;
  const int f = blockIdx.y;
  const int64_t b = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * SPW + lane / LPS;
  if (b >= B) return;
  const bool col = k < d;
  const int64_t F = n_fields;
  const mirec_ctx_field fd = fields[f];
  float e = 0.f, w1 = 0.f;
  if (fd.kind == 0) {
    const int64_t r = clamp_row(fd.ids[b] + fd.offset, fd.n_rows);
    if (col) e = fd.table[r * d + k];
    w1 = fd.table1[r];
    if (fd.keys && k == 0) fd.keys[b] = r;
  } else if (fd.kind == 1) {
    const int64_t* ids = fd.ids + b * fd.seq_len;
    float sum = 0.f, cnt = 0.f;
    for (int t = 0; t < fd.seq_len; ++t) {
      const int64_t id = ids[t];
      const float msk = id != 0 ? 1.f : 0.f;
      const int64_t r = clamp_row(id, fd.n_rows);
      if (col) sum += fd.table[r * d + k] * msk;
      w1 += fd.table1[r] * msk;
      cnt += msk;
    }
    e = sum / (cnt + 1e-8f);
  } else {
    const float x = fd.vals[b];
    if (col) e = fd.table[fd.offset * d + k] * x;
    w1 = fd.table1[fd.offset] * x;
  }
  if (col) concat[(b * F + f) * d + k] = e;
  if (k == 0) fo[b * F + f] = w1;
}

template <int LPS>
__global__ __launch_bounds__(kCtxThreads) void ctx_fm_reduce_kernel(
    const mirec_ctx_field* __restrict__ fields, int n_fields, int64_t B, int d,
    const float* __restrict__ bias, const float* __restrict__ concat,
    const float* __restrict__ fo, float* __restrict__ y_fm, float* __restrict__ fm_sum) {
  constexpr int SPW = 64 / LPS;
  const int lane = threadIdx.x & 63;
  const int k = lane % LPS;
  const int64_t b = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * SPW + lane / LPS;
  if (b >= B) return;   // whole groups exit together; no cross-group shuffles below
  const bool col = k < d;
  const int64_t F = n_fields;
  float S = 0.f, Q = 0.f;
  float fo_float = 0.f, fo_tok = 0.f, fo_seq = 0.f;
  // eight fields' loads in flight, then their sums in field order
  constexpr int U = 8;
  for (int f0 = 0; f0 < n_fields; f0 += U) {
    float e[U], w1[U];
    int kind[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int f = f0 + j;
      const bool ok = f < n_fields;
      kind[j] = ok ? fields[f].kind : -1;
      e[j] = ok && col ? concat[(b * F + f) * d + k] : 0.f;
      w1[j] = ok ? fo[b * F + f] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (kind[j] < 0) break;
      if (kind[j] == 0) fo_tok += w1[j];
      else if (kind[j] == 1) fo_seq += w1[j];
      else fo_float += w1[j];
      S += e[j];
      Q += e[j] * e[j];
    }
  }
  if (col) fm_sum[b * d + k] = S;
  const float fm = 0.5f * group_sum<LPS>(col ? S * S - Q : 0.f);
  if (k == 0) y_fm[b] = ((fo_float + fo_tok) + fo_seq) + bias[0] + fm;
}

// Backward, one block row per field as the gather. g_concat: dL/d concat [B, F*d] (may
// be NULL = 0); g_fm: dL/d y_fm [B]; fm_sum: the forward's S.
// grad_e = g_concat + g_fm * (S_k - e) (d fm / d e_fk = S_k - e_fk).
template <int LPS>
__global__ __launch_bounds__(kCtxThreads) void ctx_fm_bwd_kernel(
    const mirec_ctx_field* __restrict__ fields, int n_fields, int64_t B, int d,
    const float* __restrict__ concat, const float* __restrict__ g_concat,
    const float* __restrict__ g_fm, const float* __restrict__ fm_sum) {
  constexpr int SPW = 64 / LPS;
  const int lane = threadIdx.x & 63;
  const int k = lane % LPS;
  const int f = blockIdx.y;
  const int64_t b = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * SPW + lane / LPS;
  if (b >= B) return;
  const bool col = k < d;
  const int64_t F = n_fields;
  const float gf = g_fm[b];
  const mirec_ctx_field fd = fields[f];
  float ge = 0.f;
  if (col) {
    const int64_t c = (b * F + f) * d + k;
    ge = (g_concat ? g_concat[c] : 0.f) + gf * (fm_sum[b * d + k] - concat[c]);
  }
  if (fd.kind == 0) {
    if (col && fd.grad) fd.grad[b * fd.grad_ld + k] = ge;
    if (k == 0 && fd.grad1) fd.grad1[b * fd.grad1_ld] = gf;
  } else if (fd.kind == 1) {
    const int64_t* ids = fd.ids + b * fd.seq_len;
    float cnt = 0.f;
    for (int t = 0; t < fd.seq_len; ++t) cnt += ids[t] != 0 ? 1.f : 0.f;
    const float gm = ge / (cnt + 1e-8f);
    for (int t = 0; t < fd.seq_len; ++t) {
      const float msk = ids[t] != 0 ? 1.f : 0.f;
      if (col && fd.grad) fd.grad[(b * fd.seq_len + t) * d + k] = gm * msk;
      if (k == 0 && fd.grad1) fd.grad1[b * fd.seq_len + t] = gf * msk;
    }
  } else {
    const float x = fd.vals[b];
    if (col && fd.grad) fd.grad[b * fd.grad_ld + k] = ge * x;
    if (k == 0 && fd.grad1) fd.grad1[b * fd.grad1_ld] = gf * x;
  }
}

// z = y_fm + y_deep; p = sigmoid(z); loss_b = -(t*max(log p,-100) + (1-t)*max(log(1-p),-100))
// (torch BCELoss), dz_b = grad_scale * (p - t) / max((1-p)*p, 1e-12) * (1-p) * p
// (BCELoss backward then sigmoid backward, torch's op order).
__global__ __launch_bounds__(256) void sigmoid_bce_kernel(const float* __restrict__ y_fm,
                                                          const float* __restrict__ y_deep,
                                                          const float* __restrict__ label,
                                                          int64_t B, float grad_scale,
                                                          float* __restrict__ prob,
                                                          float* __restrict__ loss,
                                                          float* __restrict__ dz) {
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < B;
       b += (int64_t)gridDim.x * blockDim.x) {
    const float z = y_fm[b] + (y_deep ? y_deep[b] : 0.f);
    const float p = 1.f / (1.f + expf(-z));
    const float t = label ? label[b] : 0.f;
    if (prob) prob[b] = p;
    if (loss) {
      const float lp = fmaxf(logf(p), -100.f);
      const float l1p = fmaxf(logf(1.f - p), -100.f);
      loss[b] = (t - 1.f) * l1p - t * lp;
    }
    if (dz) {
      const float gp = grad_scale * (p - t) / fmaxf((1.f - p) * p, 1e-12f);
      dz[b] = gp * (1.f - p) * p;
    }
  }
}

// out[j] = sum_i x[i*m + j] (column sums; float-field, bias, position and
// LayerNorm gradients). One 1024-thread block per tile of CB columns: thread
// (c, r) sums rows r, r + RG, ... (RG = 1024 / CB row groups, coalesced across c),
// then the RG partials of a column are added in r order. Fixed order,
// independent of timing.
template <int CB>
__global__ __launch_bounds__(1024) void colsum_kernel(const float* __restrict__ x, int64_t n,
                                                      int64_t m, float* __restrict__ out) {
  constexpr int RG = 1024 / CB;
  __shared__ float part[RG][CB + 1];
  const int c = threadIdx.x % CB, r = threadIdx.x / CB;
  const int64_t j = (int64_t)blockIdx.x * CB + c;
  float s = 0.f;
  if (j < m) {
    // 8 rows' loads in flight per thread, added in the same (row) order
    constexpr int U = 8;
    int64_t i = r;
    for (; i + (U - 1) * RG < n; i += U * RG) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = x[(i + u * RG) * m + j];
#pragma unroll
      for (int u = 0; u < U; ++u) s += v[u];
    }
    for (; i < n; i += RG) s += x[i * m + j];
  }
  part[r][c] = s;
  __syncthreads();
  if (r == 0 && j < m) {
    float t = 0.f;
    for (int q = 0; q < RG; ++q) t += part[q][c];
    out[j] = t;
  }
}

// Several column sums in ONE launch (DeepFM's float-field [B, nf*d] and [B, nf] gradients
// and the bias [B, 1]: three launches before): block b takes the job whose block range holds
// it and runs colsum_kernel's body with that job's column tile — the same tile choice as
// mirec_colsum_f32 for its width, so every sum is the one-launch form's bit for bit.
constexpr int kColsumJobs = 4;
struct ColsumJobs {
  const float* x[kColsumJobs];
  float* out[kColsumJobs];
  int64_t n[kColsumJobs], m[kColsumJobs];
  int32_t cb[kColsumJobs];
  int64_t block_start[kColsumJobs + 1];
  int n_jobs;
};

template <int CB>
__device__ __forceinline__ void colsum_tile(const float* __restrict__ x, int64_t n, int64_t m,
                                            float* __restrict__ out, int64_t tile,
                                            float* part) {     // [RG][CB + 1]
  constexpr int RG = 1024 / CB;
  const int c = threadIdx.x % CB, r = threadIdx.x / CB;
  const int64_t j = tile * CB + c;
  float s = 0.f;
  if (j < m) {
    constexpr int U = 8;
    int64_t i = r;
    for (; i + (U - 1) * RG < n; i += U * RG) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = x[(i + u * RG) * m + j];
#pragma unroll
      for (int u = 0; u < U; ++u) s += v[u];
    }
    for (; i < n; i += RG) s += x[i * m + j];
  }
  part[r * (CB + 1) + c] = s;
  __syncthreads();
  if (r == 0 && j < m) {
    float t = 0.f;
    for (int q = 0; q < RG; ++q) t += part[q * (CB + 1) + c];
    out[j] = t;
  }
}

__global__ __launch_bounds__(1024) void colsum_multi_kernel(const ColsumJobs J) {
  __shared__ float part[2048];         // [RG][CB + 1] of the largest form (CB = 1: 1024 x 2)
  int q = 0;
#pragma unroll
  for (int t = 1; t < kColsumJobs; ++t)
    if (t < J.n_jobs && (int64_t)blockIdx.x >= J.block_start[t]) q = t;
  const int64_t tile = (int64_t)blockIdx.x - J.block_start[q];
  if (J.cb[q] == 64)
    colsum_tile<64>(J.x[q], J.n[q], J.m[q], J.out[q], tile, part);
  else if (J.cb[q] == 8)
    colsum_tile<8>(J.x[q], J.n[q], J.m[q], J.out[q], tile, part);
  else
    colsum_tile<1>(J.x[q], J.n[q], J.m[q], J.out[q], tile, part);
}

// The tail of a Linear's backward over a tall input (SASRec's 12 Linears at K = B x L =
// 10^5 rows, model/layers.py _SplitKLinearFn): the sum of the C split-K weight-gradient
// partials and the bias gradient (the column sum of g [K, n_out]) in ONE launch, where
// torch ran two reductions (24 reduce launches per C3 step). Fixed orders: the partials
// in c order; the bias rows in chunks of kLgRows, each chunk's rows in row order (8 row
// lanes, added in lane order), the chunks in chunk order — the last block to finish a
// chunk (agent-scope ticket; write-through partial stores drained before it, an agent
// acquire after, then plain loads) adds them.
constexpr int kLgThreads = 256;
#ifndef MIREC_LG_ROWS
#define MIREC_LG_ROWS 512
#endif
constexpr int kLgRows = MIREC_LG_ROWS;  // bias rows per chunk (C3: 512 -> 15.6 us, 1024 -> 20.1,
                                        // 256 no better; 2048: 50 blocks for K = 10^5
                                        // rows, too few waves to stream g)
constexpr int kLgSumThreads = 64;     // lanes per block of the partial sum (256: 16 blocks for
                                      // a 128 x 128 dW, each lane walking C partials)
struct LinearGradFinish {
  const float* P; int C; int64_t n4;  // partials [C, 4 n4] -> dW
  float* dW;
  const float* g; int64_t K; int n_out; float* db;
  float* scratch; int32_t* ticket;
  int nS;                             // blocks of the partial sum
  int nB;                             // bias chunks
};

__global__ __launch_bounds__(kLgThreads) void linear_grad_finish_kernel(const LinearGradFinish F) {
  const int tid = threadIdx.x;
  if ((int)blockIdx.x < F.nS) {
    // the first kLgSumThreads lanes of each block (the launch's block size serves the
    // bias chunks); eight partials' loads in flight, added in c order
    const int64_t i = (int64_t)blockIdx.x * kLgSumThreads + tid;
    if (tid >= kLgSumThreads || i >= F.n4) return;
    const float4* P4 = reinterpret_cast<const float4*>(F.P);
    float4 v = P4[i];
    int c = 1;
    for (; c + 8 <= F.C; c += 8) {
      float4 w[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) w[u] = P4[(int64_t)(c + u) * F.n4 + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        v.x += w[u].x; v.y += w[u].y; v.z += w[u].z; v.w += w[u].w;
      }
    }
    for (; c < F.C; ++c) {
      const float4 w = P4[(int64_t)c * F.n4 + i];
      v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
    }
    reinterpret_cast<float4*>(F.dW)[i] = v;
    return;
  }
  // bias chunk: thread = (row lane rl of 8, column float4 cg); 256 / 8 = 32 float4 groups
  // per pass over the columns
  __shared__ float4 part[8][33];
  __shared__ int s_last;
  const int chunk = (int)blockIdx.x - F.nS;
  const int rl = tid >> 5, cgl = tid & 31;
  const int64_t r0 = (int64_t)chunk * kLgRows;
  const int64_t r1 = r0 + kLgRows < F.K ? r0 + kLgRows : F.K;
  const int ng = F.n_out / 4;
  float* mine = F.scratch + (int64_t)chunk * F.n_out;
  for (int cg0 = 0; cg0 < ng; cg0 += 32) {
    const int cg = cg0 + cgl;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (cg < ng) {
      const float4* g4 = reinterpret_cast<const float4*>(F.g) + cg;
      int64_t r = r0 + rl;
      for (; r + 24 < r1; r += 32) {                   // 4 rows' loads in flight
        const float4 a = g4[r * ng], b = g4[(r + 8) * ng], c = g4[(r + 16) * ng],
                     d = g4[(r + 24) * ng];
        s.x = (((s.x + a.x) + b.x) + c.x) + d.x;
        s.y = (((s.y + a.y) + b.y) + c.y) + d.y;
        s.z = (((s.z + a.z) + b.z) + c.z) + d.z;
        s.w = (((s.w + a.w) + b.w) + c.w) + d.w;
      }
      for (; r < r1; r += 8) {
        const float4 a = g4[r * ng];
        s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
      }
    }
    part[rl][cgl] = s;
    __syncthreads();
    if (rl == 0 && cg < ng) {
      float4 t = part[0][cgl];
#pragma unroll
      for (int q = 1; q < 8; ++q) {
        t.x += part[q][cgl].x; t.y += part[q][cgl].y; t.z += part[q][cgl].z; t.w += part[q][cgl].w;
      }
      auto q8 = (__attribute__((address_space(1))) unsigned long long*)(mine + 4 * cg);
      __hip_atomic_store(q8, (unsigned long long)__float_as_uint(t.x) |
                                 ((unsigned long long)__float_as_uint(t.y) << 32),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(q8 + 1, (unsigned long long)__float_as_uint(t.z) |
                                     ((unsigned long long)__float_as_uint(t.w) << 32),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
  }
  // hand-off: every storing wave drained, meet, one add; the last chunk sums them all
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int prev = __hip_atomic_fetch_add(F.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == F.nB - 1;
    if (s_last) {
      __hip_atomic_store(F.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!s_last) return;
  // after the acquire: plain loads (the guide's consumer form). Thread = (float4 column
  // group, chunk slice): each slice sums its consecutive chunks in chunk order (8 loads in
  // flight), then the slices are added in slice order — a fixed order, and a few dependent
  // load rounds where one lane per column walking all nB chunks took nB / 16
  const int ns = ng >= kLgThreads ? 1 : kLgThreads / ng;     // slices
  const int cpp = kLgThreads / ns;                            // column groups per pass
  const int per = (F.nB + ns - 1) / ns;
  float4* tp = &part[0][0];                                   // 264 >= kLgThreads float4
  const int sl = tid / cpp, cgt = tid % cpp;
  for (int cg0 = 0; cg0 < ng; cg0 += cpp) {
    const int cg = cg0 + cgt;
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    if (cg < ng) {
      const float4* src = reinterpret_cast<const float4*>(F.scratch) + cg;
      const int c1 = min(F.nB, (sl + 1) * per);
      int c = sl * per;
      for (; c + 8 <= c1; c += 8) {
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = src[(int64_t)(c + u) * ng];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          t.x += v[u].x; t.y += v[u].y; t.z += v[u].z; t.w += v[u].w;
        }
      }
      for (; c < c1; ++c) {
        const float4 v = src[(int64_t)c * ng];
        t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
      }
    }
    tp[tid] = t;
    __syncthreads();
    if (sl == 0 && cg < ng) {
      float4 u = tp[cgt];
      for (int q = 1; q < ns; ++q) {
        const float4 w = tp[q * cpp + cgt];
        u.x += w.x; u.y += w.y; u.z += w.z; u.w += w.w;
      }
      reinterpret_cast<float4*>(F.db)[cg] = u;
    }
    __syncthreads();
  }
}

// keys[f * B + i] = cols[f][i] + offsets[f]: DeepFM's token keys (every token field's ids at
// its offset in the shared table) in one launch (a stack + add in torch: two)
constexpr int kKeyFields = 64;
struct KeyFields {
  const int64_t* col[kKeyFields];
  int64_t off[kKeyFields];
};

__global__ __launch_bounds__(256) void offset_keys_kernel(const KeyFields F, int n_fields,
                                                          int64_t B, int64_t* __restrict__ out) {
  const int f = blockIdx.y;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < B; i += (int64_t)gridDim.x * 256)
    out[(int64_t)f * B + i] = F.col[f][i] + F.off[f];
}

static unsigned ctx_grid(int64_t B, int lps) {
  const int64_t spb = (kCtxThreads / 64) * (64 / lps);
  return (unsigned)((B + spb - 1) / spb);
}

}  // namespace mirec

using namespace mirec;

#define MIREC_CTX_DISPATCH(KERNEL, NY, ...)                                                   \
  do {                                                                                        \
    hipStream_t st = (hipStream_t)stream;                                                     \
    const unsigned ny = (unsigned)(NY);                                                       \
    if (d <= 4)                                                                               \
      hipLaunchKernelGGL(KERNEL<4>, dim3(ctx_grid(B, 4), ny), dim3(kCtxThreads), 0, st,       \
                         __VA_ARGS__);                                                        \
    else if (d <= 8)                                                                          \
      hipLaunchKernelGGL(KERNEL<8>, dim3(ctx_grid(B, 8), ny), dim3(kCtxThreads), 0, st,       \
                         __VA_ARGS__);                                                        \
    else if (d <= 16)                                                                         \
      hipLaunchKernelGGL(KERNEL<16>, dim3(ctx_grid(B, 16), ny), dim3(kCtxThreads), 0, st,     \
                         __VA_ARGS__);                                                        \
    else if (d <= 32)                                                                         \
      hipLaunchKernelGGL(KERNEL<32>, dim3(ctx_grid(B, 32), ny), dim3(kCtxThreads), 0, st,     \
                         __VA_ARGS__);                                                        \
    else                                                                                      \
      hipLaunchKernelGGL(KERNEL<64>, dim3(ctx_grid(B, 64), ny), dim3(kCtxThreads), 0, st,     \
                         __VA_ARGS__);                                                        \
  } while (0)

extern "C" size_t mirec_ctx_fm_work_floats(int64_t B, int32_t n_fields, int32_t d) {
  return B < 0 || n_fields < 0 || d < 0 ? 0 : (size_t)B * ((size_t)n_fields + (size_t)d);
}

extern "C" int mirec_ctx_fm_fwd_f32(const mirec_ctx_field* fields_dev, int32_t n_fields,
                                    int64_t B, int32_t d, const float* bias, float* concat,
                                    float* y_fm, float* work, void* stream) {
  if (B == 0) return 0;
  if (!fields_dev || n_fields <= 0 || n_fields > 65535 || B < 0 || d < 1 || d > 64 || !bias ||
      !concat || !y_fm || !work) {
    set_error("mirec_ctx_fm_fwd_f32: bad arguments (1 <= d <= 64, 1 <= fields <= 65535)");
    return -1;
  }
  float* fo = work;
  float* fm_sum = work + B * n_fields;
  MIREC_CTX_DISPATCH(ctx_fm_gather_kernel, n_fields, fields_dev, n_fields, B, d, concat, fo);
  const int rc = launch_status("mirec_ctx_fm_fwd_f32: gather");
  if (rc) return rc;
  MIREC_CTX_DISPATCH(ctx_fm_reduce_kernel, 1, fields_dev, n_fields, B, d, bias, concat, fo, y_fm,
                     fm_sum);
  return launch_status("mirec_ctx_fm_fwd_f32");
}

extern "C" int mirec_ctx_fm_bwd_f32(const mirec_ctx_field* fields_dev, int32_t n_fields,
                                    int64_t B, int32_t d, const float* concat,
                                    const float* g_concat, const float* g_fm, const float* work,
                                    void* stream) {
  if (B == 0) return 0;
  if (!fields_dev || n_fields <= 0 || n_fields > 65535 || B < 0 || d < 1 || d > 64 || !concat ||
      !g_fm || !work) {
    set_error("mirec_ctx_fm_bwd_f32: bad arguments (1 <= d <= 64, 1 <= fields <= 65535)");
    return -1;
  }
  MIREC_CTX_DISPATCH(ctx_fm_bwd_kernel, n_fields, fields_dev, n_fields, B, d, concat, g_concat,
                     g_fm, work + B * n_fields);
  return launch_status("mirec_ctx_fm_bwd_f32");
}

// The loss and its gradient in one launch for the training step: one 1024-lane block,
// lane t computes samples t, t + 1024, ... (loss terms and dz as sigmoid_bce_kernel) and
// sums its loss terms in that order, then a fixed binary tree over the 1024 partials
// (capi.hip block_fixed_sum's order) and the mean = sum / B — what mirec_sigmoid_bce_f32 +
// mirec_sum_f32 + a division gave, bit for bit, in one launch instead of three.
__global__ __launch_bounds__(1024) void sigmoid_bce_mean_kernel(
    const float* __restrict__ y_fm, const float* __restrict__ y_deep,
    const float* __restrict__ label, int64_t B, float grad_scale, float* __restrict__ loss_b,
    float* __restrict__ loss_mean, float* __restrict__ dz) {
  __shared__ float lds[1024];
  float acc = 0.f;
  for (int64_t b = threadIdx.x; b < B; b += 1024) {
    const float z = y_fm[b] + (y_deep ? y_deep[b] : 0.f);
    const float p = 1.f / (1.f + expf(-z));
    const float t = label[b];
    const float lp = fmaxf(logf(p), -100.f);
    const float l1p = fmaxf(logf(1.f - p), -100.f);
    const float lb = (t - 1.f) * l1p - t * lp;
    if (loss_b) loss_b[b] = lb;
    acc += lb;
    const float gp = grad_scale * (p - t) / fmaxf((1.f - p) * p, 1e-12f);
    dz[b] = gp * (1.f - p) * p;
  }
  lds[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 512; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) lds[threadIdx.x] += lds[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss_mean[0] = lds[0] / (float)B;
}

extern "C" int mirec_sigmoid_bce_mean_f32(const float* y_fm, const float* y_deep,
                                          const float* label, int64_t B, float grad_scale,
                                          float* loss_b, float* loss_mean, float* dz,
                                          void* stream) {
  if (!y_fm || !label || !loss_mean || !dz || B <= 0 || B > (1 << 24)) {
    set_error("mirec_sigmoid_bce_mean_f32: bad arguments (0 < B <= 2^24)");
    return -1;
  }
  hipLaunchKernelGGL(sigmoid_bce_mean_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, y_fm,
                     y_deep, label, B, grad_scale, loss_b, loss_mean, dz);
  return launch_status("mirec_sigmoid_bce_mean_f32");
}

extern "C" int mirec_sigmoid_bce_f32(const float* y_fm, const float* y_deep, const float* label,
                                     int64_t B, float grad_scale, float* prob, float* loss,
                                     float* dz, void* stream) {
  if (B == 0) return 0;
  if (!y_fm || B < 0 || (!label && (loss || dz))) {
    set_error("mirec_sigmoid_bce_f32: bad arguments (loss / dz need labels)");
    return -1;
  }
  int64_t blocks = (B + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(sigmoid_bce_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     (hipStream_t)stream, y_fm, y_deep, label, B, grad_scale, prob, loss, dz);
  return launch_status("mirec_sigmoid_bce_f32");
}

extern "C" int mirec_colsum_multi_f32(const float* const* x, const int64_t* n, const int64_t* m,
                                      float* const* out, int32_t n_jobs, void* stream) {
  if (n_jobs < 0 || n_jobs > kColsumJobs || (n_jobs > 0 && (!x || !n || !m || !out))) {
    set_error("mirec_colsum_multi_f32: bad arguments (at most %d jobs)", kColsumJobs);
    return -1;
  }
  ColsumJobs J;
  memset(&J, 0, sizeof(J));
  int64_t blocks = 0;
  int k = 0;
  for (int q = 0; q < n_jobs; ++q) {
    if (m[q] == 0) continue;
    if (!x[q] || !out[q] || n[q] < 0 || m[q] < 0) {
      set_error("mirec_colsum_multi_f32: bad job %d", q);
      return -1;
    }
    const int cb = m[q] >= 64 ? 64 : (m[q] >= 8 ? 8 : 1);   // mirec_colsum_f32's tile
    J.x[k] = x[q];
    J.out[k] = out[q];
    J.n[k] = n[q];
    J.m[k] = m[q];
    J.cb[k] = cb;
    J.block_start[k] = blocks;
    blocks += (m[q] + cb - 1) / cb;
    ++k;
  }
  J.n_jobs = k;
  for (int q = k; q <= kColsumJobs; ++q) J.block_start[q] = blocks;
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(colsum_multi_kernel, dim3((unsigned)blocks), dim3(1024), 0,
                     (hipStream_t)stream, J);
  return launch_status("mirec_colsum_multi_f32");
}

extern "C" int mirec_offset_keys(const int64_t* const* cols, const int64_t* offsets,
                                 int32_t n_fields, int64_t B, int64_t* out, void* stream) {
  if (n_fields < 0 || n_fields > kKeyFields || B < 0 || (n_fields > 0 && B > 0 &&
      (!cols || !offsets || !out))) {
    set_error("mirec_offset_keys: bad arguments (at most %d fields)", kKeyFields);
    return -1;
  }
  if (n_fields == 0 || B == 0) return 0;
  KeyFields F;
  memset(&F, 0, sizeof(F));
  for (int f = 0; f < n_fields; ++f) {
    if (!cols[f]) {
      set_error("mirec_offset_keys: field %d has no column", f);
      return -1;
    }
    F.col[f] = cols[f];
    F.off[f] = offsets[f];
  }
  const unsigned gx = (unsigned)std::min<int64_t>((B + 255) / 256, 64);
  hipLaunchKernelGGL(offset_keys_kernel, dim3(gx, (unsigned)n_fields), dim3(256), 0,
                     (hipStream_t)stream, F, n_fields, B, out);
  return launch_status("mirec_offset_keys");
}

extern "C" int64_t mirec_linear_grad_finish_scratch(int64_t K, int32_t n_out) {
  if (K < 0 || n_out < 0) return -1;
  return ((K + kLgRows - 1) / kLgRows) * (int64_t)n_out;
}

extern "C" int mirec_linear_grad_finish_f32(const float* P, int32_t C, int64_t n_w, float* dW,
                                            const float* g, int64_t K, int32_t n_out, float* db,
                                            float* scratch, int32_t* ticket, void* stream) {
  const char* what = "mirec_linear_grad_finish_f32";
  const bool sum = P && C >= 1 && n_w > 0 && !(C == 1 && P == dW);
  const bool bias = db != nullptr && K > 0;
  if (C < 1 || n_w < 0 || (n_w % 4) != 0 || (sum && !dW) ||
      ((uintptr_t)P % 16) != 0 || ((uintptr_t)dW % 16) != 0 ||
      (bias && (!g || n_out <= 0 || (n_out % 4) != 0 || ((uintptr_t)g % 16) != 0 || !scratch ||
                !ticket || ((uintptr_t)scratch % 16) != 0 || ((uintptr_t)db % 16) != 0))) {
    set_error("%s: bad arguments", what);
    return -1;
  }
  LinearGradFinish F;
  memset(&F, 0, sizeof(F));
  F.P = P; F.C = C; F.n4 = n_w / 4; F.dW = dW;
  F.g = g; F.K = K; F.n_out = n_out; F.db = db; F.scratch = scratch; F.ticket = ticket;
  F.nS = sum ? (int)((F.n4 + kLgSumThreads - 1) / kLgSumThreads) : 0;
  F.nB = bias ? (int)((K + kLgRows - 1) / kLgRows) : 0;
  if (F.nS + F.nB == 0) return 0;
  hipLaunchKernelGGL(linear_grad_finish_kernel, dim3((unsigned)(F.nS + F.nB)), dim3(kLgThreads), 0,
                     (hipStream_t)stream, F);
  return launch_status(what);
}

extern "C" int mirec_colsum_f32(const float* x, int64_t n, int64_t m, float* out, void* stream) {
  if (m == 0) return 0;
  if (!x || !out || n < 0 || m < 0) {
    set_error("mirec_colsum_f32: bad arguments");
    return -1;
  }
  hipStream_t st = (hipStream_t)stream;
  if (m >= 64)
    hipLaunchKernelGGL(colsum_kernel<64>, dim3((unsigned)((m + 63) / 64)), dim3(1024), 0, st, x,
                       n, m, out);
  else if (m >= 8)
    hipLaunchKernelGGL(colsum_kernel<8>, dim3((unsigned)((m + 7) / 8)), dim3(1024), 0, st, x, n,
                       m, out);
  else
    hipLaunchKernelGGL(colsum_kernel<1>, dim3((unsigned)m), dim3(1024), 0, st, x, n, m, out);
  return launch_status("mirec_colsum_f32");
}
