// K9 — sequential recommender (SASRec) embedding side and sampled softmax.
//
// K9a  seq_embed_ln: restates the input block of SASRec.forward
//   (recbole/model/sequential_recommender/sasrec.py:107-117):
//     x[b,t] = item_embedding[item_seq[b,t]] + position_embedding[t]
//     y[b,t] = LayerNorm(x[b,t]) = (x - mean) * rstd * gamma + beta
//   and its autograd backward: dx = rstd * (g*gamma - mean(g*gamma)
//   - xhat * mean(g*gamma*xhat)); dgamma = sum g*xhat, dbeta = sum g (per-block
//   partials in a fixed order, then a fixed-order column sum); the item rows'
//   gradient is returned per contribution for the K2 grouping (row 0 = the
//   padding_idx row receives none, nn.Embedding(padding_idx=0)).
// K9b  sampled softmax over [positive | N negatives] per sequence (the C3
//   config's loss, a build extension — the reference has BPR and full CE only):
//     logit_j = <s_b, E[item_bj]>, loss_b = logsumexp_j(logit) - logit_0,
//     dS_b = scale * (sum_j p_j E_j - E_0), dE_bj = scale * (p_j - [j==0]) s_b.
//   One wave per sequence, ONE pass over the N+1 rows: an online (running-max)
//   softmax accumulates sum_j p_j E_j while the rows stream in; the logits stay
//   in LDS for the row gradients, which need only s_b (no second gather).
//
// Layout: D/4 lanes per row (float4 per lane), 64/(D/4) rows per wave for K9a.
#include "common.h"

namespace mirec {

template <int LPR>
__device__ __forceinline__ float lane_group_sum(float x) {
#pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
  return x;
}

__device__ __forceinline__ float sum4(float4 a) { return (a.x + a.y) + (a.z + a.w); }

constexpr int kLnRowsPerBlock = 64;   // K9a backward partial-sum chunk (fixed)

// Dropout folded into K9a / K9d (counter-based draws; the K9d header below spells them out)
struct LnDrop {
  uint32_t thr;
  float scale;
  uint64_t seed;
  int64_t* counter;     // forward: read; backward: set to drawn + 1
  int64_t* drawn;       // forward writes the counter value used; backward reads it
};

__device__ __forceinline__ uint64_t ln_mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// keep flags of the four elements e0 .. e0 + 3 (e0 a multiple of 4)
__device__ __forceinline__ void ln_keep4(uint64_t key, uint64_t e0, uint32_t thr, bool (&k)[4]) {
  const uint64_t h0 = ln_mix(key ^ (e0 >> 1)), h1 = ln_mix(key ^ ((e0 >> 1) + 1));
  k[0] = (uint32_t)h0 < thr;
  k[1] = (uint32_t)(h0 >> 32) < thr;
  k[2] = (uint32_t)h1 < thr;
  k[3] = (uint32_t)(h1 >> 32) < thr;
}


// DROP: SASRec's embedding dropout (sasrec.py:107-114, after the LayerNorm) folded in: the
// output is drop(LayerNorm(...)), the backward masks the incoming gradient the same way.
template <int D, bool DROP = false>
__global__ __launch_bounds__(256) void seq_embed_ln_fwd_kernel(
    const float* __restrict__ E, int64_t n_items, const float* __restrict__ P,
    const int64_t* __restrict__ seq, int64_t n_rows, int L, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, float* __restrict__ out,
    float* __restrict__ mean_out, float* __restrict__ rstd_out, LnDrop dr) {
  constexpr int LPR = D / 4, GPW = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const int g = lane / LPR, l = lane % LPR;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t r = wave * GPW + g;
  uint64_t key = 0;
  if (DROP) {
    const int64_t cv = dr.counter[0];
    key = ln_mix(dr.seed + (uint64_t)cv);
    if (blockIdx.x == 0 && threadIdx.x == 0) dr.drawn[0] = cv;
  }
  if (r >= n_rows) return;
  int64_t id = seq[r];
  id = id < 0 ? 0 : (id >= n_items ? n_items - 1 : id);
  const int t = (int)(r % L);
  const float4 e = reinterpret_cast<const float4*>(E + id * D)[l];
  const float4 p = reinterpret_cast<const float4*>(P + (int64_t)t * D)[l];
  float4 x = make_float4(e.x + p.x, e.y + p.y, e.z + p.z, e.w + p.w);
  const float mean = lane_group_sum<LPR>(sum4(x)) * (1.0f / D);
  float4 c = make_float4(x.x - mean, x.y - mean, x.z - mean, x.w - mean);
  const float var = lane_group_sum<LPR>(c.x * c.x + c.y * c.y + c.z * c.z + c.w * c.w) *
                    (1.0f / D);
  const float rstd = 1.0f / sqrtf(var + eps);
  const float4 gm = reinterpret_cast<const float4*>(gamma)[l];
  const float4 bt = reinterpret_cast<const float4*>(beta)[l];
  float4 y;
  y.x = c.x * rstd * gm.x + bt.x;
  y.y = c.y * rstd * gm.y + bt.y;
  y.z = c.z * rstd * gm.z + bt.z;
  y.w = c.w * rstd * gm.w + bt.w;
  if (DROP) {
    bool k[4];
    ln_keep4(key, (uint64_t)r * D + 4 * l, dr.thr, k);
    y.x = k[0] ? y.x * dr.scale : 0.f;
    y.y = k[1] ? y.y * dr.scale : 0.f;
    y.z = k[2] ? y.z * dr.scale : 0.f;
    y.w = k[3] ? y.w * dr.scale : 0.f;
  }
  reinterpret_cast<float4*>(out + r * D)[l] = y;
  if (l == 0) {
    mean_out[r] = mean;
    rstd_out[r] = rstd;
  }
}

// Block = 4 waves over kLnRowsPerBlock consecutive rows; writes dx rows, the
// item-row gradient (0 for padding id 0) and the block's partial dgamma / dbeta.
template <int D, bool DROP = false>
__global__ __launch_bounds__(256) void seq_embed_ln_bwd_kernel(
    const float* __restrict__ E, int64_t n_items, const float* __restrict__ P,
    const int64_t* __restrict__ seq, int64_t n_rows, int L, const float* __restrict__ gamma,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const float* __restrict__ gy, float* __restrict__ dx, float* __restrict__ ditem,
    float* __restrict__ part_gamma, float* __restrict__ part_beta, LnDrop dr) {
  constexpr int LPR = D / 4, GPW = 64 / LPR;
  const int64_t cv = DROP ? dr.drawn[0] : 0;
  const uint64_t key = DROP ? ln_mix(dr.seed + (uint64_t)cv) : 0ull;
  if (DROP && blockIdx.x == 0 && threadIdx.x == 0) dr.counter[0] = cv + 1;   // the next draw
  __shared__ float4 red_g[4 * GPW][LPR];
  __shared__ float4 red_b[4 * GPW][LPR];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int g = lane / LPR, l = lane % LPR;
  const float4 gm = reinterpret_cast<const float4*>(gamma)[l];
  float4 ag = make_float4(0.f, 0.f, 0.f, 0.f), ab = ag;
  const int64_t base = (int64_t)blockIdx.x * kLnRowsPerBlock;
  for (int i = w * GPW + g; i < kLnRowsPerBlock; i += 4 * GPW) {
    const int64_t r = base + i;
    if (r >= n_rows) break;
    int64_t id = seq[r];
    const bool pad = id == 0;
    id = id < 0 ? 0 : (id >= n_items ? n_items - 1 : id);
    const int t = (int)(r % L);
    const float4 e = reinterpret_cast<const float4*>(E + id * D)[l];
    const float4 p = reinterpret_cast<const float4*>(P + (int64_t)t * D)[l];
    const float mean = mean_in[r], rstd = rstd_in[r];
    float4 xh;
    xh.x = (e.x + p.x - mean) * rstd;
    xh.y = (e.y + p.y - mean) * rstd;
    xh.z = (e.z + p.z - mean) * rstd;
    xh.w = (e.w + p.w - mean) * rstd;
    float4 gv = reinterpret_cast<const float4*>(gy + r * D)[l];
    if (DROP) {
      bool k[4];
      ln_keep4(key, (uint64_t)r * D + 4 * l, dr.thr, k);
      gv.x = k[0] ? gv.x * dr.scale : 0.f;
      gv.y = k[1] ? gv.y * dr.scale : 0.f;
      gv.z = k[2] ? gv.z * dr.scale : 0.f;
      gv.w = k[3] ? gv.w * dr.scale : 0.f;
    }
    const float4 gg = make_float4(gv.x * gm.x, gv.y * gm.y, gv.z * gm.z, gv.w * gm.w);
    const float m1 = lane_group_sum<LPR>(sum4(gg)) * (1.0f / D);
    const float m2 =
        lane_group_sum<LPR>(gg.x * xh.x + gg.y * xh.y + gg.z * xh.z + gg.w * xh.w) *
        (1.0f / D);
    float4 o;
    o.x = rstd * (gg.x - m1 - xh.x * m2);
    o.y = rstd * (gg.y - m1 - xh.y * m2);
    o.z = rstd * (gg.z - m1 - xh.z * m2);
    o.w = rstd * (gg.w - m1 - xh.w * m2);
    if (dx) reinterpret_cast<float4*>(dx + r * D)[l] = o;
    if (ditem)
      reinterpret_cast<float4*>(ditem + r * D)[l] = pad ? make_float4(0.f, 0.f, 0.f, 0.f) : o;
    ag.x += gv.x * xh.x;
    ag.y += gv.y * xh.y;
    ag.z += gv.z * xh.z;
    ag.w += gv.w * xh.w;
    ab.x += gv.x;
    ab.y += gv.y;
    ab.z += gv.z;
    ab.w += gv.w;
  }
  red_g[w * GPW + g][l] = ag;
  red_b[w * GPW + g][l] = ab;
  __syncthreads();
  if (threadIdx.x < LPR) {
    float4 sg = make_float4(0.f, 0.f, 0.f, 0.f), sb = sg;
    for (int q = 0; q < 4 * GPW; ++q) {
      const float4 a = red_g[q][threadIdx.x], b = red_b[q][threadIdx.x];
      sg.x += a.x; sg.y += a.y; sg.z += a.z; sg.w += a.w;
      sb.x += b.x; sb.y += b.y; sb.z += b.z; sb.w += b.w;
    }
    reinterpret_cast<float4*>(part_gamma + (int64_t)blockIdx.x * D)[threadIdx.x] = sg;
    reinterpret_cast<float4*>(part_beta + (int64_t)blockIdx.x * D)[threadIdx.x] = sb;
  }
}

// K9d  residual + LayerNorm of the transformer blocks (layers.py MultiHeadAttention /
//   FeedForward: LayerNorm(dropout(hidden) + input_tensor), reference layers.py:338-552):
//   y = LayerNorm(drop(a) + b) in one pass (the sum is never written), and its backward
//   from the saved mean / rstd with x = drop(a) + b recomputed; same arithmetic as K9a.
//   DROP: the hidden dropout folded in (torch ran it as its own kernel each way). Draws are
//   counter-based: key = splitmix64(seed + c), c the device counter's value at the forward
//   (saved in drawn[0]); the backward redraws from drawn[0] and sets the counter to c + 1
//   (one store: a last-block ticket over the forward's 12,800 workgroups serialised that
//   many atomics on one word, 153 us against 28 for the kernel itself);
//   element e = row * D + column is kept iff the 32-bit half e & 1 of
//   splitmix64(key ^ (e >> 1)) is below thr; a kept element is scaled by 1 / (1 - p).
template <int D, bool DROP>
__global__ __launch_bounds__(256) void add_ln_fwd_kernel(
    const float* __restrict__ A, const float* __restrict__ Bv, int64_t n_rows,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
    float* __restrict__ out, float* __restrict__ mean_out, float* __restrict__ rstd_out,
    LnDrop dr) {
  constexpr int LPR = D / 4, GPW = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const int g = lane / LPR, l = lane % LPR;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t r = wave * GPW + g;
  uint64_t key = 0;
  if (DROP) {
    const int64_t c = dr.counter[0];
    key = ln_mix(dr.seed + (uint64_t)c);
    if (blockIdx.x == 0 && threadIdx.x == 0) dr.drawn[0] = c;
  }
  if (r < n_rows) {
    float4 a = reinterpret_cast<const float4*>(A + r * D)[l];
    if (DROP) {
      bool k[4];
      ln_keep4(key, (uint64_t)r * D + 4 * l, dr.thr, k);
      a.x = k[0] ? a.x * dr.scale : 0.f;
      a.y = k[1] ? a.y * dr.scale : 0.f;
      a.z = k[2] ? a.z * dr.scale : 0.f;
      a.w = k[3] ? a.w * dr.scale : 0.f;
    }
    const float4 b = reinterpret_cast<const float4*>(Bv + r * D)[l];
    float4 x = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    const float mean = lane_group_sum<LPR>(sum4(x)) * (1.0f / D);
    float4 c = make_float4(x.x - mean, x.y - mean, x.z - mean, x.w - mean);
    const float var = lane_group_sum<LPR>(c.x * c.x + c.y * c.y + c.z * c.z + c.w * c.w) *
                      (1.0f / D);
    const float rstd = 1.0f / sqrtf(var + eps);
    const float4 gm = reinterpret_cast<const float4*>(gamma)[l];
    const float4 bt = reinterpret_cast<const float4*>(beta)[l];
    float4 y;
    y.x = c.x * rstd * gm.x + bt.x;
    y.y = c.y * rstd * gm.y + bt.y;
    y.z = c.z * rstd * gm.z + bt.z;
    y.w = c.w * rstd * gm.w + bt.w;
    reinterpret_cast<float4*>(out + r * D)[l] = y;
    if (l == 0) {
      mean_out[r] = mean;
      rstd_out[r] = rstd;
    }
  }
}

// DROP: dx_a = dLN * keep * scale (the gradient of the dropped input), dx_b = dLN; else the
// one dx (both inputs' gradient) in dxb.
template <int D, bool DROP>
__global__ __launch_bounds__(256) void add_ln_bwd_kernel(
    const float* __restrict__ A, const float* __restrict__ Bv, int64_t n_rows,
    const float* __restrict__ gamma, const float* __restrict__ mean_in,
    const float* __restrict__ rstd_in, const float* __restrict__ gy, float* __restrict__ dxb,
    float* __restrict__ dxa, float* __restrict__ part_gamma, float* __restrict__ part_beta,
    LnDrop dr) {
  constexpr int LPR = D / 4, GPW = 64 / LPR;
  __shared__ float4 red_g[4 * GPW][LPR];
  __shared__ float4 red_b[4 * GPW][LPR];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int g = lane / LPR, l = lane % LPR;
  const float4 gm = reinterpret_cast<const float4*>(gamma)[l];
  const int64_t c = DROP ? dr.drawn[0] : 0;
  const uint64_t key = DROP ? ln_mix(dr.seed + (uint64_t)c) : 0ull;
  if (DROP && blockIdx.x == 0 && threadIdx.x == 0) dr.counter[0] = c + 1;   // the next draw
  float4 ag = make_float4(0.f, 0.f, 0.f, 0.f), ab = ag;
  const int64_t base = (int64_t)blockIdx.x * kLnRowsPerBlock;
  for (int i = w * GPW + g; i < kLnRowsPerBlock; i += 4 * GPW) {
    const int64_t r = base + i;
    if (r >= n_rows) break;
    float4 a = reinterpret_cast<const float4*>(A + r * D)[l];
    bool k[4] = {true, true, true, true};
    if (DROP) {
      ln_keep4(key, (uint64_t)r * D + 4 * l, dr.thr, k);
      a.x = k[0] ? a.x * dr.scale : 0.f;
      a.y = k[1] ? a.y * dr.scale : 0.f;
      a.z = k[2] ? a.z * dr.scale : 0.f;
      a.w = k[3] ? a.w * dr.scale : 0.f;
    }
    const float4 b = reinterpret_cast<const float4*>(Bv + r * D)[l];
    const float mean = mean_in[r], rstd = rstd_in[r];
    float4 xh;
    xh.x = (a.x + b.x - mean) * rstd;
    xh.y = (a.y + b.y - mean) * rstd;
    xh.z = (a.z + b.z - mean) * rstd;
    xh.w = (a.w + b.w - mean) * rstd;
    const float4 gv = reinterpret_cast<const float4*>(gy + r * D)[l];
    const float4 gg = make_float4(gv.x * gm.x, gv.y * gm.y, gv.z * gm.z, gv.w * gm.w);
    const float m1 = lane_group_sum<LPR>(sum4(gg)) * (1.0f / D);
    const float m2 =
        lane_group_sum<LPR>(gg.x * xh.x + gg.y * xh.y + gg.z * xh.z + gg.w * xh.w) *
        (1.0f / D);
    float4 o;
    o.x = rstd * (gg.x - m1 - xh.x * m2);
    o.y = rstd * (gg.y - m1 - xh.y * m2);
    o.z = rstd * (gg.z - m1 - xh.z * m2);
    o.w = rstd * (gg.w - m1 - xh.w * m2);
    reinterpret_cast<float4*>(dxb + r * D)[l] = o;
    if (DROP)
      reinterpret_cast<float4*>(dxa + r * D)[l] =
          make_float4(k[0] ? o.x * dr.scale : 0.f, k[1] ? o.y * dr.scale : 0.f,
                      k[2] ? o.z * dr.scale : 0.f, k[3] ? o.w * dr.scale : 0.f);
    ag.x += gv.x * xh.x;
    ag.y += gv.y * xh.y;
    ag.z += gv.z * xh.z;
    ag.w += gv.w * xh.w;
    ab.x += gv.x;
    ab.y += gv.y;
    ab.z += gv.z;
    ab.w += gv.w;
  }
  red_g[w * GPW + g][l] = ag;
  red_b[w * GPW + g][l] = ab;
  __syncthreads();
  if (threadIdx.x < LPR) {
    float4 sg = make_float4(0.f, 0.f, 0.f, 0.f), sb = sg;
    for (int q = 0; q < 4 * GPW; ++q) {
      const float4 a = red_g[q][threadIdx.x], b = red_b[q][threadIdx.x];
      sg.x += a.x; sg.y += a.y; sg.z += a.z; sg.w += a.w;
      sb.x += b.x; sb.y += b.y; sb.z += b.z; sb.w += b.w;
    }
    reinterpret_cast<float4*>(part_gamma + (int64_t)blockIdx.x * D)[threadIdx.x] = sg;
    reinterpret_cast<float4*>(part_beta + (int64_t)blockIdx.x * D)[threadIdx.x] = sb;
  }
}

// GELU of the feed-forward block (layers.py FeedForward.gelu, erf form):
//   y = x * 0.5 * (1 + erf(x / sqrt(2)))   (torch's op order; x / sqrt(2) as its
//   scalar division, multiplication by the reciprocal), and
//   dx = g * (0.5 * (1 + erf(u)) + x * exp(-u^2) / sqrt(2 pi)),  u = x / sqrt(2).
__global__ __launch_bounds__(256) void gelu_fwd_kernel(const float* __restrict__ x,
                                                       int64_t n, float* __restrict__ y) {
  const float rs2 = (float)(1.0 / 1.4142135623730951);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float v = x[i];
    y[i] = v * 0.5f * (1.0f + erff(v * rs2));
  }
}

__global__ __launch_bounds__(256) void gelu_bwd_kernel(const float* __restrict__ x,
                                                       const float* __restrict__ g, int64_t n,
                                                       float* __restrict__ dx) {
  const float rs2 = (float)(1.0 / 1.4142135623730951);
  const float k = (float)(0.3989422804014327);      // 1 / sqrt(2 pi)
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float v = x[i];
    const float u = v * rs2;
    dx[i] = g[i] * (0.5f * (1.0f + erff(u)) + v * k * expf(-u * u));
  }
}

// The same per element, four elements per lane (float4 loads / stores: four independent
// erf chains in flight per lane; n % 4 == 0 and 16-byte aligned pointers)
__device__ __forceinline__ float gelu_f(float v, float rs2) {
  return v * 0.5f * (1.0f + erff(v * rs2));
}
__device__ __forceinline__ float gelu_d(float v, float g, float rs2, float k) {
  const float u = v * rs2;
  return g * (0.5f * (1.0f + erff(u)) + v * k * expf(-u * u));
}

__global__ __launch_bounds__(256) void gelu_fwd4_kernel(const float4* __restrict__ x, int64_t n4,
                                                        float4* __restrict__ y) {
  const float rs2 = (float)(1.0 / 1.4142135623730951);
  const int64_t st = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + st < n4; i += 2 * st) {               // two float4 loads in flight per lane
    const float4 v = x[i], w = x[i + st];
    y[i] = make_float4(gelu_f(v.x, rs2), gelu_f(v.y, rs2), gelu_f(v.z, rs2), gelu_f(v.w, rs2));
    y[i + st] =
        make_float4(gelu_f(w.x, rs2), gelu_f(w.y, rs2), gelu_f(w.z, rs2), gelu_f(w.w, rs2));
  }
  if (i < n4) {
    const float4 v = x[i];
    y[i] = make_float4(gelu_f(v.x, rs2), gelu_f(v.y, rs2), gelu_f(v.z, rs2), gelu_f(v.w, rs2));
  }
}

__global__ __launch_bounds__(256) void gelu_bwd4_kernel(const float4* __restrict__ x,
                                                        const float4* __restrict__ g, int64_t n4,
                                                        float4* __restrict__ dx) {
  const float rs2 = (float)(1.0 / 1.4142135623730951);
  const float k = (float)(0.3989422804014327);      // 1 / sqrt(2 pi)
  const int64_t st = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + st < n4; i += 2 * st) {               // four float4 loads in flight per lane
    const float4 v = x[i], gv = g[i], w = x[i + st], gw = g[i + st];
    dx[i] = make_float4(gelu_d(v.x, gv.x, rs2, k), gelu_d(v.y, gv.y, rs2, k),
                        gelu_d(v.z, gv.z, rs2, k), gelu_d(v.w, gv.w, rs2, k));
    dx[i + st] = make_float4(gelu_d(w.x, gw.x, rs2, k), gelu_d(w.y, gw.y, rs2, k),
                             gelu_d(w.z, gw.z, rs2, k), gelu_d(w.w, gw.w, rs2, k));
  }
  if (i < n4) {
    const float4 v = x[i], gv = g[i];
    dx[i] = make_float4(gelu_d(v.x, gv.x, rs2, k), gelu_d(v.y, gv.y, rs2, k),
                        gelu_d(v.z, gv.z, rs2, k), gelu_d(v.w, gv.w, rs2, k));
  }
}

// x *= g[0] in place, skipped when g[0] == 1 (x * 1 == x for every non-NaN x, zeros and
// infinities included): a loss Function's backward scales its saved per-row gradients by
// the incoming gradient, which a plain loss.backward() makes 1 — the read of g is the whole
// launch then (K9b's item rows: 26.5 M floats, a 34.5 us torch multiply at C3's shape).
__global__ __launch_bounds__(256) void scale_by_kernel(float4* __restrict__ x, int64_t n4,
                                                       const float* __restrict__ g) {
  const float s = g[0];
  if (s == 1.0f) return;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    float4 v = x[i];
    v.x *= s; v.y *= s; v.z *= s; v.w *= s;
    x[i] = v;
  }
}

// K9b. items: pos [B] and negs [N*B] (layout j*B + b, the sampler's).
template <int D>
__global__ __launch_bounds__(256) void sampled_softmax_kernel(
    const float* __restrict__ S, const float* __restrict__ E, int64_t n_items,
    const int64_t* __restrict__ pos, const int64_t* __restrict__ neg, int64_t B, int N,
    float scale, float* __restrict__ loss, float* __restrict__ gS, float* __restrict__ gI) {
  extern __shared__ float lds_logits[];   // (N+1) per wave
  constexpr int V = D / 64;   // floats per lane (D in {64, 128, 256})
  const int lane = threadIdx.x & 63;
  const int64_t b = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (b >= B) return;
  float s[V], acc[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    s[v] = S[b * D + v * 64 + lane];
    acc[v] = 0.f;
  }
  // every lane writes the same value to its wave's slot and reads only what it
  // wrote itself: no cross-lane ordering is involved
  float* lg = lds_logits + (threadIdx.x >> 6) * (N + 1);
  float m = -__builtin_inff(), lsum = 0.f, l0 = 0.f;
  float e0[V];
  // the ids of [pos | negs] up front (lane l holds items l and l + 64), then the rows
  // eight at a time: their loads in flight together, the dots reduced side by side,
  // the online softmax folded in item order as before
  auto item_id = [&](int j) -> int64_t {
    int64_t id = j == 0 ? pos[b] : neg[(int64_t)(j - 1) * B + b];
    return id < 0 ? 0 : (id >= n_items ? n_items - 1 : id);
  };
  const int64_t ida = lane <= N ? item_id(lane) : 0;
  const int64_t idb = lane + 64 <= N ? item_id(lane + 64) : 0;
  for (int j0 = 0; j0 <= N; j0 += 8) {
    float row[8][V], dot[8];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const int j = min(j0 + jj, N);
      int64_t id;
      if (j < 64) {
        id = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(ida >> 32), j) << 32) |
                       (uint32_t)__builtin_amdgcn_readlane((int)ida, j));
      } else if (j < 128) {
        id = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(idb >> 32), j - 64)
                        << 32) | (uint32_t)__builtin_amdgcn_readlane((int)idb, j - 64));
      } else {
        id = item_id(j);
      }
#pragma unroll
      for (int v = 0; v < V; ++v) row[jj][v] = E[id * D + v * 64 + lane];
    }
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      float d0 = 0.f;
#pragma unroll
      for (int v = 0; v < V; ++v) d0 = fmaf(s[v], row[jj][v], d0);
      dot[jj] = d0;
    }
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) dot[jj] = wave_sum(dot[jj]);
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const int j = j0 + jj;
      if (j > N) break;
      lg[j] = dot[jj];
      if (j == 0) l0 = dot[jj];
      const float mn = fmaxf(m, dot[jj]);
      const float cold = expf(m - mn), cnew = expf(dot[jj] - mn);
      lsum = lsum * cold + cnew;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        acc[v] = acc[v] * cold + cnew * row[jj][v];
        if (j == 0) e0[v] = row[jj][v];
      }
      m = mn;
    }
  }
  const float lse = m + logf(lsum);
  if (lane == 0) loss[b] = lse - l0;
  const float inv = 1.f / lsum;
#pragma unroll
  for (int v = 0; v < V; ++v) gS[b * D + v * 64 + lane] = scale * (acc[v] * inv - e0[v]);
  for (int j = 0; j <= N; ++j) {
    const float p = expf(lg[j] - lse);
    const float c = scale * (p - (j == 0 ? 1.f : 0.f));
    float* out = gI + ((j == 0 ? b : (int64_t)j * B + b)) * D;
#pragma unroll
    for (int v = 0; v < V; ++v) out[v * 64 + lane] = c * s[v];
  }
}

}  // namespace mirec

using namespace mirec;

static int seq_embed_ln_fwd_impl(const float* item_table, int64_t n_items,
                                 const float* pos_table, const int64_t* item_seq, int64_t B,
                                 int32_t L, int32_t d, const float* gamma, const float* beta,
                                 float eps, float* out, float* mean, float* rstd,
                                 const LnDrop* dr, void* stream, const char* what) {
  const int64_t n = B * L;
  if (n == 0) return 0;
  if (!item_table || !pos_table || !item_seq || !gamma || !beta || !out || !mean || !rstd ||
      B < 0 || L <= 0 || n_items <= 0) {
    set_error("%s: bad arguments", what);
    return -1;
  }
  hipStream_t st = (hipStream_t)stream;
  LnDrop none;
  memset(&none, 0, sizeof(none));
#define MIREC_LNF(DD)                                                                        \
  case DD: {                                                                                 \
    constexpr int GPW = 64 / (DD / 4);                                                       \
    const int64_t waves = (n + GPW - 1) / GPW;                                               \
    const dim3 grd((unsigned)((waves + 3) / 4));                                             \
    if (dr)                                                                                  \
      hipLaunchKernelGGL((seq_embed_ln_fwd_kernel<DD, true>), grd, dim3(256), 0, st,         \
                         item_table, n_items, pos_table, item_seq, n, L, gamma, beta, eps,   \
                         out, mean, rstd, *dr);                                              \
    else                                                                                     \
      hipLaunchKernelGGL((seq_embed_ln_fwd_kernel<DD, false>), grd, dim3(256), 0, st,        \
                         item_table, n_items, pos_table, item_seq, n, L, gamma, beta, eps,   \
                         out, mean, rstd, none);                                             \
  } break;
  switch (d) {
    MIREC_LNF(32)
    MIREC_LNF(64)
    MIREC_LNF(128)
    MIREC_LNF(256)
    default:
      set_error("%s: hidden size %d not in {32,64,128,256}", what, d);
      return -1;
  }
#undef MIREC_LNF
  return launch_status(what);
}

extern "C" int64_t mirec_seq_embed_ln_partials(int64_t n_rows) {
  return (n_rows + kLnRowsPerBlock - 1) / kLnRowsPerBlock;
}

static int seq_embed_ln_bwd_impl(const float* item_table, int64_t n_items,
                                 const float* pos_table, const int64_t* item_seq, int64_t B,
                                 int32_t L, int32_t d, const float* gamma, const float* mean,
                                 const float* rstd, const float* grad_out, float* dx,
                                 float* ditem, float* part_gamma, float* part_beta,
                                 const LnDrop* dr, void* stream, const char* what) {
  const int64_t n = B * L;
  if (n == 0) return 0;
  if (!item_table || !pos_table || !item_seq || !gamma || !mean || !rstd || !grad_out ||
      !part_gamma || !part_beta || B < 0 || L <= 0 || n_items <= 0) {
    set_error("%s: bad arguments", what);
    return -1;
  }
  hipStream_t st = (hipStream_t)stream;
  const dim3 grd((unsigned)mirec_seq_embed_ln_partials(n));
  LnDrop none;
  memset(&none, 0, sizeof(none));
#define MIREC_LNB(DD)                                                                        \
  case DD:                                                                                   \
    if (dr)                                                                                  \
      hipLaunchKernelGGL((seq_embed_ln_bwd_kernel<DD, true>), grd, dim3(256), 0, st,         \
                         item_table, n_items, pos_table, item_seq, n, L, gamma, mean, rstd,  \
                         grad_out, dx, ditem, part_gamma, part_beta, *dr);                   \
    else                                                                                     \
      hipLaunchKernelGGL((seq_embed_ln_bwd_kernel<DD, false>), grd, dim3(256), 0, st,        \
                         item_table, n_items, pos_table, item_seq, n, L, gamma, mean, rstd,  \
                         grad_out, dx, ditem, part_gamma, part_beta, none);                  \
    break;
  switch (d) {
    MIREC_LNB(32)
    MIREC_LNB(64)
    MIREC_LNB(128)
    MIREC_LNB(256)
    default:
      set_error("%s: hidden size %d not in {32,64,128,256}", what, d);
      return -1;
  }
#undef MIREC_LNB
  return launch_status(what);
}

static int add_ln_fwd_impl(const float* a, const float* b, int64_t n, int32_t d,
                           const float* gamma, const float* beta, float eps, float* out,
                           float* mean, float* rstd, const LnDrop* dr, void* stream,
                           const char* what) {
  if (n == 0) return 0;
  if (!a || !b || !gamma || !beta || !out || !mean || !rstd || n < 0) {
    set_error("%s: bad arguments", what);
    return -1;
  }
  hipStream_t st = (hipStream_t)stream;
  LnDrop none;
  memset(&none, 0, sizeof(none));
#define MIREC_ALF(DD)                                                                        \
  case DD: {                                                                                 \
    constexpr int GPW = 64 / (DD / 4);                                                       \
    const int64_t waves = (n + GPW - 1) / GPW;                                               \
    const dim3 grd((unsigned)((waves + 3) / 4));                                             \
    if (dr)                                                                                  \
      hipLaunchKernelGGL((add_ln_fwd_kernel<DD, true>), grd, dim3(256), 0, st, a, b, n,      \
                         gamma, beta, eps, out, mean, rstd, *dr);                            \
    else                                                                                     \
      hipLaunchKernelGGL((add_ln_fwd_kernel<DD, false>), grd, dim3(256), 0, st, a, b, n,     \
                         gamma, beta, eps, out, mean, rstd, none);                           \
  } break;
  switch (d) {
    MIREC_ALF(32)
    MIREC_ALF(64)
    MIREC_ALF(128)
    MIREC_ALF(256)
    default:
      set_error("%s: hidden size %d not in {32,64,128,256}", what, d);
      return -1;
  }
#undef MIREC_ALF
  return launch_status(what);
}

static int add_ln_bwd_impl(const float* a, const float* b, int64_t n, int32_t d,
                           const float* gamma, const float* mean, const float* rstd,
                           const float* grad_out, float* dxb, float* dxa, float* part_gamma,
                           float* part_beta, const LnDrop* dr, void* stream, const char* what) {
  if (n == 0) return 0;
  if (!a || !b || !gamma || !mean || !rstd || !grad_out || !dxb || !part_gamma || !part_beta ||
      n < 0 || (dr && !dxa)) {
    set_error("%s: bad arguments", what);
    return -1;
  }
  hipStream_t st = (hipStream_t)stream;
  const dim3 grd((unsigned)mirec_seq_embed_ln_partials(n));
  LnDrop none;
  memset(&none, 0, sizeof(none));
#define MIREC_ALB(DD)                                                                        \
  case DD:                                                                                   \
    if (dr)                                                                                  \
      hipLaunchKernelGGL((add_ln_bwd_kernel<DD, true>), grd, dim3(256), 0, st, a, b, n,      \
                         gamma, mean, rstd, grad_out, dxb, dxa, part_gamma, part_beta, *dr); \
    else                                                                                     \
      hipLaunchKernelGGL((add_ln_bwd_kernel<DD, false>), grd, dim3(256), 0, st, a, b, n,     \
                         gamma, mean, rstd, grad_out, dxb, nullptr, part_gamma, part_beta,   \
                         none);                                                              \
    break;
  switch (d) {
    MIREC_ALB(32)
    MIREC_ALB(64)
    MIREC_ALB(128)
    MIREC_ALB(256)
    default:
      set_error("%s: hidden size %d not in {32,64,128,256}", what, d);
      return -1;
  }
#undef MIREC_ALB
  return launch_status(what);
}

static int ln_drop_args(float p, uint64_t seed, int64_t* counter, int64_t* drawn, LnDrop* dr,
                        const char* what) {
  if (!(p > 0.f && p < 1.f) || !drawn || !counter) {
    set_error("%s: dropout %g needs 0 < p < 1, the counter and the drawn word", what, (double)p);
    return -1;
  }
  dr->thr = (uint32_t)fmin(4294967295.0, ldexp(1.0 - (double)p, 32));
  dr->scale = 1.0f / (1.0f - p);
  dr->seed = seed;
  dr->counter = counter;
  dr->drawn = drawn;
  return 0;
}

extern "C" int mirec_add_ln_fwd_f32(const float* a, const float* b, int64_t n, int32_t d,
                                    const float* gamma, const float* beta, float eps, float* out,
                                    float* mean, float* rstd, void* stream) {
  return add_ln_fwd_impl(a, b, n, d, gamma, beta, eps, out, mean, rstd, nullptr, stream,
                         "mirec_add_ln_fwd_f32");
}

extern "C" int mirec_add_ln_bwd_f32(const float* a, const float* b, int64_t n, int32_t d,
                                    const float* gamma, const float* mean, const float* rstd,
                                    const float* grad_out, float* dx, float* part_gamma,
                                    float* part_beta, void* stream) {
  return add_ln_bwd_impl(a, b, n, d, gamma, mean, rstd, grad_out, dx, nullptr, part_gamma,
                         part_beta, nullptr, stream, "mirec_add_ln_bwd_f32");
}

extern "C" int mirec_seq_embed_ln_fwd_f32(const float* item_table, int64_t n_items,
                                          const float* pos_table, const int64_t* item_seq,
                                          int64_t B, int32_t L, int32_t d, const float* gamma,
                                          const float* beta, float eps, float* out, float* mean,
                                          float* rstd, void* stream) {
  return seq_embed_ln_fwd_impl(item_table, n_items, pos_table, item_seq, B, L, d, gamma, beta,
                               eps, out, mean, rstd, nullptr, stream,
                               "mirec_seq_embed_ln_fwd_f32");
}

extern "C" int mirec_seq_embed_ln_bwd_f32(const float* item_table, int64_t n_items,
                                          const float* pos_table, const int64_t* item_seq,
                                          int64_t B, int32_t L, int32_t d, const float* gamma,
                                          const float* mean, const float* rstd,
                                          const float* grad_out, float* dx, float* ditem,
                                          float* part_gamma, float* part_beta, void* stream) {
  return seq_embed_ln_bwd_impl(item_table, n_items, pos_table, item_seq, B, L, d, gamma, mean,
                               rstd, grad_out, dx, ditem, part_gamma, part_beta, nullptr, stream,
                               "mirec_seq_embed_ln_bwd_f32");
}

extern "C" int mirec_seq_embed_ln_drop_fwd_f32(const float* item_table, int64_t n_items,
                                               const float* pos_table, const int64_t* item_seq,
                                               int64_t B, int32_t L, int32_t d,
                                               const float* gamma, const float* beta, float eps,
                                               float p, uint64_t seed, int64_t* counter,
                                               int64_t* drawn, float* out, float* mean,
                                               float* rstd, void* stream) {
  LnDrop dr;
  if (ln_drop_args(p, seed, counter, drawn, &dr, "mirec_seq_embed_ln_drop_fwd_f32")) return -1;
  return seq_embed_ln_fwd_impl(item_table, n_items, pos_table, item_seq, B, L, d, gamma, beta,
                               eps, out, mean, rstd, &dr, stream,
                               "mirec_seq_embed_ln_drop_fwd_f32");
}

extern "C" int mirec_seq_embed_ln_drop_bwd_f32(const float* item_table, int64_t n_items,
                                               const float* pos_table, const int64_t* item_seq,
                                               int64_t B, int32_t L, int32_t d,
                                               const float* gamma, const float* mean,
                                               const float* rstd, const float* grad_out,
                                               float p, uint64_t seed, int64_t* drawn,
                                               int64_t* counter, float* dx, float* ditem,
                                               float* part_gamma, float* part_beta,
                                               void* stream) {
  LnDrop dr;
  if (ln_drop_args(p, seed, counter, drawn, &dr, "mirec_seq_embed_ln_drop_bwd_f32")) return -1;
  return seq_embed_ln_bwd_impl(item_table, n_items, pos_table, item_seq, B, L, d, gamma, mean,
                               rstd, grad_out, dx, ditem, part_gamma, part_beta, &dr, stream,
                               "mirec_seq_embed_ln_drop_bwd_f32");
}

extern "C" int mirec_add_ln_drop_fwd_f32(const float* a, const float* b, int64_t n, int32_t d,
                                         const float* gamma, const float* beta, float eps,
                                         float p, uint64_t seed, int64_t* counter,
                                         int64_t* drawn, float* out, float* mean, float* rstd,
                                         void* stream) {
  LnDrop dr;
  if (ln_drop_args(p, seed, counter, drawn, &dr, "mirec_add_ln_drop_fwd_f32")) return -1;
  return add_ln_fwd_impl(a, b, n, d, gamma, beta, eps, out, mean, rstd, &dr, stream,
                         "mirec_add_ln_drop_fwd_f32");
}

extern "C" int mirec_add_ln_drop_bwd_f32(const float* a, const float* b, int64_t n, int32_t d,
                                         const float* gamma, const float* mean,
                                         const float* rstd, const float* grad_out, float p,
                                         uint64_t seed, int64_t* drawn, int64_t* counter,
                                         float* dx_a, float* dx_b, float* part_gamma,
                                         float* part_beta, void* stream) {
  LnDrop dr;
  if (ln_drop_args(p, seed, counter, drawn, &dr, "mirec_add_ln_drop_bwd_f32")) return -1;
  return add_ln_bwd_impl(a, b, n, d, gamma, mean, rstd, grad_out, dx_b, dx_a, part_gamma,
                         part_beta, &dr, stream, "mirec_add_ln_drop_bwd_f32");
}

// SASRec.get_attention_mask (reference sasrec.py:91-105) in one launch: mask[b][i][j] =
// (1 - [item_seq[b][j] > 0] * [j <= i]) * -10000 as the reference's float ops round it —
// -0.0 where attention is allowed ((1 - 1) * -10000), -10000 elsewhere.
__global__ __launch_bounds__(256) void seq_attn_mask_kernel(const int64_t* __restrict__ seq,
                                                            int64_t B, int L,
                                                            float* __restrict__ mask) {
  const int64_t n = B * (int64_t)L * L;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e / ((int64_t)L * L);
    const int i = (int)((e / L) % L), j = (int)(e % L);
    const float keep = (seq[b * L + j] > 0 && j <= i) ? 1.0f : 0.0f;
    mask[e] = (1.0f - keep) * -10000.0f;
  }
}

static unsigned elem_grid(int64_t n) {
  const int64_t g = (n + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > 256 * 32 ? 256 * 32 : g));
}

extern "C" int mirec_seq_attn_mask_f32(const int64_t* item_seq, int64_t B, int32_t L,
                                       float* mask, void* stream) {
  if (B == 0 || L == 0) return 0;
  if (!item_seq || !mask || B < 0 || L < 0) {
    set_error("mirec_seq_attn_mask_f32: bad arguments");
    return -1;
  }
  hipLaunchKernelGGL(seq_attn_mask_kernel, dim3(elem_grid(B * (int64_t)L * L)), dim3(256), 0,
                     (hipStream_t)stream, item_seq, B, L, mask);
  return launch_status("mirec_seq_attn_mask_f32");
}

extern "C" int mirec_gelu_fwd_f32(const float* x, int64_t n, float* y, void* stream) {
  if (n == 0) return 0;
  if (!x || !y || n < 0) {
    set_error("mirec_gelu_fwd_f32: bad arguments");
    return -1;
  }
  if (n % 4 == 0 && ((uintptr_t)x | (uintptr_t)y) % 16 == 0)
    hipLaunchKernelGGL(gelu_fwd4_kernel, dim3(elem_grid(n / 4)), dim3(256), 0,
                       (hipStream_t)stream, reinterpret_cast<const float4*>(x), n / 4,
                       reinterpret_cast<float4*>(y));
  else
    hipLaunchKernelGGL(gelu_fwd_kernel, dim3(elem_grid(n)), dim3(256), 0, (hipStream_t)stream,
                       x, n, y);
  return launch_status("mirec_gelu_fwd_f32");
}

extern "C" int mirec_gelu_bwd_f32(const float* x, const float* g, int64_t n, float* dx,
                                  void* stream) {
  if (n == 0) return 0;
  if (!x || !g || !dx || n < 0) {
    set_error("mirec_gelu_bwd_f32: bad arguments");
    return -1;
  }
  if (n % 4 == 0 && ((uintptr_t)x | (uintptr_t)g | (uintptr_t)dx) % 16 == 0)
    hipLaunchKernelGGL(gelu_bwd4_kernel, dim3(elem_grid(n / 4)), dim3(256), 0,
                       (hipStream_t)stream, reinterpret_cast<const float4*>(x),
                       reinterpret_cast<const float4*>(g), n / 4, reinterpret_cast<float4*>(dx));
  else
    hipLaunchKernelGGL(gelu_bwd_kernel, dim3(elem_grid(n)), dim3(256), 0, (hipStream_t)stream,
                       x, g, n, dx);
  return launch_status("mirec_gelu_bwd_f32");
}

extern "C" int mirec_scale_by_f32(float* x, int64_t n, const float* g, void* stream) {
  if (n == 0) return 0;
  if (!x || !g || n < 0 || n % 4 || ((uintptr_t)x & 15)) {
    set_error("mirec_scale_by_f32: bad arguments (n %% 4 == 0, 16-byte aligned x)");
    return -1;
  }
  const int64_t n4 = n / 4;
  const unsigned grid = (unsigned)std::min<int64_t>((n4 + 255) / 256, 2048);
  hipLaunchKernelGGL(scale_by_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<float4*>(x), n4, g);
  return launch_status("mirec_scale_by_f32");
}

extern "C" int mirec_sampled_softmax_f32(const float* seq_out, const float* item_table,
                                         int64_t n_items, int32_t d, const int64_t* pos,
                                         const int64_t* neg, int64_t B, int32_t n_neg,
                                         float grad_scale, float* loss, float* g_seq,
                                         float* g_items, void* stream) {
  if (B == 0) return 0;
  if (!seq_out || !item_table || !pos || (n_neg > 0 && !neg) || !loss || !g_seq || !g_items ||
      B < 0 || n_neg < 0 || n_items <= 0) {
    set_error("mirec_sampled_softmax_f32: bad arguments");
    return -1;
  }
  const dim3 grd((unsigned)((B + 3) / 4));
  const size_t lds = (size_t)4 * (n_neg + 1) * sizeof(float);
  if (lds > 64 * 1024) {
    set_error("mirec_sampled_softmax_f32: %d negatives exceed the LDS logit buffer", n_neg);
    return -1;
  }
  hipStream_t st = (hipStream_t)stream;
  switch (d) {
    case 64:
      hipLaunchKernelGGL(sampled_softmax_kernel<64>, grd, dim3(256), lds, st, seq_out,
                         item_table, n_items, pos, neg, B, n_neg, grad_scale, loss, g_seq, g_items);
      break;
    case 128:
      hipLaunchKernelGGL(sampled_softmax_kernel<128>, grd, dim3(256), lds, st, seq_out,
                         item_table, n_items, pos, neg, B, n_neg, grad_scale, loss, g_seq, g_items);
      break;
    case 256:
      hipLaunchKernelGGL(sampled_softmax_kernel<256>, grd, dim3(256), lds, st, seq_out,
                         item_table, n_items, pos, neg, B, n_neg, grad_scale, loss, g_seq, g_items);
      break;
    default:
      set_error("mirec_sampled_softmax_f32: hidden size %d not in {64,128,256}", d);
      return -1;
  }
  return launch_status("mirec_sampled_softmax_f32");
}

// K9c — sampled evaluation of a sequential model (uni-N, the fork's validation):
// rank of the positive among [pos | N sampled items] per query, i.e. the number
// of sampled items whose score is greater or equal (a sampled copy of the positive
// item ties it exactly; torch.topk leaves the order of ties unspecified, this
// counts them ahead of the positive — the pessimistic order). Replaces
// the repeat x (1+N) of every sequence through the whole model (predict on each
// copy) + sample_collect + topk of Trainer.evaluate for these loaders.
namespace mirec {

template <int D>
__global__ __launch_bounds__(256) void rank_of_pos_kernel(
    const float* __restrict__ S, const float* __restrict__ E, int64_t n_items,
    const int64_t* __restrict__ pos, const int64_t* __restrict__ neg, int64_t n, int m,
    int32_t* __restrict__ rank) {
  constexpr int LPR = D / 4, GPW = 64 / LPR, NB = 4;
  const int lane = threadIdx.x & 63;
  const int g = lane / LPR, l = lane % LPR;
  const int64_t q = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * GPW + g;
  if (q >= n) return;
  const float4 s = reinterpret_cast<const float4*>(S + q * D)[l];
  auto row = [&](int64_t id) {
    id = id < 0 ? 0 : (id >= n_items ? n_items - 1 : id);
    return reinterpret_cast<const float4*>(E + id * D)[l];
  };
  auto dot = [&](const float4& e) {   // explicit fma chain: every call site rounds alike
    float x = fmaf(s.w, e.w, fmaf(s.z, e.z, fmaf(s.y, e.y, s.x * e.x)));
#pragma unroll
    for (int off = LPR / 2; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
  };
  const float sp = dot(row(pos[q]));
  const int64_t* nq = neg + q * (int64_t)m;
  int cnt = 0;
  for (int j0 = 0; j0 < m; j0 += NB) {
    float4 e[NB];
#pragma unroll
    for (int t = 0; t < NB; ++t)
      e[t] = j0 + t < m ? row(nq[j0 + t]) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      const float sc = dot(e[t]);
      cnt += (j0 + t < m && sc >= sp) ? 1 : 0;
    }
  }
  if (l == 0) rank[q] = cnt;
}

}  // namespace mirec

extern "C" int mirec_rank_of_pos_f32(const float* seq_out, const float* item_table,
                                     int64_t n_items, int32_t d, const int64_t* pos,
                                     const int64_t* neg, int64_t n, int32_t m, int32_t* rank,
                                     void* stream) {
  if (n == 0) return 0;
  if (!seq_out || !item_table || !pos || (m > 0 && !neg) || !rank || n < 0 || m < 0 ||
      n_items <= 0) {
    set_error("mirec_rank_of_pos_f32: bad arguments");
    return -1;
  }
  hipStream_t st = (hipStream_t)stream;
#define MIREC_ROP(DD)                                                                         \
  case DD:                                                                                    \
    hipLaunchKernelGGL(rank_of_pos_kernel<DD>,                                                \
                       dim3((unsigned)((n + 4 * (256 / DD) - 1) / (4 * (256 / DD)))),          \
                       dim3(256), 0, st, seq_out, item_table, n_items, pos, neg, n, m, rank);  \
    break;
  switch (d) {
    MIREC_ROP(32)
    MIREC_ROP(64)
    MIREC_ROP(128)
    MIREC_ROP(256)
    default:
      set_error("mirec_rank_of_pos_f32: hidden size %d not in {32,64,128,256}", d);
      return -1;
  }
#undef MIREC_ROP
  return launch_status("mirec_rank_of_pos_f32");
}
