// K5 — dense Adam over every row of an embedding table in ONE streaming pass,
// with the gradient supplied in grouped (compact) form.
//
// Restates optim.Adam.step as the reference runs it (trainer.py:109-130, 173;
// torch optim/adam.py _single_tensor_adam, CPU, foreach=False) on
// nn.Embedding(sparse=False) weights: every row moves every step (rows with a
// zero gradient still decay m and v and move p).  The dense gradient buffer
// and its zero-fill are never materialised: the kernel reads p, m, v once and
// writes them once (6 * n_rows * d * 4 bytes per step — the HBM roofline of
// the whole training step at C2), and for the few rows present in `uniq` it
// sums their contributions (grouped by K2) in a fixed order on the fly.
//
// Per element, in torch's order:
//   g  = g + wd * p                       (grad.add(param, alpha=wd))
//   m  = m + (1-b1) * (g - m)             (exp_avg.lerp_(grad, 1-b1), weight < .5)
//   v  = v * b2 + ((1-b2) * g) * g        (mul_(b2).addcmul_(g, g, value=1-b2))
//   p  = p + (-step_size) * (m / (sqrt(v) / bc2_sqrt + eps))   (addcdiv_)
// step_size = lr / (1 - b1^t) and bc2_sqrt = sqrt(1 - b2^t) come from a host
// table computed in double, indexed by the device step counter.
#include "common.h"

namespace mirec {

constexpr int kAdamThreads = 256;
constexpr int kAdamRows = 64;  // table rows per block
constexpr int kMaxTables = 4;

struct AdamConsts {
  float omb1, b2, omb2, eps, wd;
};

// Up to kMaxTables tables in one launch; blocks [block_start[t], block_start[t+1])
// belong to table t (one grid over e.g. the user AND item tables, so the
// smaller table does not run as its own under-filled launch).
struct AdamTables {
  mirec_adam_table t[kMaxTables];
  int64_t block_start[kMaxTables + 1];
  int n;
};

template <int D>
__global__ __launch_bounds__(kAdamThreads) void adam_multi_kernel(
    const AdamTables tabs, const float* __restrict__ step_consts,
    const int32_t* __restrict__ step_idx, AdamConsts k) {
  constexpr int VPR = D / 4;                        // float4 per row
  constexpr int RPP = kAdamThreads / VPR;           // rows per pass
  static_assert(kAdamThreads % VPR == 0, "row width");
  __shared__ int32_t slot[kAdamRows];
  __shared__ int32_t s_range[2];

  int ti = 0;
#pragma unroll
  for (int q = 1; q < kMaxTables; ++q)
    if (q < tabs.n && (int64_t)blockIdx.x >= tabs.block_start[q]) ti = q;
  const mirec_adam_table& T = tabs.t[ti];
  float* __restrict__ P = T.p;
  float* __restrict__ M = T.m;
  float* __restrict__ V = T.v;
  const int32_t* __restrict__ uniq = T.uniq;
  const int32_t* __restrict__ seg = T.seg;
  const int32_t* __restrict__ perm = T.perm;
  const float* __restrict__ dense_grad = T.dense_grad;

  const int64_t lo = ((int64_t)blockIdx.x - tabs.block_start[ti]) * kAdamRows;
  const int64_t hi = min(T.n_rows, lo + kAdamRows);
  if (threadIdx.x < kAdamRows) slot[threadIdx.x] = -1;
  if (threadIdx.x == 0) {
    const int nu = T.n_uniq ? T.n_uniq[0] : 0;
    // lower_bound(uniq, lo), lower_bound(uniq, hi)
    int a = 0, b = nu;
    while (a < b) { int mid = (a + b) >> 1; if (uniq[mid] < lo) a = mid + 1; else b = mid; }
    int c = a, e = nu;
    while (c < e) { int mid = (c + e) >> 1; if (uniq[mid] < hi) c = mid + 1; else e = mid; }
    s_range[0] = a;
    s_range[1] = c;
  }
  __syncthreads();
  for (int u = s_range[0] + threadIdx.x; u < s_range[1]; u += kAdamThreads)
    slot[uniq[u] - lo] = u;
  __syncthreads();

  const int st = step_idx[0];
  const float step_size = step_consts[2 * st];
  const float bc2s = step_consts[2 * st + 1];
  const float4* __restrict__ R4 = reinterpret_cast<const float4*>(T.rows);

  const int rsub = threadIdx.x / VPR;
  const int c = threadIdx.x % VPR;
#pragma unroll 2
  for (int64_t r = lo + rsub; r < hi; r += RPP) {
    const int64_t off = r * VPR + c;
    float4 p = reinterpret_cast<const float4*>(P)[off];
    float4 m = reinterpret_cast<const float4*>(M)[off];
    float4 v = reinterpret_cast<const float4*>(V)[off];
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    if (dense_grad) g = reinterpret_cast<const float4*>(dense_grad)[off];
    const int s = slot[r - lo];
    if (s >= 0) {
      const int i1 = seg[s + 1];
      for (int i = seg[s]; i < i1; ++i) {
        const float4 x = R4[(int64_t)perm[i] * VPR + c];
        g.x += x.x; g.y += x.y; g.z += x.z; g.w += x.w;
      }
    }
    float* pp = &p.x; float* mm = &m.x; float* vv = &v.x; float* gg = &g.x;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float ge = gg[e];
      if (k.wd != 0.f) ge = ge + k.wd * pp[e];
      const float me = mm[e] + k.omb1 * (ge - mm[e]);
      const float ve = vv[e] * k.b2 + (k.omb2 * ge) * ge;
      const float den = sqrtf(ve) / bc2s + k.eps;
      pp[e] = pp[e] + (-step_size) * (me / den);
      mm[e] = me;
      vv[e] = ve;
    }
    reinterpret_cast<float4*>(P)[off] = p;
    reinterpret_cast<float4*>(M)[off] = m;
    reinterpret_cast<float4*>(V)[off] = v;
  }
}

}  // namespace mirec

using namespace mirec;

extern "C" int mirec_adam_multi_f32(const mirec_adam_table* tables, int32_t n_tables, int32_t d,
                                    const float* step_consts_dev, const int32_t* step_idx_dev,
                                    double beta1, double beta2, double eps, double weight_decay,
                                    void* stream) {
  if (n_tables < 1 || n_tables > kMaxTables || !tables || !step_consts_dev || !step_idx_dev) {
    set_error("mirec_adam_multi_f32: bad arguments (n_tables=%d)", n_tables);
    return -1;
  }
  AdamTables tabs;
  memset(&tabs, 0, sizeof(tabs));
  tabs.n = n_tables;
  int64_t blocks = 0;
  for (int q = 0; q < n_tables; ++q) {
    const mirec_adam_table& t = tables[q];
    if (!t.p || !t.m || !t.v || t.n_rows < 0 ||
        (t.n_uniq && (!t.uniq || !t.seg || !t.perm || !t.rows))) {
      set_error("mirec_adam_multi_f32: bad table %d", q);
      return -1;
    }
    tabs.t[q] = t;
    tabs.block_start[q] = blocks;
    blocks += (t.n_rows + kAdamRows - 1) / kAdamRows;
  }
  tabs.block_start[n_tables] = blocks;
  for (int q = n_tables + 1; q <= kMaxTables; ++q) tabs.block_start[q] = blocks;
  if (blocks == 0) return 0;
  AdamConsts k;
  k.omb1 = (float)(1.0 - beta1);
  k.b2 = (float)beta2;
  k.omb2 = (float)(1.0 - beta2);
  k.eps = (float)eps;
  k.wd = (float)weight_decay;
  const dim3 grd((unsigned)blocks);
  hipStream_t st = (hipStream_t)stream;
#define MIREC_ADAM_CASE(DD)                                                                  \
  case DD:                                                                                   \
    hipLaunchKernelGGL(adam_multi_kernel<DD>, grd, dim3(kAdamThreads), 0, st, tabs,          \
                       step_consts_dev, step_idx_dev, k);                                    \
    break;
  switch (d) {
    MIREC_ADAM_CASE(4)
    MIREC_ADAM_CASE(16)
    MIREC_ADAM_CASE(32)
    MIREC_ADAM_CASE(64)
    MIREC_ADAM_CASE(128)
    MIREC_ADAM_CASE(256)
    default:
      set_error("mirec_adam_multi_f32: row width %d not in {4,16,32,64,128,256}", d);
      return -1;
  }
#undef MIREC_ADAM_CASE
  return launch_status("mirec_adam_multi_f32");
}

extern "C" int mirec_adam_sparse_grad_f32(float* p, float* m, float* v, int64_t n_rows,
                                          int32_t d, const float* rows, const int32_t* perm,
                                          const int32_t* uniq, const int32_t* seg,
                                          const int32_t* n_uniq_dev, int64_t n_max_uniq,
                                          const float* dense_grad, const float* step_consts_dev,
                                          const int32_t* step_idx_dev, double beta1,
                                          double beta2, double eps, double weight_decay,
                                          void* stream) {
  (void)n_max_uniq;
  if (n_rows == 0) return 0;
  mirec_adam_table t;
  t.p = p; t.m = m; t.v = v; t.n_rows = n_rows;
  t.rows = rows; t.perm = perm; t.uniq = uniq; t.seg = seg; t.n_uniq = n_uniq_dev;
  t.dense_grad = dense_grad;
  return mirec_adam_multi_f32(&t, 1, d, step_consts_dev, step_idx_dev, beta1, beta2, eps,
                              weight_decay, stream);
}
