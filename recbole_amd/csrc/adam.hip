// K5 — dense Adam over every row of the embedding tables, with the gradient
// supplied in grouped (compact) form. Two schedules, bit-identical results:
//
//  * streamed (adam_multi_kernel): one pass over p, m, v of EVERY row each step
//    (6 * n_rows * d * 4 bytes per step, the HBM roofline of the step);
//  * deferred (adam_deferred_kernel + adam_flush_kernel): a row whose gradient is
//    zero at step s is advanced by exactly the same per-element operations as
//    the streamed kernel would apply — but only when the row is next touched,
//    or at a flush. `last[row]` counts the steps already applied to the row. A
//    touch at step s replays steps last..s-1 with g = 0 and then applies step s;
//    a flush replays every row up to the global step count. Same FLOPs, same
//    bits, but each step only moves the rows it touches.
//
// Restates optim.Adam.step as the reference runs it (trainer.py:109-130, 173;
// torch optim/adam.py _single_tensor_adam, CPU, foreach=False) on
// nn.Embedding(sparse=False) weights: every row moves every step (rows with a
// zero gradient still decay m and v and move p). Per element, torch's order and
// rounding (fma where ATen's vectorised CPU kernels fuse):
//   g  = fma(p, wd, g)                    (grad.add(param, alpha=wd))
//   m  = fma(1-b1, g - m, m)              (exp_avg.lerp_(grad, 1-b1), weight < .5)
//   v  = fma((1-b2) * g, g, v * b2)       (mul_(b2).addcmul_(g, g, value=1-b2))
//   p  = p + ((-step_size) * m) / (sqrt(v) / bc2_sqrt + eps)   (addcdiv_)
// Every other op is one IEEE-rounded fp32 operation (sqrt and / correctly
// rounded). This reproduces torch CPU's m, v and p bit-for-bit given the same
// sqrt; torch CPU takes sqrt from the vendor vector math library (not always
// correctly rounded), so p agrees to an ulp there, exactly elsewhere.
//
// Host table (float32, 4 per 0-based step index s), computed in double like
// torch: {step_size = lr/(1-b1^t), bc2_sqrt = sqrt(1-b2^t), rbc = RN(1/bc2_sqrt), 0}.
// x / bc2_sqrt is evaluated as q = x*rbc; q + fma(-q, bc2_sqrt, x)*rbc (fma):
// with rbc the correctly rounded reciprocal this is the correctly rounded
// quotient (Markstein's theorem; checked exhaustively over two binades of x for
// ~13k divisors of several beta2), i.e. bit-identical to IEEE division in 3
// instead of ~11 instructions. x = +inf takes the IEEE division.
#include "common.h"

// No FMA contraction: every op rounds on its own, as in torch's op-by-op
// _single_tensor_adam, and the streamed / deferred schedules stay bit-identical
// whatever the compiler could fuse in either context.
#pragma clang fp contract(off)

namespace mirec {

constexpr int kAdamThreads = 256;
constexpr int kAdamRows = 64;  // table rows per block (streamed / flush)
constexpr int kMaxTables = 4;

struct AdamConsts {
  float omb1, omb1m1, b2, omb2, eps, wd;
  int lerp_small;  // 1 - beta1 < 0.5: lerp from m (torch's is_lerp_weight_small)
};

struct StepConsts {
  float ss, bc2s, rbc;
};

__device__ __forceinline__ StepConsts step_consts(const float* __restrict__ consts, int s) {
  const float4 c = reinterpret_cast<const float4*>(consts)[s];
  return {c.x, c.y, c.z};
}

// Launch = a list of segments, each a contiguous block range over one table.
// Streamed / flush: segment q = table q. Deferred: segment 2q = table q's
// touched rows, 2q+1 = its look-ahead rows.
struct AdamTables {
  mirec_adam_table t[kMaxTables];
  int64_t block_start[2 * kMaxTables + 1];
  int n_seg;
};

// One Adam step of one element. Shared by every schedule so the arithmetic is
// the same instruction sequence wherever a step is applied.
__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g,
                                          const StepConsts& sc, const AdamConsts& k) {
  if (k.wd != 0.f) g = fmaf(p, k.wd, g);
  const float dlt = g - m;
  const float me = k.lerp_small ? fmaf(k.omb1, dlt, m) : fmaf(k.omb1m1, dlt, g);
  const float ve = fmaf(k.omb2 * g, g, v * k.b2);
  const float x = sqrtf(ve);
  float q = x * sc.rbc;                       // x / bc2s, correctly rounded
  q = fmaf(fmaf(-q, sc.bc2s, x), sc.rbc, q);
  if (__builtin_expect(x == __builtin_inff(), 0)) q = x / sc.bc2s;
  const float den = q + k.eps;
  p = p + ((-sc.ss) * me) / den;
  m = me;
  v = ve;
}

__device__ __forceinline__ void adam_vec(float4& p, float4& m, float4& v, const float4& g,
                                         const StepConsts& sc, const AdamConsts& k) {
  adam_elem(p.x, m.x, v.x, g.x, sc, k);
  adam_elem(p.y, m.y, v.y, g.y, sc, k);
  adam_elem(p.z, m.z, v.z, g.z, sc, k);
  adam_elem(p.w, m.w, v.w, g.w, sc, k);
}

// Replay steps [s0, s1) with a zero gradient (the exact per-step sequence).
__device__ __forceinline__ void adam_replay(float4& p, float4& m, float4& v, int s0, int s1,
                                            const float* __restrict__ consts,
                                            const AdamConsts& k) {
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int s = s0; s < s1; ++s) adam_vec(p, m, v, z, step_consts(consts, s), k);
}

__device__ __forceinline__ void adam_replay1(float& p, float& m, float& v, int s0, int s1,
                                             const float* __restrict__ consts,
                                             const AdamConsts& k) {
  for (int s = s0; s < s1; ++s) adam_elem(p, m, v, 0.f, step_consts(consts, s), k);
}

__device__ __forceinline__ int segment_of(const AdamTables& tabs, int64_t b) {
  int si = 0;
#pragma unroll
  for (int q = 1; q < 2 * kMaxTables; ++q)
    if (q < tabs.n_seg && b >= tabs.block_start[q]) si = q;
  return si;
}

// Sum of the grouped contributions of row slot s, in perm order, for the W
// consecutive floats starting at column c (W = 4: float4, W = 1: float).
// Loads are issued 8 at a time (hot rows of a Zipf stream have tens of
// contributions; a dependent chain of loads would serialise them); the
// additions stay in order.
template <typename V>
__device__ __forceinline__ void vadd(V& a, const V& b);
template <>
__device__ __forceinline__ void vadd<float4>(float4& a, const float4& b) {
  a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
}
template <>
__device__ __forceinline__ void vadd<float>(float& a, const float& b) { a += b; }

template <typename V>
__device__ __forceinline__ V grouped_grad(const mirec_adam_table& T, int s, int VPR, int c) {
  V g;
  memset(&g, 0, sizeof(V));
  const V* __restrict__ R = reinterpret_cast<const V*>(T.rows);
  const int32_t* __restrict__ perm = T.perm;
  int i = T.seg[s];
  const int i1 = T.seg[s + 1];
  constexpr int U = 8;
  for (; i + U <= i1; i += U) {
    int32_t pi[U];
#pragma unroll
    for (int j = 0; j < U; ++j) pi[j] = perm[i + j];
    V x[U];
#pragma unroll
    for (int j = 0; j < U; ++j) x[j] = R[(int64_t)pi[j] * VPR + c];
#pragma unroll
    for (int j = 0; j < U; ++j) vadd(g, x[j]);
  }
  for (; i < i1; ++i) vadd(g, R[(int64_t)perm[i] * VPR + c]);
  return g;
}

// ---------------------------------------------------------------- streamed
template <int D>
__global__ __launch_bounds__(kAdamThreads) void adam_multi_kernel(
    const AdamTables tabs, const float* __restrict__ consts, const int32_t* __restrict__ step_base,
    int step_off, AdamConsts k) {
  constexpr int VPR = D / 4;                        // float4 per row
  constexpr int RPP = kAdamThreads / VPR;           // rows per pass
  static_assert(kAdamThreads % VPR == 0, "row width");
  __shared__ int32_t slot[kAdamRows];
  __shared__ int32_t s_range[2];

  const int si = segment_of(tabs, blockIdx.x);
  const mirec_adam_table& T = tabs.t[si];
  float* __restrict__ P = T.p;
  float* __restrict__ M = T.m;
  float* __restrict__ V = T.v;
  const int32_t* __restrict__ uniq = T.uniq;

  const int64_t lo = ((int64_t)blockIdx.x - tabs.block_start[si]) * kAdamRows;
  const int64_t hi = min(T.n_rows, lo + kAdamRows);
  if (threadIdx.x < kAdamRows) slot[threadIdx.x] = -1;
  if (threadIdx.x == 0) {
    const int nu = T.n_uniq ? T.n_uniq[0] : 0;
    int a = 0, b = nu;                       // lower_bound(uniq, lo)
    while (a < b) { int mid = (a + b) >> 1; if (uniq[mid] < lo) a = mid + 1; else b = mid; }
    int c = a, e = nu;                       // lower_bound(uniq, hi)
    while (c < e) { int mid = (c + e) >> 1; if (uniq[mid] < hi) c = mid + 1; else e = mid; }
    s_range[0] = a;
    s_range[1] = c;
  }
  __syncthreads();
  for (int u = s_range[0] + threadIdx.x; u < s_range[1]; u += kAdamThreads)
    slot[uniq[u] - lo] = u;
  __syncthreads();

  const StepConsts sc = step_consts(consts, step_base[0] + step_off);
  const int rsub = threadIdx.x / VPR;
  const int c = threadIdx.x % VPR;
#pragma unroll 2
  for (int64_t r = lo + rsub; r < hi; r += RPP) {
    const int64_t off = r * VPR + c;
    float4 p = reinterpret_cast<const float4*>(P)[off];
    float4 m = reinterpret_cast<const float4*>(M)[off];
    float4 v = reinterpret_cast<const float4*>(V)[off];
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    if (T.dense_grad) g = reinterpret_cast<const float4*>(T.dense_grad)[off];
    const int s = slot[r - lo];
    if (s >= 0) vadd(g, grouped_grad<float4>(T, s, VPR, c));
    adam_vec(p, m, v, g, sc, k);
    reinterpret_cast<float4*>(P)[off] = p;
    reinterpret_cast<float4*>(M)[off] = m;
    reinterpret_cast<float4*>(V)[off] = v;
  }
}

// ---------------------------------------------------------------- deferred
// One thread per (row, column): the replay of a row's skipped steps is a
// serial chain per element, so one element per thread keeps the chain short.
// RPB = 256 / D whole rows per block.
//  segment 2q   (touched): row = uniq[u] of table q. Replays last..s-1 with a
//               zero gradient, applies step s with its gradient; last = s+1.
//  segment 2q+1 (look-ahead): row = ahead_uniq[u], rows the NEXT batch reads
//               and this one does not touch (the caller's set difference).
//               Replays last..s (zero gradient); last = s+1 — so the next
//               forward pass reads rows that are complete through step s.
// `last` is read by every thread of a row before the barrier and written
// after it (a row of D >= 128 spans several waves).
template <int D>
__global__ __launch_bounds__(kAdamThreads) void adam_deferred_kernel(
    const AdamTables tabs, const float* __restrict__ consts,
    const int32_t* __restrict__ step_base, int step_off, AdamConsts k) {
  constexpr int RPB = kAdamThreads / D;             // rows per block
  static_assert(kAdamThreads % D == 0, "row width");
  const int si = segment_of(tabs, blockIdx.x);
  const mirec_adam_table& T = tabs.t[si >> 1];
  const bool ahead = si & 1;
  const int u = (int)(((int64_t)blockIdx.x - tabs.block_start[si]) * RPB) + threadIdx.x / D;
  const int c = threadIdx.x % D;
  const bool valid = u < (ahead ? T.ahead_n_uniq[0] : T.n_uniq[0]);
  const int st = step_base[0] + step_off;
  int64_t row = 0;
  int last = st;
  if (valid) {
    row = ahead ? T.ahead_uniq[u] : T.uniq[u];
    last = T.last[row];
  }
  __syncthreads();
  if (!valid) return;
  const int64_t off = row * D + c;
  float p = T.p[off], m = T.m[off], v = T.v[off];
  adam_replay1(p, m, v, last, st, consts, k);       // the zero-gradient steps it skipped
  const float g = ahead ? 0.f : grouped_grad<float>(T, u, D, c);
  adam_elem(p, m, v, g, step_consts(consts, st), k);
  T.p[off] = p;
  T.m[off] = m;
  T.v[off] = v;
  if (c == 0) T.last[row] = st + 1;
}

// Bring every row up to `n_steps` applied steps (zero-gradient replays).
template <int D>
__global__ __launch_bounds__(kAdamThreads) void adam_flush_kernel(
    const AdamTables tabs, const float* __restrict__ consts, const int32_t* __restrict__ step_base,
    int step_off, AdamConsts k) {
  constexpr int VPR = D / 4;
  constexpr int RPP = kAdamThreads / VPR;
  const int si = segment_of(tabs, blockIdx.x);
  const mirec_adam_table& T = tabs.t[si];
  const int64_t lo = ((int64_t)blockIdx.x - tabs.block_start[si]) * kAdamRows;
  const int64_t hi = min(T.n_rows, lo + kAdamRows);
  const int target = step_base[0] + step_off;
  const int rsub = threadIdx.x / VPR;
  const int c = threadIdx.x % VPR;
  for (int64_t r = lo + rsub; r < hi; r += RPP) {
    const int last = T.last[r];
    if (last >= target) continue;
    const int64_t off = r * VPR + c;
    float4 p = reinterpret_cast<const float4*>(T.p)[off];
    float4 m = reinterpret_cast<const float4*>(T.m)[off];
    float4 v = reinterpret_cast<const float4*>(T.v)[off];
    adam_replay(p, m, v, last, target, consts, k);
    reinterpret_cast<float4*>(T.p)[off] = p;
    reinterpret_cast<float4*>(T.m)[off] = m;
    reinterpret_cast<float4*>(T.v)[off] = v;
    if (c == 0) T.last[r] = target;  // a row lies in one wave here (VPR <= 64)
  }
}

}  // namespace mirec

using namespace mirec;

namespace {

enum class Sched { kStreamed, kDeferred, kFlush };

int launch_adam(Sched sched, const mirec_adam_table* tables, int32_t n_tables,
                const int64_t* n_max_uniq, int32_t d, const float* consts,
                const int32_t* step_base, int32_t step_off, double beta1, double beta2,
                double eps, double weight_decay, void* stream, const char* what) {
  if (n_tables < 1 || n_tables > kMaxTables || !tables || !consts || !step_base) {
    set_error("%s: bad arguments (n_tables=%d)", what, n_tables);
    return -1;
  }
  if (((uintptr_t)consts & 15) != 0) {
    set_error("%s: step constants must be 16-byte aligned", what);
    return -1;
  }
  if (d != 4 && d != 16 && d != 32 && d != 64 && d != 128 && d != 256) {
    set_error("%s: row width %d not in {4,16,32,64,128,256}", what, d);
    return -1;
  }
  const int VPR = d / 4;
  AdamTables tabs;
  memset(&tabs, 0, sizeof(tabs));
  const bool deferred = sched == Sched::kDeferred;
  tabs.n_seg = deferred ? 2 * n_tables : n_tables;
  int64_t blocks = 0;
  for (int q = 0; q < n_tables; ++q) {
    const mirec_adam_table& t = tables[q];
    const bool grouped = t.n_uniq != nullptr;
    if (!t.p || !t.m || !t.v || t.n_rows < 0 ||
        (grouped && (!t.uniq || !t.seg || !t.perm || !t.rows)) ||
        (sched != Sched::kStreamed && !t.last) ||
        (deferred && (!grouped || t.dense_grad || !n_max_uniq || n_max_uniq[q] < 0)) ||
        (deferred && (t.ahead_uniq == nullptr) != (t.ahead_n_uniq == nullptr))) {
      set_error("%s: bad table %d", what, q);
      return -1;
    }
    tabs.t[q] = t;
    if (deferred) {
      const int rpb = kAdamThreads / d;
      const int64_t nb = (n_max_uniq[q] + rpb - 1) / rpb;
      tabs.block_start[2 * q] = blocks;
      blocks += nb;
      tabs.block_start[2 * q + 1] = blocks;
      if (t.ahead_uniq) blocks += nb;
    } else {
      tabs.block_start[q] = blocks;
      blocks += (t.n_rows + kAdamRows - 1) / kAdamRows;
    }
  }
  (void)VPR;
  for (int q = tabs.n_seg; q <= 2 * kMaxTables; ++q) tabs.block_start[q] = blocks;
  if (blocks == 0) return 0;
  AdamConsts k;
  k.omb1 = (float)(1.0 - beta1);
  k.omb1m1 = k.omb1 - 1.0f;
  k.lerp_small = fabsf(k.omb1) < 0.5f;
  k.b2 = (float)beta2;
  k.omb2 = (float)(1.0 - beta2);
  k.eps = (float)eps;
  k.wd = (float)weight_decay;
  const dim3 grd((unsigned)blocks), blk(kAdamThreads);
  hipStream_t st = (hipStream_t)stream;
#define MIREC_ADAM_SCHED(DD)                                                                 \
  case DD:                                                                                   \
    if (sched == Sched::kStreamed)                                                           \
      hipLaunchKernelGGL(adam_multi_kernel<DD>, grd, blk, 0, st, tabs, consts, step_base,    \
                         step_off, k);                                                       \
    else if (sched == Sched::kDeferred)                                                      \
      hipLaunchKernelGGL(adam_deferred_kernel<DD>, grd, blk, 0, st, tabs, consts, step_base, \
                         step_off, k);                                                       \
    else                                                                                     \
      hipLaunchKernelGGL(adam_flush_kernel<DD>, grd, blk, 0, st, tabs, consts, step_base,    \
                         step_off, k);                                                       \
    break;
  switch (d) {
    MIREC_ADAM_SCHED(4)
    MIREC_ADAM_SCHED(16)
    MIREC_ADAM_SCHED(32)
    MIREC_ADAM_SCHED(64)
    MIREC_ADAM_SCHED(128)
    MIREC_ADAM_SCHED(256)
  }
#undef MIREC_ADAM_SCHED
  return launch_status(what);
}

}  // namespace

extern "C" int mirec_adam_multi_f32(const mirec_adam_table* tables, int32_t n_tables, int32_t d,
                                    const float* step_consts_dev, const int32_t* step_base_dev,
                                    int32_t step_off, double beta1, double beta2, double eps,
                                    double weight_decay, void* stream) {
  return launch_adam(Sched::kStreamed, tables, n_tables, nullptr, d, step_consts_dev,
                     step_base_dev, step_off, beta1, beta2, eps, weight_decay, stream,
                     "mirec_adam_multi_f32");
}

extern "C" int mirec_adam_deferred_f32(const mirec_adam_table* tables, int32_t n_tables,
                                       const int64_t* n_max_uniq, int32_t d,
                                       const float* step_consts_dev,
                                       const int32_t* step_base_dev, int32_t step_off,
                                       double beta1, double beta2, double eps,
                                       double weight_decay, void* stream) {
  return launch_adam(Sched::kDeferred, tables, n_tables, n_max_uniq, d, step_consts_dev,
                     step_base_dev, step_off, beta1, beta2, eps, weight_decay, stream,
                     "mirec_adam_deferred_f32");
}

extern "C" int mirec_adam_flush_f32(const mirec_adam_table* tables, int32_t n_tables, int32_t d,
                                    const float* step_consts_dev, const int32_t* step_base_dev,
                                    int32_t step_off, double beta1, double beta2, double eps,
                                    double weight_decay, void* stream) {
  return launch_adam(Sched::kFlush, tables, n_tables, nullptr, d, step_consts_dev,
                     step_base_dev, step_off, beta1, beta2, eps, weight_decay, stream,
                     "mirec_adam_flush_f32");
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
  memset(&t, 0, sizeof(t));
  t.p = p; t.m = m; t.v = v; t.n_rows = n_rows;
  t.rows = rows; t.perm = perm; t.uniq = uniq; t.seg = seg; t.n_uniq = n_uniq_dev;
  t.dense_grad = dense_grad;
  return mirec_adam_multi_f32(&t, 1, d, step_consts_dev, step_idx_dev, 0, beta1, beta2, eps,
                              weight_decay, stream);
}
