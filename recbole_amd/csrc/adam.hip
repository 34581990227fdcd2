// K5 — dense Adam over every row of the embedding tables, with the gradient
// supplied in grouped (compact) form. Two schedules, bit-identical results:
//
//  * streamed (adam_multi_kernel): one pass over p, m, v of EVERY row each step
//    (6 * n_rows * d * 4 bytes per step, the HBM roofline of the step);
//  * deferred (adam_deferred_kernel + the flush kernels): a row whose gradient is
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
// torch: {step_size = lr/(1-b1^t), bc2_sqrt = sqrt(1-b2^t), rbc = RN(1/bc2_sqrt),
// kq = step_size*bc2_sqrt*(1+2^-20) rounded up (p_update_vanishes)}.
// x / bc2_sqrt is evaluated as q = x*rbc; q + fma(-q, bc2_sqrt, x)*rbc (fma):
// with rbc the correctly rounded reciprocal this is the correctly rounded
// quotient (Markstein's theorem; checked exhaustively over two binades of x for
// ~13k divisors of several beta2), i.e. bit-identical to IEEE division in 3
// instead of ~11 instructions. x = +inf takes the IEEE division.

#include "adam_core.h"

namespace mirec {

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
// V = float or float2 columns per thread. A row's replay is a serial chain per
// element; a launch with few rows (one 512-positive batch: a few waves per SIMD)
// takes as long as its longest chain, so one column per lane (shortest chains);
// a launch with many rows (a data-parallel global batch) is issue-bound, so two
// (half the per-wave overhead). The host picks by the launch's row bound.
// RPB = 256 / (D / |V|) whole rows per block. Segment 2q: table q's touched rows,
// 2q+1: its look-ahead rows (the entry's work: adam_core.h deferred_row).
// Block of the deferred kernel: one row when a row fills whole waves, else one
// wave of rows. Small blocks: the launch's rows differ widely in replay length,
// and a CU takes a new block only when a whole block's waves are free.
#ifndef MIREC_DEFERRED_MIN_BLOCK
// lanes per block: 256 (C3 336.9 -> 340.1 K sequences/s against 64 — a quarter of the
// workgroups to dispatch)
#define MIREC_DEFERRED_MIN_BLOCK 256
#endif
__host__ __device__ constexpr int deferred_block(int vpr) {
  return vpr > MIREC_DEFERRED_MIN_BLOCK ? vpr : MIREC_DEFERRED_MIN_BLOCK;
}

// One block of segment si (table si >> 1; touched rows, or look-ahead rows when si is odd).
template <int D, typename V>
__device__ __forceinline__ void deferred_block_rows(const AdamTables& tabs, int si,
                                                    const float* __restrict__ consts, int st,
                                                    const AdamConsts& k) {
  constexpr int VPR = D / Lanes<V>::n;              // V = float or float2 per thread
  constexpr int RPB = deferred_block(VPR) / VPR;    // rows per block
  static_assert(deferred_block(VPR) % VPR == 0, "row width");
  const mirec_adam_table& T = tabs.t[si >> 1];
  const bool ahead = si & 1;
  const int u = (int)(((int64_t)blockIdx.x - tabs.block_start[si]) * RPB) + threadIdx.x / VPR;
  const int c = threadIdx.x % VPR;
  const int n = ahead ? T.ahead_n_uniq[0] : T.n_uniq[0];
  // the grid is sized for the host's bound on the lists: blocks past the actual
  // count leave at once (block-uniform: no thread reaches the barrier below)
  if ((int)(((int64_t)blockIdx.x - tabs.block_start[si]) * RPB) >= n) return;
  deferred_row<D, V>(T, ahead, u, n, st, consts, k, c, [](bool, bool, int64_t, const V&) {});
}

template <int D, typename V>
__global__ __launch_bounds__(kAdamThreads) void adam_deferred_kernel(
    const AdamTables tabs, const float* __restrict__ consts,
    const int32_t* __restrict__ step_base, int step_off, AdamConsts k) {
  deferred_block_rows<D, V>(tabs, segment_of(tabs, blockIdx.x), consts, step_base[0] + step_off,
                            k);
}

// A [V, D] table and a [V, 1] table in one launch (DeepFM's token embeddings and their
// first-order weights: the same rows, the same step; they ran as two launches of ~6 us
// each, twice a step — catch-up and step — where each launch is a dependent-load chain
// that leaves most of the chip idle). Segments 0, 1: table 0 (width D, V columns per
// lane); 2, 3: table 1 (one float per lane). Both block shapes are 256 lanes.
template <int D, typename V>
__global__ __launch_bounds__(kAdamThreads) void adam_deferred_pair_kernel(
    const AdamTables tabs, const float* __restrict__ consts,
    const int32_t* __restrict__ step_base, int step_off, AdamConsts k) {
  static_assert(deferred_block(D / Lanes<V>::n) == deferred_block(1), "one block shape");
  const int si = segment_of(tabs, blockIdx.x);
  const int st = step_base[0] + step_off;
  if (si < 2)
    deferred_block_rows<D, V>(tabs, si, consts, st, k);
  else
    deferred_block_rows<1, float>(tabs, si, consts, st, k);
}

// Flush of narrow rows (d < 64; d = 1 is DeepFM's first-order [V, 1] table): a block owns
// kFlushRows consecutive rows. Its threads read the rows' `last` marks in one coalesced
// pass (kFlushRows / 256 independent loads per thread), the rows that lag are listed in
// LDS, and only those are loaded and replayed, VPR lanes per row (float4 columns; one
// float per lane at d = 1). The list's order depends on the LDS atomics, the results do
// not: every row's replay is its own (adam_replay's wave votes only skip p updates that
// provably round away). The form this replaces walked its rows in 16 dependent passes,
// loaded or not: 371 us for DeepFM's 33 M-row token table (+71 us for the [V, 1] one)
// where the `last` reads alone are 132 MB (~17 us at HBM rate).
template <int D> struct NarrowVec { using T = float4; static constexpr int vpr = D / 4; };
template <> struct NarrowVec<1> { using T = float; static constexpr int vpr = 1; };

template <int D>
__global__ __launch_bounds__(kAdamThreads) void adam_flush_list_kernel(
    const AdamTables tabs, const float* __restrict__ consts, const int32_t* __restrict__ step_base,
    int step_off, AdamConsts k) {
  using V = typename NarrowVec<D>::T;
  constexpr int VPR = NarrowVec<D>::vpr;
  constexpr int RPP = kAdamThreads / VPR;           // rows per pass
  constexpr int PER = kFlushRows / kAdamThreads;    // `last` loads per thread
  static_assert(kFlushRows % kAdamThreads == 0 && kAdamThreads % VPR == 0, "block shape");
  __shared__ int32_t s_row[kFlushRows];             // lagging rows (offset in the block)
  __shared__ int32_t s_last[kFlushRows];            // and their marks
  __shared__ int32_t s_n;
  const int si = segment_of(tabs, blockIdx.x);
  const mirec_adam_table& T = tabs.t[si];
  const int64_t lo = ((int64_t)blockIdx.x - tabs.block_start[si]) * kFlushRows;
  const int target = step_base[0] + step_off;
  const int lane = threadIdx.x & 63;
  if (threadIdx.x == 0) s_n = 0;
  int raw[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int64_t r = lo + j * kAdamThreads + threadIdx.x;
    raw[j] = r < T.n_rows ? T.last[r] : target;
  }
  __syncthreads();
  const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const bool need = min(raw[j], target) < target;
    const uint64_t b = __ballot(need);
    int at = 0;
    if (lane == 0 && b) at = atomicAdd(&s_n, __popcll(b));
    at = __shfl(at, 0, 64);
    if (need) {
      const int pos = at + __popcll(b & below);
      s_row[pos] = j * kAdamThreads + threadIdx.x;
      s_last[pos] = raw[j];
    }
  }
  __syncthreads();
  const int n = s_n;
  const int rsub = threadIdx.x / VPR;
  const int c = threadIdx.x % VPR;
  for (int base = 0; base < n; base += RPP) {       // block-uniform trip count
    const int i = base + rsub;
    const bool work = i < n;
    const int64_t r = lo + (work ? s_row[i] : 0);
    const int last = work ? min(s_last[i], target) : target;
    const int64_t off = r * VPR + c;
    V p, m, v;
    memset(&p, 0, sizeof(V));
    m = p;
    v = p;
    if (work) {
      p = reinterpret_cast<const V*>(T.p)[off];
      m = reinterpret_cast<const V*>(T.m)[off];
      v = reinterpret_cast<const V*>(T.v)[off];
    }
    adam_replay(p, m, v, last, target, consts, k);
    if (work) {
      reinterpret_cast<V*>(T.p)[off] = p;
      reinterpret_cast<V*>(T.m)[off] = m;
      reinterpret_cast<V*>(T.v)[off] = v;
      if (c == 0) T.last[r] = target;
    }
  }
}

// Flush with one row per wave (D >= 64: D/64 floats per lane), so every lane of
// a wave replays the same steps (the float4 kernel above puts 256/D rows in a
// wave, whose replay counts differ: the wave runs the longest of them). Rows
// already complete exit without loading.
template <int D>
struct FlushVec { using T = float; };
template <> struct FlushVec<128> { using T = float2; };
template <> struct FlushVec<256> { using T = float4; };

#ifndef MIREC_FLUSH_THREADS
#define MIREC_FLUSH_THREADS 64
#endif
constexpr int kFlushRowThreads = MIREC_FLUSH_THREADS;

template <int D>
__global__ __launch_bounds__(kFlushRowThreads) void adam_flush_row_kernel(
    const AdamTables tabs, const float* __restrict__ consts, const int32_t* __restrict__ step_base,
    int step_off, AdamConsts k) {
  using V = typename FlushVec<D>::T;
  constexpr int RPB = kFlushRowThreads / 64;        // rows (waves) per block
  const int si = segment_of(tabs, blockIdx.x);
  const mirec_adam_table& T = tabs.t[si];
  const int64_t r = ((int64_t)blockIdx.x - tabs.block_start[si]) * RPB + (threadIdx.x >> 6);
  if (r >= T.n_rows) return;
  const int target = step_base[0] + step_off;
  const int raw = __builtin_amdgcn_readfirstlane(T.last[r]);
  const int last = min(raw, target);
  const int64_t off = r * 64 + (threadIdx.x & 63);
  // parity buffers (p_alt, mirec_bpr_adam_step_f32): state t in t & 1 ? p_alt : p; the
  // flush completes every row into its target buffer AND into p (the parameter)
  const bool par = T.p_alt != nullptr;
  const bool odd = par && (target & 1);
  if (last >= target) {
    if (odd && raw != kZeroState)            // current, held in p_alt only: publish to p
      reinterpret_cast<V*>(T.p)[off] = reinterpret_cast<const V*>(T.p_alt)[off];
    return;
  }
  V p = reinterpret_cast<const V*>((par && (last & 1)) ? T.p_alt : T.p)[off];
  V m = reinterpret_cast<const V*>(T.m)[off];
  V v = reinterpret_cast<const V*>(T.v)[off];
  replay<V, true>(p, m, v, last, target, consts, k);
  MIREC_WORK(10, 1);
  if (odd) reinterpret_cast<V*>(T.p_alt)[off] = p;
  reinterpret_cast<V*>(T.p)[off] = p;
  reinterpret_cast<V*>(T.m)[off] = m;
  reinterpret_cast<V*>(T.v)[off] = v;
  if ((threadIdx.x & 63) == 0) T.last[r] = target;
}

// Flush for sparse activity (the first steps of an epoch: most rows are in the zero
// state, which is current at every step). One wave per row would dispatch a workgroup
// per table row, and the dispatcher hands out ~2-3 workgroups per ns: a C2 flush of
// 165 K one-wave blocks takes ~55 µs whatever the work. Here each wave owns R
// consecutive rows (R per table, host's choice): lanes 0..R-1 read `last`, one ballot
// lists the rows that lag (or, at an odd target, are current in p_alt only), and the
// wave completes them one after another with the one-row-per-wave body above (same
// replay engine, same results). Blocks of four waves: R = 8 makes the grid 32x smaller.
struct FlushRows {
  int32_t r[kMaxTables];
};

template <int D>
__global__ __launch_bounds__(kAdamThreads) void adam_flush_scan_kernel(
    const AdamTables tabs, const float* __restrict__ consts, const int32_t* __restrict__ step_base,
    int step_off, AdamConsts k, FlushRows rows_per_wave) {
  using V = typename FlushVec<D>::T;
  const int si = segment_of(tabs, blockIdx.x);
  const mirec_adam_table& T = tabs.t[si];
  const int R = rows_per_wave.r[si];
  const int lane = threadIdx.x & 63;
  const int64_t r0 =
      (((int64_t)blockIdx.x - tabs.block_start[si]) * (kAdamThreads / 64) + (threadIdx.x >> 6)) * R;
  if (r0 >= T.n_rows) return;                          // wave-uniform
  const int target = step_base[0] + step_off;
  const bool par = T.p_alt != nullptr;
  const bool odd = par && (target & 1);
  int raw = kZeroState;
  if (lane < R && r0 + lane < T.n_rows) raw = T.last[r0 + lane];
  const bool need = min(raw, target) < target || (odd && raw != kZeroState);
  uint64_t todo = __ballot(need);
  while (todo) {                                       // wave-uniform loop over its rows
    const int i = __builtin_ctzll(todo);
    todo &= todo - 1;
    const int64_t r = r0 + i;
    const int rraw = __shfl(raw, i, 64);
    const int last = min(rraw, target);
    const int64_t off = r * 64 + lane;
    if (last >= target) {                              // current, in p_alt only: publish
      reinterpret_cast<V*>(T.p)[off] = reinterpret_cast<const V*>(T.p_alt)[off];
      continue;
    }
    V p = reinterpret_cast<const V*>((par && (last & 1)) ? T.p_alt : T.p)[off];
    V m = reinterpret_cast<const V*>(T.m)[off];
    V v = reinterpret_cast<const V*>(T.v)[off];
    replay<V, true>(p, m, v, last, target, consts, k);
    MIREC_WORK(10, 1);
    if (odd) reinterpret_cast<V*>(T.p_alt)[off] = p;
    reinterpret_cast<V*>(T.p)[off] = p;
    reinterpret_cast<V*>(T.m)[off] = m;
    reinterpret_cast<V*>(T.v)[off] = v;
    if (lane == 0) T.last[r] = target;
  }
}

}  // namespace mirec

using namespace mirec;

namespace {

enum class Sched { kStreamed, kDeferred, kFlush, kDeferredPair };

int launch_adam(Sched sched, const mirec_adam_table* tables, int32_t n_tables,
                const int64_t* n_max_uniq, int32_t d, const float* consts,
                const int32_t* step_base, int32_t step_off, double beta1, double beta2,
                double eps, double weight_decay, void* stream, const char* what,
                const int32_t* flush_rows = nullptr) {
  if (n_tables < 1 || n_tables > kMaxTables || !tables || !consts || !step_base) {
    set_error("%s: bad arguments (n_tables=%d)", what, n_tables);
    return -1;
  }
  if (((uintptr_t)consts & 15) != 0) {
    set_error("%s: step constants must be 16-byte aligned", what);
    return -1;
  }
  if (d != 4 && d != 16 && d != 32 && d != 64 && d != 128 && d != 256 &&
      !(d == 1 && sched != Sched::kStreamed)) {
    set_error("%s: row width %d not in {4,16,32,64,128,256} (1: deferred / flush)", what, d);
    return -1;
  }
  const int VPR = d / 4;
  // deferred pair (mirec_adam_deferred_pair_f32): tables[0] width d, tables[1] width 1
  const bool pair = sched == Sched::kDeferredPair;
  if (pair) {
    if (n_tables != 2 || d == 1) {
      set_error("%s: a pair is two tables, the first of width d > 1 (got %d tables, d=%d)",
                what, n_tables, d);
      return -1;
    }
    sched = Sched::kDeferred;
  }
  // flush with R rows per wave (adam_flush_scan_kernel): d >= 64, R in [1, 64] per table
  FlushRows fr;
  bool scan = false;
  for (int q = 0; q < kMaxTables; ++q) fr.r[q] = 1;
  if (sched == Sched::kFlush && flush_rows) {
    if (d < 64) {
      set_error("%s: rows per wave need d >= 64", what);
      return -1;
    }
    for (int q = 0; q < n_tables; ++q) {
      if (flush_rows[q] < 1 || flush_rows[q] > 64) {
        set_error("%s: rows per wave %d of table %d not in [1, 64]", what, flush_rows[q], q);
        return -1;
      }
      fr.r[q] = flush_rows[q];
    }
    scan = true;
  }
  AdamTables tabs;
  memset(&tabs, 0, sizeof(tabs));
  const bool deferred = sched == Sched::kDeferred;
  tabs.n_seg = deferred ? 2 * n_tables : n_tables;
  // deferred: float columns per thread while the launch fits ~16 waves per SIMD
  int dvec = 1;
  if (deferred && n_max_uniq && d >= 4) {
    int64_t waves = 0;
    for (int q = 0; q < (pair ? 1 : n_tables); ++q)
      if (n_max_uniq[q] > 0)
        waves += n_max_uniq[q] * (tables[q].ahead_uniq ? 2 : 1) * ((d + 63) / 64);
    if (waves > 16 * 1024) dvec = 2;
    // a touched-rows-only launch (no look-ahead lists: the step after the forward's
    // catch-ups, whose rows need no replay) streams p, m, v and the gradient rows: four
    // columns per lane (C3's step launch 180 -> 149 us; rows that do lag still replay
    // exactly, through the general replay)
    bool ahead = false;
    for (int q = 0; q < n_tables; ++q) ahead = ahead || tables[q].ahead_uniq != nullptr;
    if (dvec == 2 && d >= 128 && !ahead && !pair) dvec = 4;
  }
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
    if (t.p_alt && (sched == Sched::kStreamed || d < 64 || pair)) {
      set_error("%s: table %d: parity buffer (p_alt) needs the deferred schedule and d >= 64",
                what, q);
      return -1;
    }
    tabs.t[q] = t;
    if (deferred) {
      const int rpb = (pair && q == 1) ? deferred_block(1) : deferred_block(d / dvec) / (d / dvec);
      const int64_t nb = (n_max_uniq[q] + rpb - 1) / rpb;
      tabs.block_start[2 * q] = blocks;
      blocks += nb;
      tabs.block_start[2 * q + 1] = blocks;
      if (t.ahead_uniq) blocks += nb;
    } else {
      tabs.block_start[q] = blocks;
      const int64_t rows_per_block =
          scan ? (int64_t)(kAdamThreads / 64) * fr.r[q]
          : (sched == Sched::kFlush && d >= 64) ? kFlushRowThreads / 64
          : sched == Sched::kFlush ? kFlushRows
                                   : kAdamRows;
      blocks += (t.n_rows + rows_per_block - 1) / rows_per_block;
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
    else if (deferred && pair)                                                               \
      hipLaunchKernelGGL((dvec == 2 ? adam_deferred_pair_kernel<DD, float2>                  \
                                    : adam_deferred_pair_kernel<DD, float>),                 \
                         grd, dim3(deferred_block(1)), 0, st, tabs, consts, step_base,       \
                         step_off, k);                                                       \
    else if (deferred)                                                                       \
      hipLaunchKernelGGL((dvec == 4 ? adam_deferred_kernel<DD, float4>                       \
                          : dvec == 2 ? adam_deferred_kernel<DD, float2>                     \
                                      : adam_deferred_kernel<DD, float>),                    \
                         grd, dim3(deferred_block(DD / dvec)), 0, st, tabs, consts,          \
                         step_base, step_off, k);                                            \
    else if (DD >= 64 && scan)                                                               \
      hipLaunchKernelGGL(adam_flush_scan_kernel<(DD >= 64 ? DD : 64)>, grd, blk, 0, st, tabs,  \
                         consts, step_base, step_off, k, fr);                                \
    else if (DD >= 64)                                                                       \
      hipLaunchKernelGGL(adam_flush_row_kernel<(DD >= 64 ? DD : 64)>, grd,                   \
                         dim3(kFlushRowThreads), 0, st, tabs,                                \
                         consts, step_base, step_off, k);                                    \
    else                                                                                     \
      hipLaunchKernelGGL(adam_flush_list_kernel<(DD < 64 ? DD : 16)>, grd, blk, 0, st, tabs, \
                         consts, step_base, step_off, k);                                    \
    break;
  switch (d) {
    case 1:
      if (deferred)
        hipLaunchKernelGGL((adam_deferred_kernel<1, float>), grd, dim3(deferred_block(1)), 0, st,
                           tabs, consts, step_base, step_off, k);
      else
        hipLaunchKernelGGL(adam_flush_list_kernel<1>, grd, blk, 0, st, tabs, consts, step_base,
                           step_off, k);
      break;
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

extern "C" int mirec_adam_deferred_pair_f32(const mirec_adam_table* tables,
                                            const int64_t* n_max_uniq, int32_t d,
                                            const float* step_consts_dev,
                                            const int32_t* step_base_dev, int32_t step_off,
                                            double beta1, double beta2, double eps,
                                            double weight_decay, void* stream) {
  return launch_adam(Sched::kDeferredPair, tables, 2, n_max_uniq, d, step_consts_dev,
                     step_base_dev, step_off, beta1, beta2, eps, weight_decay, stream,
                     "mirec_adam_deferred_pair_f32");
}

extern "C" int mirec_adam_flush_f32(const mirec_adam_table* tables, int32_t n_tables, int32_t d,
                                    const float* step_consts_dev, const int32_t* step_base_dev,
                                    int32_t step_off, double beta1, double beta2, double eps,
                                    double weight_decay, void* stream) {
  return launch_adam(Sched::kFlush, tables, n_tables, nullptr, d, step_consts_dev,
                     step_base_dev, step_off, beta1, beta2, eps, weight_decay, stream,
                     "mirec_adam_flush_f32");
}

#if defined(MIREC_STEP_COUNT)
// diagnostic build only: this unit's executed-work counters (the flush's replays)
extern "C" int mirec_work_counters_adam(unsigned long long* dst, int clear) {
  if (hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_work), sizeof(g_work)) != hipSuccess) return -1;
  if (clear) {
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_work), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

extern "C" int mirec_adam_flush_rows_f32(const mirec_adam_table* tables, int32_t n_tables,
                                         int32_t d, const int32_t* rows_per_wave,
                                         const float* step_consts_dev,
                                         const int32_t* step_base_dev, int32_t step_off,
                                         double beta1, double beta2, double eps,
                                         double weight_decay, void* stream) {
  if (!rows_per_wave) {
    set_error("mirec_adam_flush_rows_f32: rows_per_wave is NULL");
    return -1;
  }
  return launch_adam(Sched::kFlush, tables, n_tables, nullptr, d, step_consts_dev,
                     step_base_dev, step_off, beta1, beta2, eps, weight_decay, stream,
                     "mirec_adam_flush_rows_f32", rows_per_wave);
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

namespace mirec {

// Flat form: any number of elements (biases, [n,1] first-order tables, MLP
// weights whose numel is not a multiple of 4), dense gradient, same adam_elem.
__global__ __launch_bounds__(kAdamThreads) void adam_flat_kernel(
    float* __restrict__ p, float* __restrict__ m, float* __restrict__ v, int64_t n,
    const float* __restrict__ g, const float* __restrict__ consts,
    const int32_t* __restrict__ step_idx, AdamConsts k) {
  const StepConsts sc = step_consts(consts, step_idx[0]);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float pp = p[i], mm = m[i], vv = v[i];
    adam_elem(pp, mm, vv, g[i], sc, k);
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
  }
}

// Several flat parameters in one launch (every dense parameter of a model step: the
// MLP's weights and biases, float-field embeddings, scalar biases — C4 ran them as six
// launches): block b takes 1,024 consecutive elements of the parameter whose block
// range holds b. The same adam_elem per element as every other K5 form.
constexpr int kFlatMax = 16;
struct FlatParams {
  mirec_flat_param t[kFlatMax];
  int64_t block_start[kFlatMax + 1];
  int n;
};

// advance != nullptr: the step counter the launch read is advanced once every block has
// read it — the block that takes the last ticket (agent-scope counter, zero between
// launches) adds 1 and zeroes the ticket (graph mode's `step += 1` without a launch).
__global__ __launch_bounds__(kAdamThreads) void adam_flat_multi_kernel(
    const FlatParams fp, const float* __restrict__ consts, const int32_t* step_idx,
    AdamConsts k, int32_t* advance, int32_t* __restrict__ ticket) {
  // step_idx and advance may be the same word (mirec_adam_flat_multi_advance_f32): neither
  // is __restrict__, and the advance is an atomic add after every block has read it
  int q = 0;
#pragma unroll
  for (int t = 1; t < kFlatMax; ++t)
    if (t < fp.n && (int64_t)blockIdx.x >= fp.block_start[t]) q = t;
  const mirec_flat_param& P = fp.t[q];
  const StepConsts sc = step_consts(consts, step_idx[0]);
  const int64_t i0 = ((int64_t)blockIdx.x - fp.block_start[q]) * (4 * kAdamThreads);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t i = i0 + u * kAdamThreads + threadIdx.x;
    if (i < P.n) {
      float pp = P.p[i], mm = P.m[i], vv = P.v[i];
      adam_elem(pp, mm, vv, P.g[i], sc, k);
      P.p[i] = pp;
      P.m[i] = mm;
      P.v[i] = vv;
    }
  }
  if (advance) {
    __syncthreads();                       // every lane's read of step_idx is done
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            (int)gridDim.x - 1) {
      __hip_atomic_fetch_add(advance, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ticket[0] = 0;
    }
  }
}

}  // namespace mirec

static int flat_multi_impl(const mirec_flat_param* params, int32_t n_params,
                           const float* step_consts_dev, const int32_t* step_idx_dev,
                           double beta1, double beta2, double eps, double weight_decay,
                           int32_t* advance, int32_t* ticket, void* stream) {
  if (n_params == 0) return 0;
  if (!params || n_params < 0 || n_params > kFlatMax || !step_consts_dev || !step_idx_dev) {
    set_error("mirec_adam_flat_multi_f32: bad arguments (at most %d parameters)", kFlatMax);
    return -1;
  }
  FlatParams fp;
  memset(&fp, 0, sizeof(fp));
  fp.n = n_params;
  int64_t blocks = 0;
  for (int q = 0; q < n_params; ++q) {
    const mirec_flat_param& t = params[q];
    if (!t.p || !t.m || !t.v || !t.g || t.n < 0) {
      set_error("mirec_adam_flat_multi_f32: bad parameter %d", q);
      return -1;
    }
    fp.t[q] = t;
    fp.block_start[q] = blocks;
    blocks += (t.n + 4 * kAdamThreads - 1) / (4 * kAdamThreads);
  }
  for (int q = n_params; q <= kFlatMax; ++q) fp.block_start[q] = blocks;
  if (blocks == 0) return 0;
  AdamConsts k;
  k.omb1 = (float)(1.0 - beta1);
  k.omb1m1 = k.omb1 - 1.0f;
  k.lerp_small = fabsf(k.omb1) < 0.5f;
  k.b2 = (float)beta2;
  k.omb2 = (float)(1.0 - beta2);
  k.eps = (float)eps;
  k.wd = (float)weight_decay;
  hipLaunchKernelGGL(adam_flat_multi_kernel, dim3((unsigned)blocks), dim3(kAdamThreads), 0,
                     (hipStream_t)stream, fp, step_consts_dev, step_idx_dev, k, advance, ticket);
  return launch_status("mirec_adam_flat_multi_f32");
}

extern "C" int mirec_adam_flat_multi_f32(const mirec_flat_param* params, int32_t n_params,
                                         const float* step_consts_dev,
                                         const int32_t* step_idx_dev, double beta1, double beta2,
                                         double eps, double weight_decay, void* stream) {
  return flat_multi_impl(params, n_params, step_consts_dev, step_idx_dev, beta1, beta2, eps,
                         weight_decay, nullptr, nullptr, stream);
}

extern "C" int mirec_adam_flat_multi_advance_f32(const mirec_flat_param* params,
                                                 int32_t n_params, const float* step_consts_dev,
                                                 int32_t* step_counter_dev, int32_t* ticket_dev,
                                                 double beta1, double beta2, double eps,
                                                 double weight_decay, void* stream) {
  if (!step_counter_dev || !ticket_dev || n_params <= 0) {
    set_error("mirec_adam_flat_multi_advance_f32: bad arguments");
    return -1;
  }
  int64_t blocks = 0;
  for (int q = 0; q < n_params && q < kFlatMax; ++q)
    blocks += (params[q].n + 4 * kAdamThreads - 1) / (4 * kAdamThreads);
  if (blocks == 0) {
    set_error("mirec_adam_flat_multi_advance_f32: no elements (the counter would not advance)");
    return -1;
  }
  return flat_multi_impl(params, n_params, step_consts_dev, step_counter_dev, beta1, beta2, eps,
                         weight_decay, step_counter_dev, ticket_dev, stream);
}

extern "C" int mirec_adam_flat_f32(float* p, float* m, float* v, int64_t n,
                                   const float* grad, const float* step_consts_dev,
                                   const int32_t* step_idx_dev, double beta1, double beta2,
                                   double eps, double weight_decay, void* stream) {
  if (n == 0) return 0;
  if (!p || !m || !v || !grad || !step_consts_dev || !step_idx_dev || n < 0) {
    set_error("mirec_adam_flat_f32: bad arguments");
    return -1;
  }
  AdamConsts k;
  k.omb1 = (float)(1.0 - beta1);
  k.omb1m1 = k.omb1 - 1.0f;
  k.lerp_small = fabsf(k.omb1) < 0.5f;
  k.b2 = (float)beta2;
  k.omb2 = (float)(1.0 - beta2);
  k.eps = (float)eps;
  k.wd = (float)weight_decay;
  int64_t blocks = (n + kAdamThreads - 1) / kAdamThreads;
  if (blocks > 256 * 16) blocks = 256 * 16;
  hipLaunchKernelGGL(adam_flat_kernel, dim3((unsigned)blocks), dim3(kAdamThreads), 0,
                     (hipStream_t)stream, p, m, v, n, grad, step_consts_dev, step_idx_dev, k);
  return launch_status("mirec_adam_flat_f32");
}
