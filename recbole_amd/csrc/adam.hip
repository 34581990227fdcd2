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
// torch: {step_size = lr/(1-b1^t), bc2_sqrt = sqrt(1-b2^t), rbc = RN(1/bc2_sqrt),
// kq = step_size*bc2_sqrt*(1+2^-20) rounded up (p_update_vanishes)}.
// x / bc2_sqrt is evaluated as q = x*rbc; q + fma(-q, bc2_sqrt, x)*rbc (fma):
// with rbc the correctly rounded reciprocal this is the correctly rounded
// quotient (Markstein's theorem; checked exhaustively over two binades of x for
// ~13k divisors of several beta2), i.e. bit-identical to IEEE division in 3
// instead of ~11 instructions. x = +inf takes the IEEE division.
#include "common.h"
#include "adam_math.h"

// No FMA contraction: every op rounds on its own, as in torch's op-by-op
// _single_tensor_adam, and the streamed / deferred schedules stay bit-identical
// whatever the compiler could fuse in either context.
#pragma clang fp contract(off)

namespace mirec {

constexpr int kAdamThreads = 256;
constexpr int kAdamRows = 64;  // table rows per block (streamed / flush)
constexpr int kMaxTables = 4;
// last[row] mark of the deferred schedule (MIREC_ADAM_ZERO_STATE in mirec.h): the
// row's m and v are all +0 and weight_decay is 0, so every zero-gradient step is
// the identity (m' = fma(-(1-b1), +0, +0) = +0, v' = +0 * b2 = +0, p' = p + (-0)
// = p, bit for bit). Such a row is current at any step: a flush or a look-ahead
// leaves it untouched (no load, no store); its first real step starts from it.
constexpr int kZeroState = MIREC_ADAM_ZERO_STATE;

struct AdamConsts {
  float omb1, omb1m1, b2, omb2, eps, wd;
  int lerp_small;  // 1 - beta1 < 0.5: lerp from m (torch's is_lerp_weight_small)
};

struct StepConsts {
  float ss, bc2s, rbc, kq;  // kq >= step_size * bc2_sqrt * (1 + 2^-20), rounded up
};

__device__ __forceinline__ StepConsts step_consts(const float* __restrict__ consts, int s) {
  const float4 c = reinterpret_cast<const float4*>(consts)[s];
  return {c.x, c.y, c.z, c.w};
}

// Zero-gradient step whose p update provably rounds away: with me, ve the new
// moments, the increment q = RN(RN(-ss*me) / den), den = RN(RN(RN(sqrt(ve))/bc2s)
// + eps) >= sqrt(ve)(1-u)^3/bc2s, so |q| <= kq*|me|/sqrt(ve) (u = 2^-24; kq holds
// the (1+u)^2/(1-u)^3 margin). If that bound is below ulp(p)/4, RN(p + q) == p
// (the nearest other float is at least ulp(p)/2 away, also below a power of two).
// Tested without sqrt or division as (kq*|me| * 2^(26-e))^2 < 0.999*ve, where
// p = f*2^e, f in [0.5, 1): the power-of-two scaling is exact, the two roundings
// of the left side and the 0.999 cover the rest. Only for normal |p| >= 2^-60
// and ve >= 2^-100 (no denormal scaling error can matter there).
// me == 0 (a row never touched, or whose momentum underflowed): q = -0 / den with
// den >= eps > 0, and p + (-0) == p for every p, zeros included.
__device__ __forceinline__ bool p_update_vanishes(float p, float me, float ve,
                                                  const StepConsts& sc, float eps) {
  const uint32_t ex = (__float_as_uint(p) >> 23) & 0xffu;       // biased exponent
  const float scale = __uint_as_float((279u - ex) << 23);        // 2^(152-ex) = 2^(26-e)
  const float t = (sc.kq * fabsf(me)) * scale;
  return (me == 0.f && eps > 0.f) ||
         (ex >= 67u && ex < 255u && ve >= 0x1p-100f && t * t < 0.999f * ve);
}

// Launch = a list of segments, each a contiguous block range over one table.
// Streamed / flush: segment q = table q. Deferred: segment 2q = table q's
// touched rows, 2q+1 = its look-ahead rows.
struct AdamTables {
  mirec_adam_table t[kMaxTables];
  int64_t block_start[2 * kMaxTables + 1];
  int n_seg;
};

// x / bc2_sqrt, correctly rounded, for x = sqrt(v) >= 0 (header comment);
// branch-free so the columns of a thread interleave. +inf / bc2_sqrt = +inf.
__device__ __forceinline__ float div_bc2s(float x, const StepConsts& sc) {
  const float q = x * sc.rbc;
  const float r = fmaf(fmaf(-q, sc.bc2s, x), sc.rbc, q);
  return x == __builtin_inff() ? x : r;
}

// One Adam step of one element. Shared by every schedule so the arithmetic is
// the same instruction sequence wherever a step is applied.
__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g,
                                          const StepConsts& sc, const AdamConsts& k) {
  if (k.wd != 0.f) g = fmaf(p, k.wd, g);
  const float dlt = g - m;
  const float me = k.lerp_small ? fmaf(k.omb1, dlt, m) : fmaf(k.omb1m1, dlt, g);
  const float ve = fmaf(k.omb2 * g, g, v * k.b2);
  const float den = div_bc2s(sqrtf(ve), sc) + k.eps;
  p = p + ((-sc.ss) * me) / den;
  m = me;
  v = ve;
}

// adam_elem with g = 0, wd = 0 and 1-b1 < 0.5, rewritten with the same results:
//   fma(1-b1, 0 - m, m) == fma(-(1-b1), m, m)   (0 - m == -m up to the sign of a
//     zero, and a zero product added to m gives the same sum either way);
//   fma((1-b2)*0, 0, v*b2) == v*b2              (adding +0 to v*b2 >= +0).
__device__ __forceinline__ void adam_elem_zero(float& p, float& m, float& v, const StepConsts& sc,
                                               const AdamConsts& k) {
  const float me = fmaf(-k.omb1, m, m);
  const float ve = v * k.b2;
  const float den = div_bc2s(sqrtf(ve), sc) + k.eps;
  p = p + ((-sc.ss) * me) / den;
  m = me;
  v = ve;
}

// Element-wise over the components of a float, float2 or float4.
template <typename V> struct Lanes;
template <> struct Lanes<float> {
  static constexpr int n = 1;
  __device__ static float& at(float& x, int) { return x; }
  __device__ static float at(const float& x, int) { return x; }
};
template <> struct Lanes<float2> {
  static constexpr int n = 2;
  __device__ static float& at(float2& x, int i) { return i ? x.y : x.x; }
  __device__ static float at(const float2& x, int i) { return i ? x.y : x.x; }
};
template <> struct Lanes<float4> {
  static constexpr int n = 4;
  __device__ static float& at(float4& x, int i) {
    return i == 0 ? x.x : i == 1 ? x.y : i == 2 ? x.z : x.w;
  }
  __device__ static float at(const float4& x, int i) {
    return i == 0 ? x.x : i == 1 ? x.y : i == 2 ? x.z : x.w;
  }
};

template <typename V>
__device__ __forceinline__ void adam_vec(V& p, V& m, V& v, const V& g, const StepConsts& sc,
                                         const AdamConsts& k) {
#pragma unroll
  for (int i = 0; i < Lanes<V>::n; ++i)
    adam_elem(Lanes<V>::at(p, i), Lanes<V>::at(m, i), Lanes<V>::at(v, i), Lanes<V>::at(g, i),
              sc, k);
}

__device__ __forceinline__ int wave_min_i(int x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x = min(x, __shfl_xor(x, off, 64));
  return x;
}

// Replay steps [s0, s1) with a zero gradient (the exact per-step sequence).
// The step loop runs over the wave's smallest s0, so the step index is
// wave-uniform (scalar constant loads, one loop for all lanes); a lane applies
// step s only from its own s0 on (one row per wave for d >= 128: no idle lanes).
template <typename V>
__device__ __forceinline__ void adam_replay(V& p, V& m, V& v, int s0, int s1,
                                            const float* __restrict__ consts,
                                            const AdamConsts& k) {
  const int lo = __builtin_amdgcn_readfirstlane(wave_min_i(s0));
  if (k.wd == 0.f && k.lerp_small) {
    // Long-idle rows: once every p update of the wave provably rounds away
    // (p_update_vanishes), a step only moves m and v. The test runs every step
    // while it holds and every 4th step while it does not; a skipped step gives
    // exactly the bits the full step would.
    bool skipping = false;
    constexpr int N = Lanes<V>::n;
    for (int s = lo; s < s1; ++s) {
      const StepConsts sc = step_consts(consts, s);
      const bool act = s >= s0;
      float me[N], ve[N];
#pragma unroll
      for (int i = 0; i < N; ++i) {
        me[i] = fmaf(-k.omb1, Lanes<V>::at(m, i), Lanes<V>::at(m, i));
        ve[i] = Lanes<V>::at(v, i) * k.b2;
      }
      bool vanish = false;
      if (skipping || ((s - lo) & 3) == 0) {
        bool mine = true;
#pragma unroll
        for (int i = 0; i < N; ++i)
          mine = mine && p_update_vanishes(Lanes<V>::at(p, i), me[i], ve[i], sc, k.eps);
        vanish = __all(!act || mine);
      }
      skipping = vanish;
      if (!vanish && act) {
#pragma unroll
        for (int i = 0; i < N; ++i) {
          const float den = div_bc2s(sqrtf(ve[i]), sc) + k.eps;
          Lanes<V>::at(p, i) = Lanes<V>::at(p, i) + ((-sc.ss) * me[i]) / den;
        }
      }
      if (act) {
#pragma unroll
        for (int i = 0; i < N; ++i) {
          Lanes<V>::at(m, i) = me[i];
          Lanes<V>::at(v, i) = ve[i];
        }
      }
    }
  } else {
    V z;
    memset(&z, 0, sizeof(V));
    for (int s = lo; s < s1; ++s) {
      const StepConsts sc = step_consts(consts, s);
      if (s >= s0) adam_vec(p, m, v, z, sc, k);
    }
  }
}

// x / bc2_sqrt as div_bc2s for a finite x (the fast path: x = sqrt(v), v <= FLT_MAX).
__device__ __forceinline__ float div_bc2s_finite(float x, const StepConsts& sc) {
  const float q = x * sc.rbc;
  return fmaf(fmaf(-q, sc.bc2s, x), sc.rbc, q);
}

// Increments q = RN(RN(-ss*me) / den), den = RN(RN(sqrt(ve) / bc2s) + eps), of G
// consecutive zero-gradient steps x N elements. The fast path is computed for all
// G*N first and one wave vote on its range conditions decides (a branch per step
// would serialise the steps' chains); the library path recomputes everything.
// The range conditions are tested at the group's first and last step only: over
// consecutive zero-gradient steps ve (= RN(ve * b2)), |me| (= RN(me * (1-b1)),
// lerp_small), step_size (host table, non-increasing: FusedAdam.step_constants
// checks it) and so |num| and den (bc2s non-decreasing) never increase, and every
// operation involved is monotone, so the bounds at the two ends hold for the
// steps between them.
template <int G, int N>
__device__ __forceinline__ void incr_steps(const float (*me)[N], const float (*ve)[N],
                                           const StepConsts* sc, const AdamConsts& k,
                                           float (*q)[N]) {
  float num[G][N], den[G][N];
#pragma unroll
  for (int j = 0; j < G; ++j)
#pragma unroll
    for (int i = 0; i < N; ++i) {
      den[j][i] = div_bc2s_finite(sqrt_rn_normal(ve[j][i]), sc[j]) + k.eps;
      num[j][i] = (-sc[j].ss) * me[j][i];
    }
  int ok = 1;                                   // int: no short-circuit branches
#pragma unroll
  for (int i = 0; i < N; ++i)
    ok &= (int)(ve[0][i] <= 0x1.fffffep127f) & (int)(ve[G - 1][i] >= 0x1p-96f) &
          (int)(fabsf(num[0][i]) <= 0x1p40f) & (int)(fabsf(num[G - 1][i]) >= 0x1p-60f) &
          (int)(den[0][i] <= 0x1p40f) & (int)(den[G - 1][i] >= 0x1p-40f);
  if (__all(ok)) {
#pragma unroll
    for (int j = 0; j < G; ++j)
#pragma unroll
      for (int i = 0; i < N; ++i) q[j][i] = div_rn_normal(num[j][i], den[j][i]);
  } else {
#pragma unroll
    for (int j = 0; j < G; ++j)
#pragma unroll
      for (int i = 0; i < N; ++i)
        q[j][i] = num[j][i] / (div_bc2s(sqrtf(ve[j][i]), sc[j]) + k.eps);
  }
}

// ---- replay of a row that fills whole waves (s0 wave-uniform); the fast-path
// sqrt / division it uses live in adam_math.h.
// Zero-gradient replay of steps [s0, s1) (wd == 0, 1-b1 < 0.5) for a thread whose
// wave holds one row (s0 the same on every lane). Same per-element results as
// adam_elem_zero applied step by step.
//
// The loop-carried chain of a zero-gradient step is one fma (m) and one mul (v);
// the expensive part (sqrt, two divisions) depends on that step's m and v only,
// and p just accumulates the increments in step order. So steps go in groups of
// four: the m / v chain first, then the four increments side by side (four
// independent sqrt / division chains in flight instead of one), then the four
// additions to p in step order — the same operations and roundings as one step
// at a time. While every element's p update provably rounds away
// (p_update_vanishes; p is then fixed, so its exponent part is computed once)
// a group only moves m and v. The test runs at the first step of every group
// outside that state (as adam_replay's every 4th step); a group whose four steps
// do not all pass goes step by step. Full steps use the fast-path sqrt /
// division of adam_math.h.
template <typename V>
__device__ __forceinline__ void adam_replay_row(V& p, V& m, V& v, int s0, int s1,
                                                const float* __restrict__ consts,
                                                const AdamConsts& k) {
  constexpr int N = Lanes<V>::n;
  constexpr int G = 4;
  int s = __builtin_amdgcn_readfirstlane(s0);
  if (s >= s1) return;
  bool skipping = false;
  float scale[N];
  bool okp[N];
#pragma unroll
  for (int i = 0; i < N; ++i) { scale[i] = 0.f; okp[i] = false; }
  const bool eps_pos = k.eps > 0.f;
  float mc[N], vc[N], pc[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    mc[i] = Lanes<V>::at(m, i);
    vc[i] = Lanes<V>::at(v, i);
    pc[i] = Lanes<V>::at(p, i);
  }
  // vanishing test with p's exponent part precomputed (p fixed while skipping)
  auto fixed_p_vanish = [&](float me, float ve, const StepConsts& sc, int i) {
    const float t = (sc.kq * fabsf(me)) * scale[i];
    return (me == 0.f && eps_pos) || (okp[i] && ve >= 0x1p-100f && t * t < 0.999f * ve);
  };
  auto enter_skip = [&]() {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const uint32_t ex = (__float_as_uint(pc[i]) >> 23) & 0xffu;
      scale[i] = __uint_as_float((279u - ex) << 23);
      okp[i] = ex >= 67u && ex < 255u;
    }
  };
  // full increments of one step for every element: q = RN(RN(-ss*me) / den)
  auto incr = [&](const float* me, const float* ve, const StepConsts& sc, float* q) {
    incr_steps<1, N>(reinterpret_cast<const float(*)[N]>(me),
                     reinterpret_cast<const float(*)[N]>(ve), &sc, k,
                     reinterpret_cast<float(*)[N]>(q));
  };
  // one step, state machine of adam_replay (test every step while skipping,
  // else at `test`)
  auto one_step = [&](const float* me, const float* ve, const StepConsts& sc, bool test) {
    bool vanish = false;
    if (skipping) {
      bool mine = true;
#pragma unroll
      for (int i = 0; i < N; ++i) mine = mine && fixed_p_vanish(me[i], ve[i], sc, i);
      vanish = __all(mine);
    } else if (test) {
      bool mine = true;
#pragma unroll
      for (int i = 0; i < N; ++i)
        mine = mine && p_update_vanishes(pc[i], me[i], ve[i], sc, k.eps);
      vanish = __all(mine);
      if (vanish) enter_skip();
    }
    if (!vanish) {
      float q[N];
      incr(me, ve, sc, q);
#pragma unroll
      for (int i = 0; i < N; ++i) pc[i] = pc[i] + q[i];
    }
    skipping = vanish;
  };

  // (loading the next group's step constants under this group's arithmetic was
  // measured slower: the scalar-load wait covers both groups' loads)
  for (; s + G <= s1; s += G) {
    StepConsts sc[G];
#pragma unroll
    for (int j = 0; j < G; ++j) sc[j] = step_consts(consts, s + j);
    float me[G][N], ve[G][N];
#pragma unroll
    for (int j = 0; j < G; ++j) {
#pragma unroll
      for (int i = 0; i < N; ++i) {
        me[j][i] = fmaf(-k.omb1, mc[i], mc[i]);
        ve[j][i] = vc[i] * k.b2;
        mc[i] = me[j][i];
        vc[i] = ve[j][i];
      }
    }
    bool group_done = false;
    if (skipping) {
      bool mine = true;
#pragma unroll
      for (int j = 0; j < G; ++j)
#pragma unroll
        for (int i = 0; i < N; ++i) mine = mine && fixed_p_vanish(me[j][i], ve[j][i], sc[j], i);
      group_done = __all(mine);                 // four skipped steps
    } else {
      bool mine = true;
#pragma unroll
      for (int i = 0; i < N; ++i)
        mine = mine && p_update_vanishes(pc[i], me[0][i], ve[0][i], sc[0], k.eps);
      if (!__all(mine)) {                       // four full steps, increments side by side
        float q[G][N];
        incr_steps<G, N>(me, ve, sc, k, q);
#pragma unroll
        for (int j = 0; j < G; ++j)
#pragma unroll
          for (int i = 0; i < N; ++i) pc[i] = pc[i] + q[j][i];
        group_done = true;
      }
    }
    if (!group_done) {                          // a transition: step by step
#pragma unroll
      for (int j = 0; j < G; ++j) one_step(me[j], ve[j], sc[j], j == 0);
    }
  }
  for (int j = 0; s < s1; ++s, ++j) {           // the last s1 - s < 4 steps
    const StepConsts sc = step_consts(consts, s);
    float me[N], ve[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      me[i] = fmaf(-k.omb1, mc[i], mc[i]);
      ve[i] = vc[i] * k.b2;
      mc[i] = me[i];
      vc[i] = ve[i];
    }
    one_step(me, ve, sc, j == 0);
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    Lanes<V>::at(m, i) = mc[i];
    Lanes<V>::at(v, i) = vc[i];
    Lanes<V>::at(p, i) = pc[i];
  }
}

// Replay dispatch: whole-wave rows in the common configuration take
// adam_replay_row, everything else the general adam_replay.
template <typename V, bool kRowWave>
__device__ __forceinline__ void replay(V& p, V& m, V& v, int s0, int s1,
                                       const float* __restrict__ consts, const AdamConsts& k) {
  if (kRowWave && k.wd == 0.f && k.lerp_small)
    adam_replay_row(p, m, v, s0, s1, consts, k);
  else
    adam_replay(p, m, v, s0, s1, consts, k);
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
__device__ __forceinline__ void vadd<float2>(float2& a, const float2& b) {
  a.x += b.x; a.y += b.y;
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
// V = float or float2 columns per thread. A row's replay is a serial chain per
// element; a launch with few rows (one 512-positive batch: a few waves per SIMD)
// takes as long as its longest chain, so one column per lane (shortest chains);
// a launch with many rows (a data-parallel global batch) is issue-bound, so two
// (half the per-wave overhead). The host picks by the launch's row bound.
// RPB = 256 / (D / |V|) whole rows per block.
//  segment 2q   (touched): row = uniq[u] of table q. Replays last..s-1 with a
//               zero gradient, applies step s with its gradient; last = s+1.
//  segment 2q+1 (look-ahead): row = ahead_uniq[u], rows the NEXT batch reads
//               and this one does not touch (the caller's set difference).
//               Replays last..s (zero gradient); last = s+1 — so the next
//               forward pass reads rows that are complete through step s.
// `last` is read by every thread of a row before the barrier and written
// after it (a row of D = 256 spans two waves).
// Block of the deferred kernel: one row when a row fills whole waves, else one
// wave of rows. Small blocks: the launch's rows differ widely in replay length,
// and a CU takes a new block only when a whole block's waves are free.
__host__ __device__ constexpr int deferred_block(int vpr) { return vpr > 64 ? vpr : 64; }

template <int D, typename V>
__global__ __launch_bounds__(kAdamThreads) void adam_deferred_kernel(
    const AdamTables tabs, const float* __restrict__ consts,
    const int32_t* __restrict__ step_base, int step_off, AdamConsts k) {
  constexpr int VPR = D / Lanes<V>::n;              // V = float or float2 per thread
  constexpr int RPB = deferred_block(VPR) / VPR;    // rows per block
  static_assert(deferred_block(VPR) % VPR == 0, "row width");
  const int si = segment_of(tabs, blockIdx.x);
  const mirec_adam_table& T = tabs.t[si >> 1];
  const bool ahead = si & 1;
  const int u = (int)(((int64_t)blockIdx.x - tabs.block_start[si]) * RPB) + threadIdx.x / VPR;
  const int c = threadIdx.x % VPR;
  // Dependent-load chain kept to three levels: (count, row id) -> (last, p, m,
  // v, the row's gradient contributions) -> replay + step. The block barrier
  // that orders every thread's read of `last` before the row's write sits at
  // the end, so no thread leaves early.
  const int n = ahead ? T.ahead_n_uniq[0] : T.n_uniq[0];
  // the grid is sized for the host's bound on the lists: blocks past the actual
  // count leave at once (block-uniform: no thread reaches the barrier below)
  if ((int)(((int64_t)blockIdx.x - tabs.block_start[si]) * RPB) >= n) return;
  const int st = step_base[0] + step_off;
  const bool valid = u < n;
  int64_t row = 0;
  int last = st;
  bool idle = !valid;   // nothing to load or store: outside the list, or a look-ahead
                        // row in the zero state (already current for every step)
  V p, m, v, g;
  memset(&p, 0, sizeof(V)); m = p; v = p; g = p;
  if (valid) {
    row = ahead ? T.ahead_uniq[u] : T.uniq[u];
    const int64_t off = row * VPR + c;
    const int raw = T.last[row];
    last = raw == kZeroState ? st : raw;
    idle = ahead && raw == kZeroState;
    if (!idle) {
      p = reinterpret_cast<const V*>(T.p)[off];
      m = reinterpret_cast<const V*>(T.m)[off];
      v = reinterpret_cast<const V*>(T.v)[off];
      if (!ahead) g = grouped_grad<V>(T, u, VPR, c);
    }
  }
  // the zero-gradient steps it skipped (all lanes take part: wave-uniform loop);
  // a row already complete through st (last > st: a repeated look-ahead of the
  // same step) is left as it is
  replay<V, (VPR >= 64)>(p, m, v, idle ? st : last, st, consts, k);
  const bool fresh = !idle && last <= st;
  if (fresh) adam_vec(p, m, v, g, step_consts(consts, st), k);
  __syncthreads();
  if (!valid || !fresh) return;
  const int64_t off = row * VPR + c;
  reinterpret_cast<V*>(T.p)[off] = p;
  reinterpret_cast<V*>(T.m)[off] = m;
  reinterpret_cast<V*>(T.v)[off] = v;
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
  // wave-uniform trip count (adam_replay's step loop runs over the whole wave)
  for (int64_t base = lo; base < hi; base += RPP) {
    const int64_t r = base + rsub;
    const bool valid = r < hi;
    const int last = valid ? min(T.last[r], target) : target;
    const bool work = last < target;
    const int64_t off = r * VPR + c;
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f), m = p, v = p;
    if (work) {
      p = reinterpret_cast<const float4*>(T.p)[off];
      m = reinterpret_cast<const float4*>(T.m)[off];
      v = reinterpret_cast<const float4*>(T.v)[off];
    }
    adam_replay(p, m, v, last, target, consts, k);
    if (work) {
      reinterpret_cast<float4*>(T.p)[off] = p;
      reinterpret_cast<float4*>(T.m)[off] = m;
      reinterpret_cast<float4*>(T.v)[off] = v;
      if (c == 0) T.last[r] = target;  // a row lies in one wave here (VPR <= 64)
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
  const int last = __builtin_amdgcn_readfirstlane(min(T.last[r], target));
  if (last >= target) return;
  const int64_t off = r * 64 + (threadIdx.x & 63);
  V p = reinterpret_cast<const V*>(T.p)[off];
  V m = reinterpret_cast<const V*>(T.m)[off];
  V v = reinterpret_cast<const V*>(T.v)[off];
  replay<V, true>(p, m, v, last, target, consts, k);
  reinterpret_cast<V*>(T.p)[off] = p;
  reinterpret_cast<V*>(T.m)[off] = m;
  reinterpret_cast<V*>(T.v)[off] = v;
  if ((threadIdx.x & 63) == 0) T.last[r] = target;
}

// Flush of a width-1 table (DeepFM's first-order [V, 1] weights): one row per
// lane; the rows of a wave lag by different step counts, so the general replay
// (wave-uniform step loop from the wave's smallest count, lanes active from their
// own) applies.
__global__ __launch_bounds__(kAdamThreads) void adam_flush_scalar_kernel(
    const AdamTables tabs, const float* __restrict__ consts, const int32_t* __restrict__ step_base,
    int step_off, AdamConsts k) {
  const int si = segment_of(tabs, blockIdx.x);
  const mirec_adam_table& T = tabs.t[si];
  const int64_t r = ((int64_t)blockIdx.x - tabs.block_start[si]) * kAdamThreads + threadIdx.x;
  const int target = step_base[0] + step_off;
  const bool valid = r < T.n_rows;
  const int last = valid ? min(T.last[r], target) : target;
  if (__all(last >= target)) return;
  float p = 0.f, m = 0.f, v = 0.f;
  if (last < target) {
    p = T.p[r];
    m = T.m[r];
    v = T.v[r];
  }
  adam_replay(p, m, v, last, target, consts, k);
  if (last < target) {
    T.p[r] = p;
    T.m[r] = m;
    T.v[r] = v;
    T.last[r] = target;
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
  if (d != 4 && d != 16 && d != 32 && d != 64 && d != 128 && d != 256 &&
      !(d == 1 && sched != Sched::kStreamed)) {
    set_error("%s: row width %d not in {4,16,32,64,128,256} (1: deferred / flush)", what, d);
    return -1;
  }
  const int VPR = d / 4;
  AdamTables tabs;
  memset(&tabs, 0, sizeof(tabs));
  const bool deferred = sched == Sched::kDeferred;
  tabs.n_seg = deferred ? 2 * n_tables : n_tables;
  // deferred: float columns per thread while the launch fits ~16 waves per SIMD
  int dvec = 1;
  if (deferred && n_max_uniq && d >= 4) {
    int64_t waves = 0;
    for (int q = 0; q < n_tables; ++q)
      if (n_max_uniq[q] > 0)
        waves += n_max_uniq[q] * (tables[q].ahead_uniq ? 2 : 1) * ((d + 63) / 64);
    if (waves > 16 * 1024) dvec = 2;
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
    tabs.t[q] = t;
    if (deferred) {
      const int rpb = deferred_block(d / dvec) / (d / dvec);
      const int64_t nb = (n_max_uniq[q] + rpb - 1) / rpb;
      tabs.block_start[2 * q] = blocks;
      blocks += nb;
      tabs.block_start[2 * q + 1] = blocks;
      if (t.ahead_uniq) blocks += nb;
    } else {
      tabs.block_start[q] = blocks;
      const int64_t rows_per_block = d == 1 ? kAdamThreads
                                     : (sched == Sched::kFlush && d >= 64) ? kFlushRowThreads / 64
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
    else if (deferred)                                                                       \
      hipLaunchKernelGGL((dvec == 2 ? adam_deferred_kernel<DD, float2>                       \
                                    : adam_deferred_kernel<DD, float>),                      \
                         grd, dim3(deferred_block(DD / dvec)), 0, st, tabs, consts,          \
                         step_base, step_off, k);                                            \
    else if (DD >= 64)                                                                       \
      hipLaunchKernelGGL(adam_flush_row_kernel<(DD >= 64 ? DD : 64)>, grd,                   \
                         dim3(kFlushRowThreads), 0, st, tabs,                                \
                         consts, step_base, step_off, k);                                    \
    else                                                                                     \
      hipLaunchKernelGGL(adam_flush_kernel<DD>, grd, blk, 0, st, tabs, consts, step_base,    \
                         step_off, k);                                                       \
    break;
  switch (d) {
    case 1:
      if (deferred)
        hipLaunchKernelGGL((adam_deferred_kernel<1, float>), grd, dim3(deferred_block(1)), 0, st,
                           tabs, consts, step_base, step_off, k);
      else
        hipLaunchKernelGGL(adam_flush_scalar_kernel, grd, blk, 0, st, tabs, consts, step_base,
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

}  // namespace mirec

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
