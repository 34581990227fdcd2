// K5 device arithmetic shared by the Adam kernels (adam.hip) and the fused BPR step
// (step.hip): torch's per-element Adam step, the zero-gradient replay engines and the
// grouped-gradient sum. Header comment of adam.hip: the arithmetic contract.
#pragma once
#include "common.h"
#include "adam_math.h"

// No FMA contraction: every op rounds on its own, as in torch's op-by-op
// _single_tensor_adam, and the streamed / deferred schedules stay bit-identical
// whatever the compiler could fuse in either context.
#pragma clang fp contract(off)

namespace mirec {

// Executed-work counters (diagnostic build only: tools/build_variant.sh work
// -DMIREC_STEP_COUNT; tools/probe_step_work.py). Element-steps actually executed, by
// kind, so a roofline can be put on the work done rather than on the dense formula:
// [0] zero-gradient steps with the p update, [1] vanishing steps (m, v only), [2]
// gradient steps, [3] the look-ahead's own zero-gradient step, [4] touched rows stepped,
// [5] look-ahead row halves replayed, [6..8] contributions formed (user row / item as
// positive / item as negative), [9] split-row participants, [10] flush rows replayed.
// Each translation unit has its own copy (read by its mirec_work_counters*).
#if defined(MIREC_STEP_COUNT)
static __device__ unsigned long long g_work[16];
#define MIREC_WORK(i, n)                                                                  \
  do {                                                                                    \
    const uint64_t act_ = __ballot(1);                                                    \
    if ((int)(threadIdx.x & 63) == __ffsll((unsigned long long)act_) - 1)                 \
      atomicAdd(&g_work[(i)], (unsigned long long)(n));                                   \
  } while (0)
#define MIREC_WORK_LANES() ((unsigned long long)__popcll(__ballot(1)))
#else
#define MIREC_WORK(i, n) do {} while (0)
#define MIREC_WORK_LANES() 0ull
#endif

constexpr int kAdamThreads = 256;
constexpr int kAdamRows = 64;  // table rows per block (streamed)
// Flush of narrow rows (d < 64, d = 1; adam_flush_list_kernel): rows per block (their
// `last` marks are read in one pass, the lagging ones listed in LDS)
constexpr int kFlushRows = 1024;
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
// The fast-path increments two at a time on gfx950's packed fp32 pipe (v_pk_fma_f32 /
// v_pk_mul_f32 / v_pk_add_f32: two IEEE fp32 operations per lane and instruction, each
// rounded as its scalar form), for G*N independent (step, element) pairs. Same operations,
// same roundings, same order per value as sqrt_rn_normal / div_bc2s_finite / div_rn_normal.
typedef float mirec_f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ mirec_f2 pk_fma(mirec_f2 a, mirec_f2 b, mirec_f2 c) {
  return __builtin_elementwise_fma(a, b, c);
}

// q = RN(RN(-ss*me) / den), den = RN(RN(RN(sqrt(ve)) / bc2s) + eps), for two pairs at once
// (each pair with its own step constants)
__device__ __forceinline__ mirec_f2 incr_pair(mirec_f2 me, mirec_f2 ve, mirec_f2 ss,
                                              mirec_f2 bc2s, mirec_f2 rbc, float eps) {
  // sqrt_rn_normal, component-wise selects
  const mirec_f2 s = {__builtin_amdgcn_sqrtf(ve.x), __builtin_amdgcn_sqrtf(ve.y)};
  const mirec_f2 sd = {__uint_as_float(__float_as_uint(s.x) - 1u),
                       __uint_as_float(__float_as_uint(s.y) - 1u)};
  const mirec_f2 su = {__uint_as_float(__float_as_uint(s.x) + 1u),
                       __uint_as_float(__float_as_uint(s.y) + 1u)};
  const mirec_f2 rd = pk_fma(-sd, s, ve);
  const mirec_f2 ru = pk_fma(-su, s, ve);
  mirec_f2 sq;
  sq.x = ru.x > 0.f ? su.x : (rd.x <= 0.f ? sd.x : s.x);
  sq.y = ru.y > 0.f ? su.y : (rd.y <= 0.f ? sd.y : s.y);
  // div_bc2s_finite + eps
  const mirec_f2 q = sq * rbc;
  const mirec_f2 den = pk_fma(pk_fma(-q, bc2s, sq), rbc, q) + (mirec_f2){eps, eps};
  // div_rn_normal(-ss * me, den)
  const mirec_f2 a = (-ss) * me;
  const mirec_f2 y0 = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
  const mirec_f2 one = {1.0f, 1.0f};
  const mirec_f2 e = pk_fma(-den, y0, one);
  const mirec_f2 y = pk_fma(e, y0, y0);
  const mirec_f2 q0 = a * y;
  const mirec_f2 r0 = pk_fma(-den, q0, a);
  const mirec_f2 q1 = pk_fma(r0, y, q0);
  const mirec_f2 r1 = pk_fma(-den, q1, a);
  return pk_fma(r1, y, q1);
}

template <int G, int N>
__device__ __forceinline__ void incr_steps(const float (*me)[N], const float (*ve)[N],
                                           const StepConsts* sc, const AdamConsts& k,
                                           float (*q)[N]) {
  float num[G][N], den[G][N];
  // range conditions at the group's first and last step (see below); the values they
  // test are recomputed in the paired path exactly as here
#pragma unroll
  for (int j = 0; j < G; j += (G > 1 ? G - 1 : 1))
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
    constexpr int NE = G * N;
#if defined(MIREC_NO_PK)                        // probe build: the scalar form
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const int j = e / N, i = e % N;
      q[j][i] = div_rn_normal((-sc[j].ss) * me[j][i],
                              div_bc2s_finite(sqrt_rn_normal(ve[j][i]), sc[j]) + k.eps);
    }
    return;
#endif
#pragma unroll
    for (int e = 0; e + 1 < NE; e += 2) {
      const int ja = e / N, ia = e % N, jb = (e + 1) / N, ib = (e + 1) % N;
      const mirec_f2 r = incr_pair((mirec_f2){me[ja][ia], me[jb][ib]},
                                   (mirec_f2){ve[ja][ia], ve[jb][ib]},
                                   (mirec_f2){sc[ja].ss, sc[jb].ss},
                                   (mirec_f2){sc[ja].bc2s, sc[jb].bc2s},
                                   (mirec_f2){sc[ja].rbc, sc[jb].rbc}, k.eps);
      q[ja][ia] = r.x;
      q[jb][ib] = r.y;
    }
    if (NE & 1) {                               // an odd count: the last one alone
      constexpr int jl = (NE - 1) / N, il = (NE - 1) % N;
      const float dl = div_bc2s_finite(sqrt_rn_normal(ve[jl][il]), sc[jl]) + k.eps;
      q[jl][il] = div_rn_normal((-sc[jl].ss) * me[jl][il], dl);
    }
  } else {
#pragma unroll
    for (int j = 0; j < G; ++j)
#pragma unroll
      for (int i = 0; i < N; ++i)
        q[j][i] = ((-sc[j].ss) * me[j][i]) / (div_bc2s(sqrtf(ve[j][i]), sc[j]) + k.eps);
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
// division of adam_math.h. G = steps per group (8: eight chains in flight for a
// thread holding one element).
template <typename V, int G = 4>
__device__ __forceinline__ void adam_replay_row(V& p, V& m, V& v, int s0, int s1,
                                                const float* __restrict__ consts,
                                                const AdamConsts& k) {
  constexpr int N = Lanes<V>::n;
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
    MIREC_WORK(vanish ? 1 : 0, N * MIREC_WORK_LANES());
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
      if (group_done) MIREC_WORK(1, G * N * MIREC_WORK_LANES());
    } else {
      bool mine = true;
#pragma unroll
      for (int i = 0; i < N; ++i)
        mine = mine && p_update_vanishes(pc[i], me[0][i], ve[0][i], sc[0], k.eps);
      if (!__all(mine)) {                       // four full steps, increments side by side
        float q[G][N];
        incr_steps<G, N>(me, ve, sc, k, q);
        MIREC_WORK(0, G * N * MIREC_WORK_LANES());
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
  for (int j = 0; s < s1; ++s, ++j) {           // the last s1 - s < G steps
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
template <typename V, bool kRowWave, int G = 4>
__device__ __forceinline__ void replay(V& p, V& m, V& v, int s0, int s1,
                                       const float* __restrict__ consts, const AdamConsts& k) {
  if (kRowWave && k.wd == 0.f && k.lerp_small)
    adam_replay_row<V, G>(p, m, v, s0, s1, consts, k);
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

// One entry of the deferred schedule (adam.hip adam_deferred_kernel; comm.hip's
// exchange form): lane c of entry u of table T's touched list (ahead = false) or
// look-ahead list (ahead = true), n entries in the list, step st.
//  touched:    row = uniq[u]. Replays last..st-1 with a zero gradient, applies step st
//              with its gradient; last = st+1.
//  look-ahead: row = ahead_uniq[u], a row the NEXT batch reads and this one does not
//              touch. Replays last..st (zero gradient); last = st+1 — so the next
//              forward pass reads rows that are complete through step st.
// `last` is read by every thread of a row before the barrier and written after it (a
// row of VPR > 64 lanes spans waves: every thread of the block calls this together).
// done(valid, loaded, row, p): after the row's stores, p = the row's state through
// st+1 when loaded (false: an idle zero-state row, p not read).
template <int D, typename V, typename Done>
__device__ __forceinline__ void deferred_row(const mirec_adam_table& T, bool ahead, int u, int n,
                                             int st, const float* __restrict__ consts,
                                             const AdamConsts& k, int c, Done&& done) {
  constexpr int VPR = D / Lanes<V>::n;
  // Dependent-load chain kept to three levels: (count, row id) -> (last, p, m, v, the
  // row's gradient contributions) -> replay + step.
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
      // parity buffers (p_alt): the row's state `last` lives in last & 1 ? p_alt : p
      const float* src = (T.p_alt && (last & 1)) ? T.p_alt : T.p;
      p = reinterpret_cast<const V*>(src)[off];
      m = reinterpret_cast<const V*>(T.m)[off];
      v = reinterpret_cast<const V*>(T.v)[off];
      if (!ahead) g = grouped_grad<V>(T, u, VPR, c);
    }
  }
  // the zero-gradient steps it skipped (all lanes take part: wave-uniform loop); a row
  // already complete through st (last > st: a repeated look-ahead of the same step) is
  // left as it is
  replay<V, (VPR >= 64)>(p, m, v, idle ? st : last, st, consts, k);
  const bool fresh = !idle && last <= st;
  if (fresh) adam_vec(p, m, v, g, step_consts(consts, st), k);
  if (VPR > 64) __syncthreads();     // a row spans waves; else the row's lanes are one wave's
  if (valid && fresh) {
    const int64_t off = row * VPR + c;
    reinterpret_cast<V*>((T.p_alt && ((st + 1) & 1)) ? T.p_alt : T.p)[off] = p;
    reinterpret_cast<V*>(T.m)[off] = m;
    reinterpret_cast<V*>(T.v)[off] = v;
    if (c == 0) T.last[row] = st + 1;
  }
  done(valid, !idle, row, p);
}

}  // namespace mirec
