// K35 — the whole model side of one C2 training step in ONE launch: BPR forward +
// backward (K3's arithmetic) and the deferred dense-Adam step (K5's arithmetic) of
// every touched row, plus the look-ahead replays — without gradient rows in HBM and
// without the K3 -> K5 kernel boundary.
//
// Reference: BPR.calculate_loss (bpr.py:74-83) + BPRLoss (loss.py:43-49), the
// nn.Embedding backward (index_add into a dense gradient) and optim.Adam.step over
// every row (trainer.py:157-174; torch optim/adam.py _single_tensor_adam).
//
// Who computes what. K3 formed one gradient row per contribution (per positive for the
// user table, per pos / neg slot for the item table) and K5 summed them per table row
// in the K2 grouping's order. Here the OWNER of a touched row forms its own
// contributions: for each one it gathers the rows of that contribution's positive
// (u, p, the T negatives), recomputes the scores and coefficients with K3's exact
// arithmetic (bpr_math.h; same lane layout, same reductions), builds the contribution
// vector, and the block adds them in grouping order and applies the Adam step — the
// same sums and the same bits as K3 + K5. The scores of a positive are recomputed by
// each of its rows' owners (≈ 3x the dot products, ≈ 4x the row reads of K3; the rows
// sit in L2 / MALL: 2.5 MB of a batch's rows against 84.6 MB tables).
//
// Parity double buffer. A touched row's new p cannot overwrite the row other blocks
// are reading as a partner in the same launch, so p lives in two buffers: the state
// after t applied steps is in P[t & 1]. Step s reads partners (and its own rows) from
// P[s & 1] — every row a step reads is complete through s - 1 (look-ahead of step s-1,
// the chunk entry catch-up, or a flush) — and writes the touched and look-ahead rows
// at state s + 1 into P[(s + 1) & 1]. m and v are private to a row's owner: one
// buffer. Zero-state rows (never updated, adam.hip) are valid in both buffers (the
// caller copies P[0] to P[1] when it marks them). mirec_adam_flush_f32 with p_alt set
// completes every row into P[t & 1] and, for an odd t, also into P[0] (the parameter).
//
// Block = one table row, one element per thread (D threads, D in {64, 128, 256}).
// Touched rows: the block's D/4-lane groups take the row's contributions in turn
// (float4 slices, K3's layout), write them to LDS; every thread adds its element of
// each contribution in order, then replays (if behind) and applies the step.
// Look-ahead rows: the deferred kernel's replay of steps last..s.
#include "adam_core.h"
#include "bpr_math.h"

namespace mirec {

struct StepLaunch {
  mirec_adam_table t[2];       // [0] users, [1] items: p (+ p_alt), m, v, last, grouping
  int64_t block_start[5];      // segments: ahead U, ahead I, touched U, touched I, end
};

// rows of one contribution of the positive k: u = EU[user[k]], p = EI[items[k]],
// n_j = EI[items[Bc + j*Bc + k]] (ids clamped as K3 clamps them)
__device__ __forceinline__ int64_t clamp_id(int64_t id, int64_t n) {
  return id < 0 ? 0 : (id >= n ? n - 1 : id);
}

template <int D>
__global__ __launch_bounds__(D) void bpr_adam_step_kernel(
    const StepLaunch L, const int64_t* __restrict__ user, const int64_t* __restrict__ items,
    int64_t Bc, int T, float gamma, float grad_scale, float* __restrict__ loss_k,
    const float* __restrict__ consts, const int32_t* __restrict__ step_base, int step_off,
    AdamConsts k) {
  constexpr int LPR = D / 4;               // lanes per contribution (float4 each)
  constexpr int NG = D / LPR;              // contribution groups per block (4)
  __shared__ float cont[NG][D];
  int si = 0;
#pragma unroll
  for (int q = 1; q < 4; ++q)
    if ((int64_t)blockIdx.x >= L.block_start[q]) si = q;
  const bool ahead = si < 2;
  const int tb = si & 1;                   // 0 users, 1 items
  const mirec_adam_table& T_ = L.t[tb];
  const int u = (int)((int64_t)blockIdx.x - L.block_start[si]);
  const int n = ahead ? T_.ahead_n_uniq[0] : T_.n_uniq[0];
  if (u >= n) return;                      // block-uniform
  const int st = step_base[0] + step_off;
  const int t = threadIdx.x;
  const float* __restrict__ Pr[2] = {T_.p, T_.p_alt};
  float* __restrict__ Pw = ((st + 1) & 1) ? T_.p_alt : T_.p;
  const int64_t row = ahead ? T_.ahead_uniq[u] : T_.uniq[u];
  const int raw = T_.last[row];

  if (ahead) {
    // rows the next step reads and this one does not touch: replay last..st (zero
    // gradient), as adam_deferred_kernel's look-ahead segment
    if (raw == kZeroState || raw > st) return;    // current at every step / already done
    const int64_t off = row * D + t;
    float p = Pr[raw & 1][off], m = T_.m[off], v = T_.v[off];
    replay<float, (D >= 64)>(p, m, v, raw, st, consts, k);
    adam_elem(p, m, v, 0.f, step_consts(consts, st), k);   // step st: zero gradient
    __syncthreads();                               // every thread read `last`
    Pw[off] = p;
    T_.m[off] = m;
    T_.v[off] = v;
    if (t == 0) T_.last[row] = st + 1;
    return;
  }

  // ---- touched row: contributions in grouping order -> gradient element t
  const float* __restrict__ EU = L.t[0].p;         // partner rows at state st
  const float* __restrict__ EI = L.t[1].p;
  if (st & 1) {
    EU = L.t[0].p_alt;
    EI = L.t[1].p_alt;
  }
  const int64_t nU = L.t[0].n_rows, nI = L.t[1].n_rows;
  const int i0 = T_.seg[u], i1 = T_.seg[u + 1];
  const int grp = t / LPR;
  const int l = t - grp * LPR;
  const float ng = -grad_scale;
  float g = 0.f;
  for (int base = i0; base < i1; base += NG) {
    const int i = base + grp;
    if (i < i1) {
      const int q = T_.perm[i];                     // contribution index
      // the positive of this contribution and, for a negative slot, which negative
      int64_t kk;
      int jn = -1;
      if (tb == 0 || q < Bc) {
        kk = q;
      } else {
        const int64_t r = q - Bc;
        jn = (int)(r / Bc);
        kk = r - (int64_t)jn * Bc;
      }
      const int64_t uid = clamp_id(user[kk], nU);
      const int64_t pid = clamp_id(items[kk], nI);
      const float4 uv = reinterpret_cast<const float4*>(EU + uid * D)[l];
      const float4 pv = reinterpret_cast<const float4*>(EI + pid * D)[l];
      const float sp = group_sum<LPR>(dot4(uv, pv));
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      if (jn >= 0) {                                  // item row as the negative jn
        const int64_t nid = clamp_id(items[Bc + (int64_t)jn * Bc + kk], nI);
        const float4 nv = reinterpret_cast<const float4*>(EI + nid * D)[l];
        const float sn = group_sum<LPR>(dot4(uv, nv));
        acc = contrib_n(bpr_coef(sp, sn, gamma, ng).dx, uv);
      } else {                                        // user row, or item row as the positive
        float lsum = 0.f;
        for (int j0 = 0; j0 < T; j0 += 4) {
          float4 nv[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int j = j0 + e;
            nv[e] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (j < T) {
              const int64_t nid = clamp_id(items[Bc + (int64_t)j * Bc + kk], nI);
              nv[e] = reinterpret_cast<const float4*>(EI + nid * D)[l];
            }
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int j = j0 + e;
            if (j < T) {
              const float sn = group_sum<LPR>(dot4(uv, nv[e]));
              const BprCoef cf = bpr_coef(sp, sn, gamma, ng);
              lsum += cf.nll;
              if (tb == 0)
                contrib_u(acc, cf.dx, pv, nv[e]);
              else
                contrib_p(acc, cf.dx, uv);
            }
          }
        }
        if (tb == 0 && l == 0 && loss_k) loss_k[kk] = lsum;   // one user slot per positive
      }
      cont[grp][4 * l + 0] = acc.x;
      cont[grp][4 * l + 1] = acc.y;
      cont[grp][4 * l + 2] = acc.z;
      cont[grp][4 * l + 3] = acc.w;
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < NG; ++h)
      if (base + h < i1) g += cont[h][t];
    __syncthreads();                                 // cont is rewritten next round
  }

  // ---- Adam step of the row (replaying skipped zero-gradient steps first)
  const int64_t off = row * D + t;
  const int last = raw == kZeroState ? st : raw;
  float p = Pr[last & 1][off], m = T_.m[off], v = T_.v[off];
  replay<float, (D >= 64)>(p, m, v, last, st, consts, k);
  const bool fresh = last <= st;
  if (fresh) adam_elem(p, m, v, g, step_consts(consts, st), k);
  __syncthreads();
  if (!fresh) return;
  Pw[off] = p;
  T_.m[off] = m;
  T_.v[off] = v;
  if (t == 0) T_.last[row] = st + 1;
}

}  // namespace mirec

using namespace mirec;

extern "C" int mirec_bpr_adam_step_f32(const mirec_adam_table* tables,
                                       const int64_t* n_max_uniq, int32_t d,
                                       const int64_t* user, const int64_t* items, int64_t Bc,
                                       int32_t T, float gamma, float grad_scale, float* loss_k,
                                       const float* step_consts_dev,
                                       const int32_t* step_base_dev, int32_t step_off,
                                       double beta1, double beta2, double eps,
                                       double weight_decay, void* stream) {
  const char* what = "mirec_bpr_adam_step_f32";
  if (!tables || !n_max_uniq || !user || !items || Bc < 0 || T < 1 || !step_consts_dev ||
      !step_base_dev || ((uintptr_t)step_consts_dev & 15) != 0) {
    set_error("%s: bad arguments", what);
    return -1;
  }
  if (d != 64 && d != 128 && d != 256) {
    set_error("%s: embedding_size %d not in {64,128,256}", what, d);
    return -1;
  }
  StepLaunch L;
  memset(&L, 0, sizeof(L));
  for (int q = 0; q < 2; ++q) {
    const mirec_adam_table& t = tables[q];
    if (!t.p || !t.p_alt || !t.m || !t.v || !t.last || !t.uniq || !t.seg || !t.perm ||
        !t.n_uniq || t.n_rows <= 0 || n_max_uniq[q] < 0 || t.dense_grad ||
        (t.ahead_uniq == nullptr) != (t.ahead_n_uniq == nullptr)) {
      set_error("%s: bad table %d", what, q);
      return -1;
    }
    L.t[q] = t;
  }
  // segments: look-ahead rows first (their replays are the longest chains), then touched
  int64_t b = 0;
  L.block_start[0] = b;
  b += L.t[0].ahead_uniq ? n_max_uniq[0] : 0;
  L.block_start[1] = b;
  b += L.t[1].ahead_uniq ? n_max_uniq[1] : 0;
  L.block_start[2] = b;
  b += n_max_uniq[0];
  L.block_start[3] = b;
  b += n_max_uniq[1];
  L.block_start[4] = b;
  if (b == 0) return 0;
  AdamConsts k;
  k.omb1 = (float)(1.0 - beta1);
  k.omb1m1 = k.omb1 - 1.0f;
  k.lerp_small = fabsf(k.omb1) < 0.5f;
  k.b2 = (float)beta2;
  k.omb2 = (float)(1.0 - beta2);
  k.eps = (float)eps;
  k.wd = (float)weight_decay;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grd((unsigned)b);
#define MIREC_STEP_CASE(DD)                                                                  \
  case DD:                                                                                   \
    hipLaunchKernelGGL(bpr_adam_step_kernel<DD>, grd, dim3(DD), 0, st, L, user, items, Bc, T, \
                       gamma, grad_scale, loss_k, step_consts_dev, step_base_dev, step_off, k); \
    break;
  switch (d) {
    MIREC_STEP_CASE(64)
    MIREC_STEP_CASE(128)
    MIREC_STEP_CASE(256)
  }
#undef MIREC_STEP_CASE
  return launch_status(what);
}
