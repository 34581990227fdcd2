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
// Block = one table row (D in {64, 128, 256}). Touched rows: the block's D/4-lane groups
// take the row's contributions in turn (float4 slices, K3's layout), write them to LDS;
// every thread adds its elements of each contribution in order, then replays (if
// behind) and applies the step. Look-ahead rows: the deferred kernel's replay of steps
// last..s. Per element the arithmetic is adam_deferred_kernel's (adam_core.h), whatever
// the number of elements a thread holds.
#include "adam_core.h"
#include "bpr_math.h"

namespace mirec {

struct StepLaunch {
  mirec_adam_table t[2];       // [0] users, [1] items: p (+ p_alt), m, v, last, grouping
  const int32_t* rec[2];       // row records per touched-row slot (mirec_step_records)
  const int32_t* crec[2];      // contribution records per grouped position
  int64_t block_start[5];      // segments: ahead U, ahead I, touched U, touched I, end
};

// rows of one contribution of the positive k: u = EU[user[k]], p = EI[items[k]],
// n_j = EI[items[Bc + j*Bc + k]] (ids clamped as K3 clamps them)
__device__ __forceinline__ int64_t clamp_id(int64_t id, int64_t n) {
  return id < 0 ? 0 : (id >= n ? n - 1 : id);
}

// Block = one table row, EPT elements per thread (float for D = 64, float2 for D >= 128:
// one wave per row at D = 128, so a step's ~6,000 row blocks are resident at once and
// the look-ahead replays overlap the touched rows' gather chains).
// Diagnostic build only (tools/build_variant.sh step_stamps -DMIREC_STEP_STAMPS,
// tools/probe_step_stamps.py): real-time (100 MHz, chip-wide) stamps per block at entry,
// after the first load levels, after the contributions (touched) / the loads
// (look-ahead), and at the end,
// into a buffer of their own that no other code reads. No stamp executes in the product.
#if defined(MIREC_STEP_STAMPS)
constexpr int kStampBlocks = 16384;
__device__ unsigned long long g_step_stamps[kStampBlocks * 4];
#define MIREC_STAMP(slot)                                                                  \
  do {                                                                                     \
    __builtin_amdgcn_sched_barrier(0);                                                     \
    unsigned long long t_;                                                                 \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_) :: "memory");           \
    __builtin_amdgcn_sched_barrier(0);                                                     \
    if (threadIdx.x == 0 && blockIdx.x < kStampBlocks) g_step_stamps[blockIdx.x * 4 + (slot)] = t_; \
  } while (0)
#else
#define MIREC_STAMP(slot) \
  do {                    \
  } while (0)
#endif

// Contribution records, built per chunk on the prep stream (mirec_step_records, after
// the K2 grouping) so that a step's touched row reaches its partner rows in two
// dependent loads (its record, then the rows) instead of four (segment, perm, ids,
// rows). Contribution record (8 int32): positive k, negative slot j (-1: the positive
// or the user slot), user id, positive item id, the negatives' ids (the first 4; more
// are read from the keys). Row record (kRowRec int32) per touched-row slot u: row id,
// first position i0, contribution count, 0, then the records of its first kRecInline
// contributions; the others are at crec[i0 + c].
constexpr int kRecInts = 8;
constexpr int kRecInline = 2;
constexpr int kRowRec = 4 + kRecInline * kRecInts;
constexpr int kStepExtraCap = 62;       // extra records staged in LDS per touched row

__device__ __forceinline__ void contrib_record(int q, int tb, int Bc, int T,
                                               const int64_t* __restrict__ user,
                                               const int64_t* __restrict__ items, int64_t nU,
                                               int64_t nI, int32_t* __restrict__ out) {
  int kk = q, jn = -1;
  if (tb == 1 && q >= Bc) {                      // item row as a negative slot
    const int r = q - Bc;
    jn = r / Bc;
    kk = r - jn * Bc;
  }
  int32_t r[kRecInts];
  r[0] = kk;
  r[1] = jn;
  r[2] = (int32_t)clamp_id(user[kk], nU);
  r[3] = (int32_t)clamp_id(items[kk], nI);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int jj = jn >= 0 ? (j == 0 ? jn : -1) : (j < T ? j : -1);
    r[4 + j] = jj >= 0 ? (int32_t)clamp_id(items[Bc + (int64_t)jj * Bc + kk], nI) : 0;
  }
  reinterpret_cast<int4*>(out)[0] = make_int4(r[0], r[1], r[2], r[3]);
  reinterpret_cast<int4*>(out)[1] = make_int4(r[4], r[5], r[6], r[7]);
}

// One block per (table, batch): row records of the batch's touched-row slots and
// contribution records of its grouped positions.
__global__ __launch_bounds__(256) void step_records_kernel(
    const int64_t* __restrict__ ukeys, const int64_t* __restrict__ ikeys, int n_batches, int Bc,
    int T, int64_t nU, int64_t nI, const int32_t* __restrict__ u_perm,
    const int32_t* __restrict__ u_uniq, const int32_t* __restrict__ u_seg,
    const int32_t* __restrict__ u_nu, const int32_t* __restrict__ i_perm,
    const int32_t* __restrict__ i_uniq, const int32_t* __restrict__ i_seg,
    const int32_t* __restrict__ i_nu, int32_t* __restrict__ u_rec, int32_t* __restrict__ u_crec,
    int32_t* __restrict__ i_rec, int32_t* __restrict__ i_crec) {
  const int tb = blockIdx.x >= (unsigned)n_batches;
  const int b = tb ? blockIdx.x - n_batches : blockIdx.x;
  const int KI = (1 + T) * Bc;
  const int per = tb ? KI : Bc;
  const int64_t* __restrict__ user = ukeys + (int64_t)b * Bc;
  const int64_t* __restrict__ items = ikeys + (int64_t)b * KI;
  const int32_t* __restrict__ perm = (tb ? i_perm : u_perm) + (int64_t)b * per;
  const int32_t* __restrict__ uniq = (tb ? i_uniq : u_uniq) + (int64_t)b * per;
  const int32_t* __restrict__ seg = (tb ? i_seg : u_seg) + (int64_t)b * (per + 1);
  const int nu = (tb ? i_nu : u_nu)[b];
  int32_t* __restrict__ rec = (tb ? i_rec : u_rec) + (int64_t)b * per * kRowRec;
  int32_t* __restrict__ crec = (tb ? i_crec : u_crec) + (int64_t)b * per * kRecInts;
  const int n = seg[nu];
  for (int i = threadIdx.x; i < n; i += blockDim.x)
    contrib_record(perm[i], tb, Bc, T, user, items, nU, nI, crec + (int64_t)i * kRecInts);
  for (int x = threadIdx.x; x < nu; x += blockDim.x) {
    const int i0 = seg[x], i1 = seg[x + 1];
    int32_t* r = rec + (int64_t)x * kRowRec;
    reinterpret_cast<int4*>(r)[0] = make_int4(uniq[x], i0, i1 - i0, 0);
    for (int c = 0; c < kRecInline; ++c)
      if (i0 + c < i1) contrib_record(perm[i0 + c], tb, Bc, T, user, items, nU, nI,
                                      r + 4 + c * kRecInts);
  }
}

template <int D> struct StepVec { using T = float2; };
template <> struct StepVec<64> { using T = float; };

template <int D>
__global__ __launch_bounds__(D / Lanes<typename StepVec<D>::T>::n, 6) void bpr_adam_step_kernel(
    const StepLaunch L, const int64_t* __restrict__ items, int Bc, int T, float gamma,
    float grad_scale, float* __restrict__ loss_k, const float* __restrict__ consts,
    const int32_t* __restrict__ step_base, int step_off, AdamConsts k) {
  using V = typename StepVec<D>::T;
  constexpr int EPT = Lanes<V>::n;         // elements per thread
  constexpr int TPB = D / EPT;             // threads per block (one row)
  constexpr int LPR = D / 4;               // lanes per contribution (float4 each, K3's layout)
  constexpr int NG = TPB / LPR;            // contributions in flight per block
  __shared__ float cont[NG][D];
  MIREC_STAMP(0);
  int si = 0;
#pragma unroll
  for (int q = 1; q < 4; ++q)
    if ((int64_t)blockIdx.x >= L.block_start[q]) si = q;
  const bool ahead = si < 2;
  const int tb = si & 1;                   // 0 users, 1 items
  const mirec_adam_table& T_ = L.t[tb];
  const int u = (int)((int64_t)blockIdx.x - L.block_start[si]);
  const int t = threadIdx.x;
  const int grp = t / LPR;
  const int l = t - grp * LPR;
  // first load level, all independent of each other: the count and the row id (look-
  // ahead) or the row record (touched: row, first position, count, and this lane
  // group's inline contribution record); u < the launch's bound, so the loads stay in
  // the buffers even past the count
  const int n = ahead ? T_.ahead_n_uniq[0] : T_.n_uniq[0];
  const int32_t* __restrict__ R = L.rec[tb] + (int64_t)u * kRowRec;
  int4 hdr = make_int4(0, 0, 0, 0), ra = hdr, rb = hdr;
  int64_t row;
  if (ahead) {
    row = T_.ahead_uniq[u];
  } else {
    hdr = reinterpret_cast<const int4*>(R)[0];
    if (grp < kRecInline) {
      ra = reinterpret_cast<const int4*>(R + 4 + grp * kRecInts)[0];
      rb = reinterpret_cast<const int4*>(R + 4 + grp * kRecInts)[1];
    }
    row = hdr.x;
  }
  const int st = step_base[0] + step_off;
  if (u >= n) return;                      // block-uniform
#if defined(MIREC_STEP_PROBE_NO_AHEAD)     // timing probes only (tools/build_variant.sh)
  if (ahead) return;
#endif
#if defined(MIREC_STEP_PROBE_NO_TOUCHED)
  if (!ahead) return;
#endif
  const float* __restrict__ Pr[2] = {T_.p, T_.p_alt};
  float* __restrict__ Pw = ((st + 1) & 1) ? T_.p_alt : T_.p;
  const int raw = T_.last[row];
  const int64_t off = row * (D / EPT) + t;           // in units of V
  MIREC_STAMP(1);

  if (ahead) {
    // rows the next step reads and this one does not touch: replay last..st (zero
    // gradient), as adam_deferred_kernel's look-ahead segment
    if (raw == kZeroState || raw > st) return;    // current at every step / already done
    V p = reinterpret_cast<const V*>(Pr[raw & 1])[off];
    V m = reinterpret_cast<const V*>(T_.m)[off];
    V v = reinterpret_cast<const V*>(T_.v)[off];
    MIREC_STAMP(2);
    replay<V, true>(p, m, v, raw, st, consts, k);
    V z;
    memset(&z, 0, sizeof(V));
    adam_vec(p, m, v, z, step_consts(consts, st), k);   // step st: zero gradient
    __syncthreads();                               // every thread read `last`
    reinterpret_cast<V*>(Pw)[off] = p;
    reinterpret_cast<V*>(T_.m)[off] = m;
    reinterpret_cast<V*>(T_.v)[off] = v;
    if (t == 0) T_.last[row] = st + 1;
    MIREC_STAMP(3);
    return;
  }

  // ---- touched row: own state in flight while the contributions are formed. Every
  // row a step reads is complete through st - 1 (look-ahead / entry catch-up / flush)
  // or in the zero state (the same p in both buffers), so its p is in buffer st & 1;
  // a row behind (never, by that invariant) reloads from its own buffer below.
  const int last = raw == kZeroState ? st : raw;
  V p = reinterpret_cast<const V*>(Pr[st & 1])[off];
  V m = reinterpret_cast<const V*>(T_.m)[off];
  V v = reinterpret_cast<const V*>(T_.v)[off];
  const float* __restrict__ EU = L.t[0].p;         // partner rows at state st
  const float* __restrict__ EI = L.t[1].p;
  if (st & 1) {
    EU = L.t[0].p_alt;
    EI = L.t[1].p_alt;
  }
  const int i0 = hdr.y, nc = hdr.z;
  const float ng = -grad_scale;
  V g;
  memset(&g, 0, sizeof(V));
  // records of contributions kRecInline.. into LDS (one level, beside round 0's rows)
  __shared__ int4 xrec[kStepExtraCap][2];
  if (nc > kRecInline) {                           // block-uniform
    const int32_t* __restrict__ C = L.crec[tb] + (int64_t)(i0 + kRecInline) * kRecInts;
    for (int c = t; c < min(nc - kRecInline, kStepExtraCap); c += TPB) {
      xrec[c][0] = reinterpret_cast<const int4*>(C + (int64_t)c * kRecInts)[0];
      xrec[c][1] = reinterpret_cast<const int4*>(C + (int64_t)c * kRecInts)[1];
    }
    __syncthreads();
  }
  for (int base = 0; base < nc; base += NG) {
    const int c = base + grp;
    if (c < nc) {
      int4 r0 = ra, r1 = rb;                        // contribution c's record
      if (c >= kRecInline) {
        if (c - kRecInline < kStepExtraCap) {
          r0 = xrec[c - kRecInline][0];
          r1 = xrec[c - kRecInline][1];
        } else {
          const int32_t* C = L.crec[tb] + (int64_t)(i0 + c) * kRecInts;
          r0 = reinterpret_cast<const int4*>(C)[0];
          r1 = reinterpret_cast<const int4*>(C)[1];
        }
      }
      const int kk = r0.x, jn = r0.y;
      const float4 uv = reinterpret_cast<const float4*>(EU + (int64_t)r0.z * D)[l];
      const float4 pv = reinterpret_cast<const float4*>(EI + (int64_t)r0.w * D)[l];
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      if (jn >= 0) {                                  // item row as the negative jn
        const float4 nv = reinterpret_cast<const float4*>(EI + (int64_t)r1.x * D)[l];
        const float sp = group_sum<LPR>(dot4(uv, pv));
        const float sn = group_sum<LPR>(dot4(uv, nv));
        acc = contrib_n(bpr_coef(sp, sn, gamma, ng).dx, uv);
      } else {                                        // user row, or item row as the positive
        const int nid4[4] = {r1.x, r1.y, r1.z, r1.w};
        float lsum = 0.f;
        for (int j0 = 0; j0 < T; j0 += 4) {
          float4 nv[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int j = j0 + e;
            nv[e] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (j < T) {
              const int64_t nid = j < 4 ? (int64_t)nid4[e]
                                        : clamp_id(items[Bc + (int64_t)j * Bc + kk],
                                                   L.t[1].n_rows);
              nv[e] = reinterpret_cast<const float4*>(EI + nid * D)[l];
            }
          }
          const float sp = group_sum<LPR>(dot4(uv, pv));
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
      *reinterpret_cast<float4*>(&cont[grp][4 * l]) = acc;
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < NG; ++h)
      if (base + h < nc) {
        const V cv = *reinterpret_cast<const V*>(&cont[h][EPT * t]);
#pragma unroll
        for (int e = 0; e < EPT; ++e) Lanes<V>::at(g, e) += Lanes<V>::at(cv, e);
      }
    __syncthreads();                                 // cont is rewritten next round
  }
  if (last < st) {                                   // behind (not expected): own buffer
    p = reinterpret_cast<const V*>(Pr[last & 1])[off];
  }

  // ---- Adam step of the row (replaying skipped zero-gradient steps first)
  MIREC_STAMP(2);
  replay<V, true>(p, m, v, last, st, consts, k);
  const bool fresh = last <= st;
  if (fresh) adam_vec(p, m, v, g, step_consts(consts, st), k);
  __syncthreads();
  if (!fresh) return;
  reinterpret_cast<V*>(Pw)[off] = p;
  reinterpret_cast<V*>(T_.m)[off] = m;
  reinterpret_cast<V*>(T_.v)[off] = v;
  if (t == 0) T_.last[row] = st + 1;
  MIREC_STAMP(3);
}

}  // namespace mirec

using namespace mirec;

extern "C" int mirec_step_records(const int64_t* user_keys, const int64_t* item_keys,
                                  int64_t n_batches, int64_t Bc, int32_t T, int64_t n_users,
                                  int64_t n_items, const int32_t* u_perm, const int32_t* u_uniq,
                                  const int32_t* u_seg, const int32_t* u_nu,
                                  const int32_t* i_perm, const int32_t* i_uniq,
                                  const int32_t* i_seg, const int32_t* i_nu, int32_t* u_rec,
                                  int32_t* u_crec, int32_t* i_rec, int32_t* i_crec,
                                  void* stream) {
  if (n_batches < 0 || Bc < 0 || T < 1 || (int64_t)(1 + T) * Bc > INT32_MAX || n_users <= 0 ||
      n_items <= 0 || !user_keys || !item_keys || !u_perm || !u_uniq || !u_seg || !u_nu ||
      !i_perm || !i_uniq || !i_seg || !i_nu || !u_rec || !u_crec || !i_rec || !i_crec) {
    set_error("mirec_step_records: bad arguments");
    return -1;
  }
  if (n_batches == 0 || Bc == 0) return 0;
  hipLaunchKernelGGL(step_records_kernel, dim3((unsigned)(2 * n_batches)), dim3(256), 0,
                     (hipStream_t)stream, user_keys, item_keys, (int)n_batches, (int)Bc, T,
                     n_users, n_items, u_perm, u_uniq, u_seg, u_nu, i_perm, i_uniq, i_seg, i_nu,
                     u_rec, u_crec, i_rec, i_crec);
  return launch_status("mirec_step_records");
}

extern "C" int mirec_bpr_adam_step_f32(const mirec_adam_table* tables,
                                       const int64_t* n_max_uniq, int32_t d,
                                       const int64_t* items, int64_t Bc, int32_t T, float gamma,
                                       float grad_scale, float* loss_k, const int32_t* u_rec,
                                       const int32_t* u_crec, const int32_t* i_rec,
                                       const int32_t* i_crec, const float* step_consts_dev,
                                       const int32_t* step_base_dev, int32_t step_off,
                                       double beta1, double beta2, double eps,
                                       double weight_decay, void* stream) {
  const char* what = "mirec_bpr_adam_step_f32";
  if (!tables || !n_max_uniq || !items || Bc < 0 || T < 1 || !step_consts_dev ||
      (int64_t)(1 + T) * Bc > INT32_MAX || !u_rec || !u_crec || !i_rec || !i_crec ||
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
    if (!t.p || !t.p_alt || !t.m || !t.v || !t.last || !t.n_uniq || t.n_rows <= 0 ||
        n_max_uniq[q] < 0 || t.dense_grad ||
        (t.ahead_uniq == nullptr) != (t.ahead_n_uniq == nullptr)) {
      set_error("%s: bad table %d", what, q);
      return -1;
    }
    L.t[q] = t;
  }
  L.rec[0] = u_rec;
  L.crec[0] = u_crec;
  L.rec[1] = i_rec;
  L.crec[1] = i_crec;
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
    hipLaunchKernelGGL(bpr_adam_step_kernel<DD>, grd,                                        \
                       dim3(DD / Lanes<typename StepVec<DD>::T>::n), 0, st, L, items,        \
                       (int)Bc, T, gamma, grad_scale, loss_k, step_consts_dev, step_base_dev,\
                       step_off, k);                                                         \
    break;
  switch (d) {
    MIREC_STEP_CASE(64)
    MIREC_STEP_CASE(128)
    MIREC_STEP_CASE(256)
  }
#undef MIREC_STEP_CASE
  return launch_status(what);
}

#if defined(MIREC_STEP_STAMPS)
// diagnostic build only: copy / clear the stamps (4 x kStampBlocks u64)
extern "C" int mirec_step_stamps(void* dst, size_t bytes) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_step_stamps), bytes) == hipSuccess ? 0 : -1;
}
extern "C" int mirec_step_stamps_clear(void) {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_step_stamps)) != hipSuccess) return -1;
  return hipMemset(p, 0, sizeof(g_step_stamps)) == hipSuccess ? 0 : -1;
}
#endif
