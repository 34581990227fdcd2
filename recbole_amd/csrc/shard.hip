// Row-sharded embedding tables over G ranks: the index plans of
// the two per-step row exchanges and the owner's slice of the global grouping.
//
// Ownership is cyclic — row `id` lives on rank id % G at local row id / G — so the
// Zipf head rows of a table spread over every rank. Every rank walks the sampler
// and groups the GLOBAL batch itself (replicated, cheap, on the prep stream), so
// each rank knows, without any exchange, which rows every other rank needs:
//
//   global slots of a batch of Bc positives (the reference's pairwise layout,
//   general_dataloader.py:235-241):   user slot t = k,  item slot t = Bc + j*Bc + k
//   (k < Bc positive, j = 0 the positive item, j >= 1 the negatives);
//   slice of a slot: g = k / B (rank g computes positives [g*B, g*B + n_g));
//   message (g, o): the slots of slice g whose row rank o owns, ascending t; a slot's
//   index in it is idx(t); every message is padded to `cap` rows.
//
// Forward: owner o sends rows -> rank g receives them at o*cap + idx(t) (one
// all-to-all of equal blocks). Rank g runs K3 on its slice reading rows at those
// positions, writes the slice's per-slot gradient rows, and sends each back in the
// same (g, o) message position (the second all-to-all). The owner finds
// contribution t of its rows at g*cap + idx(t), so K5 sums every owned row's
// contributions in the GLOBAL grouping order — the same sums, the same Adam step,
// the same bits as one GPU running the global batch.
//
// The K2 grouping sorts owner-major keys key(id) = (id % G) * S + id / G (S = rows per
// shard), so rank r's rows are the contiguous key range [r*S, (r+1)*S) of every
// sorted list and its slice of the grouping is a sub-range found by binary search.
#include "common.h"

namespace mirec {

constexpr int kPlanThreads = 256;
constexpr int kMaxRanks = 64;

__global__ void shard_keys_kernel(const int64_t* __restrict__ ids, int64_t n, int32_t G,
                                  int64_t S, int64_t* __restrict__ keys) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t id = ids[i];
  keys[i] = (id % G) * S + id / G;
}

// One workgroup per (batch c, slice g). Scans slice g's slots in ascending t and
// numbers them per owner; writes what rank r needs as owner and as requester.
__global__ __launch_bounds__(kPlanThreads) void shard_plan_kernel(
    const int64_t* __restrict__ users, const int64_t* __restrict__ items, int64_t Bc,
    int64_t B, int32_t T, int32_t G, int32_t r, int64_t cap, int64_t* __restrict__ fwd_rows,
    int32_t* __restrict__ map2, int64_t* __restrict__ pos, int32_t* __restrict__ bwd_src,
    int32_t* __restrict__ status) {
  __shared__ int wave_cnt[kMaxRanks][kPlanThreads / 64];
  __shared__ int run[kMaxRanks];
  const int64_t c = blockIdx.x / G;
  const int g = blockIdx.x % G;
  const int64_t KI = (1 + (int64_t)T) * Bc;
  const int64_t* __restrict__ u_c = users + c * Bc;
  const int64_t* __restrict__ i_c = items + c * KI;
  const int64_t k0 = (int64_t)g * B;
  const int64_t n_g = max((int64_t)0, min(B, Bc - k0));
  const int64_t n_slots = (2 + (int64_t)T) * n_g;
  const int64_t M = (int64_t)G * cap;
  int64_t* __restrict__ fr = fwd_rows + c * M;
  int32_t* __restrict__ m2 = map2 + c * (Bc + KI);
  int64_t* __restrict__ ps = pos + c * (2 + (int64_t)T) * B;
  int32_t* __restrict__ bs = bwd_src + c * M;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  for (int o = threadIdx.x; o < G; o += kPlanThreads) run[o] = 0;
  __syncthreads();
  int overflow = 0;
  for (int64_t base = 0; base < n_slots; base += kPlanThreads) {
    const int64_t s = base + threadIdx.x;       // slot of the slice: users, then items j-major
    const bool act = s < n_slots;
    int64_t t = 0, id = 0, ls = s;
    bool is_user = false;
    if (act) {
      if (s < n_g) {
        is_user = true;
        t = k0 + s;
        id = u_c[t];
      } else {
        const int64_t q = s - n_g;
        const int64_t j = q / n_g, kk = q % n_g;
        t = Bc + j * Bc + k0 + kk;
        id = i_c[j * Bc + k0 + kk];
      }
    }
    const int o = act ? (int)(id % G) : -1;
    // per-owner ranks of this tile's slots: ballots, then the waves before this one
    int pre = 0;
    for (int q = 0; q < G; ++q) {
      const uint64_t m = __ballot(o == q);
      if (q == o) pre = __popcll(m & ((1ull << lane) - 1ull));
      if (lane == 0) wave_cnt[q][wid] = __popcll(m);
    }
    __syncthreads();
    int64_t idx = 0;
    if (act) {
      int before = run[o];
      for (int w = 0; w < wid; ++w) before += wave_cnt[o][w];
      idx = before + pre;
    }
    __syncthreads();
    if (threadIdx.x < G) {
      int tot = 0;
      for (int w = 0; w < kPlanThreads / 64; ++w) tot += wave_cnt[threadIdx.x][w];
      run[threadIdx.x] += tot;
    }
    if (act) {
      if (idx >= cap) {
        // no room in the message: the slot gets a harmless in-range position (row 0
        // of the first message) so no kernel reads outside the buffers; the chunk is
        // re-planned with a larger cap before it runs (status, ShardedBPRTrainStep)
        overflow = 1;
        if (o == r) m2[t] = 0;
        if (g == r) ps[ls] = 0;
      } else {
        const int64_t local = id / G;
        if (o == r) {                                   // owner side: rows to send to g
          fr[(int64_t)g * cap + idx] = is_user ? local : -(local + 1);
          m2[t] = (int32_t)((int64_t)g * cap + idx);
        }
        if (g == r) {                                   // requester side: where my slot's row lands
          ps[ls] = (int64_t)o * cap + idx;
          bs[(int64_t)o * cap + idx] = (int32_t)ls;
        }
      }
    }
    __syncthreads();
  }
  // padding of the messages this workgroup owns (harmless rows: user row 0 / slot 0)
  for (int q = 0; q < G; ++q) {
    const int64_t cnt = min((int64_t)run[q], cap);
    if (q == r)
      for (int64_t i = cnt + threadIdx.x; i < cap; i += kPlanThreads) fr[(int64_t)g * cap + i] = 0;
    if (g == r)
      for (int64_t i = cnt + threadIdx.x; i < cap; i += kPlanThreads) bs[(int64_t)q * cap + i] = 0;
  }
  // status[0] = -4 if any message of this (batch, slice) overflowed, status[1] = the
  // largest message (rows) — every rank's launch counts every (slice, owner) message,
  // so every rank sees the same status without a collective
  if (threadIdx.x == 0) {
    int most = 0;
    for (int q = 0; q < G; ++q) most = max(most, run[q]);
    atomicMax(status + 1, most);
  }
  if (overflow) atomicExch(status, -4);
}

__device__ __forceinline__ int32_t lower_bound_i32(const int32_t* __restrict__ a, int32_t n,
                                                   int64_t key) {
  int32_t lo = 0, hi = n;
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    if ((int64_t)a[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// Owner-filtered grouping input (each rank sorts only the slots whose rows it owns, ~1/G
// of the global batch, instead of every rank sorting all of it): per batch, the slots i
// with ids[i] % G == r in slot order (a stable compaction), keyed r*S + ids[i]/G — the
// owner-major keys of the global path, so the sort, the look-ahead diff and shard_own
// work unchanged — with sel_pos = i; padded to cap_sel with the key (r+1)*S (just past the
// rank's range: shard_own's binary search leaves it out). sel_most[0] = max over the
// batches of the owned count (atomicMax; zero it first): a count over cap_sel is
// truncated here and the chunk must be re-planned with a larger cap_sel.
constexpr int kSelThreads = 1024;
__global__ __launch_bounds__(kSelThreads) void shard_select_kernel(
    const int64_t* __restrict__ ids, int64_t per, int32_t G, int64_t S, int32_t r,
    int64_t cap_sel, int64_t* __restrict__ keys, int32_t* __restrict__ sel_pos,
    int32_t* __restrict__ sel_most) {
  __shared__ int wtot[kSelThreads / 64];
  const int64_t c = blockIdx.x;
  const int64_t* __restrict__ id_c = ids + c * per;
  int64_t* __restrict__ k_c = keys + c * cap_sel;
  int32_t* __restrict__ p_c = sel_pos + c * cap_sel;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t kb = (int64_t)r * S;
  int64_t base = 0;
  for (int64_t i0 = 0; i0 < per; i0 += kSelThreads) {
    const int64_t i = i0 + threadIdx.x;
    int64_t id = 0;
    bool own = false;
    if (i < per) {
      id = id_c[i];
      own = id % G == r;
    }
    const uint64_t m = __ballot(own);
    if (lane == 0) wtot[wid] = __popcll(m);
    __syncthreads();
    int64_t j = base + __popcll(m & ((1ull << lane) - 1ull));
    int tot = 0;
    for (int w = 0; w < kSelThreads / 64; ++w) {
      if (w < wid) j += wtot[w];
      tot += wtot[w];
    }
    if (own && j < cap_sel) {
      k_c[j] = kb + id / G;
      p_c[j] = (int32_t)i;
    }
    base += tot;
    __syncthreads();                      // wtot is rewritten next round
  }
  for (int64_t j = base + threadIdx.x; j < cap_sel; j += kSelThreads) {
    k_c[j] = kb + S;
    p_c[j] = 0;
  }
  if (threadIdx.x == 0) atomicMax(sel_most, (int)base);
}

// Workgroups (batch, tile) — tile y of gridDim.y strides the batch's entries, so a chunk
// of a few large batches still spreads over the chip (one workgroup per batch took
// 48 µs for 16 batches of 20 K item slots): rank r's sub-range [lo, hi) of the sorted (keyed) uniq
// list -> local row ids, its segment offsets, and the contributions of those
// segments remapped to their positions in the backward receive buffer; the same
// for the look-ahead list.
// With sel_pos (the owner-filtered grouping, shard_select_kernel): the input lists have
// stride per_batch (= cap_sel), a grouped position's slot is sel_pos[perm[p]], and the
// outputs keep the stride out_per of the global lists.
__global__ __launch_bounds__(kPlanThreads) void shard_own_kernel(
    const int32_t* __restrict__ uniq, const int32_t* __restrict__ seg,
    const int32_t* __restrict__ n_uniq, const int32_t* __restrict__ perm, int64_t per_batch,
    const int32_t* __restrict__ ahead, const int32_t* __restrict__ n_ahead,
    const int32_t* __restrict__ map2, int64_t map_stride, int64_t map_off, int64_t S, int32_t r,
    int32_t* __restrict__ own_uniq, int32_t* __restrict__ own_seg, int32_t* __restrict__ own_n,
    int32_t* __restrict__ perm2, int32_t* __restrict__ own_ahead, int32_t* __restrict__ own_nah,
    const int32_t* __restrict__ sel_pos, int64_t out_per) {
  const int64_t c = blockIdx.x;
  const int32_t* __restrict__ uq = uniq + c * per_batch;
  const int32_t* __restrict__ sg = seg + c * (per_batch + 1);
  const int32_t* __restrict__ pm = perm + c * per_batch;
  const int32_t* __restrict__ sp = sel_pos ? sel_pos + c * per_batch : nullptr;
  const int32_t* __restrict__ m2 = map2 + c * map_stride + map_off;
  const int64_t kb = (int64_t)r * S, ke = kb + S;
  const int32_t n = n_uniq[c];
  const int32_t lo = lower_bound_i32(uq, n, kb), hi = lower_bound_i32(uq, n, ke);
  int32_t* __restrict__ ou = own_uniq + c * out_per;
  int32_t* __restrict__ os = own_seg + c * (out_per + 1);
  int32_t* __restrict__ p2 = perm2 + c * out_per;
  const int32_t t0 = (int32_t)(blockIdx.y * kPlanThreads + threadIdx.x);
  const int32_t ts = (int32_t)(gridDim.y * kPlanThreads);
  for (int32_t j = lo + t0; j < hi; j += ts) ou[j - lo] = (int32_t)(uq[j] - kb);
  for (int32_t j = lo + t0; j <= hi; j += ts) os[j - lo] = sg[j];
  for (int32_t p = sg[lo] + t0; p < sg[hi]; p += ts) p2[p] = m2[sp ? sp[pm[p]] : pm[p]];
  if (t0 == 0) own_n[c] = hi - lo;
  if (ahead) {
    const int32_t* __restrict__ ah = ahead + c * per_batch;
    const int32_t na = n_ahead[c];
    const int32_t alo = lower_bound_i32(ah, na, kb), ahi = lower_bound_i32(ah, na, ke);
    int32_t* __restrict__ oa = own_ahead + c * out_per;
    for (int32_t j = alo + t0; j < ahi; j += ts) oa[j - alo] = (int32_t)(ah[j] - kb);
    if (t0 == 0) own_nah[c] = ahi - alo;
  }
}

// tiles per batch of the (batch, tile) grids: ~4 entries per lane
inline unsigned plan_tiles(int64_t per_batch) {
  const int64_t t = (per_batch + 4 * kPlanThreads - 1) / (4 * kPlanThreads);
  return (unsigned)(t < 1 ? 1 : t > 64 ? 64 : t);
}

// Where each entry of step c's owned lists sits in step c+1's owned list (the owner
// folds step c+1's forward exchange into step c's optimizer launch: comm.hip
// adam_xchg_kernel pushes a row right after its update). Workgroups (step, tile) for
// c < n_batches - 1 (the lists are sorted local row ids): next_t[c][i] = the index of
// own[c][i] in own[c+1], -1 when step c+1 does not read it; next_a[c][a] = the index of
// own_ahead[c][a] in own[c+1] (the look-ahead list is own[c+1] minus own[c]).
__global__ __launch_bounds__(kPlanThreads) void shard_next_kernel(
    const int32_t* __restrict__ own, const int32_t* __restrict__ own_n,
    const int32_t* __restrict__ own_ah, const int32_t* __restrict__ own_nah, int64_t per_batch,
    int32_t* __restrict__ next_t, int32_t* __restrict__ next_a) {
  const int64_t c = blockIdx.x;
  const int32_t* __restrict__ nx = own + (c + 1) * per_batch;
  const int32_t nn = own_n[c + 1];
  const int32_t* __restrict__ cur = own + c * per_batch;
  const int32_t n = own_n[c];
  const int32_t t0 = (int32_t)(blockIdx.y * kPlanThreads + threadIdx.x);
  const int32_t ts = (int32_t)(gridDim.y * kPlanThreads);
  for (int32_t i = t0; i < n; i += ts) {
    const int32_t key = cur[i];
    const int32_t j = lower_bound_i32(nx, nn, key);
    next_t[c * per_batch + i] = (j < nn && nx[j] == key) ? j : -1;
  }
  const int32_t* __restrict__ ah = own_ah + c * per_batch;
  const int32_t na = own_nah[c];
  for (int32_t a = t0; a < na; a += ts) {
    const int32_t key = ah[a];
    const int32_t j = lower_bound_i32(nx, nn, key);
    next_a[c * per_batch + a] = (j < nn && nx[j] == key) ? j : -1;
  }
}

// out[i, :] = idx[i] >= 0 ? U[idx[i], :] : I[-idx[i] - 1, :]  (d/4 lanes per row,
// 16-B vectors): the forward message of an owner, rows of its two shards.
template <int D>
__global__ __launch_bounds__(256) void shard_gather_kernel(const float* __restrict__ U,
                                                           const float* __restrict__ I,
                                                           const int64_t* __restrict__ idx,
                                                           int64_t n, float* __restrict__ out) {
  constexpr int LPR = D / 4;
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int c = threadIdx.x % LPR;
  if (row >= n) return;
  const int64_t s = idx[row];
  const float4* src = reinterpret_cast<const float4*>(s >= 0 ? U + s * D : I + (-s - 1) * D);
  reinterpret_cast<float4*>(out + row * D)[c] = src[c];
}

}  // namespace mirec

using namespace mirec;

extern "C" int mirec_shard_keys(const int64_t* ids, int64_t n, int32_t G, int64_t S,
                                int64_t* keys, void* stream) {
  if (n < 0 || G < 1 || S < 1 || (n > 0 && (!ids || !keys))) {
    set_error("mirec_shard_keys: bad arguments");
    return -1;
  }
  if (n == 0) return 0;
  hipLaunchKernelGGL(shard_keys_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, ids, n, G, S, keys);
  return launch_status("mirec_shard_keys");
}

extern "C" int mirec_shard_plan(const int64_t* users, const int64_t* items, int64_t n_batches,
                                int64_t Bc, int64_t B, int32_t T, int32_t G, int32_t rank,
                                int64_t cap, int64_t* fwd_rows, int32_t* map2, int64_t* pos,
                                int32_t* bwd_src, int32_t* status, void* stream) {
  if (n_batches < 0 || Bc < 0 || B < 1 || T < 0 || G < 1 || G > kMaxRanks || rank < 0 ||
      rank >= G || cap < 1 || (Bc > (int64_t)G * B) || !users || !items || !fwd_rows ||
      !map2 || !pos || !bwd_src || !status) {
    set_error("mirec_shard_plan: bad arguments (G=%d rank=%d Bc=%lld B=%lld)", G, rank,
              (long long)Bc, (long long)B);
    return -1;
  }
  if (n_batches == 0 || Bc == 0) return 0;
  hipLaunchKernelGGL(shard_plan_kernel, dim3((unsigned)(n_batches * G)), dim3(kPlanThreads), 0,
                     (hipStream_t)stream, users, items, Bc, B, T, G, rank, cap, fwd_rows, map2,
                     pos, bwd_src, status);
  return launch_status("mirec_shard_plan");
}

extern "C" int mirec_shard_own(const int32_t* uniq, const int32_t* seg, const int32_t* n_uniq,
                               const int32_t* perm, int64_t per_batch, int64_t n_batches,
                               const int32_t* ahead, const int32_t* n_ahead, const int32_t* map2,
                               int64_t map_stride, int64_t map_off, int64_t S, int32_t rank,
                               int32_t* own_uniq, int32_t* own_seg, int32_t* own_n,
                               int32_t* perm2, int32_t* own_ahead, int32_t* own_nah,
                               void* stream) {
  if (!uniq || !seg || !n_uniq || !perm || !map2 || !own_uniq || !own_seg || !own_n ||
      !perm2 || per_batch < 1 || n_batches < 0 || S < 1 || rank < 0 ||
      (ahead && (!n_ahead || !own_ahead || !own_nah))) {
    set_error("mirec_shard_own: bad arguments");
    return -1;
  }
  if (n_batches == 0) return 0;
  hipLaunchKernelGGL(shard_own_kernel, dim3((unsigned)n_batches, plan_tiles(per_batch)),
                     dim3(kPlanThreads), 0,
                     (hipStream_t)stream, uniq, seg, n_uniq, perm, per_batch, ahead, n_ahead, map2,
                     map_stride, map_off, S, rank, own_uniq, own_seg, own_n, perm2, own_ahead,
                     own_nah, (const int32_t*)nullptr, per_batch);
  return launch_status("mirec_shard_own");
}

extern "C" int mirec_shard_select(const int64_t* ids, int64_t n_batches, int64_t per, int32_t G,
                                  int64_t S, int32_t rank, int64_t cap_sel, int64_t* keys,
                                  int32_t* sel_pos, int32_t* sel_most, void* stream) {
  if (!ids || !keys || !sel_pos || !sel_most || n_batches < 0 || per < 1 || G < 1 || S < 1 ||
      rank < 0 || rank >= G || cap_sel < 1 || cap_sel > per) {
    set_error("mirec_shard_select: bad arguments");
    return -1;
  }
  if (n_batches == 0) return 0;
  hipLaunchKernelGGL(shard_select_kernel, dim3((unsigned)n_batches), dim3(kSelThreads), 0,
                     (hipStream_t)stream, ids, per, G, S, rank, cap_sel, keys, sel_pos, sel_most);
  return launch_status("mirec_shard_select");
}

extern "C" int mirec_shard_own_sel(const int32_t* uniq, const int32_t* seg, const int32_t* n_uniq,
                                   const int32_t* perm, int64_t cap_sel, int64_t n_batches,
                                   const int32_t* ahead, const int32_t* n_ahead,
                                   const int32_t* map2, int64_t map_stride, int64_t map_off,
                                   int64_t S, int32_t rank, const int32_t* sel_pos, int64_t per,
                                   int32_t* own_uniq, int32_t* own_seg, int32_t* own_n,
                                   int32_t* perm2, int32_t* own_ahead, int32_t* own_nah,
                                   void* stream) {
  if (!uniq || !seg || !n_uniq || !perm || !map2 || !sel_pos || !own_uniq || !own_seg ||
      !own_n || !perm2 || cap_sel < 1 || per < cap_sel || n_batches < 0 || S < 1 || rank < 0 ||
      (ahead && (!n_ahead || !own_ahead || !own_nah))) {
    set_error("mirec_shard_own_sel: bad arguments");
    return -1;
  }
  if (n_batches == 0) return 0;
  hipLaunchKernelGGL(shard_own_kernel, dim3((unsigned)n_batches, plan_tiles(cap_sel)),
                     dim3(kPlanThreads), 0, (hipStream_t)stream, uniq, seg, n_uniq, perm, cap_sel,
                     ahead, n_ahead, map2, map_stride, map_off, S, rank, own_uniq, own_seg, own_n,
                     perm2, own_ahead, own_nah, sel_pos, per);
  return launch_status("mirec_shard_own_sel");
}

extern "C" int mirec_shard_next(const int32_t* own, const int32_t* own_n, const int32_t* own_ahead,
                                const int32_t* own_nah, int64_t per_batch, int64_t n_batches,
                                int32_t* next_t, int32_t* next_a, void* stream) {
  if (!own || !own_n || !own_ahead || !own_nah || !next_t || !next_a || per_batch < 1 ||
      n_batches < 0) {
    set_error("mirec_shard_next: bad arguments");
    return -1;
  }
  if (n_batches < 2) return 0;
  hipLaunchKernelGGL(shard_next_kernel, dim3((unsigned)(n_batches - 1), plan_tiles(per_batch)),
                     dim3(kPlanThreads), 0,
                     (hipStream_t)stream, own, own_n, own_ahead, own_nah, per_batch, next_t, next_a);
  return launch_status("mirec_shard_next");
}

extern "C" int mirec_shard_gather_f32(const float* U, const float* I, int32_t d,
                                      const int64_t* idx, int64_t n, float* out, void* stream) {
  if (n < 0 || !U || !I || !out || (n > 0 && !idx)) {
    set_error("mirec_shard_gather_f32: bad arguments");
    return -1;
  }
  if (n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const unsigned blocks = (unsigned)((n * (d / 4) + 255) / 256);
  switch (d) {
    case 32: hipLaunchKernelGGL(shard_gather_kernel<32>, dim3(blocks), dim3(256), 0, st, U, I, idx, n, out); break;
    case 64: hipLaunchKernelGGL(shard_gather_kernel<64>, dim3(blocks), dim3(256), 0, st, U, I, idx, n, out); break;
    case 128: hipLaunchKernelGGL(shard_gather_kernel<128>, dim3(blocks), dim3(256), 0, st, U, I, idx, n, out); break;
    case 256: hipLaunchKernelGGL(shard_gather_kernel<256>, dim3(blocks), dim3(256), 0, st, U, I, idx, n, out); break;
    default:
      set_error("mirec_shard_gather_f32: d must be 32, 64, 128 or 256 (got %d)", d);
      return -1;
  }
  return launch_status("mirec_shard_gather_f32");
}
