// K4 — bit-exact negative sampler: cyclic walk over the shuffled random_list
// with rejection of "used" items, refilled in ascending slot order.
//
// Restates AbstractSampler.random_num + sample_by_key_ids
// (recbole/sampler/sampler.py:82-101, 103-154):
//   random_num(num): value[t] = random_list[(random_pr + t) mod L], random_pr += num
//   round 0:  value[0..K*num) = random_num(K*num); key of slot t = keys[t mod K]
//   round i:  check = [t in check (ascending) if value[t] in used[key(t)]]
//             value[check] = random_num(len(check))
// Both branches of sample_by_key_ids (single key / many keys) have exactly this
// semantics. The walk is inherently sequential in `random_pr`, so one
// workgroup walks the batches in order: round 0 tests kPer consecutive slots
// per lane (independent loads in flight) and one block scan orders the
// rejected slots; refill rounds with more than 64 pending slots run over the
// block, the tail (<= 64 pending, the common case) runs in ONE wave with
// ballots and no block barrier. Pending lists and the batch's keys live in LDS.
// Membership: a per-key bitmap (one load per test) when the caller provides
// one, else binary search in the CSR of used ids.
// The sampler only depends on the data pipeline (never on model state), so the
// trainer runs it ahead of the model step on a side stream.
#include "common.h"

namespace mirec {

// Phase profile of the single-block walk (build variant -DMIREC_WALK_PROF, see
// tools/probe_walk.py): thread 0 accumulates shader-clock deltas per phase.
#ifdef MIREC_WALK_PROF
__device__ unsigned long long g_walk_prof[16];
#define WALK_MARK(slot, t0)                                                          \
  do {                                                                               \
    if (threadIdx.x == 0) {                                                          \
      const unsigned long long t1_ = __builtin_amdgcn_s_memtime();                   \
      atomicAdd(&g_walk_prof[slot], t1_ - (t0));                                     \
      (t0) = t1_;                                                                    \
    }                                                                                \
  } while (0)
#define WALK_COUNT(slot, n) do { if (threadIdx.x == 0) atomicAdd(&g_walk_prof[slot], (unsigned long long)(n)); } while (0)
#else
#define WALK_MARK(slot, t0) do {} while (0)
#define WALK_COUNT(slot, n) do {} while (0)
#endif

constexpr int kSampThreads = 1024;
constexpr int kPer = 4;          // round-0 slots per lane per pass
constexpr int kListLds = 4096;   // pending-slot lists in LDS up to this many slots
constexpr int kKeyLds = 4096;    // batch keys cached in LDS up to this many keys

struct UsedSet {
  const int64_t* ptr;
  const int32_t* cols;
  const uint32_t* bits;  // [n_keys, words] bitmap or NULL
  int64_t words;
  int64_t nbits;
};

__device__ __forceinline__ bool is_used(const UsedSet& u, int64_t key, int32_t v) {
  if (u.bits)
    return (uint64_t)(uint32_t)v < (uint64_t)u.nbits &&
           ((u.bits[key * u.words + (v >> 5)] >> (v & 31)) & 1u);
  return sorted_contains(u.cols, u.ptr[key], u.ptr[key + 1], v);
}

// Exclusive scan of 0/1 flags over the block with ballots: one barrier.
// `lds` (blockDim/64 ints) must not be reused before the next block barrier.
__device__ __forceinline__ int block_flag_scan(int flag, int* lds, int* total) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  const uint64_t m = __ballot(flag);
  const int pre = __popcll(m & ((1ull << lane) - 1ull));
  if (lane == 0) lds[wid] = __popcll(m);
  __syncthreads();
  int before = 0, tot = 0;
  for (int w = 0; w < nw; ++w) {
    const int c = lds[w];
    before += (w < wid) ? c : 0;
    tot += c;
  }
  *total = tot;
  return before + pre;
}

// Refill rounds of one batch: the i-th rejected slot (ascending) takes the i-th
// next walk value, until no slot is rejected. The reference loops until done;
// on adversarial inputs (a key whose free ids all sit outside the walk
// positions its slots can reach) that never ends, so give up after a bound and
// set `livelock`. Called by every thread of the block; `cur` holds the nrej
// pending slots, `nxt` is scratch of the same capacity.
template <class KeyOf>
__device__ __forceinline__ void walk_refill(const int32_t* __restrict__ rl, int64_t L,
                                            int64_t& pr, const UsedSet& used, KeyOf key_of,
                                            int64_t* __restrict__ bout, int32_t* cur,
                                            int32_t* nxt, int32_t nrej,
                                            int (*scan_lds)[kSampThreads / 64 + 1],
                                            int32_t* wl, int64_t* pr_lds, int& livelock) {
  const int lane = threadIdx.x & 63;
  int64_t rounds = 0;
  const int64_t max_rounds = 4 * L + 1024;
  int sel = 0;
  while (nrej > 64) {                       // wide rounds: whole block
    if (++rounds > max_rounds) { livelock = 1; break; }
    WALK_COUNT(9, 1);
    int32_t nnew = 0;
    for (int32_t base = 0; base < nrej; base += kSampThreads) {
      const int32_t i = base + threadIdx.x;
      int rej = 0;
      int32_t t = 0;
      if (i < nrej) {
        t = cur[i];
        int64_t pos = pr + i;
        if (pos >= L) pos %= L;
        const int32_t v = rl[pos];
        bout[t] = v;
        rej = is_used(used, key_of(t), v) ? 1 : 0;
      }
      int tot;
      const int excl = block_flag_scan(rej, scan_lds[sel], &tot);
      sel ^= 1;
      if (rej) nxt[nnew + excl] = t;
      nnew += tot;
    }
    pr = (pr + nrej) % L;
    int32_t* tmp = cur; cur = nxt; nxt = tmp;
    nrej = nnew;
    __syncthreads();
  }
  WALK_COUNT(10, nrej);
  if (nrej > 0 && !livelock) {              // tail: one wave, no block barriers
    if (threadIdx.x < 64) {
      int n = nrej;
      int64_t p = pr;
      int32_t t = lane < n ? cur[lane] : 0;
      int ll = 0;
      while (n > 0) {
        if (++rounds > max_rounds) { ll = 1; break; }
        WALK_COUNT(11, 1);
        int rej = 0;
        if (lane < n) {
          int64_t pos = p + lane;
          if (pos >= L) pos %= L;
          const int32_t v = rl[pos];
          bout[t] = v;
          rej = is_used(used, key_of(t), v) ? 1 : 0;
        }
        const uint64_t m = __ballot(rej);
        if (rej) wl[__popcll(m & ((1ull << lane) - 1ull))] = t;
        __builtin_amdgcn_wave_barrier();
        p = (p + n) % L;
        n = __popcll(m);
        t = lane < n ? wl[lane] : 0;
        __builtin_amdgcn_wave_barrier();
      }
      if (lane == 0) { *pr_lds = p; scan_lds[1][kSampThreads / 64] = ll; }
    }
    __syncthreads();
    pr = *pr_lds;
    livelock = scan_lds[1][kSampThreads / 64];
  }
}

// Shared memory of the single-block walk (sample_walk_kernel, and the fallback block of
// the speculative walk below).
struct WalkLds {
  int scan[2][kSampThreads / 64 + 1];
  int32_t listA[kListLds];
  int32_t listB[kListLds];
  int32_t key_lds[kKeyLds];
  int32_t wl[64];
  int64_t pr;
  uint64_t wsum[kSampThreads / 64];
};

// Walk batches [b_begin, b_end) in order from pointer `pr` (advanced in place), every
// thread of the block taking part. bad_key / livelock are set (block-uniform for
// livelock) as the batches go; a livelock stops the walk.
__device__ void walk_serial(const int32_t* __restrict__ rl, int64_t L, int64_t& pr,
                            const int64_t* __restrict__ keys, int64_t n_keys, int64_t batch_keys,
                            int64_t b_begin, int64_t n_batches, int64_t num, const UsedSet& used,
                            int64_t key_space, int reject, int64_t* __restrict__ out,
                            int64_t out_stride, int32_t* __restrict__ rejA_g,
                            int32_t* __restrict__ rejB_g, const int64_t* __restrict__ seg_ptr,
                            WalkLds& S, int& bad_key, int& livelock) {
  auto& scan_lds = S.scan;
  int32_t* listA = S.listA;
  int32_t* listB = S.listB;
  int32_t* key_lds = S.key_lds;
  int32_t* wl = S.wl;
  int64_t& pr_lds = S.pr;
#ifdef MIREC_WALK_PROF
  unsigned long long tp = __builtin_amdgcn_s_memtime();
#endif
  for (int64_t b = b_begin; b < n_batches && !livelock; ++b) {
    // batch b = one sample_by_key_ids call: fixed-size batches, or the segments
    // [seg_ptr[b], seg_ptr[b+1]) of the key list (output packed at k0 * num)
    const int64_t k0 = seg_ptr ? seg_ptr[b] : b * batch_keys;
    const int64_t Kb = seg_ptr ? seg_ptr[b + 1] - k0 : min(batch_keys, n_keys - k0);
    if (seg_ptr && Kb == 0) continue;
    if (Kb <= 0) break;
    const int64_t total = Kb * num;
    const int64_t* __restrict__ bkeys = keys + k0;
    int64_t* __restrict__ bout = out + (seg_ptr ? k0 * num : b * out_stride);
    const bool lds_lists = total <= kListLds;
    int32_t* cur = lds_lists ? listA : rejA_g;
    int32_t* nxt = lds_lists ? listB : rejB_g;
    const bool lds_keys = Kb <= kKeyLds;
    if (reject && lds_keys) {
      for (int64_t k = threadIdx.x; k < Kb; k += kSampThreads) {
        const int64_t key = bkeys[k];
        key_lds[k] = (key < 0 || key >= key_space) ? -1 : (int32_t)key;
      }
      __syncthreads();
    }
    // key of slot t (-1 = out of range)
    auto key_of = [&](int64_t t) -> int64_t {
      const int64_t k = t % Kb;
      if (lds_keys) return key_lds[k];
      const int64_t key = bkeys[k];
      return (key < 0 || key >= key_space) ? -1 : key;
    };

    WALK_MARK(0, tp);                         // batch setup + keys to LDS
    // ---- round 0: fill every slot, collect rejected slots in ascending order
    int32_t nrej = 0;
    if (Kb <= kSampThreads && num <= 4 && lds_keys) {
      // one thread per key k: its slots t = j*Kb + k (j < num) — positions of one j
      // are consecutive over the threads (coalesced), the key is read once and its
      // membership rows are hit num times; ascending t = (j, k) order comes from one
      // block scan of the num per-j flags packed as 16-bit fields
      const int k = threadIdx.x;
      const bool has = k < Kb;
      const int64_t key = has && reject ? key_lds[k] : 0;
      int32_t v4[4];
      int64_t pos = pr + k;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (pos >= L) pos %= L;
        v4[j] = (has && j < num) ? rl[pos] : 0;
        pos += Kb;
      }
      uint64_t packed = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (has && j < num) {
          bout[(int64_t)j * Kb + k] = v4[j];
          if (reject) {
            if (key < 0) bad_key = 1;
            else if (is_used(used, key, v4[j])) packed |= 1ull << (16 * j);
          }
        }
      }
      WALK_MARK(3, tp);                       // round 0 values + membership (thread 0)
      // exclusive scan of the packed per-j counts (each field < 2^16: Kb <= 1024)
      const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
      uint64_t incl = packed;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint64_t y = __shfl_up(incl, off, 64);
        if (lane >= off) incl += y;
      }
      uint64_t* wsum = S.wsum;
      if (lane == 63) wsum[wid] = incl;
      __syncthreads();
      uint64_t before = 0, tot = 0;
      for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
        const uint64_t c = wsum[w];
        before += w < wid ? c : 0;
        tot += c;
      }
      const uint64_t excl = before + incl - packed;
      int base_j = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int cj = (int)((tot >> (16 * j)) & 0xffff);
        if ((packed >> (16 * j)) & 1ull)
          cur[base_j + (int)((excl >> (16 * j)) & 0xffff)] = (int32_t)((int64_t)j * Kb + k);
        base_j += cj;
      }
      nrej = base_j;
      WALK_MARK(4, tp);                       // round 0 scan
    } else
    for (int64_t base = 0; base < total; base += (int64_t)kSampThreads * kPer) {
      const int64_t t0 = base + (int64_t)threadIdx.x * kPer;
      int32_t vals[kPer];
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        int64_t pos = pr + t0 + j;
        if (pos >= L) pos %= L;
        vals[j] = (t0 + j < total) ? rl[pos] : 0;
      }
      int flags = 0, cnt = 0;
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const int64_t t = t0 + j;
        if (t < total) {
          bout[t] = vals[j];
          if (reject) {
            const int64_t key = key_of(t);
            if (key < 0) {
              bad_key = 1;
            } else if (is_used(used, key, vals[j])) {
              flags |= 1 << j;
              ++cnt;
            }
          }
        }
      }
      int tot;
      int excl = block_exclusive_scan(cnt, scan_lds[0], &tot);
#pragma unroll
      for (int j = 0; j < kPer; ++j)
        if ((flags >> j) & 1) cur[nrej + excl++] = (int32_t)(t0 + j);
      nrej += tot;
    }
    pr = (pr + total) % L;
    __syncthreads();
    WALK_MARK(1, tp);                         // round 0 incl. its scan
    WALK_COUNT(8, nrej);

    walk_refill(rl, L, pr, used, key_of, bout, cur, nxt, nrej, scan_lds, wl, &pr_lds,
                livelock);
    __syncthreads();                          // LDS lists / keys reused by the next batch
    WALK_MARK(2, tp);                         // refill rounds
  }
}

__global__ __launch_bounds__(kSampThreads) void sample_walk_kernel(
    const int32_t* __restrict__ rl, int64_t L, int64_t* __restrict__ pr_dev,
    const int64_t* __restrict__ keys, int64_t n_keys, int64_t batch_keys, int64_t n_batches,
    int64_t num, UsedSet used, int64_t key_space, int reject, int64_t* __restrict__ out,
    int64_t out_stride, int32_t* __restrict__ status, int32_t* __restrict__ rejA_g,
    int32_t* __restrict__ rejB_g, const int64_t* __restrict__ seg_ptr) {
  __shared__ WalkLds S;
  int64_t pr = pr_dev[0] % L;
  int bad_key = 0;
  int livelock = 0;
  walk_serial(rl, L, pr, keys, n_keys, batch_keys, 0, n_batches, num, used, key_space, reject,
              out, out_stride, rejA_g, rejB_g, seg_ptr, S, bad_key, livelock);
  if (bad_key) atomicExch(status, -2);
  if (livelock && threadIdx.x == 0) atomicExch(status, -3);
  __syncthreads();
  if (threadIdx.x == 0) pr_dev[0] = pr;
}

// ---- wide path (batches of more than kWideMin slots: a data-parallel global
// batch of G x 512 positives walks G x 2,048 slots per step on every rank).
// The single-block kernel above spends ~3 ns per round-0 slot in one CU, so a
// 16k-slot batch took ~50 us. Round 0 only depends on the batch's start
// position, so it runs over the whole chip (walk_round0_kernel: values, and a
// 64-slot rejection mask per wave); one block then orders the rejected slots
// from the masks and runs the refill rounds (walk_refill_kernel), which
// publishes the next batch's start position in pr_dev. Two launches per batch,
// stream-ordered; same walk, same values as the single-block kernel.
constexpr int64_t kWideMin = 4096;
constexpr int kR0Threads = 256;
constexpr int kR0PerThread = 4;   // slots per thread (lane-strided: coalesced)

__global__ __launch_bounds__(kR0Threads) void walk_round0_kernel(
    const int32_t* __restrict__ rl, int64_t L, const int64_t* __restrict__ pr_dev,
    const int64_t* __restrict__ bkeys, int32_t Kb, int64_t total, UsedSet used,
    int64_t key_space, int reject, int64_t* __restrict__ bout, uint64_t* __restrict__ masks,
    int32_t* __restrict__ status) {
  if (status[0] == -3) return;                      // an earlier batch gave up
  const int64_t pr = pr_dev[0] % L;
  const int lane = threadIdx.x & 63;
  const int64_t w0 = ((int64_t)blockIdx.x * (kR0Threads / 64) + (threadIdx.x >> 6)) *
                     kR0PerThread;                  // first 64-slot word of this wave
  int32_t vals[kR0PerThread];
  int64_t keyv[kR0PerThread];
#pragma unroll
  for (int j = 0; j < kR0PerThread; ++j) {
    const int64_t t = (w0 + j) * 64 + lane;
    int64_t pos = pr + t;
    if (pos >= L) pos %= L;
    vals[j] = t < total ? rl[pos] : 0;
    int64_t key = -1;
    if (reject && t < total) {
      key = bkeys[(int32_t)(t % Kb)];
      if (key < 0 || key >= key_space) key = -1;
    }
    keyv[j] = key;
  }
  int bad = 0;
#pragma unroll
  for (int j = 0; j < kR0PerThread; ++j) {
    const int64_t t = (w0 + j) * 64 + lane;
    int rej = 0;
    if (t < total) {
      bout[t] = vals[j];
      if (reject) {
        if (keyv[j] < 0) bad = 1;
        else rej = is_used(used, keyv[j], vals[j]) ? 1 : 0;
      }
    }
    const uint64_t m = __ballot(rej);
    if (lane == 0 && (w0 + j) * 64 < total) masks[w0 + j] = m;
  }
  if (bad) atomicExch(status, -2);
}

__global__ __launch_bounds__(kSampThreads) void walk_refill_kernel(
    const int32_t* __restrict__ rl, int64_t L, int64_t* __restrict__ pr_dev,
    const int64_t* __restrict__ bkeys, int32_t Kb, int64_t total, UsedSet used,
    int64_t key_space, int64_t* __restrict__ bout, const uint64_t* __restrict__ masks,
    int32_t* __restrict__ status, int32_t* __restrict__ rejA_g, int32_t* __restrict__ rejB_g) {
  __shared__ int scan_lds[2][kSampThreads / 64 + 1];
  __shared__ int32_t listA[kListLds];
  __shared__ int32_t listB[kListLds];
  __shared__ int32_t wl[64];
  __shared__ int64_t pr_lds;
  if (status[0] == -3) return;
  int64_t pr = pr_dev[0] % L;
  // count the rejected slots (popcounts of the masks, block-reduced)
  const int64_t n_words = (total + 63) / 64;
  int cnt = 0;
  for (int64_t w = threadIdx.x; w < n_words; w += kSampThreads) cnt += __popcll(masks[w]);
  int nrej;
  block_exclusive_scan(cnt, scan_lds[0], &nrej);
  const bool lds_lists = nrej <= kListLds;
  int32_t* cur = lds_lists ? listA : rejA_g;
  int32_t* nxt = lds_lists ? listB : rejB_g;
  // ascending list: words are taken in order, kSampThreads at a time
  int32_t base = 0;
  for (int64_t w0 = 0; w0 < n_words; w0 += kSampThreads) {
    const int64_t w = w0 + threadIdx.x;
    const uint64_t m = w < n_words ? masks[w] : 0ull;
    int tot;
    int excl = block_exclusive_scan(__popcll(m), scan_lds[1], &tot);
    uint64_t mm = m;
    while (mm) {
      const int b = __ffsll((unsigned long long)mm) - 1;
      cur[base + excl++] = (int32_t)(w * 64 + b);
      mm &= mm - 1;
    }
    base += tot;
  }
  __syncthreads();
  pr = (pr + total) % L;
  auto key_of = [&](int64_t t) -> int64_t {
    const int64_t key = bkeys[(int32_t)(t % Kb)];
    return (key < 0 || key >= key_space) ? -1 : key;
  };
  int livelock = 0;
  walk_refill(rl, L, pr, used, key_of, bout, cur, nxt, nrej, scan_lds, wl, &pr_lds,
              livelock);
  __syncthreads();
  if (threadIdx.x == 0) {
    pr_dev[0] = pr;
    if (livelock) atomicExch(status, -3);
  }
}

// ---- K4s: the walk of a chunk by speculation, exact.
// The walk is sequential only through its pointer: batch b of a chunk starts at
// s_b = s_0 + b * total + R_b, R_b = the refill draws of the batches before it
// (r_b = the values batch b takes beyond its total round-0 slots). Given its start, a
// batch's walk is a pure function of it: r_b(s_b) and its values. So every batch is
// walked at EVERY start it can plausibly have — R in [lo_b, lo_b + W_b), a window the
// host sizes from the sampler's rejection statistics (mirec_sample_walk_spec) — one wave
// per (batch, candidate) in ONE chip-wide launch (walk_spec_kernel: round 0 as 64-slot
// ballots, the refill rounds in the wave, r and the final values of the slots round 0
// rejected kept per candidate). A second launch (walk_commit_kernel) chains the exact
// starts (R_{b+1} = R_b + r_b(R_b), a lookup per batch) and writes each batch's values
// from its chosen candidate. A batch whose start falls outside its window (or whose
// candidate could not be resolved in the wave: too many round-0 rejections, or more than
// kSpecRounds refill rounds) and every batch after it are walked by the single-block
// walk from that exact start — so the result is the serial walk's, bit for bit, always;
// speculation only decides how fast. Up to kSpecMaxBatches batches per launch pair.
constexpr int kSpecMaxBatches = 16;
constexpr int kSpecWaves = 4;            // candidates (waves) per block
constexpr int kSpecMaxTotal = 4096;      // slots per batch (uint16 pending lists)
constexpr int kSpecMaxKeys = 1024;       // keys per batch (LDS)
constexpr int kSpecFinCap = 256;         // round-0 rejections a candidate may resolve
constexpr int kSpecRounds = 64;          // refill rounds a candidate may take
constexpr int kSpecGroup = 16;           // round-0 words with their loads in flight
constexpr int kSpecCommitLds = 6144;     // resolve results the commit stages in LDS

struct SpecPlan {
  int32_t nb;                            // batches
  int32_t lo[kSpecMaxBatches];           // candidates of batch b: R = lo[b] + c, c < W[b]
  int32_t W[kSpecMaxBatches];
  int32_t cand0[kSpecMaxBatches + 1];    // first candidate index of batch b (prefix of W)
  int32_t xblocks;                       // blocks per XCD slice of the resolve grid
  int64_t mbase[kSpecMaxBatches + 1];    // batch b's rejection masks: words from mbase[b]
};

// block g of the spec grid -> (batch, first candidate): batch b's blocks sit on the
// grid positions g = b % 8 (mod 8) — one XCD under the observed round-robin placement,
// so a batch's bitmap rows stay in one L2 (speed only)
__device__ __forceinline__ bool spec_block(const SpecPlan& P, int g, int& b, int& c0) {
  const int x = g & 7;
  int m = g >> 3;
  for (int q = x; q < P.nb; q += 8) {
    const int nbk = (P.W[q] + kSpecWaves - 1) / kSpecWaves;
    if (m < nbk) {
      b = q;
      c0 = m * kSpecWaves;
      return true;
    }
    m -= nbk;
  }
  return false;
}

__device__ __forceinline__ int64_t wrap_pos(int64_t p, int64_t L) { return p < L ? p : p % L; }

// Round 0 of every candidate, key-major (walk_mask_kernel): candidate c of batch b tests
// slot t = j*Kb + k against value rl[s_b + lo_b + c + t] — for a fixed slot the
// candidates read CONSECUTIVE values and one key's used-id row. So one wave per
// (batch, key) runs its num slots with the candidates across its lanes: the value loads
// are coalesced, the membership loads stay inside one bitmap row (a few cache lines),
// and a ballot per 64 candidates writes the slot's rejection bits M[b][t][c / 64].
// (One wave per candidate made 2,048 random row loads per wave: 183 candidates of a
// 4-batch chunk took 34 us.)
__global__ __launch_bounds__(kSpecWaves * 64) void walk_mask_kernel(
    const int32_t* __restrict__ rl, int64_t L, const int64_t* __restrict__ pr_dev,
    const int64_t* __restrict__ keys, int32_t Kb, int32_t num, UsedSet used, int64_t key_space,
    int reject, SpecPlan P, uint64_t* __restrict__ M, int64_t* __restrict__ s0_out) {
  const int64_t s0 = pr_dev[0] % L;
  if (blockIdx.x == 0 && threadIdx.x == 0) s0_out[0] = s0;   // the later launches' start
  const int64_t gw = (int64_t)blockIdx.x * kSpecWaves + (threadIdx.x >> 6);
  const int b = (int)(gw / Kb);
  const int k = (int)(gw - (int64_t)b * Kb);
  if (b >= P.nb) return;                                      // wave-uniform
  const int lane = threadIdx.x & 63;
  const int64_t key = keys[(int64_t)b * Kb + k];
  const bool valid = reject && key >= 0 && key < key_space;
  const int total = Kb * num;
  const int W = P.W[b];
  const int nW = (W + 63) >> 6;
  const int64_t sb = (s0 + (int64_t)b * total + P.lo[b]) % L;
  uint64_t* __restrict__ Mb = M + P.mbase[b];
  // the (j, c) words of this key, kMaskGroup at a time: every value load of the group,
  // then every membership load, then the ballots
  constexpr int kMaskGroup = 16;
  const int nwords = num * nW;
  for (int q0 = 0; q0 < nwords; q0 += kMaskGroup) {
    int32_t v[kMaskGroup];
    bool act[kMaskGroup];
#pragma unroll
    for (int i = 0; i < kMaskGroup; ++i) {
      const int q = q0 + i;
      const int j = q / nW, c = q - j * nW;
      const int d = c * 64 + lane;
      act[i] = valid && q < nwords && d < W;
      v[i] = act[i] ? rl[wrap_pos(sb + j * Kb + k + d, L)] : 0;
    }
    int rej[kMaskGroup];
#pragma unroll
    for (int i = 0; i < kMaskGroup; ++i) rej[i] = act[i] && is_used(used, key, v[i]) ? 1 : 0;
#pragma unroll
    for (int i = 0; i < kMaskGroup; ++i) {
      const int q = q0 + i;
      const uint64_t m = __ballot(rej[i]);
      if (lane == 0 && q < nwords) {
        const int j = q / nW, c = q - j * nW;
        Mb[(int64_t)(j * Kb + k) * nW + c] = m;
      }
    }
  }
}

// Per candidate (one wave): its round-0 rejections from the masks, then its refill rounds.
__global__ __launch_bounds__(kSpecWaves * 64) void walk_spec_kernel(
    const int32_t* __restrict__ rl, int64_t L, const int64_t* __restrict__ s0_in,
    const int64_t* __restrict__ keys, int32_t Kb, int32_t num, UsedSet used, int64_t key_space,
    int reject, SpecPlan P, const uint64_t* __restrict__ M, int32_t* __restrict__ rtab,
    int32_t* __restrict__ n0tab, int2* __restrict__ fin) {
  __shared__ int32_t K[kSpecMaxKeys];
  __shared__ uint16_t lst[kSpecWaves][kSpecMaxTotal];
  const int64_t s0 = s0_in[0];
  int b, c0;
  if (!spec_block(P, blockIdx.x, b, c0)) return;              // block-uniform
  const int64_t* __restrict__ bkeys = keys + (int64_t)b * Kb;
  for (int k = threadIdx.x; k < Kb; k += kSpecWaves * 64) {
    const int64_t key = bkeys[k];
    K[k] = (key < 0 || key >= key_space) ? -1 : (int32_t)key;
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = c0 + wave;
  if (c >= P.W[b]) return;                                    // wave-uniform, no barrier after
  const int cand = P.cand0[b] + c;
  const int total = Kb * num;
  const uint64_t lt = (1ull << lane) - 1ull;
  const int64_t s = (s0 + (int64_t)b * total + P.lo[b] + c) % L;
  uint16_t* __restrict__ l = lst[wave];
  const int nW = (P.W[b] + 63) >> 6;
  const uint64_t* __restrict__ Mb = M + P.mbase[b] + (c >> 6);
  const int cb = c & 63;
  // round 0: the candidate's bit of every slot's mask, kSpecGroup words in flight
  int n0 = 0;
  for (int w0 = 0; w0 * 64 < total; w0 += kSpecGroup) {
    uint64_t mw[kSpecGroup];
#pragma unroll
    for (int i = 0; i < kSpecGroup; ++i) {
      const int t = (w0 + i) * 64 + lane;
      mw[i] = t < total ? Mb[(int64_t)t * nW] : 0ull;
    }
#pragma unroll
    for (int i = 0; i < kSpecGroup; ++i) {
      const int rej = (int)((mw[i] >> cb) & 1ull);
      const uint64_t m = __ballot(rej);
      if (rej) l[n0 + __popcll(m & lt)] = (uint16_t)((w0 + i) * 64 + lane);
      n0 += __popcll(m);
    }
  }
  n0tab[cand] = n0;
  if (n0 > kSpecFinCap) {                                     // left to the serial walk
    if (lane == 0) rtab[cand] = -1;
    return;
  }
  // refill rounds: pending slot i (ascending) takes the i-th next value
  int2* __restrict__ F = fin + (int64_t)cand * kSpecFinCap;
  int n = n0, nfin = 0, rounds = 0;
  int64_t p = wrap_pos(s + total, L);
  int64_t r = 0;
  bool ok = true;
  while (n > 0) {
    if (++rounds > kSpecRounds) { ok = false; break; }
    int nn = 0;
    for (int i0 = 0; i0 < n; i0 += 64) {
      const int i = i0 + lane;
      int rj = 0, acc = 0, t = 0, v = 0;
      if (i < n) {
        t = l[i];
        v = rl[wrap_pos(p + i, L)];
        rj = is_used(used, K[t % Kb], v) ? 1 : 0;
        acc = !rj;
      }
      const uint64_t mr = __ballot(rj), ma = __ballot(acc);
      if (rj) l[nn + __popcll(mr & lt)] = (uint16_t)t;        // in place: nn <= i0
      if (acc) F[nfin + __popcll(ma & lt)] = make_int2(t, v);
      nn += __popcll(mr);
      nfin += __popcll(ma);
    }
    r += n;
    p = wrap_pos(p + n, L);
    n = nn;
  }
  if (lane == 0) rtab[cand] = ok ? (int32_t)r : -1;
}

// Chains the starts, writes every resolved batch (plus the chunk's key rows), and —
// block nb — walks the unresolved tail serially or publishes the next start.
__global__ __launch_bounds__(kSampThreads) void walk_commit_kernel(
    const int32_t* __restrict__ rl, int64_t L, int64_t* __restrict__ pr_dev,
    const int64_t* __restrict__ s0_in, const int64_t* __restrict__ users,
    const int64_t* __restrict__ items, int32_t Kb, int32_t num, UsedSet used, int64_t key_space,
    int reject, SpecPlan P, const int32_t* __restrict__ rtab, const int32_t* __restrict__ n0tab,
    const int2* __restrict__ fin, int64_t* __restrict__ out, int64_t out_stride,
    int64_t* __restrict__ ukeys_dst, int64_t* __restrict__ ikeys_dst, int64_t key_stride,
    int32_t* __restrict__ status, int32_t* __restrict__ rejA_g, int32_t* __restrict__ rejB_g) {
  __shared__ WalkLds S;
  __shared__ int32_t Rs[kSpecMaxBatches + 1];
  __shared__ int s_fail;
  __shared__ int32_t rt[kSpecCommitLds];      // the resolve results (one load level)
  const int b = blockIdx.x;
  const int64_t total = (int64_t)Kb * num;
  const int64_t s0 = s0_in[0];
  // the chunk's key rows (users; positives at the head of each item row): do not depend
  // on the walk
  if (b < P.nb && ukeys_dst) {
    for (int k = threadIdx.x; k < Kb; k += kSampThreads) {
      ukeys_dst[(int64_t)b * Kb + k] = users[(int64_t)b * Kb + k];
      ikeys_dst[(int64_t)b * key_stride + k] = items[(int64_t)b * Kb + k];
    }
  }
  const int ncand = P.cand0[P.nb];
  const bool lds_rt = ncand <= kSpecCommitLds;
  if (lds_rt)
    for (int i = threadIdx.x; i < ncand; i += kSampThreads) rt[i] = rtab[i];
  __syncthreads();
  if (threadIdx.x == 0) {                     // chain the starts (a lookup per batch)
    int32_t R = 0;
    int f = P.nb;
    for (int q = 0; q < P.nb; ++q) {
      const int idx = R - P.lo[q];
      const int32_t rq = (idx >= 0 && idx < P.W[q])
                             ? (lds_rt ? rt[P.cand0[q] + idx] : rtab[P.cand0[q] + idx]) : -1;
      Rs[q] = R;
      if (rq < 0) { f = q; break; }
      R += rq;
    }
    if (f == P.nb) Rs[P.nb] = R;
    s_fail = f;
  }
  __syncthreads();
  const int f = s_fail;
  if (b < P.nb) {
    if (b >= f) return;                       // the tail block walks it
    const int64_t sb = (s0 + (int64_t)b * total + Rs[b]) % L;
    const int cand = P.cand0[b] + (Rs[b] - P.lo[b]);
    int64_t* __restrict__ bout = out + (int64_t)b * out_stride;
    int bad = 0;
    for (int64_t t = threadIdx.x; t < total; t += kSampThreads) {
      bout[t] = rl[wrap_pos(sb + t, L)];
      if (reject) {
        const int64_t key = users[(int64_t)b * Kb + t % Kb];
        bad |= (key < 0 || key >= key_space) ? 1 : 0;
      }
    }
    if (bad) atomicExch(status, -2);
    __syncthreads();                          // round-0 values before the refilled ones
    const int n0 = n0tab[cand];
    const int2* __restrict__ F = fin + (int64_t)cand * kSpecFinCap;
    for (int i = threadIdx.x; i < n0; i += kSampThreads) bout[F[i].x] = F[i].y;
    return;
  }
  // block nb: the unresolved tail, or the next start
  if (f == P.nb) {
    if (threadIdx.x == 0) pr_dev[0] = (s0 + (int64_t)P.nb * total + Rs[P.nb]) % L;
    return;
  }
  int64_t pr = (s0 + (int64_t)f * total + Rs[f]) % L;
  int bad_key = 0, livelock = 0;
  walk_serial(rl, L, pr, users, (int64_t)P.nb * Kb, Kb, f, P.nb, num, used, key_space, reject,
              out, out_stride, rejA_g, rejB_g, nullptr, S, bad_key, livelock);
  if (bad_key) atomicExch(status, -2);
  if (livelock && threadIdx.x == 0) atomicExch(status, -3);
  __syncthreads();
  if (threadIdx.x == 0) pr_dev[0] = pr;
}

// bits[key, v>>5] |= 1 << (v & 31) for every used id; one wave per key.
__global__ __launch_bounds__(256) void used_bitmap_kernel(const int64_t* __restrict__ ptr,
                                                          const int32_t* __restrict__ cols,
                                                          int64_t n_keys, int64_t words,
                                                          int64_t nbits,
                                                          uint32_t* __restrict__ bits) {
  const int64_t key = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (key >= n_keys) return;
  const int64_t j1 = ptr[key + 1];
  for (int64_t j = ptr[key] + (threadIdx.x & 63); j < j1; j += 64) {
    const int32_t v = cols[j];
    if ((uint64_t)(uint32_t)v < (uint64_t)nbits)
      atomicOr(&bits[key * words + (v >> 5)], 1u << (v & 31));
  }
}

// ---- alias-table fast mode (labelled non-parity; include/mirec.h mirec_sample_alias)
// Each draw is independent: one lane per (batch, j, k) slot, counter-based
// random bits (splitmix64 of seed and draw id), Walker/Vose column + threshold,
// rejection by redrawing with the next attempt number. No serial walk, so a
// whole chunk of batches is one wide launch.
constexpr int kAliasTries = 4096;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ int32_t alias_draw(const uint32_t* __restrict__ thr,
                                              const int32_t* __restrict__ alias, uint64_t n_cols,
                                              uint64_t seed, uint64_t id, uint32_t attempt) {
  const uint64_t r = mix64(seed ^ mix64(id * (uint64_t)kAliasTries + attempt));
  const uint32_t col = (uint32_t)(((r >> 32) * n_cols) >> 32);   // multiply-shift, < n_cols
  return (uint32_t)r < __ldg(thr + col) ? (int32_t)col : __ldg(alias + col);
}

__global__ __launch_bounds__(256) void alias_sample_kernel(
    const uint32_t* __restrict__ thr, const int32_t* __restrict__ alias, uint64_t n_cols,
    uint64_t seed, uint64_t counter, const int64_t* __restrict__ keys, int64_t n_keys,
    int64_t batch_keys, int64_t num, UsedSet u, int64_t n_key_space, int reject,
    int64_t* __restrict__ out, int64_t out_stride, int32_t* __restrict__ status) {
  const int64_t total = n_keys * num;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * blockDim.x) {
    // g enumerates batches in order, slot j*Kb + k inside a batch
    const int64_t b = g / (batch_keys * num);
    const int64_t k0 = b * batch_keys;
    const int64_t Kb = min(batch_keys, n_keys - k0);
    const int64_t s = g - k0 * num;
    const int64_t k = s % Kb;
    const int64_t key = keys[k0 + k];
    const uint64_t id = counter + (uint64_t)g;
    if (key < 0 || key >= n_key_space) {
      atomicExch(status, -2);
      out[b * out_stride + s] = 0;
      continue;
    }
    int32_t v = alias_draw(thr, alias, n_cols, seed, id, 0);
    if (reject) {
      uint32_t a = 1;
      for (; is_used(u, key, v) && a < (uint32_t)kAliasTries; ++a)
        v = alias_draw(thr, alias, n_cols, seed, id, a);
      if (a == (uint32_t)kAliasTries && is_used(u, key, v)) atomicExch(status, -3);
    }
    out[b * out_stride + s] = v;
  }
}

}  // namespace mirec

using namespace mirec;

#ifdef MIREC_WALK_PROF
extern "C" int mirec_walk_prof(unsigned long long* out16, int reset) {
  if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_walk_prof), sizeof(unsigned long long) * 16) !=
      hipSuccess) return -1;
  if (reset) {
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_walk_prof), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

extern "C" size_t mirec_sample_walk_workspace_size(int64_t batch_keys, int64_t num) {
  if (batch_keys <= 0 || num <= 0) return 256;
  const int64_t total = batch_keys * num;
  return (size_t)(2 * total) * sizeof(int32_t) + (size_t)((total + 63) / 64 + 1) * 8 + 256;
}

extern "C" size_t mirec_used_bitmap_bytes(int64_t n_keys, int64_t n_bits) {
  if (n_keys <= 0 || n_bits <= 0) return 0;
  return (size_t)n_keys * (size_t)((n_bits + 31) / 32) * sizeof(uint32_t);
}

extern "C" int mirec_used_bitmap_build(const int64_t* used_ptr, const int32_t* used_cols,
                                       int64_t n_keys, int64_t n_bits, uint32_t* bits,
                                       void* stream) {
  if (!used_ptr || !used_cols || !bits || n_keys < 0 || n_bits <= 0) {
    set_error("mirec_used_bitmap_build: bad arguments");
    return -1;
  }
  if (n_keys == 0) return 0;
  const int64_t words = (n_bits + 31) / 32;
  hipStream_t st = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(bits, 0, (size_t)n_keys * words * sizeof(uint32_t), st);
  if (e != hipSuccess) return hip_status(e, "mirec_used_bitmap_build: memset");
  hipLaunchKernelGGL(used_bitmap_kernel, dim3((unsigned)((n_keys + 3) / 4)), dim3(256), 0, st,
                     used_ptr, used_cols, n_keys, words, n_bits, bits);
  return launch_status("mirec_used_bitmap_build");
}

extern "C" int mirec_sample_walk(const int32_t* random_list, int64_t L, int64_t* pr_dev,
                                 const int64_t* keys, int64_t n_keys, int64_t batch_keys,
                                 int64_t n_batches, int64_t num, const int64_t* used_ptr,
                                 const int32_t* used_cols, const uint32_t* used_bits,
                                 int64_t n_bits, int64_t n_key_space, int reject, int64_t* out,
                                 int64_t out_stride, int32_t* status_dev, void* ws,
                                 size_t ws_bytes, void* stream) {
  if (L <= 0 || !random_list || !pr_dev || !out || !status_dev || n_keys < 0 || num < 0 ||
      batch_keys <= 0 || n_batches < 0) {
    set_error("mirec_sample_walk: bad arguments (L=%lld)", (long long)L);
    return -1;
  }
  if (n_keys == 0 || num == 0 || n_batches == 0) return 0;
  if (reject && ((!used_ptr || !used_cols) && !used_bits)) {
    set_error("mirec_sample_walk: reject=1 needs the used-id CSR or bitmap");
    return -1;
  }
  if (used_bits && n_bits <= 0) {
    set_error("mirec_sample_walk: bitmap needs n_bits > 0");
    return -1;
  }
  if (batch_keys * num > INT32_MAX) {
    set_error("mirec_sample_walk: batch_keys*num exceeds int32");
    return -1;
  }
  const size_t need = mirec_sample_walk_workspace_size(batch_keys, num);
  if (!ws || ws_bytes < need) {
    set_error("mirec_sample_walk: workspace %zu < %zu", ws_bytes, need);
    return -1;
  }
  if (out_stride == 0) out_stride = batch_keys * num;
  int32_t* rejA = (int32_t*)ws;
  int32_t* rejB = rejA + batch_keys * num;
  UsedSet u;
  u.ptr = used_ptr;
  u.cols = used_cols;
  u.bits = used_bits;
  u.nbits = n_bits;
  u.words = used_bits ? (n_bits + 31) / 32 : 0;
  hipStream_t st = (hipStream_t)stream;
  if (batch_keys * num <= kWideMin) {
    hipLaunchKernelGGL(sample_walk_kernel, dim3(1), dim3(kSampThreads), 0, st, random_list, L,
                       pr_dev, keys, n_keys, batch_keys, n_batches, num, u, n_key_space, reject,
                       out, out_stride, status_dev, rejA, rejB, (const int64_t*)nullptr);
    return launch_status("mirec_sample_walk");
  }
  // 8-byte aligned mask words after the two lists
  uint64_t* masks = (uint64_t*)(((uintptr_t)(rejB + batch_keys * num) + 7) & ~(uintptr_t)7);
  for (int64_t b = 0; b < n_batches; ++b) {
    const int64_t k0 = b * batch_keys;
    const int64_t Kb = min(batch_keys, n_keys - k0);
    if (Kb <= 0) break;
    const int64_t total = Kb * num;
    const int64_t words = (total + 63) / 64;
    const unsigned blocks =
        (unsigned)((words + (kR0Threads / 64) * kR0PerThread - 1) / ((kR0Threads / 64) * kR0PerThread));
    hipLaunchKernelGGL(walk_round0_kernel, dim3(blocks), dim3(kR0Threads), 0, st, random_list, L,
                       pr_dev, keys + k0, (int32_t)Kb, total, u, n_key_space, reject,
                       out + b * out_stride, masks, status_dev);
    hipLaunchKernelGGL(walk_refill_kernel, dim3(1), dim3(kSampThreads), 0, st, random_list, L,
                       pr_dev, keys + k0, (int32_t)Kb, total, u, n_key_space, out + b * out_stride,
                       masks, status_dev, rejA, rejB);
  }
  return launch_status("mirec_sample_walk");
}

// ---- K4s host side
namespace {
struct SpecShape {
  SpecPlan P;
  int64_t cands;
};

// Windows of a sub-chunk of nb batches: R_b in b*mean -+ (z*sd*sqrt(b) + slack). The
// statistics only size the windows (a miss costs speed, never exactness).
SpecShape spec_plan(int nb, double mean, double sd) {
  SpecShape sh;
  memset(&sh, 0, sizeof(sh));
  sh.P.nb = nb;
  const double z = 4.5;
  int64_t c = 0;
  for (int b = 0; b < nb; ++b) {
    int64_t lo = 0, hi = 0;
    if (b > 0 && (mean > 0.0 || sd > 0.0)) {
      const double half = z * sd * sqrt((double)b) + 3.0;
      lo = (int64_t)floor(b * mean - half);
      hi = (int64_t)ceil(b * mean + half);
      if (lo < 0) lo = 0;
      if (hi < lo) hi = lo;
    }
    sh.P.lo[b] = (int32_t)lo;
    sh.P.W[b] = (int32_t)(hi - lo + 1);
    sh.P.cand0[b] = (int32_t)c;
    c += hi - lo + 1;
  }
  sh.P.cand0[nb] = (int32_t)c;
  int xb = 0;
  for (int x = 0; x < 8; ++x) {
    int m = 0;
    for (int q = x; q < nb; q += 8) m += (sh.P.W[q] + kSpecWaves - 1) / kSpecWaves;
    xb = std::max(xb, m);
  }
  sh.P.xblocks = xb;
  sh.cands = c;
  return sh;
}

// rejection-mask words of a plan (walk_mask_kernel), and each batch's base
int64_t spec_masks(SpecPlan& P, int64_t total) {
  int64_t w = 0;
  for (int b = 0; b < P.nb; ++b) {
    P.mbase[b] = w;
    w += total * ((P.W[b] + 63) / 64);
  }
  P.mbase[P.nb] = w;
  return w;
}
}  // namespace

extern "C" size_t mirec_sample_walk_spec_workspace_size(int64_t batch_keys, int64_t num,
                                                        int64_t max_batches, double r_mean,
                                                        double r_sd) {
  if (batch_keys <= 0 || num <= 0 || max_batches <= 0) return 256;
  const int nb = (int)std::min<int64_t>(max_batches, kSpecMaxBatches);
  SpecShape sh = spec_plan(nb, r_mean, r_sd);
  const int64_t masks = spec_masks(sh.P, batch_keys * num);
  // serial-walk lists | s0 | rtab | n0tab | fin | masks
  return mirec_sample_walk_workspace_size(batch_keys, num) + 16 + (size_t)sh.cands * 8 +
         (size_t)sh.cands * kSpecFinCap * sizeof(int2) + (size_t)masks * 8 + 512;
}

extern "C" int mirec_sample_walk_spec(const int32_t* random_list, int64_t L, int64_t* pr_dev,
                                      const int64_t* users, const int64_t* items,
                                      int64_t n_batches, int64_t batch_keys, int64_t num,
                                      const int64_t* used_ptr, const int32_t* used_cols,
                                      const uint32_t* used_bits, int64_t n_bits,
                                      int64_t n_key_space, int reject, double r_mean,
                                      double r_sd, int64_t* out, int64_t out_stride,
                                      int64_t* user_keys, int64_t* item_keys, int64_t key_stride,
                                      int32_t* status_dev, void* ws, size_t ws_bytes,
                                      void* stream) {
  const char* what = "mirec_sample_walk_spec";
  if (L <= 0 || !random_list || !pr_dev || !users || !out || !status_dev || n_batches < 0 ||
      batch_keys <= 0 || num <= 0 || !(r_mean >= 0.0) || !(r_sd >= 0.0) ||
      (!user_keys) != (!item_keys) || (user_keys && (!items || key_stride < batch_keys))) {
    set_error("%s: bad arguments", what);
    return -1;
  }
  if (n_batches == 0) return 0;
  if (batch_keys > kSpecMaxKeys || batch_keys * num > kSpecMaxTotal) {
    set_error("%s: batch of %lld keys x %lld exceeds the speculative walk's %d keys / %d slots",
              what, (long long)batch_keys, (long long)num, kSpecMaxKeys, kSpecMaxTotal);
    return -1;
  }
  if (reject && ((!used_ptr || !used_cols) && !used_bits)) {
    set_error("%s: reject=1 needs the used-id CSR or bitmap", what);
    return -1;
  }
  const int nbmax = (int)std::min<int64_t>(n_batches, kSpecMaxBatches);
  const size_t need = mirec_sample_walk_spec_workspace_size(batch_keys, num, nbmax, r_mean, r_sd);
  if (!ws || ws_bytes < need) {
    set_error("%s: workspace %zu < %zu", what, ws_bytes, need);
    return -1;
  }
  if (out_stride == 0) out_stride = batch_keys * num;
  UsedSet u;
  u.ptr = used_ptr;
  u.cols = used_cols;
  u.bits = used_bits;
  u.nbits = n_bits;
  u.words = used_bits ? (n_bits + 31) / 32 : 0;
  const int64_t total = batch_keys * num;
  int32_t* rejA = (int32_t*)ws;
  int32_t* rejB = rejA + total;
  char* q = (char*)ws + mirec_sample_walk_workspace_size(batch_keys, num);
  q = (char*)(((uintptr_t)q + 15) & ~(uintptr_t)15);
  int64_t* s0 = (int64_t*)q;
  q += 16;
  hipStream_t st = (hipStream_t)stream;
  for (int64_t b0 = 0; b0 < n_batches; b0 += kSpecMaxBatches) {
    const int nb = (int)std::min<int64_t>(kSpecMaxBatches, n_batches - b0);
    SpecShape sh = spec_plan(nb, r_mean, r_sd);
    spec_masks(sh.P, total);
    int32_t* rtab = (int32_t*)q;
    int32_t* n0tab = rtab + sh.cands;
    int2* fin = (int2*)(((uintptr_t)(n0tab + sh.cands) + 15) & ~(uintptr_t)15);
    uint64_t* masks = (uint64_t*)(fin + sh.cands * kSpecFinCap);
    const int64_t* ub = users + b0 * batch_keys;
    const int64_t mwaves = (int64_t)nb * batch_keys;
    hipLaunchKernelGGL(walk_mask_kernel, dim3((unsigned)((mwaves + kSpecWaves - 1) / kSpecWaves)),
                       dim3(kSpecWaves * 64), 0, st, random_list, L, pr_dev, ub,
                       (int32_t)batch_keys, (int32_t)num, u, n_key_space, reject, sh.P, masks,
                       s0);
    int rc = launch_status(what);
    if (rc) return rc;
    hipLaunchKernelGGL(walk_spec_kernel, dim3((unsigned)(8 * sh.P.xblocks)),
                       dim3(kSpecWaves * 64), 0, st, random_list, L, s0, ub,
                       (int32_t)batch_keys, (int32_t)num, u, n_key_space, reject, sh.P, masks,
                       rtab, n0tab, fin);
    rc = launch_status(what);
    if (rc) return rc;
    hipLaunchKernelGGL(walk_commit_kernel, dim3((unsigned)(nb + 1)), dim3(kSampThreads), 0, st,
                       random_list, L, pr_dev, s0, ub, items ? items + b0 * batch_keys : nullptr,
                       (int32_t)batch_keys, (int32_t)num, u, n_key_space, reject, sh.P, rtab,
                       n0tab, fin, out + b0 * out_stride, out_stride,
                       user_keys ? user_keys + b0 * batch_keys : nullptr,
                       item_keys ? item_keys + b0 * key_stride : nullptr, key_stride, status_dev,
                       rejA, rejB);
    rc = launch_status(what);
    if (rc) return rc;
  }
  return 0;
}

// Vose's alias method in exact integer arithmetic: column capacity W = sum(counts),
// item weight counts[i] * n; a small column s keeps floor(w_s * 2^32 / W) of its
// 2^32 threshold units for itself and gives the rest to a large column l, whose
// remaining weight drops by W - w_s (exact, so the last columns hold exactly W and
// become full: threshold 2^32 - 1, alias = itself). Host-side table setup.
extern "C" int mirec_alias_build(const int64_t* counts, int64_t n, uint32_t* thr, int32_t* alias) {
  if (!counts || !thr || !alias || n <= 0 || n > (int64_t)UINT32_MAX) {
    set_error("mirec_alias_build: bad arguments");
    return -1;
  }
  unsigned __int128 W = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (counts[i] < 0) {
      set_error("mirec_alias_build: negative count at %lld", (long long)i);
      return -1;
    }
    W += (unsigned __int128)counts[i];
  }
  if (W == 0) {
    set_error("mirec_alias_build: all counts are zero");
    return -1;
  }
  std::vector<unsigned __int128> w((size_t)n);
  std::vector<int64_t> small, large;
  small.reserve((size_t)n);
  large.reserve((size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    w[(size_t)i] = (unsigned __int128)counts[i] * (unsigned __int128)n;
    (w[(size_t)i] < W ? small : large).push_back(i);
  }
  while (!small.empty() && !large.empty()) {
    const int64_t s = small.back(), l = large.back();
    small.pop_back();
    thr[s] = (uint32_t)((w[(size_t)s] << 32) / W);
    alias[s] = (int32_t)l;
    w[(size_t)l] -= W - w[(size_t)s];
    if (w[(size_t)l] < W) {
      large.pop_back();
      small.push_back(l);
    }
  }
  for (int64_t i : large) { thr[i] = UINT32_MAX; alias[i] = (int32_t)i; }
  for (int64_t i : small) { thr[i] = UINT32_MAX; alias[i] = (int32_t)i; }  // unreachable in exact arithmetic
  return 0;
}

extern "C" int mirec_sample_alias(const uint32_t* thr, const int32_t* alias, int64_t n_cols,
                                  uint64_t seed, uint64_t counter, const int64_t* keys,
                                  int64_t n_keys, int64_t batch_keys, int64_t num,
                                  const int64_t* used_ptr, const int32_t* used_cols,
                                  const uint32_t* used_bits, int64_t n_bits, int64_t n_key_space,
                                  int reject, int64_t* out, int64_t out_stride,
                                  int32_t* status_dev, void* stream) {
  if (!thr || !alias || n_cols <= 0 || n_cols > (int64_t)UINT32_MAX || !out || !status_dev ||
      n_keys < 0 || num < 0 || batch_keys <= 0 || (n_keys > 0 && !keys)) {
    set_error("mirec_sample_alias: bad arguments");
    return -1;
  }
  if (n_keys == 0 || num == 0) return 0;
  if (reject && ((!used_ptr || !used_cols) && !used_bits)) {
    set_error("mirec_sample_alias: reject=1 needs the used-id CSR or bitmap");
    return -1;
  }
  if (used_bits && n_bits <= 0) {
    set_error("mirec_sample_alias: bitmap needs n_bits > 0");
    return -1;
  }
  if (out_stride == 0) out_stride = batch_keys * num;
  if (out_stride < min(batch_keys, n_keys) * num) {
    set_error("mirec_sample_alias: out_stride %lld < batch values", (long long)out_stride);
    return -1;
  }
  UsedSet u;
  u.ptr = used_ptr;
  u.cols = used_cols;
  u.bits = used_bits;
  u.nbits = n_bits;
  u.words = used_bits ? (n_bits + 31) / 32 : 0;
  const int64_t total = n_keys * num;
  const unsigned blocks = (unsigned)std::min<int64_t>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(alias_sample_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, thr,
                     alias, (uint64_t)n_cols, seed, counter, keys, n_keys, batch_keys, num, u,
                     n_key_space, reject, out, out_stride, status_dev);
  return launch_status("mirec_sample_alias");
}

// Many consecutive sample_by_key_ids calls of different sizes in one launch: call
// s samples `num` values for keys[seg_ptr[s] .. seg_ptr[s+1]) (its values packed
// at out + seg_ptr[s] * num, layout j * K_s + k), in call order — the walk pointer
// continues from call to call exactly as the reference's successive calls do
// (GeneralNegSampleDataLoader._next_batch_data in evaluation: one call per user,
// general_dataloader.py:210-221). seg_ptr is a DEVICE int64 [n_seg + 1];
// max_seg_keys bounds K_s (workspace = mirec_sample_walk_workspace_size(max_seg_keys, num)).
extern "C" int mirec_sample_walk_segments(const int32_t* random_list, int64_t L, int64_t* pr_dev,
                                          const int64_t* keys, const int64_t* seg_ptr,
                                          int64_t n_seg, int64_t max_seg_keys, int64_t num,
                                          const int64_t* used_ptr, const int32_t* used_cols,
                                          const uint32_t* used_bits, int64_t n_bits,
                                          int64_t n_key_space, int reject, int64_t* out,
                                          int32_t* status_dev, void* ws, size_t ws_bytes,
                                          void* stream) {
  if (L <= 0 || !random_list || !pr_dev || !out || !status_dev || !seg_ptr || n_seg < 0 ||
      num < 0 || max_seg_keys < 0 || (n_seg > 0 && !keys)) {
    set_error("mirec_sample_walk_segments: bad arguments (L=%lld)", (long long)L);
    return -1;
  }
  if (n_seg == 0 || num == 0 || max_seg_keys == 0) return 0;
  if (reject && ((!used_ptr || !used_cols) && !used_bits)) {
    set_error("mirec_sample_walk_segments: reject=1 needs the used-id CSR or bitmap");
    return -1;
  }
  if (used_bits && n_bits <= 0) {
    set_error("mirec_sample_walk_segments: bitmap needs n_bits > 0");
    return -1;
  }
  if (max_seg_keys * num > INT32_MAX) {
    set_error("mirec_sample_walk_segments: max_seg_keys*num exceeds int32");
    return -1;
  }
  const size_t need = mirec_sample_walk_workspace_size(max_seg_keys, num);
  if (!ws || ws_bytes < need) {
    set_error("mirec_sample_walk_segments: workspace %zu < %zu", ws_bytes, need);
    return -1;
  }
  int32_t* rejA = (int32_t*)ws;
  int32_t* rejB = rejA + max_seg_keys * num;
  UsedSet u;
  u.ptr = used_ptr;
  u.cols = used_cols;
  u.bits = used_bits;
  u.nbits = n_bits;
  u.words = used_bits ? (n_bits + 31) / 32 : 0;
  hipLaunchKernelGGL(sample_walk_kernel, dim3(1), dim3(kSampThreads), 0, (hipStream_t)stream,
                     random_list, L, pr_dev, keys, (int64_t)0, max_seg_keys, n_seg, num, u,
                     n_key_space, reject, out, (int64_t)0, status_dev, rejA, rejB, seg_ptr);
  return launch_status("mirec_sample_walk_segments");
}
