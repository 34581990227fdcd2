// K2 — deterministic grouping of gradient contributions by table row.
//
// torch's nn.Embedding(sparse=False) backward (bpr.py:40-41) zero-fills a dense
// [n_rows, d] gradient and index_adds every looked-up row into it.  Here the
// contributions are grouped instead: a stable LSD radix sort of (row id,
// contribution index) gives, per distinct row, the ordered list of its
// contributions, which K5 (adam.hip) or the dense scatter below sums in that
// fixed order — bitwise reproducible, no float atomics.
//
// The sort runs in ONE workgroup (512 lanes): n is a training batch's
// contribution count (C2: 512 user keys, 2,560 item keys), far too small to
// fill the chip, and the sort depends only on ids, so the trainer runs it
// ahead of the model step on a side stream.  Up to kLdsMax keys the whole
// sort lives in LDS (stable kDigitBits-bit digit passes, packed per-thread digit
// counts, one block scan per pass). Larger batches: one large batch takes a
// device-wide LSD radix sort (upsweep histograms, scan, stable downsweep), several
// take one workgroup each over global ping-pong buffers (1-bit stable splits).
#include "common.h"
#include "ahead.h"

namespace mirec {

#ifndef MIREC_SORT_THREADS
#define MIREC_SORT_THREADS 512
#endif
// 512 lanes: each 4-bit pass pays a fixed cross-wave cost (wave scan, per-wave totals,
// two barriers) that grows with the wave count — one C2 batch (512 user keys / 2,560 item
// keys) sorts in 14.7 / 20.3 us with 8 waves against 27.1 / 29.1 us with 16
// (tools/probe_segsort.py, variants by tools/build_variant.sh -DMIREC_SORT_THREADS=N).
constexpr int kSortThreads = MIREC_SORT_THREADS;
#ifndef MIREC_SORT_DIGIT_BITS
#define MIREC_SORT_DIGIT_BITS 4
#endif
constexpr int kDigitBits = MIREC_SORT_DIGIT_BITS;      // radix digit width of the LDS sort
constexpr int kDigitWords = (1 << kDigitBits) / 4;     // four 16-bit counters per 64-bit word
constexpr int kLdsMax = 8192;
constexpr int kIpt = kLdsMax / kSortThreads;  // items per thread in the LDS path
// knobs of the probing builds (tools/build_variant.sh): digits of 2..6 bits (kDigitWords
// packed words of four 16-bit counters each), whole waves dividing the LDS capacity
static_assert(kDigitBits >= 2 && kDigitBits <= 6, "MIREC_SORT_DIGIT_BITS must be in [2, 6]");
static_assert(kSortThreads % 64 == 0 && kSortThreads <= 1024 && kLdsMax % kSortThreads == 0,
              "MIREC_SORT_THREADS: a multiple of 64, at most 1024, dividing kLdsMax");

__host__ __device__ __forceinline__ int nbits_for(int64_t key_space) {
  int b = 0;
  while (b < 31 && ((int64_t)1 << b) < key_space) ++b;
  return b;
}

// uniq/seg from sorted keys held in `skey` (LDS or global), blocked arrangement
template <typename KeyPtr>
__device__ void emit_segments(KeyPtr skey, int n, int32_t* __restrict__ uniq,
                              int32_t* __restrict__ seg, int32_t* __restrict__ n_uniq,
                              int* scan_lds) {
  int base_u = 0;
  for (int c0 = 0; c0 < n; c0 += kSortThreads) {
    const int i = c0 + threadIdx.x;
    int f = 0;
    int32_t kv = 0;
    if (i < n) {
      kv = skey[i];
      f = (i == 0 || skey[i - 1] != kv) ? 1 : 0;
    }
    int tot;
    const int ex = block_exclusive_scan(f, scan_lds, &tot);
    if (f) {
      uniq[base_u + ex] = kv;
      seg[base_u + ex] = i;
    }
    base_u += tot;
  }
  if (threadIdx.x == 0) {
    seg[base_u] = n;
    n_uniq[0] = base_u;
  }
}

// One workgroup per batch: batch b sorts keys[b*batch_n, min((b+1)*batch_n, n_total))
// and writes perm/uniq at b*batch_n, seg at b*(batch_n+1), n_uniq[b].
struct SortLds {
  int32_t kA[kLdsMax], vA[kLdsMax], kB[kLdsMax], vB[kLdsMax];
  int scan[kSortThreads / 64 + 1];
  uint64_t wtot[kSortThreads / 64][kDigitWords];  // per-wave packed digit counts
};
// the two-job kernel (segsort_lds2_kernel) holds one SortLds; gfx950 has 160 KiB per CU
static_assert(sizeof(SortLds) <= 160 * 1024, "SortLds exceeds the gfx950 LDS");

__device__ __forceinline__ void segsort_lds_batch(
    const int64_t* __restrict__ keys_all, int64_t n_total, int batch_n, int nbits,
    int32_t* __restrict__ perm_all, int32_t* __restrict__ uniq_all,
    int32_t* __restrict__ seg_all, int32_t* __restrict__ n_uniq_all, int64_t b, SortLds& L) {
  int32_t* kA = L.kA;
  int32_t* vA = L.vA;
  int32_t* kB = L.kB;
  int32_t* vB = L.vB;
  int* scan_lds = L.scan;
  const int n = (int)min((int64_t)batch_n, n_total - b * batch_n);
  const int64_t* __restrict__ keys = keys_all + b * batch_n;
  int32_t* __restrict__ perm = perm_all + b * batch_n;
  int32_t* __restrict__ uniq = uniq_all + b * batch_n;
  int32_t* __restrict__ seg = seg_all + b * (batch_n + 1);
  int32_t* __restrict__ n_uniq = n_uniq_all + b;
  for (int i = threadIdx.x; i < n; i += kSortThreads) {
    kA[i] = (int32_t)keys[i];
    vA[i] = i;
  }
  __syncthreads();
  int32_t *ks = kA, *vs = vA, *kd = kB, *vd = vB;
  const int ipt = (n + kSortThreads - 1) / kSortThreads;
  const int lo = threadIdx.x * ipt;
  const int hi = min(n, lo + ipt);
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  constexpr int nw = kSortThreads / 64;  // every launch of these kernels: kSortThreads lanes
  // Stable LSD passes of kDigitBits-bit digits (a blocked arrangement: thread t owns
  // positions [lo, hi)). Per-digit counts travel packed, four 16-bit fields per
  // 64-bit word (n <= 8192 < 2^16: no carries), so one wave scan of kDigitWords words
  // and one barrier give every thread its per-digit exclusive prefix; the
  // destination of an item is (items of smaller digits) + (items of its digit
  // before it) — the same permutation as 1-bit splits, in 1/kDigitBits of the
  // passes.
  for (int shift = 0; shift < nbits; shift += kDigitBits) {
    constexpr int kMask = (1 << kDigitBits) - 1;
    uint64_t c[kDigitWords];
#pragma unroll
    for (int w = 0; w < kDigitWords; ++w) c[w] = 0ull;
    for (int i = lo; i < hi; ++i) {
      const int d = (ks[i] >> shift) & kMask;
#pragma unroll
      for (int w = 0; w < kDigitWords; ++w) c[w] += (d >> 2) == w ? 1ull << (16 * (d & 3)) : 0ull;
    }
    uint64_t inc[kDigitWords];
#pragma unroll
    for (int w = 0; w < kDigitWords; ++w) inc[w] = c[w];
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
#pragma unroll
      for (int w = 0; w < kDigitWords; ++w) {
        const uint64_t y = __shfl_up(inc[w], off, 64);
        if (lane >= off) inc[w] += y;
      }
    }
    if (lane == 63) {
#pragma unroll
      for (int w = 0; w < kDigitWords; ++w) L.wtot[wid][w] = inc[w];
    }
    __syncthreads();
    uint64_t ex[kDigitWords], tot[kDigitWords];
#pragma unroll
    for (int w = 0; w < kDigitWords; ++w) { ex[w] = inc[w] - c[w]; tot[w] = 0ull; }
#pragma unroll
    for (int v = 0; v < nw; ++v) {
#pragma unroll
      for (int w = 0; w < kDigitWords; ++w) {
        const uint64_t x = L.wtot[v][w];
        ex[w] += v < wid ? x : 0ull;
        tot[w] += x;
      }
    }
    auto fsum = [](uint64_t x) {     // sum of the four 16-bit fields
      return (int)((x & 0xffff) + ((x >> 16) & 0xffff) + ((x >> 32) & 0xffff) + (x >> 48));
    };
    for (int i = lo; i < hi; ++i) {
      const int32_t kv = ks[i];
      const int d = (kv >> shift) & kMask;
      const int w = d >> 2, f = 16 * (d & 3);
      int base = 0;
      uint64_t e = 0ull;
#pragma unroll
      for (int q = 0; q < kDigitWords; ++q) {
        base += q < w ? fsum(tot[q]) : 0;
        if (q == w) {
          base += fsum(tot[q] & ((1ull << f) - 1ull));
          e = ex[q];
          ex[q] += 1ull << f;
        }
      }
      const int dst = base + (int)((e >> f) & 0xffff);
      kd[dst] = kv;
      vd[dst] = vs[i];
    }
    __syncthreads();
    int32_t* t;
    t = ks; ks = kd; kd = t;
    t = vs; vs = vd; vd = t;
  }
  for (int i = threadIdx.x; i < n; i += kSortThreads) perm[i] = vs[i];
  emit_segments(ks, n, uniq, seg, n_uniq, scan_lds);
}

__global__ __launch_bounds__(kSortThreads) void segsort_lds_kernel(
    const int64_t* __restrict__ keys_all, int64_t n_total, int batch_n, int nbits,
    int32_t* __restrict__ perm_all, int32_t* __restrict__ uniq_all,
    int32_t* __restrict__ seg_all, int32_t* __restrict__ n_uniq_all) {
  __shared__ SortLds L;
  segsort_lds_batch(keys_all, n_total, batch_n, nbits, perm_all, uniq_all, seg_all, n_uniq_all,
                    blockIdx.x, L);
}

// Per-block stable sort for blocks of <= kR8Max keys whatever the key space or the
// duplicates (DeepFM's field blocks: 2,048 ids of up to 10 M rows, Zipf heads and
// small-vocabulary fields alike): LSD passes of 8-bit digits over (key - the block's
// minimum) — ceil(bits of the block's key span / 8) passes instead of 4-bit passes over
// the table's id width. Wave w owns a contiguous run of 64-key chunks; in each chunk the
// 8 digit-bit ballots intersect to every lane's set of same-digit lanes, so a key's rank
// is (its digit's count in the wave's earlier chunks, an LDS counter [digit][wave] the
// digit's leader lane advances) + (same-digit lanes below it). One block scan of the
// 256 x 8 counters (digit-major) gives every (digit, wave) its output offset — stable,
// no atomics. Same perm / uniq / seg / n_uniq as segsort_lds_batch.
#ifndef MIREC_R8_THREADS
#define MIREC_R8_THREADS 512
#endif
// (1,024 lanes — half the chunks per wave — measured the same: C4 grouping 24.6 vs 25.3 us
// by events, 11.81 vs 11.82 M samples/s)
constexpr int kR8Threads = MIREC_R8_THREADS;
constexpr int kR8Waves = kR8Threads / 64;
constexpr int kR8Max = 4096;
constexpr int kChainMaxBlocks = 256;       // chained look-back: at most 4 loads per lane
struct R8Lds {
  uint32_t k[2][kR8Max];                   // the block's keys (int32 bit patterns)
  uint16_t v[2][kR8Max];                   // their positions in the block
  uint16_t rank[kR8Max];                   // a key's rank among its digit in its wave
  int hist[256 * kR8Waves];                // [digit][wave] counts, then their offsets
  int scan[kR8Waves + 1];
  int32_t kmin, kmax, base, last;
};

#ifdef MIREC_R8_PROBE
__device__ uint64_t g_r8_probe[16];
#define R8T(k) do { if (threadIdx.x == 0 && blockIdx.x == 0) g_r8_probe[k] = wall_clock64(); } while (0)
#define R8C(k) do { if (threadIdx.x == 0 && blockIdx.x == 0) g_r8_probe[k] = clock64(); } while (0)
extern "C" int mirec_r8_probe_read(uint64_t* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_r8_probe), sizeof(g_r8_probe)) == hipSuccess ? 0 : -1;
}
#else
#define R8T(k) do {} while (0)
#define R8C(k) do {} while (0)
#endif
// status == nullptr: block b writes its own perm / uniq / seg / n_uniq at b's offsets in
// the outputs (block-local positions; blocks_concat_kernel joins them). status != nullptr
// (chained, one launch): block b publishes its unique count in status[b] (count + 1,
// release), sums the counts of blocks < b (acquire; every one of them was dispatched
// before b and publishes without waiting, so the wait ends) and writes straight into the
// concatenated outputs; the block that takes the last ticket in status[nblocks] zeroes
// status again for the next launch.
// Keys given as fields (DeepFM: block b = field b's column + the field's table offset):
// the kernel forms them itself and writes them out for the forward's gathers.
constexpr int kSortFields = 64;
struct SortFields {
  const int64_t* col[kSortFields];
  int64_t off[kSortFields];
  int64_t* keys_out;
};

__global__ __launch_bounds__(kR8Threads) void segsort_radix8_kernel(
    const int64_t* __restrict__ keys_all, int64_t n_total, int batch_n,
    int32_t* __restrict__ perm_all, int32_t* __restrict__ uniq_all,
    int32_t* __restrict__ seg_all, int32_t* __restrict__ n_uniq_all,
    int32_t* __restrict__ status, int32_t* __restrict__ pu_all, const SortFields SF) {
  __shared__ R8Lds L;
  R8T(0);
  R8C(12);
  const int64_t b = blockIdx.x;
  const int n = (int)min((int64_t)batch_n, n_total - b * batch_n);
  const int64_t* __restrict__ keys = keys_all + b * batch_n;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  int lo = INT32_MAX, hi = INT32_MIN;
  for (int i = tid; i < n; i += kR8Threads) {
    int32_t kv;
    if (SF.keys_out) {                           // field b's id + its table offset
      const int64_t k64 = SF.col[b][i] + SF.off[b];
      SF.keys_out[b * (int64_t)batch_n + i] = k64;
      kv = (int32_t)k64;
    } else {
      kv = (int32_t)keys[i];
    }
    L.k[0][i] = (uint32_t)kv;
    L.v[0][i] = (uint16_t)i;
    lo = min(lo, kv);
    hi = max(hi, kv);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    lo = min(lo, __shfl_xor(lo, off, 64));
    hi = max(hi, __shfl_xor(hi, off, 64));
  }
  if (tid == 0) {
    L.kmin = INT32_MAX;
    L.kmax = INT32_MIN;
  }
  __syncthreads();
  if (lane == 0) {
    atomicMin(&L.kmin, lo);
    atomicMax(&L.kmax, hi);
  }
  __syncthreads();
  R8T(1);
  const uint32_t kmin = (uint32_t)L.kmin;
  const uint32_t span = n > 0 ? (uint32_t)L.kmax - kmin : 0u;
  int bits = 0;
  while (bits < 32 && (span >> bits) != 0u) ++bits;
  const int nch = (n + 63) >> 6;
  const int cpw = (nch + kR8Waves - 1) / kR8Waves;   // chunks of this wave: [wid*cpw, +cpw)
  const uint64_t lt = (1ull << lane) - 1ull;
  int cur = 0;
  for (int shift = 0; shift < bits; shift += 8) {
    for (int q = tid; q < 256 * kR8Waves; q += kR8Threads) L.hist[q] = 0;
    __syncthreads();                             // keys of the pass in place, counters zeroed
#pragma unroll 1
    for (int cc = 0; cc < cpw; ++cc) {           // rolled: a short code path (one pass of
      const int i = (wid * cpw + cc) * 64 + lane;  // one block runs cold in the I-cache)
      const bool valid = i < n;
      const uint32_t dd = valid ? ((L.k[cur][i] - kmin) >> shift) & 255u : 0u;
      uint64_t m = __ballot(valid);
#pragma unroll
      for (int bb = 0; bb < 8; ++bb) {           // same-digit lanes: AND of xnor(ballot, bit)
        const int32_t sb = __builtin_amdgcn_sbfe((int32_t)dd, bb, 1);
        const uint64_t bl = __ballot(sb != 0);
        const uint64_t s64 = (uint64_t)(int64_t)sb;
        m &= ~(bl ^ s64);
      }
      const int r = __popcll(m & lt);
      int* h = &L.hist[(int)dd * kR8Waves + wid];
      const int before = valid ? *h : 0;
      __builtin_amdgcn_wave_barrier();
      if (valid && r == 0) *h = before + __popcll(m);
      __builtin_amdgcn_wave_barrier();
      if (valid) L.rank[i] = (uint16_t)(before + r);
    }
    if (shift == 8) R8T(8);
    __syncthreads();
    {                                            // exclusive scan of the counters, digit-major
      constexpr int per = 256 * kR8Waves / kR8Threads;
      int c[per], sum = 0;
#pragma unroll
      for (int q = 0; q < per; ++q) {
        c[q] = L.hist[tid * per + q];
        sum += c[q];
      }
      int tot;
      int run = block_exclusive_scan(sum, L.scan, &tot);
#pragma unroll
      for (int q = 0; q < per; ++q) {
        L.hist[tid * per + q] = run;
        run += c[q];
      }
    }
    __syncthreads();
    if (shift == 8) R8T(9);
#pragma unroll 1
    for (int cc = 0; cc < cpw; ++cc) {
      const int i = (wid * cpw + cc) * 64 + lane;
      if (i < n) {
        const uint32_t kv = L.k[cur][i];
        const int dst = L.hist[(int)(((kv - kmin) >> shift) & 255u) * kR8Waves + wid] + L.rank[i];
        L.k[cur ^ 1][dst] = kv;
        L.v[cur ^ 1][dst] = L.v[cur][i];
      }
    }
    cur ^= 1;
    if (shift == 8) R8T(10);
    __syncthreads();                             // offsets read before the next zeroing
    R8T(2 + shift / 8);
  }
  R8T(6);
  const uint32_t* __restrict__ ks = L.k[cur];
  const int per = (n + kR8Threads - 1) / kR8Threads;  // uniq / seg: one scan over runs of
  const int i0 = min(n, tid * per), i1 = min(n, i0 + per);   // per keys a thread
  int f = 0;
  for (int i = i0; i < i1; ++i) f += (i == 0 || ks[i - 1] != ks[i]) ? 1 : 0;
  int nu;
  int o = block_exclusive_scan(f, L.scan, &nu);
  const int64_t pos0 = b * (int64_t)batch_n;
  int32_t *perm, *uniq, *seg;
  int32_t voff;                                  // added to block-local positions
  if (status) {
    // the count is the whole message: relaxed agent-scope store and loads (an agent
    // release / acquire is buffer_wbl2 / buffer_inv on gfx950 — see step.hip, part_store)
    if (tid == 0) __hip_atomic_store(&status[b], nu + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (wid == 0) {
      int acc = 0;
      for (int64_t j0 = 0; j0 < b; j0 += 64) {
        const int64_t j = j0 + lane;
        int c = 0;
        if (j < b) {
          while ((c = __hip_atomic_load(&status[j], __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT)) == 0)
            __builtin_amdgcn_s_sleep(1);
          c -= 1;
        }
        acc += wave_sum_i(c);
      }
      if (lane == 0) L.base = acc;
    }
    __syncthreads();
    perm = perm_all + pos0;
    uniq = uniq_all + L.base;
    seg = seg_all + L.base;
    voff = (int32_t)pos0;
  } else {
    perm = perm_all + pos0;
    uniq = uniq_all + pos0;
    seg = seg_all + b * (int64_t)(batch_n + 1);
    voff = 0;
  }
  for (int i = tid; i < n; i += kR8Threads) perm[i] = voff + L.v[cur][i];
  int32_t* __restrict__ pu = pu_all ? pu_all + pos0 : nullptr;   // chained only
  const int ubase = status ? L.base : 0;
  for (int i = i0; i < i1; ++i) {
    if (i == 0 || ks[i - 1] != ks[i]) {
      uniq[o] = (int32_t)ks[i];
      seg[o] = voff + i;
      ++o;
    }
    if (pu) pu[i] = ubase + o - 1;               // the segment of sorted position i
  }
  if (!status) {
    if (tid == 0) {
      seg[nu] = n;
      n_uniq_all[b] = nu;
    }
  } else {
    const int nblocks = (int)gridDim.x;
    if (tid == 0) {
      if (b == nblocks - 1) {
        seg[nu] = (int32_t)n_total;
        n_uniq_all[0] = L.base + nu;
      }
      // relaxed: this block's look-back loads have returned (their sum is in L.base)
      L.last = __hip_atomic_fetch_add(&status[nblocks], 1, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT) == nblocks - 1;
    }
    __syncthreads();
    if (L.last)                                  // every block is past its look-back
      for (int q = tid; q <= nblocks; q += kR8Threads) status[q] = 0;
  }
  R8T(7);
  R8C(13);
}

// Block-partitioned sort (keys in n_blocks blocks of block_n, every key of block b
// below every key of block b+1 — DeepFM's token keys, one block per field at its
// table offset): each block sorted in LDS by its own workgroup, then concatenated —
// the global stable sort, in two launches instead of a device-wide radix sort.
__global__ __launch_bounds__(256) void blocks_concat_kernel(
    const int32_t* __restrict__ perm_t, const int32_t* __restrict__ uniq_t,
    const int32_t* __restrict__ seg_t, const int32_t* __restrict__ nu_t, int64_t n,
    int block_n, int n_blocks, int32_t* __restrict__ perm, int32_t* __restrict__ uniq,
    int32_t* __restrict__ seg, int32_t* __restrict__ n_uniq) {
  const int b = blockIdx.x;
  int off = 0;
  for (int c = 0; c < b; ++c) off += nu_t[c];
  const int nu = nu_t[b];
  const int64_t base = (int64_t)b * block_n;
  const int nb = (int)min((int64_t)block_n, n - base);
  for (int i = threadIdx.x; i < nb; i += blockDim.x) perm[base + i] = (int32_t)base + perm_t[base + i];
  for (int i = threadIdx.x; i < nu; i += blockDim.x) {
    uniq[off + i] = uniq_t[base + i];
    seg[off + i] = (int32_t)base + seg_t[(int64_t)b * (block_n + 1) + i];
  }
  if (b == n_blocks - 1 && threadIdx.x == 0) {
    seg[off + nu] = (int32_t)n;
    n_uniq[0] = off + nu;
  }
}

// Two batched sorts in one launch (the user and the item keys of a chunk):
// workgroups [0, nbA) sort table A's batches, the rest table B's.
struct SortJob {
  const int64_t* keys; int64_t n_total; int batch_n; int nbits;
  int32_t *perm, *uniq, *seg, *n_uniq;
};

__global__ __launch_bounds__(kSortThreads) void segsort_lds2_kernel(SortJob A, SortJob B,
                                                                    int64_t nbA) {
  __shared__ SortLds L;
  const bool a = (int64_t)blockIdx.x < nbA;
  const SortJob& J = a ? A : B;
  segsort_lds_batch(J.keys, J.n_total, J.batch_n, J.nbits, J.perm, J.uniq, J.seg, J.n_uniq,
                    a ? (int64_t)blockIdx.x : (int64_t)blockIdx.x - nbA, L);
}

// Same algorithm, global ping-pong buffers, processed in chunks of
// kSortThreads*kIpt with running offsets (any n up to INT32_MAX).
__global__ __launch_bounds__(kSortThreads) void segsort_global_kernel(
    const int64_t* __restrict__ keys_all, int64_t n_total, int batch_n, int nbits,
    int32_t* __restrict__ perm_all, int32_t* __restrict__ uniq_all,
    int32_t* __restrict__ seg_all, int32_t* __restrict__ n_uniq_all, int32_t* __restrict__ ws) {
  __shared__ int scan_lds[kSortThreads / 64 + 1];
  const int64_t b = blockIdx.x;
  const int n = (int)min((int64_t)batch_n, n_total - b * batch_n);
  const int64_t* __restrict__ keys = keys_all + b * batch_n;
  int32_t* __restrict__ perm = perm_all + b * batch_n;
  int32_t* __restrict__ uniq = uniq_all + b * batch_n;
  int32_t* __restrict__ seg = seg_all + b * (batch_n + 1);
  int32_t* __restrict__ n_uniq = n_uniq_all + b;
  int32_t* kA = ws + b * 4 * (int64_t)batch_n;
  int32_t* vA = kA + batch_n;
  int32_t* kB = vA + batch_n;
  int32_t* vB = kB + batch_n;
  for (int i = threadIdx.x; i < n; i += kSortThreads) {
    kA[i] = (int32_t)keys[i];
    vA[i] = i;
  }
  __syncthreads();
  int32_t *ks = kA, *vs = vA, *kd = kB, *vd = vB;
  constexpr int CH = kSortThreads * kIpt;
  for (int bit = 0; bit < nbits; ++bit) {
    // total zeros
    int zloc = 0;
    for (int i = threadIdx.x; i < n; i += kSortThreads) zloc += ((ks[i] >> bit) & 1) ? 0 : 1;
    int Z;
    (void)block_exclusive_scan(zloc, scan_lds, &Z);
    int zrun = 0;  // zeros in earlier chunks
    for (int c0 = 0; c0 < n; c0 += CH) {
      const int lo = c0 + threadIdx.x * kIpt;
      const int hi = min(n, lo + kIpt);
      int z = 0;
      for (int i = lo; i < hi; ++i) z += ((ks[i] >> bit) & 1) ? 0 : 1;
      int zc;
      const int ez = block_exclusive_scan(z, scan_lds, &zc);
      int zb = zrun + ez;
      for (int i = lo; i < hi; ++i) {
        const int32_t kv = ks[i];
        const int one = (kv >> bit) & 1;
        const int dst = one ? (Z + (i - zb)) : zb;
        kd[dst] = kv;
        vd[dst] = vs[i];
        zb += 1 - one;
      }
      zrun += zc;
    }
    __threadfence_block();
    __syncthreads();
    int32_t* t;
    t = ks; ks = kd; kd = t;
    t = vs; vs = vd; vd = t;
  }
  for (int i = threadIdx.x; i < n; i += kSortThreads) perm[i] = vs[i];
  __syncthreads();
  emit_segments(ks, n, uniq, seg, n_uniq, scan_lds);
}

// Dense scatter of grouped sums (autograd-compatible path): one wave per
// distinct row, lanes over the row's columns, contributions in fixed order.
__global__ __launch_bounds__(256) void segment_scatter_add_kernel(
    const float* __restrict__ rows, int d, const int32_t* __restrict__ perm,
    const int32_t* __restrict__ uniq, const int32_t* __restrict__ seg,
    const int32_t* __restrict__ n_uniq_dev, float* __restrict__ dense, int64_t n_rows) {
  const int nu = n_uniq_dev[0];
  const int lane = threadIdx.x & 63;
  for (int u = blockIdx.x * 4 + (threadIdx.x >> 6); u < nu; u += gridDim.x * 4) {
    const int64_t row = uniq[u];
    if (row < 0 || row >= n_rows) continue;
    const int s0 = seg[u], s1 = seg[u + 1];
    for (int c = lane; c < d; c += 64) {
      float acc = 0.f;
      for (int i = s0; i < s1; ++i) acc += rows[(int64_t)perm[i] * d + c];
      dense[row * d + c] += acc;
    }
  }
}

// ---------------------------------------------------------------------------
// Large single-batch sorts (n > kLdsMax: the autograd paths of the context and
// sequential models group 10^5..10^6 contributions per step). Device-wide
// stable LSD radix sort, 5-bit digits, one tile of kRadixTile keys per block:
//   upsweep   per-tile digit histogram            -> hist[digit * n_tiles + tile]
//   scan      exclusive scan of hist (digit-major) -> global destination bases
//   downsweep stable in-tile ranking (blocked layout, per-thread digit counts
//             scanned digit-major in LDS) -> scatter of (key, index)
// then segments: per-tile head-flag counts -> scan -> uniq / seg writes.
constexpr int kRadixThreads = 256;
constexpr int kRadixIpt = 8;
constexpr int kRadixTile = kRadixThreads * kRadixIpt;
constexpr int kRadixBits = 5;     // digit width: 5 passes for 25-bit key spaces (was 4 bits, 7)
constexpr int kRadixBins = 1 << kRadixBits;

__global__ __launch_bounds__(kRadixThreads) void radix_init_kernel(
    const int64_t* __restrict__ keys, int n, int32_t* __restrict__ k32, int32_t* __restrict__ v32) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    k32[i] = (int32_t)keys[i];
    v32[i] = i;
  }
}

// per-thread digit counts of the thread's kRadixIpt consecutive keys -> cnt[bin][t]
__device__ __forceinline__ void tile_counts(const int32_t* __restrict__ k, int n, int base,
                                            int shift, int* cnt, int32_t* my, int* nmy) {
  const int t = threadIdx.x;
  int c[kRadixBins];
#pragma unroll
  for (int b = 0; b < kRadixBins; ++b) c[b] = 0;
  int m = 0;
#pragma unroll
  for (int j = 0; j < kRadixIpt; ++j) {
    const int i = base + t * kRadixIpt + j;
    if (i < n) {
      my[j] = k[i];
      const int dg = (my[j] >> shift) & (kRadixBins - 1);
#pragma unroll
      for (int b = 0; b < kRadixBins; ++b) c[b] += (dg == b) ? 1 : 0;
      ++m;
    }
  }
#pragma unroll
  for (int b = 0; b < kRadixBins; ++b) cnt[b * kRadixThreads + t] = c[b];
  *nmy = m;
}

__global__ __launch_bounds__(kRadixThreads) void radix_upsweep_kernel(
    const int32_t* __restrict__ k, int n, int shift, int n_tiles, int32_t* __restrict__ hist) {
  __shared__ int cnt[kRadixBins * kRadixThreads];
  int32_t my[kRadixIpt];
  int nmy;
  tile_counts(k, n, blockIdx.x * kRadixTile, shift, cnt, my, &nmy);
  __syncthreads();
  if (threadIdx.x < kRadixBins) {
    int s = 0;
    for (int t = 0; t < kRadixThreads; ++t) s += cnt[threadIdx.x * kRadixThreads + t];
    hist[threadIdx.x * n_tiles + blockIdx.x] = s;
  }
}

// exclusive scan of a[0..m) in place (one block), a[m] = total
__global__ __launch_bounds__(1024) void scan_exclusive_kernel(int32_t* __restrict__ a, int m) {
  __shared__ int lds[1024 / 64 + 1];
  int run = 0;
  for (int c0 = 0; c0 < m; c0 += 1024) {
    const int i = c0 + threadIdx.x;
    const int x = i < m ? a[i] : 0;
    int tot;
    const int ex = block_exclusive_scan(x, lds, &tot);
    if (i < m) a[i] = run + ex;
    run += tot;
  }
  if (threadIdx.x == 0) a[m] = run;
}

__global__ __launch_bounds__(kRadixThreads) void radix_downsweep_kernel(
    const int32_t* __restrict__ k, const int32_t* __restrict__ v, int n, int shift, int n_tiles,
    const int32_t* __restrict__ hist, int32_t* __restrict__ ko, int32_t* __restrict__ vo) {
  __shared__ int cnt[kRadixBins * kRadixThreads];
  __shared__ int part[kRadixThreads / 64 + 1];
  __shared__ int bin_start[kRadixBins];
  int32_t my[kRadixIpt];
  int nmy;
  const int base = blockIdx.x * kRadixTile;
  tile_counts(k, n, base, shift, cnt, my, &nmy);
  __syncthreads();
  // exclusive scan of cnt (thread-major, kRadixBins per thread: kRadixBins * kRadixThreads
  // entries), each thread's own bins serially, then a block scan of the thread totals
  const int t = threadIdx.x;
  int loc[kRadixBins];
  int s = 0;
#pragma unroll
  for (int j = 0; j < kRadixBins; ++j) {
    loc[j] = s;
    s += cnt[t * kRadixBins + j];
  }
  int tot;
  const int ex = block_exclusive_scan(s, part, &tot);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kRadixBins; ++j) cnt[t * kRadixBins + j] = ex + loc[j];
  __syncthreads();
  if (t < kRadixBins) bin_start[t] = cnt[t * kRadixThreads];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kRadixIpt; ++j) {
    if (j < nmy) {
      const int dg = (my[j] >> shift) & (kRadixBins - 1);
      int before = 0;
#pragma unroll
      for (int q = 0; q < kRadixIpt; ++q) before += (q < j && ((my[q] >> shift) & (kRadixBins - 1)) == dg) ? 1 : 0;
      const int local = cnt[dg * kRadixThreads + t] - bin_start[dg] + before;
      const int dst = hist[dg * n_tiles + blockIdx.x] + local;
      const int i = base + t * kRadixIpt + j;
      ko[dst] = my[j];
      vo[dst] = v[i];
    }
  }
}

__global__ __launch_bounds__(kRadixThreads) void seg_count_kernel(const int32_t* __restrict__ k,
                                                                  int n,
                                                                  int32_t* __restrict__ tcnt) {
  __shared__ int part[kRadixThreads / 64 + 1];
  const int base = blockIdx.x * kRadixTile;
  int f = 0;
  for (int j = 0; j < kRadixIpt; ++j) {
    const int i = base + threadIdx.x * kRadixIpt + j;
    if (i < n) f += (i == 0 || k[i - 1] != k[i]) ? 1 : 0;
  }
  int tot;
  (void)block_exclusive_scan(f, part, &tot);
  if (threadIdx.x == 0) tcnt[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kRadixThreads) void seg_write_kernel(
    const int32_t* __restrict__ k, int n, int n_tiles, const int32_t* __restrict__ tbase,
    int32_t* __restrict__ uniq, int32_t* __restrict__ seg, int32_t* __restrict__ n_uniq) {
  __shared__ int part[kRadixThreads / 64 + 1];
  const int base = blockIdx.x * kRadixTile;
  int f = 0;
  for (int j = 0; j < kRadixIpt; ++j) {
    const int i = base + threadIdx.x * kRadixIpt + j;
    if (i < n) f += (i == 0 || k[i - 1] != k[i]) ? 1 : 0;
  }
  int tot;
  int o = tbase[blockIdx.x] + block_exclusive_scan(f, part, &tot);
  for (int j = 0; j < kRadixIpt; ++j) {
    const int i = base + threadIdx.x * kRadixIpt + j;
    if (i < n && (i == 0 || k[i - 1] != k[i])) {
      uniq[o] = k[i];
      seg[o] = i;
      ++o;
    }
  }
  if (blockIdx.x == n_tiles - 1 && threadIdx.x == 0) {
    const int total = tbase[n_tiles];
    seg[total] = n;
    n_uniq[0] = total;
  }
}

static size_t radix_ws_bytes(int64_t n) {
  const int64_t tiles = (n + kRadixTile - 1) / kRadixTile;
  return (size_t)4 * (size_t)n * sizeof(int32_t) +
         (size_t)(kRadixBins * tiles + 1 + tiles + 1) * sizeof(int32_t) + 256;
}

static int radix_segment_sort(const int64_t* keys, int n, int nbits, int32_t* perm,
                              int32_t* uniq, int32_t* seg, int32_t* n_uniq, void* ws,
                              hipStream_t st) {
  const int tiles = (n + kRadixTile - 1) / kRadixTile;
  int32_t* kA = (int32_t*)ws;
  int32_t* vA = kA + n;
  int32_t* kB = vA + n;
  int32_t* vB = kB + n;
  int32_t* hist = vB + n;                       // kRadixBins * tiles + 1
  int32_t* tcnt = hist + kRadixBins * tiles + 1;  // tiles + 1
  int g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(radix_init_kernel, dim3(g), dim3(256), 0, st, keys, n, kA, vA);
  const int passes = nbits == 0 ? 0 : (nbits + kRadixBits - 1) / kRadixBits;
  for (int p = 0; p < passes; ++p) {
    const int shift = kRadixBits * p;
    hipLaunchKernelGGL(radix_upsweep_kernel, dim3(tiles), dim3(kRadixThreads), 0, st, kA, n,
                       shift, tiles, hist);
    hipLaunchKernelGGL(scan_exclusive_kernel, dim3(1), dim3(1024), 0, st, hist,
                       kRadixBins * tiles);
    hipLaunchKernelGGL(radix_downsweep_kernel, dim3(tiles), dim3(kRadixThreads), 0, st, kA, vA,
                       n, shift, tiles, hist, kB, vB);
    int32_t* t = kA; kA = kB; kB = t;
    t = vA; vA = vB; vB = t;
  }
  {
    const int rc = hip_status(
        hipMemcpyAsync(perm, vA, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToDevice, st),
        "mirec_segment_sort (perm copy)");
    if (rc) return rc;
  }
  hipLaunchKernelGGL(seg_count_kernel, dim3(tiles), dim3(kRadixThreads), 0, st, kA, n, tcnt);
  hipLaunchKernelGGL(scan_exclusive_kernel, dim3(1), dim3(1024), 0, st, tcnt, tiles);
  hipLaunchKernelGGL(seg_write_kernel, dim3(tiles), dim3(kRadixThreads), 0, st, kA, n, tiles,
                     tcnt, uniq, seg, n_uniq);
  return launch_status("mirec_segment_sort (radix)");
}

// ---------------------------------------------------------------------------
// Device-wide sort in few launches ("onesweep" form): one launch builds every pass's
// global digit histogram (8-bit digits: ceil(bits / 8) passes, 3 for a 3 M-row table
// instead of 5 five-bit passes of upsweep + scan + downsweep), one launch per pass ranks
// a 2,048-key tile stably in LDS (the ballot ranking of segsort_radix8_kernel) and finds
// its digit offsets among the tiles by decoupled look-back, and one launch emits the
// segments (with pos_seg) by a look-back scan of the run heads. 2 + passes launches,
// against 5 x 3 + 5. Same perm / uniq / seg / n_uniq (stable sort: unique).
//
// status (int32, zero before the first call, left zero: the last block of each launch
// zeroes what that launch used): hist [kOsMaxPasses][256] | look-back words [passes]
// [tiles][256] | segment look-back words [tiles] | tickets [kOsMaxPasses + 1]. A look-back
// word holds 1 << 30 | the tile's own count; a tile sums its predecessors' words.
constexpr int kOsThreads = 512;
constexpr int kOsWaves = kOsThreads / 64;
constexpr int kOsTile = 2048;
constexpr int kOsIpt = kOsTile / kOsThreads;       // keys per thread (loads)
constexpr int kOsChunks = kOsTile / 64 / kOsWaves;  // 64-key chunks per wave
constexpr int kOsMaxPasses = 4;
constexpr uint32_t kOsFlagA = 1u << 30, kOsVal = (1u << 30) - 1;

__host__ __device__ inline int64_t os_tiles(int64_t n) { return (n + kOsTile - 1) / kOsTile; }
__host__ __device__ inline int64_t os_status_words(int64_t n) {
  const int64_t t = os_tiles(n);
  return (int64_t)kOsMaxPasses * 256 + (int64_t)kOsMaxPasses * t * 256 + t + kOsMaxPasses + 1;
}

// The look-back words carry only their own count (flag 1 << 30 | count): no data is
// published through them, so relaxed agent-scope loads and stores suffice, and the loads
// of many predecessors can be in flight together (an acquire load waits for itself).
__device__ __forceinline__ uint32_t os_load(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void os_store(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// sum of the counts of tiles h, h + H, h + 2H, ... < tile in column `words` (stride per
// tile): every tile publishes its count before it sums, so no wait chains through
// predecessors — 16 loads in flight per batch, a word not yet published is re-read
__device__ __forceinline__ uint32_t os_sum_before(const uint32_t* words, int64_t tile,
                                                  int64_t stride, int h, int H) {
  uint32_t s = 0;
  for (int64_t t0 = h; t0 < tile; t0 += 16 * (int64_t)H) {
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int64_t t = t0 + j * (int64_t)H;
      w[j] = t < tile ? os_load(words + t * stride) : kOsFlagA;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int64_t t = t0 + j * (int64_t)H;
      while ((w[j] >> 30) == 0) {
        __builtin_amdgcn_s_sleep(1);
        w[j] = os_load(words + t * stride);
      }
      s += t < tile ? (w[j] & kOsVal) : 0u;
    }
  }
  return s;
}

// the last of the launch's blocks (ticket) zeroes `words` [0, n_words)
__device__ __forceinline__ void os_cleanup(uint32_t* ticket, uint32_t* words, int64_t n_words,
                                           int* flag_lds) {
  __syncthreads();
  if (threadIdx.x == 0)
    *flag_lds = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                gridDim.x - 1;
  __syncthreads();
  if (*flag_lds) {
    for (int64_t q = threadIdx.x; q < n_words; q += blockDim.x) words[q] = 0u;
    if (threadIdx.x == 0) *ticket = 0u;
  }
}

__global__ __launch_bounds__(kOsThreads) void os_hist_kernel(
    const int64_t* __restrict__ keys, int n, int passes, int32_t* __restrict__ k32,
    int32_t* __restrict__ v32, uint32_t* __restrict__ hist) {
  __shared__ int h[kOsMaxPasses][256];
  for (int q = threadIdx.x; q < kOsMaxPasses * 256; q += kOsThreads) (&h[0][0])[q] = 0;
  __syncthreads();
  const int base = blockIdx.x * kOsTile;
#pragma unroll
  for (int j = 0; j < kOsIpt; ++j) {
    const int i = base + j * kOsThreads + threadIdx.x;
    if (i < n) {
      const uint32_t kv = (uint32_t)keys[i];
      k32[i] = (int32_t)kv;
      v32[i] = i;
      for (int p = 0; p < passes; ++p) atomicAdd(&h[p][(kv >> (8 * p)) & 255u], 1);
    }
  }
  __syncthreads();
  for (int q = threadIdx.x; q < passes * 256; q += kOsThreads) {
    const int c = (&h[0][0])[q];
    if (c) __hip_atomic_fetch_add(hist + q, (uint32_t)c, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
  }
}

struct OsPassLds {
  uint32_t k[kOsTile];
  int32_t v[kOsTile];
  int cnt[256 * kOsWaves];           // [digit][wave] counts, then their offsets in the tile
  uint16_t rank[kOsTile];
  int gbase[256];                    // global start of each digit (this pass)
  int tstart[257];                   // start of each digit inside the tile
  int scan[kOsWaves + 1];
  uint32_t half[256];
  int last;
};

__global__ __launch_bounds__(kOsThreads) void os_pass_kernel(
    const int32_t* __restrict__ kin, const int32_t* __restrict__ vin, int n, int shift,
    int64_t tiles, uint32_t* __restrict__ hist_p, uint32_t* __restrict__ look_p,
    uint32_t* __restrict__ ticket_p, int32_t* __restrict__ kout, int32_t* __restrict__ vout) {
  __shared__ OsPassLds L;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t tile = blockIdx.x;
  const int base = (int)(tile * kOsTile);
  const int tn = min(kOsTile, n - base);
#pragma unroll
  for (int j = 0; j < kOsIpt; ++j) {
    const int i = j * kOsThreads + tid;
    if (i < tn) {
      L.k[i] = (uint32_t)kin[base + i];
      L.v[i] = vin[base + i];
    }
  }
  for (int q = tid; q < 256 * kOsWaves; q += kOsThreads) L.cnt[q] = 0;
  // the pass's global digit starts: an exclusive scan of its histogram
  {
    const int c = tid < 256 ? (int)hist_p[tid] : 0;
    int tot;
    const int ex = block_exclusive_scan(c, L.scan, &tot);
    if (tid < 256) L.gbase[tid] = ex;
  }
  __syncthreads();
  const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
  for (int cc = 0; cc < kOsChunks; ++cc) {       // wave wid owns chunks [wid * kOsChunks, ..)
    const int i = (wid * kOsChunks + cc) * 64 + lane;
    const bool valid = i < tn;
    const uint32_t dd = valid ? (L.k[i] >> shift) & 255u : 0u;
    uint64_t m = __ballot(valid);
#pragma unroll
    for (int bb = 0; bb < 8; ++bb) {
      const int32_t sb = __builtin_amdgcn_sbfe((int32_t)dd, bb, 1);
      const uint64_t bl = __ballot(sb != 0);
      m &= ~(bl ^ (uint64_t)(int64_t)sb);
    }
    const int r = __popcll(m & lt);
    int* h = &L.cnt[(int)dd * kOsWaves + wid];
    const int before = valid ? *h : 0;
    __builtin_amdgcn_wave_barrier();
    if (valid && r == 0) *h = before + __popcll(m);
    __builtin_amdgcn_wave_barrier();
    if (valid) L.rank[i] = (uint16_t)(before + r);
  }
  __syncthreads();
  {                                              // digit-major offsets inside the tile
    constexpr int per = 256 * kOsWaves / kOsThreads;
    int c[per], sum = 0;
#pragma unroll
    for (int q = 0; q < per; ++q) {
      c[q] = L.cnt[tid * per + q];
      sum += c[q];
    }
    int tot;
    int run = block_exclusive_scan(sum, L.scan, &tot);
#pragma unroll
    for (int q = 0; q < per; ++q) {
      L.cnt[tid * per + q] = run;
      run += c[q];
    }
  }
  __syncthreads();
  if (tid < 256) L.tstart[tid] = L.cnt[tid * kOsWaves];
  if (tid == 0) L.tstart[256] = tn;
  __syncthreads();
  if (tid < 256)                                 // digit tid: this tile's count
    os_store(look_p + tile * 256 + tid,
             kOsFlagA | (uint32_t)(L.tstart[tid + 1] - L.tstart[tid]));
  {                                              // the counts of the tiles before: thread
    const int dg = tid & 255, h = tid >> 8;      // (digit, half) sums every other tile
    const uint32_t part = os_sum_before(look_p + dg, tile, 256, h, kOsThreads / 256);
    if (h == 1) L.half[dg] = part;
    __syncthreads();
    if (h == 0)                                  // + the key's offset inside the tile
      L.gbase[dg] += (int)(part + L.half[dg]) - L.tstart[dg];
  }
  __syncthreads();
#pragma unroll
  for (int cc = 0; cc < kOsChunks; ++cc) {
    const int i = (wid * kOsChunks + cc) * 64 + lane;
    if (i < tn) {
      const uint32_t kv = L.k[i];
      const int dd = (int)((kv >> shift) & 255u);
      const int dst = L.gbase[dd] + L.cnt[dd * kOsWaves + wid] + L.rank[i];
      kout[dst] = (int32_t)kv;
      vout[dst] = L.v[i];
    }
  }
  // this pass's histogram and look-back words, zeroed by its last block
  os_cleanup(ticket_p, look_p, tiles * 256, &L.last);
  if (L.last)
    for (int q = tid; q < 256; q += kOsThreads) hist_p[q] = 0u;
}

__global__ __launch_bounds__(kOsThreads) void os_seg_kernel(
    const int32_t* __restrict__ k, int n, int64_t tiles, uint32_t* __restrict__ look,
    uint32_t* __restrict__ ticket, int32_t* __restrict__ uniq, int32_t* __restrict__ seg,
    int32_t* __restrict__ n_uniq, int32_t* __restrict__ pos_seg) {
  __shared__ int scan[kOsWaves + 1];
  __shared__ int prefix;
  __shared__ int last;
  const int64_t tile = blockIdx.x;
  const int base = (int)(tile * kOsTile);
  const int i0 = base + threadIdx.x * kOsIpt;      // blocked: kOsIpt consecutive keys
  int32_t kk[kOsIpt];
  int f = 0;
#pragma unroll
  for (int j = 0; j < kOsIpt; ++j) {
    const int i = i0 + j;
    kk[j] = i < n ? k[i] : 0;
    if (i < n) f += (i == 0 || k[i - 1] != kk[j]) ? 1 : 0;
  }
  int tot;
  const int ex = block_exclusive_scan(f, scan, &tot);
  if (threadIdx.x == 0) os_store(look + tile, kOsFlagA | (uint32_t)tot);
  {                                              // run heads of the tiles before this one
    const uint32_t part = os_sum_before(look, tile, 1, threadIdx.x, kOsThreads);
    int all;
    (void)block_exclusive_scan((int)part, scan, &all);
    if (threadIdx.x == 0) {
      prefix = all;
      if (tile == tiles - 1) {
        seg[all + tot] = n;
        n_uniq[0] = (int32_t)(all + tot);
      }
    }
  }
  __syncthreads();
  int o = prefix + ex;
#pragma unroll
  for (int j = 0; j < kOsIpt; ++j) {
    const int i = i0 + j;
    if (i < n) {
      if (i == 0 || k[i - 1] != kk[j]) {
        uniq[o] = kk[j];
        seg[o] = i;
        ++o;
      }
      if (pos_seg) pos_seg[i] = o - 1;
    }
  }
  os_cleanup(ticket, look, tiles, &last);
}

// ---------------------------------------------------------------------------
// Chunked segmented scatter-add (hot rows: a Zipf head row may own 10^4..10^5
// contributions, far too many for one wave to sum serially). Every segment is cut
// into pieces of CH = scat_chunk(d) positions counted from ITS OWN start, so a row's
// sum depends only on its own contributions and their order — not on where the row
// sits in the sorted array (a row-sharded owner's shorter array gives the one-process
// sums bit for bit). Work is dealt by absolute chunks of CH positions: the group of G
// lanes of chunk c sums every piece that STARTS in c (reading past c's end when the
// piece does) — the pieces of the segments that start in c, plus at most one later
// piece of the segment that started before c. A one-piece segment is written
// directly; a longer one leaves its first piece in tail[chunk of its start] and
// piece k in head[that chunk + k] (at most one of each per chunk), which the fixup
// kernel (owner: the block of the first boundary after the segment's start) adds in
// piece order. Deterministic, no float atomics.
// positions per chunk: short chunks for wide rows (more lane groups in flight),
// longer ones for narrow rows; the workspace is sized for the smallest
#ifndef MIREC_SCAT_NARROW_CH
#define MIREC_SCAT_NARROW_CH 8
#endif
// 8 positions per piece up to d = 16 (DeepFM tokens: C4 4.34 -> 4.54 M samples/s against 32)
__host__ __device__ __forceinline__ int scat_chunk(int d) {
  return d == 1 ? 8 : d <= 16 ? MIREC_SCAT_NARROW_CH : 32;
}
constexpr int kScatChunkMin = 8;

__device__ __forceinline__ int seg_of(const int32_t* __restrict__ seg, int nu, int p) {
  int lo = 0, hi = nu - 1;   // largest u with seg[u] <= p
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (seg[mid] <= p) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// PAIR (mirec_segment_reduce2_f32): a second, one-column source grouped by the same
// segments (DeepFM's first-order [V, 1] weights beside the [V, d] token rows) is summed
// by lane 0 of each group in the same pass, position by position in the same order as
// the one-column kernel; its pieces go to head1 / tail1.
template <int G, int DMAX, bool PAIR = false>
__global__ __launch_bounds__(256) void scatter_chunks_kernel(
    const float* __restrict__ rows, int d, const int32_t* __restrict__ perm,
    const int32_t* __restrict__ uniq, const int32_t* __restrict__ seg,
    const int32_t* __restrict__ n_uniq_dev, float* __restrict__ dense, int64_t n_rows,
    float* __restrict__ head, float* __restrict__ tail, int32_t* __restrict__ tail_seg,
    int n_chunks, int compact, const float* __restrict__ rows1 = nullptr,
    float* __restrict__ dense1 = nullptr, float* __restrict__ head1 = nullptr,
    float* __restrict__ tail1 = nullptr) {
  const int nu = n_uniq_dev[0];
  const int n = seg[nu];
  const int lane = threadIdx.x & 63;
  const int gi = lane / G, l = lane % G;
  const int c = (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64) * (64 / G) + gi;
  if (c >= n_chunks) return;
  const int CH = scat_chunk(d);
  const int p0 = c * CH;
  if (nu == 0 || p0 >= n) {
    if (l == 0) tail_seg[c] = -1;
    return;
  }
  const int p1 = min(n, p0 + CH);
  constexpr int MAXC = DMAX / G;    // columns per lane, d <= DMAX
  // sums positions [q0, q1) of one segment into acc (loads 4 positions ahead of the adds)
  float acc1 = 0.f;                         // PAIR: the one-column source (lane 0)
  auto piece = [&](int q0, int q1, float* acc) {
    int q = q0;
#pragma unroll
    for (int j = 0; j < MAXC; ++j) acc[j] = 0.f;
    acc1 = 0.f;
    for (; q + 4 <= q1; q += 4) {
      int pr[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) pr[t] = perm[q + t];
      float v[4][MAXC];
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int j = 0; j < MAXC; ++j) {
          const int col = l + j * G;
          v[t][j] = col < d ? rows[(int64_t)pr[t] * d + col] : 0.f;
        }
      float v1[4];
      if (PAIR) {
#pragma unroll
        for (int t = 0; t < 4; ++t) v1[t] = l == 0 ? rows1[pr[t]] : 0.f;
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int j = 0; j < MAXC; ++j) acc[j] += v[t][j];
      if (PAIR) {
#pragma unroll
        for (int t = 0; t < 4; ++t) acc1 += v1[t];
      }
    }
    for (; q < q1; ++q) {
      const float* r = rows + (int64_t)perm[q] * d;
#pragma unroll
      for (int j = 0; j < MAXC; ++j) {
        const int col = l + j * G;
        if (col < d) acc[j] += r[col];
      }
      if (PAIR && l == 0) acc1 += rows1[perm[q]];
    }
  };
  auto store1 = [&](float* dst) {
    if (PAIR && l == 0 && dst) *dst = acc1;
  };
  auto store = [&](float* dst, const float* acc, bool add) {
#pragma unroll
    for (int j = 0; j < MAXC; ++j) {
      const int col = l + j * G;
      if (dst && col < d) {
        if (add) dst[col] += acc[j]; else dst[col] = acc[j];
      }
    }
  };
  float acc[MAXC];
  int u = seg_of(seg, nu, p0);
  if (seg[u] < p0) {                       // the segment that started before this chunk
    const int s0 = seg[u], e = seg[u + 1];
    const int ps = s0 + (p0 - s0 + CH - 1) / CH * CH;   // its next piece start >= p0
    if (ps < p1 && ps < e) {
      piece(ps, min(e, ps + CH), acc);
      store(head + (int64_t)c * d, acc, false);
      store1(PAIR ? head1 + c : nullptr);
    }
    ++u;
  }
  int ts = -1;                              // the multi-piece segment starting here, if any
  for (; u < nu && seg[u] < p1; ++u) {     // the segments that start in this chunk
    const int s0 = seg[u], e = seg[u + 1];
    piece(s0, min(e, s0 + CH), acc);
    if (e - s0 <= CH) {
      const int64_t row = compact ? (int64_t)u : (int64_t)uniq[u];
      store((row >= 0 && row < n_rows) ? dense + row * d : nullptr, acc, !compact);
      store1(PAIR ? dense1 + u : nullptr);       // PAIR: compact outputs only
    } else {
      store(tail + (int64_t)c * d, acc, false);
      store1(PAIR ? tail1 + c : nullptr);
      ts = u;
    }
  }
  if (l == 0) tail_seg[c] = ts;            // the fixup's owner list: no search there
}

// Fixup of the multi-piece segments: the owner of boundary b is the segment that starts
// in chunk b - 1 and continues (tail_seg, written by the chunk kernel). Its sum is
// defined by 256 partial sums per column block of CW = d rounded up to a power of two
// columns: "thread" i (column cb + i % CW, kl = i / CW, KL = 256 / CW) sums
// [tail[b-1] if kl = 0] + head[b + kl] + head[b + kl + KL] + ..., and the column's sum
// is t = s_0 + s_1 + ... + s_{KL-1} in kl order — deterministic. One wave per boundary
// forms the 256 partial sums (four per lane, their loads in flight together), stages
// them in its LDS slice and folds them; four boundaries per workgroup. The one-column
// source of a pair uses the same rule with CW = 1 (KL = 256).
constexpr int kFixWaves = 4;
__global__ __launch_bounds__(64 * kFixWaves) void scatter_fixup_kernel(
    int d, const int32_t* __restrict__ uniq, const int32_t* __restrict__ seg,
    const int32_t* __restrict__ tail_seg, float* __restrict__ dense, int64_t n_rows,
    const float* __restrict__ head, const float* __restrict__ tail, int n_chunks, int compact,
    float* __restrict__ dense1 = nullptr, const float* __restrict__ head1 = nullptr,
    const float* __restrict__ tail1 = nullptr) {
  __shared__ float red[kFixWaves][256];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b = 1 + (int)blockIdx.x * kFixWaves + w;           // this wave's boundary
  if (b >= n_chunks) return;
  const int u = tail_seg[b - 1];
  if (u < 0) return;
  const int CH = scat_chunk(d);
  const int s0 = seg[u], e = seg[u + 1];
  const int kend = b - 2 + (e - s0 + CH - 1) / CH;     // chunk holding its last piece's start
  const int64_t row = compact ? (int64_t)u : (int64_t)uniq[u];
  if (row < 0 || row >= n_rows) return;
  float* R = red[w];
  // partial sums of "threads" i = lane + 64 j over src (ld columns, CW, KL), into R
  auto partials = [&](const float* __restrict__ hs, const float* __restrict__ ts, int ld, int cb,
                      int CW, int KL) {
    float acc[4];
    int col[4], kl[4];
    // loads are unconditional (clamped to a valid address) and the term is selected
    // afterwards: loads under per-lane branches wait for each other
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = lane + 64 * j;
      col[j] = cb + i % CW;
      kl[j] = i / CW;
      const float tv = ts[(int64_t)(b - 1) * ld + min(col[j], ld - 1)];
      acc[j] = (kl[j] == 0 && col[j] < ld) ? tv : 0.f;
    }
    for (int r0 = 0; b + r0 * KL <= kend; r0 += 4) {   // four rounds' loads in flight
      float hv[4][4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int k = min(b + kl[j] + (r0 + rr) * KL, kend);
          hv[rr][j] = hs[(int64_t)k * ld + min(col[j], ld - 1)];
        }
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (col[j] < ld && b + kl[j] + (r0 + rr) * KL <= kend) acc[j] += hv[rr][j];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) R[lane + 64 * j] = acc[j];
  };
  int cw = 1;
  while (cw < d && cw < 256) cw <<= 1;
  const int KL = 256 / cw;
  for (int cb = 0; cb < d; cb += cw) {
    partials(head, tail, d, cb, cw, KL);
    __builtin_amdgcn_wave_barrier();                // one wave: its LDS ops stay in order
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = lane + 64 * j;
      if (i < cw && cb + i < d) {
        float t = R[i];
        for (int z = 1; z < KL; ++z) t += R[z * cw + i];
        if (compact) dense[row * d + cb + i] = t; else dense[row * d + cb + i] += t;
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (dense1) {          // PAIR: the one-column source, as the d = 1 fixup sums it
    partials(head1, tail1, 1, 0, 1, 256);
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
      // partial sums without a term are +0: adding them in order only turns a -0 running
      // sum into +0, which one add of +0 does as well
      const int m = min(256, kend - b + 1);
      float t = R[0];
      for (int z = 1; z < m; ++z) t += R[z];
      if (m < 256) t += 0.f;
      dense1[row] = t;
    }
  }
}

static inline unsigned fixup_blocks(int n_chunks) {
  return (unsigned)((n_chunks - 1 + kFixWaves - 1) / kFixWaves);
}

// Narrow rows (2 <= d <= 16) with pos_seg (the segment of every sorted position, from
// the chained block sort): chunk c of CH = 8 sorted positions owns the same pieces as
// in scatter_chunks_kernel (pieces counted from each segment's first position) — those
// whose start lies in [p0, p1) — and sums them in the same order, so the outputs are
// bit for bit the same. No search and no serial walk over segments: the 16 lanes of a
// group each resolve one position of the window [p0, p0 + 2 CH) (its perm, segment,
// piece, whether the chunk owns it, piece start / end), every lane then loads its
// column of the 16 window rows at once and folds them in order.
constexpr int kWinKindFinal = 0, kWinKindTail = 1, kWinKindHead = 2;
template <bool PAIR>
__global__ __launch_bounds__(256) void scatter_window_kernel(
    const float* __restrict__ rows, int d, const int32_t* __restrict__ perm,
    const int32_t* __restrict__ pos_seg, const int32_t* __restrict__ uniq,
    const int32_t* __restrict__ seg, const int32_t* __restrict__ n_uniq_dev,
    float* __restrict__ dense, int64_t n_rows, float* __restrict__ head,
    float* __restrict__ tail, int32_t* __restrict__ tail_seg, int n_chunks, int compact,
    const float* __restrict__ rows1, float* __restrict__ dense1, float* __restrict__ head1,
    float* __restrict__ tail1) {
  constexpr int G = 16, CH = 8, W = 2 * CH;
  const int nu = n_uniq_dev[0];
  const int n = seg[nu];
  const int lane = threadIdx.x & 63, gb = lane & ~(G - 1), l = lane & (G - 1);
  const int c = (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G);
  if (c >= n_chunks) return;
  const int p0 = c * CH;
  if (nu == 0 || p0 >= n) {
    if (l == 0) tail_seg[c] = -1;
    return;
  }
  const int p1 = min(n, p0 + CH);
  // lane l resolves window position q = p0 + l
  const int q = p0 + l;
  int pq = 0, info = 0, dst = 0;      // info: 1 owned | 2 piece start | 4 piece end | kind << 3
  if (q < n) {
    pq = perm[q];
    const int u = pos_seg[q];
    const int s0 = seg[u], e = seg[u + 1];
    const int ps = s0 + (q - s0) / CH * CH;
    if (ps >= p0 && ps < p1) {
      const int pe = min(e, ps + CH);
      const int kind = ps != s0 ? kWinKindHead : (e - s0 <= CH ? kWinKindFinal : kWinKindTail);
      info = 1 | (q == ps ? 2 : 0) | (q == pe - 1 ? 4 : 0) | (kind << 3);
      dst = kind == kWinKindFinal ? (compact ? u : uniq[u]) : u;
    }
  }
  // the multi-piece segment starting here (its first piece is a tail piece), if any
  const uint64_t tb = __ballot((info & 2) && (info >> 3) == kWinKindTail);
  const uint64_t gm = tb & (0xFFFFull << gb);
  const int tl = gm ? __builtin_ctzll(gm) : gb;
  const int tsu = __shfl(dst, tl, 64);
  if (l == 0) tail_seg[c] = gm ? tsu : -1;
  int pt[W], it[W], dt[W];
#pragma unroll
  for (int t = 0; t < W; ++t) {
    pt[t] = __shfl(pq, gb + t, 64);
    it[t] = __shfl(info, gb + t, 64);
    dt[t] = __shfl(dst, gb + t, 64);
  }
  // every lane loads all W rows (unowned positions read row pt = 0 of a valid position;
  // their terms are skipped below): loads under per-lane branches wait for each other
  float v[W], v1[W];
  const int lc = min(l, d - 1);
#pragma unroll
  for (int t = 0; t < W; ++t) {
    v[t] = rows[(int64_t)pt[t] * d + lc];
    if (PAIR) v1[t] = rows1[pt[t]];
  }
  float acc = 0.f, acc1 = 0.f;
#pragma unroll
  for (int t = 0; t < W; ++t) {
    if (!(it[t] & 1)) continue;
    acc = ((it[t] & 2) ? 0.f : acc) + v[t];
    if (PAIR) acc1 = ((it[t] & 2) ? 0.f : acc1) + v1[t];
    if (!(it[t] & 4)) continue;
    const int kind = it[t] >> 3;
    if (kind == kWinKindFinal) {
      const int64_t row = dt[t];
      if (l < d && row >= 0 && row < n_rows) {
        if (compact) dense[row * d + l] = acc; else dense[row * d + l] += acc;
      }
      if (PAIR && l == 0) dense1[dt[t]] = acc1;
    } else {
      float* out = (kind == kWinKindTail ? tail : head) + (int64_t)c * d;
      if (l < d) out[l] = acc;
      if (PAIR && l == 0) (kind == kWinKindTail ? tail1 : head1)[c] = acc1;
    }
  }
}

// Wide rows (16 < d <= 256) with pos_seg: chunk c of CH = 32 sorted positions owns the
// same pieces as scatter_chunks_kernel and sums them in the same order (bit for bit).
// One wave per chunk: lane l resolves window position p0 + l of [p0, p0 + 64) (perm,
// segment, piece, ownership); then the wave walks the window in order, eight positions'
// row loads in flight at a time — position t's perm and flags come from lane t by
// readlane, so the walk is uniform (scalar branches) and every row read is one coalesced
// access of the lanes' columns (l, l + 64, ...).
template <int MAXC>
__global__ __launch_bounds__(256) void scatter_wide_window_kernel(
    const float* __restrict__ rows, int d, const int32_t* __restrict__ perm,
    const int32_t* __restrict__ pos_seg, const int32_t* __restrict__ uniq,
    const int32_t* __restrict__ seg, const int32_t* __restrict__ n_uniq_dev,
    float* __restrict__ dense, int64_t n_rows, float* __restrict__ head,
    float* __restrict__ tail, int32_t* __restrict__ tail_seg, int n_chunks, int compact) {
  constexpr int CH = 32, W = 64;
  const int nu = n_uniq_dev[0];
  const int n = seg[nu];
  const int lane = threadIdx.x & 63;
  const int c = __builtin_amdgcn_readfirstlane(
      (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6));
  if (c >= n_chunks) return;
  const int p0 = c * CH;
  if (nu == 0 || p0 >= n) {
    if (lane == 0) tail_seg[c] = -1;
    return;
  }
  const int p1 = min(n, p0 + CH);
  const int q = p0 + lane;
  int pq = 0, info = 0, dst = 0;      // info: 1 owned | 2 piece start | 4 piece end | kind << 3
  if (q < n) {
    pq = perm[q];
    const int u = pos_seg[q];
    const int s0 = seg[u], e = seg[u + 1];
    const int ps = s0 + (q - s0) / CH * CH;
    if (ps >= p0 && ps < p1) {
      const int pe = min(e, ps + CH);
      const int kind = ps != s0 ? kWinKindHead : (e - s0 <= CH ? kWinKindFinal : kWinKindTail);
      info = 1 | (q == ps ? 2 : 0) | (q == pe - 1 ? 4 : 0) | (kind << 3);
      dst = kind == kWinKindFinal ? (compact ? u : uniq[u]) : u;
    }
  }
  const uint64_t tb = __ballot((info & 2) && (info >> 3) == kWinKindTail);
  const int tsu = tb ? __builtin_amdgcn_readlane(dst, __builtin_ctzll(tb)) : -1;
  if (lane == 0) tail_seg[c] = tsu;
  int col[MAXC];
#pragma unroll
  for (int j = 0; j < MAXC; ++j) col[j] = min(lane + 64 * j, d - 1);
  float acc[MAXC];
#pragma unroll
  for (int j = 0; j < MAXC; ++j) acc[j] = 0.f;
  for (int t0 = 0; t0 < W; t0 += 8) {
    int it[8], pt[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      it[j] = __builtin_amdgcn_readlane(info, t0 + j);
      pt[j] = __builtin_amdgcn_readlane(pq, t0 + j);
    }
    float v[8][MAXC];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int cc = 0; cc < MAXC; ++cc)
        v[j][cc] = (it[j] & 1) ? rows[(int64_t)pt[j] * d + col[cc]] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (!(it[j] & 1)) continue;
#pragma unroll
      for (int cc = 0; cc < MAXC; ++cc) acc[cc] = ((it[j] & 2) ? 0.f : acc[cc]) + v[j][cc];
      if (!(it[j] & 4)) continue;
      const int kind = it[j] >> 3;
      const int dt = __builtin_amdgcn_readlane(dst, t0 + j);
      if (kind == kWinKindFinal) {
        const int64_t row = dt;
        if (row >= 0 && row < n_rows) {
#pragma unroll
          for (int cc = 0; cc < MAXC; ++cc) {
            const int cl = lane + 64 * cc;
            if (cl < d) {
              if (compact) dense[row * d + cl] = acc[cc]; else dense[row * d + cl] += acc[cc];
            }
          }
        }
      } else {
        float* out = (kind == kWinKindTail ? tail : head) + (int64_t)c * d;
#pragma unroll
        for (int cc = 0; cc < MAXC; ++cc) {
          const int cl = lane + 64 * cc;
          if (cl < d) out[cl] = acc[cc];
        }
      }
    }
  }
}

// Union of two reduced gradients (the deferred optimizer's second level, one table read
// by two autograd Functions): A = (uA[0..nA), rowsA), B = (uB[0..nB), rowsB), each
// ascending and distinct. Output: the union rows ascending, each row's sum formed as the
// second-level segment_reduce of [A's rows; B's rows] formed it — (0 + a) + b, 0 + a,
// 0 + b — where a_pre = 1 takes a as already carrying its leading 0 + (a previous
// merge's output): the same bits, with no sort of the concatenated keys and no reduce.
// Two launches: a stable merge of the key lists (A before B on equal keys) into the
// merged order, then the run heads (tile counts summed over the tiles before, as in
// os_seg_kernel) with each head's one or two rows summed by a wave.
__device__ __forceinline__ int merge_lower(const int32_t* __restrict__ a, int n, int32_t key) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ int merge_upper(const int32_t* __restrict__ a, int n, int32_t key) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] <= key) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(256) void merge_place_kernel(
    const int32_t* __restrict__ uA, const int32_t* __restrict__ nA_dev, int capA,
    const int32_t* __restrict__ uB, const int32_t* __restrict__ nB_dev, int capB,
    int32_t* __restrict__ mk, int32_t* __restrict__ ref) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int nA = nA_dev[0], nB = nB_dev[0];
  if (i < capA) {
    if (i >= nA) return;
    const int32_t key = uA[i];
    const int pos = (int)i + merge_lower(uB, nB, key);
    mk[pos] = key;
    ref[pos] = (int32_t)i;
  } else if (i < (int64_t)capA + capB) {
    const int j = (int)(i - capA);
    if (j >= nB) return;
    const int32_t key = uB[j];
    const int pos = j + merge_upper(uA, nA, key);
    mk[pos] = key;
    ref[pos] = (int32_t)(0x80000000u | (uint32_t)j);
  }
}

constexpr int kMergeThreads = 256;
constexpr int kMergeIpt = 2;
constexpr int kMergeTile = kMergeThreads * kMergeIpt;   // merged positions per workgroup

// one output row's (up to two) source rows folded, V floats at column c
template <int V>
__device__ __forceinline__ void merge_fold(const float* __restrict__ s0,
                                           const float* __restrict__ s1, bool pre0, bool two,
                                           float* __restrict__ dst) {
#pragma unroll
  for (int e = 0; e < V; ++e) {
    float v = s0[e];
    if (!pre0) v = 0.f + v;
    if (two) v = v + s1[e];
    dst[e] = v;
  }
}

template <int V>
__global__ __launch_bounds__(kMergeThreads) void merge_compact_kernel(
    const int32_t* __restrict__ mk, const int32_t* __restrict__ ref,
    const int32_t* __restrict__ nA_dev, const int32_t* __restrict__ nB_dev,
    const float* __restrict__ rowsA, const float* __restrict__ rowsB, int d, int a_pre,
    int32_t* __restrict__ uniq_out, int32_t* __restrict__ n_out, float* __restrict__ rows_out,
    uint32_t* __restrict__ look, uint32_t* __restrict__ ticket) {
  __shared__ int scan[kMergeThreads / 64 + 1];
  __shared__ int hp[kMergeTile];                  // merged position of each run head
  __shared__ int h0[kMergeTile], h1[kMergeTile];  // each head's source rows
  __shared__ int prefix, n_heads, last;
  const int m = nA_dev[0] + nB_dev[0];
  const int64_t tile = blockIdx.x;
  const int base = (int)(tile * kMergeTile);
  const int i0 = base + threadIdx.x * kMergeIpt;
  int f = 0;
#pragma unroll
  for (int j = 0; j < kMergeIpt; ++j) {
    const int p = i0 + j;
    if (p < m) f += (p == 0 || mk[p - 1] != mk[p]) ? 1 : 0;
  }
  int tot;
  const int ex = block_exclusive_scan(f, scan, &tot);
  if (threadIdx.x == 0) os_store(look + tile, kOsFlagA | (uint32_t)tot);
  {
    const uint32_t part = os_sum_before(look, tile, 1, threadIdx.x, kMergeThreads);
    int all;
    (void)block_exclusive_scan((int)part, scan, &all);
    if (threadIdx.x == 0) {
      prefix = all;
      n_heads = tot;
      if (tile == gridDim.x - 1) n_out[0] = all + tot;
    }
  }
  int o = ex;
#pragma unroll
  for (int j = 0; j < kMergeIpt; ++j) {
    const int p = i0 + j;
    if (p < m && (p == 0 || mk[p - 1] != mk[p])) hp[o++] = p;
  }
  __syncthreads();
  // per head: its one or two source rows, resolved once (LDS), uniq written
  for (int h = threadIdx.x; h < n_heads; h += kMergeThreads) {
    const int p = hp[h];
    const int32_t key = mk[p];
    const int r0 = ref[p];
    const bool two = p + 1 < m && mk[p + 1] == key;
    h0[h] = r0;                                    // A row, or B row | 0x80000000
    h1[h] = two ? (ref[p + 1] & 0x7fffffff) : -1;  // the B row of a row in both
    uniq_out[prefix + h] = key;
  }
  __syncthreads();
  // (head, column group) items over the block's lanes, eight items' loads in flight
  const int dv = d / V;
  const int items = n_heads * dv;
  for (int it0 = threadIdx.x; it0 < items; it0 += 8 * kMergeThreads) {
    float a[8][V], b[8][V];
    int hh[8], cc[8];
    bool tw[8], pre[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int it = min(it0 + j * kMergeThreads, items - 1);
      const int h = it / dv;
      cc[j] = (it - h * dv) * V;
      hh[j] = h;
      const int r0 = h0[h], r1 = h1[h];
      tw[j] = r1 >= 0;
      const bool fromA = r0 >= 0;
      pre[j] = fromA && a_pre;
      const float* s0 = (fromA ? rowsA + (int64_t)r0 * d
                               : rowsB + (int64_t)(r0 & 0x7fffffff) * d) + cc[j];
      const float* s1 = rowsB + (int64_t)(tw[j] ? r1 : 0) * d + cc[j];
#pragma unroll
      for (int e = 0; e < V; ++e) {
        a[j][e] = s0[e];
        b[j][e] = s1[e];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (it0 + j * kMergeThreads >= items) continue;
      merge_fold<V>(a[j], b[j], pre[j], tw[j], rows_out + (int64_t)(prefix + hh[j]) * d + cc[j]);
    }
  }
  os_cleanup(ticket, look, gridDim.x, &last);
}

}  // namespace mirec

using namespace mirec;

extern "C" size_t mirec_segment_sort_workspace_size(int64_t n, int64_t key_space) {
  (void)key_space;
  if (n <= kLdsMax) return 256;
  return radix_ws_bytes(n);
}

extern "C" int mirec_segment_sort_batched(const int64_t* keys, int64_t n, int64_t batch_n,
                                          int64_t key_space, int32_t* perm, int32_t* uniq,
                                          int32_t* seg, int32_t* n_uniq_dev, void* ws,
                                          size_t ws_bytes, void* stream) {
  if (n < 0 || key_space <= 0 || key_space > INT32_MAX || n > INT32_MAX || batch_n < 0 ||
      !seg || !n_uniq_dev || (n > 0 && (!keys || !perm || !uniq || batch_n == 0))) {
    set_error("mirec_segment_sort: bad arguments");
    return -1;
  }
  hipStream_t st = (hipStream_t)stream;
  int nb = 0;
  while (nb < 31 && ((int64_t)1 << nb) < key_space) ++nb;
  if (n == 0) {  // one empty batch: seg[0] = 0, n_uniq = 0
    hipLaunchKernelGGL(segsort_lds_kernel, dim3(1), dim3(kSortThreads), 0, st, keys, (int64_t)0,
                       1, nb, perm, uniq, seg, n_uniq_dev);
    return launch_status("mirec_segment_sort");
  }
  const int64_t n_batches = (n + batch_n - 1) / batch_n;
  if (n_batches == 1 && n > kLdsMax) {
    if (!ws || ws_bytes < radix_ws_bytes(n)) {
      set_error("mirec_segment_sort: workspace %zu < %zu", ws_bytes, radix_ws_bytes(n));
      return -1;
    }
    return radix_segment_sort(keys, (int)n, nb, perm, uniq, seg, n_uniq_dev, ws, st);
  }
  if (batch_n <= kLdsMax) {
    hipLaunchKernelGGL(segsort_lds_kernel, dim3((unsigned)n_batches), dim3(kSortThreads), 0, st,
                       keys, n, (int)batch_n, nb, perm, uniq, seg, n_uniq_dev);
  } else {
    const size_t need = (size_t)4 * (size_t)(n_batches * batch_n) * sizeof(int32_t);
    if (!ws || ws_bytes < need) {
      set_error("mirec_segment_sort: workspace %zu < %zu", ws_bytes, need);
      return -1;
    }
    hipLaunchKernelGGL(segsort_global_kernel, dim3((unsigned)n_batches), dim3(kSortThreads), 0,
                       st, keys, n, (int)batch_n, nb, perm, uniq, seg, n_uniq_dev,
                       (int32_t*)ws);
  }
  return launch_status("mirec_segment_sort");
}

extern "C" size_t mirec_segment_sort_blocks_workspace_size(int64_t n, int64_t block_n) {
  if (n <= 0 || block_n <= 0) return 256;
  const int64_t nb = (n + block_n - 1) / block_n;
  return (size_t)(2 * nb * block_n + nb * (block_n + 1) + nb) * sizeof(int32_t) + 256;
}

extern "C" int mirec_segment_sort_blocks(const int64_t* keys, int64_t n, int64_t block_n,
                                         int64_t key_space, int32_t* perm, int32_t* uniq,
                                         int32_t* seg, int32_t* n_uniq_dev, void* ws,
                                         size_t ws_bytes, void* stream) {
  if (n <= 0 || block_n <= 0 || block_n > kLdsMax || key_space <= 0 ||
      key_space > INT32_MAX || n > INT32_MAX || !keys || !perm || !uniq || !seg || !n_uniq_dev) {
    set_error("mirec_segment_sort_blocks: bad arguments (0 < block_n <= %d)", kLdsMax);
    return -1;
  }
  if (!ws || ws_bytes < mirec_segment_sort_blocks_workspace_size(n, block_n)) {
    set_error("mirec_segment_sort_blocks: workspace too small");
    return -1;
  }
  const int64_t nb = (n + block_n - 1) / block_n;
  int32_t* perm_t = (int32_t*)ws;
  int32_t* uniq_t = perm_t + nb * block_n;
  int32_t* seg_t = uniq_t + nb * block_n;
  int32_t* nu_t = seg_t + nb * (block_n + 1);
  int nbits = 0;
  while (nbits < 31 && ((int64_t)1 << nbits) < key_space) ++nbits;
  hipStream_t st = (hipStream_t)stream;
  if (block_n <= kR8Max)       // 8-bit digits over the block's key span
    hipLaunchKernelGGL(segsort_radix8_kernel, dim3((unsigned)nb), dim3(kR8Threads), 0, st, keys,
                       n, (int)block_n, perm_t, uniq_t, seg_t, nu_t, (int32_t*)nullptr,
                       (int32_t*)nullptr, SortFields{});
  else
    hipLaunchKernelGGL(segsort_lds_kernel, dim3((unsigned)nb), dim3(kSortThreads), 0, st, keys,
                       n, (int)block_n, nbits, perm_t, uniq_t, seg_t, nu_t);
  hipLaunchKernelGGL(blocks_concat_kernel, dim3((unsigned)nb), dim3(256), 0, st, perm_t, uniq_t,
                     seg_t, nu_t, n, (int)block_n, (int)nb, perm, uniq, seg, n_uniq_dev);
  return launch_status("mirec_segment_sort_blocks");
}

extern "C" int mirec_segment_sort_blocks_chained(const int64_t* keys, int64_t n,
                                                 int64_t block_n, int64_t key_space,
                                                 int32_t* perm, int32_t* uniq, int32_t* seg,
                                                 int32_t* n_uniq_dev, int32_t* status,
                                                 int64_t n_status, int32_t* pos_seg,
                                                 void* stream) {
  if (n <= 0 || block_n <= 0 || block_n > kR8Max || key_space <= 0 || key_space > INT32_MAX ||
      n > INT32_MAX || !keys || !perm || !uniq || !seg || !n_uniq_dev || !status) {
    set_error("mirec_segment_sort_blocks_chained: bad arguments (0 < block_n <= %d)", kR8Max);
    return -1;
  }
  const int64_t nb = (n + block_n - 1) / block_n;
  if (nb > kChainMaxBlocks || n_status < nb + 1) {
    set_error("mirec_segment_sort_blocks_chained: %lld blocks need status[%lld] (at most %d "
              "blocks)", (long long)nb, (long long)(nb + 1), kChainMaxBlocks);
    return -1;
  }
  hipLaunchKernelGGL(segsort_radix8_kernel, dim3((unsigned)nb), dim3(kR8Threads), 0,
                     (hipStream_t)stream, keys, n, (int)block_n, perm, uniq, seg, n_uniq_dev,
                     status, pos_seg, SortFields{});
  return launch_status("mirec_segment_sort_blocks_chained");
}

extern "C" int mirec_segment_sort_fields_chained(const int64_t* const* cols,
                                                 const int64_t* offsets, int32_t n_fields,
                                                 int64_t B, int64_t key_space, int64_t* keys_out,
                                                 int32_t* perm, int32_t* uniq, int32_t* seg,
                                                 int32_t* n_uniq_dev, int32_t* status,
                                                 int64_t n_status, int32_t* pos_seg,
                                                 void* stream) {
  if (n_fields <= 0 || n_fields > kSortFields || B <= 0 || B > kR8Max || key_space <= 0 ||
      key_space > INT32_MAX || !cols || !offsets || !keys_out || !perm || !uniq || !seg ||
      !n_uniq_dev || !status || n_status < n_fields + 1) {
    set_error("mirec_segment_sort_fields_chained: bad arguments (1..%d fields of 1..%d keys)",
              kSortFields, kR8Max);
    return -1;
  }
  SortFields SF;
  memset(&SF, 0, sizeof(SF));
  for (int f = 0; f < n_fields; ++f) {
    if (!cols[f]) {
      set_error("mirec_segment_sort_fields_chained: field %d has no column", f);
      return -1;
    }
    SF.col[f] = cols[f];
    SF.off[f] = offsets[f];
  }
  SF.keys_out = keys_out;
  hipLaunchKernelGGL(segsort_radix8_kernel, dim3((unsigned)n_fields), dim3(kR8Threads), 0,
                     (hipStream_t)stream, (const int64_t*)keys_out, (int64_t)n_fields * B, (int)B,
                     perm, uniq, seg, n_uniq_dev, status, pos_seg, SF);
  return launch_status("mirec_segment_sort_fields_chained");
}

extern "C" int64_t mirec_segment_sort_onesweep_status_words(int64_t n) {
  return n > 0 ? os_status_words(n) : 0;
}

extern "C" int mirec_segment_sort_onesweep(const int64_t* keys, int64_t n, int64_t key_space,
                                           int32_t* perm, int32_t* uniq, int32_t* seg,
                                           int32_t* n_uniq_dev, int32_t* pos_seg, void* ws,
                                           size_t ws_bytes, int32_t* status, int64_t n_status,
                                           void* stream) {
  if (n <= 0 || n > (int64_t)kOsVal || key_space <= 0 || key_space > INT32_MAX || !keys ||
      !perm || !uniq || !seg || !n_uniq_dev || !status) {
    set_error("mirec_segment_sort_onesweep: bad arguments (0 < n < 2^30)");
    return -1;
  }
  if (n_status < os_status_words(n) || !ws || ws_bytes < (size_t)4 * (size_t)n * 4) {
    set_error("mirec_segment_sort_onesweep: status (%lld words) or workspace too small",
              (long long)os_status_words(n));
    return -1;
  }
  int nbits = 0;
  while (nbits < 31 && ((int64_t)1 << nbits) < key_space) ++nbits;
  const int passes = nbits == 0 ? 1 : (nbits + 7) / 8;
  const int64_t tiles = os_tiles(n);
  uint32_t* hist = (uint32_t*)status;
  uint32_t* look = hist + kOsMaxPasses * 256;
  uint32_t* slook = look + (int64_t)kOsMaxPasses * tiles * 256;
  uint32_t* tickets = slook + tiles;
  int32_t* kA = (int32_t*)ws;
  int32_t* vA = kA + n;
  int32_t* kB = vA + n;
  int32_t* vB = kB + n;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(os_hist_kernel, dim3((unsigned)tiles), dim3(kOsThreads), 0, st, keys,
                     (int)n, passes, kA, vA, hist);
  for (int p = 0; p < passes; ++p) {
    int32_t* vo = p == passes - 1 ? perm : vB;     // the last pass writes perm itself
    hipLaunchKernelGGL(os_pass_kernel, dim3((unsigned)tiles), dim3(kOsThreads), 0, st, kA, vA,
                       (int)n, 8 * p, tiles, hist + p * 256, look + (int64_t)p * tiles * 256,
                       tickets + p, kB, vo);
    int32_t* t = kA; kA = kB; kB = t;
    t = vA; vA = vB; vB = t;
  }
  hipLaunchKernelGGL(os_seg_kernel, dim3((unsigned)tiles), dim3(kOsThreads), 0, st, kA, (int)n,
                     tiles, slook, tickets + kOsMaxPasses, uniq, seg, n_uniq_dev, pos_seg);
  return launch_status("mirec_segment_sort_onesweep");
}

extern "C" int mirec_segment_sort(const int64_t* keys, int64_t n, int64_t key_space,
                                  int32_t* perm, int32_t* uniq, int32_t* seg,
                                  int32_t* n_uniq_dev, void* ws, size_t ws_bytes, void* stream) {
  return mirec_segment_sort_batched(keys, n, n > 0 ? n : 1, key_space, perm, uniq, seg,
                                    n_uniq_dev, ws, ws_bytes, stream);
}

extern "C" size_t mirec_segment_scatter_add_workspace_size(int64_t n, int32_t d) {
  const int64_t chunks = (n + kScatChunkMin - 1) / kScatChunkMin;
  return (size_t)2 * (size_t)chunks * (size_t)(d > 0 ? d : 1) * sizeof(float) +
         (size_t)chunks * sizeof(int32_t) + 256;
}

static int scatter_impl(const float* rows, int32_t d, const int32_t* perm, const int32_t* uniq,
                        const int32_t* seg, const int32_t* n_uniq_dev, int64_t n, float* dense,
                        int64_t n_rows, void* ws, size_t ws_bytes, int compact, void* stream) {
  if (n == 0) return 0;
  if (!rows || !perm || !uniq || !seg || !n_uniq_dev || !dense || d <= 0 || d > 256 || n < 0 ||
      n > INT32_MAX) {
    set_error("mirec_segment_scatter_add_f32: bad arguments (1 <= d <= 256)");
    return -1;
  }
  if (!ws || ws_bytes < mirec_segment_scatter_add_workspace_size(n, d)) {
    set_error("mirec_segment_scatter_add_f32: workspace too small");
    return -1;
  }
  const int chunks = (int)((n + scat_chunk(d) - 1) / scat_chunk(d));
  float* head = (float*)ws;
  float* tail = head + (int64_t)chunks * d;
  int32_t* tail_seg = (int32_t*)(tail + (int64_t)chunks * d);
  hipStream_t st = (hipStream_t)stream;
#define MIREC_SCAT(GG, DM)                                                                    \
  {                                                                                          \
    const int64_t groups_per_block = 4 * (64 / GG);                                          \
    hipLaunchKernelGGL((scatter_chunks_kernel<GG, DM>),                                       \
                       dim3((unsigned)((chunks + groups_per_block - 1) / groups_per_block)),  \
                       dim3(256), 0, st, rows, d, perm, uniq, seg, n_uniq_dev, dense, n_rows, \
                       head, tail, tail_seg, chunks, compact);                                \
  }
  if (d == 1) MIREC_SCAT(1, 1)
  else if (d <= 4) MIREC_SCAT(4, 4)
  else if (d <= 16) MIREC_SCAT(16, 16)
  else if (d <= 32) MIREC_SCAT(32, 32)
  else if (d <= 64) MIREC_SCAT(64, 64)
  else MIREC_SCAT(64, 256)
#undef MIREC_SCAT
  if (chunks > 1)
    hipLaunchKernelGGL(scatter_fixup_kernel, dim3(fixup_blocks(chunks)), dim3(64 * kFixWaves), 0,
                       st, d,
                       uniq, seg, tail_seg, dense, n_rows, head, tail, chunks, compact);
  return launch_status("mirec_segment_scatter_add_f32");
}

extern "C" int mirec_segment_scatter_add_f32(const float* rows, int32_t d, const int32_t* perm,
                                             const int32_t* uniq, const int32_t* seg,
                                             const int32_t* n_uniq_dev, int64_t n, float* dense,
                                             int64_t n_rows, void* ws, size_t ws_bytes,
                                             void* stream) {
  return scatter_impl(rows, d, perm, uniq, seg, n_uniq_dev, n, dense, n_rows, ws, ws_bytes, 0,
                      stream);
}

static int reduce2_impl(const float* rows, int32_t d, const float* rows1, const int32_t* perm,
                        const int32_t* pos_seg, const int32_t* uniq, const int32_t* seg,
                        const int32_t* n_uniq_dev, int64_t n, float* out, float* out1, void* ws,
                        size_t ws_bytes, void* stream) {
  if (n == 0) return 0;
  if (!rows || !rows1 || !perm || !uniq || !seg || !n_uniq_dev || !out || !out1 || d < 2 ||
      d > 16 || n < 0 || n > INT32_MAX) {
    set_error("mirec_segment_reduce2_f32: bad arguments (2 <= d <= 16)");
    return -1;
  }
  if (!ws || ws_bytes < mirec_segment_scatter_add_workspace_size(n, d + 1)) {
    set_error("mirec_segment_reduce2_f32: workspace too small");
    return -1;
  }
  static_assert(MIREC_SCAT_NARROW_CH == 8, "the pair needs the one-column chunk size");
  const int chunks = (int)((n + scat_chunk(d) - 1) / scat_chunk(d));
  float* head = (float*)ws;
  float* tail = head + (int64_t)chunks * d;
  float* head1 = tail + (int64_t)chunks * d;
  float* tail1 = head1 + chunks;
  int32_t* tail_seg = (int32_t*)(tail1 + chunks);
  hipStream_t st = (hipStream_t)stream;
  const int64_t gpb = 4 * (64 / 16);
  if (pos_seg)
    hipLaunchKernelGGL((scatter_window_kernel<true>), dim3((unsigned)((chunks + gpb - 1) / gpb)),
                       dim3(256), 0, st, rows, d, perm, pos_seg, uniq, seg, n_uniq_dev, out, n,
                       head, tail, tail_seg, chunks, 1, rows1, out1, head1, tail1);
  else if (d <= 4)
    hipLaunchKernelGGL((scatter_chunks_kernel<4, 4, true>),
                       dim3((unsigned)((chunks + 4 * 16 - 1) / (4 * 16))), dim3(256), 0, st, rows,
                       d, perm, uniq, seg, n_uniq_dev, out, n, head, tail, tail_seg, chunks, 1,
                       rows1, out1, head1, tail1);
  else
    hipLaunchKernelGGL((scatter_chunks_kernel<16, 16, true>),
                       dim3((unsigned)((chunks + gpb - 1) / gpb)), dim3(256), 0, st, rows, d,
                       perm, uniq, seg, n_uniq_dev, out, n, head, tail, tail_seg, chunks, 1,
                       rows1, out1, head1, tail1);
  if (chunks > 1)
    hipLaunchKernelGGL(scatter_fixup_kernel, dim3(fixup_blocks(chunks)), dim3(64 * kFixWaves), 0,
                       st, d,
                       uniq, seg, tail_seg, out, n, head, tail, chunks, 1, out1, head1, tail1);
  return launch_status("mirec_segment_reduce2_f32");
}

extern "C" int mirec_segment_reduce2_f32(const float* rows, int32_t d, const float* rows1,
                                         const int32_t* perm, const int32_t* uniq,
                                         const int32_t* seg, const int32_t* n_uniq_dev, int64_t n,
                                         float* out, float* out1, void* ws, size_t ws_bytes,
                                         void* stream) {
  return reduce2_impl(rows, d, rows1, perm, nullptr, uniq, seg, n_uniq_dev, n, out, out1, ws,
                      ws_bytes, stream);
}

extern "C" int mirec_segment_reduce2_pos_seg_f32(const float* rows, int32_t d,
                                                 const float* rows1, const int32_t* perm,
                                                 const int32_t* pos_seg, const int32_t* uniq,
                                                 const int32_t* seg, const int32_t* n_uniq_dev,
                                                 int64_t n, float* out, float* out1, void* ws,
                                                 size_t ws_bytes, void* stream) {
  if (!pos_seg) {
    set_error("mirec_segment_reduce2_pos_seg_f32: pos_seg is null");
    return -1;
  }
  return reduce2_impl(rows, d, rows1, perm, pos_seg, uniq, seg, n_uniq_dev, n, out, out1, ws,
                      ws_bytes, stream);
}

extern "C" int mirec_segment_reduce_pos_seg_f32(const float* rows, int32_t d,
                                                const int32_t* perm, const int32_t* pos_seg,
                                                const int32_t* uniq, const int32_t* seg,
                                                const int32_t* n_uniq_dev, int64_t n, float* out,
                                                void* ws, size_t ws_bytes, void* stream) {
  if (n == 0) return 0;
  if (!rows || !perm || !pos_seg || !uniq || !seg || !n_uniq_dev || !out || d <= 0 ||
      d > 256 || n < 0 || n > INT32_MAX) {
    set_error("mirec_segment_reduce_pos_seg_f32: bad arguments (1 <= d <= 256)");
    return -1;
  }
  if (!ws || ws_bytes < mirec_segment_scatter_add_workspace_size(n, d)) {
    set_error("mirec_segment_reduce_pos_seg_f32: workspace too small");
    return -1;
  }
  const int chunks = (int)((n + scat_chunk(d) - 1) / scat_chunk(d));
  float* head = (float*)ws;
  float* tail = head + (int64_t)chunks * d;
  int32_t* tail_seg = (int32_t*)(tail + (int64_t)chunks * d);
  hipStream_t st = (hipStream_t)stream;
  if (d <= 16) {
    const int64_t gpb = 4 * (64 / 16);
    hipLaunchKernelGGL((scatter_window_kernel<false>), dim3((unsigned)((chunks + gpb - 1) / gpb)),
                       dim3(256), 0, st, rows, d, perm, pos_seg, uniq, seg, n_uniq_dev, out, n,
                       head, tail, tail_seg, chunks, 1, nullptr, nullptr, nullptr, nullptr);
  } else {
    const dim3 grd((unsigned)((chunks + 3) / 4));   // four waves (chunks) per workgroup
#define MIREC_WIDE(MC)                                                                         hipLaunchKernelGGL((scatter_wide_window_kernel<MC>), grd, dim3(256), 0, st, rows, d, perm,                        pos_seg, uniq, seg, n_uniq_dev, out, n, head, tail, tail_seg, chunks, 1)
    if (d <= 64) MIREC_WIDE(1);
    else if (d <= 128) MIREC_WIDE(2);
    else MIREC_WIDE(4);
#undef MIREC_WIDE
  }
  if (chunks > 1)
    hipLaunchKernelGGL(scatter_fixup_kernel, dim3(fixup_blocks(chunks)), dim3(64 * kFixWaves), 0,
                       st, d, uniq, seg, tail_seg, out, n, head, tail, chunks, 1);
  return launch_status("mirec_segment_reduce_pos_seg_f32");
}

extern "C" int mirec_segment_merge2_f32(const int32_t* uA, const int32_t* nA_dev, int64_t capA,
                                        const float* rowsA, const int32_t* uB,
                                        const int32_t* nB_dev, int64_t capB, const float* rowsB,
                                        int32_t d, int32_t a_pre, int32_t* uniq_out,
                                        int32_t* n_out_dev, float* rows_out, void* ws,
                                        size_t ws_bytes, int32_t* status, int64_t n_status,
                                        void* stream) {
  const int64_t cap = capA + capB;
  if (!uA || !nA_dev || !rowsA || !uB || !nB_dev || !rowsB || !uniq_out || !n_out_dev ||
      !rows_out || !status || capA < 0 || capB < 0 || cap <= 0 || cap >= (int64_t)kOsVal ||
      d <= 0 || d > 1024) {
    set_error("mirec_segment_merge2_f32: bad arguments");
    return -1;
  }
  const int64_t tiles = (cap + kMergeTile - 1) / kMergeTile;
  if (!ws || ws_bytes < (size_t)(2 * cap) * sizeof(int32_t) || n_status < tiles + 1) {
    set_error("mirec_segment_merge2_f32: workspace (%lld B) or status (%lld words) too small",
              (long long)(2 * cap * 4), (long long)(tiles + 1));
    return -1;
  }
  int32_t* mk = (int32_t*)ws;
  int32_t* ref = mk + cap;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(merge_place_kernel, dim3((unsigned)((cap + 255) / 256)), dim3(256), 0, st,
                     uA, nA_dev, (int)capA, uB, nB_dev, (int)capB, mk, ref);
  if (d % 4 == 0)
    hipLaunchKernelGGL(merge_compact_kernel<4>, dim3((unsigned)tiles), dim3(kMergeThreads), 0, st,
                       mk, ref, nA_dev, nB_dev, rowsA, rowsB, d, a_pre, uniq_out, n_out_dev,
                       rows_out, (uint32_t*)status, (uint32_t*)status + tiles);
  else
    hipLaunchKernelGGL(merge_compact_kernel<1>, dim3((unsigned)tiles), dim3(kMergeThreads), 0, st,
                       mk, ref, nA_dev, nB_dev, rowsA, rowsB, d, a_pre, uniq_out, n_out_dev,
                       rows_out, (uint32_t*)status, (uint32_t*)status + tiles);
  return launch_status("mirec_segment_merge2_f32");
}

extern "C" int mirec_segment_reduce_f32(const float* rows, int32_t d, const int32_t* perm,
                                        const int32_t* uniq, const int32_t* seg,
                                        const int32_t* n_uniq_dev, int64_t n, float* out,
                                        void* ws, size_t ws_bytes, void* stream) {
  return scatter_impl(rows, d, perm, uniq, seg, n_uniq_dev, n, out, n, ws, ws_bytes, 1, stream);
}

// ---------------------------------------------------------------------------
// Look-ahead lists of the deferred Adam (adam.hip): for consecutive batches b,
// b+1 of a chunk, out_b = uniq(b+1) \ uniq(b) in ascending order — the rows the
// next forward pass reads that step b's Adam does not touch (device code: ahead.h).
namespace mirec {

__global__ __launch_bounds__(kSortThreads) void uniq_ahead_diff_kernel(
    const int32_t* __restrict__ uniq, const int32_t* __restrict__ n_uniq, int64_t stride,
    int64_t n_batches, int32_t* __restrict__ out, int32_t* __restrict__ n_out) {
  __shared__ int32_t a_lds[kDiffLds];
  __shared__ int scan_lds[kSortThreads / 64 + 1];
  uniq_ahead_diff_batch(uniq, n_uniq, stride, n_batches, out, n_out, blockIdx.x, a_lds, scan_lds);
}

struct DiffJob {
  const int32_t* uniq; const int32_t* n_uniq; int64_t stride; int32_t* out; int32_t* n_out;
};

// Both tables' look-ahead lists in one launch: workgroups [0, nb) table A, the rest B.
__global__ __launch_bounds__(kSortThreads) void uniq_ahead_diff2_kernel(DiffJob A, DiffJob B,
                                                                        int64_t nb) {
  __shared__ int32_t a_lds[kDiffLds];
  __shared__ int scan_lds[kSortThreads / 64 + 1];
  const bool a = (int64_t)blockIdx.x < nb;
  const DiffJob& J = a ? A : B;
  uniq_ahead_diff_batch(J.uniq, J.n_uniq, J.stride, nb, J.out, J.n_out,
                        a ? (int64_t)blockIdx.x : (int64_t)blockIdx.x - nb, a_lds, scan_lds);
}

}  // namespace mirec

extern "C" int mirec_uniq_ahead_diff(const int32_t* uniq, const int32_t* n_uniq, int64_t stride,
                                     int64_t n_batches, int32_t* out, int32_t* n_out,
                                     void* stream) {
  if (!uniq || !n_uniq || !out || !n_out || stride <= 0 || n_batches < 0) {
    mirec::set_error("mirec_uniq_ahead_diff: bad arguments");
    return -1;
  }
  if (n_batches == 0) return 0;
  hipLaunchKernelGGL(mirec::uniq_ahead_diff_kernel, dim3((unsigned)n_batches),
                     dim3(mirec::kSortThreads), 0, (hipStream_t)stream, uniq, n_uniq, stride,
                     n_batches, out, n_out);
  return mirec::launch_status("mirec_uniq_ahead_diff");
}

// ---- both tables of a chunk (mirec_prepare_chunk, gather.hip): one sort launch
// and one look-ahead launch when both fit the LDS path, else the separate calls.
namespace mirec {
int sort_chunk_pair(const int64_t* ukeys, int64_t nU_keys, int64_t Bu, int64_t u_space,
                    int32_t* u_perm, int32_t* u_uniq, int32_t* u_seg, int32_t* u_nu,
                    const int64_t* ikeys, int64_t nI_keys, int64_t Bi, int64_t i_space,
                    int32_t* i_perm, int32_t* i_uniq, int32_t* i_seg, int32_t* i_nu,
                    int64_t n_batches, int32_t* u_ahead, int32_t* u_nah, int32_t* i_ahead,
                    int32_t* i_nah, void* ws, size_t ws_bytes, hipStream_t st) {
  if (Bu <= kLdsMax && Bi <= kLdsMax && u_space <= INT32_MAX && i_space <= INT32_MAX &&
      nU_keys == n_batches * Bu && nI_keys == n_batches * Bi && n_batches > 0) {
    SortJob A = {ukeys, nU_keys, (int)Bu, nbits_for(u_space), u_perm, u_uniq, u_seg, u_nu};
    SortJob B = {ikeys, nI_keys, (int)Bi, nbits_for(i_space), i_perm, i_uniq, i_seg, i_nu};
    hipLaunchKernelGGL(segsort_lds2_kernel, dim3((unsigned)(2 * n_batches)), dim3(kSortThreads),
                       0, st, A, B, n_batches);
    int rc = launch_status("mirec_prepare_chunk: sort");
    if (rc || !u_ahead) return rc;
    DiffJob DA = {u_uniq, u_nu, Bu, u_ahead, u_nah};
    DiffJob DB = {i_uniq, i_nu, Bi, i_ahead, i_nah};
    hipLaunchKernelGGL(uniq_ahead_diff2_kernel, dim3((unsigned)(2 * n_batches)),
                       dim3(kSortThreads), 0, st, DA, DB, n_batches);
    return launch_status("mirec_prepare_chunk: look-ahead");
  }
  int rc = mirec_segment_sort_batched(ukeys, nU_keys, Bu, u_space, u_perm, u_uniq, u_seg, u_nu,
                                      ws, ws_bytes, st);
  if (rc) return rc;
  rc = mirec_segment_sort_batched(ikeys, nI_keys, Bi, i_space, i_perm, i_uniq, i_seg, i_nu, ws,
                                  ws_bytes, st);
  if (rc || !u_ahead) return rc;
  rc = mirec_uniq_ahead_diff(u_uniq, u_nu, Bu, n_batches, u_ahead, u_nah, st);
  if (rc) return rc;
  return mirec_uniq_ahead_diff(i_uniq, i_nu, Bi, n_batches, i_ahead, i_nah, st);
}
}  // namespace mirec
