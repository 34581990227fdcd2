// Cross-GPU exchange for the row-sharded C2 step: one process per
// GPU, every rank's receive WINDOW mapped into every other rank's address space (HIP
// IPC over xGMI), and the per-step exchanges done by kernels storing straight into the
// peers' windows, with a flag per (source, exchange) instead of RCCL collectives.
//
// Why: a row-sharded step exchanges ~1.5 MB per rank twice (the rows each slice reads,
// then its gradient rows back): latency-bound RCCL all-to-alls of ~10-20 µs each, two
// extra launches per step. Here the owner's gather stores each message row directly
// into the receiving rank's window and the last block raises one flag per peer; the
// consumer's next launch waits for the flags on the GPU (no host, no collective).
//
// Window (one uncached device allocation per rank, hipDeviceMallocUncached: no cache
// on either side holds its lines, so a peer's stores are what a later load reads):
//   [fwd rows: G x wcap x d floats][bwd rows: G x wcap x d][flags: kFlagSets x kMaxPeers int32]
// wcap = the largest message a plan can ask for; the step's exchanges use the plan's own
// cap (<= wcap) as the block stride, so a region holds block `src` (the rows rank src
// sent) at src * cap — the layout of the equal-block all-to-all it replaces.
//
// Hand-off. Everything a peer reads is in the windows, and the windows (rows and flags)
// are UNCACHED memory: a store to them is not held in any L2 and is visible once it is
// acknowledged (s_waitcnt vmcnt(0)), and a load of them is served from memory. The
// memory model's system-scope release (buffer_wbl2 + waitcnt) and acquire (buffer_inv)
// add L2 write-back / invalidation for CACHED data only — here that is pure cost: with
// one such release + acquire per block, a 3,072-block owner-Adam launch took 104 µs
// against 15.6 µs for the same rows without them (profiles/r06_ipc_adam_probe.txt).
// So: every block of a pushing launch drains its stores (s_waitcnt vmcnt(0) in each
// wave), meets, and one lane adds to the launch's arrival counter (a relaxed agent-scope
// add: an L2 atomic, coherent across the XCDs); the block whose add is last stores the
// exchange's sequence number into flag[set][me] of every peer (a relaxed system-scope
// store to uncached memory). The waiting side polls its own flags with system-scope
// loads and then reads the window (uncached) — a workgroup-scope acquire keeps the
// compiler from hoisting the window loads above the poll. Build with
// -DMIREC_COMM_FORMAL_FENCES for the memory model's own system-scope forms.
//
// Sequence numbers: each exchange set keeps a device counter per rank (cnt); a push
// raises flags to cnt + 1 and the wait for it sets cnt = cnt + 1 — every rank runs the
// same exchanges in the same order, so the counters agree without communication, and
// captured graphs replay with advancing values. A rank cannot run ahead by a whole
// exchange of the same set (its next push of a set needs the other set's flags, which
// need the peer's wait), so a flag never exceeds the value being waited for by more
// than nothing, and a window block is never overwritten while its reader still reads.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "adam_core.h"
#include "bpr_math.h"

namespace mirec {

constexpr int kMaxPeers = 64;
// 0 forward rows, 1 backward rows (the step), 2 alltoallv rows, 3 allreduce blocks, 4 the
// generic calls' entry / exit barriers
constexpr int kFlagSets = 5;
constexpr int kBarrierSet = 4;
constexpr int kXThreads = 256;
#ifdef MIREC_COMM_FORMAL_FENCES
constexpr int kArriveOrder = __ATOMIC_ACQ_REL, kFlagOrder = __ATOMIC_RELEASE;
constexpr int kArriveScope = __HIP_MEMORY_SCOPE_SYSTEM;
#else
constexpr int kArriveOrder = __ATOMIC_RELAXED, kFlagOrder = __ATOMIC_RELAXED;
constexpr int kArriveScope = __HIP_MEMORY_SCOPE_AGENT;
#endif

struct Peers {
  char* base[kMaxPeers];                // every rank's window in this process
};

struct XSig {                           // the flag raised at the end of a pushing launch
  int32_t* arrive;                      // arrival counters (kArriveInts, zero between)
  const int32_t* cnt;                   // this exchange set's counter (read)
  int64_t flag_off;                     // byte offset of flag set 0 in a window
  int32_t set, G, me;
};

__device__ __forceinline__ int32_t* flag_at(char* win, int64_t flag_off, int set, int src) {
  return reinterpret_cast<int32_t*>(win + flag_off) + set * kMaxPeers + src;
}

// Arrival of a launch's blocks in two levels (lane 0 of each block; true for the block
// that arrives last): block b counts into group b % kArriveGroups (its own 64-B line),
// the block completing a group into the top counter. A launch of a few thousand blocks
// on one counter serialises that many L2 atomics on one address (the owner-Adam launch:
// ~30 µs of its 47); here no address takes more than ~50. Counters are left zero.
constexpr int kArriveGroups = 64, kArriveStride = 16;   // int32s: one 64-B line each
constexpr int kArriveInts = (1 + kArriveGroups) * kArriveStride;

__device__ __forceinline__ bool arrive_last(int32_t* arrive) {
#ifdef MIREC_COMM_PROBE_NO_ARRIVE   // timing probe only (one rank: nothing waits on the flags)
  return false;
#endif
  const int nb = (int)(gridDim.x * gridDim.y);
  const int b = (int)(blockIdx.y * gridDim.x + blockIdx.x);
  const int g = b % kArriveGroups;
  const int gsz = (nb - g + kArriveGroups - 1) / kArriveGroups;
  if (gsz > 1) {
    int32_t* cg = arrive + (1 + g) * kArriveStride;
    if (__hip_atomic_fetch_add(cg, 1, kArriveOrder, kArriveScope) != gsz - 1) return false;
    __hip_atomic_store(cg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const int ng = nb < kArriveGroups ? nb : kArriveGroups;
  if (__hip_atomic_fetch_add(arrive, 1, kArriveOrder, kArriveScope) != ng - 1) return false;
  __hip_atomic_store(arrive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// the end of a pushing launch: this block's stores drained and published; the last
// block raises the flags
__device__ __forceinline__ void push_done(const Peers& P, const XSig& s) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x != 0) return;
  if (!arrive_last(s.arrive)) return;
  const int32_t v = s.cnt[0] + 1;
  for (int q = 0; q < s.G; ++q)
    if (q != s.me)
      __hip_atomic_store(flag_at(P.base[q], s.flag_off, s.set, s.me), v, kFlagOrder,
                         __HIP_MEMORY_SCOPE_SYSTEM);
}

// The step form of a hand-off (the row-sharded step's two launches, bpr_xchg_kernel and
// adam_xchg_kernel): every block first waits for the exchange set it consumes (its
// flags from every peer at the set's counter + 1); the last block to finish advances
// that counter and raises the flags of the set it produces (none: raise_cnt null).
struct XStep {
  int32_t* arrive;                      // arrival counters (kArriveInts, zero between)
  int32_t* wait_cnt;                    // counter of the consumed set (null: no wait)
  const int32_t* raise_cnt;             // counter of the produced set (null: no flags)
  int32_t* status;                      // -5 when a wait gave up
  int64_t flag_off, max_polls;
  int32_t wait_set, raise_set, G, me;
};

// All threads of the block: the flags of the consumed set from every peer, then a
// system-scope acquire (the peers' rows in this window are visible to the block).
__device__ __forceinline__ void xstep_wait(char* win, const XStep& x) {
  if (!x.wait_cnt) return;
  if (threadIdx.x < 64) {
    const int32_t target = x.wait_cnt[0] + 1;
    bool ok = true;
    for (int q = threadIdx.x; q < x.G; q += 64) {
      if (q == x.me) continue;
      const int32_t* f = flag_at(win, x.flag_off, x.wait_set, q);
      int64_t n = 0;
      while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < target) {
        if (++n > x.max_polls) {
          ok = false;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    if (!ok) __hip_atomic_store(x.status, -5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef MIREC_COMM_FORMAL_FENCES
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
#endif
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// The end of a step launch: this block's stores drained; the last block advances the
// consumed set's counter and raises the produced set's flags in every peer's window.
__device__ __forceinline__ void xstep_end(const Peers& P, const XStep& x) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x != 0) return;
  if (!arrive_last(x.arrive)) return;
  if (x.wait_cnt) x.wait_cnt[0] = x.wait_cnt[0] + 1;
  if (!x.raise_cnt) return;
  const int32_t v = x.raise_cnt[0] + 1;
  for (int q = 0; q < x.G; ++q)
    if (q != x.me)
      __hip_atomic_store(flag_at(P.base[q], x.flag_off, x.raise_set, x.me), v, kFlagOrder,
                         __HIP_MEMORY_SCOPE_SYSTEM);
}

// Wait for flag[set][src] >= cnt + 1 of every src != me, then cnt += 1 (advance; without
// it the wait only makes sure the flags are there: the pre-wait of a step launch, whose
// own blocks wait again at once and advance the counter). One block; a bounded spin
// (status -5 and an early exit instead of a hang).
__global__ __launch_bounds__(64) void xchg_wait_kernel(char* win, int64_t flag_off, int set,
                                                       int G, int me, int32_t* cnt,
                                                       int32_t* status, int64_t max_polls,
                                                       int advance) {
  const int32_t target = cnt[0] + 1;
  bool ok = true;
  for (int q = threadIdx.x; q < G; q += 64) {
    if (q == me) continue;
    const int32_t* f = flag_at(win, flag_off, set, q);
    int64_t n = 0;
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < target) {
      if (++n > max_polls) {
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
  }
  if (!ok) __hip_atomic_store(status, -5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  __syncthreads();
  if (threadIdx.x == 0 && advance) cnt[0] = target;
}

// One lane: flag[set][me] = cnt[set] + 1 in every peer's window (system-scope release
// after this stream's earlier work): a barrier's arrival, waited for by xchg_wait_kernel.
__global__ __launch_bounds__(64) void xchg_raise_kernel(Peers P, int64_t flag_off, int set, int G,
                                                        int me, const int32_t* cnt) {
  if (threadIdx.x != 0) return;
  const int32_t v = cnt[0] + 1;
  for (int q = 0; q < G; ++q)
    if (q != me)
      __hip_atomic_store(flag_at(P.base[q], flag_off, set, me), v, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_SYSTEM);
}

// The owner's forward message rows into the readers' windows: entry q = g * cap + j
// of idx (the exchange plan, mirec_shard_plan fwd_rows: >= 0 a user-shard row, < 0 an
// item-shard row -id - 1) goes to rank g's window, block `me`, row j. D/4 lanes per row.
template <int D>
__global__ __launch_bounds__(kXThreads) void xchg_push_rows_kernel(
    const float* __restrict__ U, const float* __restrict__ I, const int64_t* __restrict__ idx,
    int64_t cap, int64_t region_off, Peers P, XSig s) {
  constexpr int LPR = D / 4;
  const int64_t q = ((int64_t)blockIdx.x * kXThreads + threadIdx.x) / LPR;
  const int c = threadIdx.x % LPR;
  const int64_t n = (int64_t)s.G * cap;
  if (q < n) {
    const int g = (int)(q / cap);
    const int64_t j = q - (int64_t)g * cap;
    const int64_t r = idx[q];
    const float4 v = reinterpret_cast<const float4*>(r >= 0 ? U + r * D : I + (-r - 1) * D)[c];
    float* dst = reinterpret_cast<float*>(P.base[g] + region_off) + ((int64_t)s.me * cap + j) * D;
    reinterpret_cast<float4*>(dst)[c] = v;
  }
  push_done(P, s);
}

// Rows of this rank's send buffer [G x wcap x D] (block g for rank g, its first counts[g]
// rows; counts NULL: all) into the readers' windows (block `me` of the forward region),
// and each count into the reader's count slot `me` (published by the same flag).
template <int D>
__global__ __launch_bounds__(kXThreads) void xchg_push_blocks_kernel(
    const float* __restrict__ send, const int64_t* __restrict__ counts, int64_t wcap,
    int64_t count_off, Peers P, XSig s) {
  constexpr int LPR = D / 4;
  const int64_t q = ((int64_t)blockIdx.x * kXThreads + threadIdx.x) / LPR;
  const int c = threadIdx.x % LPR;
  if (blockIdx.x == 0 && threadIdx.x < (unsigned)s.G) {
    const int g = threadIdx.x;
    const int64_t n = counts ? counts[g] : wcap;
    reinterpret_cast<int64_t*>(P.base[g] + count_off)[s.me] = n < 0 ? 0 : (n > wcap ? wcap : n);
  }
  if (q < (int64_t)s.G * wcap) {
    const int g = (int)(q / wcap);
    const int64_t j = q - (int64_t)g * wcap;
    if (!counts || j < counts[g]) {
      const float4 v = reinterpret_cast<const float4*>(send + q * D)[c];
      float* dst = reinterpret_cast<float*>(P.base[g]) + ((int64_t)s.me * wcap + j) * D;
      reinterpret_cast<float4*>(dst)[c] = v;
    }
  }
  push_done(P, s);
}

// After the wait: every source's block of the forward region (its first count rows) into
// the caller's recv [G x wcap x D] at the same place; the counts into recv_counts.
template <int D>
__global__ __launch_bounds__(kXThreads) void xchg_copy_out_kernel(
    const char* __restrict__ win, int64_t wcap, int64_t count_off, int G, float* __restrict__ recv,
    int64_t* __restrict__ recv_counts) {
  constexpr int LPR = D / 4;
  const int64_t q = ((int64_t)blockIdx.x * kXThreads + threadIdx.x) / LPR;
  const int c = threadIdx.x % LPR;
  const int64_t* cnt = reinterpret_cast<const int64_t*>(win + count_off);
  if (recv_counts && blockIdx.x == 0 && threadIdx.x < (unsigned)G) recv_counts[threadIdx.x] = cnt[threadIdx.x];
  if (q >= (int64_t)G * wcap) return;
  const int g = (int)(q / wcap);
  const int64_t j = q - (int64_t)g * wcap;
  if (j < cnt[g])
    reinterpret_cast<float4*>(recv + q * D)[c] =
        reinterpret_cast<const float4*>(reinterpret_cast<const float*>(win) + q * D)[c];
}

// K3 of this rank's slice on the received rows, its gradient rows straight into the
// owners' windows. The BPR arithmetic is K3's (bpr_math.h, bpr.hip AT_IDS): a slot's
// row sits at message position pos = o * cap + j of the forward region (owner o's
// message), and its gradient row goes to owner o's backward region at me * cap + j —
// the position the owner's plan (shard.hip: perm2 = g * cap + j) reads it from. The
// last block raises the backward flags.
template <int D>
__global__ __launch_bounds__(kXThreads) void bpr_xchg_kernel(
    const char* __restrict__ win, int64_t fwd_off, int64_t bwd_off, const int64_t* __restrict__ user,
    const int64_t* __restrict__ pos, const int64_t* __restrict__ neg, int64_t B, int times,
    float gamma, float grad_scale, float* __restrict__ loss_k, int64_t cap, Peers P, XStep s) {
  constexpr int LPR = D / 4;
  constexpr int GPW = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const int g = lane / LPR;
  const int l = lane - g * LPR;
  const int64_t k = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * GPW + g;
  xstep_wait(const_cast<char*>(win), s);        // the owners' rows of this step are here
  const float* __restrict__ E = reinterpret_cast<const float*>(win + fwd_off);
  auto row_of = [&](int64_t p) -> int64_t { return p; };
  auto out_of = [&](int64_t p) -> float* {    // message position -> the owner's window row
    const int64_t o = p / cap;
    return reinterpret_cast<float*>(P.base[o] + bwd_off) + ((int64_t)s.me * cap + (p - o * cap)) * D;
  };
  if (k < B) {
    const int64_t pu = user[k], pp = pos[k];
    const float4 u = reinterpret_cast<const float4*>(E + row_of(pu) * D)[l];
    const float4 p = reinterpret_cast<const float4*>(E + row_of(pp) * D)[l];
    const float sp = group_sum<LPR>(dot4(u, p));
    float4 gu = make_float4(0.f, 0.f, 0.f, 0.f), gp = gu;
    float lsum = 0.f;
    const float ng = -grad_scale;
    for (int j0 = 0; j0 < times; j0 += 4) {
      float4 n[4];
      int64_t pn[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = j0 + q;
        pn[q] = j < times ? neg[(int64_t)j * B + k] : 0;
        n[q] = j < times ? reinterpret_cast<const float4*>(E + row_of(pn[q]) * D)[l]
                         : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      float sn[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) sn[q] = group_sum<LPR>(dot4(u, n[q]));
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (j0 + q < times) {
          const BprCoef cf = bpr_coef(sp, sn[q], gamma, ng);
          lsum += cf.nll;
          float4 gn;
          pair_contrib(gu, gp, gn, cf.dx, u, p, n[q]);
          reinterpret_cast<float4*>(out_of(pn[q]))[l] = gn;
        }
      }
    }
    reinterpret_cast<float4*>(out_of(pu))[l] = gu;
    reinterpret_cast<float4*>(out_of(pp))[l] = gp;
    if (l == 0 && loss_k) loss_k[k] = lsum;
  }
  xstep_end(P, s);
}

// The same n floats (n4 float4) of this rank into block `me` (stride floats apart) of
// every rank's region: the all-reduce's contribution.
__global__ __launch_bounds__(kXThreads) void xchg_push_bcast_kernel(
    const float* __restrict__ buf, int64_t n4, int64_t stride, int64_t region_off, Peers P,
    XSig s) {
  const int64_t q = (int64_t)blockIdx.x * kXThreads + threadIdx.x;
  if (q < (int64_t)s.G * n4) {
    const int g = (int)(q / n4);
    const int64_t i = q - (int64_t)g * n4;
    float* dst = reinterpret_cast<float*>(P.base[g] + region_off) + (int64_t)s.me * stride;
    reinterpret_cast<float4*>(dst)[i] = reinterpret_cast<const float4*>(buf)[i];
  }
  push_done(P, s);
}

// buf <- the sum over ranks (in rank order: the same bits on every rank) of every
// rank's n floats in region rows [src * wcap * d ...) of the window (after the wait)
__global__ __launch_bounds__(kXThreads) void xchg_sum_kernel(const char* __restrict__ win,
                                                             int64_t region_off, int64_t stride,
                                                             int G, int64_t n,
                                                             float* __restrict__ buf) {
  const int64_t i = (int64_t)blockIdx.x * kXThreads + threadIdx.x;
  if (i >= n) return;
  const float* r = reinterpret_cast<const float*>(win + region_off);
  float t = r[i];
  for (int q = 1; q < G; ++q) t += r[(int64_t)q * stride + i];
  buf[i] = t;
}

// Where the rows of the next step go (the owner's fold of the next forward exchange
// into this step's optimizer launch): entry u of segment si (2q touched, 2q+1 look-ahead
// of table q) is entry next[si][u] (-1: none) of the next step's owned list of table q,
// whose slots' message positions are dst[q][seg[q][j] .. seg[q][j+1]) (g * cap + idx:
// reader g's forward region, block me, row idx). next[si] null: no push.
struct XNext {
  const int32_t* next[2 * kMaxTables];
  const int32_t* seg[kMaxTables];
  const int32_t* dst[kMaxTables];
  int64_t cap;
};

// The owner's deferred Adam of a row-sharded step (adam_core.h deferred_row: the same
// rows, the same arithmetic, the same bits as mirec_adam_deferred_f32) with both
// exchanges folded in: every block waits for the backward flags (the readers' gradient
// rows in this window), and every row the NEXT step reads — each is in this launch's
// touched or look-ahead list, current through st+1 once its entry is done — is stored
// from registers into each reader's forward region at its message positions; the last
// block raises the forward flags. The blocks map onto the segments as in
// adam_deferred_kernel (the host's block_start: each segment's rows on blocks of their
// own, sized by the host's bound; blocks past a segment's count do no row work but
// still arrive). A grid-stride form, where the first blocks walked all four segments
// one after the other, took 6 µs more per launch (profiles/r06_ipc_adam_probe.txt).
template <int D, typename V>
__global__ __launch_bounds__(kAdamThreads) void adam_xchg_kernel(
    const AdamTables tabs, const float* __restrict__ consts, const int32_t* __restrict__ step_base,
    int step_off, AdamConsts k, XNext nx, char* win, Peers P, XStep xs) {
  constexpr int VPR = D / Lanes<V>::n;
  constexpr int RPB = (VPR >= kAdamThreads ? VPR : kAdamThreads) / VPR;
  const int si = segment_of(tabs, blockIdx.x);
  const mirec_adam_table& T = tabs.t[si >> 1];
  const bool ahead = si & 1;
  const int base = (int)(((int64_t)blockIdx.x - tabs.block_start[si]) * RPB);
  const int n = (ahead && !T.ahead_uniq) ? 0 : ahead ? T.ahead_n_uniq[0] : T.n_uniq[0];
  const int32_t* __restrict__ nxt = nx.next[si];
  const int32_t* __restrict__ sg = nx.seg[si >> 1];
  const int32_t* __restrict__ ds = nx.dst[si >> 1];
  const int u = base + threadIdx.x / VPR;
  const int c = threadIdx.x % VPR;
  int e0 = 0, e1 = 0;                      // the next step's slots of this row (issued early)
  if (nxt && u < n) {
    const int j = nxt[u];
    if (j >= 0) {
      e0 = sg[j];
      e1 = sg[j + 1];
    }
  }
  if (base < n) {                          // block-uniform; idle blocks only arrive
    xstep_wait(win, xs);
    deferred_row<D, V>(T, ahead, u, n, step_base[0] + step_off, consts, k, c,
                       [&](bool valid, bool loaded, int64_t row, V p) {
      if (!valid || e0 >= e1) return;
      if (!loaded) p = reinterpret_cast<const V*>(T.p)[row * VPR + c];   // zero-state row
      for (int e = e0; e < e1; ++e) {
        const int32_t q = ds[e];
        const int g = (int)(q / nx.cap);
        const int64_t idx = q - (int64_t)g * nx.cap;
        float* dst = reinterpret_cast<float*>(P.base[g]) + ((int64_t)xs.me * nx.cap + idx) * D;
        reinterpret_cast<V*>(dst)[c] = p;
      }
    });
  }
  xstep_end(P, xs);
}

}  // namespace mirec

using namespace mirec;

struct mirec_comm {
  int rank, world;
  char* window;
  size_t window_bytes;
  int64_t wcap;                         // rows per source block of a row region
  int32_t d;
  char* peers[kMaxPeers];
  bool opened[kMaxPeers];
  int32_t* ctl;                         // device: [unused | cnt[kFlagSets] | status]
  int32_t* arrive;                      // device: the launches' arrival counters
  int prewait;                          // MIREC_COMM_PREWAIT (mirec_comm_config)
};

namespace {
int64_t region_bytes(const mirec_comm* c) { return (int64_t)c->world * c->wcap * c->d * 4; }
int64_t flag_off(const mirec_comm* c) { return 2 * region_bytes(c); }
// the alltoallv row counts: kMaxPeers int64 after the flags
int64_t count_off(const mirec_comm* c) {
  return flag_off(c) + kFlagSets * kMaxPeers * (int64_t)sizeof(int32_t);
}
Peers peers_of(const mirec_comm* c) {
  Peers P;
  memset(&P, 0, sizeof(P));
  for (int q = 0; q < c->world; ++q) P.base[q] = c->peers[q];
  return P;
}
XSig sig_of(const mirec_comm* c, int set) {
  XSig s;
  s.arrive = c->arrive;
  s.cnt = c->ctl + 1 + set;
  s.flag_off = flag_off(c);
  s.set = set;
  s.G = c->world;
  s.me = c->rank;
  return s;
}
// A step launch that consumes set `wait` (-1: none) and produces set `raise` (-1: none).
XStep xstep_of(const mirec_comm* c, int wait, int raise, int64_t max_polls) {
  XStep x;
  x.arrive = c->arrive;
  x.wait_cnt = wait >= 0 ? c->ctl + 1 + wait : nullptr;
  x.raise_cnt = raise >= 0 ? c->ctl + 1 + raise : nullptr;
  x.status = c->ctl + 1 + kFlagSets;
  x.flag_off = flag_off(c);
  x.max_polls = max_polls;
  x.wait_set = wait;
  x.raise_set = raise;
  x.G = c->world;
  x.me = c->rank;
  return x;
}
bool connected(const mirec_comm* c) {
  for (int q = 0; q < c->world; ++q)
    if (!c->peers[q]) return false;
  return true;
}
}  // namespace

// unique_id: the job's 64-byte token (every rank passes the same one; the windows of
// different jobs never meet: their handles come only through the caller's exchange).
extern "C" int mirec_comm_init(int rank, int world, const void* unique_id, mirec_comm** out) {
  if (!out || !unique_id || world < 1 || world > kMaxPeers || rank < 0 || rank >= world) {
    set_error("mirec_comm_init: bad arguments (world 1..%d)", kMaxPeers);
    return -1;
  }
  mirec_comm* c = new mirec_comm;
  memset(c, 0, sizeof(*c));
  c->rank = rank;
  c->world = world;
  hipError_t e = hipMalloc(&c->ctl, (2 + kFlagSets) * sizeof(int32_t));
  if (e == hipSuccess) e = hipMemset(c->ctl, 0, (2 + kFlagSets) * sizeof(int32_t));
  if (e == hipSuccess) e = hipMalloc(&c->arrive, kArriveInts * sizeof(int32_t));
  if (e == hipSuccess) e = hipMemset(c->arrive, 0, kArriveInts * sizeof(int32_t));
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    if (c->ctl) (void)hipFree(c->ctl);
    if (c->arrive) (void)hipFree(c->arrive);
    delete c;
    return hip_status(e, "mirec_comm_init");
  }
  *out = c;
  return 0;
}

// This rank's window for rows of d floats, wcap rows per source block; its IPC handle
// (HIP_IPC_HANDLE_SIZE bytes) goes to handle_out for the caller to share.
extern "C" int mirec_comm_window(mirec_comm* c, int64_t wcap, int32_t d, void** local,
                                 void* handle_out) {
  if (!c || wcap < 1 || d < 4 || d % 4 || !handle_out || c->window) {
    set_error("mirec_comm_window: bad arguments (one window per communicator)");
    return -1;
  }
  c->wcap = wcap;
  c->d = d;
  c->window_bytes = (size_t)count_off(c) + kMaxPeers * sizeof(int64_t);
  hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void**>(&c->window), c->window_bytes,
                                       hipDeviceMallocUncached);
  if (e == hipSuccess) e = hipMemset(c->window, 0, c->window_bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  hipIpcMemHandle_t h;
  if (e == hipSuccess) e = hipIpcGetMemHandle(&h, c->window);
  if (e != hipSuccess) return hip_status(e, "mirec_comm_window");
  memcpy(handle_out, &h, sizeof(h));
  c->peers[c->rank] = c->window;
  if (local) *local = c->window;
  return 0;
}

extern "C" int64_t mirec_comm_handle_bytes(void) { return (int64_t)sizeof(hipIpcMemHandle_t); }

// Map every other rank's window (handles: world x mirec_comm_handle_bytes(), rank order).
extern "C" int mirec_comm_connect(mirec_comm* c, const void* handles) {
  if (!c || !handles || !c->window) {
    set_error("mirec_comm_connect: bad arguments (window first)");
    return -1;
  }
  for (int q = 0; q < c->world; ++q) {
    if (q == c->rank || c->peers[q]) continue;
    hipIpcMemHandle_t h;
    memcpy(&h, static_cast<const char*>(handles) + (size_t)q * sizeof(h), sizeof(h));
    void* p = nullptr;
    const hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return hip_status(e, "mirec_comm_connect");
    c->peers[q] = static_cast<char*>(p);
    c->opened[q] = true;
  }
  return 0;
}

// Byte offsets of the forward / backward row regions and the device status word (-5:
// a wait timed out; never reset by the library).
extern "C" int mirec_comm_layout(const mirec_comm* c, int64_t* fwd_off, int64_t* bwd_off,
                                 int32_t** status_dev) {
  if (!c || !c->window) {
    set_error("mirec_comm_layout: no window");
    return -1;
  }
  if (fwd_off) *fwd_off = 0;
  if (bwd_off) *bwd_off = region_bytes(c);
  if (status_dev) *status_dev = c->ctl + 1 + kFlagSets;
  return 0;
}

// The status word to the host (synchronous: after the device's work), then cleared: 0,
// or -5 when a wait gave up on a peer since the last read.
extern "C" int mirec_comm_status(mirec_comm* c, int32_t* out) {
  if (!c || !out) {
    set_error("mirec_comm_status: bad arguments");
    return -1;
  }
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess)
    e = hipMemcpy(out, c->ctl + 1 + kFlagSets, sizeof(int32_t), hipMemcpyDeviceToHost);
  if (e == hipSuccess && *out != 0) e = hipMemset(c->ctl + 1 + kFlagSets, 0, sizeof(int32_t));
  if (e == hipSuccess) e = hipDeviceSynchronize();
  return e == hipSuccess ? 0 : hip_status(e, "mirec_comm_status");
}

// flags: MIREC_COMM_PREWAIT (1) — each step launch (mirec_comm_bpr_f32,
// mirec_comm_adam_deferred_f32) is preceded by a one-block wait for its flags, so its
// own blocks never spin while a rank sharing this device needs the compute units to
// raise them (ranks on one GPU; on a node of one rank per GPU the in-kernel waits alone
// save the launch).
extern "C" int mirec_comm_config(mirec_comm* c, int32_t flags) {
  if (!c || (flags & ~1)) {
    set_error("mirec_comm_config: bad arguments");
    return -1;
  }
  c->prewait = flags & 1;
  return 0;
}

extern "C" int mirec_comm_destroy(mirec_comm* c) {
  if (!c) return 0;
  (void)hipDeviceSynchronize();
  for (int q = 0; q < c->world; ++q)
    if (c->opened[q]) (void)hipIpcCloseMemHandle(c->peers[q]);
  if (c->window) (void)hipFree(c->window);
  if (c->ctl) (void)hipFree(c->ctl);
  if (c->arrive) (void)hipFree(c->arrive);
  delete c;
  return 0;
}

namespace {
constexpr int64_t kMaxPolls = 1ll << 24;   // seconds of polling: a lost peer ends as status -5

int wait_set(mirec_comm* c, int set, hipStream_t st, const char* what, int advance = 1) {
  hipLaunchKernelGGL(xchg_wait_kernel, dim3(1), dim3(64), 0, st, c->window, flag_off(c), set,
                     c->world, c->rank, c->ctl + 1 + set, c->ctl + 1 + kFlagSets, kMaxPolls,
                     advance);
  return launch_status(what);
}

// Every rank's stream has reached this point (its earlier launches, which read its own
// window, are done) before any rank's stream goes on: the generic calls' entry and exit.
int barrier(mirec_comm* c, hipStream_t st, const char* what) {
  hipLaunchKernelGGL(xchg_raise_kernel, dim3(1), dim3(64), 0, st, peers_of(c), flag_off(c),
                     kBarrierSet, c->world, c->rank, (const int32_t*)(c->ctl + 1 + kBarrierSet));
  const int rc = launch_status(what);
  return rc ? rc : wait_set(c, kBarrierSet, st, what);
}
}  // namespace

// The exchange's wait, alone (set 0 forward rows, 1 backward rows).
extern "C" int mirec_comm_wait(mirec_comm* c, int32_t set, void* stream) {
  if (!c || !c->window || !connected(c) || set < 0 || set >= kFlagSets) {
    set_error("mirec_comm_wait: bad arguments");
    return -1;
  }
  return wait_set(c, set, (hipStream_t)stream, "mirec_comm_wait");
}

#define MIREC_XD(DD, ...)                     \
  switch (DD) {                               \
    case 32: { constexpr int D = 32; __VA_ARGS__; break; }   \
    case 64: { constexpr int D = 64; __VA_ARGS__; break; }   \
    case 128: { constexpr int D = 128; __VA_ARGS__; break; } \
    case 256: { constexpr int D = 256; __VA_ARGS__; break; } \
    default: set_error("d must be 32, 64, 128 or 256"); return -1; \
  }

// Forward rows of the row-sharded step (shard.hip plan): owner -> readers' windows.
extern "C" int mirec_comm_push_rows_f32(mirec_comm* c, const float* U, const float* I,
                                        const int64_t* idx, int64_t cap, void* stream) {
  if (!c || !c->window || !connected(c) || !U || !I || !idx || cap < 1 || cap > c->wcap) {
    set_error("mirec_comm_push_rows_f32: bad arguments (cap <= the window's)");
    return -1;
  }
  const int64_t n = (int64_t)c->world * cap;
  const unsigned blocks = (unsigned)((n * (c->d / 4) + kXThreads - 1) / kXThreads);
  hipStream_t st = (hipStream_t)stream;
  const Peers P = peers_of(c);
  const XSig s = sig_of(c, 0);
  MIREC_XD(c->d, hipLaunchKernelGGL(xchg_push_rows_kernel<D>, dim3(blocks), dim3(kXThreads), 0,
                                    st, U, I, idx, cap, (int64_t)0, P, s));
  return launch_status("mirec_comm_push_rows_f32");
}

// K3 on the received rows (its blocks wait for the forward flags); gradient rows to the
// owners, backward flags raised by its last block.
extern "C" int mirec_comm_bpr_f32(mirec_comm* c, const int64_t* user, const int64_t* pos,
                                  const int64_t* neg, int64_t B, int32_t times, float gamma,
                                  float grad_scale, float* loss_k, int64_t cap, void* stream) {
  if (!c || !c->window || !connected(c) || B < 0 || times < 0 || cap < 1 || cap > c->wcap ||
      (B > 0 && (!user || !pos || (times > 0 && !neg)))) {
    set_error("mirec_comm_bpr_f32: bad arguments");
    return -1;
  }
  const int64_t GPW = 64 / (c->d / 4);
  const unsigned blocks = (unsigned)std::max<int64_t>(1, (B + (kXThreads / 64) * GPW - 1) /
                                                            ((kXThreads / 64) * GPW));
  hipStream_t st = (hipStream_t)stream;
  const Peers P = peers_of(c);
  const XStep s = xstep_of(c, 0, 1, kMaxPolls);
  if (c->prewait) {
    const int rc = wait_set(c, 0, st, "mirec_comm_bpr_f32", 0);
    if (rc) return rc;
  }
  MIREC_XD(c->d, hipLaunchKernelGGL(bpr_xchg_kernel<D>, dim3(blocks), dim3(kXThreads), 0, st,
                                    (const char*)c->window, (int64_t)0, region_bytes(c), user,
                                    pos, neg, B, times, gamma, grad_scale, loss_k, cap, P, s));
  return launch_status("mirec_comm_bpr_f32");
}

// The owner's deferred Adam of a row-sharded step with both exchanges folded in
// (adam_xchg_kernel). tables: as mirec_adam_deferred_f32 (rows = this window's backward
// region); next / next_seg / next_dst: XNext (per segment / per table; next NULL: no
// push — the chunk's last step). n_max: host bounds of the lists (the grid).
extern "C" int mirec_comm_adam_deferred_f32(mirec_comm* c, const mirec_adam_table* tables,
                                            int32_t n_tables, const int64_t* n_max, int32_t d,
                                            const float* consts, const int32_t* step_base,
                                            int32_t step_off, double beta1, double beta2,
                                            double eps, double weight_decay,
                                            const int32_t* const* next,
                                            const int32_t* const* next_seg,
                                            const int32_t* const* next_dst, int64_t cap,
                                            void* stream) {
  if (!c || !c->window || !connected(c) || !tables || n_tables < 1 || n_tables > kMaxTables ||
      !n_max || !consts || !step_base || d != c->d || cap < 1 || cap > c->wcap ||
      ((uintptr_t)consts & 15) != 0) {
    set_error("mirec_comm_adam_deferred_f32: bad arguments");
    return -1;
  }
  AdamTables tabs;
  memset(&tabs, 0, sizeof(tabs));
  tabs.n_seg = 2 * n_tables;
  const int rpb = std::max(1, kAdamThreads / d);
  int64_t blocks = 0;
  XNext nx;
  memset(&nx, 0, sizeof(nx));
  nx.cap = cap;
  for (int q = 0; q < n_tables; ++q) {
    const mirec_adam_table& t = tables[q];
    if (!t.p || !t.m || !t.v || !t.last || !t.uniq || !t.seg || !t.perm || !t.rows ||
        !t.n_uniq || t.dense_grad || t.p_alt || n_max[q] < 0 ||
        (t.ahead_uniq == nullptr) != (t.ahead_n_uniq == nullptr)) {
      set_error("mirec_comm_adam_deferred_f32: bad table %d", q);
      return -1;
    }
    tabs.t[q] = t;
    const int64_t nb = (n_max[q] + rpb - 1) / rpb;     // segment 2q, then 2q + 1
    tabs.block_start[2 * q] = blocks;
    blocks += nb;
    tabs.block_start[2 * q + 1] = blocks;
    if (t.ahead_uniq) blocks += nb;
    if (next) {
      if (!next[2 * q] || (t.ahead_uniq && !next[2 * q + 1]) || !next_seg || !next_seg[q] ||
          !next_dst || !next_dst[q]) {
        set_error("mirec_comm_adam_deferred_f32: table %d: incomplete push lists", q);
        return -1;
      }
      nx.next[2 * q] = next[2 * q];
      nx.next[2 * q + 1] = next[2 * q + 1];
      nx.seg[q] = next_seg[q];
      nx.dst[q] = next_dst[q];
    }
  }
  AdamConsts k;
  k.omb1 = (float)(1.0 - beta1);
  k.omb1m1 = k.omb1 - 1.0f;
  k.lerp_small = fabsf(k.omb1) < 0.5f;
  k.b2 = (float)beta2;
  k.omb2 = (float)(1.0 - beta2);
  k.eps = (float)eps;
  k.wd = (float)weight_decay;
  for (int q = tabs.n_seg; q <= 2 * kMaxTables; ++q) tabs.block_start[q] = blocks;
  if (blocks == 0) blocks = 1;             // still one arrival: the flags are raised
  hipStream_t st = (hipStream_t)stream;
  const Peers P = peers_of(c);
  const XStep xs = xstep_of(c, 1, next ? 0 : -1, kMaxPolls);
  if (c->prewait) {
    const int rc = wait_set(c, 1, st, "mirec_comm_adam_deferred_f32", 0);
    if (rc) return rc;
  }
  // the forward region sits at offset 0 of every window (Peers point at window starts)
  MIREC_XD(d, hipLaunchKernelGGL((adam_xchg_kernel<D, float>), dim3((unsigned)blocks),
                                 dim3(kAdamThreads), 0, st, tabs, consts, step_base, step_off, k,
                                 nx, c->window, P, xs));
  return launch_status("mirec_comm_adam_deferred_f32");
}

// rows of send [world x wcap x d] (block g for rank g, its first
// send_counts[g] rows; counts on the device, NULL: all wcap) to every rank; afterwards
// recv [world x wcap x d] (the caller's buffer, not the window) holds block src at
// src * wcap — its first recv_counts[src] rows (device, written when non-NULL) — as
// rank src sent them. Stream-ordered: an entry barrier (every peer's earlier work on its
// window is done), the pushes (set 2), the wait, the copy out, an exit barrier (every
// peer has copied out before anyone's next exchange writes its window).
extern "C" int mirec_alltoallv_rows_f32(mirec_comm* c, const float* send,
                                        const int64_t* send_counts, float* recv,
                                        int64_t* recv_counts, int32_t d, void* stream) {
  if (!c || !c->window || !connected(c) || !send || !recv || d != c->d ||
      (reinterpret_cast<const char*>(recv) < c->window + c->window_bytes &&
       reinterpret_cast<const char*>(recv) + region_bytes(c) > c->window)) {
    set_error("mirec_alltoallv_rows_f32: bad arguments (recv: the caller's buffer, d = the window's)");
    return -1;
  }
  const int64_t n = (int64_t)c->world * c->wcap;
  const unsigned blocks = (unsigned)((n * (d / 4) + kXThreads - 1) / kXThreads);
  hipStream_t st = (hipStream_t)stream;
  const Peers P = peers_of(c);
  const XSig s = sig_of(c, 2);
  int rc = barrier(c, st, "mirec_alltoallv_rows_f32");
  if (rc) return rc;
  MIREC_XD(d, hipLaunchKernelGGL(xchg_push_blocks_kernel<D>, dim3(blocks), dim3(kXThreads), 0, st,
                                 send, send_counts, c->wcap, count_off(c), P, s));
  rc = launch_status("mirec_alltoallv_rows_f32");
  if (!rc) rc = wait_set(c, 2, st, "mirec_alltoallv_rows_f32");
  if (rc) return rc;
  MIREC_XD(d, hipLaunchKernelGGL(xchg_copy_out_kernel<D>, dim3(blocks), dim3(kXThreads), 0, st,
                                 (const char*)c->window, c->wcap, count_off(c), c->world, recv,
                                 recv_counts));
  rc = launch_status("mirec_alltoallv_rows_f32");
  return rc ? rc : barrier(c, st, "mirec_alltoallv_rows_f32");
}

// buf[n] <- the sum over ranks of every rank's buf, added in rank order
// (bit-identical on every rank). n <= wcap x d, a multiple of 4, buf 16-B aligned. Entry
// barrier, every rank's buf into block `me` of every window's backward region (set 3),
// the wait, the sum, exit barrier.
extern "C" int mirec_allreduce_sum_f32(mirec_comm* c, float* buf, int64_t n, void* stream) {
  if (!c || !c->window || !connected(c) || !buf || n < 0 || n > c->wcap * c->d ||
      ((uintptr_t)buf % 16) != 0 || n % 4) {
    set_error("mirec_allreduce_sum_f32: bad arguments (n <= wcap * d, a multiple of 4)");
    return -1;
  }
  if (n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const Peers P = peers_of(c);
  const XSig s = sig_of(c, 3);
  const int64_t stride = c->wcap * c->d;
  const unsigned blocks = (unsigned)(((int64_t)c->world * (n / 4) + kXThreads - 1) / kXThreads);
  int rc = barrier(c, st, "mirec_allreduce_sum_f32");
  if (rc) return rc;
  hipLaunchKernelGGL(xchg_push_bcast_kernel, dim3(blocks), dim3(kXThreads), 0, st, buf, n / 4,
                     stride, region_bytes(c), P, s);
  rc = launch_status("mirec_allreduce_sum_f32");
  if (!rc) rc = wait_set(c, 3, st, "mirec_allreduce_sum_f32");
  if (rc) return rc;
  hipLaunchKernelGGL(xchg_sum_kernel, dim3((unsigned)((n + kXThreads - 1) / kXThreads)),
                     dim3(kXThreads), 0, st, (const char*)c->window, region_bytes(c), stride,
                     c->world, n, buf);
  rc = launch_status("mirec_allreduce_sum_f32");
  return rc ? rc : barrier(c, st, "mirec_allreduce_sum_f32");
}
