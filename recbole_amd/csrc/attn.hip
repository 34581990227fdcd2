// K9e — the attention core of SASRec's MultiHeadAttention (reference
// recbole/model/layers.py:338-407: scores = Q K^T / sqrt(dh) + attention_mask, softmax,
// attn_dropout, @ V) for the sequence lengths SASRec runs (L <= 64) and dh = 64, forward
// and backward, one workgroup per (sequence, head). torch ran it as its fused attention
// library kernels (aotriton attn_fwd / bwd_kernel_fuse: 130 + 471 us per layer at C3's
// 2,048 x 2 heads x 50 x 64, ~18 TFLOP/s on tiles sized for long sequences) plus a
// permute copy of the context; here a whole (sequence, head) problem fits one workgroup:
//
//   forward   the sequence's K and V rows in LDS; wave w owns query rows 16w..16w+15:
//             S = Q K^T on fp32 MFMA (16x16x4, the exact fp32 products), scale + the
//             additive mask, row softmax (max / exp / sum across the 16 lanes of a row),
//             dropout, P V on MFMA; the context goes straight to [B, L, H * dh] (no
//             permute copy) with each row's log-sum-exp and the dropout's keep bits.
//   backward  K, V, Q, dO in LDS; wave w recomputes its rows' P from the saved
//             log-sum-exp, forms dP = dO V^T, dS = P (dP' - rowsum(P dP')) (dP' = dP
//             through the dropout), then all waves take 16-row strips of
//             dQ = dS K / sqrt(dh), dK = dS^T Q / sqrt(dh), dV = P'^T dO.
//
// Dropout draws are counter-based: key = splitmix64(seed + c), c the forward's counter
// value; for a row i = 16w + 4lk + r with r even and a column j, one draw
// x = splitmix64(key ^ (((b H + h) 64 + i) 64 + j)) decides element (i, j) by its low 32
// bits and element (i + 1, j) by its high 32 bits (kept iff < thr);
// the keep bits are saved as the forward's ballot words (64 per (b, h): wave w, column
// tile c, row r -> word (w 4 + c) 4 + r, bit li + 16 lk for row 16w + 4lk + r, column
// 16c + li) and read back by the backward, which advances the device counter by one store
// (captured steps draw new masks every replay; a last-block ticket in the forward serialised
// 4,096 atomics on one word, ~11 us a launch).
#include "common.h"

namespace mirec {

typedef float floatx4 __attribute__((ext_vector_type(4)));

// exp / log / the softmax's division in their hardware forms (v_exp_f32, v_log_f32, one
// reciprocal per row: a few ulp, inside the path's 1e-4 tolerance; fwd 71 -> 66 us at C3's
// shapes); MIREC_ATTN_EXACTMATH builds the libm forms
#if !defined(MIREC_ATTN_EXACTMATH)
#define AT_EXP(x) __expf(x)
#define AT_LOG(x) __logf(x)
#define AT_RCP(x) __frcp_rn(x)
#define AT_DIV(x, y, ry) ((x) * (ry))
#else
#define AT_EXP(x) expf(x)
#define AT_LOG(x) logf(x)
#define AT_RCP(x) (x)
#define AT_DIV(x, y, ry) ((x) / (y))
#endif

constexpr int kAtL = 64;         // padded sequence length (one 64-row tile)
constexpr int kAtD = 64;         // head dimension
constexpr int kAtLd = 68;        // LDS row stride (floats)
constexpr int kAtThreads = 256;  // four waves: 16 query rows each
constexpr int kAtWords = 64;     // keep-bit words per (b, h)

struct AttnArgs {
  const float* q;       // [B, L, H*64] (the query / key / value Linear outputs)
  const float* k;
  const float* v;
  const float* mask;    // [B, L, L] additive
  const float* dout;    // backward: dL/d context [B, L, H*64]
  float* out;           // forward: context [B, L, H*64]
  float* dq;            // backward outputs [B, L, H*64]
  float* dk;
  float* dv;
  float* lse;           // [B*H, 64] log-sum-exp of each query row (forward writes)
  uint64_t* keep;       // [B*H, 64] keep-bit words, or nullptr (no dropout)
  int64_t B;
  int L, H;
  float scale;          // 1 / sqrt(dh)
  uint32_t keep_thr;    // keep iff draw < keep_thr
  float keep_scale;     // 1 / (1 - p)
  uint64_t seed;
  int64_t* counter;     // forward: read; backward: advanced (one store)
};

__device__ __forceinline__ uint64_t at_mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ floatx4 at_mfma(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Tiles of rows 0..63 of one head's [L, 64] slice (row stride ld floats; rows >= L zero):
// at_load issues every float4 load of NT tiles into registers, at_store writes them to LDS
// (a load -> store loop per float4 waited a full memory latency per iteration).
constexpr int kAtPer = kAtL * (kAtD / 4) / kAtThreads;   // float4 per thread per tile

template <int NT>
__device__ __forceinline__ void at_load(float4 (&x)[NT][kAtPer], const float* const (&src)[NT],
                                        int L, int ld) {
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int j = 0; j < kAtPer; ++j) {
      const int e = threadIdx.x + j * kAtThreads;
      const int r = e >> 4, c4 = (e & 15) * 4;
      x[t][j] = r < L ? *reinterpret_cast<const float4*>(src[t] + (int64_t)r * ld + c4)
                      : make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

__device__ __forceinline__ void at_store(float (*T)[kAtLd], const float4 (&x)[kAtPer]) {
#pragma unroll
  for (int j = 0; j < kAtPer; ++j) {
    const int e = threadIdx.x + j * kAtThreads;
    *reinterpret_cast<float4*>(&T[e >> 4][(e & 15) * 4]) = x[j];
  }
}

// A operand rows of this wave straight from global memory: lane (li, lk) holds
// row r0 + li, floats 16u + 4lk .. +3 for u = 0..3 (zero for rows >= L)
__device__ __forceinline__ void at_rows(float4 (&a)[4], const float* __restrict__ src, int r0,
                                        int L, int ld, int li, int lk) {
#pragma unroll
  for (int u = 0; u < 4; ++u)
    a[u] = r0 + li < L ? *reinterpret_cast<const float4*>(src + (int64_t)(r0 + li) * ld + 16 * u + 4 * lk)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
}

// acc[c] += A x B^T for the wave's 16 A rows (registers, at_rows layout) and B^T's column
// n = row 16c + n of Bt (LDS, k along the row): the S = Q K^T / dP = dO V^T form. Lane
// (li, lk) supplies A[row li][k] and B[k][col li] for k = 16u + 4lk + e.
// live: the column tiles c to form (bit c; wave-uniform). (Skipping the zero tiles of dP,
// dQ, dK, dV in the backward measured slower: 172 against 153 us at C3's shapes, the
// predicated form taking 180 registers against 138.)
__device__ __forceinline__ void at_abt(floatx4 (&acc)[4], const float4 (&a)[4],
                                       const float (*Bt)[kAtLd], int li, int lk,
                                       uint32_t live = 0xFu) {
#pragma unroll
  for (int u = 0; u < kAtD / 16; ++u) {
    float4 b[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) b[c] = *reinterpret_cast<const float4*>(&Bt[16 * c + li][16 * u + 4 * lk]);
    // the four accumulators interleaved: consecutive MFMAs are independent (one chain
    // would wait the 40-cycle dependent latency per MFMA); each still sums x, y, z, w in
    // order
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if ((live >> c) & 1u) acc[c] = at_mfma(a[u].x, b[c].x, acc[c]);
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if ((live >> c) & 1u) acc[c] = at_mfma(a[u].y, b[c].y, acc[c]);
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if ((live >> c) & 1u) acc[c] = at_mfma(a[u].z, b[c].z, acc[c]);
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if ((live >> c) & 1u) acc[c] = at_mfma(a[u].w, b[c].w, acc[c]);
  }
}

// acc[c] += A x B with A = 16 rows of a row-major LDS tile (k along the row: A[li][k]) and
// B = a row-major LDS tile indexed [k][16c + li] (the P V / dS K form), k over 0..63; live:
// the k slices u to add (bit u, wave-uniform: a slice whose A tile is all zero adds nothing).
__device__ __forceinline__ void at_ab(floatx4 (&acc)[4], const float (*A)[kAtLd],
                                      const float (*Bm)[kAtLd], int li, int lk,
                                      uint32_t live = 0xFu) {
#pragma unroll 2
  for (int u = 0; u < kAtL / 16; ++u) {
    if (!((live >> u) & 1u)) continue;
    const float4 a = *reinterpret_cast<const float4*>(&A[li][16 * u + 4 * lk]);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = 16 * u + 4 * lk + e;
      const float ae = e == 0 ? a.x : e == 1 ? a.y : e == 2 ? a.z : a.w;
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = at_mfma(ae, Bm[k][16 * c + li], acc[c]);
    }
  }
}

// acc[c] += A^T x B with A^T's row li = column j0 + li of a row-major LDS tile At ([k][j]),
// B = a row-major LDS tile [k][16c + li] (the dS^T Q / P'^T dO form), k over 0..63. Lane
// group lk takes k = 16u + 4lk + e (rows 4 apart: with the 68-float stride the 64 lanes
// of one read hit 64 different banks).
__device__ __forceinline__ void at_atb(floatx4 (&acc)[4], const float (*At)[kAtLd], int j0,
                                       const float (*Bm)[kAtLd], int li, int lk,
                                       uint32_t live = 0xFu) {
#pragma unroll 2
  for (int u = 0; u < kAtL / 16; ++u) {
    if (!((live >> u) & 1u)) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = 16 * u + 4 * lk + e;
      const float a = At[k][j0 + li];
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = at_mfma(a, Bm[k][16 * c + li], acc[c]);
    }
  }
}

// ------------------------------------------------------------------------------- forward
// LDS: K and V (34.8 KB: four workgroups per CU); Q rows come straight from global memory
// in the A-operand layout, and P' replaces K once every wave has its scores.
__global__ __launch_bounds__(kAtThreads) void attn_fwd_kernel(AttnArgs a) {
  __shared__ float Ks[kAtL][kAtLd];      // K, then each wave's P' rows
  __shared__ float Vs[kAtL][kAtLd];
  const int64_t bh = blockIdx.x;
  const int64_t b = bh / a.H;
  const int h = (int)(bh % a.H);
  const int L = a.L, ld = a.H * kAtD;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, lk = lane >> 4;
  const int64_t base = b * L * ld + h * kAtD;
  const bool drop = a.keep != nullptr;
  const uint64_t key = drop ? at_mix(a.seed + (uint64_t)a.counter[0]) : 0ull;
  {
    float4 kv[2][kAtPer];
    const float* const srcs[2] = {a.k + base, a.v + base};
    at_load<2>(kv, srcs, L, ld);
    at_store(Ks, kv[0]);
    at_store(Vs, kv[1]);
  }
  float4 qa[4];
  at_rows(qa, a.q + base, 16 * w, L, ld, li, lk);
  // the mask values of this lane's 16 scores
  float mk[4][4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * w + 4 * lk + r, col = 16 * c + li;
      mk[c][r] = (row < L && col < L) ? a.mask[(b * L + row) * L + col] : 0.f;
    }
  __syncthreads();

  floatx4 s[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) s[c] = floatx4{0.f, 0.f, 0.f, 0.f};
  at_abt(s, qa, Ks, li, lk);

  // scale + mask, row softmax (row 16w + 4lk + r lives in the 16 lanes of group lk)
  float p[4][4], mx[4], sum[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) mx[r] = -__builtin_inff();
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float x = (16 * c + li < L) ? s[c][r] * a.scale + mk[c][r] : -__builtin_inff();
      p[c][r] = x;
      mx[r] = fmaxf(mx[r], x);
    }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) mx[r] = fmaxf(mx[r], __shfl_xor(mx[r], o, 64));
    sum[r] = 0.f;
  }
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      p[c][r] = AT_EXP(p[c][r] - mx[r]);
      sum[r] += p[c][r];
    }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) sum[r] += __shfl_xor(sum[r], o, 64);
  uint64_t word = 0ull;
  float rsum[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) rsum[r] = AT_RCP(sum[r]);
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < 4; r += 2) {
      // one draw per two elements (rows r, r + 1 of column 16c + li): its halves
      uint64_t d = 0ull;
      if (drop) {
        const int row = 16 * w + 4 * lk + r, col = 16 * c + li;
        d = at_mix(key ^ (((uint64_t)bh * kAtL + row) * kAtL + col));
      }
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        float x = AT_DIV(p[c][r + h2], sum[r + h2], rsum[r + h2]);
        if (drop) {
          const bool kept = (uint32_t)(h2 ? d >> 32 : d) < a.keep_thr;
          const uint64_t bal = __ballot(kept);
          if (lane == c * 4 + r + h2) word = bal;
          x = kept ? x * a.keep_scale : 0.f;
        }
        p[c][r + h2] = x;
      }
    }
  if (drop && lane < 16) a.keep[bh * kAtWords + w * 16 + lane] = word;
  // column tiles of this wave's P' that are not all zero (a causal mask zeroes the tiles
  // past the diagonal exactly: exp underflows): O = P' V skips the others' k slices
  uint32_t live = 0;
#pragma unroll
  for (int c = 0; c < 4; ++c)
    live |= (__ballot(p[c][0] != 0.f || p[c][1] != 0.f || p[c][2] != 0.f || p[c][3] != 0.f) != 0ull
                 ? 1u : 0u) << c;
  if (li == 0)
#pragma unroll
    for (int r = 0; r < 4; ++r) a.lse[bh * kAtL + 16 * w + 4 * lk + r] = mx[r] + AT_LOG(sum[r]);
  __syncthreads();                         // every wave's K reads are done: Ks takes P'
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) Ks[16 * w + 4 * lk + r][16 * c + li] = p[c][r];
  __syncthreads();

  floatx4 o[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) o[c] = floatx4{0.f, 0.f, 0.f, 0.f};
  at_ab(o, &Ks[16 * w], Vs, li, lk, live);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = 16 * w + 4 * lk + r;
    if (row < L)
#pragma unroll
      for (int c = 0; c < 4; ++c) a.out[base + (int64_t)row * ld + 16 * c + li] = o[c][r];
  }
}

// ------------------------------------------------------------------------------ backward
// LDS: four tiles (69.6 KB: two workgroups per CU). Phase 1 (S, dP from the wave's Q / dO
// rows in registers against K, V); the Q and dO tiles wait in registers and take the LDS
// slots of V (after phase 1) and of K (after dQ, dK).
__global__ __launch_bounds__(kAtThreads) void attn_bwd_kernel(AttnArgs a) {
  __shared__ float Ks[kAtL][kAtLd];      // K, then dO
  __shared__ float Vs[kAtL][kAtLd];      // V, then Q
  __shared__ float Ds[kAtL][kAtLd];      // dS
  __shared__ float Ps[kAtL][kAtLd];      // P' (after the dropout)
  const int64_t bh = blockIdx.x;
  const int64_t b = bh / a.H;
  const int h = (int)(bh % a.H);
  const int L = a.L, ld = a.H * kAtD;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, lk = lane >> 4;
  const int64_t base = b * L * ld + h * kAtD;
  const bool drop = a.keep != nullptr;
  float4 later[2][kAtPer];                 // the Q and dO tiles for phase 2
  {
    float4 kv[2][kAtPer];
    const float* const srcs[2] = {a.k + base, a.v + base};
    at_load<2>(kv, srcs, L, ld);
    const float* const srcs2[2] = {a.q + base, a.dout + base};
    at_load<2>(later, srcs2, L, ld);
    at_store(Ks, kv[0]);
    at_store(Vs, kv[1]);
  }
  float4 qa[4], da[4];
  at_rows(qa, a.q + base, 16 * w, L, ld, li, lk);
  at_rows(da, a.dout + base, 16 * w, L, ld, li, lk);
  float mk[4][4], lse[4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * w + 4 * lk + r, col = 16 * c + li;
      mk[c][r] = (row < L && col < L) ? a.mask[(b * L + row) * L + col] : 0.f;
    }
#pragma unroll
  for (int r = 0; r < 4; ++r) lse[r] = a.lse[bh * kAtL + 16 * w + 4 * lk + r];
  const uint64_t word = (drop && lane < 16) ? a.keep[bh * kAtWords + w * 16 + lane] : 0ull;
  if (drop && a.counter && bh == 0 && tid == 0) a.counter[0] += 1;   // the next draw
  __syncthreads();

  floatx4 s[4], dp[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    s[c] = floatx4{0.f, 0.f, 0.f, 0.f};
    dp[c] = s[c];
  }
  at_abt(s, qa, Ks, li, lk);
  at_abt(dp, da, Vs, li, lk);
  float pr[4][4], rs[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) rs[r] = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * w + 4 * lk + r, col = 16 * c + li;
      const float pv = (row < L && col < L) ? AT_EXP(s[c][r] * a.scale + mk[c][r] - lse[r]) : 0.f;
      float g = dp[c][r];
      float pd = pv;
      if (drop) {
        const uint64_t wd = __shfl(word, c * 4 + r, 64);
        const bool kept = (wd >> (li + 16 * lk)) & 1ull;
        g = kept ? g * a.keep_scale : 0.f;
        pd = kept ? pv * a.keep_scale : 0.f;
      }
      pr[c][r] = pd;
      s[c][r] = pv;             // P
      dp[c][r] = g;             // dL/dP
      rs[r] += pv * g;
    }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) rs[r] += __shfl_xor(rs[r], o, 64);
  __syncthreads();                         // every wave's V reads are done: Vs takes Q
  at_store(Vs, later[0]);
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      Ps[16 * w + 4 * lk + r][16 * c + li] = pr[c][r];
      Ds[16 * w + 4 * lk + r][16 * c + li] = s[c][r] * (dp[c][r] - rs[r]);
    }
  __syncthreads();

  floatx4 acc[4];
  // dQ rows 16w.. = dS K * scale
#pragma unroll
  for (int c = 0; c < 4; ++c) acc[c] = floatx4{0.f, 0.f, 0.f, 0.f};
  at_ab(acc, &Ds[16 * w], Ks, li, lk);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = 16 * w + 4 * lk + r;
    if (row < L)
#pragma unroll
      for (int c = 0; c < 4; ++c) a.dq[base + (int64_t)row * ld + 16 * c + li] = acc[c][r] * a.scale;
  }
  // dK rows 16w.. = dS^T Q * scale
#pragma unroll
  for (int c = 0; c < 4; ++c) acc[c] = floatx4{0.f, 0.f, 0.f, 0.f};
  at_atb(acc, Ds, 16 * w, Vs, li, lk);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = 16 * w + 4 * lk + r;
    if (row < L)
#pragma unroll
      for (int c = 0; c < 4; ++c) a.dk[base + (int64_t)row * ld + 16 * c + li] = acc[c][r] * a.scale;
  }
  __syncthreads();                         // every wave's K reads are done: Ks takes dO
  at_store(Ks, later[1]);
  __syncthreads();
  // dV rows 16w.. = P'^T dO
#pragma unroll
  for (int c = 0; c < 4; ++c) acc[c] = floatx4{0.f, 0.f, 0.f, 0.f};
  at_atb(acc, Ps, 16 * w, Ks, li, lk);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = 16 * w + 4 * lk + r;
    if (row < L)
#pragma unroll
      for (int c = 0; c < 4; ++c) a.dv[base + (int64_t)row * ld + 16 * c + li] = acc[c][r];
  }
}

static int attn_check(const AttnArgs& a, const char* what) {
  if (a.B < 0 || a.L < 1 || a.L > kAtL || a.H < 1 || !a.q || !a.k || !a.v || !a.mask || !a.lse) {
    set_error("%s: bad arguments (B=%lld L=%d H=%d; L must be in [1, %d], dh = %d)", what,
              (long long)a.B, a.L, a.H, kAtL, kAtD);
    return -1;
  }
  if ((((uintptr_t)a.q | (uintptr_t)a.k | (uintptr_t)a.v) & 15) != 0) {
    set_error("%s: q, k, v must be 16-byte aligned", what);
    return -1;
  }
  return 0;
}

}  // namespace mirec

using namespace mirec;

extern "C" int mirec_attn_fwd_f32(const float* q, const float* k, const float* v,
                                  const float* mask, int64_t B, int32_t L, int32_t H,
                                  float dropout_p, uint64_t seed, int64_t* counter, float* out,
                                  float* lse, uint64_t* keep_words, void* stream) {
  AttnArgs a;
  memset(&a, 0, sizeof(a));
  a.q = q; a.k = k; a.v = v; a.mask = mask; a.out = out; a.lse = lse;
  a.B = B; a.L = L; a.H = H;
  a.scale = 1.0f / sqrtf((float)kAtD);
  if (attn_check(a, "mirec_attn_fwd_f32") || !out) {
    if (!out) set_error("mirec_attn_fwd_f32: out is NULL");
    return -1;
  }
  if (dropout_p > 0.f) {
    if (dropout_p >= 1.f || !counter || !keep_words) {
      set_error("mirec_attn_fwd_f32: dropout %g needs p < 1, a counter and keep words",
                (double)dropout_p);
      return -1;
    }
    a.keep = keep_words;
    a.keep_thr = (uint32_t)fmin(4294967295.0, ldexp(1.0 - (double)dropout_p, 32));
    a.keep_scale = 1.0f / (1.0f - dropout_p);
    a.seed = seed;
    a.counter = counter;
  }
  if (B == 0) return 0;
  hipLaunchKernelGGL(attn_fwd_kernel, dim3((unsigned)(B * H)), dim3(kAtThreads), 0,
                     (hipStream_t)stream, a);
  return launch_status("mirec_attn_fwd_f32");
}

extern "C" int mirec_attn_bwd_f32(const float* q, const float* k, const float* v,
                                  const float* mask, const float* dout, const float* lse,
                                  const uint64_t* keep_words, int64_t* counter, int64_t B,
                                  int32_t L, int32_t H, float dropout_p, float* dq, float* dk,
                                  float* dv, void* stream) {
  AttnArgs a;
  memset(&a, 0, sizeof(a));
  a.q = q; a.k = k; a.v = v; a.mask = mask; a.dout = dout; a.lse = const_cast<float*>(lse);
  a.dq = dq; a.dk = dk; a.dv = dv;
  a.B = B; a.L = L; a.H = H;
  a.scale = 1.0f / sqrtf((float)kAtD);
  if (attn_check(a, "mirec_attn_bwd_f32")) return -1;
  if (!dout || !dq || !dk || !dv || (((uintptr_t)dout & 15) != 0)) {
    set_error("mirec_attn_bwd_f32: dout / dq / dk / dv missing or dout not 16-byte aligned");
    return -1;
  }
  if (dropout_p > 0.f) {
    if (dropout_p >= 1.f || !keep_words) {
      set_error("mirec_attn_bwd_f32: dropout %g needs p < 1 and the forward's keep words",
                (double)dropout_p);
      return -1;
    }
    a.keep = const_cast<uint64_t*>(keep_words);
    a.keep_scale = 1.0f / (1.0f - dropout_p);
    a.counter = counter;          // may be NULL: the caller advances it
  }
  if (B == 0) return 0;
  hipLaunchKernelGGL(attn_bwd_kernel, dim3((unsigned)(B * H)), dim3(kAtThreads), 0,
                     (hipStream_t)stream, a);
  return launch_status("mirec_attn_bwd_f32");
}
