// K10  The deep part of DeepFM in three launches: MLPLayers (Dropout -> Linear -> ReLU
// per hidden layer, reference recbole/model/layers.py:30-86) followed by
// deep_predict_layer (Linear to one logit, deepfm.py:40-43,61). torch runs this as
// ~10 forward and ~17 backward launches (dropout, addmm, relu, threshold_backward,
// masked_scale, two GEMMs and a bias reduction per layer); here:
//
//   forward      one block per 16 rows runs every layer: its input tile (after the
//                dropout) in LDS, the layer's product on fp32 MFMA (16x16x4, exact
//                fp32 fma chains), bias + ReLU + the next layer's dropout in the
//                epilogue, the result back to LDS for the next layer. Saves each
//                layer's (dropped) input for the backward, and layer 0's mask.
//   data grad    one block per 16 rows walks the layers backwards: g_x = g_z W, then
//                g_z of the layer below = g_x * scale * [x > 0] (dropout backward and
//                ReLU backward in one test: x = h * mask * scale > 0 iff the element
//                was kept and h > 0); writes every g_z and the input gradient.
//   weight grad  one block per 16x16 tile of every dW (plus, for the tiles of the
//                first input column, the bias gradient): dW = g_z^T x over the batch,
//                the eight waves each take an eighth of the rows and their partial
//                tiles are added in wave order (fixed order, run to run identical).
// Every loop issues the next group's loads before the current group's MFMAs (the
// first version, one dependent load level per 16-wide slice, ran the forward at 83 µs).
//
// Dropout draws are counter-based (mirec_mlp_draw below; restated in numpy by
// tests/mlp_spec.py): element e of layer l in the forward with counter value c is
// kept iff  splitmix64(splitmix64(seed + c) ^ (e * 8 + l)) >> 32  <  keep_threshold.
// The counter lives on the device and the last block of each training forward
// advances it, so captured steps (HIP graph replays) draw new masks every step.
#include "common.h"

#include <cstdlib>

namespace mirec {

constexpr int kMlpRows = 16;       // rows per forward / data-grad block
constexpr int kMlpThreads = 512;   // eight waves
constexpr int kMlpWaves = kMlpThreads / 64;
constexpr int kMlpU = 4;           // 16-wide slices per prefetch group (data grad)
#ifndef MIREC_FWD_U
#define MIREC_FWD_U 8
#endif
constexpr int kFwdU = MIREC_FWD_U; // forward: 8 slices (32 MFMAs) per group

typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ bool mlp_keep(uint64_t key, int layer, uint64_t elem, uint32_t thr) {
  return (uint32_t)(splitmix64(key ^ (elem * 8ull + (uint64_t)layer)) >> 32) < thr;
}

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Row strides (floats) of the two LDS tiles: widths dims[j] of even j live in tile A,
// of odd j in tile B (a layer reads one and writes the other); layers from l0 on.
static void mlp_ld(const mirec_mlp& a, int* ldA, int* ldB, int l0 = 0) {
  int m[2] = {0, 0};
  for (int j = l0; j <= a.n_layers; ++j) m[j & 1] = a.dims[j] > m[j & 1] ? a.dims[j] : m[j & 1];
  *ldA = (m[0] + 15) / 16 * 16 + 4;
  *ldB = (m[1] + 15) / 16 * 16 + 4;
}

// -------------------------------------------------------------------------- forward
// One 16 x 16 output tile: rows of A [16, K] (LDS, row stride ld) times columns c0..c0+15
// of W [N, K] over the 16-wide K slices [s0, s1). k = 16 s + 16 u + 4 lk + e: the four
// MFMAs of a slice cover it once each; the next group's loads are issued before this
// group's MFMAs (two accumulators, added at the end).
template <int U = kFwdU>
__device__ __forceinline__ floatx4 tile_dot(const float* cur, int ld, const float* __restrict__ W,
                                            int K, int N, int c0, int s0, int s1, int li, int lk) {
  constexpr int kFwdU = U;          // slices per prefetch group (shadows the file default)
  const int c = c0 + li;
  const float* wr = W + (int64_t)(c < N ? c : N - 1) * K;
  const int kend = min(16 * s1, K);
  float4 pa[kFwdU], pb[kFwdU];
  // branch-free loads (addresses clamped into the row, out-of-range slices zeroed after
  // the load): straight-line code lets the compiler wait on the older group only
  // (vmcnt(N)) while the next group is in flight
  auto load = [&](int k0) {
#pragma unroll
    for (int u = 0; u < kFwdU; ++u) {
      const int k = k0 + 16 * u + 4 * lk;
      const int kc = k < K ? k : K - 4;
      pa[u] = *reinterpret_cast<const float4*>(cur + li * ld + kc);
      pb[u] = *reinterpret_cast<const float4*>(wr + kc);
      if (k >= kend) pb[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  floatx4 accA = {0.f, 0.f, 0.f, 0.f}, accB = {0.f, 0.f, 0.f, 0.f};
  if (s0 >= s1) return accA;
  load(16 * s0);
  for (int k0 = 16 * s0; k0 < kend; k0 += 16 * kFwdU) {
    float4 ca[kFwdU], cb[kFwdU];
#pragma unroll
    for (int u = 0; u < kFwdU; ++u) { ca[u] = pa[u]; cb[u] = pb[u]; }
    if (k0 + 16 * kFwdU < kend) load(k0 + 16 * kFwdU);
#pragma unroll
    for (int u = 0; u < kFwdU; ++u) {
      floatx4& acc = (u & 1) ? accB : accA;
      acc = mfma4(ca[u].x, cb[u].x, acc);
      acc = mfma4(ca[u].y, cb[u].y, acc);
      acc = mfma4(ca[u].z, cb[u].z, acc);
      acc = mfma4(ca[u].w, cb[u].w, acc);
    }
  }
  return accA + accB;
}

// Rows r0.. of layer l0's input into the LDS tile `t` (row stride ld): layer 0 reads x
// and applies its dropout (saving the dropped input and the keep flags), a later layer
// reads its saved input xs[l0] (already dropped). Every float4 is loaded before any is
// processed (stores to the saved buffers may alias x as far as the compiler knows,
// which would otherwise serialise one load per element). NT threads.
template <int NT>
__device__ __forceinline__ void stage_rows(const mirec_mlp& a, const float* __restrict__ x,
                                           int l0, int64_t B, int64_t r0, bool drop,
                                           bool save, uint64_t key, float* t, int ld) {
  const int tid = threadIdx.x;
  const int K = a.dims[l0];
  const float* src = l0 ? a.xs[l0] : x;
  constexpr int kV = kMlpRows * 1024 / 4 / NT;            // float4 per thread, K <= 1024
  const int nv = kMlpRows * K / 4;
  const int64_t lim = (B - r0) * K / 4;                   // float4 of valid rows
  const float4* x4 = reinterpret_cast<const float4*>(src + r0 * K);
  float4 xv[kV];
#pragma unroll
  for (int j = 0; j < kV; ++j) {
    const int q = tid + j * NT;
    xv[j] = (q < nv && q < lim) ? x4[q] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int j = 0; j < kV; ++j) {
    const int q = tid + j * NT;
    if (q >= nv) break;
    const int e0 = 4 * q, i = e0 / K, k = e0 - i * K;
    float4 v = xv[j];
    if (q < lim && l0 == 0) {
      const int64_t e = r0 * K + e0;
      if (drop) {
        const bool k0 = mlp_keep(key, 0, (uint64_t)e, a.keep_threshold);
        const bool k1 = mlp_keep(key, 0, (uint64_t)e + 1, a.keep_threshold);
        const bool k2 = mlp_keep(key, 0, (uint64_t)e + 2, a.keep_threshold);
        const bool k3 = mlp_keep(key, 0, (uint64_t)e + 3, a.keep_threshold);
        v.x = k0 ? v.x * a.scale : 0.f;
        v.y = k1 ? v.y * a.scale : 0.f;
        v.z = k2 ? v.z * a.scale : 0.f;
        v.w = k3 ? v.w * a.scale : 0.f;
        if (save)
          *reinterpret_cast<uint32_t*>(a.mask0 + e) =
              (k0 ? 1u : 0u) | (k1 ? 1u << 8 : 0u) | (k2 ? 1u << 16 : 0u) | (k3 ? 1u << 24 : 0u);
      }
      if (save && a.xs[0] && a.xs[0] != x) *reinterpret_cast<float4*>(a.xs[0] + e) = v;
    }
    *reinterpret_cast<float4*>(t + i * ld + k) = v;
  }
}

// Layers l0..L-1 for one block of 16 rows (l0 = 0: every layer; l0 = 1 behind the wide
// layer-0 kernel below). KS waves per 16-column output tile, each over 1/KS of the K
// slices, their partial tiles added in LDS in kh order: the forward is latency-bound (one
// block per 16 rows: 128 blocks on half the chip at C4, waves waiting on W's loads 43 % and
// on MFMA results 34 % of their time with KS = 1, profiles/r06_C4_mlp_pmc.txt), and KS = 2
// doubles the waves in flight and halves each wave's dependent chain.
#ifndef MIREC_MLP_FWD_KS
#define MIREC_MLP_FWD_KS 2
#endif
constexpr int kFwdKS = MIREC_MLP_FWD_KS;
template <int KS>
__global__ __launch_bounds__(kMlpThreads * KS) void mlp_fwd_kernel(mirec_mlp a, const float* __restrict__ x,
                                                              int64_t B, float* __restrict__ y,
                                                              int train, int ldA, int ldB, int l0) {
  extern __shared__ float lds[];
  float* const tA = lds;
  float* const tB = lds + kMlpRows * ldA;
  floatx4* const red = reinterpret_cast<floatx4*>(tB + kMlpRows * ldB);   // [KS-1][waves][64]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = (tid >> 6) % kMlpWaves, kh = (tid >> 6) / kMlpWaves;
  const int li = lane & 15, lk = lane >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * kMlpRows;
  const int L = a.n_layers;
  bool any_drop = false;
  for (int l = 0; l < L; ++l) any_drop |= train && a.dropout[l];
  const uint64_t key = any_drop ? splitmix64(a.seed + (uint64_t)a.counter[0]) : 0ull;

  stage_rows<kMlpThreads * KS>(a, x, l0, B, r0, train && a.dropout[0], true, key,
                               (l0 & 1) ? tB : tA, (l0 & 1) ? ldB : ldA);
  __syncthreads();

  for (int l = l0; l < L; ++l) {
    const int K = a.dims[l], N = a.dims[l + 1];
    const float* cur = (l & 1) ? tB : tA;
    float* nxt = (l & 1) ? tA : tB;
    const int ld = (l & 1) ? ldB : ldA, ldn = (l & 1) ? ldA : ldB;
    const float* __restrict__ bias = a.b[l];
    const bool last = l == L - 1;
    const bool drop_next = !last && train && a.dropout[l + 1];
    const bool relu = a.relu[l] != 0;
    float* __restrict__ save = last ? nullptr : a.xs[l + 1];
    const int ntile = (N + 15) / 16;
    const int nsl = (K + 15) / 16, spk = (nsl + KS - 1) / KS;
    for (int t0 = 0; t0 < ntile; t0 += kMlpWaves) {    // rounds: every wave at every barrier
      const int t = t0 + wave;                          // one 16-column tile per wave (group)
      const int c = t * 16 + li;
      floatx4 acc0 = {0.f, 0.f, 0.f, 0.f};
      if (t < ntile)
        acc0 = tile_dot<(kFwdU / KS > 1 ? kFwdU / KS : 1)>(cur, ld, a.W[l], K, N, t * 16, kh * spk,
                                                           min(nsl, (kh + 1) * spk), li, lk);
      if (KS > 1) {
        if (kh > 0) red[((kh - 1) * kMlpWaves + wave) * 64 + lane] = acc0;
        __syncthreads();
        if (kh == 0)
#pragma unroll
          for (int h = 1; h < KS; ++h) acc0 = acc0 + red[((h - 1) * kMlpWaves + wave) * 64 + lane];
      }
      // epilogue: lane holds rows 4*lk + r of column c
      if (kh == 0 && t < ntile && c < N) {
        const float bc = bias ? bias[c] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 4 * lk + r;
          const int64_t row = r0 + i;
          float z = acc0[r] + bc;
          if (relu) z = z < 0.f ? 0.f : z;           // NaN passes, as torch.relu
          if (last) {
            if (row < B) y[row * N + c] = z;
            continue;
          }
          if (drop_next && row < B) {
            const bool kp = mlp_keep(key, l + 1, (uint64_t)(row * N + c), a.keep_threshold);
            z = kp ? z * a.scale : 0.f;
          }
          if (row < B && save) save[row * N + c] = z;
          nxt[i * ldn + c] = z;
        }
      }
      if (KS > 1) __syncthreads();                      // red is rewritten next round
    }
    __syncthreads();
  }

  // the last block of a training forward with dropout advances the draw counter (every
  // block has read it above, before its first barrier)
  if (any_drop && tid == 0) {
    const int prev = atomicAdd(a.arrive, 1);
    if (prev == (int)gridDim.x - 1) {
      atomicExch(a.arrive, 0);
      atomicAdd(reinterpret_cast<unsigned long long*>(a.counter), 1ull);
    }
  }
}

// Wide layer 0 (dims[0] >= kWideMin, training / grad mode) over the whole chip: the
// fused kernel above runs it with one 16-row block per CU on half the chip, each block
// streaming all of W0 (C4: 128 blocks x 320 KB). Here a block of 4 waves takes 16 rows x
// 32 columns: the rows (after layer 0's dropout) staged once in LDS, waves (tile ct, K
// half kh) each form one 16 x 16 tile over half the K slices, the two halves added in
// LDS (kh 0 + kh 1), and the epilogue (bias, ReLU, layer 1's dropout) writes layer 1's
// saved input xs[1], which mlp_fwd_kernel(l0 = 1) then reads. Blocks of column group 0
// save layer 0's dropped input and keep flags. The draw counter is read, not advanced
// (the l0 = 1 launch advances it).
constexpr int kWideMin = 256;
constexpr int kWideThreads = 256;
constexpr int kL0Cols = 32;
__global__ __launch_bounds__(kWideThreads) void mlp_l0_fwd_kernel(mirec_mlp a,
                                                                  const float* __restrict__ x,
                                                                  int64_t B, int train, int ld) {
  extern __shared__ float lds[];
  float* const tA = lds;
  floatx4* const red = reinterpret_cast<floatx4*>(lds + kMlpRows * ld);   // [2 tiles][64]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int li = lane & 15, lk = lane >> 4;
  const int ct = wave & 1, kh = wave >> 1;
  const int64_t r0 = (int64_t)blockIdx.x * kMlpRows;
  const int K = a.dims[0], N = a.dims[1], L = a.n_layers;
  bool any_drop = false;
  for (int l = 0; l < L; ++l) any_drop |= train && a.dropout[l];
  const uint64_t key = any_drop ? splitmix64(a.seed + (uint64_t)a.counter[0]) : 0ull;
  stage_rows<kWideThreads>(a, x, 0, B, r0, train && a.dropout[0], blockIdx.y == 0, key, tA, ld);
  __syncthreads();
  const int nsl = (K + 15) / 16, half = (nsl + 1) / 2;
  const int c0 = blockIdx.y * kL0Cols + ct * 16;
  floatx4 acc = tile_dot(tA, ld, a.W[0], K, N, c0, kh ? half : 0, kh ? nsl : half, li, lk);
  if (kh) red[ct * 64 + lane] = acc;
  __syncthreads();
  if (kh) return;
  acc = acc + red[ct * 64 + lane];
  const int c = c0 + li;
  if (c >= N) return;
  const float bc = a.b[0] ? a.b[0][c] : 0.f;
  const bool drop_next = train && a.dropout[1];
  const bool relu = a.relu[0] != 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t row = r0 + 4 * lk + r;
    if (row >= B) continue;
    float z = acc[r] + bc;
    if (relu) z = z < 0.f ? 0.f : z;
    if (drop_next) {
      const bool kp = mlp_keep(key, 1, (uint64_t)(row * N + c), a.keep_threshold);
      z = kp ? z * a.scale : 0.f;
    }
    a.xs[1][row * N + c] = z;
  }
}

// ------------------------------------------------------------------------ data grad
// l_end = 1 (the wide backward below takes layer 0): layers L-1..1 only.
__global__ __launch_bounds__(kMlpThreads) void mlp_bwd_data_kernel(mirec_mlp a,
                                                                   const float* __restrict__ dy,
                                                                   int64_t B,
                                                                   float* __restrict__ gx0,
                                                                   int ldA, int ldB, int split,
                                                                   int l_end) {
  extern __shared__ float lds[];
  float* const tA = lds;
  float* const tB = lds + kMlpRows * ldA;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int li = lane & 15, lk = lane >> 4;
  // split = 2: two blocks per 16 rows; both run the narrow layers above layer 0 (block
  // half 0 alone stores their g_z), and they share layer 0's wide output tiles (even /
  // odd), which is where the time goes (C4: 39 tiles of 624 columns)
  const int half = split > 1 ? (int)(blockIdx.x & 1) : 0;
  const int64_t r0 = (int64_t)(blockIdx.x / split) * kMlpRows;
  const int L = a.n_layers;
  {
    const int N = a.dims[L];
    float* t = (L & 1) ? tB : tA;
    const int ld = (L & 1) ? ldB : ldA;
    for (int idx = tid; idx < kMlpRows * N; idx += kMlpThreads) {
      const int i = idx / N, n = idx - i * N;
      const int64_t row = r0 + i;
      t[i * ld + n] = row < B ? dy[row * N + n] : 0.f;
    }
  }
  __syncthreads();
  for (int l = L - 1; l >= l_end; --l) {
    const int K = a.dims[l], N = a.dims[l + 1];     // g_x [16, K] = g_z [16, N] . W [N, K]
    const float* cur = ((l + 1) & 1) ? tB : tA;      // g_z: width dims[l + 1]
    float* nxt = (l & 1) ? tB : tA;                  // g_z of the layer below: width dims[l]
    const int ld = ((l + 1) & 1) ? ldB : ldA, ldn = (l & 1) ? ldB : ldA;
    const float* __restrict__ W = a.W[l];
    const float* __restrict__ xs = l > 0 ? a.xs[l] : nullptr;
    float* __restrict__ gz = l > 0 ? a.gz[l - 1] : nullptr;
    const float sc = (a.dropout[l] ? a.scale : 1.f);
    const int ntile = (K + 15) / 16;
    // this wave's (tile, group) sequence — tiles t = wave, wave + 8, ..., groups of
    // kMlpU 16-wide slices of N — with the next item's loads (and, at a tile's first
    // group, the tile's saved-input loads for its epilogue) issued before the current
    // item's MFMAs, across tile boundaries too
    const int ng = (N + 16 * kMlpU - 1) / (16 * kMlpU);
    // tiles of this wave: t0, t0 + stride, ... (layer 0 split over the block pair)
    const int t0 = l == 0 ? half + split * wave : wave;
    const int tstride = l == 0 ? split * kMlpWaves : kMlpWaves;
    const int my_tiles = t0 < ntile ? (ntile - t0 + tstride - 1) / tstride : 0;
    const bool store_gz = half == 0;
    const int items = my_tiles * ng;
    float pa[kMlpU][4], pb[kMlpU][4], px[4];
    auto load = [&](int it) {         // branch-free, as in the forward
      const int t = t0 + (it / ng) * tstride, g0 = (it % ng) * 16 * kMlpU;
      const int c = t * 16 + li;
      const bool cin = c < K;
      const int cc = cin ? c : K - 1;
#pragma unroll
      for (int u = 0; u < kMlpU; ++u) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int n = g0 + 16 * u + 4 * lk + s;
          const int nc = n < N ? n : N - 1;
          pa[u][s] = cur[li * ld + nc];
          // a multiply by 0 / 1, not a select: the compiler sinks `cond ? load : 0` into
          // a conditional load followed by a full vmcnt(0) wait, one load at a time
          pb[u][s] = W[(int64_t)nc * K + cc] * ((n < N && cin) ? 1.f : 0.f);
        }
      }
      if (it % ng == 0) {             // the tile's saved inputs / layer-0 keep flags
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = r0 + 4 * lk + r;
          const int64_t e = (row < B ? row : B - 1) * K + cc;
          px[r] = l > 0 ? xs[e] : (a.dropout[0] ? (float)a.mask0[e] : 1.f);
        }
      }
    };
    floatx4 accA = {0.f, 0.f, 0.f, 0.f}, accB = {0.f, 0.f, 0.f, 0.f};
    float xv[4] = {0.f, 0.f, 0.f, 0.f};
    if (items > 0) load(0);
    for (int it = 0; it < items; ++it) {
      float ca[kMlpU][4], cb[kMlpU][4];
#pragma unroll
      for (int u = 0; u < kMlpU; ++u)
#pragma unroll
        for (int s = 0; s < 4; ++s) { ca[u][s] = pa[u][s]; cb[u][s] = pb[u][s]; }
      if (it % ng == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) xv[r] = px[r];
      }
      if (it + 1 < items) load(it + 1);
#pragma unroll
      for (int u = 0; u < kMlpU; ++u) {
        floatx4& acc = (u & 1) ? accB : accA;
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = mfma4(ca[u][s], cb[u][s], acc);
      }
      if (it % ng != ng - 1) continue;
      // the tile is complete: epilogue
      const int t = t0 + (it / ng) * tstride;
      const int c = t * 16 + li;
      const floatx4 acc = accA + accB;
      accA = floatx4{0.f, 0.f, 0.f, 0.f};
      accB = accA;
      if (c < K) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 4 * lk + r;
          const int64_t row = r0 + i;
          float g = acc[r];
          if (l > 0) {
            // dropout backward (g * mask * scale) then ReLU backward ([h > 0])
            const bool live = row < B && xv[r] > 0.f;
            g = live ? g * sc : 0.f;
            if (row < B && store_gz) gz[row * K + c] = g;
            nxt[i * ldn + c] = g;
          } else if (row < B) {
            if (a.dropout[0]) g = xv[r] != 0.f ? g * sc : 0.f;
            gx0[row * K + c] = g;
          }
        }
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------- weight grad
// Block -> (layer l, 16-row tile of dW_l's outputs, 16-column tile of its inputs).
__global__ __launch_bounds__(kMlpThreads) void mlp_bwd_weight_kernel(mirec_mlp a, int64_t B,
                                                                     const float* __restrict__ x0,
                                                                     const float* __restrict__ dy) {
  __shared__ float part[kMlpWaves][64][5];
  __shared__ float bpart[kMlpWaves][16];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int li = lane & 15, lk = lane >> 4;
  int l = 0;
  while (l + 1 < a.n_layers && (int)blockIdx.x >= a.tile_start[l + 1]) ++l;
  const int K = a.dims[l], N = a.dims[l + 1];
  const int nti = (K + 15) / 16;
  const int rel = (int)blockIdx.x - a.tile_start[l];
  const int ot = rel / nti, it = rel - ot * nti;
  const float* __restrict__ gz = l == a.n_layers - 1 ? dy : a.gz[l];
  const float* __restrict__ xs = (l == 0 && !a.xs[0]) ? x0 : a.xs[l];
  const int o = ot * 16 + li, i = it * 16 + li;
  const bool oin = o < N, iin = i < K;
  const bool with_bias = it == 0 && a.db[l];
  // rows of this wave: an eighth of the batch (multiple of 4)
  const int64_t q = ((B + 4 * kMlpWaves - 1) / (4 * kMlpWaves)) * 4;
  const int64_t b_lo = wave * q, b_hi = (b_lo + q < B) ? b_lo + q : B;
  floatx4 accA = {0.f, 0.f, 0.f, 0.f}, accB = {0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;
  // groups of 64 rows: row b0 + 4s + lk (s < 16); the next group's 32 loads are issued
  // before this group's sixteen MFMAs
  constexpr int S = 16;
  float pa[S], pb[S];
  const int oc = oin ? o : N - 1, ic = iin ? i : K - 1;
  auto load = [&](int64_t b0) {     // branch-free: clamped rows, zeroed after the load
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int64_t b = b0 + 4 * s + lk;
      const bool bin = b < b_hi;
      const int64_t bc = bin ? b : b_lo;
      const float g = gz[bc * N + oc];
      const float x = xs[bc * K + ic];
      pa[s] = (oin && bin) ? g : 0.f;
      pb[s] = (iin && bin) ? x : 0.f;
    }
  };
  if (b_lo < b_hi) load(b_lo);
  for (int64_t b0 = b_lo; b0 < b_hi; b0 += 4 * S) {
    float ca[S], cb[S];
#pragma unroll
    for (int s = 0; s < S; ++s) { ca[s] = pa[s]; cb[s] = pb[s]; }
    if (b0 + 4 * S < b_hi) load(b0 + 4 * S);
#pragma unroll
    for (int s = 0; s < S; ++s) {
      floatx4& acc = (s & 1) ? accB : accA;
      acc = mfma4(ca[s], cb[s], acc);
      bsum += ca[s];
    }
  }
  const floatx4 acc = accA + accB;
#pragma unroll
  for (int r = 0; r < 4; ++r) part[wave][lane][r] = acc[r];
  if (with_bias) {       // the four row phases of column o, in phase order
    const float s1 = __shfl(bsum, li + 16, 64), s2 = __shfl(bsum, li + 32, 64),
                s3 = __shfl(bsum, li + 48, 64);
    if (lk == 0) bpart[wave][li] = ((bsum + s1) + s2) + s3;
  }
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = part[0][lane][r];
#pragma unroll
      for (int w = 1; w < kMlpWaves; ++w) v += part[w][lane][r];
      const int oo = ot * 16 + 4 * lk + r;
      if (oo < N && iin) a.dW[l][(int64_t)oo * K + i] = v;
    }
    if (with_bias && lk == 0 && oin) {
      float v = bpart[0][li];
#pragma unroll
      for (int w = 1; w < kMlpWaves; ++w) v += bpart[w][li];
      a.db[l][o] = v;
    }
  }
}

// --------------------------------------------------------------- wide backward (one launch)
// Behind mlp_bwd_data_kernel(l_end = 1), which leaves g_z of every layer output in
// gz[0..L-2]: layer 0's data gradient and every layer's weight (and bias) gradient, as
// 64-column wave tiles over the whole chip.
//
// Column permutation: a wave's 64 output columns c0..c0+63 form four 16 x 16 MFMA tiles
// j = 0..3 whose lane column li holds output column c0 + 4 li + j, so one float4 load of
// the B operand (4 consecutive columns of a row) feeds the four tiles' MFMAs, and the
// results go out as float4 stores (4 consecutive columns of one row).
//
// Role D (blocks [0, nD)): g_x0 [B, K0] = g_z0 [B, N0] . W0 [N0, K0] per 16 rows x 64
//   columns; epilogue: layer 0's dropout backward (keep flag ? scale : 0).
// Role W (blocks [nD, ..)): dW_l [N, K] = g_z_l^T . x_l over the batch, per 16 output rows
//   x 64 columns; the batch is cut into 4G slices — the 4 waves of a block take 4 of
//   them (partials added in LDS in wave order), the G blocks of one tile hand their
//   partials over (scratch, write-through 8-B agent stores, one agent-scope add per
//   block; the block whose add comes last takes an agent acquire, sums the G partials in
//   block order and writes dW / db): every sum in a fixed order, run-to-run identical.
constexpr int kWideG = 4;
struct WidePlan {
  int nD;                                  // role-D blocks
  int ncbD, nrtD;                          // role D: column groups of 64, row tiles of 16
  int tile0[MIREC_MLP_MAX_LAYERS + 1];     // role W: first wave tile of layer l
  int ncb[MIREC_MLP_MAX_LAYERS];           // role W: column groups of layer l
  int64_t q;                               // rows per batch slice (multiple of 16)
};
constexpr int kWideTileFloats = 64 * 16 + 16;   // a wave tile's partial: 64 lanes x 16 + bias

__device__ __forceinline__ void st8_agent(float* p, float a, float b) {
  auto q = (__attribute__((address_space(1))) unsigned long long*)(p);
  const unsigned long long w =
      (unsigned long long)__float_as_uint(a) | ((unsigned long long)__float_as_uint(b) << 32);
  __hip_atomic_store(q, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float2 ld8_agent(const float* p) {
  auto q = (const __attribute__((address_space(1))) unsigned long long*)(p);
  const unsigned long long w = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return make_float2(__uint_as_float((unsigned)w), __uint_as_float((unsigned)(w >> 32)));
}

__global__ __launch_bounds__(kWideThreads) void mlp_bwd_wide_kernel(
    mirec_mlp a, const float* __restrict__ x0, const float* __restrict__ dy, int64_t B,
    float* __restrict__ gx0, WidePlan P) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int li = lane & 15, lk = lane >> 4;
  const int L = a.n_layers;
  floatx4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};

  if ((int)blockIdx.x < P.nD) {                      // ---- role D
    const int t = blockIdx.x * 4 + wave;
    if (t >= P.ncbD * P.nrtD) return;
    const int rt = t / P.ncbD, cb = t - rt * P.ncbD;
    const int K = a.dims[0], N = a.dims[1];
    const int64_t r0 = (int64_t)rt * kMlpRows;
    const int c = cb * 64 + 4 * li;                  // this lane's 4 output columns
    const bool cin = c < K;                          // K % 4 == 0: a float4 is all in or out
    const int cc = cin ? c : K - 4;
    const int64_t row = r0 + li < B ? r0 + li : B - 1;
    const float* __restrict__ gz = a.gz[0];
    const float* __restrict__ W = a.W[0];
    float4 pa, pb[4];
    auto load = [&](int n0) {                        // K index of MFMA e: n0 + 4 lk + e
      const int n = n0 + 4 * lk;
      const int nc = n < N ? n : N - 4;
      pa = *reinterpret_cast<const float4*>(gz + row * N + nc);
      if (n >= N) pa = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        pb[e] = *reinterpret_cast<const float4*>(W + (int64_t)(nc + e) * K + cc);
        if (!cin) pb[e] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    };
    load(0);
    for (int n0 = 0; n0 < N; n0 += 16) {
      const float4 ca = pa;
      float4 cbv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) cbv[e] = pb[e];
      if (n0 + 16 < N) load(n0 + 16);
      const float av[4] = {ca.x, ca.y, ca.z, ca.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[0] = mfma4(av[e], cbv[e].x, acc[0]);
        acc[1] = mfma4(av[e], cbv[e].y, acc[1]);
        acc[2] = mfma4(av[e], cbv[e].z, acc[2]);
        acc[3] = mfma4(av[e], cbv[e].w, acc[3]);
      }
    }
    if (!cin) return;
    const float sc = a.dropout[0] ? a.scale : 1.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t rr = r0 + 4 * lk + r;
      if (rr >= B) continue;
      float4 g = make_float4(acc[0][r], acc[1][r], acc[2][r], acc[3][r]);
      if (a.dropout[0]) {
        const uint32_t m = *reinterpret_cast<const uint32_t*>(a.mask0 + rr * K + c);
        g.x = (m & 0xFFu) ? g.x * sc : 0.f;
        g.y = (m & 0xFF00u) ? g.y * sc : 0.f;
        g.z = (m & 0xFF0000u) ? g.z * sc : 0.f;
        g.w = (m & 0xFF000000u) ? g.w * sc : 0.f;
      }
      *reinterpret_cast<float4*>(gx0 + rr * K + c) = g;
    }
    return;
  }

  // ---- role W: block -> (wave tile wt, block group g); wave -> batch slice 4 g + wave
  __shared__ float red[4][64][17];
  const int wb = (int)blockIdx.x - P.nD;
  const int wt = wb / kWideG, g = wb - wt * kWideG;
  int l = 0;
  while (l + 1 < L && wt >= P.tile0[l + 1]) ++l;
  const int K = a.dims[l], N = a.dims[l + 1];
  const int rel = wt - P.tile0[l];
  const int ot = rel / P.ncb[l], cb = rel - ot * P.ncb[l];
  const float* __restrict__ gz = l == L - 1 ? dy : a.gz[l];
  const float* __restrict__ xs = (l == 0 && !a.xs[0]) ? x0 : a.xs[l];
  const int o = ot * 16 + li;                        // this lane's output row (A row)
  const bool oin = o < N;
  const int oc = oin ? o : N - 1;
  const int c = cb * 64 + 4 * li;
  const bool cin = c < K;
  const int cc = cin ? c : K - 4;
  const int64_t b_lo = (int64_t)(4 * g + wave) * P.q;
  const int64_t b_hi = b_lo + P.q < B ? b_lo + P.q : B;
  float bsum = 0.f;
  float pa[4];
  float4 pb[4];
  auto load = [&](int64_t b0) {                      // batch row of MFMA e: b0 + 4 lk + e
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t b = b0 + 4 * lk + e;
      const bool bin = b < b_hi;
      const int64_t bc = bin ? b : b_lo;
      const float gv = gz[bc * N + oc];
      pb[e] = *reinterpret_cast<const float4*>(xs + bc * K + cc);
      pa[e] = (oin && bin) ? gv : 0.f;
      if (!(cin && bin)) pb[e] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  if (b_lo < b_hi) load(b_lo);
  for (int64_t b0 = b_lo; b0 < b_hi; b0 += 16) {
    float ca[4];
    float4 cbv[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) { ca[e] = pa[e]; cbv[e] = pb[e]; }
    if (b0 + 16 < b_hi) load(b0 + 16);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc[0] = mfma4(ca[e], cbv[e].x, acc[0]);
      acc[1] = mfma4(ca[e], cbv[e].y, acc[1]);
      acc[2] = mfma4(ca[e], cbv[e].z, acc[2]);
      acc[3] = mfma4(ca[e], cbv[e].w, acc[3]);
      bsum += ca[e];
    }
  }
  // this wave's partial: 16 values per lane, the bias partial of row li (its 4 lk lanes)
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave][lane][4 * j + r] = acc[j][r];
  {
    const float s1 = __shfl(bsum, li + 16, 64), s2 = __shfl(bsum, li + 32, 64),
                s3 = __shfl(bsum, li + 48, 64);
    if (lk == 0) red[wave][li][16] = ((bsum + s1) + s2) + s3;
  }
  __syncthreads();
  if (wave != 0) return;
  float v[17];
#pragma unroll
  for (int k = 0; k < 16; ++k)
    v[k] = ((red[0][lane][k] + red[1][lane][k]) + red[2][lane][k]) + red[3][lane][k];
  v[16] = ((red[0][li][16] + red[1][li][16]) + red[2][li][16]) + red[3][li][16];
  // hand-off of the block partials (scratch [tile][g][kWideTileFloats]; the guide's first
  // form: write-through 8-B agent stores, this wave drained, one agent-scope add; the
  // block whose add returns G - 1 takes an agent acquire and reads them back with
  // agent-scope loads). Only wave 0 stores, adds and reads.
  float* __restrict__ part = a.wscratch + (int64_t)wt * kWideG * kWideTileFloats;
  float* mine = part + (int64_t)g * kWideTileFloats;
#pragma unroll
  for (int k = 0; k < 16; k += 2) st8_agent(mine + lane * 16 + k, v[k], v[k + 1]);
  if (lk == 0) {
    auto q = (__attribute__((address_space(1))) unsigned int*)(mine + 1024 + li);
    __hip_atomic_store(q, __float_as_uint(v[16]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int prev = 0;
  if (lane == 0)
    prev = __hip_atomic_fetch_add(a.wcount + wt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  prev = __shfl(prev, 0, 64);
  if (prev != kWideG - 1) return;                    // wave-uniform
  if (lane == 0)
    __hip_atomic_store(a.wcount + wt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float tot[17];
#pragma unroll
  for (int k = 0; k < 17; ++k) tot[k] = 0.f;
  for (int gg = 0; gg < kWideG; ++gg) {              // block order: a fixed summation order
    const float* src = part + (int64_t)gg * kWideTileFloats;
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
      const float2 w = ld8_agent(src + lane * 16 + k);
      tot[k] = gg ? tot[k] + w.x : w.x;
      tot[k + 1] = gg ? tot[k + 1] + w.y : w.y;
    }
    auto q = (const __attribute__((address_space(1))) unsigned int*)(src + 1024 + li);
    const float bv = __uint_as_float(__hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    tot[16] = gg ? tot[16] + bv : bv;
  }
  if (cin) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int oo = ot * 16 + 4 * lk + r;
      if (oo < N)
        *reinterpret_cast<float4*>(a.dW[l] + (int64_t)oo * K + c) =
            make_float4(tot[r], tot[4 + r], tot[8 + r], tot[12 + r]);
    }
  }
  if (cb == 0 && a.db[l] && lk == 0 && oin) a.db[l][o] = tot[16];
}

static int mlp_check(const mirec_mlp* a, const char* what) {
  bool ok = a && a->n_layers >= 1 && a->n_layers <= MIREC_MLP_MAX_LAYERS;
  if (ok) {
    for (int l = 0; l <= a->n_layers; ++l)
      ok = ok && a->dims[l] >= 1 && a->dims[l] <= 1024 && (l == a->n_layers || a->dims[l] % 4 == 0);
    for (int l = 0; l < a->n_layers; ++l) {
      ok = ok && a->W[l] && ((uintptr_t)a->W[l] % 16 == 0);
      if (l + 1 < a->n_layers) ok = ok && a->relu[l];       // hidden layers: ReLU
    }
  }
  if (!ok) {
    set_error("%s: bad MLP descriptor (1..%d layers, widths <= 1024 and multiples of 4 except "
              "the output, ReLU after every hidden layer, 16-B aligned weights)",
              what, MIREC_MLP_MAX_LAYERS);
    return -1;
  }
  return 0;
}

// The two tiles must fit the 64 KB of dynamic LDS a launch gets without attributes
// (C4: 16 x (628 + 132) floats = 48.6 KB).
static int mlp_lds_limit(size_t shm, const char* what) {
  if (shm > 65536) {
    set_error("%s: layer widths need %zu B of LDS (> 64 KB)", what, shm);
    return -1;
  }
  return 0;
}

}  // namespace mirec

using namespace mirec;

namespace mirec {
// LDS of the wide layer-0 forward: the 16-row A tile + the K-half partials
static size_t wide_fwd_shm(const mirec_mlp& a) {
  const int ld = (a.dims[0] + 15) / 16 * 16 + 4;
  return (size_t)kMlpRows * ld * sizeof(float) + 2 * 64 * sizeof(floatx4);
}
// The wide layer-0 forward is OFF by default: with layers 1.. behind it in a second launch
// it measured 37.5 µs for the C4 forward against 31.0 µs for the one fused launch
// (profiles/r04_models.json vs round 5's models run). MIREC_MLP_WIDE_FWD=1 turns it on.
static bool wide_fwd_on() {
  static const bool on = [] {
    const char* e = getenv("MIREC_MLP_WIDE_FWD");
    return e && e[0] == '1';
  }();
  return on;
}
static bool wide_fwd_ok(const mirec_mlp& a) {
  return wide_fwd_on() && a.n_layers >= 2 && a.dims[0] >= kWideMin && a.xs[1] != nullptr &&
         wide_fwd_shm(a) <= 65536;
}
// the wide backward's plan (WidePlan) and wave tiles; false: the one-block-per-16-rows path
static bool wide_bwd_plan(const mirec_mlp& a, int64_t B, WidePlan* P, int* tiles) {
  if (a.n_layers < 2 || a.dims[0] < kWideMin || B <= 0) return false;
  memset(P, 0, sizeof(*P));
  P->nrtD = (int)((B + kMlpRows - 1) / kMlpRows);
  P->ncbD = (a.dims[0] + 63) / 64;
  P->nD = (int)(((int64_t)P->nrtD * P->ncbD + 3) / 4);
  int t = 0;
  for (int l = 0; l < a.n_layers; ++l) {
    P->tile0[l] = t;
    P->ncb[l] = (a.dims[l] + 63) / 64;
    t += ((a.dims[l + 1] + 15) / 16) * P->ncb[l];
  }
  P->tile0[a.n_layers] = t;
  P->q = ((B + 4 * kWideG - 1) / (4 * kWideG) + 15) / 16 * 16;
  *tiles = t;
  return true;
}
}  // namespace mirec

// Scratch of the wide backward (mirec_mlp.wscratch / .wcount): 1 and the sizes when the
// descriptor's shapes take it, 0 when they do not (wscratch may stay NULL then).
extern "C" int mirec_mlp_bwd_workspace(const mirec_mlp* mlp, int64_t B, int64_t* scratch_floats,
                                       int64_t* counters) {
  if (!mlp || !scratch_floats || !counters || mlp_check(mlp, "mirec_mlp_bwd_workspace")) return -1;
  WidePlan P;
  int tiles = 0;
  *scratch_floats = 0;
  *counters = 0;
  if (!wide_bwd_plan(*mlp, B, &P, &tiles)) return 0;
  *scratch_floats = (int64_t)tiles * kWideG * kWideTileFloats;
  *counters = tiles;
  return 1;
}

extern "C" int mirec_mlp_fwd_f32(const mirec_mlp* mlp, const float* x, int64_t B, float* y,
                                 int32_t train, void* stream) {
  if (B == 0) return 0;
  if (mlp_check(mlp, "mirec_mlp_fwd_f32")) return -1;
  const mirec_mlp& a = *mlp;
  bool any_drop = false;
  for (int l = 0; l < a.n_layers; ++l) any_drop |= train && a.dropout[l];
  if (!x || !y || B < 0 || (any_drop && (!a.counter || !a.arrive)) ||
      (train && a.dropout[0] && (!a.mask0 || !a.xs[0])) || ((uintptr_t)x % 16) != 0) {
    set_error("mirec_mlp_fwd_f32: bad arguments");
    return -1;
  }
  if (train) {
    for (int l = 1; l < a.n_layers; ++l)
      if (!a.xs[l]) { set_error("mirec_mlp_fwd_f32: training needs the saved inputs"); return -1; }
  }
  const unsigned row_blocks = (unsigned)((B + kMlpRows - 1) / kMlpRows);
  hipStream_t st = (hipStream_t)stream;
  // wide layer 0 over the whole chip (it writes xs[1]), then layers 1.. in row blocks
  const int l0 = wide_fwd_ok(a) ? 1 : 0;
  if (l0) {
    const int ld = (a.dims[0] + 15) / 16 * 16 + 4;
    hipLaunchKernelGGL(mlp_l0_fwd_kernel, dim3(row_blocks, (unsigned)((a.dims[1] + kL0Cols - 1) / kL0Cols)),
                       dim3(kWideThreads), wide_fwd_shm(a), st, a, x, B, (int)train, ld);
    const int rc = launch_status("mirec_mlp_fwd_f32: layer 0");
    if (rc) return rc;
  }
  int ldA, ldB;
  mlp_ld(a, &ldA, &ldB, l0);
  const size_t shm1 = (size_t)kMlpRows * (ldA + ldB) * sizeof(float);
  const size_t shmK = shm1 + (size_t)(kFwdKS - 1) * kMlpWaves * 64 * sizeof(floatx4);
  const bool ks = kFwdKS > 1 && shmK <= 65536;
  const size_t shm = ks ? shmK : shm1;
  if (mlp_lds_limit(shm, "mirec_mlp_fwd_f32")) return -1;
  if (ks)
    hipLaunchKernelGGL(mlp_fwd_kernel<kFwdKS>, dim3(row_blocks), dim3(kMlpThreads * kFwdKS), shm,
                       st, a, x, B, y, (int)train, ldA, ldB, l0);
  else
    hipLaunchKernelGGL(mlp_fwd_kernel<1>, dim3(row_blocks), dim3(kMlpThreads), shm, st, a, x, B,
                       y, (int)train, ldA, ldB, l0);
  return launch_status("mirec_mlp_fwd_f32");
}

extern "C" int mirec_mlp_bwd_f32(const mirec_mlp* mlp, const float* x, const float* dy, int64_t B,
                                 float* gx, void* stream) {
  if (B == 0) return 0;
  if (mlp_check(mlp, "mirec_mlp_bwd_f32")) return -1;
  mirec_mlp a = *mlp;
  bool ok = x && dy && gx && B > 0;
  for (int l = 0; l < a.n_layers; ++l) ok = ok && a.dW[l];
  for (int l = 1; l < a.n_layers; ++l) ok = ok && a.xs[l] && a.gz[l - 1];
  if (a.dropout[0]) ok = ok && a.mask0;
  if (!ok) {
    set_error("mirec_mlp_bwd_f32: bad arguments (saved inputs, g_z buffers and dW needed)");
    return -1;
  }
  hipStream_t st = (hipStream_t)stream;
  const int64_t row_blocks = (B + kMlpRows - 1) / kMlpRows;
  WidePlan P;
  int wtiles = 0;
  if (a.wscratch && a.wcount && ((uintptr_t)x % 16) == 0 && wide_bwd_plan(a, B, &P, &wtiles)) {
    // layers L-1..1 in row blocks (g_z of every layer output), then layer 0's data
    // gradient and every weight gradient over the whole chip
    int ldA, ldB;
    mlp_ld(a, &ldA, &ldB, 1);
    const size_t shm = (size_t)kMlpRows * (ldA + ldB) * sizeof(float);
    if (mlp_lds_limit(shm, "mirec_mlp_bwd_f32")) return -1;
    hipLaunchKernelGGL(mlp_bwd_data_kernel, dim3((unsigned)row_blocks), dim3(kMlpThreads), shm, st,
                       a, dy, B, gx, ldA, ldB, 1, 1);
    int rc = launch_status("mirec_mlp_bwd_f32: data");
    if (rc) return rc;
    hipLaunchKernelGGL(mlp_bwd_wide_kernel, dim3((unsigned)(P.nD + wtiles * kWideG)),
                       dim3(kWideThreads), 0, st, a, x, dy, B, gx, P);
    return launch_status("mirec_mlp_bwd_f32: wide");
  }
  int tiles = 0;
  for (int l = 0; l < a.n_layers; ++l) {
    a.tile_start[l] = tiles;
    tiles += ((a.dims[l + 1] + 15) / 16) * ((a.dims[l] + 15) / 16);
  }
  int ldA, ldB;
  mlp_ld(a, &ldA, &ldB);
  const size_t shm = (size_t)kMlpRows * (ldA + ldB) * sizeof(float);
  if (mlp_lds_limit(shm, "mirec_mlp_bwd_f32")) return -1;
  // two blocks per 16 rows while that still fits one wave of blocks on the chip and
  // layer 0 has tiles for both
  const int split = (row_blocks * 2 <= 256 && (a.dims[0] + 15) / 16 >= 2 * kMlpWaves) ? 2 : 1;
  hipLaunchKernelGGL(mlp_bwd_data_kernel, dim3((unsigned)(row_blocks * split)),
                     dim3(kMlpThreads), shm, st, a, dy, B, gx, ldA, ldB, split, 0);
  int rc = launch_status("mirec_mlp_bwd_f32: data");
  if (rc) return rc;
  hipLaunchKernelGGL(mlp_bwd_weight_kernel, dim3((unsigned)tiles), dim3(kMlpThreads), 0, st, a, B,
                     x, dy);
  return launch_status("mirec_mlp_bwd_f32: weight");
}
