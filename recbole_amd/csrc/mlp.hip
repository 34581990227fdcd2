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
// of odd j in tile B (a layer reads one and writes the other).
static void mlp_ld(const mirec_mlp& a, int* ldA, int* ldB) {
  int m[2] = {0, 0};
  for (int j = 0; j <= a.n_layers; ++j) m[j & 1] = a.dims[j] > m[j & 1] ? a.dims[j] : m[j & 1];
  *ldA = (m[0] + 15) / 16 * 16 + 4;
  *ldB = (m[1] + 15) / 16 * 16 + 4;
}

// -------------------------------------------------------------------------- forward
__global__ __launch_bounds__(kMlpThreads) void mlp_fwd_kernel(mirec_mlp a, const float* __restrict__ x,
                                                              int64_t B, float* __restrict__ y,
                                                              int train, int ldA, int ldB) {
  extern __shared__ float lds[];
  float* const tA = lds;
  float* const tB = lds + kMlpRows * ldA;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int li = lane & 15, lk = lane >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * kMlpRows;
  const int L = a.n_layers;
  bool any_drop = false;
  for (int l = 0; l < L; ++l) any_drop |= train && a.dropout[l];
  const uint64_t key = any_drop ? splitmix64(a.seed + (uint64_t)a.counter[0]) : 0ull;

  // layer 0's input rows, after its dropout: the block's 16 rows are one contiguous
  // range of x; every float4 of it is loaded before any is processed (stores to the
  // saved buffers may alias x as far as the compiler knows, which would otherwise
  // serialise one load per element)
  {
    const int K = a.dims[0];
    const bool drop = train && a.dropout[0];
    constexpr int kV = kMlpRows * 1024 / 4 / kMlpThreads;   // float4 per thread, K <= 1024
    const int nv = kMlpRows * K / 4;
    const int64_t lim = (B - r0) * K / 4;                   // float4 of valid rows
    const float4* x4 = reinterpret_cast<const float4*>(x + r0 * K);
    float4 xv[kV];
#pragma unroll
    for (int j = 0; j < kV; ++j) {
      const int q = tid + j * kMlpThreads;
      xv[j] = (q < nv && q < lim) ? x4[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int j = 0; j < kV; ++j) {
      const int q = tid + j * kMlpThreads;
      if (q >= nv) break;
      const int e0 = 4 * q, i = e0 / K, k = e0 - i * K;
      float4 v = xv[j];
      if (q < lim) {
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
          *reinterpret_cast<uint32_t*>(a.mask0 + e) =
              (k0 ? 1u : 0u) | (k1 ? 1u << 8 : 0u) | (k2 ? 1u << 16 : 0u) | (k3 ? 1u << 24 : 0u);
        }
        if (a.xs[0] && a.xs[0] != x) *reinterpret_cast<float4*>(a.xs[0] + e) = v;
      }
      *reinterpret_cast<float4*>(tA + i * ldA + k) = v;
    }
  }
  __syncthreads();

  for (int l = 0; l < L; ++l) {
    const int K = a.dims[l], N = a.dims[l + 1];
    const float* cur = (l & 1) ? tB : tA;
    float* nxt = (l & 1) ? tA : tB;
    const int ld = (l & 1) ? ldB : ldA, ldn = (l & 1) ? ldA : ldB;
    const float* __restrict__ W = a.W[l];
    const float* __restrict__ bias = a.b[l];
    const bool last = l == L - 1;
    const bool drop_next = !last && train && a.dropout[l + 1];
    const bool relu = a.relu[l] != 0;
    float* __restrict__ save = last ? nullptr : a.xs[l + 1];
    const int ntile = (N + 15) / 16;
    for (int t = wave; t < ntile; t += kMlpWaves) {     // one 16-column tile per wave
      const int c = t * 16 + li;
      const float* wr = W + (int64_t)(c < N ? c : N - 1) * K;
      // k = k0 + 16u + 4*lk + s: the four MFMAs of a 16-wide slice cover it once each;
      // the next group's loads are issued before this group's MFMAs (two accumulators)
      float4 pa[kFwdU], pb[kFwdU];
      // branch-free loads (addresses clamped into the row, out-of-range slices zeroed
      // after the load): straight-line code lets the compiler wait on the older group
      // only (vmcnt(N)) while the next group is in flight
      auto load = [&](int k0) {
#pragma unroll
        for (int u = 0; u < kFwdU; ++u) {
          const int k = k0 + 16 * u + 4 * lk;
          const int kc = k < K ? k : K - 4;
          pa[u] = *reinterpret_cast<const float4*>(cur + li * ld + kc);
          pb[u] = *reinterpret_cast<const float4*>(wr + kc);
          if (k >= K) pb[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      };
      floatx4 accA = {0.f, 0.f, 0.f, 0.f}, accB = {0.f, 0.f, 0.f, 0.f};
      auto mfma_group = [&](const float4* ca, const float4* cb) {
#pragma unroll
        for (int u = 0; u < kFwdU; ++u) {
          floatx4& acc = (u & 1) ? accB : accA;
          acc = mfma4(ca[u].x, cb[u].x, acc);
          acc = mfma4(ca[u].y, cb[u].y, acc);
          acc = mfma4(ca[u].z, cb[u].z, acc);
          acc = mfma4(ca[u].w, cb[u].w, acc);
        }
      };
#if defined(MIREC_FWD_PF2)
      // two groups' loads in flight while one group's MFMAs run: buffers q (even groups)
      // and p (odd groups), taken two groups per iteration so every index is static
      constexpr int GW = 16 * kFwdU;
      float4 qa[kFwdU], qb[kFwdU];
      auto load_q = [&](int k0) {
#pragma unroll
        for (int u = 0; u < kFwdU; ++u) {
          const int k = k0 + 16 * u + 4 * lk;
          const int kc = k < K ? k : K - 4;
          qa[u] = *reinterpret_cast<const float4*>(cur + li * ld + kc);
          qb[u] = *reinterpret_cast<const float4*>(wr + kc);
          if (k >= K) qb[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      };
      load_q(0);
      if (GW < K) load(GW);
      for (int k0 = 0; k0 < K; k0 += 2 * GW) {
        mfma_group(qa, qb);                       // group k0 (its loads were issued first)
        if (k0 + 2 * GW < K) load_q(k0 + 2 * GW);
        if (k0 + GW < K) {
          mfma_group(pa, pb);                     // group k0 + GW
          if (k0 + 3 * GW < K) load(k0 + 3 * GW);
        }
      }
#else
      load(0);
      for (int k0 = 0; k0 < K; k0 += 16 * kFwdU) {
        float4 ca[kFwdU], cb[kFwdU];
#pragma unroll
        for (int u = 0; u < kFwdU; ++u) { ca[u] = pa[u]; cb[u] = pb[u]; }
        if (k0 + 16 * kFwdU < K) load(k0 + 16 * kFwdU);
        mfma_group(ca, cb);
      }
#endif
      const floatx4 acc0 = accA + accB;
      // epilogue: lane holds rows 4*lk + r of column c
      if (c < N) {
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

// ------------------------------------------------------------------------ data grad
__global__ __launch_bounds__(kMlpThreads) void mlp_bwd_data_kernel(mirec_mlp a,
                                                                   const float* __restrict__ dy,
                                                                   int64_t B,
                                                                   float* __restrict__ gx0,
                                                                   int ldA, int ldB, int split) {
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
  for (int l = L - 1; l >= 0; --l) {
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
  int ldA, ldB;
  mlp_ld(a, &ldA, &ldB);
  const size_t shm = (size_t)kMlpRows * (ldA + ldB) * sizeof(float);
  if (mlp_lds_limit(shm, "mirec_mlp_fwd_f32")) return -1;
  hipLaunchKernelGGL(mlp_fwd_kernel, dim3((unsigned)((B + kMlpRows - 1) / kMlpRows)),
                     dim3(kMlpThreads), shm, (hipStream_t)stream, a, x, B, y, (int)train, ldA,
                     ldB);
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
  int tiles = 0;
  for (int l = 0; l < a.n_layers; ++l) {
    a.tile_start[l] = tiles;
    tiles += ((a.dims[l + 1] + 15) / 16) * ((a.dims[l] + 15) / 16);
  }
  int ldA, ldB;
  mlp_ld(a, &ldA, &ldB);
  const size_t shm = (size_t)kMlpRows * (ldA + ldB) * sizeof(float);
  if (mlp_lds_limit(shm, "mirec_mlp_bwd_f32")) return -1;
  hipStream_t st = (hipStream_t)stream;
  // two blocks per 16 rows while that still fits one wave of blocks on the chip and
  // layer 0 has tiles for both
  const int64_t row_blocks = (B + kMlpRows - 1) / kMlpRows;
  const int split = (row_blocks * 2 <= 256 && (a.dims[0] + 15) / 16 >= 2 * kMlpWaves) ? 2 : 1;
  hipLaunchKernelGGL(mlp_bwd_data_kernel, dim3((unsigned)(row_blocks * split)),
                     dim3(kMlpThreads), shm, st, a, dy, B, gx, ldA, ldB, split);
  int rc = launch_status("mirec_mlp_bwd_f32: data");
  if (rc) return rc;
  hipLaunchKernelGGL(mlp_bwd_weight_kernel, dim3((unsigned)tiles), dim3(kMlpThreads), 0, st, a, B,
                     x, dy);
  return launch_status("mirec_mlp_bwd_f32: weight");
}
