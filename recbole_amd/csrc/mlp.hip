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
//                the four waves each take a quarter of the rows and their partial
//                tiles are added in wave order (fixed order, run to run identical).
//
// Dropout draws are counter-based (mirec_mlp_draw below; restated in numpy by
// tests/mlp_spec.py): element e of layer l in the forward with counter value c is
// kept iff  splitmix64(splitmix64(seed + c) ^ (e * 8 + l)) >> 32  <  keep_threshold.
// The counter lives on the device and the last block of each training forward
// advances it, so captured steps (HIP graph replays) draw new masks every step.
#include "common.h"

namespace mirec {

constexpr int kMlpRows = 16;       // rows per forward / data-grad block
constexpr int kMlpThreads = 256;   // four waves

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

  // layer 0's input rows, after its dropout
  {
    const int K = a.dims[0];
    const bool drop = train && a.dropout[0];
    for (int idx = tid; idx < kMlpRows * K; idx += kMlpThreads) {
      const int i = idx / K, k = idx - i * K;
      const int64_t row = r0 + i;
      float v = 0.f;
      if (row < B) {
        const int64_t e = row * K + k;
        v = x[e];
        if (drop) {
          const bool kp = mlp_keep(key, 0, (uint64_t)e, a.keep_threshold);
          v = kp ? v * a.scale : 0.f;
          a.mask0[e] = kp ? 1 : 0;
        }
        if (a.xs[0] && a.xs[0] != x) a.xs[0][e] = v;
      }
      tA[i * ldA + k] = v;
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
    for (int t0 = wave; t0 < ntile; t0 += 8) {      // two column tiles per wave: t0, t0 + 4
      const int t1 = t0 + 4;
      const bool has1 = t1 < ntile;
      const int c0 = t0 * 16 + li, c1 = t1 * 16 + li;
      const float* w0 = W + (int64_t)(c0 < N ? c0 : N - 1) * K;
      const float* w1 = W + (int64_t)(c1 < N ? c1 : N - 1) * K;
      floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      // k = k0 + 4*lk + s: the four MFMAs of a 16-wide slice cover it once each
      for (int k0 = 0; k0 < K; k0 += 16) {
        const int k = k0 + 4 * lk;
        const bool kin = k < K;
        const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 av = kin ? *reinterpret_cast<const float4*>(cur + li * ld + k) : z4;
        const float4 b0 = kin ? *reinterpret_cast<const float4*>(w0 + k) : z4;
        const float4 b1 = (kin && has1) ? *reinterpret_cast<const float4*>(w1 + k) : z4;
        acc0 = mfma4(av.x, b0.x, acc0);
        acc0 = mfma4(av.y, b0.y, acc0);
        acc0 = mfma4(av.z, b0.z, acc0);
        acc0 = mfma4(av.w, b0.w, acc0);
        if (has1) {
          acc1 = mfma4(av.x, b1.x, acc1);
          acc1 = mfma4(av.y, b1.y, acc1);
          acc1 = mfma4(av.z, b1.z, acc1);
          acc1 = mfma4(av.w, b1.w, acc1);
        }
      }
      // epilogue: lane holds rows 4*lk + r of column c
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h == 1 && !has1) break;
        const int c = h ? c1 : c0;
        if (c >= N) continue;
        const floatx4 acc = h ? acc1 : acc0;
        const float bc = bias ? bias[c] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 4 * lk + r;
          const int64_t row = r0 + i;
          float z = acc[r] + bc;
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
    __threadfence();
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
                                                                   int ldA, int ldB) {
  extern __shared__ float lds[];
  float* const tA = lds;
  float* const tB = lds + kMlpRows * ldA;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int li = lane & 15, lk = lane >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * kMlpRows;
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
    for (int t0 = wave; t0 < ntile; t0 += 8) {
      const int t1 = t0 + 4;
      const bool has1 = t1 < ntile;
      const int c0 = t0 * 16 + li, c1 = t1 * 16 + li;
      const bool in0 = c0 < K, in1 = has1 && c1 < K;
      floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      for (int n0 = 0; n0 < N; n0 += 16) {
        float av[4], b0[4], b1[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int n = n0 + 4 * lk + s;
          const bool nin = n < N;
          av[s] = nin ? cur[li * ld + n] : 0.f;
          b0[s] = (nin && in0) ? W[(int64_t)n * K + c0] : 0.f;
          b1[s] = (nin && in1) ? W[(int64_t)n * K + c1] : 0.f;
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) acc0 = mfma4(av[s], b0[s], acc0);
        if (has1) {
#pragma unroll
          for (int s = 0; s < 4; ++s) acc1 = mfma4(av[s], b1[s], acc1);
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h == 1 && !has1) break;
        const int c = h ? c1 : c0;
        if (c >= K) continue;
        const floatx4 acc = h ? acc1 : acc0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 4 * lk + r;
          const int64_t row = r0 + i;
          float g = acc[r];
          if (l > 0) {
            // dropout backward (g * mask * scale) then ReLU backward ([h > 0])
            const bool live = row < B && xs[row * K + c] > 0.f;
            g = live ? g * sc : 0.f;
            if (row < B) gz[row * K + c] = g;
            nxt[i * ldn + c] = g;
          } else if (row < B) {
            if (a.dropout[0]) g = a.mask0[row * K + c] ? g * sc : 0.f;
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
  __shared__ float part[4][64][5];
  __shared__ float bpart[4][16];
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
  // rows of this wave: a quarter of the batch (multiple of 4)
  const int64_t q = ((B + 15) / 16) * 4;
  const int64_t b_lo = wave * q, b_hi = (b_lo + q < B) ? b_lo + q : B;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;
  int64_t b0 = b_lo;
  for (; b0 + 16 <= b_hi; b0 += 16) {     // 16 rows: eight loads in flight, four MFMAs
    float av[4], bv[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int64_t b = b0 + 4 * s + lk;
      av[s] = oin ? gz[b * N + o] : 0.f;
      bv[s] = iin ? xs[b * K + i] : 0.f;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      acc = mfma4(av[s], bv[s], acc);
      bsum += av[s];
    }
  }
  for (; b0 < b_hi; b0 += 4) {
    const int64_t b = b0 + lk;
    const float av = (oin && b < b_hi) ? gz[b * N + o] : 0.f;
    const float bv = (iin && b < b_hi) ? xs[b * K + i] : 0.f;
    acc = mfma4(av, bv, acc);
    bsum += av;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) part[wave][lane][r] = acc[r];
  if (with_bias) {       // the four row phases of column o, in phase order
    float s1 = __shfl(bsum, li + 16, 64), s2 = __shfl(bsum, li + 32, 64),
          s3 = __shfl(bsum, li + 48, 64);
    if (lk == 0) bpart[wave][li] = ((bsum + s1) + s2) + s3;
  }
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = ((part[0][lane][r] + part[1][lane][r]) + part[2][lane][r]) + part[3][lane][r];
      const int oo = ot * 16 + 4 * lk + r;
      if (oo < N && iin) a.dW[l][(int64_t)oo * K + i] = v;
    }
    if (with_bias && lk == 0 && oin)
      a.db[l][o] = ((bpart[0][li] + bpart[1][li]) + bpart[2][li]) + bpart[3][li];
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
  hipLaunchKernelGGL(mlp_bwd_data_kernel, dim3((unsigned)((B + kMlpRows - 1) / kMlpRows)),
                     dim3(kMlpThreads), shm, st, a, dy, B, gx, ldA, ldB);
  int rc = launch_status("mirec_mlp_bwd_f32: data");
  if (rc) return rc;
  hipLaunchKernelGGL(mlp_bwd_weight_kernel, dim3((unsigned)tiles), dim3(kMlpThreads), 0, st, a, B,
                     x, dy);
  return launch_status("mirec_mlp_bwd_f32: weight");
}
