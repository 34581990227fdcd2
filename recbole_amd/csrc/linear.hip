// K11 — the Linear layers of SASRec's transformer blocks (reference layers.py:338-461:
// MultiHeadAttention's query / key / value / dense and FeedForward's dense_1 / dense_2,
// nn.Linear over B x L = 10^5 rows of width 64..256) on fp32 MFMA, forward
// Y = X W^T + b and the data gradient dX = dY W. The library GEMMs ran these tall, narrow
// products at ~0.25 of the fp32 MFMA peak (tiles of 128 x 32 with most of each workgroup's
// time in its prologue); here a workgroup keeps the weight in LDS:
//
//   * the whole weight staged once per workgroup as Bs[n][k] (the B operand's column n
//     along k, row stride K + 4 floats; W itself for the forward, W transposed for dX);
//     one or two persistent workgroups per CU (the slice fits once or twice in LDS);
//   * eight waves, each walking 16-row slabs on its own (no barrier after the staging),
//     A rows straight from global memory in the 16x16x4 MFMA's A layout, the next slab's
//     loaded while the current slab's products run;
//   * per 16-wide k slice: the B float4 of four 16-column tiles from LDS, 16 MFMAs with the
//     four accumulators interleaved; bias in the epilogue.
// The weight gradient (dW = dY^T X over the 10^5 rows) stays the split-K batched product
// + mirec_linear_grad_finish_f32.
#include "common.h"

#include <algorithm>

namespace mirec {

typedef float floatx4 __attribute__((ext_vector_type(4)));

#ifndef MIREC_LN_GW
#define MIREC_LN_GW 4
#endif
constexpr int kLnThreads = 512;           // eight waves
constexpr int kLnWaves = kLnThreads / 64;

__device__ __forceinline__ floatx4 ln_mfma(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Y[M, N] = X[M, K] B[K, N] (+ bias), B[k][n] = WT ? W[k][n] : W[n][k] (W row-major). One
// workgroup per CU stages the whole weight once; each of its waves then walks 16-row slabs
// s = its global wave index + i * (waves in the grid), the next slab's A rows loaded while
// the current slab's products run (no workgroup barrier after the staging).
template <int K, int N, bool WT, bool ACC>
__global__ __launch_bounds__(kLnThreads) void linear_mfma_kernel(
    const float* __restrict__ X, int64_t M, const float* __restrict__ W,
    const float* __restrict__ bias, const float* __restrict__ R, float* __restrict__ Y) {
  // ACC: Y = R + X B. R may be Y (in place): each element is read once and then written
  // once by the same lane, so no other access depends on their order (the restrict
  // qualifiers keep the epilogue's loads batched: without them 48.6 -> 78 us)
  constexpr int KP = K + 4;               // LDS row stride (floats)
  constexpr int NU = K / 16;              // 16-wide k slices
  constexpr int NC = N / 16;              // 16-wide column tiles
  extern __shared__ __attribute__((aligned(16))) float Bs[];   // [N][KP], float4-aligned
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, lk = lane >> 4;
  const int64_t slabs = (M + 15) / 16;
  const int64_t nw = (int64_t)gridDim.x * kLnWaves;
  int64_t s = (int64_t)blockIdx.x * kLnWaves + w;
  // lane (li, lk) holds row 16 s + li, floats 16u + 4lk .. +3 of slab s
  auto load_a = [&](float4 (&a)[NU], int64_t ss) {
    const int64_t r = 16 * ss + li;
    const bool ok = ss < slabs && r < M;
    const float* src = X + (ok ? r : 0) * K + 4 * lk;
#pragma unroll
    for (int u = 0; u < NU; ++u)
      a[u] = ok ? *reinterpret_cast<const float4*>(src + 16 * u) : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  float4 a[NU];
  load_a(a, s);                           // in flight with the staging

  // ---- the weight into LDS as Bs[n][k]
  if (!WT) {                              // W [N][K]: row n of W is Bs row n
    for (int e = tid; e < N * K / 4; e += kLnThreads) {
      const int n = e / (K / 4), k4 = (e % (K / 4)) * 4;
      *reinterpret_cast<float4*>(&Bs[n * KP + k4]) =
          *reinterpret_cast<const float4*>(W + (int64_t)n * K + k4);
    }
  } else {                                // W [K][N]: Bs[n][k] = W[k][n]
    for (int e = tid; e < N * K / 4; e += kLnThreads) {
      const int k = e / (N / 4), n4 = (e % (N / 4)) * 4;
      const float4 x = *reinterpret_cast<const float4*>(W + (int64_t)k * N + n4);
      Bs[(n4 + 0) * KP + k] = x.x;
      Bs[(n4 + 1) * KP + k] = x.y;
      Bs[(n4 + 2) * KP + k] = x.z;
      Bs[(n4 + 3) * KP + k] = x.w;
    }
  }
  float bv[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) bv[c] = bias ? bias[16 * c + li] : 0.f;
  __syncthreads();

  for (; s < slabs; s += nw) {
    constexpr bool kPre = NU <= 8 && NC <= 8;   // K or N = 256: no room for a second A slab
    float4 an[kPre ? NU : 1];
    if (kPre) load_a(reinterpret_cast<float4(&)[NU]>(an), s + nw);   // next slab, in flight
    floatx4 acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = floatx4{0.f, 0.f, 0.f, 0.f};
    // groups g = (k slice u, GW column tiles cg..): the next group's B reads are issued
    // before this group's MFMAs (their LDS latency under the products); GW accumulators
    // interleaved, so a dependent MFMA follows its predecessor GW issues later
    constexpr int GW = NC < MIREC_LN_GW ? NC : MIREC_LN_GW;
    constexpr int NG = NU * (NC / GW);
    auto load_b = [&](float4 (&b)[GW], int g) {
      const int u = g / (NC / GW), cg = GW * (g % (NC / GW));
#pragma unroll
      for (int c = 0; c < GW; ++c)
        b[c] = *reinterpret_cast<const float4*>(&Bs[(16 * (cg + c) + li) * KP + 16 * u + 4 * lk]);
    };
    float4 bc[GW];
    load_b(bc, 0);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int u = g / (NC / GW), cg = GW * (g % (NC / GW));
      float4 bn[GW];
      if (g + 1 < NG) load_b(bn, g + 1);
      __builtin_amdgcn_sched_barrier(0);   // the reads stay ahead of this group's MFMAs
#pragma unroll
      for (int c = 0; c < GW; ++c) acc[cg + c] = ln_mfma(a[u].x, bc[c].x, acc[cg + c]);
#pragma unroll
      for (int c = 0; c < GW; ++c) acc[cg + c] = ln_mfma(a[u].y, bc[c].y, acc[cg + c]);
#pragma unroll
      for (int c = 0; c < GW; ++c) acc[cg + c] = ln_mfma(a[u].z, bc[c].z, acc[cg + c]);
#pragma unroll
      for (int c = 0; c < GW; ++c) acc[cg + c] = ln_mfma(a[u].w, bc[c].w, acc[cg + c]);
      // the scheduler keeps this order (no hoisting of later groups' reads)
      __builtin_amdgcn_sched_barrier(0);
      if (g + 1 < NG)
#pragma unroll
        for (int c = 0; c < GW; ++c) bc[c] = bn[c];
    }
    // C layout: acc[c][i] = Y[16 s + 4lk + i][16c + li]
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t r = 16 * s + 4 * lk + i;
      if (r < M)
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int64_t o = r * N + 16 * c + li;
          Y[o] = ACC ? R[o] + (acc[c][i] + bv[c]) : acc[c][i] + bv[c];
        }
    }
    if (kPre) {
#pragma unroll
      for (int u = 0; u < NU; ++u) a[u] = an[kPre ? u : 0];
    } else if (s + nw < slabs) {
      load_a(a, s + nw);
    }
  }
}

template <int K, int N, bool WT, bool ACC>
int launch_linear(const float* X, int64_t M, const float* W, const float* bias, const float* R,
                  float* Y, hipStream_t st, const char* what) {
  constexpr size_t lds = (size_t)N * (K + 4) * sizeof(float);
  static bool attr = false;
  if (!attr) {
    if (hip_status(hipFuncSetAttribute((const void*)linear_mfma_kernel<K, N, WT, ACC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                   what))
      return -1;
    attr = true;
  }
  const int per_cu = 1;   // eight waves per CU (the VGPR budget of the wider forms: 2 per SIMD)
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  }
  const int64_t slabs = (M + 15) / 16;
  const int64_t grid = std::min<int64_t>((slabs + kLnWaves - 1) / kLnWaves, (int64_t)cus * per_cu);
  hipLaunchKernelGGL((linear_mfma_kernel<K, N, WT, ACC>), dim3((unsigned)grid), dim3(kLnThreads),
                     lds, st, X, M, W, bias, R, Y);
  return launch_status(what);
}

template <bool WT>
int linear_dispatch(const float* X, int64_t M, int K, int N, const float* W, const float* bias,
                    const float* R, float* Y, hipStream_t st, const char* what) {
#define MIREC_LN(KK, NN) \
  if (K == KK && N == NN)                                                                    \
    return R ? launch_linear<KK, NN, WT, WT>(X, M, W, bias, R, Y, st, what)                  \
             : launch_linear<KK, NN, WT, false>(X, M, W, bias, nullptr, Y, st, what);
  MIREC_LN(64, 64)
  MIREC_LN(64, 128)
  MIREC_LN(64, 256)
  MIREC_LN(128, 64)
  MIREC_LN(128, 128)
  MIREC_LN(128, 256)
  MIREC_LN(256, 64)
  MIREC_LN(256, 128)
#undef MIREC_LN
  set_error("%s: widths K=%d N=%d not in the built set ({64,128,256}^2 minus 256 x 256)", what, K,
            N);
  return -1;
}

}  // namespace mirec

using namespace mirec;

extern "C" int mirec_linear_shape_ok(int32_t K, int32_t N) {
  const bool k = K == 64 || K == 128 || K == 256, n = N == 64 || N == 128 || N == 256;
  return k && n && !(K == 256 && N == 256);
}

extern "C" int mirec_linear_fwd_f32(const float* x, int64_t M, int32_t K, int32_t N,
                                    const float* w, const float* bias, float* y, void* stream) {
  if (M < 0 || !x || !w || !y || (((uintptr_t)x | (uintptr_t)w) & 15)) {
    set_error("mirec_linear_fwd_f32: bad arguments (16-byte aligned x, w)");
    return -1;
  }
  if (M == 0) return 0;
  return linear_dispatch<false>(x, M, K, N, w, bias, nullptr, y, (hipStream_t)stream,
                                "mirec_linear_fwd_f32");
}

extern "C" int mirec_linear_bwd_data_f32(const float* gy, int64_t M, int32_t n_out,
                                         int32_t n_in, const float* w, float* gx,
                                         int32_t accumulate, void* stream) {
  if (M < 0 || !gy || !w || !gx || (((uintptr_t)gy | (uintptr_t)w) & 15)) {
    set_error("mirec_linear_bwd_data_f32: bad arguments (16-byte aligned gy, w)");
    return -1;
  }
  if (M == 0) return 0;
  // dX[M, n_in] = dY[M, n_out] W[n_out, n_in]: reduction n_out, B[k][n] = W[k][n]
  return linear_dispatch<true>(gy, M, n_out, n_in, w, nullptr, accumulate ? gx : nullptr, gx,
                               (hipStream_t)stream, "mirec_linear_bwd_data_f32");
}

extern "C" int mirec_linear_bwd_data_acc_f32(const float* gy, int64_t M, int32_t n_out,
                                             int32_t n_in, const float* w, const float* acc,
                                             float* gx, void* stream) {
  if (M < 0 || !gy || !w || !gx || !acc || (((uintptr_t)gy | (uintptr_t)w) & 15)) {
    set_error("mirec_linear_bwd_data_acc_f32: bad arguments (16-byte aligned gy, w; acc)");
    return -1;
  }
  if (M == 0) return 0;
  // dX = acc + dY W, into gx (acc == gx: in place, as mirec_linear_bwd_data_f32 accumulating)
  return linear_dispatch<true>(gy, M, n_out, n_in, w, nullptr, acc, gx, (hipStream_t)stream,
                               "mirec_linear_bwd_data_acc_f32");
}
