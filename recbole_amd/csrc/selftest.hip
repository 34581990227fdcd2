// Built-in self-test of the K5 fast paths (csrc/adam_math.h + the replay's
// increment): the fast correctly rounded sqrt and division used by the deferred
// Adam replay against the library sqrtf / IEEE division, bit for bit, on the GPU
// that runs them. The exhaustive / 2^34-pair version is tools/check_adam_math.hip;
// this entry point runs a sampled subset fast enough for the -m gpu test suite.
#include "common.h"
#include "adam_math.h"

#pragma clang fp contract(off)

namespace mirec {

// sqrt: every `stride`-th float of [2^-96, FLT_MAX], plus every float within 64
// ulps of each power of two in the range (binade edges).
__global__ __launch_bounds__(256) void selftest_sqrt(uint64_t stride,
                                                     unsigned long long* __restrict__ out) {
  const uint32_t lo = 0x0f800000u, hi = 0x7f7fffffu;
  const uint64_t n_stride = ((uint64_t)(hi - lo)) / stride + 1;
  const uint64_t n_edge = (uint64_t)(254 - 31) * 128;          // exponents 31..254, +-64 ulps
  unsigned long long bad = 0, tested = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_stride + n_edge;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t u;
    if (i < n_stride) {
      u = lo + (uint32_t)(i * stride);
    } else {
      const uint64_t e = i - n_stride;
      const uint32_t p2 = (uint32_t)(31 + e / 128) << 23;
      u = p2 + (uint32_t)(e % 128) - 64u;
    }
    const float x = __uint_as_float(u);
    if (!sqrt_fast_ok(x)) continue;
    ++tested;
    if (__float_as_uint(sqrt_rn_normal(x)) != __float_as_uint(sqrtf(x))) ++bad;
  }
  atomicAdd(&out[0], bad);
  atomicAdd(&out[1], tested);
}

__device__ __forceinline__ uint64_t st_mix(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float st_make(uint64_t r, int elo, int ehi, int edge) {
  const int e = elo + (int)((r >> 32) % (uint64_t)(ehi - elo));
  uint32_t mant = (uint32_t)r & 0x7fffffu;
  if (edge == 1) mant = 0;
  if (edge == 2) mant = 0x7fffffu;
  if (edge == 3) mant &= 0xffu;
  return __uint_as_float(((uint32_t)(e + 127) << 23) | mant);
}

// division: n pseudo-random pairs of the fast range (log-uniform exponents,
// binade-edge mantissas one time in four)
__global__ __launch_bounds__(256) void selftest_div(uint64_t seed, uint64_t n,
                                                    unsigned long long* __restrict__ out) {
  unsigned long long bad = 0, tested = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r1 = st_mix(seed ^ (2 * i)), r2 = st_mix(seed ^ (2 * i + 1));
    const int edge = (int)(r2 & 15);
    float a = st_make(r1, -60, 40, edge == 4 ? 1 : edge == 5 ? 2 : edge == 6 ? 3 : 0);
    const float b = st_make(r2, -40, 40, edge == 7 ? 1 : edge == 8 ? 2 : edge == 9 ? 3 : 0);
    if (r1 & 1) a = -a;
    if (!div_fast_ok(a, b)) continue;
    ++tested;
    if (__float_as_uint(div_rn_normal(a, b)) != __float_as_uint(a / b)) ++bad;
  }
  atomicAdd(&out[2], bad);
  atomicAdd(&out[3], tested);
}

}  // namespace mirec

extern "C" int mirec_selftest_adam_math(uint64_t sqrt_stride, uint64_t n_div, uint64_t seed,
                                        unsigned long long* out4_dev, void* stream) {
  if (!out4_dev || sqrt_stride == 0) {
    mirec::set_error("mirec_selftest_adam_math: bad arguments");
    return -1;
  }
  hipStream_t st = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(out4_dev, 0, 4 * sizeof(unsigned long long), st);
  if (e != hipSuccess) return mirec::hip_status(e, "mirec_selftest_adam_math: memset");
  hipLaunchKernelGGL(mirec::selftest_sqrt, dim3(4096), dim3(256), 0, st, sqrt_stride, out4_dev);
  hipLaunchKernelGGL(mirec::selftest_div, dim3(4096), dim3(256), 0, st, seed, n_div, out4_dev);
  return mirec::launch_status("mirec_selftest_adam_math");
}
