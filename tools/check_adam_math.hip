// Checks the fast-path sqrt / division of the Adam replay (csrc/adam_math.h)
// against the library sqrtf and IEEE division on the GPU:
//  * sqrt: EVERY float in [2^-96, FLT_MAX] (exhaustive);
//  * division: 2^34 pseudo-random (a, b) pairs inside the fast range (|a| in
//    [2^-60, 2^40], b in [2^-40, 2^40]), log-uniform exponents, uniform
//    mantissas, plus pairs whose b or a sits on a binade edge.
// Bitwise comparison; prints mismatch counts and exits non-zero on any.
//   hipcc -O3 --offload-arch=gfx950 -I recbole_amd/csrc tools/check_adam_math.hip -o /tmp/chk
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "adam_math.h"

using namespace mirec;

__global__ void sqrt_all(uint32_t lo, uint64_t n, unsigned long long* bad, uint32_t* first) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t u = lo + (uint32_t)i;
    const float x = __uint_as_float(u);
    if (!sqrt_fast_ok(x)) continue;
    const float a = sqrt_rn_normal(x), b = sqrtf(x);
    if (__float_as_uint(a) != __float_as_uint(b)) {
      atomicAdd(bad, 1ull);
      atomicMin(first, u);
    }
  }
}

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float make(uint64_t r, int elo, int ehi, int edge) {
  const int e = elo + (int)((r >> 32) % (uint64_t)(ehi - elo));
  uint32_t mant = (uint32_t)r & 0x7fffffu;
  if (edge == 1) mant = 0;                 // power of two
  if (edge == 2) mant = 0x7fffffu;         // just below the next power of two
  if (edge == 3) mant &= 0xffu;            // near a power of two
  return __uint_as_float(((uint32_t)(e + 127) << 23) | mant);
}

__global__ void div_rand(uint64_t seed, uint64_t n, unsigned long long* bad, unsigned long long* tested,
                         float* ex) {
  unsigned long long cnt = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r1 = mix(seed ^ (2 * i)), r2 = mix(seed ^ (2 * i + 1));
    const int edge = (int)(r2 & 15);
    float a = make(r1, -60, 40, edge == 4 ? 1 : edge == 5 ? 2 : edge == 6 ? 3 : 0);
    float b = make(r2, -40, 40, edge == 7 ? 1 : edge == 8 ? 2 : edge == 9 ? 3 : 0);
    if (r1 & 1) a = -a;
    if (!div_fast_ok(a, b)) continue;
    ++cnt;
    const float q1 = div_rn_normal(a, b), q2 = a / b;
    if (__float_as_uint(q1) != __float_as_uint(q2)) {
      atomicAdd(bad, 1ull);
      ex[0] = a; ex[1] = b;
    }
  }
  atomicAdd(tested, cnt);
}

int main() {
  unsigned long long* d;
  uint32_t* first;
  float* ex;
  hipMalloc(&d, 4 * sizeof(unsigned long long));
  hipMalloc(&first, 4);
  hipMalloc(&ex, 8);
  hipMemset(d, 0, 4 * sizeof(unsigned long long));
  hipMemset(first, 0xff, 4);
  const uint32_t lo = 0x0f800000u;          // 2^-96
  const uint32_t hi = 0x7f7fffffu;          // FLT_MAX
  hipLaunchKernelGGL(sqrt_all, dim3(8192), dim3(256), 0, 0, lo, (uint64_t)(hi - lo) + 1, d, first);
  const uint64_t n = 1ull << 34;
  hipLaunchKernelGGL(div_rand, dim3(16384), dim3(256), 0, 0, 12345ull, n, d + 1, d + 2, ex);
  hipDeviceSynchronize();
  unsigned long long h[4];
  uint32_t f;
  float e[2];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  hipMemcpy(&f, first, 4, hipMemcpyDeviceToHost);
  hipMemcpy(e, ex, 8, hipMemcpyDeviceToHost);
  printf("sqrt: %u values checked, %llu mismatches (first 0x%08x)\n", hi - lo + 1, h[0], f);
  printf("div: %llu pairs checked, %llu mismatches", h[2], h[1]);
  if (h[1]) printf(" (e.g. %a / %a)", e[0], e[1]);
  printf("\n");
  return (h[0] || h[1]) ? 1 : 0;
}
