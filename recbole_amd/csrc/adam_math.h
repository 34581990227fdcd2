// Fast-path correctly rounded sqrt and division for the Adam replay (adam.hip),
// shared with the exhaustive / randomized checker tools/check_adam_math.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace mirec {

// sqrtf and IEEE division as the compiler expands them, minus the parts that are
// identities on the ranges tested before use: sqrt_rn_normal drops the
// small-input scaling and the 0 / inf fix-up of the correctly rounded sqrt
// expansion (both select the unscaled value on [2^-96, FLT_MAX]); div_rn_normal
// is the refinement sequence of the correctly rounded division expansion
// without v_div_scale / v_div_fmas scaling and v_div_fixup, which are no-ops
// when numerator, denominator, reciprocal and quotient are normal with exponent
// difference < 96 (|a| in [2^-60, 2^40], b in [2^-40, 2^40]). Any lane outside
// its range sends the wave down the library path, so the results are those of
// sqrtf and / everywhere (tools/check_adam_math.hip checks both on the GPU).
__device__ __forceinline__ float sqrt_rn_normal(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sd = __uint_as_float(__float_as_uint(s) - 1u);
  const float su = __uint_as_float(__float_as_uint(s) + 1u);
  const float rd = fmaf(-sd, s, x);
  const float ru = fmaf(-su, s, x);
  const float r = rd <= 0.f ? sd : s;
  return ru > 0.f ? su : r;
}

__device__ __forceinline__ bool sqrt_fast_ok(float x) {
  return x >= 0x1p-96f && x <= 0x1.fffffep127f;
}

__device__ __forceinline__ float div_rn_normal(float a, float b) {
  const float y0 = __builtin_amdgcn_rcpf(b);
  const float e = fmaf(-b, y0, 1.0f);
  const float y = fmaf(e, y0, y0);
  const float q0 = a * y;
  const float r0 = fmaf(-b, q0, a);
  const float q1 = fmaf(r0, y, q0);
  const float r1 = fmaf(-b, q1, a);
  return fmaf(r1, y, q1);
}

__device__ __forceinline__ bool div_fast_ok(float a, float b) {
  const float aa = fabsf(a);
  return aa >= 0x1p-60f && aa <= 0x1p40f && b >= 0x1p-40f && b <= 0x1p40f;
}

}  // namespace mirec
