// Arithmetic of the BPR step shared by K3 (bpr.hip) and the fused step kernel
// (step.hip): the two form the same scores, coefficients, losses and gradient
// contributions bit for bit. Every operation is written out — fmaf where one is
// wanted, contraction off elsewhere — so no compiler fusing decision can differ
// between the kernels that inline these functions.
//
// Restates BPR.calculate_loss (recbole/model/general_recommender/bpr.py:74-83) and
// BPRLoss (recbole/model/loss.py:43-49) with torch's backward op order:
//   x = s+ - s-;  s = sigmoid(x);  loss term = -log(gamma + s)
//   g = -(1/R) / (gamma + s);  dx = g * (1 - s) * s      (d loss / d x)
//   du += dx*p - dx*n,  dp += dx*u,  dn = -dx*u
#pragma once
#include "common.h"

namespace mirec {

// <a, b> of one float4 lane slice: x*x + three fused steps
__device__ __forceinline__ float dot4(const float4& a, const float4& b) {
  return fmaf(a.w, b.w, fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)));
}

template <int CTRL>
__device__ __forceinline__ float dpp_f32(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xf, 0xf, false));
}

// Sum over the LPR lanes of an aligned lane group; every lane gets the same bits. A
// butterfly pairing lanes i, i^1, then i^2, ... : xor 1 and 2 are DPP quad permutations,
// xor 4 and 8 the DPP half-row / row mirrors (after the quad steps every lane of a quad
// holds the quad sum, so pairing i with 7 - i, then with 15 - i, adds the same values as
// i^4, i^8), xor 16 a swizzle inside 32 lanes and xor 32 one bpermute: four VALU-latency
// steps instead of ds_bpermute round trips. a + b = b + a exactly, so both partners agree.
template <int LPR>
__device__ __forceinline__ float group_sum(float x) {
  static_assert(LPR >= 1 && LPR <= 64 && (LPR & (LPR - 1)) == 0, "LPR: a power of two <= 64");
  if (LPR >= 2) x += dpp_f32<0xB1>(x);     // quad_perm [1,0,3,2]
  if (LPR >= 4) x += dpp_f32<0x4E>(x);     // quad_perm [2,3,0,1]
  if (LPR >= 8) x += dpp_f32<0x141>(x);    // row_half_mirror
  if (LPR >= 16) x += dpp_f32<0x140>(x);   // row_mirror
  if (LPR >= 32) x += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(x), 0x401F));
  if (LPR >= 64) x += __shfl_xor(x, 32, 64);
  return x;
}

struct BprCoef {
  float dx;    // d loss / d (pos_score - neg_score), scaled by -ng = 1/R
  float nll;   // -log(gamma + sigmoid(x)), this row's loss term (before the mean)
};

__device__ __forceinline__ BprCoef bpr_coef(float sp, float sn, float gamma, float ng) {
#pragma clang fp contract(off)
  const float x = sp - sn;
  const float s = 1.f / (1.f + expf(-x));
  const float gs = gamma + s;
  const float gg = ng / gs;
  return {(gg * (1.f - s)) * s, -logf(gs)};
}

// the three gradient contributions of one (positive, negative) row, each product and
// sum rounded on its own; gu / gp accumulate over the rows of a positive (j order)
__device__ __forceinline__ void contrib_u(float4& gu, float dx, const float4& p,
                                          const float4& n) {
#pragma clang fp contract(off)
  gu.x += dx * p.x - dx * n.x;
  gu.y += dx * p.y - dx * n.y;
  gu.z += dx * p.z - dx * n.z;
  gu.w += dx * p.w - dx * n.w;
}
__device__ __forceinline__ void contrib_p(float4& gp, float dx, const float4& u) {
#pragma clang fp contract(off)
  gp.x += dx * u.x;
  gp.y += dx * u.y;
  gp.z += dx * u.z;
  gp.w += dx * u.w;
}
__device__ __forceinline__ float4 contrib_n(float dx, const float4& u) {
#pragma clang fp contract(off)
  return make_float4(-dx * u.x, -dx * u.y, -dx * u.z, -dx * u.w);
}

__device__ __forceinline__ void pair_contrib(float4& gu, float4& gp, float4& gn, float dx,
                                             const float4& u, const float4& p,
                                             const float4& n) {
  contrib_u(gu, dx, p, n);
  contrib_p(gp, dx, u);
  gn = contrib_n(dx, u);
}

}  // namespace mirec
