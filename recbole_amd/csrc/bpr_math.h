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

// sum over the LPR lanes of a lane group (xor butterfly: every lane gets the sum)
template <int LPR>
__device__ __forceinline__ float group_sum(float x) {
#pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
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
