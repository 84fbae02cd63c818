// Linear BN-backward fold for expansion 1 x 1 convolutions (net.cpp, unit_backward).
//
// The training BN backward of a bottleneck's conv3 (reference: slim BN as normalizer_fn,
// models/resnet50_extended_model_hierarchical.py:298-339; the gradient TF derives for
// FusedBatchNorm) is, per channel c of the conv output z3 (x-hat = (z3 - mean) * invstd):
//   dz3 = A_c dyhat + B_c + D_c z3,   A = gamma * invstd,   D = -A * mean(dyhat * x-hat) * invstd,
//   B = -A * mean(dyhat) - D * mean
// (dyhat = the ReLU-gated output gradient). It is affine in (dyhat, z3), and z3 = y2 W3^T is
// itself linear in the conv input y2, so the two consumers of dz3 need neither dz3 nor z3:
//   data gradient   dy2 = dz3 W3 = dyhat (A o W3) + y2 H + b,   H = W3^T diag(D) W3 [ci x ci],
//                                                                b = B W3 [ci]
//   weight gradient dW3 = dz3^T y2 = A o (dyhat^T y2) + B (x) colsum(y2) + D o (W3 G),
//                                                                G = y2^T y2 [ci x ci]
// With ci = co / 4 the data gradient becomes one K-concatenated GEMM of K = co + ci (+25 %) and
// the separate BN-backward apply pass over dz3 (read dyhat, z3, bits; write dz3: 6 B per
// element) disappears. The constant b is added by the next BN backward (BnBwdArgs::dshift).
#pragma once
#include "seg_common.h"

struct LbfPrepArgs {
  int co, ci;
  const float* mean; const float* invstd; const float* scale; const float* sdy; const float* sdyx;
  const void* w;    // W3 as the forward ran it: 16-bit [co][ci]
  const void* wt;   // its transpose (data-gradient weights): 16-bit [ci][co]
  void* wts;        // out: [ci][co] 16-bit, A_c * wt[k][c]
  void* xd;         // out: [co][ci] 16-bit, D_c * w[c][k] (the H product's first operand)
  float* bpart;     // out: [co / 128][ci] partial sums over 128-channel chunks of B_c w[c][k]
  float* coef;      // out: [3][co] = A, B, D
};

struct LbfCombineArgs {
  int co, ci;
  const void* w;        // W3, 16-bit [co][ci]
  const float* g;       // [ci][ci] Gram matrix y2^T y2
  const float* p1;      // [co][ci] dyhat^T y2
  const float* cspart;  // [rb][ci] column-sum partials of y2 (the unit's conv2 BN-backward reduce,
                        // BnBwdArgs::cs_part)
  int rb;
  const float* coef;    // [3][co] = A, B, D
  float* out;           // [co][ci] weight gradient (fp32)
};

hipError_t launch_lbf_prep(int dtype, const LbfPrepArgs& a, hipStream_t s);
// h[i] = sum_s slab[s * n + i] rounded to the 16-bit type (fixed split order); bias[k] = sum over
// the co / 128 chunk partials of the prep (fixed order)
hipError_t launch_lbf_hreduce(int dtype, const float* slab, int splits, long n, void* h,
                              const float* bpart, int nbp, int ci, float* bias, hipStream_t s);
hipError_t launch_lbf_combine(int dtype, const LbfCombineArgs& a, hipStream_t s);
