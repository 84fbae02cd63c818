// Group normalisation (norm_layer='group', hierarchical.py:293-333 -> TF 1.12
// tf.contrib.layers.group_norm): per image n and channel group g, moments over H x W x C/G
// (biased variance, epsilon 1e-5), then out = (x - mean_ng) * rsqrt(var_ng + eps) * gamma_c +
// beta_c. groups = 32 everywhere except the logits convs (softmax_classifier arg scope,
// groups = 1: a layer norm over H x W x C). No moving statistics.
//
// The per-image affine is a per-channel one, so the batch-norm apply / backward streaming
// kernels run per image with per-image BnState vectors (mean, invstd, scale = gamma * invstd);
// these kernels produce those vectors:
//   forward : gn_partial (per image and row chunk, per channel (sum, M2) by an exact two-pass
//             over the chunk) -> gn_stats_final (Chan merge over the group's chunks and
//             channels in fixed order);
//   backward: the batch-norm reduce per image gives S1 = sum dyhat, S2 = sum dyhat * xhat per
//             channel; gn_bwd_final sums them into dbeta / dgamma (fixed image order) and
//             sets sdy = mean_g(gamma S1), sdyx = mean_g(gamma S2) per (image, group), so the
//             batch-norm apply with scale = invstd and the gradient pre-scaled by gamma gives
//             dx = invstd (gamma dyhat - mean_g(gamma dyhat) - xhat mean_g(gamma dyhat xhat)).
#pragma once
#include "bn.h"

#define SEG_GN_EPS 1e-5f   // module_arg_scope norm_epsilon (group_norm_params, :313-317)

struct GnPartArgs {
  const void* y; int ldy;   // conv output, N images of hw rows each
  int N; long hw; int C;
  int chunk;                // rows per chunk; nchunks = ceil(hw / chunk)
  float* part;              // [N][nchunks][C][2] = (sum, M2)
};

int gn_chunks(long hw);
hipError_t launch_gn_partial(int dtype, int y_f32, const GnPartArgs& a, hipStream_t s);
// st: N per-image states (device array of BnState)
hipError_t launch_gn_stats_final(const float* part, int N, long hw, int C, int groups,
                                 const float* gamma, const BnState* st, hipStream_t s);
// part: [N][rb][C][2] reduce partials of the per-image batch-norm reduce
hipError_t launch_gn_bwd_final(const float* part, int N, int rb, long hw, int C, int groups,
                               const float* gamma, const BnState* st, float* dgamma,
                               float* dbeta, hipStream_t s);
// dst[r][c] = src[r][c] * scale[c] (fp32 rows of stride ld, c < C)
hipError_t launch_gn_chscale(const float* src, float* dst, long rows, int ld, int C,
                             const float* scale, hipStream_t s);
