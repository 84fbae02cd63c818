// Batch normalisation (TF 1.12 fused training semantics) as HBM-streaming kernels.
//   forward : per-channel (mean, biased var) from the conv epilogue's tile partials
//             (Chan merge, fixed order), out = act((y-mean)*gamma*rsqrt(var+eps) + beta [+res])
//   backward: dyhat = dz * [z>0]; dgamma = sum dyhat*xhat; dbeta = sum dyhat;
//             dy = gamma*invstd*(dyhat - mean(dyhat) - xhat*mean(dyhat*xhat))
#pragma once
#include "seg_common.h"

#define SEG_BN_EPS 1.001e-5f  // tf.nn.fused_batch_norm clamps 1e-5 up to this

struct BnState {     // per-layer per-step device vectors, each [C]
  float* mean;
  float* invstd;
  float* scale;      // gamma * invstd
  float* var_unb;    // Bessel-corrected batch variance (moving-average input)
  float* sdy;        // backward: mean(dyhat)
  float* sdyx;       // backward: mean(dyhat * xhat)
};

struct BnApplyArgs {
  const void* y; int ldy;          // conv output (T)
  long M; int C;
  const float* mean; const float* scale; const float* beta;
  int relu;
  // residual 1: plain tensor (T) with optional spatial subsampling (stride rs over an
  // [N][Hr][Wr] grid; the output grid is [N][Ho][Wo])
  const void* res; int ldres; int rs; int Ho, Wo, Hr, Wr;
  // residual 2: second BN (shortcut conv): (y2-mean2)*scale2+beta2
  const void* y2; int ldy2; const float* mean2; const float* scale2; const float* beta2;
  void* out; int ldo;              // output (T or f32)
  uint8_t* mask;                   // optional ReLU bits of out: [M][C/8], bit e = out[c0+e] > 0
};

struct BnBwdArgs {
  const void* dz; int lddz;        // incoming gradient (T or f32)
  const void* z; int ldz;          // activation whose >0 mask gates dz (nullable)
  const uint8_t* mask;             // the same gate as bits [M][C/8] (preferred over z when set)
  const void* y; int ldy;          // conv output (T)
  long M; int C;
  const float* mean; const float* invstd; const float* scale;
  const float* sdy; const float* sdyx;   // apply: means from finalize
  void* dy; int lddy;              // output gradient wrt y (T)
  void* dyhat; int lddyhat;        // optional masked gradient (T)
  const float* dzscale;            // optional per-channel factor applied to dz
  // optional per-channel term added to dz before the gate (8-wide masked path only): the
  // constant part of a data gradient whose producer left it out (net.cpp, linear BN-backward
  // fold of the consumer's expansion conv)
  const float* dshift;
  int reduce_dyhat;                // the reduce (not the apply) stores the gated gradient in dyhat
  // optional (8-wide masked reduce with dshift): per row block column sums of the forward
  // output relu((y - mean) * scale + beta) rounded to T as the forward BN apply stored it,
  // recomputed from y, [rb][C] (the linear BN-backward fold's colsum of the next conv's input)
  const float* beta;
  float* cs_part;
  float* part;                     // reduce partials [rb][C][2]
  int rb;                          // number of row blocks
  // dual (launch_bn_bwd_*_dual): a second BN layer gated by the same dz and bits, e.g. a
  // projection unit's conv3 and shortcut BN; dz and the bits are read once for both
  const void* y2; int ldy2;
  const float* mean2; const float* invstd2; const float* scale2;
  const float* sdy2; const float* sdyx2;
  void* dy2; int lddy2;
  float* part2;
};

// pack (nullable, [2C]): also writes [mean | E[x^2]] for a cross-replica exchange
hipError_t launch_bn_stats_finalize(const float* tile_part, long M, int C, int tile_rows,
                                    float* scratch, const float* gamma, BnState st,
                                    hipStream_t s, float* pack = nullptr);
// cross-replica BN: the replica-summed pack -> global mean / biased variance in st
hipError_t launch_bn_sync_unpack(const float* pack, int C, float inv_world, const float* gamma,
                                 BnState st, hipStream_t s);
// inference mode, every layer in one launch (one workgroup per job)
struct BnInferJob { const float* mov_mean; const float* mov_var; const float* gamma; BnState st; int C; };
hipError_t launch_bn_infer_finalize_all(const BnInferJob* jobs, int n, hipStream_t s);
// inference mode: st from the moving statistics (no batch statistics)
hipError_t launch_bn_infer_finalize(const float* mov_mean, const float* mov_var, int C,
                                    const float* gamma, BnState st, hipStream_t s);
hipError_t launch_bn_apply(int dtype, int out_f32, const BnApplyArgs& a, hipStream_t s);
int bn_bwd_rowblocks(long M, int C);
hipError_t launch_bn_bwd_reduce(int dtype, int dz_f32, const BnBwdArgs& a, hipStream_t s);
// frozen: is_training=False statistics (moving averages): the batch means do not depend on
// the input, so sdy = sdyx = 0 and dy = gamma * invstd * dyhat (FusedBatchNormGrad, inference)
hipError_t launch_bn_bwd_finalize(const float* part, int rb, long M, int C, BnState st,
                                  float* dgamma, float* dbeta, hipStream_t s, int frozen = 0);
hipError_t launch_bn_bwd_apply(int dtype, int dz_f32, const BnBwdArgs& a, hipStream_t s);
// dual forms (16-bit or fp32 dz of the storage type, ReLU bits, no dzscale / dyhat)
hipError_t launch_bn_bwd_reduce_dual(int dtype, const BnBwdArgs& a, hipStream_t s);
hipError_t launch_bn_bwd_apply_dual(int dtype, const BnBwdArgs& a, hipStream_t s);
hipError_t launch_moving_update(float* mov_mean, float* mov_var, const float* bmean,
                                const float* bvar, int n, float decay, hipStream_t s);
