// Fused optimizer update: L2 regulariser gradient + MomentumOptimizer + optional EMA shadow
// + refresh of the compute-dtype (bf16) weight copy, and the regularisation loss value.
#pragma once
#include "seg_common.h"

struct SgdmArgs {
  float* w;            // fp32 master weights
  const float* g;      // gradient of the segmentation loss (already all-reduced / averaged)
  float* v;            // momentum accumulator
  float* ema;          // optional EMA shadow (nullptr = off)
  bf16_t* w_lp;        // optional bf16 copy to refresh (nullptr = none)
  long n;
  float lr, momentum, wd, ema_decay;
  float* reg_part;     // optional [blocks] partial sums of 0.5*wd*w_old^2
};

int sgdm_blocks(long n);
hipError_t launch_sgdm(const SgdmArgs& a, hipStream_t s);
hipError_t launch_sum_partials(const float* part, int n, float* out, hipStream_t s);
hipError_t launch_cast_f32_bf16(const float* src, bf16_t* dst, long n, hipStream_t s);
hipError_t launch_scale_inplace(float* x, long n, float f, hipStream_t s);
