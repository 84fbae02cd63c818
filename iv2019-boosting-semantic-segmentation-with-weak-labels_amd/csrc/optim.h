// Fused optimizer update: L2 regulariser gradient + MomentumOptimizer + optional EMA shadow
// + refresh of the compute-dtype (bf16 / fp16) weight copy, and the regularisation loss value;
// a device flag (non-finite loss-scaled gradients, fp16) skips the update of the step.
#pragma once
#include "seg_common.h"

struct SgdmArgs {
  float* w;            // fp32 master weights
  const float* g;      // gradient of the segmentation loss (already all-reduced / averaged)
  float* v;            // momentum accumulator
  float* ema;          // optional EMA shadow (nullptr = off)
  void* w_lp;          // optional 16-bit copy to refresh (nullptr = none)
  int lp_f16;          // w_lp is fp16 (else bf16)
  long n;
  float lr, momentum, wd, ema_decay;
  float* reg_part;     // optional [blocks] partial sums of 0.5*wd*w_old^2
  const int* skip;     // optional device flag: != 0 = non-finite gradients, keep the weights
  int nesterov;        // MomentumOptimizer(use_nesterov=True): var -= lr * (g + m * accum)
};

int sgdm_blocks(long n);
hipError_t launch_sgdm(const SgdmArgs& a, hipStream_t s);
hipError_t launch_sum_partials(const float* part, int n, float* out, hipStream_t s);
hipError_t launch_cast_f32_bf16(const float* src, bf16_t* dst, long n, hipStream_t s);
// fp32 -> 16-bit storage of dtype (SEG_BF16 / SEG_F16)
hipError_t launch_cast_f32_half(int dtype, const float* src, void* dst, long n, hipStream_t s);
// flag = 1 if any of x[0..n) is not finite (flag must be zeroed before; benign same-value race)
hipError_t launch_nonfinite(const float* x, long n, int* flag, hipStream_t s);
// x[0..n1) *= f1, x[n1..n1+n2) *= f2
hipError_t launch_scale2(float* x, long n1, float f1, long n2, float f2, hipStream_t s);
hipError_t launch_scale_inplace(float* x, long n, float f, hipStream_t s);
