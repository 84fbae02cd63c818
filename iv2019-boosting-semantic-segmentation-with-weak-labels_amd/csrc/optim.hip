// Optimizer kernels (see optim.h).
#include "optim.h"

namespace {

constexpr int SG_THREADS = 256;
constexpr int SG_PER_BLOCK = SG_THREADS * 16;

__global__ void sgdm_kernel(SgdmArgs a) {
  const long base = (long)blockIdx.x * SG_PER_BLOCK;
  const bool skip = a.skip && *a.skip;   // dynamic loss scaling: overflowed step
  float reg = 0.f;
  if (base + SG_PER_BLOCK <= a.n && !skip) {
    // whole block: branch-free, so every element's loads are issued ahead of the arithmetic
    // (the bounds check in the general loop serialised one memory latency per element)
    float w_old[16], g[16], v[16], e[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const long i = base + (long)k * SG_THREADS + threadIdx.x;
      w_old[k] = a.w[i];
      g[k] = a.g[i];
      v[k] = a.v[i];
      if (a.ema) e[k] = a.ema[i];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const long i = base + (long)k * SG_THREADS + threadIdx.x;
      reg += w_old[k] * w_old[k];
      const float gt = g[k] + a.wd * w_old[k];
      const float vn = v[k] * a.momentum + gt;
      a.v[i] = vn;
      const float w_new = a.nesterov ? w_old[k] - a.lr * (gt + a.momentum * vn) : w_old[k] - a.lr * vn;
      a.w[i] = w_new;
      if (a.ema) a.ema[i] = e[k] - (1.f - a.ema_decay) * (e[k] - w_old[k]);
      if (a.w_lp) {
        if (a.lp_f16) ((f16_t*)a.w_lp)[i] = (f16_t)w_new;
        else ((bf16_t*)a.w_lp)[i] = f2bf(w_new);
      }
    }
  } else
  for (int k = 0; k < 16; ++k) {
    const long i = base + (long)k * SG_THREADS + threadIdx.x;
    if (i >= a.n) break;
    const float w_old = a.w[i];
    reg += w_old * w_old;
    if (skip) continue;
    // total gradient = d(seg)/dw + d(wd * sum(w^2)/2)/dw
    const float gt = a.g[i] + a.wd * w_old;
    // tf.train.MomentumOptimizer: accum = accum*m + g; var -= lr*accum, or with
    // use_nesterov var -= lr*(g + m*accum) (training_ops ApplyMomentum)
    const float v = a.v[i] * a.momentum + gt;
    a.v[i] = v;
    const float w_new = a.nesterov ? w_old - a.lr * (gt + a.momentum * v) : w_old - a.lr * v;
    a.w[i] = w_new;
    if (a.ema) a.ema[i] -= (1.f - a.ema_decay) * (a.ema[i] - w_old);
    if (a.w_lp) {
      if (a.lp_f16) ((f16_t*)a.w_lp)[i] = (f16_t)w_new;
      else ((bf16_t*)a.w_lp)[i] = f2bf(w_new);
    }
  }
  if (a.reg_part) {
    __shared__ float sh[SG_THREADS / 64];
    float s = wave_sum(reg);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = 0.f;
      for (int q = 0; q < SG_THREADS / 64; ++q) t += sh[q];
      a.reg_part[blockIdx.x] = 0.5f * a.wd * t;
    }
  }
}

__global__ void sum_partials_kernel(const float* __restrict__ p, int n, float* out) {
  __shared__ double sh[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) s += p[i];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) sh[threadIdx.x] += sh[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = (float)sh[0];
}

__global__ void cast_kernel(const float* __restrict__ s, bf16_t* __restrict__ d, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    d[i] = f2bf(s[i]);
}

__global__ void cast_f16_kernel(const float* __restrict__ s, f16_t* __restrict__ d, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    d[i] = (f16_t)s[i];
}

__global__ void nonfinite_kernel(const float* __restrict__ x, long n, int* flag) {
  bool bad = false;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    bad |= !isfinite(x[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) *flag = 1;
}

__global__ void scale2_kernel(float* x, long n1, float f1, long n2, float f2) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n1 + n2; i += (long)gridDim.x * blockDim.x)
    x[i] *= i < n1 ? f1 : f2;
}

__global__ void scale_kernel(float* x, long n, float f) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    x[i] *= f;
}

}  // namespace

int sgdm_blocks(long n) { return ceil_div(n, SG_PER_BLOCK); }

hipError_t launch_sgdm(const SgdmArgs& a, hipStream_t s) {
  if (a.n <= 0) return hipSuccess;
  hipLaunchKernelGGL(sgdm_kernel, dim3(sgdm_blocks(a.n)), dim3(SG_THREADS), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_sum_partials(const float* part, int n, float* out, hipStream_t s) {
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, s, part, n, out);
  return hipGetLastError();
}

hipError_t launch_cast_f32_bf16(const float* src, bf16_t* dst, long n, hipStream_t s) {
  long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(cast_kernel, dim3((int)g), dim3(256), 0, s, src, dst, n);
  return hipGetLastError();
}

hipError_t launch_scale_inplace(float* x, long n, float f, hipStream_t s) {
  long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(scale_kernel, dim3((int)g), dim3(256), 0, s, x, n, f);
  return hipGetLastError();
}

hipError_t launch_cast_f32_half(int dtype, const float* src, void* dst, long n, hipStream_t s) {
  if (dtype != SEG_F16) return launch_cast_f32_bf16(src, (bf16_t*)dst, n, s);
  long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(cast_f16_kernel, dim3((int)(g < 1 ? 1 : g)), dim3(256), 0, s, src, (f16_t*)dst, n);
  return hipGetLastError();
}

hipError_t launch_nonfinite(const float* x, long n, int* flag, hipStream_t s) {
  long g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(nonfinite_kernel, dim3((int)(g < 1 ? 1 : g)), dim3(256), 0, s, x, n, flag);
  return hipGetLastError();
}

hipError_t launch_scale2(float* x, long n1, float f1, long n2, float f2, hipStream_t s) {
  long g = (n1 + n2 + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(scale2_kernel, dim3((int)(g < 1 ? 1 : g)), dim3(256), 0, s, x, n1, f1, n2, f2);
  return hipGetLastError();
}
