// Linear BN-backward fold kernels (see lbf.h). Every sum runs in a fixed order: bitwise
// reproducible run to run.
#include "lbf.h"

namespace {

// dz3 = A dyhat + B + D z3 from the layer's BN state (the apply kernel's formula
// sc * (dyhat - sdy - x-hat * sdyx), x-hat = (z3 - mean) * invstd, expanded)
__device__ __forceinline__ void lbf_coefs(const LbfPrepArgs& a, int c, float& A, float& B, float& D) {
  const float sc = a.scale[c];
  A = sc;
  D = -sc * a.sdyx[c] * a.invstd[c];
  B = -sc * a.sdy[c] - D * a.mean[c];
}

// four roles by block range: the scaled data-gradient weights, the D-scaled forward weights
// (the H product's first operand), the constant b of the data gradient, the coefficient table
template <typename T>
__global__ __launch_bounds__(256) void lbf_prep_kernel(LbfPrepArgs a, int nb_wt, int nb_xd, int nb_b) {
  __shared__ float bsh[2048];
  const int b = blockIdx.x, t = threadIdx.x;
  if (b < nb_wt) {   // wts[k][c] = A_c wt[k][c], 8 output channels c per thread
    const long i = (long)b * 256 + t;
    const int cpr = a.co / 8;
    if (i >= (long)a.ci * cpr) return;
    const int k = (int)(i / cpr), c0 = (int)(i - (long)k * cpr) * 8;
    float v[8];
    Vec8<T>::load((const T*)a.wt + (size_t)k * a.co + c0, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= a.scale[c0 + e];
    Vec8<T>::store((T*)a.wts + (size_t)k * a.co + c0, v);
  } else if (b < nb_wt + nb_xd) {   // xd[c][k] = D_c w[c][k], 8 input channels k per thread
    const long i = (long)(b - nb_wt) * 256 + t;
    const int cpr = a.ci / 8;
    if (i >= (long)a.co * cpr) return;
    const int c = (int)(i / cpr), k0 = (int)(i - (long)c * cpr) * 8;
    float A, B, D;
    lbf_coefs(a, c, A, B, D);
    float v[8];
    Vec8<T>::load((const T*)a.w + (size_t)c * a.ci + k0, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= D;
    Vec8<T>::store((T*)a.xd + (size_t)c * a.ci + k0, v);
  } else if (b < nb_wt + nb_xd + nb_b) {
    // bias partials: block = 64 input channels k x one 128-channel chunk of c, 4 c-lanes per k,
    // lanes combined in order through LDS (the chunks are summed by lbf_hreduce)
    const int nkc = a.ci / 64;
    const int bb = b - nb_wt - nb_xd;
    const int kc = bb % nkc, cc = bb / nkc;
    const int kk = t % 64, cl = t / 64;
    if (t < 128) {
      float A, B, D;
      lbf_coefs(a, cc * 128 + t, A, B, D);
      bsh[t] = B;
    }
    __syncthreads();
    const T* W = (const T*)a.w + (size_t)(cc * 128) * a.ci + kc * 64 + kk;
    float sacc = 0.f;
#pragma unroll 8
    for (int j = 0; j < 32; ++j) {
      const int c = cl + 4 * j;
      sacc = __builtin_fmaf(bsh[c], ldf(W + (size_t)c * a.ci), sacc);
    }
    bsh[128 + t] = sacc;
    __syncthreads();
    if (t < 64)
      a.bpart[(size_t)cc * a.ci + kc * 64 + t] =
          (bsh[128 + t] + bsh[128 + 64 + t]) + (bsh[128 + 128 + t] + bsh[128 + 192 + t]);
  } else {   // coefficient table [3][co]
    const int c = (b - nb_wt - nb_xd - nb_b) * 256 + t;
    if (c >= a.co) return;
    float A, B, D;
    lbf_coefs(a, c, A, B, D);
    a.coef[c] = A;
    a.coef[a.co + c] = B;
    a.coef[2 * a.co + c] = D;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void lbf_hreduce_kernel(const float* __restrict__ slab, int splits, long n,
                                                          T* __restrict__ h, const float* __restrict__ bpart,
                                                          int nbp, int ci, float* __restrict__ bias) {
  const long g = (long)blockIdx.x * 256 + threadIdx.x, stride = (long)gridDim.x * 256;
  for (long i = g; i < n; i += stride) {
    // the splits' loads issued 8 at a time before their (ordered) adds
    float s = 0.f;
    int z = 0;
    for (; z + 8 <= splits; z += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = slab[(size_t)(z + u) * n + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; z < splits; ++z) s += slab[(size_t)z * n + i];
    h[i] = TypeOps<T>::from_f(s);
  }
  for (long k = g; k < ci; k += stride) {
    float s = 0.f;
    for (int z = 0; z < nbp; ++z) s += bpart[(size_t)z * ci + k];
    bias[k] = s;
  }
}

// out[c][k] = A_c p1[c][k] + B_c colsum_k + D_c (W3 G)[c][k]: a 32 x 64 output tile per block,
// 2 x 4 per thread, the W3 G product in fp32 through LDS in 32-deep chunks, the next chunk's
// global loads issued before the current chunk's FMAs
template <typename T>
__global__ __launch_bounds__(256) void lbf_combine_kernel(LbfCombineArgs a) {
  __shared__ float sw[2][32][33];
  __shared__ float sg[2][32][68];
  __shared__ float scs[4][64];
  const int tid = threadIdx.x;
  const int tx = tid % 16, ty = tid / 16;
  const int ntk = a.ci / 64;
  const int c0 = (blockIdx.x / ntk) * 32, k0 = (blockIdx.x % ntk) * 64;
  {   // the tile's 64 column sums: 4 interleaved groups of partial rows, then in order; 16
      // loads in flight per thread (a dependent add per load was ~60 us per launch)
    const int kk = tid % 64, q = tid / 64;
    const float* P = a.cspart + k0 + kk;
    float s = 0.f;
    int r = q;
    for (; r + 60 < a.rb; r += 64) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = P[(size_t)(r + 4 * u) * a.ci];
#pragma unroll
      for (int u = 0; u < 16; ++u) s += v[u];
    }
    for (; r < a.rb; r += 4) s += P[(size_t)r * a.ci];
    scs[q][kk] = s;
  }
  // chunk loaders: W3 rows c0..c0+31 x 32 k (4 bf16 per thread), G 32 rows x 64 k (8 floats)
  const int wr = tid / 8, wq = (tid % 8) * 4;
  const int gr = tid / 8, gq = (tid % 8) * 8;
  const T* Wp = (const T*)a.w + (size_t)(c0 + wr) * a.ci + wq;
  const float* Gp = a.g + (size_t)gr * a.ci + k0 + gq;
  uint2 wn;
  float4 g0n, g1n;
  auto fetch = [&](int j0) {
    wn = *(const uint2*)(Wp + j0);
    g0n = *(const float4*)(Gp + (size_t)j0 * a.ci);
    g1n = *(const float4*)(Gp + (size_t)j0 * a.ci + 4);
  };
  auto stage = [&](int buf) {
    float v[4];
    v[0] = TypeOps<T>::to_f(__builtin_bit_cast(T, (uint16_t)(wn.x & 0xffff)));
    v[1] = TypeOps<T>::to_f(__builtin_bit_cast(T, (uint16_t)(wn.x >> 16)));
    v[2] = TypeOps<T>::to_f(__builtin_bit_cast(T, (uint16_t)(wn.y & 0xffff)));
    v[3] = TypeOps<T>::to_f(__builtin_bit_cast(T, (uint16_t)(wn.y >> 16)));
#pragma unroll
    for (int e = 0; e < 4; ++e) sw[buf][wr][wq + e] = v[e];
    *(float4*)&sg[buf][gr][gq] = g0n;
    *(float4*)&sg[buf][gr][gq + 4] = g1n;
  };
  float acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int l = 0; l < 4; ++l) acc[i][l] = 0.f;
  fetch(0);
  stage(0);
  int buf = 0;
  for (int j0 = 0; j0 < a.ci; j0 += 32) {
    const bool more = j0 + 32 < a.ci;
    if (more) fetch(j0 + 32);
    __syncthreads();
#pragma unroll 8
    for (int j = 0; j < 32; ++j) {
      const float w0 = sw[buf][ty * 2][j], w1 = sw[buf][ty * 2 + 1][j];
      const float4 gv = *(const float4*)&sg[buf][j][tx * 4];
      acc[0][0] = __builtin_fmaf(w0, gv.x, acc[0][0]);
      acc[0][1] = __builtin_fmaf(w0, gv.y, acc[0][1]);
      acc[0][2] = __builtin_fmaf(w0, gv.z, acc[0][2]);
      acc[0][3] = __builtin_fmaf(w0, gv.w, acc[0][3]);
      acc[1][0] = __builtin_fmaf(w1, gv.x, acc[1][0]);
      acc[1][1] = __builtin_fmaf(w1, gv.y, acc[1][1]);
      acc[1][2] = __builtin_fmaf(w1, gv.z, acc[1][2]);
      acc[1][3] = __builtin_fmaf(w1, gv.w, acc[1][3]);
    }
    if (more) stage(buf ^ 1);
    buf ^= 1;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = c0 + ty * 2 + i;
    const float A = a.coef[c], B = a.coef[a.co + c], D = a.coef[2 * a.co + c];
    const float4 p = *(const float4*)(a.p1 + (size_t)c * a.ci + k0 + tx * 4);
    const float pv[4] = {p.x, p.y, p.z, p.w};
    float o[4];
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      const int kk = tx * 4 + l;
      const float cs = (scs[0][kk] + scs[1][kk]) + (scs[2][kk] + scs[3][kk]);
      o[l] = A * pv[l] + B * cs + D * acc[i][l];
    }
    *(float4*)(a.out + (size_t)c * a.ci + k0 + tx * 4) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

template <typename T>
hipError_t prep_t(const LbfPrepArgs& a, hipStream_t s) {
  const int nb_wt = ceil_div((long)a.ci * (a.co / 8), 256);
  const int nb_xd = ceil_div((long)a.co * (a.ci / 8), 256);
  const int nb_b = (a.ci / 64) * (a.co / 128), nb_c = ceil_div(a.co, 256);
  hipLaunchKernelGGL(lbf_prep_kernel<T>, dim3(nb_wt + nb_xd + nb_b + nb_c), dim3(256), 0, s, a, nb_wt,
                     nb_xd, nb_b);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_lbf_prep(int dtype, const LbfPrepArgs& a, hipStream_t s) {
  if (!seg_half(dtype) || a.co % 128 || a.ci % 64 || a.co > 2048) return hipErrorInvalidValue;
  return dtype == SEG_F16 ? prep_t<f16_t>(a, s) : prep_t<bf16_t>(a, s);
}

hipError_t launch_lbf_hreduce(int dtype, const float* slab, int splits, long n, void* h,
                              const float* bpart, int nbp, int ci, float* bias, hipStream_t s) {
  const int blocks = ceil_div(n, 256) < 1024 ? ceil_div(n, 256) : 1024;
  if (dtype == SEG_F16)
    hipLaunchKernelGGL(lbf_hreduce_kernel<f16_t>, dim3(blocks), dim3(256), 0, s, slab, splits, n, (f16_t*)h,
                       bpart, nbp, ci, bias);
  else if (dtype == SEG_BF16)
    hipLaunchKernelGGL(lbf_hreduce_kernel<bf16_t>, dim3(blocks), dim3(256), 0, s, slab, splits, n, (bf16_t*)h,
                       bpart, nbp, ci, bias);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_lbf_combine(int dtype, const LbfCombineArgs& a, hipStream_t s) {
  if (a.co % 32 || a.ci % 64) return hipErrorInvalidValue;
  const dim3 g((a.co / 32) * (a.ci / 64));
  if (dtype == SEG_F16) hipLaunchKernelGGL(lbf_combine_kernel<f16_t>, g, dim3(256), 0, s, a);
  else if (dtype == SEG_BF16) hipLaunchKernelGGL(lbf_combine_kernel<bf16_t>, g, dim3(256), 0, s, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}
