// Group normalisation statistics (see gn.h).
#include "gn.h"

namespace {

constexpr int GN_THREADS = 256;
constexpr int GN_CHUNK = 512;   // rows per forward partial

// per image n and row chunk: per channel (sum, M2) over the chunk's rows, exact two-pass
// (mean of the chunk first, then squared deviations); thread = (row lane, channel)
template <typename T>
__global__ __launch_bounds__(GN_THREADS) void gn_partial_kernel(GnPartArgs a) {
  __shared__ float sh[GN_THREADS];
  __shared__ float mu[GN_THREADS];
  const int cpb = a.C - (int)blockIdx.y * GN_THREADS < GN_THREADS ? a.C - (int)blockIdx.y * GN_THREADS : GN_THREADS;
  const int rpp = GN_THREADS / cpb;
  const int cl = threadIdx.x % cpb, rl = threadIdx.x / cpb;
  const int c = blockIdx.y * GN_THREADS + cl;
  const bool act = rl < rpp;
  const int n = blockIdx.z, k = blockIdx.x;
  const long r0 = (long)k * a.chunk;
  const long r1 = r0 + a.chunk < a.hw ? r0 + a.chunk : a.hw;
  const T* Y = (const T*)a.y + (size_t)n * a.hw * a.ldy + c;
  float s = 0.f;
  if (act)
    for (long r = r0 + rl; r < r1; r += rpp) s += TypeOps<T>::to_f(Y[(size_t)r * a.ldy]);
  sh[threadIdx.x] = s;
  __syncthreads();
  if (act && rl == 0) {
    float t = sh[cl];
    for (int q = 1; q < rpp; ++q) t += sh[q * cpb + cl];
    sh[cl] = t;   // rl == 0 slots hold the chunk sums from here on
    mu[cl] = t / (float)(r1 - r0);
  }
  __syncthreads();
  const float m = act ? mu[cl] : 0.f;
  float q2 = 0.f;
  if (act)
    for (long r = r0 + rl; r < r1; r += rpp) {
      const float d = TypeOps<T>::to_f(Y[(size_t)r * a.ldy]) - m;
      q2 += d * d;
    }
  const float sum = (act && rl == 0) ? sh[cl] : 0.f;
  __syncthreads();
  sh[threadIdx.x] = q2;
  __syncthreads();
  if (act && rl == 0) {
    float t = sh[cl];
    for (int q = 1; q < rpp; ++q) t += sh[q * cpb + cl];
    const int nch = (int)((a.hw + a.chunk - 1) / a.chunk);
    float* o = a.part + 2 * (((size_t)n * nch + k) * a.C + c);
    o[0] = sum;
    o[1] = t;
  }
}

// Chan merge of (count, mean, M2) b into a
__device__ __forceinline__ void chan_merge(float& na, float& ma, float& qa, float nb, float mb, float qb) {
  const float n = na + nb;
  if (nb <= 0.f) return;
  const float d = mb - ma;
  ma += d * (nb / n);
  qa += qb + d * d * (na * nb / n);
  na = n;
}

// per (group, image): merge the chunk partials of the group's channels in fixed order
__global__ __launch_bounds__(GN_THREADS) void gn_stats_final_kernel(const float* __restrict__ part,
                                                                    int N, long hw, int C, int groups,
                                                                    const float* __restrict__ gamma,
                                                                    const BnState* __restrict__ st) {
  __shared__ float sn[GN_THREADS], sm[GN_THREADS], sq[GN_THREADS];
  const int g = blockIdx.x, n = blockIdx.y;
  const int cg = C / groups;
  const int nch = (int)((hw + GN_CHUNK - 1) / GN_CHUNK);
  float cnt = 0.f, mean = 0.f, m2 = 0.f;
  for (long e = threadIdx.x; e < (long)nch * cg; e += GN_THREADS) {
    const int k = (int)(e / cg), c = g * cg + (int)(e % cg);
    const float* p = part + 2 * (((size_t)n * nch + k) * C + c);
    const long rows = (long)(k + 1) * GN_CHUNK < hw ? GN_CHUNK : hw - (long)k * GN_CHUNK;
    chan_merge(cnt, mean, m2, (float)rows, p[0] / (float)rows, p[1]);
  }
  sn[threadIdx.x] = cnt; sm[threadIdx.x] = mean; sq[threadIdx.x] = m2;
  __syncthreads();
  for (int s = GN_THREADS / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      float na = sn[threadIdx.x], ma = sm[threadIdx.x], qa = sq[threadIdx.x];
      chan_merge(na, ma, qa, sn[threadIdx.x + s], sm[threadIdx.x + s], sq[threadIdx.x + s]);
      sn[threadIdx.x] = na; sm[threadIdx.x] = ma; sq[threadIdx.x] = qa;
    }
    __syncthreads();
  }
  const float mu = sm[0];
  const float rstd = rsqrtf(sq[0] / (float)(hw * cg) + SEG_GN_EPS);   // biased variance
  const BnState S = st[n];
  for (int j = threadIdx.x; j < cg; j += GN_THREADS) {
    const int c = g * cg + j;
    S.mean[c] = mu;
    S.invstd[c] = rstd;
    S.scale[c] = gamma[c] * rstd;
  }
}

// per channel: the per-image reduce partials -> S1, S2 (fixed order); per (image, group) the
// means of gamma * S; dgamma / dbeta summed over the images in order
__global__ __launch_bounds__(GN_THREADS) void gn_bwd_final_kernel(const float* __restrict__ part,
                                                                  int N, int rb, long hw, int C,
                                                                  int groups,
                                                                  const float* __restrict__ gamma,
                                                                  const BnState* __restrict__ st,
                                                                  float* dgamma, float* dbeta) {
  __shared__ float v1[GN_THREADS], v2[GN_THREADS];
  const int cg = C / groups;
  const int c = blockIdx.x * GN_THREADS + threadIdx.x;
  const bool act = c < C;
  const float gm = act ? gamma[c] : 0.f;
  const float inv = 1.f / (float)(hw * cg);
  float t1 = 0.f, t2 = 0.f;
  for (int n = 0; n < N; ++n) {
    float s1 = 0.f, s2 = 0.f;
    if (act)
      for (int b = 0; b < rb; ++b) {
        const float2 p = *(const float2*)(part + 2 * (((size_t)n * rb + b) * C + c));
        s1 += p.x;
        s2 += p.y;
      }
    t1 += s1;
    t2 += s2;
    v1[threadIdx.x] = gm * s1;
    v2[threadIdx.x] = gm * s2;
    __syncthreads();
    if (act && c % cg == 0) {   // group leader: its cg channels are in this block (256 % cg == 0)
      float a1 = 0.f, a2 = 0.f;
      for (int j = 0; j < cg; ++j) { a1 += v1[threadIdx.x + j]; a2 += v2[threadIdx.x + j]; }
      v1[threadIdx.x] = a1 * inv;
      v2[threadIdx.x] = a2 * inv;
    }
    __syncthreads();
    if (act) {
      const int lead = threadIdx.x - (c % cg);
      st[n].sdy[c] = v1[lead];
      st[n].sdyx[c] = v2[lead];
    }
    __syncthreads();
  }
  if (act) {
    if (dgamma) dgamma[c] = t2;
    if (dbeta) dbeta[c] = t1;
  }
}

__global__ void gn_chscale_kernel(const float* __restrict__ src, float* dst, long rows, int ld,
                                  int C, const float* __restrict__ scale) {
  const long total = rows * C;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / C;
    const int c = (int)(i - r * C);
    dst[r * ld + c] = src[r * ld + c] * scale[c];
  }
}

}  // namespace

int gn_chunks(long hw) { return (int)((hw + GN_CHUNK - 1) / GN_CHUNK); }

hipError_t launch_gn_partial(int dtype, int y_f32, const GnPartArgs& a0, hipStream_t s) {
  GnPartArgs a = a0;
  a.chunk = GN_CHUNK;
  const dim3 g(gn_chunks(a.hw), (a.C + GN_THREADS - 1) / GN_THREADS, a.N);
  if (y_f32 || dtype == SEG_F32) hipLaunchKernelGGL(gn_partial_kernel<float>, g, dim3(GN_THREADS), 0, s, a);
  else if (dtype == SEG_F16) hipLaunchKernelGGL(gn_partial_kernel<f16_t>, g, dim3(GN_THREADS), 0, s, a);
  else hipLaunchKernelGGL(gn_partial_kernel<bf16_t>, g, dim3(GN_THREADS), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_gn_stats_final(const float* part, int N, long hw, int C, int groups,
                                 const float* gamma, const BnState* st, hipStream_t s) {
  if (groups < 1 || C % groups) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gn_stats_final_kernel, dim3(groups, N), dim3(GN_THREADS), 0, s, part, N, hw, C,
                     groups, gamma, st);
  return hipGetLastError();
}

hipError_t launch_gn_bwd_final(const float* part, int N, int rb, long hw, int C, int groups,
                               const float* gamma, const BnState* st, float* dgamma,
                               float* dbeta, hipStream_t s) {
  const int cg = groups > 0 ? C / groups : 0;
  if (groups < 1 || C % groups || (cg > GN_THREADS) || (C > GN_THREADS && GN_THREADS % cg))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(gn_bwd_final_kernel, dim3((C + GN_THREADS - 1) / GN_THREADS), dim3(GN_THREADS), 0,
                     s, part, N, rb, hw, C, groups, gamma, st, dgamma, dbeta);
  return hipGetLastError();
}

hipError_t launch_gn_chscale(const float* src, float* dst, long rows, int ld, int C,
                             const float* scale, hipStream_t s) {
  long g = (rows * C + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(gn_chscale_kernel, dim3((int)(g < 1 ? 1 : g)), dim3(256), 0, s, src, dst, rows,
                     ld, C, scale);
  return hipGetLastError();
}
