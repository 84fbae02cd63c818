// Batch-norm kernels (see bn.h). All reductions use a fixed order: bitwise reproducible.
#include "bn.h"

namespace {

// ---- forward statistics: merge per-tile (sum, M2) partials with Chan's formula --------
// stage 1: grid (ceil(C/64), G); block 256 = 64 channels x 4 tile lanes
constexpr int STAT_TPB = 64;  // tiles per block in stage 1

__device__ __forceinline__ void chan_merge(float& n, float& mean, float& m2, float nb, float meanb,
                                           float m2b) {
  if (nb <= 0.f) return;
  if (n <= 0.f) { n = nb; mean = meanb; m2 = m2b; return; }
  float tot = n + nb;
  float d = meanb - mean;
  mean = mean + d * (nb / tot);
  m2 = m2 + m2b + d * d * (n * nb / tot);
  n = tot;
}

__global__ void bn_stats_stage1(const float* __restrict__ part, long M, int C, int tile_rows,
                                int ntiles, float* __restrict__ out /* [G][C][3] */) {
  __shared__ float sh[3][4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int tl = threadIdx.x >> 6;
  const int t0 = blockIdx.y * STAT_TPB;
  float n = 0.f, mean = 0.f, m2 = 0.f;
  if (c < C) {
    for (int t = t0 + tl; t < t0 + STAT_TPB && t < ntiles; t += 4) {
      long rows = M - (long)t * tile_rows;
      float nb = (float)(rows < tile_rows ? rows : tile_rows);
      float2 v = *(const float2*)(part + 2 * ((size_t)t * C + c));
      chan_merge(n, mean, m2, nb, v.x / nb, v.y);
    }
  }
  sh[0][tl][threadIdx.x & 63] = n;
  sh[1][tl][threadIdx.x & 63] = mean;
  sh[2][tl][threadIdx.x & 63] = m2;
  __syncthreads();
  if (tl == 0 && c < C) {
    for (int k = 1; k < 4; ++k)
      chan_merge(n, mean, m2, sh[0][k][threadIdx.x], sh[1][k][threadIdx.x], sh[2][k][threadIdx.x]);
    float* o = out + 3 * ((size_t)blockIdx.y * C + c);
    o[0] = n; o[1] = mean; o[2] = m2;
  }
}

__global__ void bn_stats_stage2(const float* __restrict__ g, int G, int C, const float* gamma,
                                BnState st) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float n = 0.f, mean = 0.f, m2 = 0.f;
  for (int k = 0; k < G; ++k) {
    const float* o = g + 3 * ((size_t)k * C + c);
    chan_merge(n, mean, m2, o[0], o[1], o[2]);
  }
  float var = m2 / n;
  float inv = rsqrtf(var + SEG_BN_EPS);
  st.mean[c] = mean;
  st.invstd[c] = inv;
  st.scale[c] = gamma[c] * inv;
  st.var_unb[c] = m2 / (n > 1.f ? n - 1.f : 1.f);
}

// ---- forward apply ---------------------------------------------------------------------
template <typename T, typename TO, int VEC>
__global__ void bn_apply_kernel(BnApplyArgs a) {
  const int cg_n = a.C / VEC;
  const long total = a.M * cg_n;
  const T* Y = (const T*)a.y;
  const T* RES = (const T*)a.res;
  const T* Y2 = (const T*)a.y2;
  TO* O = (TO*)a.out;
  for (long it = (long)blockIdx.x * blockDim.x + threadIdx.x; it < total;
       it += (long)gridDim.x * blockDim.x) {
    const long m = it / cg_n;
    const int c0 = (int)(it - m * cg_n) * VEC;
    float v[VEC];
    if constexpr (VEC == 8) {
      Vec8<T>::load(Y + (size_t)m * a.ldy + c0, v);
    } else {
      v[0] = ldf(Y + (size_t)m * a.ldy + c0);
    }
#pragma unroll
    for (int e = 0; e < VEC; ++e) v[e] = (v[e] - a.mean[c0 + e]) * a.scale[c0 + e] + a.beta[c0 + e];
    if (Y2) {
      float u[VEC];
      if constexpr (VEC == 8) Vec8<T>::load(Y2 + (size_t)m * a.ldy2 + c0, u);
      else u[0] = ldf(Y2 + (size_t)m * a.ldy2 + c0);
#pragma unroll
      for (int e = 0; e < VEC; ++e)
        v[e] = ((u[e] - a.mean2[c0 + e]) * a.scale2[c0 + e] + a.beta2[c0 + e]) + v[e];
    } else if (RES) {
      size_t rm = (size_t)m;
      if (a.rs > 1) {
        long wo = m % a.Wo;
        long t = m / a.Wo;
        long ho = t % a.Ho;
        long n = t / a.Ho;
        rm = (size_t)((n * a.Hr + ho * a.rs) * a.Wr + wo * a.rs);
      }
      float u[VEC];
      if constexpr (VEC == 8) Vec8<T>::load(RES + rm * a.ldres + c0, u);
      else u[0] = ldf(RES + rm * a.ldres + c0);
#pragma unroll
      for (int e = 0; e < VEC; ++e) v[e] = u[e] + v[e];  // shortcut + residual
    }
    if (a.relu) {
#pragma unroll
      for (int e = 0; e < VEC; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    if constexpr (VEC == 8) Vec8<TO>::store(O + (size_t)m * a.ldo + c0, v);
    else stf(O + (size_t)m * a.ldo + c0, v[0]);
  }
}

// ---- backward reduce: per row block partial sums of dyhat and dyhat*xhat -----------------
// block: 256 threads = RL row lanes x CGB channel groups (VEC channels each)
template <typename T, typename TZ, int VEC>
__global__ void bn_bwd_reduce_kernel(BnBwdArgs a) {
  const int cg_n = a.C / VEC;
  const int cgb = cg_n < 256 ? cg_n : 256;       // channel groups per block pass
  const int rl_n = 256 / cgb;                     // row lanes
  const int tcg = threadIdx.x % cgb, trl = threadIdx.x / cgb;
  const long rows_per = (a.M + a.rb - 1) / a.rb;
  const long r0 = (long)blockIdx.x * rows_per;
  const long r1 = (r0 + rows_per < a.M) ? r0 + rows_per : a.M;
  const TZ* DZ = (const TZ*)a.dz;
  const TZ* Z = (const TZ*)a.z;
  const T* Y = (const T*)a.y;
  __shared__ float sh[2][256 * VEC];
  for (int base = 0; base < cg_n; base += cgb) {
    const int cg = base + tcg;
    const bool act = cg < cg_n;
    const int c0 = act ? cg * VEC : 0;
    float s1[VEC], s2[VEC], mu[VEC], inv[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) { s1[e] = 0.f; s2[e] = 0.f; mu[e] = a.mean[c0 + e]; inv[e] = a.invstd[c0 + e]; }
    if (act && trl < rl_n) {
      for (long m = r0 + trl; m < r1; m += rl_n) {
        float dz[VEC], y[VEC];
        if constexpr (VEC == 8) {
          Vec8<TZ>::load(DZ + (size_t)m * a.lddz + c0, dz);
          Vec8<T>::load(Y + (size_t)m * a.ldy + c0, y);
        } else {
          dz[0] = ldf(DZ + (size_t)m * a.lddz + c0);
          y[0] = ldf(Y + (size_t)m * a.ldy + c0);
        }
        if (Z) {
          float z[VEC];
          if constexpr (VEC == 8) Vec8<TZ>::load(Z + (size_t)m * a.ldz + c0, z);
          else z[0] = ldf(Z + (size_t)m * a.ldz + c0);
#pragma unroll
          for (int e = 0; e < VEC; ++e) dz[e] = z[e] > 0.f ? dz[e] : 0.f;
        }
        if (a.dzscale) {
#pragma unroll
          for (int e = 0; e < VEC; ++e) dz[e] *= a.dzscale[c0 + e];
        }
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          s1[e] += dz[e];
          s2[e] += dz[e] * ((y[e] - mu[e]) * inv[e]);
        }
      }
    }
    // reduce over row lanes through LDS (fixed order)
    __syncthreads();
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      sh[0][threadIdx.x * VEC + e] = s1[e];
      sh[1][threadIdx.x * VEC + e] = s2[e];
    }
    __syncthreads();
    if (act && trl == 0) {
      for (int r = 1; r < rl_n; ++r) {
        int t = r * cgb + tcg;
#pragma unroll
        for (int e = 0; e < VEC; ++e) { s1[e] += sh[0][t * VEC + e]; s2[e] += sh[1][t * VEC + e]; }
      }
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        float* o = a.part + 2 * ((size_t)blockIdx.x * a.C + c0 + e);
        o[0] = s1[e];
        o[1] = s2[e];
      }
    }
  }
}

// block = 8 channels (fast) x 32 row-block lanes; fixed-order float sums, then an LDS tree
__global__ void bn_bwd_finalize_kernel(const float* __restrict__ part, int rb, long M, int C,
                                       BnState st, float* dgamma, float* dbeta) {
  __shared__ float sh[2][32][9];
  const int cl = threadIdx.x & 7, lane = threadIdx.x >> 3;
  const int c = blockIdx.x * 8 + cl;
  float s1 = 0.f, s2 = 0.f;
  if (c < C) {
    for (int k = lane; k < rb; k += 32) {
      const float2 v = *(const float2*)(part + 2 * ((size_t)k * C + c));
      s1 += v.x;
      s2 += v.y;
    }
  }
  sh[0][lane][cl] = s1;
  sh[1][lane][cl] = s2;
  __syncthreads();
  for (int st2 = 16; st2 > 0; st2 >>= 1) {
    if (lane < st2) {
      sh[0][lane][cl] += sh[0][lane + st2][cl];
      sh[1][lane][cl] += sh[1][lane + st2][cl];
    }
    __syncthreads();
  }
  if (lane == 0 && c < C) {
    s1 = sh[0][0][cl];
    s2 = sh[1][0][cl];
    st.sdy[c] = s1 / (float)M;
    st.sdyx[c] = s2 / (float)M;
    if (dgamma) dgamma[c] = s2;
    if (dbeta) dbeta[c] = s1;
  }
}

template <typename T, typename TZ, int VEC>
__global__ void bn_bwd_apply_kernel(BnBwdArgs a) {
  const int cg_n = a.C / VEC;
  const long total = a.M * cg_n;
  const TZ* DZ = (const TZ*)a.dz;
  const TZ* Z = (const TZ*)a.z;
  const T* Y = (const T*)a.y;
  T* DY = (T*)a.dy;
  T* DH = (T*)a.dyhat;
  for (long it = (long)blockIdx.x * blockDim.x + threadIdx.x; it < total;
       it += (long)gridDim.x * blockDim.x) {
    const long m = it / cg_n;
    const int c0 = (int)(it - m * cg_n) * VEC;
    float dz[VEC], y[VEC];
    if constexpr (VEC == 8) {
      Vec8<TZ>::load(DZ + (size_t)m * a.lddz + c0, dz);
      Vec8<T>::load(Y + (size_t)m * a.ldy + c0, y);
    } else {
      dz[0] = ldf(DZ + (size_t)m * a.lddz + c0);
      y[0] = ldf(Y + (size_t)m * a.ldy + c0);
    }
    if (Z) {
      float z[VEC];
      if constexpr (VEC == 8) Vec8<TZ>::load(Z + (size_t)m * a.ldz + c0, z);
      else z[0] = ldf(Z + (size_t)m * a.ldz + c0);
#pragma unroll
      for (int e = 0; e < VEC; ++e) dz[e] = z[e] > 0.f ? dz[e] : 0.f;
    }
    if (a.dzscale) {
#pragma unroll
      for (int e = 0; e < VEC; ++e) dz[e] *= a.dzscale[c0 + e];
    }
    if (DH) {
      if constexpr (VEC == 8) Vec8<T>::store(DH + (size_t)m * a.lddyhat + c0, dz);
      else stf(DH + (size_t)m * a.lddyhat + c0, dz[0]);
    }
    float o[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      const int c = c0 + e;
      float xh = (y[e] - a.mean[c]) * a.invstd[c];
      o[e] = a.scale[c] * (dz[e] - a.sdy[c] - xh * a.sdyx[c]);
    }
    if constexpr (VEC == 8) Vec8<T>::store(DY + (size_t)m * a.lddy + c0, o);
    else stf(DY + (size_t)m * a.lddy + c0, o[0]);
  }
}

__global__ void moving_update_kernel(float* mm, float* mv, const float* bm, const float* bv, int n,
                                     float decay) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // assign_moving_average(zero_debias=False): v -= (1-decay)*(v - value)
  mm[i] -= (1.f - decay) * (mm[i] - bm[i]);
  mv[i] -= (1.f - decay) * (mv[i] - bv[i]);
}

int grid_for(long items) {
  long g = (items + 255) / 256;
  return (int)(g < 4096 ? (g < 1 ? 1 : g) : 4096);
}

template <typename T, typename TO>
hipError_t apply_t(const BnApplyArgs& a, hipStream_t s) {
  bool v8 = (a.C % 8 == 0) && (a.ldy % 8 == 0) && (a.ldo % 8 == 0) &&
            (!a.res || a.ldres % 8 == 0) && (!a.y2 || a.ldy2 % 8 == 0) &&
            (((uintptr_t)a.out) % 16 == 0);
  if (v8) hipLaunchKernelGGL((bn_apply_kernel<T, TO, 8>), dim3(grid_for(a.M * a.C / 8)), dim3(256), 0, s, a);
  else hipLaunchKernelGGL((bn_apply_kernel<T, TO, 1>), dim3(grid_for(a.M * a.C)), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <typename T, typename TZ>
bool bwd_v8(const BnBwdArgs& a) {
  return (a.C % 8 == 0) && (a.lddz % 8 == 0) && (a.ldy % 8 == 0) && (!a.z || a.ldz % 8 == 0) &&
         (!a.dy || a.lddy % 8 == 0) && (!a.dyhat || a.lddyhat % 8 == 0) &&
         ((uintptr_t)a.dz % 16 == 0);
}

template <typename T, typename TZ>
hipError_t bwd_reduce_t(const BnBwdArgs& a, hipStream_t s) {
  if (bwd_v8<T, TZ>(a)) hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, TZ, 8>), dim3(a.rb), dim3(256), 0, s, a);
  else hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, TZ, 1>), dim3(a.rb), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <typename T, typename TZ>
hipError_t bwd_apply_t(const BnBwdArgs& a, hipStream_t s) {
  if (bwd_v8<T, TZ>(a)) hipLaunchKernelGGL((bn_bwd_apply_kernel<T, TZ, 8>), dim3(grid_for(a.M * a.C / 8)), dim3(256), 0, s, a);
  else hipLaunchKernelGGL((bn_bwd_apply_kernel<T, TZ, 1>), dim3(grid_for(a.M * a.C)), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_bn_stats_finalize(const float* tile_part, long M, int C, int tile_rows,
                                    float* scratch, const float* gamma, BnState st,
                                    hipStream_t s) {
  int ntiles = ceil_div(M, tile_rows);
  int G = ceil_div(ntiles, STAT_TPB);
  hipLaunchKernelGGL(bn_stats_stage1, dim3(ceil_div(C, 64), G), dim3(256), 0, s, tile_part, M, C,
                     tile_rows, ntiles, scratch);
  hipLaunchKernelGGL(bn_stats_stage2, dim3(ceil_div(C, 64)), dim3(64), 0, s, scratch, G, C, gamma,
                     st);
  return hipGetLastError();
}

hipError_t launch_bn_apply(int dtype, int out_f32, const BnApplyArgs& a, hipStream_t s) {
  if (dtype == SEG_BF16) {
    if (out_f32) return apply_t<bf16_t, float>(a, s);
    return apply_t<bf16_t, bf16_t>(a, s);
  }
  return apply_t<float, float>(a, s);
}

int bn_bwd_rowblocks(long M, int C) {
  // ~1024 blocks, each >= 64 rows
  long rb = (M + 63) / 64;
  if (rb > 1024) rb = 1024;
  (void)C;
  return (int)(rb < 1 ? 1 : rb);
}

hipError_t launch_bn_bwd_reduce(int dtype, int dz_f32, const BnBwdArgs& a, hipStream_t s) {
  if (dtype == SEG_BF16) {
    if (dz_f32) return bwd_reduce_t<bf16_t, float>(a, s);
    return bwd_reduce_t<bf16_t, bf16_t>(a, s);
  }
  return bwd_reduce_t<float, float>(a, s);
}

hipError_t launch_bn_bwd_finalize(const float* part, int rb, long M, int C, BnState st,
                                  float* dgamma, float* dbeta, hipStream_t s) {
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(ceil_div(C, 8)), dim3(256), 0, s, part, rb, M,
                     C, st, dgamma, dbeta);
  return hipGetLastError();
}

hipError_t launch_bn_bwd_apply(int dtype, int dz_f32, const BnBwdArgs& a, hipStream_t s) {
  if (dtype == SEG_BF16) {
    if (dz_f32) return bwd_apply_t<bf16_t, float>(a, s);
    return bwd_apply_t<bf16_t, bf16_t>(a, s);
  }
  return bwd_apply_t<float, float>(a, s);
}

hipError_t launch_moving_update(float* mov_mean, float* mov_var, const float* bmean,
                                const float* bvar, int n, float decay, hipStream_t s) {
  hipLaunchKernelGGL(moving_update_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, s, mov_mean,
                     mov_var, bmean, bvar, n, decay);
  return hipGetLastError();
}
