// Batch-norm kernels (see bn.h). All reductions use a fixed order: bitwise reproducible.
#include "bn.h"
#include <cstdlib>
#include <type_traits>

// (non-temporal stores for the apply kernels' outputs measured no faster)
#define BN_STORE8(T, p, v) Vec8<T>::store(p, v)

namespace {

// ---- forward statistics: one-launch finalize (a two-launch Chan merge measured slower) ----
// per-tile (sum, M2) partials of tile_rows rows (the last one ragged) merged as shifted sums
// around tile 0's mean p: A = sum_t n_t (mean_t - p), B = sum_t (M2_t + n_t (mean_t - p)^2), so
// mean = p + A / N and var = B / N - (A / N)^2, with no division per merge. Block = 8 channels
// (consecutive lanes: each tile's 8 partials are one 64-B read) x 64 tile lanes; a lane issues
// FIN_U tiles' loads before using any, then a fixed xor butterfly over the wave's 8 tile lanes
// and a fixed-order sum of the 8 waves (bitwise reproducible). (A per-lane-tile layout with 8
// strided 8-B loads per tile ran 1.1-1.9x slower beside the side stream: 8x the cache-line
// requests.)
constexpr int FIN_CH = 8, FIN_LANES = 64, FIN_U = 16;

__global__ __launch_bounds__(FIN_CH * FIN_LANES) void bn_stats_final_kernel(
    const float* __restrict__ part, long M, int C, int tile_rows, int ntiles,
    const float* __restrict__ gamma, BnState st, float* pack) {
  __shared__ float sh[2][FIN_LANES / 8][FIN_CH];
  const int cl = threadIdx.x % FIN_CH, tl = threadIdx.x / FIN_CH;
  const int c = blockIdx.x * FIN_CH + cl;
  float A = 0.f, B = 0.f, p = 0.f;
  if (c < C) {
    const float fr = (float)tile_rows, inv_fr = 1.f / fr;
    const float s0 = part[2 * (size_t)c];
    p = M < tile_rows ? s0 / (float)M : s0 * inv_fr;
    for (int t0 = tl; t0 < ntiles; t0 += FIN_LANES * FIN_U) {
      float2 v[FIN_U];
#pragma unroll
      for (int u = 0; u < FIN_U; ++u) {
        const int t = t0 + u * FIN_LANES;
        v[u] = t < ntiles ? *(const float2*)(part + 2 * ((size_t)t * C + c)) : make_float2(0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < FIN_U; ++u) {
        const int t = t0 + u * FIN_LANES;
        const long rows = M - (long)t * tile_rows;
        const bool rag = rows < tile_rows;
        const float n = t >= ntiles ? 0.f : (rag ? (float)rows : fr);   // absent tiles weigh 0
        const float d = (rag ? v[u].x / fmaxf(n, 1.f) : v[u].x * inv_fr) - p;
        A = __builtin_fmaf(n, d, A);
        B += __builtin_fmaf(n * d, d, v[u].y);
      }
    }
  }
#pragma unroll
  for (int o = FIN_CH; o < 64; o <<= 1) {   // the wave's 8 tile lanes of this channel
    A += __shfl_xor(A, o, 64);
    B += __shfl_xor(B, o, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) < FIN_CH) {
    sh[0][w][cl] = A;
    sh[1][w][cl] = B;
  }
  __syncthreads();
  if (threadIdx.x < FIN_CH && c < C) {
    A = sh[0][0][cl];
    B = sh[1][0][cl];
#pragma unroll
    for (int k = 1; k < FIN_LANES / 8; ++k) {
      A += sh[0][k][cl];
      B += sh[1][k][cl];
    }
    const float N = (float)M;
    const float dm = A / N;
    const float mean = p + dm;
    const float var = fmaxf(B / N - dm * dm, 0.f);
    const float inv = rsqrtf(var + SEG_BN_EPS);
    st.mean[c] = mean;
    st.invstd[c] = inv;
    st.scale[c] = gamma[c] * inv;
    st.var_unb[c] = var * (N / (N > 1.f ? N - 1.f : 1.f));
    if (pack) {
      pack[c] = mean;
      pack[C + c] = var + mean * mean;
    }
  }
}

// backward finalize: sums of the per-row-block (sum dyhat, sum dyhat*xhat) partials, the same
// layout and fixed reduction order
__global__ __launch_bounds__(FIN_CH * FIN_LANES) void bn_bwd_final_kernel(
    const float* __restrict__ part, int rb, long M, int C, BnState st, float* dgamma,
    float* dbeta, int frozen) {
  __shared__ float sh[2][FIN_LANES / 8][FIN_CH];
  const int cl = threadIdx.x % FIN_CH, tl = threadIdx.x / FIN_CH;
  const int c = blockIdx.x * FIN_CH + cl;
  float s1 = 0.f, s2 = 0.f;
  if (c < C) {
    for (int k0 = tl; k0 < rb; k0 += FIN_LANES * FIN_U) {
      float2 v[FIN_U];
#pragma unroll
      for (int u = 0; u < FIN_U; ++u) {
        const int k = k0 + u * FIN_LANES;
        v[u] = k < rb ? *(const float2*)(part + 2 * ((size_t)k * C + c)) : make_float2(0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < FIN_U; ++u) {
        s1 += v[u].x;
        s2 += v[u].y;
      }
    }
  }
#pragma unroll
  for (int o = FIN_CH; o < 64; o <<= 1) {
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) < FIN_CH) {
    sh[0][w][cl] = s1;
    sh[1][w][cl] = s2;
  }
  __syncthreads();
  if (threadIdx.x < FIN_CH && c < C) {
    s1 = sh[0][0][cl];
    s2 = sh[1][0][cl];
#pragma unroll
    for (int k = 1; k < FIN_LANES / 8; ++k) {
      s1 += sh[0][k][cl];
      s2 += sh[1][k][cl];
    }
    st.sdy[c] = frozen ? 0.f : s1 / (float)M;
    st.sdyx[c] = frozen ? 0.f : s2 / (float)M;
    if (dgamma) dgamma[c] = s2;
    if (dbeta) dbeta[c] = s1;
  }
}

// cross_replica_batch_normalization.py:400-425: global mean = mean of the replica means,
// global variance = mean of the replica E[x^2] - mean^2 (no Bessel factor: the non-fused
// path's variance also feeds the moving average, :452-466 with _bessels_correction_test_only)
__global__ void bn_sync_unpack_kernel(const float* __restrict__ pack, int C, float inv_world,
                                      const float* gamma, BnState st) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float mean = pack[c] * inv_world;
  const float var = pack[C + c] * inv_world - mean * mean;
  const float inv = rsqrtf(var + SEG_BN_EPS);
  st.mean[c] = mean;
  st.invstd[c] = inv;
  st.scale[c] = gamma[c] * inv;
  st.var_unb[c] = var;
}

// inference-mode BN (tf.contrib.layers.batch_norm is_training=False, i.e.
// batch_norm_accumulate_statistics unset; hierarchical.py:306-307): the moving statistics
// take the place of the batch statistics in the same apply kernel
__global__ void bn_infer_finalize_kernel(const float* __restrict__ mov_mean,
                                         const float* __restrict__ mov_var, int C,
                                         const float* gamma, BnState st) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float inv = rsqrtf(mov_var[c] + SEG_BN_EPS);
  st.mean[c] = mov_mean[c];
  st.invstd[c] = inv;
  st.scale[c] = gamma[c] * inv;
  st.var_unb[c] = mov_var[c];
}

__global__ void bn_infer_finalize_all_kernel(const BnInferJob* __restrict__ jobs) {
  const BnInferJob j = jobs[blockIdx.x];
  for (int c = threadIdx.x; c < j.C; c += blockDim.x) {
    const float inv = rsqrtf(j.mov_var[c] + SEG_BN_EPS);
    j.st.mean[c] = j.mov_mean[c];
    j.st.invstd[c] = inv;
    j.st.scale[c] = j.gamma[c] * inv;
    j.st.var_unb[c] = j.mov_var[c];
  }
}

// ---- forward apply ---------------------------------------------------------------------
template <typename T, typename TO, int VEC, typename IDX>
__device__ __forceinline__ void bn_apply_body(const BnApplyArgs& a) {
  const int cg_n = a.C / VEC;
  const IDX total = (IDX)(a.M * cg_n);
  const T* Y = (const T*)a.y;
  const T* RES = (const T*)a.res;
  const T* Y2 = (const T*)a.y2;
  TO* O = (TO*)a.out;
  for (IDX it = (IDX)blockIdx.x * blockDim.x + threadIdx.x; it < total;
       it += (IDX)gridDim.x * blockDim.x) {
    const IDX m = it / (IDX)cg_n;
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
        long wo = (long)m % a.Wo;
        long t = (long)m / a.Wo;
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

// generic-layout apply (the narrow logits layers: C = 14 / 7 / 3): 32-bit element indices when
// they fit (round 5: the 64-bit division per element was most of these launches' ~10 us)
template <typename T, typename TO, int VEC>
__global__ void bn_apply_kernel(BnApplyArgs a) {
  if (a.M * (a.C / VEC) < (1L << 31)) bn_apply_body<T, TO, VEC, unsigned>(a);
  else bn_apply_body<T, TO, VEC, long>(a);
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

template <typename T, typename TZ, int VEC, typename IDX>
__device__ __forceinline__ void bn_bwd_apply_body(const BnBwdArgs& a) {
  const int cg_n = a.C / VEC;
  const IDX total = (IDX)(a.M * cg_n);
  const TZ* DZ = (const TZ*)a.dz;
  const TZ* Z = (const TZ*)a.z;
  const T* Y = (const T*)a.y;
  T* DY = (T*)a.dy;
  T* DH = (T*)a.dyhat;
  for (IDX it = (IDX)blockIdx.x * blockDim.x + threadIdx.x; it < total;
       it += (IDX)gridDim.x * blockDim.x) {
    const IDX m = it / (IDX)cg_n;
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
    if (DH) {   // the masked gradient before any per-channel factor
      if constexpr (VEC == 8) Vec8<T>::store(DH + (size_t)m * a.lddyhat + c0, dz);
      else stf(DH + (size_t)m * a.lddyhat + c0, dz[0]);
    }
    if (a.dzscale) {
#pragma unroll
      for (int e = 0; e < VEC; ++e) dz[e] *= a.dzscale[c0 + e];
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

template <typename T, typename TZ, int VEC>
__global__ void bn_bwd_apply_kernel(BnBwdArgs a) {
  if (a.M * (a.C / VEC) < (1L << 31)) bn_bwd_apply_body<T, TZ, VEC, unsigned>(a);
  else bn_bwd_apply_body<T, TZ, VEC, long>(a);
}

// ---- 8-channel streaming kernels (C % 8 == 0): thread -> fixed channel group ------------
// A thread owns one 8-channel group for the whole launch (per-channel constants loaded once)
// and walks rows; U rows are loaded before any is consumed, so U x (2..3) 16-B loads are in
// flight per lane. No integer division in the row loop. C/8 > 256 spills into blockIdx.y.
constexpr int BN_U = 4;   // rows in flight per thread (reduce combines 4 slots explicitly)

struct RowLane {
  int cg, rl, rpp;
  bool act;
};

__device__ __forceinline__ RowLane row_lane(int cg_n) {
  RowLane r;
  if (cg_n >= 256) {
    r.cg = blockIdx.y * 256 + threadIdx.x; r.rl = 0; r.rpp = 1; r.act = r.cg < cg_n;
  } else {
    r.rpp = 256 / cg_n; r.cg = threadIdx.x % cg_n; r.rl = threadIdx.x / cg_n; r.act = r.rl < r.rpp;
  }
  return r;
}

// per-channel constants: scalar loads (BN vectors of small heads break 16-B alignment)
__device__ __forceinline__ void ld8(const float* p, int c0, float* o) {
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = p[c0 + e];
}

// Row loops are split into full groups (U valid rows: no bounds tests, all loads issued
// before any use) and one guarded tail group, and every optional input is a template
// parameter, so the compiler emits straight-line load batches.
enum { RES_NONE = 0, RES_PLAIN = 1, RES_SUB = 2, RES_BN2 = 3 };

template <typename T, typename TO, int RES, int RELU>
__global__ __launch_bounds__(256) void bn_apply8_kernel(BnApplyArgs a) {
  const RowLane L = row_lane(a.C / 8);
  if (!L.act) return;
  const int c0 = L.cg * 8;
  float mu[8], sc[8], be[8], mu2[8], sc2[8], be2[8];
  ld8(a.mean, c0, mu); ld8(a.scale, c0, sc); ld8(a.beta, c0, be);
  if constexpr (RES == RES_BN2) { ld8(a.mean2, c0, mu2); ld8(a.scale2, c0, sc2); ld8(a.beta2, c0, be2); }
  const T* Y = (const T*)a.y + c0;
  const T* RS = (const T*)(RES == RES_BN2 ? a.y2 : a.res) + c0;
  const int ldr = RES == RES_BN2 ? a.ldy2 : a.ldres;
  TO* O = (TO*)a.out + c0;
  const long step = (long)L.rpp * BN_U;
  auto res_row = [&](long m) -> size_t {
    if constexpr (RES == RES_SUB) {
      const int mi = (int)m;
      const int wo = mi % a.Wo, t = mi / a.Wo;
      const int ho = t % a.Ho, n = t / a.Ho;
      return ((size_t)n * a.Hr + (size_t)ho * a.rs) * a.Wr + (size_t)wo * a.rs;
    } else {
      return (size_t)m;
    }
  };
  auto body = [&](long base, int nrows) {
    float v[BN_U][8], u[BN_U][8];
#pragma unroll
    for (int k = 0; k < BN_U; ++k)
      if (k < nrows) Vec8<T>::load(Y + (size_t)(base + k * L.rpp) * a.ldy, v[k]);
    if constexpr (RES != RES_NONE) {
#pragma unroll
      for (int k = 0; k < BN_U; ++k)
        if (k < nrows) Vec8<T>::load(RS + res_row(base + k * L.rpp) * ldr, u[k]);
    }
#pragma unroll
    for (int k = 0; k < BN_U; ++k) {
      if (k >= nrows) continue;
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float x = __builtin_fmaf(v[k][e] - mu[e], sc[e], be[e]);
        if constexpr (RES == RES_BN2) x = __builtin_fmaf(u[k][e] - mu2[e], sc2[e], be2[e]) + x;
        else if constexpr (RES != RES_NONE) x = u[k][e] + x;
        o[e] = RELU ? fmaxf(x, 0.f) : x;
      }
      BN_STORE8(TO, O + (size_t)(base + k * L.rpp) * a.ldo, o);
      if (RELU && a.mask) {   // bits of the value as stored (> 0 after rounding)
        uint32_t bits = 0;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const bool pos = sizeof(TO) == 2 ? TypeOps<TO>::to_f(TypeOps<TO>::from_f(o[e])) > 0.f : o[e] > 0.f;
          bits |= (uint32_t)pos << e;
        }
        a.mask[(size_t)(base + k * L.rpp) * (a.C >> 3) + L.cg] = (uint8_t)bits;
      }
    }
  };
  long base = (long)blockIdx.x * step + L.rl;
  for (; base + (BN_U - 1) * L.rpp < a.M; base += (long)gridDim.x * step) body(base, BN_U);
  if (base < a.M) body(base, (int)((a.M - base + L.rpp - 1) / L.rpp));
}

// raw 8-element row chunk: loaded first for every row of a group, converted afterwards, so
// that all of a group's loads are in flight together
template <typename T> struct Raw8;
template <> struct Raw8<bf16_t> {
  uint4 u;
  __device__ __forceinline__ void load(const bf16_t* p) { u = *(const uint4*)p; }
  __device__ __forceinline__ void cvt(float* o) const {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) { o[2 * i] = bf2f((bf16_t)(w[i] & 0xffff)); o[2 * i + 1] = bf2f((bf16_t)(w[i] >> 16)); }
  }
};
template <> struct Raw8<f16_t> {
  uint4 u;
  __device__ __forceinline__ void load(const f16_t* p) { u = *(const uint4*)p; }
  __device__ __forceinline__ void cvt(float* o) const { Half<f16_t>::unpack(u, o); }
};
template <> struct Raw8<float> {
  float4 a, b;
  __device__ __forceinline__ void load(const float* p) { a = *(const float4*)p; b = *(const float4*)(p + 4); }
  __device__ __forceinline__ void cvt(float* o) const {
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
  }
};

// masked incoming gradient for n rows (dz * [z > 0] * dzscale) and the matching y rows
template <typename T, typename TZ, int HZ, int HS, bool FULL>
__device__ __forceinline__ void bwd_load(const BnBwdArgs& a, int c0, long base, int rpp, int nrows,
                                         float (&dz)[BN_U][8], float (&y)[BN_U][8]) {
  if constexpr (FULL) nrows = BN_U;
  const TZ* DZ = (const TZ*)a.dz + c0;
  const TZ* Z = (const TZ*)a.z + c0;
  const T* Y = (const T*)a.y + c0;
  Raw8<TZ> rdz[BN_U], rz[BN_U];
  Raw8<T> ry[BN_U];
  uint32_t mk[BN_U];
  const int cg = c0 >> 3, cgn = a.C >> 3;
#pragma unroll
  for (int k = 0; k < BN_U; ++k) {
    if (FULL || k < nrows) {
      const size_t m = (size_t)(base + k * rpp);
      rdz[k].load(DZ + m * a.lddz);
      ry[k].load(Y + m * a.ldy);
      if constexpr (HZ == 1) rz[k].load(Z + m * a.ldz);
      if constexpr (HZ == 2) mk[k] = a.mask[m * cgn + cg];
    }
  }
  __builtin_amdgcn_sched_barrier(0);   // keep the group's loads ahead of every conversion
  float sft[8];
  if constexpr (HS == 2) ld8(a.dshift, c0, sft);
#pragma unroll
  for (int k = 0; k < BN_U; ++k) {
    if (FULL || k < nrows) {
      rdz[k].cvt(dz[k]);
      ry[k].cvt(y[k]);
      if constexpr (HS == 2) {
#pragma unroll
        for (int e = 0; e < 8; ++e) dz[k][e] += sft[e];
      }
      if constexpr (HZ == 1) {
        float z[8];
        rz[k].cvt(z);
#pragma unroll
        for (int e = 0; e < 8; ++e) dz[k][e] = z[e] > 0.f ? dz[k][e] : 0.f;
      } else if constexpr (HZ == 2) {
#pragma unroll
        for (int e = 0; e < 8; ++e) dz[k][e] = (mk[k] >> e) & 1u ? dz[k][e] : 0.f;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) { dz[k][e] = 0.f; y[k][e] = 0.f; }
    }
  }
  if constexpr (HS == 1) {
    float ds[8];
    ld8(a.dzscale, c0, ds);
#pragma unroll
    for (int k = 0; k < BN_U; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) dz[k][e] *= ds[e];
  }
}

// per row block partial (sum dyhat, sum dyhat*xhat); rows of block b: [b*rows_per, ...)
// HS: 1 = dz times dzscale, 2 = dz plus dshift before the gate; HD: the gated gradient (dyhat)
// is also stored (the linear BN-backward fold's masked gradient, read by the data and weight
// gradients in place of the apply's output)
// CS: also the column sums of the forward output (BnBwdArgs::cs_part), recomputed per element
// exactly as bn_apply8_kernel forms it (fma, ReLU, rounding to T)
template <typename T, typename TZ, int HZ, int HS, int HD = 0, int CS = 0>
__global__ __launch_bounds__(256) void bn_bwd_reduce8_kernel(BnBwdArgs a) {
  __shared__ float sh[CS ? 3 : 2][256 * 8];
  const RowLane L = row_lane(a.C / 8);
  const int c0 = (L.act ? L.cg : 0) * 8;
  const long rows_per = (a.M + a.rb - 1) / a.rb;
  const long r0 = (long)blockIdx.x * rows_per;
  const long r1 = (r0 + rows_per < a.M) ? r0 + rows_per : a.M;
  float s1[8], s2[8], mu[8], inv[8];
  // one accumulator set per row slot k: the U rows of a group stay independent (no loop
  // rerolling), so their loads are issued together
  float t1[BN_U][8], t2[BN_U][8];
  float s3[8], fsc[8], fbe[8];
#pragma unroll
  for (int k = 0; k < BN_U; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) { t1[k][e] = 0.f; t2[k][e] = 0.f; }
#pragma unroll
  for (int e = 0; e < 8; ++e) s3[e] = 0.f;
  if (L.act) {
    ld8(a.mean, c0, mu); ld8(a.invstd, c0, inv);
    if constexpr (CS) { ld8(a.scale, c0, fsc); ld8(a.beta, c0, fbe); }
    auto acc = [&](long base, int nrows, auto full) {
      float dz[BN_U][8], y[BN_U][8];
      bwd_load<T, TZ, HZ, HS, decltype(full)::value>(a, c0, base, L.rpp, nrows, dz, y);
      if constexpr (HD) {
        T* DH = (T*)a.dyhat + c0;
#pragma unroll
        for (int k = 0; k < BN_U; ++k)
          if (decltype(full)::value || k < nrows) BN_STORE8(T, DH + (size_t)(base + k * L.rpp) * a.lddyhat, dz[k]);
      }
#pragma unroll
      for (int k = 0; k < BN_U; ++k)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          t1[k][e] += dz[k][e];
          t2[k][e] += dz[k][e] * ((y[k][e] - mu[e]) * inv[e]);
        }
      if constexpr (CS) {   // rows past the block are zero in y: skip them, not their value
#pragma unroll
        for (int k = 0; k < BN_U; ++k)
          if (decltype(full)::value || k < nrows)
#pragma unroll
            for (int e = 0; e < 8; ++e)
              s3[e] += TypeOps<T>::to_f(TypeOps<T>::from_f(fmaxf(__builtin_fmaf(y[k][e] - mu[e], fsc[e], fbe[e]), 0.f)));
      }
    };
    long base = r0 + L.rl;
    for (; base + (BN_U - 1) * L.rpp < r1; base += (long)L.rpp * BN_U) acc(base, BN_U, std::true_type{});
    if (base < r1) acc(base, (int)((r1 - base + L.rpp - 1) / L.rpp), std::false_type{});
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    s1[e] = (t1[0][e] + t1[1][e]) + (t1[2][e] + t1[3][e]);
    s2[e] = (t2[0][e] + t2[1][e]) + (t2[2][e] + t2[3][e]);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sh[0][threadIdx.x * 8 + e] = s1[e];
    sh[1][threadIdx.x * 8 + e] = s2[e];
    if constexpr (CS) sh[CS ? 2 : 0][threadIdx.x * 8 + e] = s3[e];
  }
  __syncthreads();
  if (L.act && L.rl == 0) {
    const int cg_b = a.C / 8 >= 256 ? 256 : a.C / 8;
    for (int r = 1; r < L.rpp; ++r) {
      const int t = r * cg_b + threadIdx.x;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[e] += sh[0][t * 8 + e]; s2[e] += sh[1][t * 8 + e];
        if constexpr (CS) s3[e] += sh[CS ? 2 : 0][t * 8 + e];
      }
    }
    float* o = a.part + 2 * ((size_t)blockIdx.x * a.C + c0);
#pragma unroll
    for (int e = 0; e < 8; e += 2)
      *(float4*)(o + 2 * e) = make_float4(s1[e], s2[e], s1[e + 1], s2[e + 1]);
    if constexpr (CS) {
      float* q = a.cs_part + (size_t)blockIdx.x * a.C + c0;
      *(float4*)q = make_float4(s3[0], s3[1], s3[2], s3[3]);
      *(float4*)(q + 4) = make_float4(s3[4], s3[5], s3[6], s3[7]);
    }
  }
}

template <typename T, typename TZ, int HZ, int HS, int HD>
__global__ __launch_bounds__(256) void bn_bwd_apply8_kernel(BnBwdArgs a) {
  const RowLane L = row_lane(a.C / 8);
  if (!L.act) return;
  const int c0 = L.cg * 8;
  float mu[8], inv[8], sc[8], sdy[8], sdyx[8];
  ld8(a.mean, c0, mu); ld8(a.invstd, c0, inv); ld8(a.scale, c0, sc);
  ld8(a.sdy, c0, sdy); ld8(a.sdyx, c0, sdyx);
  T* DY = (T*)a.dy + c0;
  T* DH = (T*)a.dyhat + c0;
  float ds[8];
  if constexpr (HS == 1) ld8(a.dzscale, c0, ds);
  const long step = (long)L.rpp * BN_U;
  auto body = [&](long base, int nrows, auto full) {
    float dz[BN_U][8], y[BN_U][8];
    if constexpr (decltype(full)::value) nrows = BN_U;
    bwd_load<T, TZ, HZ, HS == 2 ? 2 : 0, decltype(full)::value>(a, c0, base, L.rpp, nrows, dz, y);
#pragma unroll
    for (int k = 0; k < BN_U; ++k) {
      if (k >= nrows) continue;
      const size_t m = (size_t)(base + k * L.rpp);
      // dyhat: the masked gradient before the per-channel factor (group norm's gamma)
      if constexpr (HD) BN_STORE8(T, DH + m * a.lddyhat, dz[k]);
      if constexpr (HS == 1) {
#pragma unroll
        for (int e = 0; e < 8; ++e) dz[k][e] *= ds[e];
      }
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xh = (y[k][e] - mu[e]) * inv[e];
        o[e] = sc[e] * (dz[k][e] - sdy[e] - xh * sdyx[e]);
      }
      BN_STORE8(T, DY + m * a.lddy, o);
    }
  };
  long base = (long)blockIdx.x * step + L.rl;
  for (; base + (BN_U - 1) * L.rpp < a.M; base += (long)gridDim.x * step) body(base, BN_U, std::true_type{});
  if (base < a.M) body(base, (int)((a.M - base + L.rpp - 1) / L.rpp), std::false_type{});
}

// dual reduce: (sum dyhat, sum dyhat*xhat) for two BN layers gated by the same dz / bits, dz
// and the bits read once; two rows in flight per thread (the second y and accumulator set
// would push four past 256 VGPRs), rows added in order, partials in each layer's layout
template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_reduce8_dual_kernel(BnBwdArgs a) {
  constexpr int U = 2;
  __shared__ float sh[3][256 * 8];
  const RowLane L = row_lane(a.C / 8);
  const int c0 = (L.act ? L.cg : 0) * 8;
  const long rows_per = (a.M + a.rb - 1) / a.rb;
  const long r0 = (long)blockIdx.x * rows_per;
  const long r1 = (r0 + rows_per < a.M) ? r0 + rows_per : a.M;
  float s1[8], s2[8], s3[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; s3[e] = 0.f; }
  if (L.act) {
    float mu[8], inv[8], mu2[8], inv2[8];
    ld8(a.mean, c0, mu); ld8(a.invstd, c0, inv); ld8(a.mean2, c0, mu2); ld8(a.invstd2, c0, inv2);
    const T* DZ = (const T*)a.dz + c0;
    const T* Y = (const T*)a.y + c0;
    const T* Y2 = (const T*)a.y2 + c0;
    const int cg = c0 >> 3, cgn = a.C >> 3;
    for (long base = r0 + L.rl; base < r1; base += (long)L.rpp * U) {
      Raw8<T> rdz[U], ry[U], ry2[U];
      uint32_t mk[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const long m = base + k * L.rpp;
        if (m < r1) {
          rdz[k].load(DZ + (size_t)m * a.lddz);
          ry[k].load(Y + (size_t)m * a.ldy);
          ry2[k].load(Y2 + (size_t)m * a.ldy2);
          mk[k] = a.mask[(size_t)m * cgn + cg];
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < U; ++k) {
        if (base + k * L.rpp >= r1) continue;
        float dz[8], y[8], y2[8];
        rdz[k].cvt(dz); ry[k].cvt(y); ry2[k].cvt(y2);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = (mk[k] >> e) & 1u ? dz[e] : 0.f;
          s1[e] += d;
          s2[e] += d * ((y[e] - mu[e]) * inv[e]);
          s3[e] += d * ((y2[e] - mu2[e]) * inv2[e]);
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sh[0][threadIdx.x * 8 + e] = s1[e];
    sh[1][threadIdx.x * 8 + e] = s2[e];
    sh[2][threadIdx.x * 8 + e] = s3[e];
  }
  __syncthreads();
  if (L.act && L.rl == 0) {
    const int cg_b = a.C / 8 >= 256 ? 256 : a.C / 8;
    for (int r = 1; r < L.rpp; ++r) {
      const int t = r * cg_b + threadIdx.x;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[e] += sh[0][t * 8 + e];
        s2[e] += sh[1][t * 8 + e];
        s3[e] += sh[2][t * 8 + e];
      }
    }
    float* o = a.part + 2 * ((size_t)blockIdx.x * a.C + c0);
    float* o2 = a.part2 + 2 * ((size_t)blockIdx.x * a.C + c0);
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      *(float4*)(o + 2 * e) = make_float4(s1[e], s2[e], s1[e + 1], s2[e + 1]);
      *(float4*)(o2 + 2 * e) = make_float4(s1[e], s3[e], s1[e + 1], s3[e + 1]);
    }
  }
}

// dual apply: dy = scale (dyhat - sdy - xhat sdyx) for both layers from one dz / bits read
template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_apply8_dual_kernel(BnBwdArgs a) {
  constexpr int U = 2;
  const RowLane L = row_lane(a.C / 8);
  if (!L.act) return;
  const int c0 = L.cg * 8;
  float mu[8], inv[8], sc[8], sdy[8], sdyx[8], mu2[8], inv2[8], sc2[8], sdy2[8], sdyx2[8];
  ld8(a.mean, c0, mu); ld8(a.invstd, c0, inv); ld8(a.scale, c0, sc);
  ld8(a.sdy, c0, sdy); ld8(a.sdyx, c0, sdyx);
  ld8(a.mean2, c0, mu2); ld8(a.invstd2, c0, inv2); ld8(a.scale2, c0, sc2);
  ld8(a.sdy2, c0, sdy2); ld8(a.sdyx2, c0, sdyx2);
  const T* DZ = (const T*)a.dz + c0;
  const T* Y = (const T*)a.y + c0;
  const T* Y2 = (const T*)a.y2 + c0;
  T* DY = (T*)a.dy + c0;
  T* DY2 = (T*)a.dy2 + c0;
  const int cg = c0 >> 3, cgn = a.C >> 3;
  const long step = (long)L.rpp * U;
  for (long base = (long)blockIdx.x * step + L.rl; base < a.M; base += (long)gridDim.x * step) {
    Raw8<T> rdz[U], ry[U], ry2[U];
    uint32_t mk[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const long m = base + k * L.rpp;
      if (m < a.M) {
        rdz[k].load(DZ + (size_t)m * a.lddz);
        ry[k].load(Y + (size_t)m * a.ldy);
        ry2[k].load(Y2 + (size_t)m * a.ldy2);
        mk[k] = a.mask[(size_t)m * cgn + cg];
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const long m = base + k * L.rpp;
      if (m >= a.M) continue;
      float dz[8], y[8], y2[8], o[8], o2[8];
      rdz[k].cvt(dz); ry[k].cvt(y); ry2[k].cvt(y2);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = (mk[k] >> e) & 1u ? dz[e] : 0.f;
        o[e] = sc[e] * (d - sdy[e] - ((y[e] - mu[e]) * inv[e]) * sdyx[e]);
        o2[e] = sc2[e] * (d - sdy2[e] - ((y2[e] - mu2[e]) * inv2[e]) * sdyx2[e]);
      }
      BN_STORE8(T, DY + (size_t)m * a.lddy, o);
      BN_STORE8(T, DY2 + (size_t)m * a.lddy2, o2);
    }
  }
}

dim3 grid8(long M, int C) {
  const int cg_n = C / 8;
  const int rpp = cg_n >= 256 ? 1 : 256 / cg_n;
  long g = (M + (long)rpp * BN_U - 1) / ((long)rpp * BN_U);
  if (g > 2048) g = 2048;
  return dim3((unsigned)(g < 1 ? 1 : g), cg_n > 256 ? (unsigned)ceil_div(cg_n, 256) : 1u);
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
  if (v8) {
    const int res = a.y2 ? RES_BN2 : (a.res ? (a.rs > 1 ? RES_SUB : RES_PLAIN) : RES_NONE);
    const dim3 g = grid8(a.M, a.C);
#define BN_APPLY_CASE(R)                                                                      \
    if (res == R) {                                                                           \
      if (a.relu) hipLaunchKernelGGL((bn_apply8_kernel<T, TO, R, 1>), g, dim3(256), 0, s, a); \
      else hipLaunchKernelGGL((bn_apply8_kernel<T, TO, R, 0>), g, dim3(256), 0, s, a);        \
    }
    BN_APPLY_CASE(RES_NONE) BN_APPLY_CASE(RES_PLAIN) BN_APPLY_CASE(RES_SUB) BN_APPLY_CASE(RES_BN2)
#undef BN_APPLY_CASE
  }
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
  if (a.mask && !bwd_v8<T, TZ>(a)) return hipErrorInvalidValue;   // bits exist on the 8-wide path only
  const bool rdh = a.reduce_dyhat && a.dyhat;
  if ((a.dshift || rdh) && (!a.mask || a.dzscale || !bwd_v8<T, TZ>(a))) return hipErrorInvalidValue;
  if (a.cs_part && (!a.dshift || rdh || !a.beta || sizeof(T) != 2)) return hipErrorInvalidValue;
  if (bwd_v8<T, TZ>(a)) {
    const int cg_n = a.C / 8;
    const dim3 g(a.rb, cg_n > 256 ? ceil_div(cg_n, 256) : 1);
    if (a.cs_part) hipLaunchKernelGGL((bn_bwd_reduce8_kernel<T, TZ, 2, 2, 0, 1>), g, dim3(256), 0, s, a);
    else if (a.mask && a.dshift && rdh) hipLaunchKernelGGL((bn_bwd_reduce8_kernel<T, TZ, 2, 2, 1>), g, dim3(256), 0, s, a);
    else if (a.mask && a.dshift) hipLaunchKernelGGL((bn_bwd_reduce8_kernel<T, TZ, 2, 2, 0>), g, dim3(256), 0, s, a);
    else if (a.mask && rdh) hipLaunchKernelGGL((bn_bwd_reduce8_kernel<T, TZ, 2, 0, 1>), g, dim3(256), 0, s, a);
    else if (a.mask) hipLaunchKernelGGL((bn_bwd_reduce8_kernel<T, TZ, 2, 0>), g, dim3(256), 0, s, a);
    else if (a.z && a.dzscale) hipLaunchKernelGGL((bn_bwd_reduce8_kernel<T, TZ, 1, 1>), g, dim3(256), 0, s, a);
    else if (a.z) hipLaunchKernelGGL((bn_bwd_reduce8_kernel<T, TZ, 1, 0>), g, dim3(256), 0, s, a);
    else if (a.dzscale) hipLaunchKernelGGL((bn_bwd_reduce8_kernel<T, TZ, 0, 1>), g, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((bn_bwd_reduce8_kernel<T, TZ, 0, 0>), g, dim3(256), 0, s, a);
  }
  else hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, TZ, 1>), dim3(a.rb), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <typename T, typename TZ>
hipError_t bwd_apply_t(const BnBwdArgs& a, hipStream_t s) {
  if (a.mask && !bwd_v8<T, TZ>(a)) return hipErrorInvalidValue;
  if (a.dshift && (!a.mask || a.dzscale || a.dyhat || !bwd_v8<T, TZ>(a))) return hipErrorInvalidValue;
  if (bwd_v8<T, TZ>(a)) {
    const dim3 g = grid8(a.M, a.C);
    const int key = (a.z ? 4 : 0) | (a.dzscale ? 2 : 0) | (a.dyhat ? 1 : 0);
    if (a.dshift) {
      hipLaunchKernelGGL((bn_bwd_apply8_kernel<T, TZ, 2, 2, 0>), g, dim3(256), 0, s, a);
      return hipGetLastError();
    }
    if (a.mask) {   // ReLU bits; dzscale with them only under group norm (gamma)
      if (a.dzscale) {
        if (a.dyhat) hipLaunchKernelGGL((bn_bwd_apply8_kernel<T, TZ, 2, 1, 1>), g, dim3(256), 0, s, a);
        else hipLaunchKernelGGL((bn_bwd_apply8_kernel<T, TZ, 2, 1, 0>), g, dim3(256), 0, s, a);
      } else if (a.dyhat) {
        hipLaunchKernelGGL((bn_bwd_apply8_kernel<T, TZ, 2, 0, 1>), g, dim3(256), 0, s, a);
      } else {
        hipLaunchKernelGGL((bn_bwd_apply8_kernel<T, TZ, 2, 0, 0>), g, dim3(256), 0, s, a);
      }
      return hipGetLastError();
    }
    switch (key) {
      case 0: hipLaunchKernelGGL((bn_bwd_apply8_kernel<T, TZ, 0, 0, 0>), g, dim3(256), 0, s, a); break;
      case 1: hipLaunchKernelGGL((bn_bwd_apply8_kernel<T, TZ, 0, 0, 1>), g, dim3(256), 0, s, a); break;
      case 2: hipLaunchKernelGGL((bn_bwd_apply8_kernel<T, TZ, 0, 1, 0>), g, dim3(256), 0, s, a); break;
      case 3: hipLaunchKernelGGL((bn_bwd_apply8_kernel<T, TZ, 0, 1, 1>), g, dim3(256), 0, s, a); break;
      case 4: hipLaunchKernelGGL((bn_bwd_apply8_kernel<T, TZ, 1, 0, 0>), g, dim3(256), 0, s, a); break;
      case 5: hipLaunchKernelGGL((bn_bwd_apply8_kernel<T, TZ, 1, 0, 1>), g, dim3(256), 0, s, a); break;
      case 6: hipLaunchKernelGGL((bn_bwd_apply8_kernel<T, TZ, 1, 1, 0>), g, dim3(256), 0, s, a); break;
      default: hipLaunchKernelGGL((bn_bwd_apply8_kernel<T, TZ, 1, 1, 1>), g, dim3(256), 0, s, a); break;
    }
  }
  else hipLaunchKernelGGL((bn_bwd_apply_kernel<T, TZ, 1>), dim3(grid_for(a.M * a.C)), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_bn_stats_finalize(const float* tile_part, long M, int C, int tile_rows,
                                    float* scratch, const float* gamma, BnState st,
                                    hipStream_t s, float* pack) {
  int ntiles = ceil_div(M, tile_rows);
  (void)scratch;
  hipLaunchKernelGGL(bn_stats_final_kernel, dim3(ceil_div(C, FIN_CH)), dim3(FIN_CH * FIN_LANES), 0,
                     s, tile_part, M, C, tile_rows, ntiles, gamma, st, pack);
  return hipGetLastError();
}

hipError_t launch_bn_sync_unpack(const float* pack, int C, float inv_world, const float* gamma,
                                 BnState st, hipStream_t s) {
  hipLaunchKernelGGL(bn_sync_unpack_kernel, dim3(ceil_div(C, 64)), dim3(64), 0, s, pack, C,
                     inv_world, gamma, st);
  return hipGetLastError();
}

hipError_t launch_bn_infer_finalize_all(const BnInferJob* jobs, int n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(bn_infer_finalize_all_kernel, dim3(n), dim3(256), 0, s, jobs);
  return hipGetLastError();
}

hipError_t launch_bn_infer_finalize(const float* mov_mean, const float* mov_var, int C,
                                    const float* gamma, BnState st, hipStream_t s) {
  hipLaunchKernelGGL(bn_infer_finalize_kernel, dim3(ceil_div(C, 64)), dim3(64), 0, s, mov_mean,
                     mov_var, C, gamma, st);
  return hipGetLastError();
}

hipError_t launch_bn_apply(int dtype, int out_f32, const BnApplyArgs& a, hipStream_t s) {
  if (dtype == SEG_BF16) {
    if (out_f32) return apply_t<bf16_t, float>(a, s);
    return apply_t<bf16_t, bf16_t>(a, s);
  }
  if (dtype == SEG_F16) {
    if (out_f32) return apply_t<f16_t, float>(a, s);
    return apply_t<f16_t, f16_t>(a, s);
  }
  return apply_t<float, float>(a, s);
}

int bn_bwd_rowblocks(long M, int C) {
  // ~1024 blocks, each >= 64 rows
  const long cap = 1024;
  long rb = (M + 63) / 64;
  if (rb > cap) rb = cap;
  (void)C;
  return (int)(rb < 1 ? 1 : rb);
}

hipError_t launch_bn_bwd_reduce(int dtype, int dz_f32, const BnBwdArgs& a, hipStream_t s) {
  if (dtype == SEG_BF16) {
    if (dz_f32) return bwd_reduce_t<bf16_t, float>(a, s);
    return bwd_reduce_t<bf16_t, bf16_t>(a, s);
  }
  if (dtype == SEG_F16) {
    if (dz_f32) return bwd_reduce_t<f16_t, float>(a, s);
    return bwd_reduce_t<f16_t, f16_t>(a, s);
  }
  return bwd_reduce_t<float, float>(a, s);
}

hipError_t launch_bn_bwd_finalize(const float* part, int rb, long M, int C, BnState st,
                                  float* dgamma, float* dbeta, hipStream_t s, int frozen) {
  hipLaunchKernelGGL(bn_bwd_final_kernel, dim3(ceil_div(C, FIN_CH)), dim3(FIN_CH * FIN_LANES), 0, s,
                     part, rb, M, C, st, dgamma, dbeta, frozen);
  return hipGetLastError();
}

hipError_t launch_bn_bwd_apply(int dtype, int dz_f32, const BnBwdArgs& a, hipStream_t s) {
  if (dtype == SEG_BF16) {
    if (dz_f32) return bwd_apply_t<bf16_t, float>(a, s);
    return bwd_apply_t<bf16_t, bf16_t>(a, s);
  }
  if (dtype == SEG_F16) {
    if (dz_f32) return bwd_apply_t<f16_t, float>(a, s);
    return bwd_apply_t<f16_t, f16_t>(a, s);
  }
  return bwd_apply_t<float, float>(a, s);
}

template <typename T>
bool dual_ok(const BnBwdArgs& a) {
  return a.mask && !a.z && !a.dzscale && !a.dyhat && a.C % 8 == 0 && a.lddz % 8 == 0 &&
         a.ldy % 8 == 0 && a.ldy2 % 8 == 0 && a.lddy % 8 == 0 && a.lddy2 % 8 == 0 &&
         (uintptr_t)a.dz % 16 == 0;
}

hipError_t launch_bn_bwd_reduce_dual(int dtype, const BnBwdArgs& a, hipStream_t s) {
  const int cg_n = a.C / 8;
  const dim3 g(a.rb, cg_n > 256 ? ceil_div(cg_n, 256) : 1);
  if (dtype == SEG_BF16) {
    if (!dual_ok<bf16_t>(a)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(bn_bwd_reduce8_dual_kernel<bf16_t>, g, dim3(256), 0, s, a);
  } else if (dtype == SEG_F16) {
    if (!dual_ok<f16_t>(a)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(bn_bwd_reduce8_dual_kernel<f16_t>, g, dim3(256), 0, s, a);
  } else {
    if (!dual_ok<float>(a)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(bn_bwd_reduce8_dual_kernel<float>, g, dim3(256), 0, s, a);
  }
  return hipGetLastError();
}

hipError_t launch_bn_bwd_apply_dual(int dtype, const BnBwdArgs& a, hipStream_t s) {
  const dim3 g = grid8(a.M, a.C);
  if (dtype == SEG_BF16) {
    if (!dual_ok<bf16_t>(a)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(bn_bwd_apply8_dual_kernel<bf16_t>, g, dim3(256), 0, s, a);
  } else if (dtype == SEG_F16) {
    if (!dual_ok<f16_t>(a)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(bn_bwd_apply8_dual_kernel<f16_t>, g, dim3(256), 0, s, a);
  } else {
    if (!dual_ok<float>(a)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(bn_bwd_apply8_dual_kernel<float>, g, dim3(256), 0, s, a);
  }
  return hipGetLastError();
}

hipError_t launch_moving_update(float* mov_mean, float* mov_var, const float* bmean,
                                const float* bvar, int n, float decay, hipStream_t s) {
  hipLaunchKernelGGL(moving_update_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, s, mov_mean,
                     mov_var, bmean, bvar, n, decay);
  return hipGetLastError();
}
