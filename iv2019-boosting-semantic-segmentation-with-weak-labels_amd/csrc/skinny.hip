// Skinny 1x1 convolutions: y[m][n] = sum_k x[m][k] w[n][k] with one side tiny. These are the
// hierarchical heads' logits convs (hierarchical.py:78-83: 256 -> 14 / 7 / 3 channels) and their
// data gradients (14 / 7 / 3 -> 256), which the 16-bit tile kernels cannot take (channel counts
// not multiples of 8 / 64). Both are HBM-bound GEMVs in disguise, so neither is tiled: the
// narrow output one puts the whole N on one MFMA column block, the narrow reduction one is
// plain VALU with the weights held in registers.
//
//  narrow N (N <= 16, K % 32 == 0, K <= 512): one v_mfma_f32_16x16x32 per 16 rows x 32 K, the
//    weights as the MFMA's first operand (rows n >= N zero) so each lane ends with 4
//    consecutive channels of one pixel: a 16-row group's output is one contiguous 512-B store
//    (ldy = 16). Blocks of 4 waves own 128-row tiles and reduce the tile's per-channel
//    (sum, M2) BN partials from the fp32 accumulators (two-pass through LDS), the layout the
//    BN statistics finalize reads (conv_nt_stat_rows = 128).
//  narrow K (K <= 16, N % 8 == 0): a thread owns 8 output channels (weights in registers) and
//    walks rows; each row's K inputs are one or two 16-B loads shared by the row's lanes.
#include "conv.h"

namespace {

constexpr int SK_THREADS = 256;
constexpr int SK_ROWS = 128;   // rows per block = BN-statistics partial rows

template <typename E>
__global__ __launch_bounds__(SK_THREADS) void skinny_narrow_n_kernel(ConvArgs a) {
  typedef typename Half<E>::V V;
  __shared__ float sh[SK_ROWS][17];
  __shared__ float part[16][17];
  __shared__ float sum_s[16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  const long M = (long)a.N * a.Ho * a.Wo;
  const int K = a.C, N = a.Co, nkb = K / 32;
  const long row0 = (long)blockIdx.x * SK_ROWS;
  const E* X = (const E*)a.x;
  const E* Wt = (const E*)a.w;
  E* Y = (E*)a.y;
  // weights: lane supplies W[n = lr][k = 32 kb + 8 lq .. + 8], one 16-B load each (rows
  // 16-B aligned: conv_skinny_ok); round 5: these were 8 two-byte loads each, 128 per lane
  // issued before any pixel load (the l1 logits conv 46 us for 67 MB read)
  V wv[16];
  const V vzero = {};
#pragma unroll
  for (int kb = 0; kb < 16; ++kb)
    if (kb < nkb) wv[kb] = lr < N ? *(const V*)(Wt + (size_t)lr * a.ldw + kb * 32 + lq * 8) : vzero;
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int r = wave * 32 + g * 16 + lr;   // row of this lane inside the tile
    const long m = row0 + r;
    const long mc = m < M ? m : M - 1;
    V xv[16];
#pragma unroll
    for (int kb = 0; kb < 16; ++kb)
      if (kb < nkb) xv[kb] = *(const V*)(X + (size_t)mc * a.ldx + kb * 32 + lq * 8);
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < 16; ++kb)
      if (kb < nkb) acc = Half<E>::mma(wv[kb], xv[kb], acc);
    // lane: pixel m, channels 4 lq .. 4 lq + 3 (a partial last group writes zeros up to the
    // next multiple of 4, inside ldy)
    if (m < M && lq * 4 < N) {
      uint32_t w2[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) w2[h] = pack2<E>(acc[2 * h], acc[2 * h + 1]);
      *(uint2*)(Y + (size_t)m * a.ldy + lq * 4) = make_uint2(w2[0], w2[1]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) sh[r][lq * 4 + q] = acc[q];
  }
  if (!a.stats) return;
  __syncthreads();
  // per-channel (sum, M2) of the tile's valid rows: 16 segments of 8 rows x 16 channels
  const int c = threadIdx.x & 15, seg = threadIdx.x >> 4;
  const int nrows = (int)(M - row0 < SK_ROWS ? M - row0 : SK_ROWS);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = seg * 8 + i;
    s += r < nrows ? sh[r][c] : 0.f;
  }
  part[seg][c] = s;
  __syncthreads();
  if (threadIdx.x < 16) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += part[k][threadIdx.x];
    sum_s[threadIdx.x] = t;
  }
  __syncthreads();
  const float mu = sum_s[c] / (float)nrows;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = seg * 8 + i;
    const float d = sh[r][c] - mu;
    q += r < nrows ? d * d : 0.f;
  }
  __syncthreads();   // every thread has read part[] (the mean pass) before it is reused
  part[seg][c] = q;
  __syncthreads();
  if (threadIdx.x < N) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += part[k][threadIdx.x];
    float* dst = a.stats + 2 * ((size_t)blockIdx.x * N + threadIdx.x);
    dst[0] = sum_s[threadIdx.x];
    dst[1] = t;
  }
}

// 16-bit pair dot product with fp32 accumulation (v_dot2c_f32_bf16 / _f16)
template <typename E> __device__ __forceinline__ float dot2(uint32_t x, uint32_t w, float acc);
template <> __device__ __forceinline__ float dot2<bf16_t>(uint32_t x, uint32_t w, float acc) {
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(b2, x), __builtin_bit_cast(b2, w), acc, false);
}
template <> __device__ __forceinline__ float dot2<f16_t>(uint32_t x, uint32_t w, float acc) {
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  return __builtin_amdgcn_fdot2(__builtin_bit_cast(h2, x), __builtin_bit_cast(h2, w), acc, false);
}

template <typename E, int K>
__global__ __launch_bounds__(SK_THREADS) void skinny_narrow_k_kernel(ConvArgs a) {
  constexpr int KP = K / 2;   // 16-bit pairs per row
  const long M = (long)a.N * a.Ho * a.Wo;
  const int nch = a.Co / 8;
  const int per = SK_THREADS / nch;   // rows per block step (the host picks N with nch | 256)
  const int cg = threadIdx.x % nch, rl = threadIdx.x / nch;
  const E* X = (const E*)a.x;
  const uint16_t* Wt = (const uint16_t*)a.w;
  E* Y = (E*)a.y;
  // the block's weights (Co rows of ldw 16-bit values) through LDS as packed pairs [k/2][n]:
  // read once per block by consecutive threads, then each thread takes its 8 channels per pair
  // as two 16-B LDS reads; the rows are v_dot2 products (two 16-bit products per instruction,
  // fp32 accumulation). Round 5: each thread read its 8 x K weights as two-byte global loads,
  // ~8 x K of them before its first pixel, and ran one fp32 FMA per product: the l1 logits
  // data gradient took 76 us for 67 MB written
  extern __shared__ uint32_t wsh[];   // [KP][Co]
  for (int i = threadIdx.x; i < KP * a.Co; i += SK_THREADS) {
    const int kp = i / a.Co, n = i - kp * a.Co;
    const int k0 = 2 * kp, k1 = 2 * kp + 1;
    const uint32_t lo = k0 < a.C ? Wt[(size_t)n * a.ldw + k0] : 0u;
    const uint32_t hi = k1 < a.C ? Wt[(size_t)n * a.ldw + k1] : 0u;
    wsh[i] = lo | (hi << 16);
  }
  __syncthreads();
  if (rl >= per) return;
  uint32_t w[8][KP];
#pragma unroll
  for (int kp = 0; kp < KP; ++kp) {
    const uint4 lo = *(const uint4*)(wsh + kp * a.Co + cg * 8);
    const uint4 hi = *(const uint4*)(wsh + kp * a.Co + cg * 8 + 4);
    w[0][kp] = lo.x; w[1][kp] = lo.y; w[2][kp] = lo.z; w[3][kp] = lo.w;
    w[4][kp] = hi.x; w[5][kp] = hi.y; w[6][kp] = hi.z; w[7][kp] = hi.w;
  }
  // input channels >= C (the pixel's padding up to ldx) are masked out of the products
  uint32_t xm[KP];
#pragma unroll
  for (int kp = 0; kp < KP; ++kp)
    xm[kp] = 2 * kp + 1 < a.C ? 0xffffffffu : (2 * kp < a.C ? 0x0000ffffu : 0u);
  // rows m, m + per, m + 2 per, m + 3 per per trip: the four rows' loads go out together
  const long step = (long)gridDim.x * per * 4;
  for (long m0 = (long)blockIdx.x * per * 4 + rl; m0 < M; m0 += step) {
    uint32_t x[4][KP];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long m = m0 + (long)u * per;
      const long mc = m < M ? m : M - 1;
#pragma unroll
      for (int q = 0; q < KP / 4; ++q) {
        const uint4 v = *(const uint4*)(X + (size_t)mc * a.ldx + q * 8);
        x[u][4 * q] = v.x; x[u][4 * q + 1] = v.y; x[u][4 * q + 2] = v.z; x[u][4 * q + 3] = v.w;
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long m = m0 + (long)u * per;
      if (m >= M) break;
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float s = 0.f;
#pragma unroll
        for (int kp = 0; kp < KP; ++kp) s = dot2<E>(x[u][kp] & xm[kp], w[e][kp], s);
        o[e] = s;
      }
      Vec8<E>::store(Y + (size_t)m * a.ldy + cg * 8, o);
    }
  }
}

template <typename E>
hipError_t skinny_launch(const ConvArgs& a, hipStream_t s) {
  const long M = (long)a.N * a.Ho * a.Wo;
  if (a.Co <= 16) {
    hipLaunchKernelGGL(skinny_narrow_n_kernel<E>, dim3(ceil_div(M, SK_ROWS)), dim3(SK_THREADS), 0, s, a);
  } else {
    // ~4 blocks per CU: every block stages the weight table once, so the grid stays small and
    // each thread walks many rows
    const int per = SK_THREADS / (a.Co / 8);
    const long blocks = std::min<long>(1024, (M + 4L * per - 1) / (4L * per));
    const int K = a.C <= 8 ? 8 : 16;
    const size_t lds = (size_t)(K / 2) * a.Co * sizeof(uint32_t);
    if (K == 8) hipLaunchKernelGGL((skinny_narrow_k_kernel<E, 8>), dim3((int)blocks), dim3(SK_THREADS), lds, s, a);
    else hipLaunchKernelGGL((skinny_narrow_k_kernel<E, 16>), dim3((int)blocks), dim3(SK_THREADS), lds, s, a);
  }
  return hipGetLastError();
}

}  // namespace

bool conv_skinny_ok(int dtype, int out_f32, const ConvArgs& a) {
  if (!seg_half(dtype) || out_f32 || a.KH != 1 || a.KW != 1 || a.sf != 1 || a.st != 1 || a.pad_h ||
      a.pad_w || a.r || a.r2 || a.tap8)
    return false;
  if (a.Co <= 16)   // narrow N: 16-B pixel and weight loads, 4-channel stores inside ldy
    return a.C % 32 == 0 && a.C <= 512 && a.ldx % 8 == 0 && a.ldy >= (a.Co + 3) / 4 * 4 &&
           a.ldy % 4 == 0 && a.ldw % 8 == 0 && ((uintptr_t)a.w & 15) == 0;
  // narrow K (data gradient of a narrow conv): no BN statistics; the weight table (K x Co fp32)
  // fits the block's LDS
  return a.C <= 16 && a.ldx % 8 == 0 && a.ldx >= (a.C <= 8 ? 8 : 16) && a.Co % 8 == 0 &&
         a.ldy % 8 == 0 && SK_THREADS % (a.Co / 8) == 0 && a.Co / 8 <= SK_THREADS && a.Co <= 1024 &&
         !a.stats;
}

hipError_t launch_conv_skinny(int dtype, const ConvArgs& a, hipStream_t s) {
  if (dtype == SEG_F16) return skinny_launch<f16_t>(a, s);
  return skinny_launch<bf16_t>(a, s);
}
