// Pooling / pyramid / resize kernels (see pool.h). 8-channel vectors (16 B bf16, 32 B f32)
// per thread; channel counts here are always multiples of 8 (checked by the launchers).
#include "pool.h"

namespace {

inline int grid_for(long items) {
  long g = (items + 255) / 256;
  return (int)(g < 8192 ? (g < 1 ? 1 : g) : 8192);
}

// ---- max pool 3x3 stride 2, TF SAME padding (pads are -inf, i.e. ignored) ---------------
template <typename T>
__global__ void maxpool_fwd_kernel(const T* __restrict__ x, int N, int H, int W, int C, int ldx,
                                   T* __restrict__ y, int Ho, int Wo, int ldy, int ph, int pw,
                                   uint8_t* __restrict__ arg) {
  const int cg_n = C / 8;
  const long total = (long)N * Ho * Wo * cg_n;
  for (long it = (long)blockIdx.x * blockDim.x + threadIdx.x; it < total;
       it += (long)gridDim.x * blockDim.x) {
    // 32-bit index decode (launch_* checks the item count < 2^31): 64-bit div/mod per
    // element was most of these streaming kernels' time
    const unsigned ui = (unsigned)it, up = ui / (unsigned)cg_n;
    const int cg = (int)(ui - up * (unsigned)cg_n);
    const long p = up;
    const unsigned ut = up / (unsigned)Wo;
    const int wo = (int)(up - ut * (unsigned)Wo);
    const unsigned un = ut / (unsigned)Ho;
    const int ho = (int)(ut - un * (unsigned)Ho);
    const int n = (int)un;
    float mx[8];
    uint32_t am[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { mx[e] = -INFINITY; am[e] = 255; }
    // the 9 window rows are loaded before any compare (one memory latency per element, not 9);
    // padding taps read a valid in-range row and are skipped
    float v[9][8];
#pragma unroll
    for (int t9 = 0; t9 < 9; ++t9) {
      const int hi = ho * 2 - ph + t9 / 3, wi = wo * 2 - pw + t9 % 3;
      const int hc = hi < 0 ? 0 : (hi >= H ? H - 1 : hi), wc = wi < 0 ? 0 : (wi >= W ? W - 1 : wi);
      Vec8<T>::load(x + ((size_t)((long)n * H + hc) * W + wc) * ldx + cg * 8, v[t9]);
    }
#pragma unroll
    for (int t9 = 0; t9 < 9; ++t9) {
      const int hi = ho * 2 - ph + t9 / 3, wi = wo * 2 - pw + t9 % 3;
      if (hi < 0 || hi >= H || wi < 0 || wi >= W) continue;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (v[t9][e] > mx[e]) { mx[e] = v[t9][e]; am[e] = t9; }  // first max wins (row-major scan)
    }
    Vec8<T>::store(y + p * ldy + cg * 8, mx);
    uint2 packed;
    packed.x = am[0] | (am[1] << 8) | (am[2] << 16) | (am[3] << 24);
    packed.y = am[4] | (am[5] << 8) | (am[6] << 16) | (am[7] << 24);
    *(uint2*)(arg + (size_t)p * C + cg * 8) = packed;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void bn_relu_maxpool_kernel(
    const T* __restrict__ y, int N, int H, int W, int ldy, const float* __restrict__ mean,
    const float* __restrict__ scale, const float* __restrict__ beta, uint8_t* __restrict__ mask,
    T* __restrict__ p, int Ho, int Wo, int ldp, uint8_t* __restrict__ arg) {
  constexpr int C = 64;
  const unsigned total = (unsigned)N * Ho * Wo * 8;
  const unsigned it = blockIdx.x * 256u + threadIdx.x;
  if (it >= total) return;
  const unsigned up = it >> 3;
  const int cg = (int)(it & 7);
  const unsigned ut = up / (unsigned)Wo;
  const int wo = (int)(up - ut * (unsigned)Wo);
  const unsigned un = ut / (unsigned)Ho;
  const int ho = (int)(ut - un * (unsigned)Ho);
  float mu[8], sc[8], be[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { mu[e] = mean[cg * 8 + e]; sc[e] = scale[cg * 8 + e]; be[e] = beta[cg * 8 + e]; }
  // window taps (2ho + dh, 2wo + dw); taps past the bottom / right edge read a clamped row and
  // are skipped (they are the 'SAME' padding)
  float v[9][8];
#pragma unroll
  for (int t9 = 0; t9 < 9; ++t9) {
    const int hi = ho * 2 + t9 / 3, wi = wo * 2 + t9 % 3;
    const int hc = hi < H ? hi : H - 1, wc = wi < W ? wi : W - 1;
    Vec8<T>::load(y + ((size_t)((long)un * H + hc) * W + wc) * ldy + cg * 8, v[t9]);
  }
  float mx[8];
  uint32_t am[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { mx[e] = -INFINITY; am[e] = 255; }
#pragma unroll
  for (int t9 = 0; t9 < 9; ++t9) {
    const int dh = t9 / 3, dw = t9 % 3;
    const int hi = ho * 2 + dh, wi = wo * 2 + dw;
    if (hi >= H || wi >= W) continue;
    uint32_t bits = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      // the BN apply kernel's arithmetic and rounding: the value the max-pool would have read
      const float o = fmaxf(__builtin_fmaf(v[t9][e] - mu[e], sc[e], be[e]), 0.f);
      const float z = sizeof(T) == 2 ? TypeOps<T>::to_f(TypeOps<T>::from_f(o)) : o;
      bits |= (uint32_t)(z > 0.f) << e;
      if (z > mx[e]) { mx[e] = z; am[e] = t9; }   // first max wins (row-major scan)
    }
    if (dh < 2 && dw < 2)   // this window's top-left 2 x 2 owns the pixel's ReLU bits
      mask[((size_t)((long)un * H + hi) * W + wi) * (C / 8) + cg] = (uint8_t)bits;
  }
  Vec8<T>::store(p + (size_t)up * ldp + cg * 8, mx);
  uint2 packed;
  packed.x = am[0] | (am[1] << 8) | (am[2] << 16) | (am[3] << 24);
  packed.y = am[4] | (am[5] << 8) | (am[6] << 16) | (am[7] << 24);
  *(uint2*)(arg + (size_t)up * C + cg * 8) = packed;
}

// gather form: each input pixel sums the gradients of the (<= 4) windows whose stored first
// max (forward argmax byte) is this pixel — no atomics, no recomputation
// C = 64 (the stem pool): blockIdx.y is one input row (n, hi) so the row decode is scalar;
// a thread owns 8 channels of one input pixel (8 threads per pixel, 128 B per pixel)
template <typename T>
__global__ __launch_bounds__(256) void maxpool_bwd_row_kernel(
    const uint8_t* __restrict__ arg, int H, int W, const T* __restrict__ dy, int Ho, int Wo,
    int lddy, T* __restrict__ dx, int lddx, int ph, int pw) {
  constexpr int C = 64;
  const int n = blockIdx.y / H, hi = blockIdx.y - n * H;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= W * 8) return;
  const int wi = idx >> 3, cg = idx & 7;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  const int ho_lo = hi + ph - 2 < 0 ? 0 : (hi + ph - 1) >> 1;
  const int ho_hi = (hi + ph) >> 1;
  const int wo_lo = wi + pw - 2 < 0 ? 0 : (wi + pw - 1) >> 1;
  const int wo_hi = (wi + pw) >> 1;
  // the <= 2 x 2 covering windows: every argmax word and every gradient row is loaded before
  // any is used (one memory latency per thread instead of one or two per window; the
  // gradient rows of windows that did not pick this pixel are L2 reads, not HBM)
  uint2 am[2][2];
  float g[2][2][8];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ho = ho_lo + i, wo = wo_lo + j;
      const bool ok = ho <= ho_hi && ho < Ho && wo <= wo_hi && wo < Wo;
      const size_t q = (size_t)((long)n * Ho + (ok ? ho : 0)) * Wo + (ok ? wo : 0);
      am[i][j] = ok ? *(const uint2*)(arg + q * C + cg * 8) : make_uint2(~0u, ~0u);
      if (ok) Vec8<T>::load(dy + q * lddy + cg * 8, g[i][j]);
      else {
#pragma unroll
        for (int e = 0; e < 8; ++e) g[i][j][e] = 0.f;
      }
    }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      // window order and float order as the per-window loop: ho outer, wo inner
      const uint32_t me = (uint32_t)((hi - ((ho_lo + i) * 2 - ph)) * 3 + (wi - ((wo_lo + j) * 2 - pw)));
      const uint2 a = am[i][j];
      const uint32_t b[8] = {a.x & 255, (a.x >> 8) & 255, (a.x >> 16) & 255, a.x >> 24,
                             a.y & 255, (a.y >> 8) & 255, (a.y >> 16) & 255, a.y >> 24};
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (b[e] == me) acc[e] += g[i][j][e];
    }
  Vec8<T>::store(dx + ((size_t)((long)n * H + hi) * W + wi) * lddx + cg * 8, acc);
}

// tiled gather for the stem pool without padding (H = 2 Ho, W = 2 Wo, C = 64): a block owns
// input rows 2r, 2r + 1 and 64 input columns; the pooled rows r - 1, r and the 33 pooled columns
// that cover them are staged once in LDS (gradient + argmax bytes), so each pooled value is read
// ~2x from L2 instead of ~9x (one thread per input pixel and 8 channels, every covering window
// re-read); per pixel the same windows in the same order as maxpool_bwd_row_kernel
template <typename T>
__global__ __launch_bounds__(256) void maxpool_bwd_tile_kernel(
    const uint8_t* __restrict__ arg, int H, int W, const T* __restrict__ dy, int Ho, int Wo,
    int lddy, T* __restrict__ dx, int lddx) {
  constexpr int C = 64, TW = 64, PW = TW / 2 + 1;
  __shared__ uint4 gs[2][PW][8];
  __shared__ uint2 as[2][PW][8];
  const int n = blockIdx.y / Ho, r = blockIdx.y - n * Ho;
  const int w0 = blockIdx.x * TW, wo0 = w0 / 2 - 1;   // pooled column of LDS slot 0
  const int t = threadIdx.x;
  for (int i = t; i < 2 * PW * 8; i += 256) {
    const int cg = i & 7, slot = (i >> 3) % PW, rs = (i >> 3) / PW;
    const int ho = r - 1 + rs, wo = wo0 + slot;
    const bool ok = ho >= 0 && ho < Ho && wo >= 0 && wo < Wo;
    const size_t q = ok ? (size_t)((long)n * Ho + ho) * Wo + wo : 0;
    as[rs][slot][cg] = ok ? *(const uint2*)(arg + q * C + cg * 8) : make_uint2(~0u, ~0u);
    gs[rs][slot][cg] = ok ? *(const uint4*)(dy + q * lddy + cg * 8) : make_uint4(0u, 0u, 0u, 0u);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int it = t + 256 * k;            // (row, col, cg): cg fastest, then column
    const int cg = it & 7, pix = it >> 3;
    const int ri = pix / TW, cj = pix - ri * TW;
    const int hi = 2 * r + ri, wi = w0 + cj;
    if (wi >= W) continue;
    const int ho_lo = hi - 2 < 0 ? 0 : (hi - 1) >> 1, ho_hi = hi >> 1;
    const int wo_lo = wi - 2 < 0 ? 0 : (wi - 1) >> 1, wo_hi = wi >> 1;
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ho = ho_lo + i, wo = wo_lo + j;
        if (ho > ho_hi || ho >= Ho || wo > wo_hi || wo >= Wo) continue;
        const uint32_t me = (uint32_t)((hi - 2 * ho) * 3 + (wi - 2 * wo));
        const uint2 a = as[ho - (r - 1)][wo - wo0][cg];
        float g[8];
        Half<T>::unpack(gs[ho - (r - 1)][wo - wo0][cg], g);
        const uint32_t b[8] = {a.x & 255, (a.x >> 8) & 255, (a.x >> 16) & 255, a.x >> 24,
                               a.y & 255, (a.y >> 8) & 255, (a.y >> 16) & 255, a.y >> 24};
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (b[e] == me) acc[e] += g[e];
      }
    Vec8<T>::store(dx + ((size_t)((long)n * H + hi) * W + wi) * lddx + cg * 8, acc);
  }
}

template <typename T>
__global__ void maxpool_bwd_kernel(const uint8_t* __restrict__ arg, int N, int H, int W, int C,
                                   const T* __restrict__ dy, int Ho, int Wo, int lddy,
                                   T* __restrict__ dx, int lddx, int ph, int pw) {
  const int cg_n = C / 8;
  const long total = (long)N * H * W * cg_n;
  for (long it = (long)blockIdx.x * blockDim.x + threadIdx.x; it < total;
       it += (long)gridDim.x * blockDim.x) {
    // 32-bit index decode (launch_* checks the item count < 2^31): 64-bit div/mod per
    // element was most of these streaming kernels' time
    const unsigned ui = (unsigned)it, up = ui / (unsigned)cg_n;
    const int cg = (int)(ui - up * (unsigned)cg_n);
    const unsigned ut = up / (unsigned)W;
    const int wi = (int)(up - ut * (unsigned)W);
    const unsigned un = ut / (unsigned)H;
    const int hi = (int)(ut - un * (unsigned)H);
    const int n = (int)un;
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    int ho_lo = (hi + ph - 2 + 1) >> 1;  // ceil((hi+ph-2)/2) for hi+ph-2 >= -1
    if (hi + ph - 2 < 0) ho_lo = 0;
    int ho_hi = (hi + ph) >> 1;
    int wo_lo = (wi + pw - 2 + 1) >> 1;
    if (wi + pw - 2 < 0) wo_lo = 0;
    int wo_hi = (wi + pw) >> 1;
    for (int ho = ho_lo; ho <= ho_hi && ho < Ho; ++ho) {
      for (int wo = wo_lo; wo <= wo_hi && wo < Wo; ++wo) {
        const size_t q = (size_t)((long)n * Ho + ho) * Wo + wo;
        const uint2 a = *(const uint2*)(arg + q * C + cg * 8);
        const uint32_t me = (uint32_t)((hi - (ho * 2 - ph)) * 3 + (wi - (wo * 2 - pw)));
        uint32_t b[8] = {a.x & 255, (a.x >> 8) & 255, (a.x >> 16) & 255, a.x >> 24,
                         a.y & 255, (a.y >> 8) & 255, (a.y >> 16) & 255, a.y >> 24};
        bool any = false;
#pragma unroll
        for (int e = 0; e < 8; ++e) any |= b[e] == me;
        if (!any) continue;
        float g[8];
        Vec8<T>::load(dy + q * lddy + cg * 8, g);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (b[e] == me) acc[e] += g[e];
      }
    }
    Vec8<T>::store(dx + ((size_t)((long)n * H + hi) * W + wi) * lddx + cg * 8, acc);
  }
}

template <typename T>
__global__ void add_strided_kernel(T* __restrict__ dx, int H, int W, int lddx, const T* __restrict__ g,
                                   int N, int Ho, int Wo, int C, int ldg, int s) {
  const int cg_n = C / 8;
  const long total = (long)N * Ho * Wo * cg_n;
  for (long it = (long)blockIdx.x * blockDim.x + threadIdx.x; it < total;
       it += (long)gridDim.x * blockDim.x) {
    // 32-bit index decode (launch_* checks the item count < 2^31): 64-bit div/mod per
    // element was most of these streaming kernels' time
    const unsigned ui = (unsigned)it, up = ui / (unsigned)cg_n;
    const int cg = (int)(ui - up * (unsigned)cg_n);
    const long p = up;
    const unsigned ut = up / (unsigned)Wo;
    const int wo = (int)(up - ut * (unsigned)Wo);
    const unsigned un = ut / (unsigned)Ho;
    const int ho = (int)(ut - un * (unsigned)Ho);
    const int n = (int)un;
    T* d = dx + ((size_t)((long)n * H + ho * s) * W + wo * s) * lddx + cg * 8;
    float a[8], b[8];
    Vec8<T>::load(d, a);
    Vec8<T>::load(g + (size_t)p * ldg + cg * 8, b);
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] += b[e];
    Vec8<T>::store(d, a);
  }
}

// ---- separable grid reductions ------------------------------------------------------------
// block per (n, h); thread per channel; registers indexed statically by cell q
template <typename T>
__global__ void grid_rowreduce_kernel(const T* __restrict__ x, int N, int H, int W, int C, int ldx,
                                      GridSpec g, float* __restrict__ part) {
  const int n = blockIdx.x / H, h = blockIdx.x % H;
  __shared__ float tab[SEG_MAX_CELLS * 256];
  for (int cbase = 0; cbase < C; cbase += blockDim.x) {
    const int c = cbase + threadIdx.x;
    const bool act = c < C;
    float acc[SEG_MAX_CELLS];
#pragma unroll
    for (int q = 0; q < SEG_MAX_CELLS; ++q) acc[q] = 0.f;
    const T* row = x + (size_t)((long)n * H + h) * W * ldx + (act ? c : 0);
    for (int w0 = 0; w0 < W; w0 += 256) {
      const int wn = (W - w0) < 256 ? (W - w0) : 256;
      __syncthreads();
      for (int i = threadIdx.x; i < g.total_ccells * wn; i += blockDim.x) {
        int q = i / wn, w = i % wn;
        tab[q * 256 + w] = g.rowtab[(size_t)q * W + w0 + w];
      }
      __syncthreads();
      for (int w = 0; w < wn && act; ++w) {
        float v = ldf(row + (size_t)(w0 + w) * ldx);
#pragma unroll
        for (int q = 0; q < SEG_MAX_CELLS; ++q)
          if (q < g.total_ccells) acc[q] += v * tab[q * 256 + w];
      }
    }
    float* o = part + (size_t)((long)n * H + h) * g.total_ccells * C + c;
#pragma unroll
    for (int q = 0; q < SEG_MAX_CELLS; ++q)
      if (act && q < g.total_ccells) o[(size_t)q * C] = acc[q];
  }
}

// 8 channels per thread (16-B loads), RL row lanes stride the row's pixels, cells taken 6 at a
// time (a second sweep of the row for 7..12 cells keeps the accumulators in registers); per-cell
// partial sums combined over the row lanes through LDS in fixed order.
// C % 8 == 0, 256 % (C/8) == 0, total cells <= 12.
template <typename T>
__global__ __launch_bounds__(256) void grid_rowreduce8_kernel(const T* __restrict__ x, int N, int H, int W,
                                                              int C, int ldx, GridSpec g,
                                                              float* __restrict__ part) {
  constexpr int QB = 6;
  const int n = blockIdx.x / H, h = blockIdx.x % H;
  const int cgn = C >> 3, RL = 256 / cgn;
  const int cg = threadIdx.x % cgn, rl = threadIdx.x / cgn;
  __shared__ float tab[QB * 256];
  __shared__ float red[256 * 8];
  const T* row = x + (size_t)((long)n * H + h) * W * ldx + cg * 8;
  float* o = part + (size_t)((long)n * H + h) * g.total_ccells * C;
  for (int q0 = 0; q0 < g.total_ccells; q0 += QB) {
    const int nq = g.total_ccells - q0 < QB ? g.total_ccells - q0 : QB;
    float acc[QB][8];
#pragma unroll
    for (int q = 0; q < QB; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[q][e] = 0.f;
    for (int w0 = 0; w0 < W; w0 += 256) {
      const int wn = (W - w0) < 256 ? (W - w0) : 256;
      __syncthreads();
      for (int i = threadIdx.x; i < nq * wn; i += 256) {
        const int q = i / wn, w = i - q * wn;
        tab[q * 256 + w] = g.rowtab[(size_t)(q0 + q) * W + w0 + w];
      }
      __syncthreads();
      // a lane's pixels 4 at a time: the 4 loads issued before their (in-order) FMAs
      int w = rl;
      for (; w + 3 * RL < wn; w += 4 * RL) {
        float v[4][8];
#pragma unroll
        for (int u = 0; u < 4; ++u) Vec8<T>::load(row + (size_t)(w0 + w + u * RL) * ldx, v[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int q = 0; q < QB; ++q) {
            if (q < nq) {
              const float wq = tab[q * 256 + w + u * RL];
#pragma unroll
              for (int e = 0; e < 8; ++e) acc[q][e] = __builtin_fmaf(wq, v[u][e], acc[q][e]);
            }
          }
      }
      for (; w < wn; w += RL) {
        float v[8];
        Vec8<T>::load(row + (size_t)(w0 + w) * ldx, v);
#pragma unroll
        for (int q = 0; q < QB; ++q) {
          if (q < nq) {
            const float wq = tab[q * 256 + w];
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[q][e] = __builtin_fmaf(wq, v[e], acc[q][e]);
          }
        }
      }
    }
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      if (q >= nq) break;
      __syncthreads();
#pragma unroll
      for (int e = 0; e < 8; ++e) red[(rl * cgn + cg) * 8 + e] = acc[q][e];
      __syncthreads();
      for (int c = threadIdx.x; c < C; c += 256) {
        float t = 0.f;
        for (int r = 0; r < RL; ++r) t += red[r * C + c];
        o[(size_t)(q0 + q) * C + c] = t;
      }
    }
  }
}

struct OutPtrs { void* p[SEG_MAX_GRIDS]; };

template <typename T>
__global__ void grid_colreduce_kernel(const float* __restrict__ part, int N, int H, int C,
                                      GridSpec g, OutPtrs outs) {
  // output element enumeration: grid by grid, [n][i][j][c]
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (int gi = 0; gi < g.n; ++gi) {
    long cnt = (long)N * g.kr[gi] * g.kc[gi] * C;
    if (idx < cnt) {
      int c = (int)(idx % C);
      long t = idx / C;
      int j = (int)(t % g.kc[gi]);
      t /= g.kc[gi];
      int i = (int)(t % g.kr[gi]);
      int n = (int)(t / g.kr[gi]);
      const int qi = g.rcell_off[gi] + i, qj = g.ccell_off[gi] + j;
      // rows 8 at a time: every weight and partial of a group loaded before the group's adds,
      // which stay in row order (one thread per output: a dependent load per row made the
      // image-pooling reduce over 128 rows ~45 us)
      const float* ct = g.coltab + (size_t)qi * H;
      const float* pp = part + (size_t)n * H * g.total_ccells * C + (size_t)qj * C + c;
      const size_t rs = (size_t)g.total_ccells * C;
      float s = 0.f;
      int h = 0;
      for (; h + 8 <= H; h += 8) {
        float wv[8], pv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          wv[u] = ct[h + u];
          pv[u] = pp[(size_t)(h + u) * rs];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (wv[u] != 0.f) s += wv[u] * pv[u];
      }
      for (; h < H; ++h) {
        const float wgt = ct[h];
        if (wgt != 0.f) s += wgt * pp[(size_t)h * rs];
      }
      stf((T*)outs.p[gi] + idx, s * g.scale[gi]);
      return;
    }
    idx -= cnt;
  }
}

// ---- align-corners bilinear resize (TF legacy scaler, TF lerp form) ------------------------
__device__ __forceinline__ void tf_lerp(int o, int n_in, int n_out, int& lo, int& hi, float& l) {
  float scale = n_out > 1 ? (float)(n_in - 1) / (float)(n_out - 1) : 0.f;
  float fin = (float)o * scale;
  lo = (int)fin;
  hi = lo + 1 < n_in - 1 ? lo + 1 : n_in - 1;
  l = fin - (float)lo;
}

template <typename T>
__global__ void resize_fwd_kernel(const T* __restrict__ x, int N, int hi_n, int wi_n, int C,
                                  int ldx, T* __restrict__ y, int Ho, int Wo, int ldy) {
  const int cg_n = C / 8;
  const long total = (long)N * Ho * Wo * cg_n;
  for (long it = (long)blockIdx.x * blockDim.x + threadIdx.x; it < total;
       it += (long)gridDim.x * blockDim.x) {
    // 32-bit index decode (launch_* checks the item count < 2^31): 64-bit div/mod per
    // element was most of these streaming kernels' time
    const unsigned ui = (unsigned)it, up = ui / (unsigned)cg_n;
    const int cg = (int)(ui - up * (unsigned)cg_n);
    const long p = up;
    const unsigned ut = up / (unsigned)Wo;
    const int wo = (int)(up - ut * (unsigned)Wo);
    const unsigned un = ut / (unsigned)Ho;
    const int ho = (int)(ut - un * (unsigned)Ho);
    const int n = (int)un;
    if (hi_n == 1 && wi_n == 1) {   // 1 x 1 source (the image-pool branch): a broadcast, one
                                    // load (every tap is the same cell, every weight 0)
      float v[8];
      Vec8<T>::load(x + (size_t)n * ldx + cg * 8, v);
      Vec8<T>::store(y + (size_t)p * ldy + cg * 8, v);
      continue;
    }
    int y0, y1, x0, x1;
    float yl, xl;
    tf_lerp(ho, hi_n, Ho, y0, y1, yl);
    tf_lerp(wo, wi_n, Wo, x0, x1, xl);
    const T* base = x + (size_t)n * hi_n * wi_n * ldx + cg * 8;
    float tl[8], tr[8], bl[8], br[8], o[8];
    Vec8<T>::load(base + ((size_t)y0 * wi_n + x0) * ldx, tl);
    Vec8<T>::load(base + ((size_t)y0 * wi_n + x1) * ldx, tr);
    Vec8<T>::load(base + ((size_t)y1 * wi_n + x0) * ldx, bl);
    Vec8<T>::load(base + ((size_t)y1 * wi_n + x1) * ldx, br);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float top = tl[e] + (tr[e] - tl[e]) * xl;
      float bot = bl[e] + (br[e] - bl[e]) * xl;
      o[e] = top + (bot - top) * yl;
    }
    Vec8<T>::store(y + (size_t)p * ldy + cg * 8, o);
  }
}

struct InPtrs { const void* p[SEG_MAX_GRIDS]; };

template <typename T>
__global__ void psp_input_bwd_kernel(const T* __restrict__ dcat, int ldcat, GridSpec g, InPtrs dp,
                                     int N, int H, int W, int C, T* __restrict__ dx, int lddx) {
  const int cg_n = C / 8;
  const long total = (long)N * H * W * cg_n;
  for (long it = (long)blockIdx.x * blockDim.x + threadIdx.x; it < total;
       it += (long)gridDim.x * blockDim.x) {
    // 32-bit index decode (launch_* checks the item count < 2^31): 64-bit div/mod per
    // element was most of these streaming kernels' time
    const unsigned ui = (unsigned)it, up = ui / (unsigned)cg_n;
    const int cg = (int)(ui - up * (unsigned)cg_n);
    const long p = up;
    const unsigned ut = up / (unsigned)W;
    const int w = (int)(up - ut * (unsigned)W);
    const unsigned un = ut / (unsigned)H;
    const int h = (int)(ut - un * (unsigned)H);
    const int n = (int)un;
    float a[8];
    Vec8<T>::load(dcat + (size_t)p * ldcat + cg * 8, a);
    for (int gi = 0; gi < g.n; ++gi) {
      int i = h / g.kh[gi], j = w / g.kw[gi];
      if (i < g.kr[gi] && j < g.kc[gi]) {
        float b[8];
        const T* src = (const T*)dp.p[gi] + ((size_t)((long)n * g.kr[gi] + i) * g.kc[gi] + j) * C + cg * 8;
        Vec8<T>::load(src, b);
        const float sc = g.scale[gi];
#pragma unroll
        for (int e = 0; e < 8; ++e) a[e] += b[e] * sc;
      }
    }
    Vec8<T>::store(dx + (size_t)p * lddx + cg * 8, a);
  }
}

}  // namespace

hipError_t launch_maxpool_fwd(int dtype, const void* x, int N, int H, int W, int C, int ldx,
                              void* y, int Ho, int Wo, int ldy, int pad_h, int pad_w, void* arg,
                              hipStream_t s) {
  if (C % 8 || ldx % 8 || ldy % 8) return hipErrorInvalidValue;
  if ((long)N * Ho * Wo * C / 8 >= (1L << 31)) return hipErrorInvalidValue;   // 32-bit decode
  dim3 g(grid_for((long)N * Ho * Wo * C / 8));
  if (dtype == SEG_BF16)
    hipLaunchKernelGGL(maxpool_fwd_kernel<bf16_t>, g, dim3(256), 0, s, (const bf16_t*)x, N, H, W, C,
                       ldx, (bf16_t*)y, Ho, Wo, ldy, pad_h, pad_w, (uint8_t*)arg);
  else if (dtype == SEG_F16)
    hipLaunchKernelGGL(maxpool_fwd_kernel<f16_t>, g, dim3(256), 0, s, (const f16_t*)x, N, H, W, C,
                       ldx, (f16_t*)y, Ho, Wo, ldy, pad_h, pad_w, (uint8_t*)arg);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<float>, g, dim3(256), 0, s, (const float*)x, N, H, W, C,
                       ldx, (float*)y, Ho, Wo, ldy, pad_h, pad_w, (uint8_t*)arg);
  return hipGetLastError();
}

hipError_t launch_bn_relu_maxpool_fwd(int dtype, const void* y, int N, int H, int W, int ldy,
                                      const float* mean, const float* scale, const float* beta,
                                      uint8_t* mask, void* p, int Ho, int Wo, int ldp, int pad_h,
                                      int pad_w, uint8_t* arg, hipStream_t s) {
  if (pad_h || pad_w || H % 2 || W % 2 || Ho * 2 != H || Wo * 2 != W || ldy % 8 || ldp % 8)
    return hipErrorInvalidValue;
  if ((long)N * Ho * Wo * 8 >= (1L << 31)) return hipErrorInvalidValue;   // 32-bit decode
  const dim3 g((unsigned)ceil_div((long)N * Ho * Wo * 8, 256));
  if (dtype == SEG_BF16)
    hipLaunchKernelGGL(bn_relu_maxpool_kernel<bf16_t>, g, dim3(256), 0, s, (const bf16_t*)y, N, H, W,
                       ldy, mean, scale, beta, mask, (bf16_t*)p, Ho, Wo, ldp, arg);
  else if (dtype == SEG_F16)
    hipLaunchKernelGGL(bn_relu_maxpool_kernel<f16_t>, g, dim3(256), 0, s, (const f16_t*)y, N, H, W,
                       ldy, mean, scale, beta, mask, (f16_t*)p, Ho, Wo, ldp, arg);
  else
    hipLaunchKernelGGL(bn_relu_maxpool_kernel<float>, g, dim3(256), 0, s, (const float*)y, N, H, W,
                       ldy, mean, scale, beta, mask, (float*)p, Ho, Wo, ldp, arg);
  return hipGetLastError();
}

hipError_t launch_maxpool_bwd(int dtype, const void* arg, int N, int H, int W, int C,
                              const void* dy, int Ho, int Wo, int lddy, void* dx, int lddx,
                              int pad_h, int pad_w, hipStream_t s) {
  if (C % 8 || lddy % 8 || lddx % 8) return hipErrorInvalidValue;
  if ((long)N * H * W * C / 8 >= (1L << 31)) return hipErrorInvalidValue;   // 32-bit decode
  if (C == 64 && pad_h == 0 && pad_w == 0 && H == 2 * Ho && W == 2 * Wo && (dtype == SEG_BF16 || dtype == SEG_F16) &&
      (long)N * Ho < 65536) {   // the stem pool (16-bit): LDS-staged pooled tiles
    dim3 g((unsigned)ceil_div(W, 64), (unsigned)(N * Ho));
    if (dtype == SEG_BF16)
      hipLaunchKernelGGL(maxpool_bwd_tile_kernel<bf16_t>, g, dim3(256), 0, s, (const uint8_t*)arg, H, W,
                         (const bf16_t*)dy, Ho, Wo, lddy, (bf16_t*)dx, lddx);
    else
      hipLaunchKernelGGL(maxpool_bwd_tile_kernel<f16_t>, g, dim3(256), 0, s, (const uint8_t*)arg, H, W,
                         (const f16_t*)dy, Ho, Wo, lddy, (f16_t*)dx, lddx);
    return hipGetLastError();
  }
  if (C == 64 && (long)N * H < 65536) {   // the stem pool: one row of the input per grid row
    dim3 g((unsigned)ceil_div((long)W * 8, 256), (unsigned)(N * H));
    if (dtype == SEG_BF16)
      hipLaunchKernelGGL(maxpool_bwd_row_kernel<bf16_t>, g, dim3(256), 0, s, (const uint8_t*)arg, H, W,
                         (const bf16_t*)dy, Ho, Wo, lddy, (bf16_t*)dx, lddx, pad_h, pad_w);
    else if (dtype == SEG_F16)
      hipLaunchKernelGGL(maxpool_bwd_row_kernel<f16_t>, g, dim3(256), 0, s, (const uint8_t*)arg, H, W,
                         (const f16_t*)dy, Ho, Wo, lddy, (f16_t*)dx, lddx, pad_h, pad_w);
    else
      hipLaunchKernelGGL(maxpool_bwd_row_kernel<float>, g, dim3(256), 0, s, (const uint8_t*)arg, H, W,
                         (const float*)dy, Ho, Wo, lddy, (float*)dx, lddx, pad_h, pad_w);
    return hipGetLastError();
  }
  dim3 g(grid_for((long)N * H * W * C / 8));
  if (dtype == SEG_BF16)
    hipLaunchKernelGGL(maxpool_bwd_kernel<bf16_t>, g, dim3(256), 0, s, (const uint8_t*)arg, N, H, W,
                       C, (const bf16_t*)dy, Ho, Wo, lddy, (bf16_t*)dx, lddx, pad_h, pad_w);
  else if (dtype == SEG_F16)
    hipLaunchKernelGGL(maxpool_bwd_kernel<f16_t>, g, dim3(256), 0, s, (const uint8_t*)arg, N, H, W,
                       C, (const f16_t*)dy, Ho, Wo, lddy, (f16_t*)dx, lddx, pad_h, pad_w);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel<float>, g, dim3(256), 0, s, (const uint8_t*)arg, N, H, W,
                       C, (const float*)dy, Ho, Wo, lddy, (float*)dx, lddx, pad_h, pad_w);
  return hipGetLastError();
}

hipError_t launch_add_strided(int dtype, void* dx, int H, int W, int lddx, const void* g, int N,
                              int Ho, int Wo, int C, int ldg, int stride, hipStream_t s) {
  if (C % 8 || lddx % 8 || ldg % 8) return hipErrorInvalidValue;
  if ((long)N * Ho * Wo * C / 8 >= (1L << 31)) return hipErrorInvalidValue;   // 32-bit decode
  dim3 gr(grid_for((long)N * Ho * Wo * C / 8));
  if (dtype == SEG_BF16)
    hipLaunchKernelGGL(add_strided_kernel<bf16_t>, gr, dim3(256), 0, s, (bf16_t*)dx, H, W, lddx,
                       (const bf16_t*)g, N, Ho, Wo, C, ldg, stride);
  else if (dtype == SEG_F16)
    hipLaunchKernelGGL(add_strided_kernel<f16_t>, gr, dim3(256), 0, s, (f16_t*)dx, H, W, lddx,
                       (const f16_t*)g, N, Ho, Wo, C, ldg, stride);
  else
    hipLaunchKernelGGL(add_strided_kernel<float>, gr, dim3(256), 0, s, (float*)dx, H, W, lddx,
                       (const float*)g, N, Ho, Wo, C, ldg, stride);
  return hipGetLastError();
}

hipError_t launch_grid_rowreduce(int dtype, const void* x, int N, int H, int W, int C, int ldx,
                                 const GridSpec& g, float* part, hipStream_t s) {
  if (g.total_ccells > SEG_MAX_CELLS) return hipErrorInvalidValue;
  dim3 gr(N * H);
  const bool v8 = C % 8 == 0 && ldx % 8 == 0 && C / 8 <= 256 && 256 % (C / 8) == 0 && g.total_ccells <= 12;
  if (v8) {
    if (dtype == SEG_BF16)
      hipLaunchKernelGGL((grid_rowreduce8_kernel<bf16_t>), gr, dim3(256), 0, s, (const bf16_t*)x, N, H, W, C, ldx, g, part);
    else if (dtype == SEG_F16)
      hipLaunchKernelGGL((grid_rowreduce8_kernel<f16_t>), gr, dim3(256), 0, s, (const f16_t*)x, N, H, W, C, ldx, g, part);
    else
      hipLaunchKernelGGL((grid_rowreduce8_kernel<float>), gr, dim3(256), 0, s, (const float*)x, N, H, W, C, ldx, g, part);
    return hipGetLastError();
  }
  if (dtype == SEG_BF16)
    hipLaunchKernelGGL(grid_rowreduce_kernel<bf16_t>, gr, dim3(256), 0, s, (const bf16_t*)x, N, H,
                       W, C, ldx, g, part);
  else if (dtype == SEG_F16)
    hipLaunchKernelGGL(grid_rowreduce_kernel<f16_t>, gr, dim3(256), 0, s, (const f16_t*)x, N, H,
                       W, C, ldx, g, part);
  else
    hipLaunchKernelGGL(grid_rowreduce_kernel<float>, gr, dim3(256), 0, s, (const float*)x, N, H, W,
                       C, ldx, g, part);
  return hipGetLastError();
}

hipError_t launch_grid_colreduce(int dtype, const float* part, int N, int H, int W, int C,
                                 const GridSpec& g, void* const* outs, hipStream_t s) {
  (void)W;
  OutPtrs o;
  long total = 0;
  for (int i = 0; i < SEG_MAX_GRIDS; ++i) o.p[i] = i < g.n ? outs[i] : nullptr;
  for (int i = 0; i < g.n; ++i) total += (long)N * g.kr[i] * g.kc[i] * C;
  dim3 gr(ceil_div(total, 256));
  if (dtype == SEG_BF16)
    hipLaunchKernelGGL(grid_colreduce_kernel<bf16_t>, gr, dim3(256), 0, s, part, N, H, C, g, o);
  else if (dtype == SEG_F16)
    hipLaunchKernelGGL(grid_colreduce_kernel<f16_t>, gr, dim3(256), 0, s, part, N, H, C, g, o);
  else
    hipLaunchKernelGGL(grid_colreduce_kernel<float>, gr, dim3(256), 0, s, part, N, H, C, g, o);
  return hipGetLastError();
}

hipError_t launch_resize_fwd(int dtype, const void* x, int N, int hi, int wi, int C, int ldx,
                             void* y, int Ho, int Wo, int ldy, hipStream_t s) {
  if (C % 8 || ldx % 8 || ldy % 8) return hipErrorInvalidValue;
  if ((long)N * Ho * Wo * C / 8 >= (1L << 31)) return hipErrorInvalidValue;   // 32-bit decode
  dim3 gr(grid_for((long)N * Ho * Wo * C / 8));
  if (dtype == SEG_BF16)
    hipLaunchKernelGGL(resize_fwd_kernel<bf16_t>, gr, dim3(256), 0, s, (const bf16_t*)x, N, hi, wi,
                       C, ldx, (bf16_t*)y, Ho, Wo, ldy);
  else if (dtype == SEG_F16)
    hipLaunchKernelGGL(resize_fwd_kernel<f16_t>, gr, dim3(256), 0, s, (const f16_t*)x, N, hi, wi,
                       C, ldx, (f16_t*)y, Ho, Wo, ldy);
  else
    hipLaunchKernelGGL(resize_fwd_kernel<float>, gr, dim3(256), 0, s, (const float*)x, N, hi, wi, C,
                       ldx, (float*)y, Ho, Wo, ldy);
  return hipGetLastError();
}

hipError_t launch_psp_input_bwd(int dtype, const void* dcat, int ldcat, const GridSpec& g,
                                const void* const* dpooled, int N, int H, int W, int C, void* dx,
                                int lddx, hipStream_t s) {
  if (C % 8 || ldcat % 8 || lddx % 8) return hipErrorInvalidValue;
  InPtrs ip;
  for (int i = 0; i < SEG_MAX_GRIDS; ++i) ip.p[i] = i < g.n ? dpooled[i] : nullptr;
  if ((long)N * H * W * C / 8 >= (1L << 31)) return hipErrorInvalidValue;   // 32-bit decode
  dim3 gr(grid_for((long)N * H * W * C / 8));
  if (dtype == SEG_BF16)
    hipLaunchKernelGGL(psp_input_bwd_kernel<bf16_t>, gr, dim3(256), 0, s, (const bf16_t*)dcat, ldcat,
                       g, ip, N, H, W, C, (bf16_t*)dx, lddx);
  else if (dtype == SEG_F16)
    hipLaunchKernelGGL(psp_input_bwd_kernel<f16_t>, gr, dim3(256), 0, s, (const f16_t*)dcat, ldcat,
                       g, ip, N, H, W, C, (f16_t*)dx, lddx);
  else
    hipLaunchKernelGGL(psp_input_bwd_kernel<float>, gr, dim3(256), 0, s, (const float*)dcat, ldcat, g,
                       ip, N, H, W, C, (float*)dx, lddx);
  return hipGetLastError();
}
