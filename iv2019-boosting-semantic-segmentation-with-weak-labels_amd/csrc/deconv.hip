// 'hybrid' upsampling deconvolution of the logits heads (see deconv.h).
#include "deconv.h"

namespace {

constexpr int DC_THREADS = 256;

// wgrad tile: TR rows x TC columns of output pixels per block (+ a one-pixel halo of x)
template <int CT> struct DcTile { static constexpr int TR = 8, TC = CT <= 32 ? 32 : 16; };

// per-head LDS image of the parameters: D_h [C][3][3][C] then b_h [C], heads back to back
template <int C1, int C2, int C3>
__device__ void load_params(const DeconvArgs& a, float* sw) {
  const int cs[3] = {C1, C2, C3};
  int base = 0;
  for (int h = 0; h < 3; ++h) {
    const int nwh = 9 * cs[h] * cs[h];
    for (int k = threadIdx.x; k < nwh; k += blockDim.x) sw[base + k] = a.w[h][k];
    for (int k = threadIdx.x; k < cs[h]; k += blockDim.x) sw[base + nwh + k] = a.b[h][k];
    base += nwh + cs[h];
  }
  __syncthreads();
}

template <int C>
__device__ __forceinline__ void fwd_head(const DeconvArgs& a, int n, int py, int px, int off,
                                         const float* D, float* out) {
  float acc[C];
  const float* B = D + 9 * C * C;
#pragma unroll
  for (int o = 0; o < C; ++o) acc[o] = B[o];
  for (int kh = 0; kh < 3; ++kh) {
    const int qy = py + 1 - kh;
    if (qy < 0 || qy >= a.H) continue;
    for (int kw = 0; kw < 3; ++kw) {
      const int qx = px + 1 - kw;
      if (qx < 0 || qx >= a.W) continue;
      const float* xr = a.x + ((size_t)(n * a.H + qy) * a.W + qx) * a.ld + off;
      for (int i = 0; i < C; ++i) {
        const float xi = xr[i];
        const float* d = D + ((i * 3 + kh) * 3 + kw) * C;
#pragma unroll
        for (int o = 0; o < C; ++o) acc[o] += xi * d[o];
      }
    }
  }
#pragma unroll
  for (int o = 0; o < C; ++o) out[off + o] = acc[o];
}

template <int C1, int C2, int C3>
__global__ __launch_bounds__(DC_THREADS) void deconv_fwd_kernel(DeconvArgs a) {
  extern __shared__ float sw[];
  load_params<C1, C2, C3>(a, sw);
  const long total = (long)a.N * a.H * a.W;
  for (long id = (long)blockIdx.x * blockDim.x + threadIdx.x; id < total;
       id += (long)gridDim.x * blockDim.x) {
    const int px = (int)(id % a.W);
    const int py = (int)((id / a.W) % a.H);
    const int n = (int)(id / ((long)a.W * a.H));
    float* out = a.y + (size_t)id * a.ld;
    fwd_head<C1>(a, n, py, px, 0, sw, out);
    fwd_head<C2>(a, n, py, px, C1, sw + 9 * C1 * C1 + C1, out);
    fwd_head<C3>(a, n, py, px, C1 + C2, sw + 9 * (C1 * C1 + C2 * C2) + C1 + C2, out);
  }
}

// dx[q][i] = sum_{kh,kw,o} g'[qy + kh - 1][qx + kw - 1][o] * D[i][kh][kw][o], g' = g * gscale
template <int C>
__device__ __forceinline__ void dgrad_head(const DeconvArgs& a, int n, int qy, int qx, int off,
                                           const float* D, float* out) {
  float acc[C];
#pragma unroll
  for (int i = 0; i < C; ++i) acc[i] = 0.f;
  for (int kh = 0; kh < 3; ++kh) {
    const int py = qy + kh - 1;
    if (py < 0 || py >= a.H) continue;
    for (int kw = 0; kw < 3; ++kw) {
      const int px = qx + kw - 1;
      if (px < 0 || px >= a.W) continue;
      const float* gr = a.g + ((size_t)(n * a.H + py) * a.W + px) * a.ld + off;
      for (int o = 0; o < C; ++o) {
        const float go = gr[o] * a.gscale[off + o];
#pragma unroll
        for (int i = 0; i < C; ++i) acc[i] += go * D[((i * 3 + kh) * 3 + kw) * C + o];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < C; ++i) out[off + i] = acc[i];
}

template <int C1, int C2, int C3>
__global__ __launch_bounds__(DC_THREADS) void deconv_dgrad_kernel(DeconvArgs a) {
  extern __shared__ float sw[];
  load_params<C1, C2, C3>(a, sw);
  const long total = (long)a.N * a.H * a.W;
  for (long id = (long)blockIdx.x * blockDim.x + threadIdx.x; id < total;
       id += (long)gridDim.x * blockDim.x) {
    const int qx = (int)(id % a.W);
    const int qy = (int)((id / a.W) % a.H);
    const int n = (int)(id / ((long)a.W * a.H));
    float* out = a.dx + (size_t)id * a.ld;
    dgrad_head<C1>(a, n, qy, qx, 0, sw, out);
    dgrad_head<C2>(a, n, qy, qx, C1, sw + 9 * C1 * C1 + C1, out);
    dgrad_head<C3>(a, n, qy, qx, C1 + C2, sw + 9 * (C1 * C1 + C2 * C2) + C1 + C2, out);
  }
}

// weight / bias gradient partials of one TR x TC pixel tile: LDS holds g' (zero outside the
// map) and x with a one-pixel halo (zero outside: SAME padding); thread t owns partial entries
// t, t + blockDim, ... in the per-head order [D_h (i, kh, kw, o) | b_h (o)]
template <int C1, int C2, int C3>
__global__ __launch_bounds__(DC_THREADS) void deconv_wgrad_kernel(DeconvArgs a) {
  constexpr int CT = C1 + C2 + C3;
  constexpr int TR = DcTile<CT>::TR, TC = DcTile<CT>::TC;
  constexpr int NW = 9 * (C1 * C1 + C2 * C2 + C3 * C3) + CT;
  extern __shared__ float lds[];
  float* G = lds;                       // [TR][TC][CT]
  float* X = lds + TR * TC * CT;        // [TR + 2][TC + 2][CT]
  const int tiles_x = (a.W + TC - 1) / TC, tiles_y = (a.H + TR - 1) / TR;
  const int b = blockIdx.x;
  const int tx = b % tiles_x, ty = (b / tiles_x) % tiles_y, n = b / (tiles_x * tiles_y);
  const int r0 = ty * TR, c0 = tx * TC;
  for (int k = threadIdx.x; k < TR * TC * CT; k += blockDim.x) {
    const int ch = k % CT, pix = k / CT, c = pix % TC, r = pix / TC;
    const int py = r0 + r, px = c0 + c;
    G[k] = (py < a.H && px < a.W)
               ? a.g[((size_t)(n * a.H + py) * a.W + px) * a.ld + ch] * a.gscale[ch] : 0.f;
  }
  for (int k = threadIdx.x; k < (TR + 2) * (TC + 2) * CT; k += blockDim.x) {
    const int ch = k % CT, pix = k / CT, c = pix % (TC + 2), r = pix / (TC + 2);
    const int qy = r0 - 1 + r, qx = c0 - 1 + c;
    X[k] = (qy >= 0 && qy < a.H && qx >= 0 && qx < a.W)
               ? a.x[((size_t)(n * a.H + qy) * a.W + qx) * a.ld + ch] : 0.f;
  }
  __syncthreads();
  const int cs[3] = {C1, C2, C3};
  for (int w = threadIdx.x; w < NW; w += blockDim.x) {
    int h = 0, base = 0, off = 0;
    while (w - base >= 9 * cs[h] * cs[h] + cs[h]) { base += 9 * cs[h] * cs[h] + cs[h]; off += cs[h]; ++h; }
    const int C = cs[h], k = w - base;
    float s = 0.f;
    if (k < 9 * C * C) {   // D[i][kh][kw][o]: sum_p g'[p][o] * x[p + (1 - kh, 1 - kw)][i]
      const int o = k % C, kw = (k / C) % 3, kh = (k / (3 * C)) % 3, i = k / (9 * C);
      for (int r = 0; r < TR; ++r)
        for (int c = 0; c < TC; ++c)
          s += G[(r * TC + c) * CT + off + o] * X[((r + 2 - kh) * (TC + 2) + c + 2 - kw) * CT + off + i];
    } else {               // bias: sum_p g'[p][o]
      const int o = k - 9 * C * C;
      for (int r = 0; r < TR; ++r)
        for (int c = 0; c < TC; ++c) s += G[(r * TC + c) * CT + off + o];
    }
    a.part[(size_t)b * NW + w] = s;
  }
}

// fixed-order sum of the tile partials into the gradient buffer
__global__ void deconv_wreduce_kernel(DeconvArgs a, int nblocks, int nw) {
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= nw) return;
  float s = 0.f;
  for (int b = 0; b < nblocks; ++b) s += a.part[(size_t)b * nw + w];
  int h = 0, base = 0;
  while (w - base >= 9 * a.c[h] * a.c[h] + a.c[h]) { base += 9 * a.c[h] * a.c[h] + a.c[h]; ++h; }
  const int k = w - base;
  if (k < 9 * a.c[h] * a.c[h]) a.gw[h][k] = s;
  else a.gb[h][k - 9 * a.c[h] * a.c[h]] = s;
}

int grid_pixels(long total) {
  long g = (total + DC_THREADS - 1) / DC_THREADS;
  return (int)(g > 4096 ? 4096 : (g < 1 ? 1 : g));
}

template <int C1, int C2, int C3>
hipError_t fwd_t(const DeconvArgs& a, hipStream_t s) {
  const size_t lds = (size_t)(9 * (C1 * C1 + C2 * C2 + C3 * C3) + C1 + C2 + C3) * 4;
  auto k = deconv_fwd_kernel<C1, C2, C3>;
  hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k, dim3(grid_pixels((long)a.N * a.H * a.W)), dim3(DC_THREADS), lds, s, a);
  return hipGetLastError();
}

template <int C1, int C2, int C3>
hipError_t bwd_t(const DeconvArgs& a, hipStream_t s) {
  constexpr int CT = C1 + C2 + C3;
  const size_t lds = (size_t)(9 * (C1 * C1 + C2 * C2 + C3 * C3) + CT) * 4;
  auto kd = deconv_dgrad_kernel<C1, C2, C3>;
  hipError_t e = hipFuncSetAttribute((const void*)kd, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kd, dim3(grid_pixels((long)a.N * a.H * a.W)), dim3(DC_THREADS), lds, s, a);
  constexpr int TR = DcTile<CT>::TR, TC = DcTile<CT>::TC;
  const size_t lw = (size_t)(TR * TC + (TR + 2) * (TC + 2)) * CT * 4;
  auto kw = deconv_wgrad_kernel<C1, C2, C3>;
  e = hipFuncSetAttribute((const void*)kw, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lw);
  if (e != hipSuccess) return e;
  const int nb = deconv_wgrad_blocks(a.N, a.H, a.W, CT);
  hipLaunchKernelGGL(kw, dim3(nb), dim3(DC_THREADS), lw, s, a);
  const int nw = deconv_nw(a.c);
  hipLaunchKernelGGL(deconv_wreduce_kernel, dim3((nw + 255) / 256), dim3(256), 0, s, a, nb, nw);
  return hipGetLastError();
}

}  // namespace

int deconv_nw(const int c[3]) {
  return 9 * (c[0] * c[0] + c[1] * c[1] + c[2] * c[2]) + c[0] + c[1] + c[2];
}

int deconv_wgrad_blocks(int N, int H, int W, int ct) {
  const int TR = 8, TC = ct <= 32 ? 32 : 16;
  return N * ((H + TR - 1) / TR) * ((W + TC - 1) / TC);
}

hipError_t launch_deconv_fwd(const DeconvArgs& a, hipStream_t s) {
  if (a.c[0] == 14 && a.c[1] == 7 && a.c[2] == 3) return fwd_t<14, 7, 3>(a, s);
  if (a.c[0] == 53 && a.c[1] == 12 && a.c[2] == 5) return fwd_t<53, 12, 5>(a, s);
  return hipErrorInvalidValue;
}

hipError_t launch_deconv_bwd(const DeconvArgs& a, hipStream_t s) {
  if (a.c[0] == 14 && a.c[1] == 7 && a.c[2] == 3) return bwd_t<14, 7, 3>(a, s);
  if (a.c[0] == 53 && a.c[1] == 12 && a.c[2] == 5) return bwd_t<53, 12, 5>(a, s);
  return hipErrorInvalidValue;
}
