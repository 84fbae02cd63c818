// Input preprocessing kernels (see input.h). Both are one pass over the output pixels: each
// output pixel gathers its (<= 4) source pixels from the raw uint8 image in HBM; raw bytes
// are read once per output pixel neighbourhood (L2 absorbs the 2x2 reuse).
#include "input.h"

// TF 1.12 computes the resize scales and lerps on the CPU in IEEE float without FMA
// contraction (CalculateResizeScale, compute_interpolation_weights): the scales are divided
// on the host here (a device division may differ by one ulp, which moves `in_f` by one ulp of
// a value up to the source size) and contraction is off so each lerp rounds like TF's.
#pragma clang fp contract(off)

namespace {

constexpr int IN_THREADS = 256;

__device__ __forceinline__ void lerp_legacy(int o, int n_in, float scale, int& lo, int& hi,
                                            float& l) {
  const float fin = (float)o * scale;
  lo = (int)fin;                  // fin >= 0: floor
  hi = lo + 1 < n_in - 1 ? lo + 1 : n_in - 1;
  l = fin - (float)lo;
}

// (cy, cx): the output is the H x W window at that offset of the image resized to the size
// `sy` / `sx` were computed for (the aspect-preserving resize + random crop of
// resize_images_and_labels, input_pipelines/utils.py:206-232); (0, 0) with the full size is
// the plain resize
__global__ __launch_bounds__(IN_THREADS) void prepare_images_kernel(
    const uint8_t* __restrict__ raw, int n, int Hr, int Wr, int H, int W, float sy, float sx,
    int cy, int cx, float* __restrict__ out) {
  const long total = (long)n * H * W;
  const float inv255 = (float)(1.0 / 255.0);   // convert_image_dtype: cast * (1 / max)
  for (long id = (long)blockIdx.x * IN_THREADS + threadIdx.x; id < total;
       id += (long)gridDim.x * IN_THREADS) {
    const int x = (int)(id % W);
    const int y = (int)((id / W) % H);
    const int b = (int)(id / ((long)W * H));
    int ylo, yhi, xlo, xhi;
    float yl, xl;
    lerp_legacy(y + cy, Hr, sy, ylo, yhi, yl);
    lerp_legacy(x + cx, Wr, sx, xlo, xhi, xl);
    const uint8_t* img = raw + (size_t)b * Hr * Wr * 3;
    const uint8_t* tl = img + ((size_t)ylo * Wr + xlo) * 3;
    const uint8_t* tr = img + ((size_t)ylo * Wr + xhi) * 3;
    const uint8_t* bl = img + ((size_t)yhi * Wr + xlo) * 3;
    const uint8_t* br = img + ((size_t)yhi * Wr + xhi) * 3;
    float* o = out + id * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float vtl = (float)tl[c] * inv255, vtr = (float)tr[c] * inv255;
      const float vbl = (float)bl[c] * inv255, vbr = (float)br[c] * inv255;
      const float top = vtl + (vtr - vtl) * xl;
      const float bot = vbl + (vbr - vbl) * xl;
      const float v = top + (bot - top) * yl;
      o[c] = (v - 0.5f) / 0.5f;
    }
  }
}

__global__ __launch_bounds__(IN_THREADS) void prepare_labels_kernel(
    const uint8_t* __restrict__ raw, int n, int Hr, int Wr, int H, int W, float sy, float sx,
    LidMap m, int32_t* __restrict__ out) {
  const long total = (long)n * H * W;
  for (long id = (long)blockIdx.x * IN_THREADS + threadIdx.x; id < total;
       id += (long)gridDim.x * IN_THREADS) {
    const int x = (int)(id % W);
    const int y = (int)((id / W) % H);
    const int b = (int)(id / ((long)W * H));
    int ys = (int)floorf((float)y * sy), xs = (int)floorf((float)x * sx);
    ys = ys < Hr - 1 ? ys : Hr - 1;
    xs = xs < Wr - 1 ? xs : Wr - 1;
    const int lid = raw[((size_t)b * Hr + ys) * Wr + xs];
    out[id] = lid < m.n ? m.cid[lid] : -1;   // out-of-table ids: tf.gather error -> -1 marker
  }
}

}  // namespace

hipError_t launch_prepare_images(const uint8_t* raw, int n, int Hr, int Wr, int Hs, int Ws,
                                 int cy, int cx, int H, int W, float* out, hipStream_t s) {
  const long total = (long)n * H * W;
  if (total <= 0) return hipSuccess;
  const long g = std::min<long>(ceil_div(total, IN_THREADS), 16384);
  const float sy = (float)Hr / (float)Hs, sx = (float)Wr / (float)Ws;   // host IEEE division
  hipLaunchKernelGGL(prepare_images_kernel, dim3((unsigned)g), dim3(IN_THREADS), 0, s, raw, n, Hr,
                     Wr, H, W, sy, sx, cy, cx, out);
  return hipGetLastError();
}

hipError_t launch_prepare_labels(const uint8_t* raw, int n, int Hr, int Wr, int H, int W,
                                 const LidMap& m, int32_t* out, hipStream_t s) {
  const long total = (long)n * H * W;
  if (total <= 0) return hipSuccess;
  const long g = std::min<long>(ceil_div(total, IN_THREADS), 16384);
  const float sy = (float)Hr / (float)H, sx = (float)Wr / (float)W;
  hipLaunchKernelGGL(prepare_labels_kernel, dim3((unsigned)g), dim3(IN_THREADS), 0, s, raw, n, Hr,
                     Wr, H, W, sy, sx, m, out);
  return hipGetLastError();
}
