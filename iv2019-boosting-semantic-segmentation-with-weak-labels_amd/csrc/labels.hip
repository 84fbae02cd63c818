// Weak-label maps on the GPU; see labels.h for the reference semantics restated here.
#include "labels.h"

namespace {

constexpr int LB_THREADS = 256;
constexpr int LB_MAX_BOXES = 1024;   // reference MAX_N_BBOXES = 516 (input_subset_bboxes_v2.py:33)

// One block = 256 consecutive output pixels of one image (blockIdx.y). The image's boxes are
// converted to integer source rectangles once per block (float64 multiply + truncation, as
// the reference's int(coord * size) on float32 coordinates) and kept in LDS; each thread counts
// the boxes covering its source pixel per class, normalises, and the block stores its
// 256 x 15 floats through LDS as contiguous 16-byte chunks.
__global__ __launch_bounds__(LB_THREADS) void bbox_labels_kernel(const float* boxes, const int* cids,
                                                              const int* box_off, const BboxGeom* geom,
                                                              int H, int W, float* out) {
  __shared__ int4 rect[LB_MAX_BOXES];
  __shared__ int rcid[LB_MAX_BOXES];
  __shared__ float stage[LB_THREADS * SEG_WEAK_CLASSES];
  const int img = blockIdx.y;
  const BboxGeom g = geom[img];
  const int b0 = box_off[img], nb = box_off[img + 1] - b0;
  for (int b = threadIdx.x; b < nb; b += LB_THREADS) {
    const float* c = boxes + 4 * (size_t)(b0 + b);
    // the reference multiplies a float32 coordinate by an integer size in numpy, which
    // promotes to float64, then truncates (input_subset_bboxes_v2.py:85)
    const int xmin = (int)((double)c[0] * g.src_w), xmax = (int)((double)c[1] * g.src_w);
    const int ymin = (int)((double)c[2] * g.src_h), ymax = (int)((double)c[3] * g.src_h);
    rect[b] = make_int4(xmin, xmax, ymin, ymax);
    rcid[b] = cids[b0 + b];
  }
  __syncthreads();
  const long npix = (long)H * W;
  const long p = (long)blockIdx.x * LB_THREADS + threadIdx.x;
  float v[SEG_WEAK_CLASSES];
  if (p < npix) {
    const int y = (int)(p / W), x = (int)(p - (long)y * W);
    // TF 1.12 ResizeNearestNeighbor (align_corners = false): float scale in/out, floorf
    const float sh = (float)g.src_h / (float)g.rh, sw = (float)g.src_w / (float)g.rw;
    const int sy = min((int)floorf((float)(y + g.oy) * sh), g.src_h - 1);
    const int sx = min((int)floorf((float)(x + g.ox) * sw), g.src_w - 1);
    float cnt[SEG_WEAK_CLASSES];
#pragma unroll
    for (int k = 0; k < SEG_WEAK_CLASSES; ++k) cnt[k] = 0.f;
    for (int b = 0; b < nb; ++b) {
      const int4 r = rect[b];
      const bool in = (sx >= r.x) & (sx <= r.y) & (sy >= r.z) & (sy <= r.w);
      const int c = rcid[b];
#pragma unroll
      for (int k = 0; k < SEG_WEAK_CLASSES; ++k) cnt[k] += (in && c == k) ? 1.f : 0.f;
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < SEG_WEAK_CLASSES; ++k) s += cnt[k];
#pragma unroll
    for (int k = 0; k < SEG_WEAK_CLASSES; ++k)
      v[k] = s > 0.5f ? cnt[k] / s : (k == SEG_WEAK_CLASSES - 1 ? 1.f : 0.f);
  }
#pragma unroll
  for (int k = 0; k < SEG_WEAK_CLASSES; ++k) stage[threadIdx.x * SEG_WEAK_CLASSES + k] = v[k];
  __syncthreads();
  // the block's pixels are contiguous in out: 256 * 15 floats = 960 float4
  float* o = out + ((size_t)img * npix + (size_t)blockIdx.x * LB_THREADS) * SEG_WEAK_CLASSES;
  const long rem = npix - (long)blockIdx.x * LB_THREADS;
  const int nval = (int)(rem < LB_THREADS ? rem : LB_THREADS) * SEG_WEAK_CLASSES;
  if (nval == LB_THREADS * SEG_WEAK_CLASSES && ((uintptr_t)o & 15) == 0) {
    for (int i = threadIdx.x; i < nval / 4; i += LB_THREADS)
      ((float4*)o)[i] = ((const float4*)stage)[i];
  } else {
    for (int i = threadIdx.x; i < nval; i += LB_THREADS) o[i] = stage[i];
  }
}

__global__ __launch_bounds__(LB_THREADS) void tag_labels_kernel(const float* tags, long npix, float* out) {
  const int img = blockIdx.y;
  float t[SEG_WEAK_CLASSES];
#pragma unroll
  for (int k = 0; k < SEG_WEAK_CLASSES; ++k) t[k] = tags[img * SEG_WEAK_CLASSES + k];
  for (long p = (long)blockIdx.x * LB_THREADS + threadIdx.x; p < npix; p += (long)gridDim.x * LB_THREADS) {
    float* o = out + ((size_t)img * npix + p) * SEG_WEAK_CLASSES;
#pragma unroll
    for (int k = 0; k < SEG_WEAK_CLASSES; ++k) o[k] = t[k];
  }
}

}  // namespace

hipError_t launch_bbox_labels(const float* boxes, const int* cids, const int* box_off,
                              const BboxGeom* geom, int n, int H, int W, float* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const long npix = (long)H * W;
  const dim3 grid((unsigned)ceil_div(npix, LB_THREADS), (unsigned)n);
  hipLaunchKernelGGL(bbox_labels_kernel, grid, dim3(LB_THREADS), 0, s, boxes, cids, box_off, geom, H, W, out);
  return hipGetLastError();
}

hipError_t launch_tag_labels(const float* tags, int n, int H, int W, float* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const long npix = (long)H * W;
  const dim3 grid((unsigned)std::min<long>(ceil_div(npix, LB_THREADS), 4096), (unsigned)n);
  hipLaunchKernelGGL(tag_labels_kernel, grid, dim3(LB_THREADS), 0, s, tags, npix, out);
  return hipGetLastError();
}
