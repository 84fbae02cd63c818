// 'hybrid' upsampling (resnet50_extended_model_hierarchical.py:168-180): per head, a 3 x 3
// stride-1 SAME slim.conv2d_transpose C -> C with bias and no normalizer / activation, applied
// to the low-resolution logits before the align-corners bilinear resize (which stays fused
// into the loss head / eval kernels). Tiny fp32 work (24 or 70 channels at H/8 x W/8), so
// plain VALU kernels with the weights in LDS.
//
// Weight layout per head h (flat fp32, inside the weight-decay region of the parameters):
// D[i][kh][kw][o] = TF kernel[kh][kw][o][i] (conv2d_transpose filters are [h, w, out, in]), so
// the generic OHWI -> HWIO checkpoint transpose of a (C, 3, 3, C) "weights" tensor gives TF's
// layout. y[p][o] = b[o] + sum_{kh,kw,i} x[py + 1 - kh][px + 1 - kw][i] * D[i][kh][kw][o].
#pragma once
#include "seg_common.h"

struct DeconvArgs {
  const float* x;          // [N][H][W][ld] logits (l1 | l2v | l2h channels)
  float* y;                // [N][H][W][ld] forward output (bilinear-resize input)
  const float* g;          // [N][H][W][ld] gradient w.r.t. y (unnormalised, loss head)
  const float* gscale;     // [ld] per-channel factor applied to g (loss normalisation)
  float* dx;               // [N][H][W][ld] gradient w.r.t. x
  float* part;             // wgrad partials [blocks][nw]
  int N, H, W, ld;
  int c[3];                // channels per head
  const float* w[3];       // D per head (params)
  const float* b[3];       // bias per head
  float* gw[3];            // gradient destinations (grads buffer)
  float* gb[3];
};

// number of weight + bias gradient values (the partial vector length)
int deconv_nw(const int c[3]);
// wgrad partial blocks for this shape
int deconv_wgrad_blocks(int N, int H, int W, int ct);
hipError_t launch_deconv_fwd(const DeconvArgs& a, hipStream_t s);
// dx, and the weight / bias gradients (partials + fixed-order reduce into gw / gb)
hipError_t launch_deconv_bwd(const DeconvArgs& a, hipStream_t s);
