// Implicit-GEMM convolutions on CDNA4 MFMA (gfx950). No im2col buffer is ever built: the
// A-operand gather computes each source pixel (with TF padding / dilation / stride) while
// staging tiles into LDS.
//
//   forward : y[p][co]  = sum_{kh,kw,ci} x[src(p,kh,kw)][ci] * w[co][kh][kw][ci]
//   dgrad   : dx[p][ci] = sum_{kh,kw,co} dy[src_t(p,kh,kw)][co] * wT[ci][kh][kw][co]
//             (wT = spatially flipped, transposed weights; stride>1 uses the divisibility
//              gather of a transposed conv)
//   wgrad   : dw[co][kh][kw][ci] = sum_p dy[p][co] * x[src(p,kh,kw)][ci]   (split-K slabs)
#pragma once
#include "seg_common.h"

struct ConvArgs {
  const void* x;  // A source, NHWC [N][H][W][ldx]
  int N, H, W, C, ldx;
  const void* w;  // B, [Co][K] with row stride ldw (K = KH*KW*C)
  int ldw;
  void* y;        // output NHWC [N][Ho][Wo][ldy]
  int Ho, Wo, Co, ldy;
  const void* r;  // optional residual added in the epilogue (may alias y), ld = ldr
  int ldr;
  const void* r2; // optional second residual, ld = ldr2
  int ldr2;
  int KH, KW;
  int sf;         // forward stride: src = o*sf - pad + k*dil
  int st;         // transposed stride: src valid iff divisible by st (1 = plain conv)
  int pad_h, pad_w, dil;
  float* stats;   // BN partials [mtiles][Co] x {sum, M2} (nullptr = none)
  int tap8;       // tap mode: a tap is tap8 16-B chunks of K (2: the space-to-depth stem, 16
                  // channels per tap); K = KH*KW*C is padded to a multiple of 64 with zero weights
  // K-concatenated second GEMM (dense 1x1: the ping-pong path, and v2 for Co <= 128): y = x w^T + x2 w2^T, x2 [..][ldx2]
  // with C2 channels on the same pixels, w2 [Co][ldw2]; a projection unit's conv1 + shortcut
  // data gradients into the unit input in one accumulation (x2 = nullptr: single GEMM)
  const void* x2;
  int ldx2, C2;
  const void* w2;
  int ldw2;
  // optional ReLU bits of the output's consumer, [M][ldm] bytes (bit e of byte n/8 = channel n):
  // outputs whose bit is 0 are stored as zero (conv_nt_omask_ok launches only)
  const uint8_t* omask;
  int ldm;
};

struct WgradArgs {
  const void* dy;  // [P][lddy], P = N*Ho*Wo
  int lddy;
  const void* x;   // NHWC [N][H][W][ldx]
  int N, H, W, C, ldx;
  int Ho, Wo, Co;
  int KH, KW, sf, pad_h, pad_w, dil;
  float* out;      // fp32 [splits][Co][KH*KW*C]
  int splits;
  // optional second dy source (16-bit v2 / ping-pong kernels): rows co >= Co1 of the output
  // take dy2 [P][lddy2] column co - Co1 (Co1 % 8 == 0; the ping-pong kernel Co1 % 256 == 0):
  // two weight-gradient GEMMs over the same x in one launch (csrc/lbf.h: dyhat^T y2, y2^T y2)
  const void* dy2;
  int lddy2, Co1;
};

// host launchers (conv.hip); return hipError_t
hipError_t launch_conv_nt(int dtype, int out_f32, const ConvArgs& a, hipStream_t s);
hipError_t launch_conv_wgrad(int dtype, const WgradArgs& a, hipStream_t s);
hipError_t launch_splitk_reduce(const float* part, int splits, long split_stride, long n,
                                float* out, int accumulate, hipStream_t s);
// all layers' flips in one launch: table of FlipJob (device), prefix = the job's first tile;
// total = flip tiles over all jobs
struct FlipJob { const void* w; void* wt; int co, k, ci; long prefix; };
long flip_tiles(int co, int k, int ci);
hipError_t launch_weight_flip_batched(int dtype, const FlipJob* jobs, int njobs, long total,
                                      hipStream_t s);
hipError_t launch_weight_flip_transpose(int dtype, const void* w, void* wt, int co, int kh, int kw,
                                        int ci, hipStream_t s);
int conv_nt_mtiles(long M);  // upper bound on BN-stat partial tiles (128-row tiles)
// rows per BN-stat partial tile of the kernel launch_conv_nt will pick (128 or 256)
int conv_nt_stat_rows(int dtype, int out_f32, const ConvArgs& a);
bool conv_nt_v2_ok(const ConvArgs& a);
int conv_nt_v2_rows(const ConvArgs& a);   // tile rows (= BN-stat partial rows) of the v2 config
// true when launch_conv_nt runs the v2 kernel
bool conv_nt_uses_v2(int dtype, int out_f32, const ConvArgs& a);
hipError_t launch_conv_nt_v2(int dtype, const ConvArgs& a, hipStream_t s);
// the v2 kernel's K-concatenated second GEMM (ConvArgs::x2): dense 1x1, stride 1, Co <= 128, no
// residual or statistics (launch_conv_nt_v2 takes it when x2 is set)
bool conv_nt_v2_dual_ok(const ConvArgs& a);
// skinny 1x1 convs (skinny.hip): N <= 16 (the logits convs, with BN partials per 128 rows) or
// K <= 16 (their data gradients), 16-bit storage; taken where the v2 kernels cannot run
bool conv_skinny_ok(int dtype, int out_f32, const ConvArgs& a);
hipError_t launch_conv_skinny(int dtype, const ConvArgs& a, hipStream_t s);
// ping-pong 256x256 main loop (conv_pp.hip) for the v2 cases with Co > 128
bool conv_nt_pp_ok(const ConvArgs& a);
hipError_t launch_conv_nt_pp(int dtype, const ConvArgs& a, hipStream_t s);
// launches that apply ConvArgs::omask: 16-bit dense 1x1 ping-pong, one tile per workgroup (the
// identity units' conv1 data gradient with its residual; a projection unit's K-concatenated
// conv1 + shortcut data gradient; decrease_fdims' data gradient into block4)
bool conv_nt_omask_ok(int dtype, const ConvArgs& a);
// ping-pong 256x256 weight gradient (conv_pp.hip), used when the v2 tile choice is 256 x 256
bool conv_wgrad_pp_ok(const WgradArgs& a);
hipError_t launch_conv_wgrad_pp(int dtype, const WgradArgs& a, hipStream_t s);
bool conv_wgrad_v2_ok(const WgradArgs& a);
// small-channel 3 x 3 stride-1 weight gradient on input patches (wgrad_patch.hip): Co, C in
// {64, 128}, Wo % 64 == 0; grid = conv_wgrad_patch_blocks x splits
bool conv_wgrad_patch_ok(const WgradArgs& a);
int conv_wgrad_patch_blocks(const WgradArgs& a);
hipError_t launch_conv_wgrad_patch(int dtype, const WgradArgs& a, hipStream_t s);
hipError_t launch_conv_wgrad_v2(int dtype, const WgradArgs& a, hipStream_t s);
hipError_t launch_conv_wgrad_v2_tile(int dtype, const WgradArgs& a, int bm, int bn, hipStream_t s);
void conv_wgrad_v2_tile(int Co, int Ncol, long P, int* bm, int* bn);

// 7x7 / 2 stem (3 channels) in 16-bit storage as a 4x4 / 1 VALID conv over a space-to-depth
// image: X'[n][i][j][(dh*2 + dw)*3 + c] = x[n][2i + dh - pad_h][2j + dw - pad_w][c] (channels
// 12..15 zero), Hs = Ho + 3, Ws = Wo + 3; w'[co][a][b][(dh*2 + dw)*3 + c] = w[co][2a+dh][2b+dw][c]
// (zero past the 7x7 kernel), K = 4 * 4 * 16 = 256 (tap mode, tap8 = 2)
//   images f32 [N][H][W][3] -> s2d [N][Hs][Ws][16]
hipError_t launch_cast_s2d(int dtype, const float* src, void* dst, int N, int H, int W, int Hs, int Ws,
                           int pad_h, int pad_w, hipStream_t s);
//   s2d [N][Hs][Ws][16] -> [N][H][W][8] (channels 0..2 the image, 3..7 zero): parity tests' view
hipError_t launch_unshuffle_s2d(const void* src, void* dst, int N, int H, int W, int Hs, int Ws,
                                int pad_h, int pad_w, hipStream_t s);
//   weights 16-bit [Co][7][7][3] -> [Co][256]
hipError_t launch_stem_s2d_weights(const bf16_t* w, bf16_t* wp, int co, hipStream_t s);
//   split-K slabs [splits][co_pad][256] of the s2d weight gradient -> fp32 [co][7][7][3]
hipError_t launch_splitk_reduce_s2d(const float* part, int splits, long split_stride, int co,
                                    float* out, hipStream_t s);
