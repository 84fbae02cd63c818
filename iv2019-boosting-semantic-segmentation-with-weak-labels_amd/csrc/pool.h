// Pooling, subsampling, pyramid (PSP/ASPP) pooling and align-corners bilinear resize.
#pragma once
#include "seg_common.h"

// Separable "grid reduction" spec: for pyramid pools (VALID avg pool, kernel = stride) and
// for the transpose of an align_corners bilinear resize from a small k x k grid.
#define SEG_MAX_GRIDS 4
#define SEG_MAX_CELLS 24
struct GridSpec {
  int n;                          // number of grids
  int kr[SEG_MAX_GRIDS];          // grid rows (cells along H)
  int kc[SEG_MAX_GRIDS];          // grid cols (cells along W)
  int kh[SEG_MAX_GRIDS];          // avg-pool window (psp_input_bwd only)
  int kw[SEG_MAX_GRIDS];
  int ccell_off[SEG_MAX_GRIDS];   // first column-cell of grid g in a row's cell list
  int rcell_off[SEG_MAX_GRIDS];   // first row-cell of grid g in coltab
  int total_ccells;               // sum_g kc[g]
  int total_rcells;               // sum_g kr[g]
  float scale[SEG_MAX_GRIDS];     // output scale per grid (1/(kh*kw) for avg pool)
  const float* rowtab;            // device [total_ccells][W]: weight of column w for cell
  const float* coltab;            // device [total_rcells][H]: weight of row h for cell
};

// max pool 3x3/2 (TF SAME): also writes the first-max window index (0..8) per output
// element to arg[N*Ho*Wo][C] (bytes); the backward gathers through it
hipError_t launch_maxpool_fwd(int dtype, const void* x, int N, int H, int W, int C, int ldx,
                              void* y, int Ho, int Wo, int ldy, int pad_h, int pad_w, void* arg,
                              hipStream_t s);
// the stem's BN apply + ReLU fused into the 3x3/2 max-pool (C = 64, even H and W, no top / left
// padding): z = relu((y - mean) * scale + beta) is rounded to the storage type per window tap
// and pooled as the max-pool would pool the stored z; the ReLU bits of every input pixel are
// written by the one window whose top-left 2 x 2 holds it; z itself is never stored
hipError_t launch_bn_relu_maxpool_fwd(int dtype, const void* y, int N, int H, int W, int ldy,
                                      const float* mean, const float* scale, const float* beta,
                                      uint8_t* mask, void* p, int Ho, int Wo, int ldp, int pad_h,
                                      int pad_w, uint8_t* arg, hipStream_t s);
hipError_t launch_maxpool_bwd(int dtype, const void* arg, int N, int H, int W, int C,
                              const void* dy, int Ho, int Wo, int lddy, void* dx, int lddx,
                              int pad_h, int pad_w, hipStream_t s);
// dx[n][ho*s][wo*s][c] += g[n][ho][wo][c]
hipError_t launch_add_strided(int dtype, void* dx, int H, int W, int lddx, const void* g, int N,
                              int Ho, int Wo, int C, int ldg, int stride, hipStream_t s);
// rows pass: part[n][h][cell][c] = sum_w x[n][h][w][c] * weight(g, w, cell)
hipError_t launch_grid_rowreduce(int dtype, const void* x, int N, int H, int W, int C, int ldx,
                                 const GridSpec& g, float* part, hipStream_t s);
// cols pass: out_g[n][i][j][c] = scale * sum_h part[n][h][cell(g,j)][c] * weight(g, h, i)
hipError_t launch_grid_colreduce(int dtype, const float* part, int N, int H, int W, int C,
                                 const GridSpec& g, void* const* outs, hipStream_t s);
// align_corners bilinear resize small [N][k][k][C] -> [N][Ho][Wo] slice (ld)
hipError_t launch_resize_fwd(int dtype, const void* x, int N, int hi, int wi, int C, int ldx,
                             void* y, int Ho, int Wo, int ldy, hipStream_t s);
// dx = dconcat_slice + sum_g avgpool_bwd(dpooled_g)   (PSP input gradient)
hipError_t launch_psp_input_bwd(int dtype, const void* dcat, int ldcat, const GridSpec& g,
                                const void* const* dpooled, int N, int H, int W, int C, void* dx,
                                int lddx, hipStream_t s);
