// Input preprocessing on the GPU: the per-image transforms the
// reference's tf.data map functions run on decoded PNGs (input_cityscapes.py:66-96,190-209).
//   images: uint8 [n][Hr][Wr][3] -> tf.image.convert_image_dtype (x * float(1/255)) ->
//           tf.image.resize_images BILINEAR, align_corners = False (TF 1.12 legacy scaler:
//           scale = in/out, in_f = o * scale, lo = (int)in_f, hi = min(lo+1, in-1)) ->
//           from_0_1_to_m1_1 ((x - 0.5) / 0.5) -> fp32 [n][H][W][3]
//   labels: uint8 label ids [n][Hr][Wr] -> tf.gather(lids2cids (voids replaced)) ->
//           NEAREST_NEIGHBOR resize (src = min(floorf(o * in/out), in-1)) -> int32 [n][H][W]
// Host side: TFRecord / tf.train.Example / PNG decode (input_pipelines/tfrecords.py).
#pragma once
#include "seg_common.h"

#define SEG_MAX_LIDS 256

struct LidMap { int n; int cid[SEG_MAX_LIDS]; };

// resized to Hs x Ws, then the H x W window at (cy, cx) (plain resize: Hs = H, Ws = W, 0, 0)
hipError_t launch_prepare_images(const uint8_t* raw, int n, int Hr, int Wr, int Hs, int Ws,
                                 int cy, int cx, int H, int W, float* out, hipStream_t s);
hipError_t launch_prepare_labels(const uint8_t* raw, int n, int Hr, int Wr, int H, int W,
                                 const LidMap& m, int32_t* out, hipStream_t s);
