// Weak-label generation on the GPU: the bbox and image-tag label maps the
// loss head consumes, produced on device from box lists instead of host-rasterised 126 MB
// per-image tensors.
//
//   bbox (input_subset_bboxes_v2.py:74-98, then resize_images_and_labels / utils.py:181-241):
//     boxes are rasterised at the SOURCE image size (xmin = int(x0 * w) ..., float64 product,
//     rla[ymin:ymax+1, xmin:xmax+1, cid] += 1), normalised per pixel to a multinomial (void
//     channel 14 where no box covers the pixel), nearest-neighbour resized (TF 1.12
//     ResizeNearestNeighbor, align_corners = False: src = min(floorf(dst * (in/out)), in-1))
//     to the aspect-preserving size and cropped at (oy, ox). All three steps are fused: each
//     output pixel maps to one source pixel and counts the boxes covering it.
//   tag (input_subset_image_labels.py:73-107): a normalised 15-vector tiled over H x W.
#pragma once
#include "seg_common.h"

#define SEG_WEAK_CLASSES 15

struct BboxGeom {   // per image
  int src_h, src_w;   // rasterisation size (decoded image)
  int rh, rw;         // nearest-neighbour resized size (>= H, W)
  int oy, ox;         // crop offset into the resized map
};

// boxes [total][4] = (xmin, xmax, ymin, ymax) normalised, cids [total], box_off [n+1] prefix
// offsets per image, geom [n]; out [n][H][W][15] fp32
hipError_t launch_bbox_labels(const float* boxes, const int* cids, const int* box_off,
                              const BboxGeom* geom, int n, int H, int W, float* out, hipStream_t s);
// tags [n][15] (already normalised) -> out [n][H][W][15]
hipError_t launch_tag_labels(const float* tags, int n, int H, int W, float* out, hipStream_t s);
