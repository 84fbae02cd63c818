"""Weak-label tensors of the reference's OpenImages pipelines (numpy, host side).

Restates the label semantics the hot path consumes (dataset I/O itself is out of scope):

* ``generate_bbox_rla``  — ``open_images/input_subset_bboxes_v2.py:74-98``: boxes are
  rasterised into a 15-channel per-pixel count map (``rla[ymin:ymax+1, xmin:xmax+1, cid]
  += 1`` with coordinates ``int(coord * size)``), then normalised per pixel to a
  multinomial; pixels with no box get the void channel (14).
* ``generate_tag_rla``   — ``open_images/input_subset_image_labels.py:73-96``: the set of
  image-level tags becomes a normalised 15-vector (void if empty), tiled over H x W
  (``:107``).
"""
from __future__ import annotations

import numpy as np

# mid2cid (input_subset_bboxes_v2.py:38-53): 14 classes + void
N_WEAK_CLASSES = 15
VOID = 14


def generate_bbox_rla(cids, coords_normalized, size):
    """cids: iterable of class ids in [0, 13]; coords: (xmin, xmax, ymin, ymax) in [0, 1]."""
    h, w = size
    rla = np.zeros((h, w, N_WEAK_CLASSES), dtype=np.float32)
    for cid, c in zip(cids, coords_normalized):
        # float32 coordinate x integer size is promoted to float64 by numpy in the reference
        # (np.float32 * np.int32/np.int64), then truncated
        xmin, xmax, ymin, ymax = (int(float(c[0]) * w), int(float(c[1]) * w),
                                  int(float(c[2]) * h), int(float(c[3]) * h))
        rla[ymin:ymax + 1, xmin:xmax + 1, cid] += 1
    s = np.sum(rla, axis=2, keepdims=True)
    void = np.zeros(N_WEAK_CLASSES, dtype=np.float32)
    void[VOID] = 1.0
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.where(s > 0.5, rla / s, void).astype(np.float32)


def generate_tag_rla(cids):
    rla = np.zeros(N_WEAK_CLASSES, dtype=np.float32)
    for c in cids:
        rla[c] = 1.0
    if not len(cids):
        rla[VOID] = 1.0
    return rla / np.sum(rla)


# ---- resize + crop of the label maps (input_pipelines/utils.py:181-241, utils/utils.py:531-596)

def aspect_preserving_size(src_h, src_w, target_h, target_w, mode="max"):
    """resize_images_or_labels(preserve_aspect_ratio=True) target size: the scale factor is
    max (mode 'max') or min of target/src per axis in float64, dims = ceil(scale * dim)
    (utils/utils.py:567-585)."""
    sh, sw = float(target_h) / float(src_h), float(target_w) / float(src_w)
    s = max(sh, sw) if mode == "max" else min(sh, sw)
    return int(np.ceil(s * float(src_h))), int(np.ceil(s * float(src_w)))


def nearest_index(in_size, out_size):
    """TF 1.12 ResizeNearestNeighbor, align_corners=False: src = min(floorf(dst * scale),
    in - 1) with scale = in / out computed in float32."""
    scale = np.float32(in_size) / np.float32(out_size)
    d = np.arange(out_size, dtype=np.float32)
    return np.minimum(np.floor(d * scale).astype(np.int64), in_size - 1)


def bbox_label_map(cids, coords_normalized, src_size, resized_size, offset, out_size):
    """Host restatement of one bbox-weak label of the training input: rasterise at the source
    size (generate_bbox_rla), nearest-neighbour resize to resized_size, crop out_size at
    offset (the random crop of resize_images_and_labels, utils.py:219-232)."""
    rla = generate_bbox_rla(cids, coords_normalized, src_size)
    iy = nearest_index(src_size[0], resized_size[0])[offset[0]:offset[0] + out_size[0]]
    ix = nearest_index(src_size[1], resized_size[1])[offset[1]:offset[1] + out_size[1]]
    return np.ascontiguousarray(rla[iy][:, ix])


class BboxLabelsGPU:
    """Device-side bbox / tag label maps through the C ABI (seg_bbox_labels / seg_tag_labels):
    the [n][H][W][15] tensors the loss head reads are produced on the GPU from box lists."""

    def __init__(self, height, width, device):
        self.h, self.w, self.device = height, width, device

    def bbox(self, images, out=None, stream=None):
        """images: list of (cids, coords (k, 4) = (xmin, xmax, ymin, ymax), src_size (h, w),
        resized_size (h, w), offset (y, x)). Returns a device tensor [n, H, W, 15]."""
        import torch
        from seg_hip import LIB, check
        n = len(images)
        counts = [len(im[0]) for im in images]
        if max(counts, default=0) > 1024:
            raise ValueError("at most 1024 boxes per image (reference MAX_N_BBOXES = 516)")
        for cids, coords, src, rs, off in images:
            if rs[0] < off[0] + self.h or rs[1] < off[1] + self.w:
                raise ValueError(f"crop {off} + {(self.h, self.w)} outside the resized map {rs}")
            if len(cids) and (np.min(cids) < 0 or np.max(cids) >= N_WEAK_CLASSES - 1):
                raise ValueError("box class ids must be in [0, 13]")
        boxes = np.zeros((max(sum(counts), 1), 4), np.float32)
        cid = np.zeros(max(sum(counts), 1), np.int32)
        off = np.zeros(n + 1, np.int32)
        geom = np.zeros((max(n, 1), 6), np.int32)
        for i, (cids, coords, src, rs, o) in enumerate(images):
            k = counts[i]
            off[i + 1] = off[i] + k
            if k:
                boxes[off[i]:off[i + 1]] = np.asarray(coords, np.float32).reshape(k, 4)
                cid[off[i]:off[i + 1]] = np.asarray(cids, np.int32)
            geom[i] = (src[0], src[1], rs[0], rs[1], o[0], o[1])
        dev = torch.device(self.device)
        tb, tc, to, tg = (torch.as_tensor(x).to(dev) for x in (boxes, cid, off, geom))
        if out is None:
            out = torch.empty((n, self.h, self.w, N_WEAK_CLASSES), dtype=torch.float32, device=dev)
        s = (stream or torch.cuda.current_stream()).cuda_stream
        check(LIB.seg_bbox_labels(tb.data_ptr(), tc.data_ptr(), to.data_ptr(), tg.data_ptr(), n,
                                  max(counts, default=0), self.h, self.w, out.data_ptr(), s))
        return out

    def tags(self, tag_sets, out=None, stream=None):
        """tag_sets: list of class-id lists -> device tensor [n, H, W, 15] (tiled)."""
        import torch
        from seg_hip import LIB, check
        n = len(tag_sets)
        t = torch.as_tensor(np.stack([generate_tag_rla(list(c)) for c in tag_sets]).astype(np.float32))
        t = t.to(torch.device(self.device))
        if out is None:
            out = torch.empty((n, self.h, self.w, N_WEAK_CLASSES), dtype=torch.float32, device=t.device)
        s = (stream or torch.cuda.current_stream()).cuda_stream
        check(LIB.seg_tag_labels(t.data_ptr(), n, self.h, self.w, out.data_ptr(), s))
        return out


class BoxLists(list):
    """A bbox-weak sub-batch as box lists: items (cids, coords (k, 4), src_size, resized_size,
    offset), as the reference's prebatch map sees them before _generate_rla. Passed as
    labels['prolabels_per_bbox'], it is rasterised on the device by define_losses."""


class TagSets(list):
    """An image-tag sub-batch as class-id lists (labels['prolabels_per_image'])."""


def synthetic_box_lists(rng, n, out_size, max_boxes=20, src_sizes=((1024, 2048), (768, 1024), (1200, 1600))):
    """Seeded random box lists with the reference's aspect-preserving resize + random crop
    geometry (sizes drawn from src_sizes)."""
    items = BoxLists()
    for _ in range(n):
        k = int(rng.integers(0, max_boxes + 1))
        cids = rng.integers(0, N_WEAK_CLASSES - 1, size=k)
        a, b = rng.random((k, 2)).astype(np.float32), rng.random((k, 2)).astype(np.float32)
        coords = np.stack([np.minimum(a[:, 0], b[:, 0]), np.maximum(a[:, 0], b[:, 0]),
                           np.minimum(a[:, 1], b[:, 1]), np.maximum(a[:, 1], b[:, 1])], 1)
        src = src_sizes[int(rng.integers(0, len(src_sizes)))]
        rs = aspect_preserving_size(src[0], src[1], out_size[0], out_size[1])
        off = (int(rng.integers(0, rs[0] - out_size[0] + 1)), int(rng.integers(0, rs[1] - out_size[1] + 1)))
        items.append((cids, coords, src, rs, off))
    return items
