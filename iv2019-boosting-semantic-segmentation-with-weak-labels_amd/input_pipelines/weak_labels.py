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
        xmin, xmax, ymin, ymax = (int(c[0] * w), int(c[1] * w), int(c[2] * h), int(c[3] * h))
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
