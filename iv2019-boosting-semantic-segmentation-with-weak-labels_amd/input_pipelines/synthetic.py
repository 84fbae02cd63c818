"""Seeded synthetic batches in the reference's input contract.

Batch layout (per_pixel_per_bbox_per_image.py:50-77): images of the three sub-batches are
concatenated on axis 0, strong (per-pixel) first, then per-bbox, then per-image.
Images follow input_pipelines/utils.py:96-112: uint8 -> [0,1) -> (x - 0.5) / 0.5.
"""
from __future__ import annotations

import numpy as np

from input_pipelines.weak_labels import generate_bbox_rla, generate_tag_rla


def images(rng, n, h, w):
    u8 = rng.integers(0, 256, size=(n, h, w, 3), dtype=np.uint8)
    return ((u8.astype(np.float32) / 255.0) - 0.5) / 0.5


def pixel_labels(rng, n, h, w, n_classes=20, patch=32, void_frac=0.1):
    """Blocky patches of class ids; ~void_frac of the patches are void (last id)."""
    gh, gw = -(-h // patch), -(-w // patch)
    grid = rng.integers(0, n_classes - 1, size=(n, gh, gw))
    grid = np.where(rng.random((n, gh, gw)) < void_frac, n_classes - 1, grid)
    lab = np.repeat(np.repeat(grid, patch, axis=1), patch, axis=2)[:, :h, :w]
    return np.ascontiguousarray(lab.astype(np.int32))


def bbox_labels(rng, n, h, w, max_boxes=20):
    out = np.empty((n, h, w, 15), dtype=np.float32)
    for i in range(n):
        k = int(rng.integers(0, max_boxes + 1))
        cids = rng.integers(0, 14, size=k)
        a = rng.random((k, 2))
        b = rng.random((k, 2))
        coords = np.stack([np.minimum(a[:, 0], b[:, 0]), np.maximum(a[:, 0], b[:, 0]),
                           np.minimum(a[:, 1], b[:, 1]), np.maximum(a[:, 1], b[:, 1])], 1)
        out[i] = generate_bbox_rla(cids, coords, (h, w))
    return out


def tag_labels(rng, n, h, w):
    out = np.empty((n, h, w, 15), dtype=np.float32)
    for i in range(n):
        k = int(rng.integers(0, 5))
        out[i] = generate_tag_rla(sorted(set(rng.integers(0, 14, size=k).tolist())))[None, None, :]
    return out


def batch(seed, nb_pp, nb_pb, nb_pi, h, w):
    rng = np.random.default_rng(seed)
    n = nb_pp + nb_pb + nb_pi
    return dict(images=images(rng, n, h, w),
                px=pixel_labels(rng, nb_pp, h, w),
                bbox=bbox_labels(rng, nb_pb, h, w) if nb_pb else None,
                tag=tag_labels(rng, nb_pi, h, w) if nb_pi else None)


def evaluate_input(config, params, seed=1234, device=None):
    """EVAL input_fn in the reference's contract (input_cityscapes.py evaluate_input):
    endless seeded batches of ({'proimages'}, {'prolabels'}) as device tensors, Nb images
    per rank at the network size, labels at (label_height, label_width) when the settings
    carry them (default: the network size)."""
    import torch
    from input_pipelines.utils import get_temp_Nb
    nb = get_temp_Nb(config, params.Nb)
    h, w = params.height_feature_extractor, params.width_feature_extractor
    hl = getattr(params, 'label_height', None) or h
    wl = getattr(params, 'label_width', None) or w
    dev = device or torch.device('cuda', torch.cuda.current_device())
    rng = np.random.default_rng(seed)
    while True:
        imgs = torch.from_numpy(images(rng, nb, h, w)).to(dev)
        labs = torch.from_numpy(pixel_labels(rng, nb, hl, wl).astype(np.int32)).to(dev)
        yield {'proimages': imgs}, {'prolabels': labs}


def predict_input(config, params, seed=4321, device=None):
    """PREDICT input_fn: seeded ({'proimages'}, None) batches of Nb images."""
    import torch
    from input_pipelines.utils import get_temp_Nb
    nb = get_temp_Nb(config, params.Nb)
    h, w = params.height_feature_extractor, params.width_feature_extractor
    dev = device or torch.device('cuda', torch.cuda.current_device())
    rng = np.random.default_rng(seed)
    while True:
        yield {'proimages': torch.from_numpy(images(rng, nb, h, w)).to(dev)}, None
