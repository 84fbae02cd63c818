"""Seeded parameter initialisation with the reference's initializer semantics.

Conv weights: ``slim.variance_scaling_initializer()`` (factor 2.0, FAN_IN, truncated normal
with stddev sqrt(1.3 * 2 / fan_in)) — the arg scope at hierarchical.py:336-339; the hybrid
upsampler's conv2d_transpose weights the same (hierarchical.py:174-175; fan_in = 9 C, stored
(Cin, 3, 3, Cout)), its biases 0. BN: gamma 1, beta 0, moving mean 0, moving variance 1. The ImageNet warm start
(define_initializers.py:72-131) needs a checkpoint that is not available.

Seeding scheme (documented so any implementation reproduces it): the i-th conv in
TF variable-creation order draws from ``np.random.default_rng([seed, i])`` in float64,
``standard_normal`` redrawn outside +-2, scaled by the stddev, stored [Co][KH][KW][Ci].
"""
from __future__ import annotations

import math

import numpy as np


def _truncated_normal(rng, shape, std):
    x = rng.standard_normal(size=shape)
    bad = np.abs(x) > 2.0
    while bad.any():
        x[bad] = rng.standard_normal(size=int(bad.sum()))
        bad = np.abs(x) > 2.0
    return x * std


def init_params(param_info, seed=0):
    """param_info: list of seg_hip.ParamInfo in creation order (weights carry their
    (Co, KH, KW, Ci) shape)."""
    out = {}
    conv_index = 0
    for p in param_info:
        if p.kind == 'weights':
            shape = tuple(int(d) for d in p.shape)
            rng = np.random.default_rng([seed, conv_index])
            conv_index += 1
            fan_in = shape[1] * shape[2] * shape[3]
            out[p.name] = _truncated_normal(rng, shape, math.sqrt(1.3 * 2.0 / fan_in)).astype(np.float32)
        elif p.kind == 'gamma' or p.kind == 'moving_variance':   # BatchNorm or GroupNorm gamma
            out[p.name] = np.ones(p.numel, np.float32)
        else:
            out[p.name] = np.zeros(p.numel, np.float32)
    return out
