"""TEST INFRASTRUCTURE — the TF-semantics convolution restated as K*K shifted GEMMs.

Only tests/ may import this module. ``conv_tf`` (``oracle/tfseg.py``: slim ``conv2d`` with TF
'SAME' padding, or ``resnet_utils.conv2d_same``'s explicit padding for stride > 1, as called
at ``models/resnet50_extended_feature_extractor.py:25-30`` and
``models/resnet50_extended_model_hierarchical.py:59-64``) is rewritten here as a sum over the
K*K taps of a shifted read times one weight slice, for the forward, the data gradient (its
adjoint: the same shifted slices accumulated) and the weight gradient (the full pixel
reduction per tap). Nothing but slicing and matrix products, so the same code runs on CPU
tensors (``tests/test_oracle.py`` pins it to ``conv_tf`` and its autograd) and on float64
CUDA tensors, where the 1024 x 2048 layers of a C2 step are checked element by element in
about a second (torch is plumbing here: the arithmetic is the restated sum, in float64).

Tensors are NHWC; weights [Co][K][K][Ci].
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from oracle.tfseg import ConvSpec, same_pads


def geometry(H: int, W: int, spec: ConvSpec):
    """(Ho, Wo, pad_top, pad_left, pad_bottom, pad_right) exactly as conv_tf pads."""
    keff = spec.k + (spec.k - 1) * (spec.rate - 1)
    if spec.explicit_pad:
        pb = (keff - 1) // 2
        pt, pbot, pl, pr = pb, keff - 1 - pb, pb, keff - 1 - pb
    else:
        pt, pbot = same_pads(H, spec.k, spec.stride, spec.rate)
        pl, pr = same_pads(W, spec.k, spec.stride, spec.rate)
    Ho = (H + pt + pbot - keff) // spec.stride + 1
    Wo = (W + pl + pr - keff) // spec.stride + 1
    return Ho, Wo, pt, pl, pbot, pr


def _tap(xp, spec, i, j, Ho, Wo):
    """xp[:, i*r + s*ho, j*r + s*wo, :] for every output pixel (ho, wo) (a strided view)."""
    s, r = spec.stride, spec.rate
    return xp[:, i * r: i * r + s * (Ho - 1) + 1: s, j * r: j * r + s * (Wo - 1) + 1: s, :]


def conv_fwd(x, w, spec):
    """conv_tf(x, w) in NHWC: sum over taps of shifted(x) @ w[:, i, j, :]^T  ->  [N, Ho, Wo, Co]."""
    H, W = x.shape[1], x.shape[2]
    Ho, Wo, pt, pl, pb, pr = geometry(H, W, spec)
    xp = F.pad(x, (0, 0, pl, pr, pt, pb))
    out = torch.zeros(x.shape[0], Ho, Wo, w.shape[0], dtype=x.dtype, device=x.device)
    for i in range(spec.k):
        for j in range(spec.k):
            out += _tap(xp, spec, i, j, Ho, Wo) @ w[:, i, j, :].T
    return out


def conv_dgrad(dy, w, spec, H: int, W: int):
    """d conv_tf / dx applied to dy: each tap's dy @ w[:, i, j, :] added back onto the shifted
    input positions it was read from  ->  [N, H, W, Ci]."""
    Ho, Wo, pt, pl, pb, pr = geometry(H, W, spec)
    assert dy.shape[1:3] == (Ho, Wo)
    acc = torch.zeros(dy.shape[0], H + pt + pb, W + pl + pr, w.shape[3], dtype=dy.dtype,
                      device=dy.device)
    for i in range(spec.k):
        for j in range(spec.k):
            _tap(acc, spec, i, j, Ho, Wo).add_(dy @ w[:, i, j, :])
    return acc[:, pt:pt + H, pl:pl + W]


def conv_wgrad(x, dy, spec):
    """d conv_tf / dw applied to dy: dW[:, i, j, :] = dy^T @ shifted(x) over every pixel
    ->  [Co, K, K, Ci]."""
    H, W = x.shape[1], x.shape[2]
    Ho, Wo, pt, pl, pb, pr = geometry(H, W, spec)
    assert dy.shape[1:3] == (Ho, Wo)
    xp = F.pad(x, (0, 0, pl, pr, pt, pb))
    Co, Ci = dy.shape[-1], x.shape[-1]
    d2 = dy.reshape(-1, Co)
    out = torch.zeros(Co, spec.k, spec.k, Ci, dtype=x.dtype, device=x.device)
    for i in range(spec.k):
        for j in range(spec.k):
            out[:, i, j, :] = d2.T @ _tap(xp, spec, i, j, Ho, Wo).reshape(-1, Ci)
    return out
