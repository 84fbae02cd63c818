"""TEST INFRASTRUCTURE — CPU restatement of the reference training step (TF 1.12 semantics).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this module.

Everything here is written from the reference's source (cited file:line, paths relative to
the reference's ``code/`` directory) and from the published semantics of the third-party
library it calls, ``tensorflow==1.12.0`` (``requirements.txt:9``), which is not present in
the reference tree:

* slim ``resnet_v1`` / ``resnet_utils`` (``conv2d_same``, ``stack_blocks_dense``,
  ``subsample``, ``bottleneck``) — called at
  ``models/resnet50_extended_feature_extractor.py:25-30`` and
  ``models/resnet50_extended_model_hierarchical.py:59-64``;
* ``tf.contrib.layers.batch_norm`` (fused, training): batch mean, biased variance for the
  normalisation, Bessel-corrected variance for the moving average, epsilon clamped to
  1.001e-5 by ``nn.fused_batch_norm`` — used as ``normalizer_fn`` at
  ``models/resnet50_extended_model_hierarchical.py:325-339``;
* ``tf.image.resize_images(..., align_corners=True)`` (``ResizeBilinear`` legacy scaler) —
  ``models/resnet50_extended_model_hierarchical.py:167,193-202``;
* ``(sparse_)softmax_cross_entropy_with_logits`` whose backprop is ``softmax - labels``;
  ``tf.losses.compute_weighted_loss`` (``SUM_BY_NONZERO_WEIGHTS``, safe division);
  ``l2_regularizer`` (``scale * sum(w**2) / 2``); ``MomentumOptimizer``.

Tensors are NHWC at the interface; internally NCHW for torch's CPU conv. The default
arithmetic is float64 (fixtures); bench.py times the same code in float32.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

# ----------------------------------------------------------------------------------------
# configuration and architecture (slim resnet_v1 unit schedule)
# ----------------------------------------------------------------------------------------

BN_EPS = 1.001e-5  # tf.nn.fused_batch_norm clamps epsilon=1e-5 (hierarchical.py:335) up to this
GN_EPS = 1e-5      # group_norm takes norm_epsilon as given (hierarchical.py:313-317)


@dataclass
class SegConfig:
    depth: int = 50                  # 50 | 101  (add_model_arguments :239-240)
    pyramid: str = "psp"             # none | psp | aspp
    height: int = 512                # height_feature_extractor
    width: int = 1024
    nb_pp: int = 2                   # per-pixel (strong) images, first on the batch axis
    nb_pb: int = 0                   # per-bbox weak images
    nb_pi: int = 0                   # per-image (tag) weak images
    dataset: str = "cityscapes"
    output_stride: int = 8           # stride_feature_extractor default (:236)
    feature_dims_decreased: int = 256
    bn_decay: float = 0.9            # batch_norm_decay (:269)
    weight_decay: float = 0.00017    # regularization_weight (utils/utils.py:111)
    fov_k: int = 0                   # fov_expansion_kernel_size (hierarchical.py:247-250)
    fov_rate: int = 0                # fov_expansion_kernel_rate
    upsampling: str = "bilinear"     # upsampling_method (hierarchical.py:143-184): bilinear | hybrid
    norm: str = "batch"              # norm_layer (hierarchical.py:293-333): batch | group
    groups: int = 32                 # module_arg_scope groups (group norm; logits use 1)

    @property
    def nb(self) -> int:
        return self.nb_pp + self.nb_pb + self.nb_pi


@dataclass
class ConvSpec:
    name: str           # TF variable scope of the conv (weights are <name>/weights)
    ci: int
    co: int
    k: int
    stride: int = 1
    rate: int = 1
    explicit_pad: bool = False   # conv2d_same with stride>1: pad then VALID
    relu: bool = True            # activation after BN (conv3/shortcut/logits: None)


def _bottleneck_specs(scope: str, depth_in: int, depth: int, depth_bn: int, stride: int,
                      rate: int) -> List[ConvSpec]:
    """slim resnet_v1.bottleneck: shortcut(conv if depth changes) + 1x1 -> 3x3 -> 1x1."""
    specs = []
    if depth != depth_in:
        specs.append(ConvSpec(f"{scope}/shortcut", depth_in, depth, 1, stride, 1, relu=False))
    specs.append(ConvSpec(f"{scope}/conv1", depth_in, depth_bn, 1))
    specs.append(ConvSpec(f"{scope}/conv2", depth_bn, depth_bn, 3, stride, rate,
                          explicit_pad=(stride > 1)))
    specs.append(ConvSpec(f"{scope}/conv3", depth_bn, depth, 1, relu=False))
    return specs


def resnet_units(depth: int, output_stride: int):
    """stack_blocks_dense schedule for resnet_v1_{50,101} with output_stride.

    Returns a list of (scope, depth_in, depth, depth_bottleneck, stride, rate).
    Blocks: (base_depth, units, stride) = (64,3,2), (128,4,2), (256,6|23,2), (512,3,1); the
    stride sits on the LAST unit of each block; once the running stride reaches
    output_stride/4 (root block divides by 4) strides become rates.
    """
    n3 = {50: 6, 101: 23}[depth]
    blocks = [("block1", 64, 3, 2), ("block2", 128, 4, 2), ("block3", 256, n3, 2),
              ("block4", 512, 3, 1)]
    target = output_stride // 4
    current, rate = 1, 1
    depth_in = 64
    units = []
    for bname, base, n, bstride in blocks:
        for i in range(n):
            ustride = bstride if i == n - 1 else 1
            scope = f"{bname}/unit_{i + 1}/bottleneck_v1"
            if current == target:
                units.append((scope, depth_in, base * 4, base, 1, rate))
                rate *= ustride
            else:
                units.append((scope, depth_in, base * 4, base, ustride, 1))
                current *= ustride
            depth_in = base * 4
    return units


def n_classes(dataset: str):
    """(l1, l2_vehicle, l2_human) logits channels (hierarchical.py:81-83)."""
    return (53, 12, 5) if dataset == "vistas" else (14, 7, 3)


def psp_grids(hf: int, wf: int):
    """PSP pooling windows: kernel = stride = (hf/8, wf/8)//k (hierarchical.py:189-200)."""
    sd = np.array([hf, wf]) // 8
    out = []
    for k in (1, 2, 3, 6):
        kern = sd // k
        out.append((int(kern[0]), int(kern[1])))
    return out


def build_specs(cfg: SegConfig) -> List[ConvSpec]:
    """All convs in TF variable-creation order (each followed by BN)."""
    rn = f"feature_extractor/base/resnet_v1_{cfg.depth}"
    specs = [ConvSpec(f"{rn}/conv1", 3, 64, 7, 2, 1, explicit_pad=True)]
    for (scope, din, d, dbn, s, r) in resnet_units(cfg.depth, cfg.output_stride):
        specs += _bottleneck_specs(f"{rn}/{scope}", din, d, dbn, s, r)
    fd = cfg.feature_dims_decreased
    specs.append(ConvSpec("feature_extractor/extension/decrease_fdims", 2048, fd, 1))
    if cfg.fov_k > 0 and cfg.fov_rate > 0:
        # resnet50_extended_feature_extractor.py:44-49: slim.conv2d (SAME, BN, ReLU), fd -> fd
        specs.append(ConvSpec("feature_extractor/extension/increase_fov", fd, fd, cfg.fov_k, 1,
                              cfg.fov_rate))
    if cfg.pyramid == "psp":
        for i in range(4):
            specs.append(ConvSpec(f"feature_extractor/pyramid_module/Conv{'' if i == 0 else '_%d' % i}",
                                  fd, fd, 1))
        specs.append(ConvSpec("feature_extractor/pyramid_module/Conv_4", 5 * fd, fd, 1))
    elif cfg.pyramid == "aspp":
        # the commented spec at hierarchical.py:209-226, called where _create_psp_module is
        # (:55-57, variable scope 'pyramid_module'); slim names convs in creation order
        specs.append(ConvSpec("feature_extractor/pyramid_module/Conv", fd, fd, 1))    # image pool
        specs.append(ConvSpec("feature_extractor/pyramid_module/Conv_1", fd, fd, 1))  # 1x1
        for i, r in enumerate((6, 12, 18)):
            specs.append(ConvSpec(f"feature_extractor/pyramid_module/Conv_{i + 2}", fd, fd, 3, 1, r))
        specs.append(ConvSpec("feature_extractor/pyramid_module/Conv_5", 5 * fd, fd, 1))
    for head in ("l1_features", "l2_vehicle_features", "l2_human_features"):
        specs += _bottleneck_specs(f"adaptation_module/{head}", fd, fd, fd, 1, 1)
    c1, c2, c3 = n_classes(cfg.dataset)
    for nm, c in (("l1_logits", c1), ("l2_vehicle_logits", c2), ("l2_human_logits", c3)):
        specs.append(ConvSpec(f"softmax_classifier/{nm}", fd, c, 1, relu=False))
    return specs


# ----------------------------------------------------------------------------------------
# parameters: deterministic seeded init (documented PCG64 scheme)
# ----------------------------------------------------------------------------------------

def truncated_normal(rng: np.random.Generator, shape, std: float) -> np.ndarray:
    """TF truncated_normal: N(0, std) redrawn outside +-2 std."""
    x = rng.standard_normal(size=shape)
    bad = np.abs(x) > 2.0
    while bad.any():
        x[bad] = rng.standard_normal(size=int(bad.sum()))
        bad = np.abs(x) > 2.0
    return x * std


def init_params(cfg: SegConfig, seed: int = 0) -> Dict[str, np.ndarray]:
    """variance_scaling_initializer() (factor 2, FAN_IN, truncated normal, std=sqrt(1.3*2/fan_in))
    for conv weights, stored [Co][KH][KW][Ci]; BN gamma=1, beta=0, moving mean 0 / var 1.

    Seeding: conv ``i`` (creation order) draws from ``np.random.default_rng([seed, i])``
    in float64, then the product casts to its master dtype (fp32).
    """
    p = {}
    for i, s in enumerate(build_specs(cfg)):
        rng = np.random.default_rng([seed, i])
        fan_in = s.k * s.k * s.ci
        p[f"{s.name}/weights"] = truncated_normal(rng, (s.co, s.k, s.k, s.ci),
                                                 math.sqrt(1.3 * 2.0 / fan_in))
        if cfg.norm == "group":   # tf.contrib.layers.group_norm: gamma / beta only
            p[f"{s.name}/GroupNorm/gamma"] = np.ones(s.co)
            p[f"{s.name}/GroupNorm/beta"] = np.zeros(s.co)
            continue
        p[f"{s.name}/BatchNorm/gamma"] = np.ones(s.co)
        p[f"{s.name}/BatchNorm/beta"] = np.zeros(s.co)
        p[f"{s.name}/BatchNorm/moving_mean"] = np.zeros(s.co)
        p[f"{s.name}/BatchNorm/moving_variance"] = np.ones(s.co)
    if cfg.upsampling == "hybrid":
        n0 = len(build_specs(cfg))
        for h, c in enumerate(n_classes(cfg.dataset)):
            rng = np.random.default_rng([seed, n0 + h])
            name = deconv_scope(h)
            p[f"{name}/weights"] = truncated_normal(rng, (c, 3, 3, c), math.sqrt(1.3 * 2.0 / (9 * c)))
            p[f"{name}/biases"] = np.zeros(c)
    return p


def deconv_scope(h: int) -> str:
    """slim.conv2d_transpose default scope of head h's hybrid upsampler (hierarchical.py:168-180):
    created after the three logits convs inside softmax_classifier/upsampling."""
    return "softmax_classifier/upsampling/Conv2d_transpose" + ("", "_1", "_2")[h]


# ----------------------------------------------------------------------------------------
# primitive ops with TF 1.12 semantics (NCHW tensors)
# ----------------------------------------------------------------------------------------

def same_pads(n: int, k: int, s: int, rate: int = 1):
    """TF 'SAME': out = ceil(n/s); pad_total = max((out-1)*s + k_eff - n, 0); before = total//2."""
    keff = k + (k - 1) * (rate - 1)
    out = -(-n // s)
    tot = max((out - 1) * s + keff - n, 0)
    return tot // 2, tot - tot // 2


def conv_tf(x, w_ohwi, spec: ConvSpec):
    """slim.conv2d / resnet_utils.conv2d_same (no bias: normalizer_fn is set)."""
    w = w_ohwi.permute(0, 3, 1, 2)
    if spec.explicit_pad:
        keff = spec.k + (spec.k - 1) * (spec.rate - 1)
        pb = (keff - 1) // 2
        pe = keff - 1 - pb
        x = F.pad(x, (pb, pe, pb, pe))
        return F.conv2d(x, w, stride=spec.stride, dilation=spec.rate)
    ph = same_pads(x.shape[2], spec.k, spec.stride, spec.rate)
    pw = same_pads(x.shape[3], spec.k, spec.stride, spec.rate)
    x = F.pad(x, (pw[0], pw[1], ph[0], ph[1]))
    return F.conv2d(x, w, stride=spec.stride, dilation=spec.rate)


def bn_train(y, gamma, beta, eps=BN_EPS, bessel=True):
    """FusedBatchNorm training: returns (out, batch_mean, batch_var_bessel).

    bessel=False: the cross-replica path (utils/cross_replica_batch_normalization.py:400-425,
    run here over the replicas' concatenated batch): normalised by the global mean and the
    biased global variance, and that biased variance is the moving-average input (:452-466)."""
    n = y.shape[0] * y.shape[2] * y.shape[3]
    mean = y.mean(dim=(0, 2, 3))
    if bessel:
        var = ((y - mean[None, :, None, None]) ** 2).mean(dim=(0, 2, 3))
    else:   # the reference's formula (:418): E[x^2] - mean^2
        var = (y * y).mean(dim=(0, 2, 3)) - mean * mean
    scale = gamma * torch.rsqrt(var + eps)
    out = (y - mean[None, :, None, None]) * scale[None, :, None, None] + beta[None, :, None, None]
    return out, mean.detach(), (var * (n / max(n - 1, 1)) if bessel else var).detach()


def maxpool_same_3x3s2(x):
    """slim max_pool2d([3,3], stride=2, padding='SAME') (arg scope hierarchical.py:351-353)."""
    ph = same_pads(x.shape[2], 3, 2)
    pw = same_pads(x.shape[3], 3, 2)
    x = F.pad(x, (pw[0], pw[1], ph[0], ph[1]), value=float("-inf"))
    return F.max_pool2d(x, 3, 2)


def resize_tables(n_in: int, n_out: int):
    """TF ResizeBilinear(align_corners=True) legacy index/lerp computation, in float32.

    scale = (in-1)/(out-1) (float); in_f = i*scale (float); lower = (int64)in_f;
    upper = min(lower+1, in-1); lerp = in_f - lower.
    """
    scale = np.float32((n_in - 1) / np.float32(n_out - 1)) if n_out > 1 else np.float32(0.0)
    i = np.arange(n_out, dtype=np.float32)
    fin = (i * scale).astype(np.float32)
    lo = fin.astype(np.int64)
    hi = np.minimum(lo + 1, n_in - 1)
    lerp = (fin - lo.astype(np.float32)).astype(np.float32)
    return lo, hi, lerp


def nearest_ac_index(n_in: int, n_out: int):
    """TF 1.12 ResizeNearestNeighbor(align_corners=True) source rows: scale =
    (in-1)/(out-1) in float32 (in/out when out == 1), in = min(roundf(o*scale), in-1)
    (round half away from zero)."""
    scale = (np.float32(n_in - 1) / np.float32(n_out - 1) if n_out > 1
             else np.float32(n_in) / np.float32(n_out))
    f = (np.arange(n_out, dtype=np.float32) * np.float32(scale)).astype(np.float32)
    r = np.floor(f.astype(np.float64) + 0.5)   # f >= 0: roundf, exact in float64
    return torch.as_tensor(np.minimum(r.astype(np.int64), n_in - 1))


def prepare_images_np(raw_u8, H: int, W: int, resized=None, offset=(0, 0)):
    """Eval/train image preprocessing (input_cityscapes.py:190-209, 66-96):
    tf.image.convert_image_dtype (uint8 -> x * float32(1/255)), ResizeBilinear with
    align_corners=False (TF 1.12 legacy scaler: scale = in/out, in_f = o*scale, lo = (int),
    hi = min(lo+1, in-1), lerp = in_f - lo, all float32), from_0_1_to_m1_1 ((x-0.5)/0.5).
    raw_u8 [n, h, w, 3] -> float32 [n, H, W, 3]. With `resized` (h', w') and `offset` (y, x):
    the resize goes to h' x w' and the H x W window at the offset is returned (the
    preserve_aspect_ratio resize + random crop, input_pipelines/utils.py:206-232)."""
    raw = np.asarray(raw_u8)
    x = raw.astype(np.float32) * np.float32(1.0 / 255.0)
    rh, rw = resized if resized is not None else (H, W)

    def tables(n_in, n_out):
        scale = np.float32(np.float32(n_in) / np.float32(n_out))
        fin = (np.arange(n_out, dtype=np.float32) * scale).astype(np.float32)
        lo = fin.astype(np.int64)
        hi = np.minimum(lo + 1, n_in - 1)
        return lo, hi, (fin - lo.astype(np.float32)).astype(np.float32)
    cy, cx = offset
    yl, yh, ylr = (t[cy:cy + H] for t in tables(raw.shape[1], rh))
    xl, xh, xlr = (t[cx:cx + W] for t in tables(raw.shape[2], rw))
    xlr = xlr[None, None, :, None]
    ylr = ylr[None, :, None, None]
    tl, tr = x[:, yl][:, :, xl], x[:, yl][:, :, xh]
    bl, br = x[:, yh][:, :, xl], x[:, yh][:, :, xh]
    top = tl + (tr - tl) * xlr
    bot = bl + (br - bl) * xlr
    v = (top + (bot - top) * ylr).astype(np.float32)
    return ((v - np.float32(0.5)) / np.float32(0.5)).astype(np.float32)


def prepare_labels_np(raw_u8, H: int, W: int, lids2cids):
    """tf.gather(_replacevoids(lids2cids), label) then ResizeNearestNeighbor (align_corners
    False: src = min(floorf(o * float32(in/out)), in-1)). [n, h, w] uint8 -> int32."""
    raw = np.asarray(raw_u8)
    m = np.asarray(lids2cids, np.int64)
    m = np.where(m == -1, m.max() + 1, m)

    def src(n_in, n_out):
        scale = np.float32(np.float32(n_in) / np.float32(n_out))
        f = (np.arange(n_out, dtype=np.float32) * scale).astype(np.float32)
        return np.minimum(np.floor(f).astype(np.int64), n_in - 1)
    lab = m[raw.astype(np.int64)]
    return lab[:, src(raw.shape[1], H)][:, :, src(raw.shape[2], W)].astype(np.int32)


def resize_bilinear_ac(x, h_out: int, w_out: int):
    """align_corners bilinear with TF's arithmetic form:
    top = tl + (tr-tl)*xl; bottom = bl + (br-bl)*xl; out = top + (bottom-top)*yl."""
    yl, yh, ylr = resize_tables(x.shape[2], h_out)
    xl, xh, xlr = resize_tables(x.shape[3], w_out)
    ylr = torch.as_tensor(ylr, dtype=x.dtype)[None, None, :, None]
    xlr = torch.as_tensor(xlr, dtype=x.dtype)[None, None, None, :]
    yl, yh = torch.as_tensor(yl), torch.as_tensor(yh)
    xl, xh = torch.as_tensor(xl), torch.as_tensor(xh)
    top_rows = x[:, :, yl, :]
    bot_rows = x[:, :, yh, :]
    tl, tr = top_rows[:, :, :, xl], top_rows[:, :, :, xh]
    bl, br = bot_rows[:, :, :, xl], bot_rows[:, :, :, xh]
    top = tl + (tr - tl) * xlr
    bottom = bl + (br - bl) * xlr
    return top + (bottom - top) * ylr


class _XentTF(torch.autograd.Function):
    """softmax_cross_entropy_with_logits over dim=1: loss=-sum(y*log_softmax); backprop = p - y
    (TF's kernel ignores sum(y) != 1)."""

    @staticmethod
    def forward(ctx, logits, labels):
        logp = torch.log_softmax(logits, dim=1)
        ctx.save_for_backward(logp, labels)
        return -(labels * logp).sum(dim=1)

    @staticmethod
    def backward(ctx, g):
        logp, labels = ctx.saved_tensors
        return g.unsqueeze(1) * (logp.exp() - labels), None


def xent(logits, labels):
    return _XentTF.apply(logits, labels)


def weighted_loss(raw, w):
    """compute_weighted_loss, Reduction.SUM_BY_NONZERO_WEIGHTS with safe division."""
    num = (w != 0).sum()
    tot = (raw * w).sum()
    if int(num) == 0:
        return tot * 0.0, 0
    return tot / num, int(num)


# ----------------------------------------------------------------------------------------
# label tables (define_losses_hierarchical.py:37-93; hierarchical.py:88-117)
# ----------------------------------------------------------------------------------------

CITYSCAPES = dict(
    cid_l1_vehicle=12, cid_l1_human=11,
    pp2l1=[0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 11, 12, 12, 12, 12, 12, 12, 13],
    pb2l1=[12, 12, 12, 12, 12, 12, 11, 11, 11, 11, 11, 13, 13, 13, 13],
    pp2veh=[6] * 13 + [0, 1, 2, 3, 4, 5, 6],
    pb2veh=[5, 2, 0, 4, 3, 1, 6, 6, 6, 6, 6, 6, 6, 6, 6],
    pp2hum=[2] * 11 + [0, 1] + [2] * 7,
    pb2hum=[2, 2, 2, 2, 2, 2, 0, 0, 0, 0, 0, 2, 2, 2, 2],
    l1_to_common=[0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 19],
    veh_to_common=[13, 14, 15, 16, 17, 18, 19],
    hum_to_common=[11, 12, 19],
)


# Vistas: define_losses_hierarchical.py:38-74 (label remaps) and
# models/resnet50_extended_model_hierarchical.py:95-106 (decision fusion), as listed there
VISTAS = dict(
    cid_l1_vehicle=49, cid_l1_human=19,
    pp2l1=list(range(20)) + [19, 19, 19] + list(range(20, 50)) + [49] * 10 + [50, 51, 52],
    pb2l1=[49, 49, 49, 49, 49, 49, 19, 19, 19, 19, 19, 52, 52, 52, 52],
    pp2veh=[11] * 52 + list(range(11)) + [11, 11, 11],
    pb2veh=[0, 2, 3, 5, 6, 9, 11, 11, 11, 11, 11, 11, 11, 11, 11],
    pp2hum=[4] * 19 + [0, 1, 2, 3] + [4] * 43,
    pb2hum=[4, 4, 4, 4, 4, 4, 0, 0, 0, 0, 0, 4, 4, 4, 4],
    l1_to_common=list(range(20)) + list(range(23, 53)) + [63, 64, 65],
    veh_to_common=[52, 53, 54, 55, 56, 57, 58, 59, 60, 61, 62, 65],
    hum_to_common=[19, 20, 21, 22, 65],
)
assert len(VISTAS["pp2l1"]) == 66 and len(VISTAS["pp2veh"]) == 66 and len(VISTAS["pp2hum"]) == 66
assert len(VISTAS["l1_to_common"]) == 53
TABLES = {"cityscapes": CITYSCAPES, "vistas": VISTAS}


def _t(v):
    return torch.as_tensor(v, dtype=torch.long)


# ----------------------------------------------------------------------------------------
# the model (hierarchical.py:17-141) and losses (define_losses_hierarchical.py:14-217)
# ----------------------------------------------------------------------------------------

class OracleNet:
    """Functional restatement of ``model`` + ``define_losses`` + the SGDM step."""

    def __init__(self, cfg: SegConfig, params: Dict[str, np.ndarray], dtype=torch.float64):
        self.cfg = cfg
        self.specs = build_specs(cfg)
        self.spec_by_name = {s.name: s for s in self.specs}
        self.dtype = dtype
        self.p = {k: torch.tensor(v, dtype=dtype) for k, v in params.items()}
        self.batch_stats: Dict[str, tuple] = {}
        self.sync_bn = False   # cross-replica BN over a concatenated multi-replica batch
        self.bn_inference = False   # EVAL / PREDICT with batch_norm_accumulate_statistics unset

    # -- building blocks -------------------------------------------------------------
    def conv_bn(self, x, name: str, relu: Optional[bool] = None, record: Dict = None):
        s = self.spec_by_name[name]
        y = conv_tf(x, self.p[f"{name}/weights"], s)
        if self.cfg.norm == "group":
            # tf.contrib.layers.group_norm (module_arg_scope :313-333): per image, moments over
            # H x W x C/G (tf.nn.moments: biased), epsilon 1e-5; the softmax_classifier scope
            # passes groups=1 (hierarchical.py:78)
            G = 1 if name.startswith("softmax_classifier/") else self.cfg.groups
            n, c, h, w = y.shape
            yg = y.reshape(n, G, c // G, h, w)
            mean = yg.mean(dim=(2, 3, 4), keepdim=True)
            var = ((yg - mean) ** 2).mean(dim=(2, 3, 4), keepdim=True)
            xh = ((yg - mean) * torch.rsqrt(var + GN_EPS)).reshape(n, c, h, w)
            out = xh * self.p[f"{name}/GroupNorm/gamma"][None, :, None, None] + \
                self.p[f"{name}/GroupNorm/beta"][None, :, None, None]
            if record is not None:
                record[name] = y
            act = s.relu if relu is None else relu
            return torch.relu(out) if act else out
        if self.bn_inference:   # is_training=False (hierarchical.py:306-307): moving statistics
            mm = self.p[f"{name}/BatchNorm/moving_mean"]
            mv = self.p[f"{name}/BatchNorm/moving_variance"]
            sc = self.p[f"{name}/BatchNorm/gamma"] * torch.rsqrt(mv + BN_EPS)
            out = (y - mm[None, :, None, None]) * sc[None, :, None, None] + \
                self.p[f"{name}/BatchNorm/beta"][None, :, None, None]
            if record is not None:
                record[name] = y
            act = s.relu if relu is None else relu
            return torch.relu(out) if act else out
        out, m, v = bn_train(y, self.p[f"{name}/BatchNorm/gamma"], self.p[f"{name}/BatchNorm/beta"],
                             bessel=not self.sync_bn)
        self.batch_stats[name] = (m, v)
        if record is not None:
            record[name] = y
        act = s.relu if relu is None else relu
        return torch.relu(out) if act else out

    def bottleneck(self, x, scope: str, stride: int, rate: int, depth: int, record=None):
        depth_in = x.shape[1]
        if depth == depth_in:
            shortcut = x[:, :, ::stride, ::stride] if stride > 1 else x  # resnet_utils.subsample
        else:
            shortcut = self.conv_bn(x, f"{scope}/shortcut", relu=False, record=record)
        r = self.conv_bn(x, f"{scope}/conv1", record=record)
        r = self.conv_bn(r, f"{scope}/conv2", record=record)
        r = self.conv_bn(r, f"{scope}/conv3", relu=False, record=record)
        return torch.relu(shortcut + r)

    def psp(self, x, record=None):
        """_create_psp_module (hierarchical.py:186-207)."""
        cfg = self.cfg
        h, w = x.shape[2], x.shape[3]
        branches = [x]
        names = ["Conv", "Conv_1", "Conv_2", "Conv_3"]
        for (kh, kw), nm in zip(psp_grids(cfg.height, cfg.width), names):
            pooled = F.avg_pool2d(x, (kh, kw), stride=(kh, kw))
            c = self.conv_bn(pooled, f"feature_extractor/pyramid_module/{nm}", record=record)
            branches.append(resize_bilinear_ac(c, h, w))
        return self.conv_bn(torch.cat(branches, 1), "feature_extractor/pyramid_module/Conv_4",
                            record=record)

    def aspp(self, x, record=None):
        """ASPP per the commented spec (hierarchical.py:209-226); build-side, unpinned."""
        h, w = x.shape[2], x.shape[3]
        pooled = F.avg_pool2d(x, (h, w), stride=(h, w))
        c = self.conv_bn(pooled, "feature_extractor/pyramid_module/Conv", record=record)
        br = [resize_bilinear_ac(c, h, w),
              self.conv_bn(x, "feature_extractor/pyramid_module/Conv_1", record=record)]
        for i in range(3):
            br.append(self.conv_bn(x, f"feature_extractor/pyramid_module/Conv_{i + 2}", record=record))
        return self.conv_bn(torch.cat(br, 1), "feature_extractor/pyramid_module/Conv_5", record=record)

    # -- forward -------------------------------------------------------------------------
    def forward(self, images_nhwc, record=None):
        """Returns dict with low-res logits (l1, l2v, l2h) NCHW and encoder features."""
        cfg = self.cfg
        x = images_nhwc.permute(0, 3, 1, 2).to(self.dtype)
        rn = f"feature_extractor/base/resnet_v1_{cfg.depth}"
        x = self.conv_bn(x, f"{rn}/conv1", record=record)
        x = maxpool_same_3x3s2(x)
        for (scope, din, d, dbn, s, r) in resnet_units(cfg.depth, cfg.output_stride):
            x = self.bottleneck(x, f"{rn}/{scope}", s, r, d, record=record)
        x = self.conv_bn(x, "feature_extractor/extension/decrease_fdims", record=record)
        if cfg.fov_k > 0 and cfg.fov_rate > 0:
            x = self.conv_bn(x, "feature_extractor/extension/increase_fov", record=record)
        if cfg.pyramid == "psp":
            x = self.psp(x, record=record)
        elif cfg.pyramid == "aspp":
            x = self.aspp(x, record=record)
        feats = x
        heads = {}
        for h, head in enumerate(("l1", "l2_vehicle", "l2_human")):
            f = self.bottleneck(x, f"adaptation_module/{head}_features", 1, 1, x.shape[1],
                                record=record)
            heads[head] = self.conv_bn(f, f"softmax_classifier/{head}_logits", relu=False,
                                       record=record)
            if cfg.upsampling == "hybrid":
                # slim.conv2d_transpose(C, 3, SAME, stride 1, activation None, bias) before the
                # resize (hierarchical.py:168-180); TF filter [kh][kw][out][in] is stored
                # D[in][kh][kw][out], i.e. torch's conv_transpose2d weight [in][out][kh][kw]
                sc = deconv_scope(h)
                heads[head] = F.conv_transpose2d(heads[head], self.p[f"{sc}/weights"].permute(0, 3, 1, 2),
                                                 self.p[f"{sc}/biases"], padding=1)
        return {"features": feats, "l1_logits": heads["l1"],
                "l2_vehicle_logits": heads["l2_vehicle"], "l2_human_logits": heads["l2_human"]}

    # -- upsample + softmax + decisions (hierarchical.py:84-117) ------------------------
    def head_predictions(self, low):
        cfg = self.cfg
        up = {k: resize_bilinear_ac(low[k], cfg.height, cfg.width)
              for k in ("l1_logits", "l2_vehicle_logits", "l2_human_logits")}
        probs = {k: torch.softmax(v, dim=1) for k, v in up.items()}
        decs = {k: torch.argmax(v, dim=1) for k, v in probs.items()}
        t = TABLES[cfg.dataset]
        l1d, vd, hd = decs["l1_logits"], decs["l2_vehicle_logits"], decs["l2_human_logits"]
        fused = torch.where(l1d == t["cid_l1_vehicle"], _t(t["veh_to_common"])[vd],
                            torch.where(l1d == t["cid_l1_human"], _t(t["hum_to_common"])[hd],
                                        _t(t["l1_to_common"])[l1d]))
        return up, probs, decs, fused

    # -- EVAL / PREDICT decisions (define_estimator_hierarchical.py:161-194,215-232) ---
    def eval_decisions(self, low, cid_map, out_h, out_w, replace_voids=False):
        """_map_predictions_to_new_cids (:490-522) -> _replace_voids (:577-630) ->
        _resize_predictions (:524-575) of the fused decisions; returns int64 [N, out_h, out_w].

        The l1 probabilities keep their C1 channels: the segment-sum remap raises on a
        len(cid_map) != C1 map and is skipped by the reference's bare except (:509-515), so
        _replace_voids compares the MAPPED decisions with C1 - 1 and takes l1 top-k indices."""
        _, probs, decs, fused = self.head_predictions(low)
        m = np.asarray(cid_map, dtype=np.int64)
        m = np.where(m == -1, m.max() + 1, m)                  # utils._replacevoids
        assert len(m) != probs["l1_logits"].shape[1], "probability remap branch not restated"
        d = torch.as_tensor(m)[fused]                          # tf.gather(ocids2ncids, decs)
        if replace_voids:
            p1 = probs["l1_logits"]                            # [N, C1, H, W]
            c1 = p1.shape[1]
            # top_k(k=2), stable: equal values keep the lower index first
            order = torch.sort(-p1, dim=1, stable=True).indices
            d = torch.where(d == c1 - 1, order[:, 1], order[:, 0])
        hy = nearest_ac_index(self.cfg.height, out_h)
        wx = nearest_ac_index(self.cfg.width, out_w)
        return d[:, hy][:, :, wx]

    def predict_decisions(self, low, out_h, out_w, replace_voids=False):
        """PREDICT branch (define_estimator_hierarchical.py:203-232): the fused decisions in
        training cids (the cid mapping is commented out, :226-227) and the l1 probabilities go
        through _resize_predictions (:530-575: decisions NEAREST_NEIGHBOR align_corners, l1
        probabilities ResizeBilinear align_corners) and THEN _replace_voids (:577-630) on the
        resized probabilities: void = decision C1 - 1 -> the second of top_k(k=2), else the
        first (the reference's tf.equal "assertion" is not an assert: the first index replaces
        the decision everywhere else). Returns int64 [N, out_h, out_w]."""
        _, probs, _, fused = self.head_predictions(low)
        hy = nearest_ac_index(self.cfg.height, out_h)
        wx = nearest_ac_index(self.cfg.width, out_w)
        d = fused[:, hy][:, :, wx]
        if replace_voids:
            p1 = resize_bilinear_ac(probs["l1_logits"], out_h, out_w)   # [N, C1, Ho, Wo]
            c1 = p1.shape[1]
            order = torch.sort(-p1, dim=1, stable=True).indices
            d = torch.where(d == c1 - 1, order[:, 1], order[:, 0])
        return d

    # -- losses (define_losses_hierarchical.py:98-210) ---------------------------------
    def losses(self, low, px_labels, bbox_soft=None, tag_soft=None, weak_l1_decisions=None):
        """`weak_l1_decisions` (int [Nb_pb + Nb_pi, H, W], optional) replaces this forward's
        l1 argmax in the weak-pixel gate of the l2 weights (:169-177) -- the same weight mask
        as another implementation's run, so that argmax near-ties do not flip pixels in and
        out of the l2 terms when the two are compared; the losses' values and gradients are
        still this forward's."""
        cfg = self.cfg
        t = TABLES[cfg.dataset]
        up, probs, decs, _ = self.head_predictions(low)
        npp = cfg.nb_pp
        lab = torch.as_tensor(px_labels, dtype=torch.long)
        weak = []
        if cfg.nb_pb:
            weak.append(torch.as_tensor(bbox_soft, dtype=self.dtype))
        if cfg.nb_pi:
            weak.append(torch.as_tensor(tag_soft, dtype=self.dtype))

        def seg_sum(soft, table, nseg):
            out = torch.zeros(*soft.shape[:3], nseg, dtype=self.dtype)
            for c, sid in enumerate(table):
                out[..., sid] = out[..., sid] + soft[..., c]
            return out

        # l1: sparse CE on the strong slice, weight = label <= max-1 (:129-140)
        l1lab = _t(t["pp2l1"])[lab]
        l1_logits = up["l1_logits"][:npp]
        onehot_l1 = F.one_hot(l1lab, l1_logits.shape[1]).permute(0, 3, 1, 2).to(self.dtype)
        l1_raw = xent(l1_logits, onehot_l1)
        l1_w = (l1lab <= max(t["pp2l1"]) - 1).to(self.dtype)
        l1_loss, n1 = weighted_loss(l1_raw, l1_w)

        def l2_term(key, pp_table, pb_table, cid_l1):
            nseg = max(pp_table) + 1
            strong = F.one_hot(_t(pp_table)[lab], nseg).to(self.dtype)       # NHWC
            labs = [strong] + [seg_sum(wk, pb_table, nseg) for wk in weak]
            y = torch.cat(labs, 0)
            raw = xent(up[key], y.permute(0, 3, 1, 2))
            w_strong = 1.0 - y[:npp, ..., -1]
            if y.shape[0] > npp:
                yw = y[npp:]
                not_void = (1.0 - yw[..., -1]) > 0.01
                d1w = decs["l1_logits"][npp:] if weak_l1_decisions is None else \
                    torch.as_tensor(weak_l1_decisions, dtype=torch.long)
                l1c = (d1w == cid_l1) & (yw[..., :-1].max(dim=-1).values >= 0.01)
                w = torch.cat([w_strong, (not_void & l1c).to(self.dtype)], 0)
            else:
                w = w_strong
            return weighted_loss(raw, w)

        l2v_loss, n2v = l2_term("l2_vehicle_logits", t["pp2veh"], t["pb2veh"], t["cid_l1_vehicle"])
        l2h_loss, n2h = l2_term("l2_human_logits", t["pp2hum"], t["pb2hum"], t["cid_l1_human"])
        seg = l1_loss + 0.1 * (l2v_loss + l2h_loss)
        reg = sum(cfg.weight_decay * (self.p[f"{s.name}/weights"] ** 2).sum() / 2.0
                  for s in self.specs)
        return {"total": seg + reg, "segmentation": seg, "l1_segmentation": l1_loss,
                "l2_vehicle_segmentation": l2v_loss, "l2_human_segmentation": l2h_loss,
                "regularization": reg, "counts": (n1, n2v, n2h), "decisions": decs}

    # -- one full training step ----------------------------------------------------------
    def train_step(self, images, px_labels, bbox_soft=None, tag_soft=None, lr=0.01,
                   momentum=0.9, mom_state=None, ema_state=None, ema_decay=0.0, step=0,
                   nesterov=False, weak_l1_decisions=None):
        """Forward, losses, autodiff backward of the segmentation loss, SGDM with L2 term
        (MomentumOptimizer, use_nesterov per define_optimizer.py:17-20).

        Returns (losses, grads-of-seg-loss, new params, new momentum, new ema, batch stats).
        `weak_l1_decisions`: see losses().
        """
        trainable = self._trainable()
        low = self.forward(torch.as_tensor(images))
        L = self.losses(low, px_labels, bbox_soft, tag_soft, weak_l1_decisions)
        return (L, low) + self._grads_and_update(L["segmentation"], trainable, lr, momentum,
                                                 mom_state, ema_state, ema_decay, step,
                                                 nesterov)

    def train_step_replicas(self, batches, lr=0.01, momentum=0.9):
        """One data-parallel step of R replicas with cross-replica BN (--cross_replica_norm):
        `batches` = R dicts {images, px, bbox, tag}, each shaped by self.cfg (one replica's
        sub-batch). BN runs over the R concatenated sub-batches (global mean, biased global
        variance); each replica's loss is normalised over its own sub-batch; the gradient is
        that of the replica mean of the losses, i.e. the averaged per-replica gradients of a
        MirroredStrategy step whose statistics all-reduce is differentiated through.
        Returns (per-replica losses, grads, new params, new momentum, batch stats)."""
        self.sync_bn = True
        try:
            trainable = self._trainable()
            imgs = torch.cat([torch.as_tensor(b["images"]) for b in batches], 0)
            low = self.forward(imgs)
            nb = self.cfg.nb
            keys = ("l1_logits", "l2_vehicle_logits", "l2_human_logits")
            Ls = [self.losses({k: low[k][r * nb:(r + 1) * nb] for k in keys}, b["px"],
                              b.get("bbox"), b.get("tag"))
                  for r, b in enumerate(batches)]
            total = sum(L["segmentation"] for L in Ls) / len(Ls)
            g, new_p, new_m, _, stats = self._grads_and_update(total, trainable, lr, momentum,
                                                               None, None, 0.0, 0)
        finally:
            self.sync_bn = False
        return Ls, g, new_p, new_m, stats

    def _trainable(self):
        trainable = {k: v for k, v in self.p.items() if not k.endswith("moving_mean")
                     and not k.endswith("moving_variance")}
        for v in trainable.values():
            v.requires_grad_(True)
        return trainable

    def _grads_and_update(self, loss, trainable, lr, momentum, mom_state, ema_state, ema_decay,
                          step, nesterov=False):
        names = list(trainable)
        grads = torch.autograd.grad(loss, [trainable[n] for n in names], allow_unused=True)
        g = {n: (gr if gr is not None else torch.zeros_like(trainable[n])).detach()
             for n, gr in zip(names, grads)}
        for v in trainable.values():
            v.requires_grad_(False)
        new_p, new_m, new_e = {}, {}, {}
        mom_state = mom_state or {n: torch.zeros_like(self.p[n]) for n in names}
        d = min(ema_decay, (1.0 + step) / (10.0 + step)) if ema_decay > 0 else 0.0
        for n in names:
            w = self.p[n].detach()
            gt = g[n] + (self.cfg.weight_decay * w if n.endswith("/weights") else 0.0)
            v = momentum * mom_state[n] + gt                 # MomentumOptimizer accum
            new_m[n] = v
            # ApplyMomentum: var -= lr * accum, or lr * (g + momentum * accum) with use_nesterov
            new_p[n] = w - lr * (gt + momentum * v) if nesterov else w - lr * v
            if ema_decay > 0:
                s = (ema_state or {}).get(n, w)
                new_e[n] = s - (1.0 - d) * (s - w)
        dec = self.cfg.bn_decay
        for name, (m, v) in self.batch_stats.items():
            mm = self.p[f"{name}/BatchNorm/moving_mean"]
            mv = self.p[f"{name}/BatchNorm/moving_variance"]
            new_p[f"{name}/BatchNorm/moving_mean"] = mm - (1 - dec) * (mm - m)
            new_p[f"{name}/BatchNorm/moving_variance"] = mv - (1 - dec) * (mv - v)
        return g, new_p, new_m, new_e, dict(self.batch_stats)


# ----------------------------------------------------------------------------------------
# metrics (define_metrics.py:5-20; utils/utils.py:385-446)
# ----------------------------------------------------------------------------------------

def confusion_matrix(labels, decisions, num_classes):
    idx = np.asarray(labels).reshape(-1).astype(np.int64) * num_classes + \
        np.asarray(decisions).reshape(-1).astype(np.int64)
    return np.bincount(idx, minlength=num_classes * num_classes).reshape(
        num_classes, num_classes).astype(np.int32)


def mean_iou_train(cm):
    """define_metrics.mean_iou: mean over ALL classes of inter/(union+1e-9) (fp32)."""
    cm = cm.astype(np.float32)
    inter = np.diag(cm)
    union = cm.sum(0) + cm.sum(1) - inter
    return float(np.mean(inter / (union + np.float32(1e-9))))


def eval_metrics(cm):
    """print_metrics_from_confusion_matrix arithmetic (global acc, mean acc, mean IoU)."""
    cm = np.asarray(cm)
    with np.errstate(divide="ignore", invalid="ignore"):
        glob = np.trace(cm) / np.sum(cm) * 100
        acc = np.diagonal(cm) / np.sum(cm, 1) * 100
        inter = np.diagonal(cm)
        union = np.sum(cm, 0) + np.sum(cm, 1) - np.diagonal(cm)
        ious = inter / np.where(union > 0, union, np.ones_like(union)) * 100
    mask = np.logical_not(np.isnan(acc))
    return float(glob), float(np.mean(acc[mask])), float(np.mean(ious[mask])), acc, ious
