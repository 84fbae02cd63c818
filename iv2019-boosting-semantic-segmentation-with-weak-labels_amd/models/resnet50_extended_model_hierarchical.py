"""Drop-in ``model_fn`` of the reference (models/resnet50_extended_model_hierarchical.py).

``model(mode, features, labels, config, params)`` keeps the reference signature and
return value ``(features, end_points, predictions)``. The network itself is not built in
Python: the native context (``seg_hip.SegContext``, one per device per process) holds the
dilated ResNet-50/101 encoder, the PSP pyramid, the three adaptation bottlenecks and the
logits convs, and this function runs its forward pass on the device tensor ``features``
(``proimages``, NHWC fp32 in [-1, 1)).

``predictions`` has the reference's keys (hierarchical.py:121-130): ``l1_logits``,
``l1_probabilities``, ``l1_decisions`` and the same for ``l2_vehicle`` / ``l2_human`` at full
network resolution (NHWC), and ``decisions``. The training step never needs the
full-resolution tensors (the 8x align-corners upsampling of hierarchical.py:84-86, the softmax
and the argmax are fused into the loss head), so they are materialised on first access by one
``seg_full_predictions`` launch and cached; the low-resolution logits the network produces are
under ``*_logits_lowres``. In TRAIN ``decisions`` is the full-resolution fused decision map
filled by the loss head; in EVAL / PREDICT it is produced by ``seg_predict`` (no loss head)
from the logits of a forward whose batch norm uses the moving statistics unless
``batch_norm_accumulate_statistics`` is set (hierarchical.py:306-307).
"""
from __future__ import annotations

from collections.abc import MutableMapping

import numpy as np

from estimator.mode_keys import ModeKeys
from input_pipelines.utils import get_temp_Nb
from models.initializers import init_params

_CONTEXTS = {}


def _validate_params(params):
    # hierarchical.py:272-276
    if bool(getattr(params, 'fov_expansion_kernel_rate', 0)) != bool(
            getattr(params, 'fov_expansion_kernel_size', 0)):
        raise ValueError("One of params.{fov_expansion_kernel_rate, fov_expansion_kernel_size} "
                         "is set. In order to take effect both should be set.")
    if getattr(params, 'upsampling_method', 'bilinear') not in ('bilinear', 'hybrid'):
        # 'no' leaves the logits at H/8 x W/8, which the reference's own losses cannot
        # compare with full-resolution labels
        raise NotImplementedError("upsampling_method must be 'bilinear' (default) or 'hybrid'")
    if getattr(params, 'norm_layer', 'batch') not in ('batch', 'group'):
        raise ValueError('norm_type not valid.')   # module_arg_scope :291-292
    if getattr(params, 'norm_layer', 'batch') == 'group' and getattr(params, 'cross_replica_norm', False):
        # module_arg_scope :329-331
        raise ValueError('cross_replica_norm is supported only for batch normalization for now.')
    if getattr(params, 'stride_feature_extractor', 8) != 8:
        raise NotImplementedError('stride_feature_extractor must be 8')


def sub_batches(config, params, mode=ModeKeys.TRAIN):
    """Per-rank (per-tower) sub-batches: each of the three is split (get_temp_Nb).
    EVAL / PREDICT batches are Nb per-pixel images (evaluate/predict input pipelines)."""
    if mode != ModeKeys.TRAIN:
        return (get_temp_Nb(config, params.Nb), 0, 0)
    return (get_temp_Nb(config, getattr(params, 'Nb_per_pixel', params.Nb)),
            get_temp_Nb(config, getattr(params, 'Nb_per_bbox', 0)),
            get_temp_Nb(config, getattr(params, 'Nb_per_image', 0)))


def get_context(config, params, device=None, mode=ModeKeys.TRAIN):
    """The process's native context for these settings (created on first use)."""
    from seg_hip import SegContext
    import torch
    nb_pp, nb_pb, nb_pi = sub_batches(config, params, mode)
    depth = 101 if getattr(params, 'name_feature_extractor', 'resnet_v1_50') == 'resnet_v1_101' else 50
    pyramid = getattr(params, 'pyramid', None) or (
        'psp' if getattr(params, 'psp_module', False) else
        'aspp' if getattr(params, 'aspp_module', False) else 'none')
    dev = torch.cuda.current_device() if device is None else device
    key = (dev, depth, pyramid, params.height_feature_extractor, params.width_feature_extractor,
           nb_pp, nb_pb, nb_pi, getattr(params, 'compute_dtype', 'fp32'),
           params.per_pixel_dataset_name, bool(getattr(params, 'cross_replica_norm', False)),
           getattr(params, 'ema_decay', 0) > 0,
           getattr(params, 'fov_expansion_kernel_size', 0), getattr(params, 'fov_expansion_kernel_rate', 0),
           getattr(params, 'upsampling_method', 'bilinear'), getattr(params, 'norm_layer', 'batch'))
    ctx = _CONTEXTS.get(key)
    if ctx is None:
        ctx = SegContext(depth=depth, pyramid=pyramid, height=params.height_feature_extractor,
                         width=params.width_feature_extractor, nb_pp=nb_pp, nb_pb=nb_pb,
                         nb_pi=nb_pi, dtype=getattr(params, 'compute_dtype', 'fp32'),
                         dataset=params.per_pixel_dataset_name,
                         feature_dims=getattr(params, 'feature_dims_decreased', 256),
                         bn_decay=getattr(params, 'batch_norm_decay', 0.9),
                         train_bn=getattr(params, 'norm_train_variables', True),
                         weight_decay=getattr(params, 'regularization_weight', 0.00017),
                         ema=getattr(params, 'ema_decay', 0) > 0, device=dev,
                         # extension/increase_fov (resnet50_extended_feature_extractor.py:44-49)
                         fov_k=getattr(params, 'fov_expansion_kernel_size', 0),
                         fov_rate=getattr(params, 'fov_expansion_kernel_rate', 0),
                         # 'hybrid': conv2d_transpose + bias per head (hierarchical.py:168-180)
                         upsampling=getattr(params, 'upsampling_method', 'bilinear'),
                         # norm_layer='group': group_norm(groups=32) after every conv, groups=1
                         # on the logits (hierarchical.py:44-48,78,293-333)
                         norm=getattr(params, 'norm_layer', 'batch'))
        ctx.load_params(init_params(ctx.param_info, seed=getattr(params, 'init_seed', 0)))
        if getattr(params, 'cross_replica_norm', False):
            # hierarchical.py:327-328: BN statistics over all replicas (torch.distributed)
            ctx.set_bn_sync()
        _CONTEXTS[key] = ctx
    return ctx


def release_contexts():
    """Destroy every cached context (device memory back to the allocator); the next
    get_context builds a fresh one from the seeded initialisation."""
    for ctx in _CONTEXTS.values():
        ctx.close()
    _CONTEXTS.clear()


def model(mode, features, labels, config, params):
    """Forward pass (hierarchical.py:17-141). ``features``: device tensor [N, hf, wf, 3]."""
    import torch
    _validate_params(params)
    ctx = get_context(config, params, mode=mode)
    assert features.shape[-1] == 3, 'features must be NHWC with 3 channels'
    # tf.contrib.layers.batch_norm(is_training=batch_norm_accumulate_statistics)
    # (hierarchical.py:40-49,306-307) in every mode: train.py sets the flag (train.py:46); a
    # TRAIN step without it normalises with the moving statistics, differentiates through them
    # as constants and leaves them unchanged (no UPDATE_OPS)
    infer = not bool(getattr(params, 'batch_norm_accumulate_statistics', mode == ModeKeys.TRAIN))
    if getattr(ctx, 'bn_inference', False) != infer:
        ctx.set_bn_inference(infer)
    ctx.forward(features.contiguous())
    return None, {}, Predictions(ctx, params.per_pixel_dataset_name)


HEADS = ('l1', 'l2_vehicle', 'l2_human')
LAZY_KEYS = tuple(f'{h}_{k}' for h in HEADS for k in ('logits', 'probabilities', 'decisions'))


class Predictions(MutableMapping):
    """The model's ``predictions`` (hierarchical.py:121-130) for the last forward of ``ctx``.

    Eager entries: ``decisions`` (int32 [N, H, W]; filled by the loss head in TRAIN),
    ``*_logits_lowres`` (zero-copy views of the network's output, [N, H/8, W/8, c]) and
    ``_context``. The nine full-resolution entries of LAZY_KEYS are produced together by one
    ``seg_full_predictions`` launch on first access (f32 [N, H, W, c] logits and
    probabilities, int32 [N, H, W] decisions); reading them after the context has run another
    forward raises instead of returning the newer forward's values.

    Cost of generic iteration: the key set is the reference's (iteration lists the lazy keys
    too, so ``set(predictions)`` matches the reference dict), which means ``dict(predictions)``,
    ``.items()`` or ``.values()`` materialise the full-resolution outputs — about
    2·N·H·W·(c1+c2+c3)·4 bytes (4.7 GB for Vistas at 1024x2048, N = 4) — on every batch.
    Consumers that need only the decisions read ``predictions['decisions']`` (the PREDICT loop
    of ``SemanticSegmentation.predict`` and ``predict.py`` do), or ``materialised()`` for the
    entries computed so far without a launch."""

    def __init__(self, ctx, dataset='cityscapes'):
        import torch
        self._ctx = ctx
        self._forward_id = getattr(ctx, 'forward_count', 0)
        self._c = (53, 12, 5) if dataset == 'vistas' else (14, 7, 3)
        _, _, logits = ctx.outputs()
        n, h, w = logits.shape[0], ctx.cfg.height, ctx.cfg.width
        self._shape = (n, h, w)
        c1, c2, c3 = self._c
        self._store = {'decisions': torch.zeros((n, h, w), dtype=torch.int32, device=logits.device),
                       'l1_logits_lowres': logits[..., :c1],
                       'l2_vehicle_logits_lowres': logits[..., c1:c1 + c2],
                       'l2_human_logits_lowres': logits[..., c1 + c2:c1 + c2 + c3],
                       '_context': ctx}

    def _materialise(self):
        import torch
        if getattr(self._ctx, 'forward_count', 0) != self._forward_id:
            raise RuntimeError('full-resolution predictions requested after the context ran '
                               'another forward: they are computed from the last forward only')
        n, h, w = self._shape
        ct = sum(self._c)
        dev = self._store['decisions'].device
        logits = torch.empty((n, h, w, ct), dtype=torch.float32, device=dev)
        probs = torch.empty_like(logits)
        hd = torch.empty((n, h, w, 3), dtype=torch.int32, device=dev)
        self._ctx.full_predictions(logits, probs, hd)
        lo = 0
        for i, (head, c) in enumerate(zip(HEADS, self._c)):
            self._store[f'{head}_logits'] = logits[..., lo:lo + c]
            self._store[f'{head}_probabilities'] = probs[..., lo:lo + c]
            self._store[f'{head}_decisions'] = hd[..., i]
            lo += c

    def __getitem__(self, k):
        if k in LAZY_KEYS and k not in self._store:
            self._materialise()
        return self._store[k]

    def __setitem__(self, k, v):
        self._store[k] = v

    def __delitem__(self, k):
        del self._store[k]

    def __iter__(self):
        return iter(list(dict.fromkeys(LAZY_KEYS + tuple(self._store))))

    def __len__(self):
        return len(set(LAZY_KEYS) | set(self._store))

    def materialised(self):
        """The entries computed so far (no launch): a plain dict."""
        return dict(self._store)


def add_model_arguments(argparser):
    """Same flags and defaults as hierarchical.py:228-269."""
    a = argparser.add_argument
    a('--stride_feature_extractor', type=int, default=8)
    a('--name_feature_extractor', type=str, default='resnet_v1_50',
      choices=['resnet_v1_50', 'resnet_v1_101'])
    a('--feature_dims_decreased', type=int, default=256)
    a('--fov_expansion_kernel_size', type=int, default=0)
    a('--fov_expansion_kernel_rate', type=int, default=0)
    a('--upsampling_method', type=str, default='bilinear', choices=['no', 'bilinear', 'hybrid'])
    a('--psp_module', action='store_true')
    a('--norm_layer', type=str, default='batch', choices=['batch', 'group'])
    a('--cross_replica_norm', action='store_true')
    a('--norm_train_variables', action='store_true')
    a('--batch_norm_accumulate_statistics', action='store_true')
    a('--batch_norm_decay', type=float, default=0.9)
    # build-side additions
    # ASPP: the reference's commented-out _create_aspp_module (hierarchical.py:209-226), built
    # in the PSP call site's 'pyramid_module' scope; mutually exclusive with --psp_module
    a('--aspp_module', action='store_true')
    # default: the reference's fp32 arithmetic; bf16 / fp16 (with fp32 master weights) are the
    # MI355X-speed options the benchmark configs name (BASELINE C2-C5)
    a('--compute_dtype', type=str, default='fp32', choices=['bf16', 'fp16', 'fp32'])
    a('--init_seed', type=int, default=0)
