"""Drop-in ``define_losses`` (estimator/define_losses_hierarchical.py:14-217).

TRAIN runs the fused HIP loss head (``seg_loss``): align-corners upsampling of the low-res
logits on the fly, l1 sparse softmax-CE on the strong slice, l2 vehicle/human soft CE on
the whole mixed batch with the weak weights gated by the l1 argmax, SUM_BY_NONZERO_WEIGHTS
reductions, ``seg = l1 + 0.1 * (l2v + l2h)``, plus the gradient seed for the backward pass.
EVAL returns zeros like the reference (:26-30).

Returned values are device scalars; ``regularization`` (and therefore ``total``) is
produced by the fused update (it needs the weights of this step, read once there), so it
is valid after the step's train_op has run.
"""
from estimator.mode_keys import ModeKeys
from input_pipelines.weak_labels import BboxLabelsGPU, BoxLists, TagSets


def _weak_maps(ctx):
    if getattr(ctx, '_weak_maps', None) is None:
        ctx._weak_maps = BboxLabelsGPU(ctx.cfg.height, ctx.cfg.width, ctx.device)
    return ctx._weak_maps


class Losses(dict):
    """dict of device scalars; 'total' = segmentation + regularization on access."""

    def __init__(self, ctx):
        losses, reg, _ = ctx.outputs()
        super().__init__(segmentation=losses[0], l1_segmentation=losses[1],
                         l1_segmentation_hot=losses[0] * 0.0,
                         l2_vehicle_segmentation=losses[2], l2_human_segmentation=losses[3],
                         regularization=reg[0])
        self._losses, self._reg = losses, reg

    def __getitem__(self, k):
        if k == 'total':
            return self._losses[0] + self._reg[0]
        return super().__getitem__(k)

    def counts(self):
        return tuple(int(v) for v in self._losses[4:7].tolist())


def define_losses(mode, predictions, labels, config, params):  # pylint: disable=unused-argument
    if mode == ModeKeys.EVAL:
        import torch
        z = torch.zeros(())
        return {'total': z, 'segmentation': z, 'regularization': z}
    if mode != ModeKeys.TRAIN:
        raise NotImplementedError(f"mode {mode} is invalid or not yet implemented.")
    ctx = predictions['_context']
    px = labels.get('prolabels_per_pixel')
    bb = labels.get('prolabels_per_bbox')
    tg = labels.get('prolabels_per_image')
    # weak labels given as box lists / tag sets are rasterised on the device (labels.hip)
    if isinstance(bb, BoxLists):
        bb = _weak_maps(ctx).bbox(bb) if len(bb) else None
    if isinstance(tg, TagSets):
        tg = _weak_maps(ctx).tags(tg) if len(tg) else None
    ctx.loss(px if px is not None and px.numel() else None,
             bb if bb is not None and bb.numel() else None,
             tg if tg is not None and tg.numel() else None,
             predictions.get('decisions'))
    return Losses(ctx)
