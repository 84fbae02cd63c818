"""Drop-in ``define_estimator`` (estimator/define_estimator_hierarchical.py:39-239).

Signature kept: ``define_estimator(mode, features, labels, model_fn, config, params)`` is
bound with ``functools.partial(define_estimator, model_fn=...)`` by the facade exactly as in
system_factory.py:178-187. Instead of a TF graph it runs the step eagerly on the device:

  model_fn forward  ->  define_losses (fused loss head)  ->  train_op():
      backward (HIP)  ->  gradient all-reduce over RCCL when distributed  ->
      fused SGDM + L2 + BN moving averages + EMA (HIP)

The returned ``EstimatorSpec`` holds ``train_op``, a callable that finishes the step.
Gradient semantics follow TF 1.12 MirroredStrategy: every rank normalises its
loss by its own non-zero-weight counts; gradients are averaged across ranks (SUM all-reduce
then 1/N); BN batch statistics (for the moving averages) are averaged the same way. EMA is
disabled when distributed (system_factory.py:236-238).
"""
from __future__ import annotations

from collections import namedtuple

from estimator.define_losses_hierarchical import define_losses
from estimator.define_optimizer import DynamicLossScaler, define_optimizer
from estimator.mode_keys import ModeKeys

EstimatorSpec = namedtuple('EstimatorSpec',
                           ['mode', 'predictions', 'loss', 'train_op', 'losses', 'eval_metric_ops'],
                           defaults=(None,))


class GlobalStep(object):
    def __init__(self, value=0):
        self.value = int(value)


_GLOBAL_STEP = GlobalStep()


def get_or_create_global_step():
    return _GLOBAL_STEP


def world_size():
    import torch.distributed as dist
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def allreduce_grads(ctx, overlap=True, always=False, timing=None):
    """SUM all-reduce of the flat gradient buffer (gradients + BN batch-statistics tail) over
    the process group (RCCL over xGMI on MI355X; gloo on CPU tests). Returns the scale that
    turns the sum into the tower mean (applied inside the fused update).

    On GPU contexts the buffer goes bucket by bucket (ctx.grad_buckets(): conv-weight ranges
    in the order the backward writes them, then the BN tail) on a side stream, each
    collective waiting only for its bucket's event, so the all-reduce of the head and upper
    layers overlaps the backward of the lower ones; the compute stream waits for the side
    stream before the update. `always` runs the collective even in a one-rank group (tests
    of the RCCL path on one GPU); otherwise a single rank skips it.

    `timing` (a list, GPU bucketed path only): appends (backward_done, comm_done) events --
    recorded on the compute stream when its backward has been issued, and on the comm stream
    after the last bucket's collective -- so backward_done.elapsed_time(comm_done), when
    positive, is the all-reduce time the update waits for (exposed, not overlapped)."""
    import torch
    import torch.distributed as dist
    n = world_size()
    if n <= 1 and not (always and dist.is_available() and dist.is_initialized()):
        return 1.0
    buckets = ctx.grad_buckets() if overlap and hasattr(ctx, 'grad_buckets') else None
    if buckets and ctx.grads.is_cuda:
        main = torch.cuda.current_stream(ctx.grads.device)
        comm = getattr(ctx, '_comm_stream', None)
        if comm is None:
            comm = ctx._comm_stream = torch.cuda.Stream(ctx.grads.device)
        if timing is not None:
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record(main)
        for i, (lo, hi) in enumerate(buckets):
            ctx.wait_bucket(i, comm)
            with torch.cuda.stream(comm):
                dist.all_reduce(ctx.grads[lo:hi], op=dist.ReduceOp.SUM)
        if timing is not None:
            ev1.record(comm)
            timing.append((ev0, ev1))
        main.wait_stream(comm)
    elif buckets:
        for lo, hi in buckets:   # host buffers (gloo): the same bucket order, no streams
            dist.all_reduce(ctx.grads[lo:hi], op=dist.ReduceOp.SUM)
    else:
        dist.all_reduce(ctx.grads, op=dist.ReduceOp.SUM)
    return 1.0 / n


def ema_decay_effective(ema_decay, step):
    """tf.train.ExponentialMovingAverage(decay, num_updates=global_step)."""
    if not ema_decay or ema_decay <= 0:
        return 0.0
    return min(ema_decay, (1.0 + step) / (10.0 + step))


def define_estimator(mode, features, labels, model_fn, config, params):
    assert mode in (ModeKeys.TRAIN, ModeKeys.EVAL, ModeKeys.PREDICT)
    assert params.name_feature_extractor in {'resnet_v1_50', 'resnet_v1_101'}
    proimages = features['proimages']
    _, _, predictions = model_fn(mode, proimages, labels, config, params)
    if mode == ModeKeys.EVAL:
        return _eval_spec(predictions, labels, config, params)
    if mode == ModeKeys.PREDICT:
        return _predict_spec(predictions, features, params)
    global_step = get_or_create_global_step()
    ctx = predictions['_context']
    # fp16 storage: dynamic loss scaling (the scale must be set before the loss seeds the
    # backward); bf16 / fp32 need none
    if getattr(ctx, 'dtype', None) == 'fp16' and getattr(ctx, '_scaler', None) is None:
        ctx._scaler = DynamicLossScaler(ctx)
    losses = define_losses(mode, predictions, labels, config, params)
    optimizer = define_optimizer(global_step, params)
    if getattr(ctx, 'nesterov', False) != optimizer.use_nesterov:
        ctx.set_nesterov(optimizer.use_nesterov)
    # one process: nothing reads the gradients between backward and update, so the update of
    # every parameter but the stem's runs beside the stem's weight gradient (seg_set_defer_stem)
    if world_size() <= 1 and getattr(ctx, 'dtype', None) != 'fp16' and hasattr(ctx, 'set_defer_stem'):
        ctx.set_defer_stem(True)

    def train_op():
        ctx.backward()
        scale = allreduce_grads(ctx)
        ema = 0.0 if world_size() > 1 else ema_decay_effective(params.ema_decay, global_step.value)
        ctx.apply_update(optimizer.learning_rate(global_step.value), optimizer.momentum,
                         ema, scale)
        if getattr(ctx, '_scaler', None) is not None:
            ctx._scaler.update()   # an overflowed step was skipped on the device
        global_step.value += 1
        return losses

    return EstimatorSpec(mode, predictions, losses['total'], train_op, losses)


def _eval_spec(predictions, labels, config, params):
    """EVAL branch (define_estimator_hierarchical.py:161-200): zero losses, decisions mapped
    to evaluation cids, optionally void-replaced, nearest-neighbour resized to the label
    size, and the streaming confusion matrix of this batch (labels rows, decisions columns),
    max(tcids2ecids) + 1 classes. All of it runs on the device (seg_predict, seg_confusion)."""
    import torch
    from utils.utils import _replacevoids
    if getattr(params, 'preserve_aspect_ratio', False):
        raise NotImplementedError('evaluation with preserving aspect ratio is not implemented.')
    losses = define_losses(ModeKeys.EVAL, predictions, labels, config, params)
    ctx = predictions['_context']
    prolabels = labels['prolabels']
    tcids2ecids = list(params.training_cids2evaluation_cids)
    decs = torch.empty(prolabels.shape, dtype=torch.int32, device=prolabels.device)
    ctx.predict(tcids2ecids, decs, replace_voids=bool(getattr(params, 'replace_voids', False)))
    nc = max(_replacevoids(tcids2ecids)) + 1
    cm = torch.empty((nc, nc), dtype=torch.int32, device=prolabels.device)
    ctx.confusion(prolabels.to(torch.int32).contiguous(), decs, nc, cm)
    out = predictions.materialised() if hasattr(predictions, 'materialised') else dict(predictions)
    out['decisions'] = decs
    return EstimatorSpec(ModeKeys.EVAL, out, losses['total'], None, losses,
                         {'confusion_matrix': cm})


def _predict_spec(predictions, features, params):
    """PREDICT branch (define_estimator_hierarchical.py:203-238): decisions in TRAINING cids
    (the reference leaves the inference-cid mapping commented out, :226-227), resized to
    (height_system, width_system) when both are set, else to the raw image size, else kept at
    network resolution (_resize_predictions: decisions nearest align-corners, l1 probabilities
    bilinear align-corners); --replace_voids then takes the top-2 of the RESIZED l1
    probabilities (_replace_voids, :530-630), all in one device launch. The full-resolution
    logits / probabilities / per-head decisions stay lazy entries of the model's predictions
    (materialised on first access)."""
    import torch
    ctx = predictions['_context']
    img = features['proimages']
    n, h_net, w_net = img.shape[0], img.shape[1], img.shape[2]
    size = (getattr(params, 'height_system', None), getattr(params, 'width_system', None))
    if not all(size):
        raw = features.get('rawimages')
        size = (int(raw.shape[1]), int(raw.shape[2])) if raw is not None else (h_net, w_net)
    replace = bool(getattr(params, 'replace_voids', False))
    decs = torch.empty((n,) + tuple(size), dtype=torch.int32, device=img.device)
    ctx.predict(list(range(params.output_Nclasses)), decs, replace_voids=replace, order="predict")
    out = predictions
    out['decisions'] = decs
    for k in ('rawimages', 'rawimagespaths'):
        if k in features:
            out[k] = features[k]
    return EstimatorSpec(ModeKeys.PREDICT, out, None, None, None)
