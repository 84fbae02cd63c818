"""``mean_iou`` of estimator/define_metrics.py:5-20 on the device confusion-matrix kernel:
mean over ALL classes of inter / (union + 1e-9) (training-summary definition)."""
EPSILON = 1E-9


def confusion_matrix(ctx, labels, decisions, num_classes):
    import torch
    cm = torch.zeros((num_classes, num_classes), dtype=torch.int32, device=labels.device)
    ctx.confusion(labels.contiguous().view(-1), decisions.contiguous().view(-1), num_classes, cm)
    return cm


def mean_iou_from_cm(cm):
    cm = cm.float()
    inter = cm.diagonal()
    union = cm.sum(0) + cm.sum(1) - inter
    return (inter / (union + EPSILON)).mean()


def mean_iou(labels, decisions, num_classes, params, ctx=None):
    if ctx is None:
        raise ValueError('mean_iou needs the native context (predictions["_context"])')
    return mean_iou_from_cm(confusion_matrix(ctx, labels, decisions, num_classes))
