"""Settings surface and TF-free helpers, drop-in for the reference's ``code/utils/utils.py``.

``SemanticSegmentationArguments`` keeps the reference's flag names, positional arguments
and defaults (utils/utils.py:7-257) so existing command lines parse unchanged. ``mode``
takes the tf.estimator ModeKeys strings ('train', 'eval', 'infer').
"""
from __future__ import annotations

import argparse

import numpy as np

from estimator.mode_keys import ModeKeys


class SemanticSegmentationArguments(object):
    """Collects command-line arguments (reference utils/utils.py:7-30)."""

    def __init__(self, mode=None):
        self._parser = argparse.ArgumentParser()
        self.add_system_arguments()
        self.add_tf_arguments()
        if mode == ModeKeys.PREDICT:
            self.add_inference_arguments()
        elif mode == ModeKeys.TRAIN:
            self.add_train_arguments()
        elif mode == ModeKeys.EVAL:
            self.add_evaluate_arguments()

    @property
    def argparser(self):
        return self._parser

    def parse_args(self, argv):
        self.args = self._parser.parse_args(argv)
        return self.args

    # utils/utils.py:33-47
    def add_system_arguments(self):
        p = self._parser
        p.add_argument('--height_system', type=int, default=None)
        p.add_argument('--width_system', type=int, default=None)
        p.add_argument('--height_feature_extractor', type=int, default=512)
        p.add_argument('--width_feature_extractor', type=int, default=1024)

    # utils/utils.py:49-54 (XLA flag kept for command-line compatibility; no effect here)
    def add_tf_arguments(self):
        self._parser.add_argument('--enable_xla', action='store_true')

    # utils/utils.py:56-119
    def add_train_arguments(self):
        p = self._parser
        p.add_argument('log_dir', type=str)
        p.add_argument('per_pixel_dataset_name', type=str, choices=['cityscapes', 'vistas'])
        p.add_argument('--Ntrain', type=int, default=2975)
        p.add_argument('--init_ckpt_path', type=str, default='')
        p.add_argument('--training_problem_def_path', type=str)
        p.add_argument('--save_checkpoints_steps', type=int, default=None)
        p.add_argument('--save_summaries_steps', type=int, default=120)
        p.add_argument('--train_void_class', action='store_true')
        p.add_argument('--Ne', type=int, default=17)
        p.add_argument('--Nb', type=int, default=4)
        p.add_argument('--learning_rate_schedule', type=str, default='piecewise_constant',
                       choices=['piecewise_constant', 'polynomial_decay'])
        p.add_argument('--learning_rate_initial', type=float, default=0.01)
        p.add_argument('--learning_rate_boundaries', type=int, default=[8, 15, 17], nargs='*')
        g = p.add_mutually_exclusive_group()
        g.add_argument('--learning_rate_decay', type=float)
        g.add_argument('--learning_rate_values', type=float, nargs='*')
        p.add_argument('--learning_rate_decay_steps', type=float, default=0.5)
        p.add_argument('--learning_rate_final', type=float, default=0.5)
        p.add_argument('--learning_rate_power', type=float, default=0.9)
        p.add_argument('--optimizer', type=str, default='SGDM', choices=['SGD', 'SGDM'])
        p.add_argument('--ema_decay', type=float, default=0.9)
        p.add_argument('--regularization_weight', type=float, default=0.00017)
        p.add_argument('--bootstrapping_percentage', type=int, default=-1)
        p.add_argument('--momentum', type=float, default=0.9)
        p.add_argument('--use_nesterov', action='store_true')
        p.add_argument('--distribute', action='store_true')
        # build-side: also write the reference's TF V2 checkpoints (utils/tf_checkpoint.py)
        p.add_argument('--tf_checkpoints', action='store_true')

    # utils/utils.py:121-146
    def add_inference_arguments(self):
        p = self._parser
        p.add_argument('log_dir', type=str, default=None)
        p.add_argument('--ckpt_path', type=str, default=None)
        p.add_argument('training_problem_def_path', type=str)
        p.add_argument('predict_dir', type=str, default=None)
        p.add_argument('--inference_problem_def_path', type=str, default=None)
        p.add_argument('--replace_voids', action='store_true')
        p.add_argument('--Nb', type=int, default=1)
        p.add_argument('--restore_emas', action='store_true')
        p.add_argument('--train_void_class', action='store_true')

    # utils/utils.py:148-170
    def add_evaluate_arguments(self):
        p = self._parser
        p.add_argument('log_dir', type=str, default=None)
        p.add_argument('--eval_all_ckpts', action='store_true')
        p.add_argument('--ckpt_path', type=str, default=None)
        p.add_argument('Neval', type=int)
        p.add_argument('training_problem_def_path', type=str)
        p.add_argument('--evaluation_problem_def_path', type=str, default=None)
        p.add_argument('--replace_voids', action='store_true')
        p.add_argument('--train_void_class', action='store_true')
        p.add_argument('--Nb', type=int, default=1)
        p.add_argument('--restore_emas', action='store_true')


def almost_equal(num1, num2, error=10**-3):
    return abs(num1 - num2) <= error


def _replacevoids(mappings):
    """Replace void (-1) with max id + 1 (utils/utils.py:286-289)."""
    max_m = max(mappings)
    return [m if m != -1 else max_m + 1 for m in mappings]


def safe_div(num, den):
    """numpy form of the reference's safe_div (utils/utils.py:365-383): 0 where den == 0."""
    num = np.asarray(num, dtype=np.float64)
    den = np.asarray(den, dtype=np.float64)
    return np.where(den > 0, num / np.where(den == 0, 1.0, den), 0.0)


def metrics_from_confusion_matrix(cm):
    """Global accuracy, mean accuracy and mean IoU exactly as
    print_metrics_from_confusion_matrix computes them (utils/utils.py:407-425): classes with
    no ground truth are excluded from the means, zero IoUs are kept."""
    cm = np.asarray(cm)
    with np.errstate(divide='ignore', invalid='ignore'):
        global_accuracy = np.trace(cm) / np.sum(cm) * 100
        accuracies = np.diagonal(cm) / np.sum(cm, 1) * 100
        inter = np.diagonal(cm)
        union = np.sum(cm, 0) + np.sum(cm, 1) - np.diagonal(cm)
        ious = inter / np.where(union > 0, union, np.ones_like(union)) * 100
    mask = np.logical_not(np.isnan(accuracies))
    return (float(global_accuracy), float(np.mean(accuracies[mask])), float(np.mean(ious[mask])),
            accuracies, ious)


def print_metrics_from_confusion_matrix(cm, labels=None, printfile=None, printcmd=False,
                                        summary=False):
    """Reporting surface of utils/utils.py:385-446 (same numbers, same text layout)."""
    cm = np.asarray(cm)
    assert cm.dtype == np.int32 and cm.ndim == 2 and cm.shape[0] == cm.shape[1]
    labels = labels or ['unknown'] * cm.shape[0]
    g, ma, mi, acc, ious = metrics_from_confusion_matrix(cm)
    mask = np.logical_not(np.isnan(acc))
    s = f"\nGlobal accuracy: {g:5.2f}\n"
    s += "Per class accuracies (nans due to 0 #Trues) and ious (nans due to 0 #TPs):\n"
    for lab, a, i, m in zip(labels, acc, ious, mask):
        s += f"{lab:<30s}  {a:>5.2f}  {i:>5.2f}  {'' if m else '(ignored in averages)'}\n"
    s += f"Mean accuracy (ignoring nans): {ma:5.2f}\n"
    s += f"Mean iou (ignoring accuracies' nans but including ious' 0s): {mi:5.2f}\n"
    if printcmd:
        print(s)
    if printfile:
        if summary:
            printfile.write(s)
        else:
            print(f"{g:>5.2f}", f"{ma:>5.2f}", f"{mi:>5.2f}", acc, ious, file=printfile)
    return g, ma, mi
