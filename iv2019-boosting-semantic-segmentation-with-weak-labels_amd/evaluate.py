"""Evaluation entry point, drop-in for the reference's code/evaluate.py.

Same command line: ``python evaluate.py <log_dir> <Neval> <training_problem_def_path>
{cityscapes,vistas} [--ckpt_path P | --eval_all_ckpts] [--evaluation_problem_def_path P]
[--replace_voids] [--Nb N]`` plus the model flags. The reference's own ``__main__`` raises
NotImplementedError (evaluate.py:81-83); here ``main`` runs: checkpoints written by train.py
(``<log_dir>/model.ckpt-<step>.pt``) are evaluated on the eval input_fn (seeded synthetic
Cityscapes-shaped batches, or ``--tfrecords_path`` TFRecords of KEYS2FEATURES_v5 examples), the confusion matrices are
accumulated on the device and printed / saved like evaluate.py:56-68 (``all_metrics.txt``;
the raw metrics as ``all_metrics.npz`` instead of a pickle).
"""
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

from estimator.mode_keys import ModeKeys  # noqa: E402
from input_pipelines.synthetic import evaluate_input as eval_fn  # noqa: E402
from models.resnet50_extended_model_hierarchical import add_model_arguments, model as model_fn  # noqa: E402
from system_factory import SemanticSegmentation  # noqa: E402
from utils.utils import SemanticSegmentationArguments, print_metrics_from_confusion_matrix  # noqa: E402


def tfrecord_eval_fn(config, params):
    """evaluate_input over params.tfrecords_path (input_cityscapes.py:190-240): TFRecord ->
    PNG decode on the host, resize / lids2cids (evaluation problem definition) on the device."""
    from input_pipelines.tfrecords import tfrecord_input
    from input_pipelines.utils import get_temp_Nb
    return tfrecord_input(params.tfrecords_path, params.evaluation_problem_def['lids2cids'],
                          params.height_feature_extractor, params.width_feature_extractor,
                          get_temp_Nb(config, params.Nb))


def _add_extra_args(args):
    # evaluate.py:70-79: no regularizer, batch-norm decay irrelevant in inference
    args.regularization_weight = 0.0
    args.batch_norm_decay = 1.0


def main(argv, max_steps=None):
    ssargs = SemanticSegmentationArguments(mode=ModeKeys.EVAL)
    add_model_arguments(ssargs.argparser)
    ssargs.argparser.add_argument('per_pixel_dataset_name', type=str,
                                  choices=['vistas', 'cityscapes'])
    ssargs.argparser.add_argument('--eval_res_dir', type=str, default=None)
    # the reference hard-codes its TFRecord path; without one, seeded synthetic batches
    ssargs.argparser.add_argument('--tfrecords_path', type=str, default=None)
    args = ssargs.parse_args(argv)
    _add_extra_args(args)
    system = SemanticSegmentation({'eval': tfrecord_eval_fn if args.tfrecords_path else eval_fn},
                                  model_fn, args)
    all_metrics = system.evaluate(max_steps=max_steps)
    s = system.settings
    labels = s.evaluation_problem_def['cids2labels']
    if -1 in s.evaluation_problem_def['lids2cids'] and not s.train_void_class:
        labels = labels[:-1]
    res_dir = args.eval_res_dir or os.path.join(args.log_dir, 'eval')
    os.makedirs(res_dir, exist_ok=True)
    with open(os.path.join(res_dir, 'all_metrics.txt'), 'w') as f:
        for m in all_metrics:
            print(f"{m['global_step']:>05} ", end='', file=f)
            print_metrics_from_confusion_matrix(m['confusion_matrix'], labels, printfile=f)
    import numpy as np
    np.savez(os.path.join(res_dir, 'all_metrics.npz'),
             global_step=np.array([m['global_step'] for m in all_metrics]),
             confusion_matrix=np.stack([m['confusion_matrix'] for m in all_metrics]))
    return all_metrics


if __name__ == '__main__':
    main(sys.argv[1:])
