"""Training entry point, drop-in for the reference's code/train.py.

Same command line: ``python train.py <log_dir> {cityscapes,vistas} [flags]`` (plus the model
flags of add_model_arguments and ``--psp_module``). The reference hard-codes its dataset paths
(train.py:17-20, 55-66 and the OpenImages modules); here they are flags:
``--tfrecords_path_per_pixel`` (cityscapes / vistas TFRecords), ``--bboxes_index_path`` +
``--bboxes_images_dir`` and ``--image_labels_index_path`` + ``--image_labels_images_dir``
(OpenImages weak streams, JSON indices: input_pipelines/train_inputs.py). With a per-pixel
TFRecord path the real-data input runs (host decode, device preprocessing and device bbox
rasterisation, input_pipelines/train_inputs.heterogeneous_train_input); without one, the
train input_fn yields seeded synthetic batches in the same input contract
(per_pixel_per_bbox_per_image.py:50-77).
Multi-GPU: ``python train.py ... --distribute`` takes every visible GPU in one launch, as the
reference's MirroredStrategy does (system_factory.py:276-283): without WORLD_SIZE in the
environment, main() starts one rank process per GPU (utils/launch.spawn_ranks; rank 0 keeps the
console log, the settings file and the checkpoints, rank r > 0 logs to <log_dir>/rank<r>.log)
and fails if any rank fails. Under an external launcher (``torchrun --nproc-per-node N``)
WORLD_SIZE is set and the process is one rank. ``SEG_TRAIN_RANKS`` overrides the rank count
and ``SEG_TRAIN_BACKEND=gloo`` lets them share fewer GPUs (tests on one GPU).
"""
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

from estimator.mode_keys import ModeKeys  # noqa: E402
from input_pipelines.utils import get_temp_Nb  # noqa: E402
from models.resnet50_extended_model_hierarchical import add_model_arguments, model as model_fn  # noqa: E402
from system_factory import SemanticSegmentation  # noqa: E402
from utils.utils import SemanticSegmentationArguments  # noqa: E402


def rank_sub_batches(config, params):
    """This rank's share of every sub-batch: get_temp_Nb (input_pipelines/utils.py:118-125)
    applied to the per-pixel, per-bbox and per-image streams separately, as the reference's
    per-tower input does (per_pixel_per_bbox_per_image.py:20-87 under MirroredStrategy)."""
    return [get_temp_Nb(config, params.Nb_per_pixel), get_temp_Nb(config, params.Nb_per_bbox),
            get_temp_Nb(config, params.Nb_per_image)]


def synthetic_seed(rank, step):
    return 1000003 * rank + step


def synthetic_train_input(config, params):
    """Endless seeded batches shaped like the heterogeneous-supervision pipeline, per rank.

    With ``--synthetic_pool`` k > 0 (default 8) the first k batches (seeds synthetic_seed(rank,
    j)) are generated on the host once and stay resident in HBM; later steps cycle through them
    (the same tensors again: nothing downstream writes its input in place). Regenerating every
    step would cost the host ~0.1 GB of images + 126 MB of soft labels per weak image at
    1024 x 2048 plus the H2D copies, far more than the device step. k = 0 generates a fresh
    seeded batch every step (seed synthetic_seed(rank, step))."""
    import torch
    from input_pipelines.synthetic import batch
    rank = int(os.environ.get('RANK', 0))
    nb = rank_sub_batches(config, params)
    dev = torch.device('cuda', torch.cuda.current_device())
    pool_n = int(getattr(params, 'synthetic_pool', 8) or 0)
    if pool_n < 0:
        raise ValueError(f"--synthetic_pool must be >= 0, got {pool_n}")

    def make(step):
        b = batch(synthetic_seed(rank, step), *nb, params.height_feature_extractor,
                  params.width_feature_extractor)
        pin = lambda a: torch.from_numpy(a).pin_memory().to(dev, non_blocking=True)
        return ({'proimages': pin(b['images'])},
                {'prolabels_per_pixel': pin(b['px']),
                 'prolabels_per_bbox': pin(b['bbox']) if nb[1] else None,
                 'prolabels_per_image': pin(b['tag']) if nb[2] else None})
    pool = []
    step = 0
    while True:
        if pool_n == 0:
            yield make(step)
        else:
            if len(pool) < pool_n:
                pool.append(make(step))
            yield pool[step % pool_n]
        step += 1


def add_train_input_pipeline_arguments(argparser):
    argparser.add_argument('--Nb_per_pixel', type=int, default=4)
    argparser.add_argument('--Nb_per_bbox', type=int, default=8)
    argparser.add_argument('--Nb_per_image', type=int, default=4)
    argparser.add_argument('--max_steps', type=int, default=None)
    # dataset locations (hard-coded constants in the reference)
    argparser.add_argument('--tfrecords_path_per_pixel', type=str, nargs='*', default=None)
    argparser.add_argument('--bboxes_index_path', type=str, default=None)
    argparser.add_argument('--bboxes_images_dir', type=str, default=None)
    argparser.add_argument('--image_labels_index_path', type=str, default=None)
    argparser.add_argument('--image_labels_images_dir', type=str, default=None)
    argparser.add_argument('--input_workers', type=int, default=0,
                           help='real-data decode threads (0: NUM_PARALLEL_CALLS = 15, capped '
                                'at the usable cores)')
    argparser.add_argument('--input_prefetch', type=int, default=2,
                           help='real-data batches decoded ahead of the training step')
    argparser.add_argument('--synthetic_pool', type=int, default=8,
                           help='synthetic input: number of seeded batches kept resident in HBM '
                                'and cycled (default 8); 0 = a fresh seeded batch every step')
    argparser.add_argument('--input_seed', type=int, default=0,
                           help='seed of the shuffles and crop offsets (the reference seeds nothing)')


def train_input_fn(settings):
    """The real-data input when a per-pixel TFRecord path is given, else the synthetic one."""
    if settings.tfrecords_path_per_pixel:
        from input_pipelines.train_inputs import heterogeneous_train_input
        return heterogeneous_train_input
    return synthetic_train_input


def _add_extra_args(settings):
    # train.py:42-68 of the reference
    settings.norm_train_variables = True
    settings.batch_norm_accumulate_statistics = True
    if settings.per_pixel_dataset_name == 'vistas':
        settings.Ntrain = 18000
        settings.training_problem_def_path = os.path.join(_HERE, 'problem_definitions/vistas/problem01.json')
    elif settings.per_pixel_dataset_name == 'cityscapes':
        settings.Ntrain = 2975
        settings.training_problem_def_path = os.path.join(_HERE, 'problem_definitions/cityscapes/problem01.json')
    settings.Nb = settings.Nb_per_pixel
    settings.preserve_aspect_ratio_per_pixel = False
    settings.preserve_aspect_ratio_per_bbox = True
    settings.preserve_aspect_ratio_per_image = True


def build_system(argv):
    """train.py's settings and facade, without running it: (system, settings)."""
    ssargs = SemanticSegmentationArguments(mode=ModeKeys.TRAIN)
    add_train_input_pipeline_arguments(ssargs.argparser)
    add_model_arguments(ssargs.argparser)
    settings = ssargs.parse_args(argv)
    _add_extra_args(settings)
    return SemanticSegmentation({'train': train_input_fn(settings)}, model_fn, settings), settings


def launch_distributed(argv, settings):
    """`--distribute` without a launcher: one rank process of this script per visible GPU
    (module docstring). Returns 0 when every rank finished; raises if any failed."""
    from utils.launch import spawn_ranks, visible_gpus
    n = int(os.environ.get('SEG_TRAIN_RANKS', 0)) or visible_gpus()
    if n < 1:
        raise RuntimeError('--distribute: no visible GPU')
    os.makedirs(settings.log_dir, exist_ok=True)
    logs = [None] + [open(os.path.join(settings.log_dir, f'rank{r}.log'), 'w') for r in range(1, n)]
    try:
        rc = spawn_ranks(n, [sys.executable, '-u', os.path.abspath(__file__)] + list(argv),
                         outs=logs, name='train.py --distribute')
    finally:
        for f in logs[1:]:
            f.close()
    if rc != 0:
        raise RuntimeError(f'train.py --distribute: a rank failed (exit {rc}); rank logs in '
                           f'{settings.log_dir}/rank<r>.log')
    return 0


def main(argv):
    """Trains on this process (one rank, or the whole run without --distribute) and returns
    the number of steps run; with --distribute and no launcher it starts the ranks itself and
    returns 0 once all of them finished."""
    system, settings = build_system(argv)
    if settings.distribute and 'WORLD_SIZE' not in os.environ:
        return launch_distributed(argv, settings)
    return system.train(max_steps=settings.max_steps)


if __name__ == '__main__':
    main(sys.argv[1:])
