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
Multi-GPU: ``torchrun --nproc-per-node N train.py ... --distribute`` (one process per GPU).
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


def synthetic_train_input(config, params):
    """Endless seeded batches shaped like the heterogeneous-supervision pipeline, per rank."""
    import torch
    from input_pipelines.synthetic import batch
    rank = int(os.environ.get('RANK', 0))
    nb = [get_temp_Nb(config, params.Nb_per_pixel), get_temp_Nb(config, params.Nb_per_bbox),
          get_temp_Nb(config, params.Nb_per_image)]
    dev = torch.device('cuda', torch.cuda.current_device())
    step = 0
    while True:
        b = batch(1000003 * rank + step, *nb, params.height_feature_extractor,
                  params.width_feature_extractor)
        feats = {'proimages': torch.as_tensor(b['images']).to(dev)}
        labels = {'prolabels_per_pixel': torch.as_tensor(b['px']).to(dev),
                  'prolabels_per_bbox': torch.as_tensor(b['bbox']).to(dev) if nb[1] else None,
                  'prolabels_per_image': torch.as_tensor(b['tag']).to(dev) if nb[2] else None}
        yield feats, labels
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


def main(argv):
    ssargs = SemanticSegmentationArguments(mode=ModeKeys.TRAIN)
    add_train_input_pipeline_arguments(ssargs.argparser)
    add_model_arguments(ssargs.argparser)
    settings = ssargs.parse_args(argv)
    _add_extra_args(settings)
    system = SemanticSegmentation({'train': train_input_fn(settings)}, model_fn, settings)
    return system.train(max_steps=settings.max_steps)


if __name__ == '__main__':
    main(sys.argv[1:])
