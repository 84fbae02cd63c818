"""Prediction entry point, drop-in for the reference's code/predict.py.

Same command line: ``python predict.py <log_dir> <training_problem_def_path> <predict_dir>
[--ckpt_path P] [--inference_problem_def_path P] [--replace_voids] [--Nb N]
[--export_lids_images] [--export_color_decisions] [--export_overlapped_color_decisions]
[--results_dir D]`` plus the model flags and the dataset name. Images of ``predict_dir``
(png / jpg / ppm, input_cityscapes.py:248-260) are decoded on the host (PIL, as the reference
does), preprocessed on the device (``seg_prepare_images``: convert_image_dtype, bilinear resize
to the network size, [-1, 1) centring, input_cityscapes.py:262-269), run through the PREDICT
branch, and the decisions (resized to the raw image size) are exported as in
predict.py:112-135: label-id images through ``cids2lids``, colour images through
``cids2colors`` and 50 % overlays. Live matplotlib plotting is not built.
"""
import glob
import json
import os
import sys
import time

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

import numpy as np  # noqa: E402

from estimator.mode_keys import ModeKeys  # noqa: E402
from models.resnet50_extended_model_hierarchical import add_model_arguments, model as model_fn  # noqa: E402
from system_factory import SemanticSegmentation  # noqa: E402
from utils.utils import SemanticSegmentationArguments  # noqa: E402

SUPPORTED_EXTENSIONS = ['png', 'PNG', 'jpg', 'JPG', 'jpeg', 'JPEG', 'ppm', 'PPM']


def predict_dir_input(config, params):
    """predict_input (input_cityscapes.py:248-292): batches of Nb images of predict_dir. The
    reference batches without drop_remainder, so every image is predicted: the context's
    batch is fixed at Nb, so a short last batch is padded with its last image and
    'rawimagespaths' lists only the real ones (the export loop zips over it)."""
    import torch
    from PIL import Image
    from input_pipelines.tfrecords import prepare_images
    from input_pipelines.utils import get_temp_Nb
    nb = get_temp_Nb(config, params.Nb)
    dev = torch.device('cuda', torch.cuda.current_device())
    fnames = []
    for se in SUPPORTED_EXTENSIONS:
        fnames.extend(glob.glob(os.path.join(params.predict_dir, '*.' + se), recursive=True))
    for i in range(0, len(fnames), nb):
        chunk = fnames[i:i + nb]
        padded = chunk + [chunk[-1]] * (nb - len(chunk))
        raws = [np.array(Image.open(f).convert('RGB'), dtype=np.uint8) for f in padded]
        raw = torch.from_numpy(np.stack(raws)).to(dev)
        yield {'proimages': prepare_images(raw, params.height_feature_extractor,
                                           params.width_feature_extractor),
               'rawimages': raw, 'rawimagespaths': chunk}, None


def _add_predict_arguments(argparser):
    a = argparser.add_argument
    a('per_pixel_dataset_name', type=str, choices=['vistas', 'cityscapes'])
    a('--plotting', action='store_true')
    a('--plotting_overlapped', action='store_true')
    a('--plot_l1_confidence', action='store_true')
    a('--plot_l2_confidence', action='store_true')
    a('--timeout', type=float, default=10.0)
    a('--export_color_decisions', action='store_true')
    a('--export_overlapped_color_decisions', action='store_true')
    a('--export_lids_images', action='store_true')
    a('--results_dir', type=str, default=None)


def main(argv, max_steps=None):
    ssargs = SemanticSegmentationArguments(mode=ModeKeys.PREDICT)
    add_model_arguments(ssargs.argparser)
    _add_predict_arguments(ssargs.argparser)
    s = ssargs.parse_args(argv)
    s.regularization_weight = 0.0   # predict.py:168-181
    s.batch_norm_decay = 1.0
    if s.plotting or s.plotting_overlapped:
        raise NotImplementedError('live plotting is not built; use the --export_* flags')
    if s.export_lids_images or s.export_color_decisions or s.export_overlapped_color_decisions:
        assert s.results_dir is not None and os.path.isdir(s.results_dir), (
            'results_dir must a valid path if export_{lids, color}_images flags are True.')
    system = SemanticSegmentation({'predict': predict_dir_input}, model_fn, s)
    st = system.settings
    path = getattr(st, 'inference_problem_def_path', None)
    idef = json.load(open(path)) if path else st.training_problem_def
    idspal = np.array(idef['cids2lids'], dtype=np.uint8) if 'cids2lids' in idef else None
    colpal = np.array(idef['cids2colors'], dtype=np.uint8)
    n, t0 = 0, time.time()
    for out in system.predict(max_steps=max_steps):
        decs = out['decisions'].cpu().numpy()
        raws = out['rawimages'].cpu().numpy()
        for d, raw, p in zip(decs, raws, out['rawimagespaths']):
            root = os.path.splitext(os.path.split(p)[1])[0]
            from PIL import Image
            if s.export_lids_images:
                f = os.path.join(s.results_dir, root + '_result_lids.png')
                assert not os.path.exists(f), f'Output filename ({f}) already exists.'
                Image.fromarray(idspal[d]).save(f)
            if s.export_color_decisions:
                f = os.path.join(s.results_dir, root + '_result_color.png')
                assert not os.path.exists(f), f'Output filename ({f}) already exists.'
                Image.fromarray(colpal[d]).save(f)
            if s.export_overlapped_color_decisions:
                f = os.path.join(s.results_dir, root + '_result_overlapped_color.png')
                assert not os.path.exists(f), f'Output filename ({f}) already exists.'
                Image.fromarray((0.5 * raw + (1 - 0.5) * colpal[d]).astype(np.uint8)).save(f)
            n += 1
    print(f'\nTotal time (input pipeline + network): {time.time() - t0:.3f} s for {n} images')
    return n


if __name__ == '__main__':
    main(sys.argv[1:])
