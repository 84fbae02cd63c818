"""Real-data training input (the reference's heterogeneous-supervision train_input), device
preprocessing. Reference: input_pipelines/heterogeneous_supervision/per_pixel_per_bbox_per_image.py
:20-87 zips three streams and concatenates their ``proimages`` on the batch axis (strong first):

* per-pixel (cityscapes / vistas TFRecords, ``input_cityscapes.py:64-188``): shuffle_and_repeat
  over records, PNG decode, convert_image_dtype + bilinear resize to the network size
  (``preserve_aspect_ratio_per_pixel = False``, train.py:66), lids2cids + nearest resize, then
  from_0_1_to_m1_1 -- here: host decode (input_pipelines/tfrecords.py), ``seg_prepare_images``
  / ``seg_prepare_labels`` on the device;
* per-bbox (OpenImages boxes, ``open_images/input_subset_bboxes_v2.py:57-200``): image JPEG,
  box list (mid, (xmin, xmax, ymin, ymax)) -> ``_generate_rla`` at the raw size, aspect-
  preserving resize (mode 'max') + random crop (``input_pipelines/utils.py:181-241``) -- here:
  the image through ``seg_prepare_images_crop`` and the box list as a ``BoxLists`` item that
  ``define_losses`` rasterises on the device (``seg_bbox_labels``) with the same geometry;
* per-image (OpenImages image-level labels, ``input_subset_image_labels.py:57-130``): image
  JPEG + mids -> normalised 15-vector tiled over the image -- ``TagSets``.

Index files. The reference reads ``imageid -> boxes`` / ``imageid -> mids`` pickles at
hard-coded paths; pickles are not loaded here, so the same content comes as JSON:
``{"<imageid>": [["/m/0k4j", [xmin, xmax, ymin, ymax]], ...]}`` for boxes and
``{"<imageid>": ["/m/0k4j", ...]}`` for tags, with the images at ``<images_dir>/<imageid>.jpg``.

Randomness. The reference seeds nothing (shuffle buffers of 2000, tf.random_uniform crop
offsets). Here every stream draws from ``numpy.random.default_rng(seed)`` with the seed derived
from ``--input_seed``, the stream and the rank, so a run is reproducible; the shuffle is
tf.data's buffered shuffle (fill a buffer of ``SHUFFLE_BUFFER`` elements, emit a uniformly
chosen one, refill its slot), repeated per epoch; the weak streams' crop offsets come from a
second generator per stream, so neither order depends on how far decoding runs ahead. Data
parallelism: rank r of N reads the records / images r, r + N, ... (one process per GPU; each
rank batches get_temp_Nb of each sub-batch, as every tower of the reference's
MirroredStrategy does).

Parallelism (the reference's ``map(..., num_parallel_calls=15)`` + ``prefetch(None)``,
input_cityscapes.py:22,125-135,185-186; per_pixel_per_bbox_per_image.py:81-85): the element
selection runs in order on the calling thread, the PNG / JPEG decodes of the next
``--input_prefetch`` batches run on a pool of ``--input_workers`` threads (PIL releases the
GIL while it decodes), and each batch's uploads + device preprocessing are issued when the
training loop takes it.
"""
from __future__ import annotations

import collections
import io
import json
import os
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, Iterator, List, Sequence

import numpy as np

from input_pipelines.weak_labels import BoxLists, TagSets, aspect_preserving_size

SHUFFLE_BUFFER = 2000   # input_cityscapes.py:20, input_subset_bboxes_v2.py:31
NUM_PARALLEL_CALLS = 15  # input_cityscapes.py:22

# mid2cid (input_subset_bboxes_v2.py:38-53, input_subset_image_labels.py:40-56)
MID2CID = {'/m/0199g': 0, '/m/01bjv': 1, '/m/0k4j': 2, '/m/04_sv': 3, '/m/07jdr': 4,
           '/m/07r04': 5, '/m/01g317': 6, '/m/04yx4': 7, '/m/03bt1vf': 8, '/m/01bl7v': 9,
           '/m/05r655': 10, '/m/015qff': 11, '/m/01mqdt': 12, '/m/02pv19': 13}


def shuffled(items: Sequence, rng, buffer: int = SHUFFLE_BUFFER, repeat: bool = True) -> Iterator:
    """tf.data shuffle_and_repeat(buffer) over a finite sequence: per epoch, a buffered
    shuffle (buffer filled in order; each output a uniformly drawn buffer slot, refilled with
    the next element); epochs follow each other without mixing."""
    while True:
        it = iter(items)
        buf = []
        for x in it:
            buf.append(x)
            if len(buf) >= buffer:
                break
        for x in it:
            i = int(rng.integers(len(buf)))
            yield buf[i]
            buf[i] = x
        while buf:
            yield buf.pop(int(rng.integers(len(buf))))
        if not repeat:
            return


def decode_jpeg(b: bytes) -> np.ndarray:
    """tf.image.decode_jpeg(channels=3) on the host (PIL / libjpeg; the IDCT of TF's libjpeg-turbo
    build may differ by a unit in the last place on some pixels: parity unpinned for JPEG)."""
    from PIL import Image
    return np.asarray(Image.open(io.BytesIO(b)).convert('RGB'), dtype=np.uint8)


def _rank_world():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return int(os.environ.get('RANK', 0)), int(os.environ.get('WORLD_SIZE', 1))


def default_workers():
    """Decode threads: the reference's NUM_PARALLEL_CALLS, capped at the usable cores (the
    affinity set, and the cgroup CPU quota where one is set: 16 on the GPU box)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    try:
        q, per = open('/sys/fs/cgroup/cpu.max').read().split()
        if q != 'max':
            n = min(n, max(1, int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return max(1, min(NUM_PARALLEL_CALLS, n))


def _decode_record(rec: bytes):
    from input_pipelines.tfrecords import parse_cityscapes_example
    return parse_cityscapes_example(rec)[:3]


def _decode_jpeg_file(path: str):
    with open(path, 'rb') as f:
        return decode_jpeg(f.read())


class PerPixelStream:
    """Shuffled per-pixel TFRecord examples of this rank: select(n) gives the next n serialized
    records, decode_record one of them -> (image uint8 [h,w,3], label ids uint8 [h,w], path)."""

    def __init__(self, paths, rng, rank=0, world=1):
        from input_pipelines.tfrecords import read_records
        paths = [paths] if isinstance(paths, str) else list(paths)
        recs = [r for p in paths for r in read_records(p)]
        if not recs:
            raise ValueError(f'no records in {paths}')
        self._it = shuffled(recs[rank::world] or recs, rng)

    def select(self, n):
        return [next(self._it) for _ in range(n)]

    decode = staticmethod(_decode_record)

    def take(self, n):
        return [self.decode(r) for r in self.select(n)]


class OpenImagesStream:
    """Shuffled OpenImages entries of this rank from a JSON index (see module docstring):
    select(n) gives (imageid, annotations, image path); take(n) decodes them ->
    (imageid, image uint8 [h,w,3], annotations)."""

    def __init__(self, index_path, images_dir, rng, rank=0, world=1):
        with open(index_path) as f:
            index = json.load(f)
        self.images_dir = images_dir
        keys = sorted(index)
        if not keys:
            raise ValueError(f'empty index {index_path}')
        keys = keys[rank::world] or keys
        self._it = shuffled([(k, index[k]) for k in keys], rng)

    def select(self, n):
        out = []
        for _ in range(n):
            iid, ann = next(self._it)
            out.append((iid, ann, os.path.join(self.images_dir, iid + '.jpg')))
        return out

    decode = staticmethod(_decode_jpeg_file)

    def take(self, n):
        return [(iid, self.decode(path), ann) for iid, ann, path in self.select(n)]


def _weak_geometry(src, H, W, rng):
    """resize_images_and_labels(preserve_aspect_ratio=True): mode 'max' size, then a uniform
    crop offset in [0, extra] per axis (utils.py:206-232)."""
    rs = aspect_preserving_size(src[0], src[1], H, W)
    off = (int(rng.integers(0, rs[0] - H + 1)), int(rng.integers(0, rs[1] - W + 1)))
    return rs, off


def box_item(boxes, src, H, W, rng):
    """One BoxLists item from index boxes [[mid, [xmin, xmax, ymin, ymax]], ...]: unknown mids
    are dropped (the reference's mid2cid lookup covers the subset's classes only)."""
    kept = [(MID2CID[m], c) for m, c in boxes if m in MID2CID]
    cids = np.asarray([k for k, _ in kept], np.int32)
    coords = np.asarray([c for _, c in kept], np.float32).reshape(len(kept), 4)
    rs, off = _weak_geometry(src, H, W, rng)
    return (cids, coords, tuple(src), rs, off)


def heterogeneous_train_input(config, params) -> Callable:
    """input_fn(config, params) of the real-data TRAIN path: yields (features, labels) with
    features['proimages'] = [strong; bbox; tag] fp32 [Nb, H, W, 3] on the device and labels
    {'prolabels_per_pixel': int32 [Nb_pp, H, W], 'prolabels_per_bbox': BoxLists,
    'prolabels_per_image': TagSets}. Decoding runs ahead on a thread pool (module docstring)."""
    import torch
    from input_pipelines.tfrecords import prepare_images, prepare_images_crop, prepare_labels
    from input_pipelines.utils import get_temp_Nb
    rank, world = _rank_world()
    H, W = params.height_feature_extractor, params.width_feature_extractor
    nb = [get_temp_Nb(config, params.Nb_per_pixel), get_temp_Nb(config, params.Nb_per_bbox),
          get_temp_Nb(config, params.Nb_per_image)]
    seed = int(getattr(params, 'input_seed', 0))
    rngs = [np.random.default_rng([seed, s, rank]) for s in range(3)]
    geom = [np.random.default_rng([seed, s, rank, 1]) for s in range(3)]   # crop offsets
    lids2cids = list(params.training_problem_def['lids2cids'])
    pp = PerPixelStream(params.tfrecords_path_per_pixel, rngs[0], rank, world) if nb[0] else None
    if nb[1] and not (params.bboxes_index_path and params.bboxes_images_dir):
        raise ValueError('Nb_per_bbox > 0 needs --bboxes_index_path and --bboxes_images_dir')
    if nb[2] and not (params.image_labels_index_path and params.image_labels_images_dir):
        raise ValueError('Nb_per_image > 0 needs --image_labels_index_path and '
                         '--image_labels_images_dir')
    pb = OpenImagesStream(params.bboxes_index_path, params.bboxes_images_dir, rngs[1], rank,
                          world) if nb[1] else None
    pi = OpenImagesStream(params.image_labels_index_path, params.image_labels_images_dir,
                          rngs[2], rank, world) if nb[2] else None
    dev = torch.device('cuda', torch.cuda.current_device())
    workers = int(getattr(params, 'input_workers', 0) or 0) or default_workers()
    depth = max(1, int(getattr(params, 'input_prefetch', 2) or 1))
    pool = ThreadPoolExecutor(max_workers=workers, thread_name_prefix='seg-decode')

    def to_dev(a):
        return torch.from_numpy(np.require(a, requirements=["C", "W"])[None]).pin_memory().to(dev, non_blocking=True)

    def submit():
        """The next batch: its elements selected in stream order, their decodes queued."""
        job = {}
        if pp is not None:
            job['pp'] = [pool.submit(pp.decode, r) for r in pp.select(nb[0])]
        for stream, kind, n in ((pb, 'bbox', nb[1]), (pi, 'tag', nb[2])):
            if stream is not None:
                job[kind] = [(iid, ann, pool.submit(stream.decode, path))
                             for iid, ann, path in stream.select(n)]
        return job

    pending = collections.deque(submit() for _ in range(depth))
    try:
        while True:
            job = pending.popleft()
            pending.append(submit())            # keep `depth` batches decoding ahead
            ims, px = [], None
            if 'pp' in job:
                ex = [f.result() for f in job['pp']]
                same = len({e[0].shape for e in ex}) == 1
                if same:   # one upload + one launch for the sub-batch
                    raw_i = torch.from_numpy(np.stack([e[0] for e in ex])).pin_memory().to(dev, non_blocking=True)
                    raw_l = torch.from_numpy(np.stack([e[1] for e in ex])).pin_memory().to(dev, non_blocking=True)
                    ims.append(prepare_images(raw_i, H, W))
                    px = prepare_labels(raw_l, H, W, lids2cids)
                else:
                    ims += [prepare_images(to_dev(e[0]), H, W) for e in ex]
                    px = torch.cat([prepare_labels(to_dev(e[1]), H, W, lids2cids) for e in ex])
            boxes, tags = BoxLists(), TagSets()
            for kind in ('bbox', 'tag'):
                if kind not in job:
                    continue
                g = geom[1] if kind == 'bbox' else geom[2]
                for iid, ann, fut in job[kind]:
                    im = fut.result()
                    src = im.shape[:2]
                    if kind == 'bbox':
                        item = box_item(ann, src, H, W, g)
                        boxes.append(item)
                        rs, off = item[3], item[4]
                    else:
                        tags.append([MID2CID[m] for m in ann if m in MID2CID])
                        rs, off = _weak_geometry(src, H, W, g)
                    ims.append(prepare_images_crop(to_dev(im), rs, off, H, W))
            feats = {'proimages': torch.cat(ims) if len(ims) > 1 else ims[0]}
            labels = {'prolabels_per_pixel': px,
                      'prolabels_per_bbox': boxes if nb[1] else None,
                      'prolabels_per_image': tags if nb[2] else None}
            yield feats, labels
    finally:
        pool.shutdown(wait=False, cancel_futures=True)
