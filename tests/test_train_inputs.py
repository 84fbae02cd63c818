"""Host side of the real-data TRAIN input (input_pipelines/train_inputs.py) on the committed
tiny training set (tests/golden/tiny_train, made by make_tiny_train.py): tf.data's buffered
shuffle_and_repeat, the per-pixel TFRecord stream, the OpenImages-style box / tag indices and
the mid2cid map, and the aspect-preserving resize + crop geometry of the weak streams."""
import os
from types import SimpleNamespace

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
TINY = os.path.join(HERE, "golden", "tiny_train")


def test_shuffle_is_a_permutation_per_epoch_and_seeded():
    from input_pipelines.train_inputs import shuffled
    items = list(range(37))
    for buf in (1, 5, 37, 100):
        it = shuffled(items, np.random.default_rng(3), buffer=buf)
        ep = [[next(it) for _ in items] for _ in range(3)]
        for e in ep:
            assert sorted(e) == items
        it2 = shuffled(items, np.random.default_rng(3), buffer=buf)
        assert [next(it2) for _ in items] == ep[0]
    # buffer 1 keeps the order (tf.data: shuffle(1) is the identity)
    it = shuffled(items, np.random.default_rng(0), buffer=1)
    assert [next(it) for _ in items] == items
    # a small buffer only moves elements a bounded distance forward
    it = shuffled(items, np.random.default_rng(0), buffer=4)
    out = [next(it) for _ in items]
    assert all(out.index(x) >= x - 3 for x in items[:30])
    assert list(shuffled(items, np.random.default_rng(1), buffer=8, repeat=False)).__len__() == 37


def test_per_pixel_stream_reads_tfrecords():
    from input_pipelines.train_inputs import PerPixelStream
    path = os.path.join(TINY, "cityscapes.tfrecord")
    s = PerPixelStream(path, np.random.default_rng(0))
    ex = s.take(8)   # two epochs of 4 records
    paths = [e[2] for e in ex]
    assert sorted(paths[:4]) == sorted(paths[4:]) == [f"img_{i}.png".encode() for i in range(4)]
    for im, la, _ in ex:
        assert im.shape == (96, 192, 3) and im.dtype == np.uint8
        assert la.shape == (96, 192) and la.max() < 34
    # data parallel: rank r of N reads records r, r + N, ...
    r1 = PerPixelStream(path, np.random.default_rng(0), rank=1, world=2)
    assert sorted({e[2] for e in r1.take(6)}) == [b"img_1.png", b"img_3.png"]


def test_openimages_streams_and_box_items():
    import json
    from input_pipelines.train_inputs import MID2CID, OpenImagesStream, box_item
    from input_pipelines.weak_labels import aspect_preserving_size
    idx = os.path.join(TINY, "bboxes.json")
    raw = json.load(open(idx))
    s = OpenImagesStream(idx, os.path.join(TINY, "images"), np.random.default_rng(0))
    got = s.take(4)
    assert sorted(g[0] for g in got) == sorted(raw)
    rng = np.random.default_rng(5)
    for iid, im, ann in got:
        assert im.dtype == np.uint8 and im.ndim == 3 and im.shape[2] == 3
        cids, coords, src, rs, off = box_item(ann, im.shape[:2], 64, 128, rng)
        known = [a for a in ann if a[0] in MID2CID]
        assert list(cids) == [MID2CID[a[0]] for a in known]
        assert coords.shape == (len(known), 4)
        assert rs == aspect_preserving_size(src[0], src[1], 64, 128)
        assert rs[0] >= 64 and rs[1] >= 128 and (rs[0] == 64 or rs[1] == 128 or
                                                  abs(rs[0] / rs[1] - src[0] / src[1]) < 0.05)
        assert 0 <= off[0] <= rs[0] - 64 and 0 <= off[1] <= rs[1] - 128


def test_real_data_input_requires_weak_indices():
    from input_pipelines.train_inputs import heterogeneous_train_input

    class Cfg:
        class train_distribute:
            num_towers = 1
    p = SimpleNamespace(height_feature_extractor=64, width_feature_extractor=128, Nb_per_pixel=1,
                        Nb_per_bbox=1, Nb_per_image=0, input_seed=0,
                        training_problem_def={"lids2cids": list(range(34))},
                        tfrecords_path_per_pixel=[os.path.join(TINY, "cityscapes.tfrecord")],
                        bboxes_index_path=None, bboxes_images_dir=None,
                        image_labels_index_path=None, image_labels_images_dir=None)
    with pytest.raises(ValueError, match="bboxes_index_path"):
        next(heterogeneous_train_input(Cfg, p))


def test_train_cli_flags():
    import train
    from estimator.mode_keys import ModeKeys
    from utils.utils import SemanticSegmentationArguments
    a = SemanticSegmentationArguments(mode=ModeKeys.TRAIN)
    train.add_train_input_pipeline_arguments(a.argparser)
    s = a.parse_args(["logs", "cityscapes", "--tfrecords_path_per_pixel", "a.tfrecord",
                      "b.tfrecord", "--bboxes_index_path", "i.json", "--input_seed", "3"])
    assert s.tfrecords_path_per_pixel == ["a.tfrecord", "b.tfrecord"] and s.input_seed == 3
    assert train.train_input_fn(s).__name__ == "heterogeneous_train_input"
    s = a.parse_args(["logs", "cityscapes"])
    assert train.train_input_fn(s) is train.synthetic_train_input


def test_oracle_crop_resize_is_resize_then_slice():
    from oracle.tfseg import prepare_images_np
    raw = np.random.default_rng(2).integers(0, 256, (1, 70, 150, 3), dtype=np.uint8)
    full = prepare_images_np(raw, 64, 138)
    for off in [(0, 0), (0, 10), (0, 5)]:
        np.testing.assert_array_equal(
            prepare_images_np(raw, 64, 128, resized=(64, 138), offset=off),
            full[:, off[0]:off[0] + 64, off[1]:off[1] + 128])
