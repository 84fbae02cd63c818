"""Device input preprocessing (csrc/input.hip) against the oracle's
restatement, bit-exact for images and labels (the kernel divides its scales on the host and
keeps FMA contraction off, as TF's CPU resize rounds); and the TFRecord -> PNG -> device batch
path end to end."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

L2C = [-1] * 7 + list(range(19)) + [-1] * 8


@pytest.mark.parametrize("src,dst", [((37, 53), (64, 96)), ((100, 200), (48, 64)),
                                     ((64, 128), (64, 128)), ((1024, 2048), (512, 1024))])
def test_prepare_images_and_labels(cuda, src, dst):
    from input_pipelines.tfrecords import prepare_images, prepare_labels
    from oracle.tfseg import prepare_images_np, prepare_labels_np
    rng = np.random.default_rng(sum(src) + sum(dst))
    raw = rng.integers(0, 256, (2,) + src + (3,), dtype=np.uint8)
    lab = rng.integers(0, 34, (2,) + src, dtype=np.uint8)
    im = prepare_images(torch.from_numpy(raw).to(cuda), *dst).cpu().numpy()
    la = prepare_labels(torch.from_numpy(lab).to(cuda), *dst, L2C).cpu().numpy()
    ref_i = prepare_images_np(raw, *dst)
    np.testing.assert_array_equal(im, ref_i)
    np.testing.assert_array_equal(la, prepare_labels_np(lab, *dst, L2C))


@pytest.mark.parametrize("src,dst", [((80, 120), (64, 128)), ((100, 100), (64, 128)),
                                     ((70, 150), (64, 128)), ((768, 1024), (512, 1024))])
def test_prepare_images_crop(cuda, src, dst):
    """Aspect-preserving resize (mode 'max') + crop window of the weak streams, bit-exact vs
    resizing and slicing on the host (input_pipelines/utils.py:181-241), at several offsets
    including both extremes."""
    from input_pipelines.tfrecords import prepare_images_crop
    from input_pipelines.weak_labels import aspect_preserving_size
    from oracle.tfseg import prepare_images_np
    rng = np.random.default_rng(sum(src))
    raw = rng.integers(0, 256, (1,) + src + (3,), dtype=np.uint8)
    rs = aspect_preserving_size(src[0], src[1], *dst)
    full = prepare_images_np(raw, *rs)
    for off in [(0, 0), (rs[0] - dst[0], rs[1] - dst[1]),
                (int(rng.integers(0, rs[0] - dst[0] + 1)), int(rng.integers(0, rs[1] - dst[1] + 1)))]:
        got = prepare_images_crop(torch.from_numpy(raw).to(cuda), rs, off, *dst).cpu().numpy()
        ref = prepare_images_np(raw, *dst, resized=rs, offset=off)
        np.testing.assert_array_equal(ref, full[:, off[0]:off[0] + dst[0], off[1]:off[1] + dst[1]])
        np.testing.assert_array_equal(got, ref)
    with pytest.raises(RuntimeError, match="outside"):
        prepare_images_crop(torch.from_numpy(raw).to(cuda), rs, (rs[0] - dst[0] + 1, 0), *dst)


def test_prepare_labels_out_of_table_ids(cuda):
    from input_pipelines.tfrecords import prepare_labels
    lab = torch.tensor([[[0, 40], [33, 255]]], dtype=torch.uint8, device=cuda)
    out = prepare_labels(lab, 2, 2, L2C).cpu().numpy()
    assert out.tolist() == [[[19, -1], [19, -1]]]


def test_tfrecord_input_end_to_end(cuda, tmp_path):
    from input_pipelines.tfrecords import (encode_example, encode_png, tfrecord_input,
                                           write_records)
    from oracle.tfseg import prepare_images_np, prepare_labels_np
    rng = np.random.default_rng(7)
    ims = rng.integers(0, 256, (4, 40, 80, 3), dtype=np.uint8)
    las = rng.integers(0, 34, (4, 40, 80), dtype=np.uint8)
    recs = [encode_example({"image/encoded": [encode_png(ims[i])],
                            "label/encoded": [encode_png(las[i])],
                            "image/path": [f"im{i}.png".encode()],
                            "label/path": [f"la{i}.png".encode()]}) for i in range(4)]
    p = str(tmp_path / "eval.tfrecord")
    write_records(p, recs)
    batches = list(tfrecord_input(p, L2C, 32, 64, nb=2))
    assert len(batches) == 2
    for b, (f, l) in enumerate(batches):
        ref_i = prepare_images_np(ims[2 * b:2 * b + 2], 32, 64)
        np.testing.assert_array_equal(f["proimages"].cpu().numpy(), ref_i)
        np.testing.assert_array_equal(l["prolabels"].cpu().numpy(),
                                      prepare_labels_np(las[2 * b:2 * b + 2], 32, 64, L2C))
        assert f["rawimagespaths"] == [f"im{2 * b}.png".encode(), f"im{2 * b + 1}.png".encode()]


def test_evaluate_from_tfrecords(cuda, tmp_path, init_ckpt):
    """evaluate.py --tfrecords_path: the confusion matrix of the TFRecord batches equals the
    one built from the oracle-preprocessed labels and the native decisions."""
    import importlib.util
    import os
    from input_pipelines.tfrecords import encode_example, encode_png, write_records
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pkg = os.path.join(repo, "iv2019-boosting-semantic-segmentation-with-weak-labels_amd")
    rng = np.random.default_rng(9)
    ims = rng.integers(0, 256, (2, 60, 100, 3), dtype=np.uint8)
    las = rng.integers(0, 34, (2, 60, 100), dtype=np.uint8)
    recs = [encode_example({"image/encoded": [encode_png(ims[i])],
                            "label/encoded": [encode_png(las[i])]}) for i in range(2)]
    p = str(tmp_path / "val.tfrecord")
    write_records(p, recs)
    init_ckpt(tmp_path, pyramid="none", height=48, width=64, nb_pp=1, dtype="fp32")
    spec = importlib.util.spec_from_file_location("seg_eval_tfr", os.path.join(pkg, "evaluate.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    res = mod.main([str(tmp_path), "2", os.path.join(pkg, "problem_definitions", "cityscapes",
                                                      "problem01.json"),
                    "cityscapes", "--Nb", "1", "--height_feature_extractor", "48",
                    "--width_feature_extractor", "64", "--compute_dtype", "fp32",
                    "--tfrecords_path", p])
    cm = res[0]["confusion_matrix"]
    assert cm.shape == (19, 19) and 0 < int(cm.sum()) <= 2 * 48 * 64
