"""GPU weak-label maps (seg_bbox_labels / seg_tag_labels) against the host restatement and
the reference's own rasterisation fixtures: bit-exact (integer box geometry, fp32 counts and
one fp32 division per channel on both sides)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "reference_fixtures.npz"))


@pytest.mark.parametrize("case", range(8))
def test_bbox_labels_match_reference_fixture(cuda, case):
    """No resize, no crop: the device map equals the reference's _generate_rla output."""
    from input_pipelines.weak_labels import BboxLabelsGPU
    cids = GOLD[f"bbox{case}_cids"]
    coords = GOLD[f"bbox{case}_coords"]
    keep = cids >= 0
    h, w = (int(v) for v in GOLD[f"bbox{case}_size"])
    out = BboxLabelsGPU(h, w, cuda).bbox([(cids[keep], coords[keep], (h, w), (h, w), (0, 0))])
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out[0].cpu().numpy(), GOLD[f"bbox{case}_rla"])


def _random_image(rng, src, target):
    from input_pipelines.weak_labels import aspect_preserving_size
    k = int(rng.integers(0, 40))
    cids = rng.integers(0, 14, size=k)
    a, b = rng.random((k, 2)).astype(np.float32), rng.random((k, 2)).astype(np.float32)
    coords = np.stack([np.minimum(a[:, 0], b[:, 0]), np.maximum(a[:, 0], b[:, 0]),
                       np.minimum(a[:, 1], b[:, 1]), np.maximum(a[:, 1], b[:, 1])], 1)
    if k:
        coords[0] = (0.0, 1.0, 0.0, 1.0)   # whole image (xmax = w: clipped by the slice)
    if k > 1:
        coords[1] = (0.1, 0.7, 0.3, 0.9)   # float64 products just below an integer (0.7 * 10)
    rs = aspect_preserving_size(src[0], src[1], target[0], target[1])
    off = (int(rng.integers(0, rs[0] - target[0] + 1)), int(rng.integers(0, rs[1] - target[1] + 1)))
    return cids, coords, src, rs, off


@pytest.mark.parametrize("seed", range(4))
def test_bbox_labels_resize_crop_match_host(cuda, seed):
    from input_pipelines.weak_labels import BboxLabelsGPU, bbox_label_map
    rng = np.random.default_rng(seed)
    H, W = 48, 80
    srcs = [(37, 53), (120, 90), (48, 80), (301, 517), (100, 1000)]
    ims = [_random_image(rng, s, (H, W)) for s in srcs]
    ims.append((np.zeros(0, np.int64), np.zeros((0, 4), np.float32), (40, 70), (48, 84), (0, 2)))
    out = BboxLabelsGPU(H, W, cuda).bbox(ims).cpu().numpy()
    for i, (cids, coords, src, rs, off) in enumerate(ims):
        exp = bbox_label_map(cids, coords, src, rs, off, (H, W))
        np.testing.assert_array_equal(out[i], exp)
    assert np.all(np.abs(out.sum(-1) - 1.0) < 1e-3)   # input_subset_bboxes_v2_test.py:40-43
    assert np.all(out[-1][..., 14] == 1.0)             # no boxes: void everywhere


def test_tag_labels_tiled(cuda):
    from input_pipelines.weak_labels import BboxLabelsGPU, generate_tag_rla
    sets = [[3], [], [0, 5, 13]]
    out = BboxLabelsGPU(9, 13, cuda).tags(sets).cpu().numpy()
    for i, s in enumerate(sets):
        np.testing.assert_array_equal(out[i], np.broadcast_to(generate_tag_rla(s), (9, 13, 15)))


def test_bbox_labels_reject_too_many_boxes(cuda):
    from input_pipelines.weak_labels import BboxLabelsGPU
    k = 1025
    with pytest.raises(ValueError):
        BboxLabelsGPU(8, 8, cuda).bbox([(np.zeros(k, np.int64), np.zeros((k, 4), np.float32),
                                         (8, 8), (8, 8), (0, 0))])


def test_loss_with_device_weak_labels_equals_dense(cuda):
    """define_losses with box lists / tag sets (rasterised on the device) gives exactly the
    losses of the same labels rasterised on the host."""
    from estimator.define_losses_hierarchical import define_losses
    from estimator.mode_keys import ModeKeys
    from input_pipelines.synthetic import images, pixel_labels
    from input_pipelines.weak_labels import (BoxLists, TagSets, bbox_label_map, generate_tag_rla,
                                             synthetic_box_lists)
    from models.initializers import init_params
    from seg_hip import SegContext
    H, W = 64, 128
    rng = np.random.default_rng(5)
    ctx = SegContext(pyramid="psp", height=H, width=W, nb_pp=1, nb_pb=2, nb_pi=1, dtype="bf16")
    ctx.load_params(init_params(ctx.param_info, seed=2))
    img = torch.as_tensor(images(rng, 4, H, W)).to(cuda)
    px = torch.as_tensor(pixel_labels(rng, 1, H, W)).to(cuda)
    boxes = synthetic_box_lists(rng, 2, (H, W), src_sizes=((100, 150), (64, 128)))
    tags = TagSets([[1, 4]])
    dense_bb = np.stack([bbox_label_map(c, co, s, r, o, (H, W)) for c, co, s, r, o in boxes])
    dense_tg = np.broadcast_to(generate_tag_rla([1, 4]), (1, H, W, 15)).copy()
    ctx.forward(img)
    ctx.loss(px, torch.as_tensor(dense_bb).to(cuda), torch.as_tensor(dense_tg).to(cuda))
    ref = ctx.outputs()[0].cpu().numpy().copy()
    labels = {"prolabels_per_pixel": px, "prolabels_per_bbox": BoxLists(boxes),
              "prolabels_per_image": tags}
    define_losses(ModeKeys.TRAIN, {"_context": ctx}, labels, None, None)
    got = ctx.outputs()[0].cpu().numpy()
    ctx.close()
    np.testing.assert_array_equal(got, ref)
