"""CPU tests: the oracle against the reference's own golden vectors (tests/golden) and
against known answers of the TF 1.12 semantics it restates."""
import math
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import tfseg
from oracle.tfseg import (CITYSCAPES, OracleNet, SegConfig, build_specs, eval_metrics,
                          init_params, resize_bilinear_ac, resize_tables, resnet_units, same_pads,
                          weighted_loss, xent)

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "reference_fixtures.npz"))


# ---------------------------------------------------------------- reference golden vectors
@pytest.mark.parametrize("case", range(8))
def test_bbox_rasterisation_matches_reference(case):
    from input_pipelines.weak_labels import generate_bbox_rla
    cids = GOLD[f"bbox{case}_cids"]
    coords = GOLD[f"bbox{case}_coords"]
    keep = cids >= 0  # unknown mids are ignored by the reference
    got = generate_bbox_rla(cids[keep], coords[keep], tuple(GOLD[f"bbox{case}_size"]))
    exp = GOLD[f"bbox{case}_rla"]
    np.testing.assert_allclose(got, exp, rtol=0, atol=1e-7)
    # the reference's own assertion (input_subset_bboxes_v2_test.py:40-43)
    assert np.all(np.abs(got.sum(-1) - 1.0) < 1e-3)


@pytest.mark.parametrize("case", range(6))
def test_tag_labels_match_reference(case):
    from input_pipelines.weak_labels import generate_tag_rla
    got = generate_tag_rla(list(GOLD[f"tag{case}_cids"]))
    np.testing.assert_allclose(got, GOLD[f"tag{case}_rla"], atol=1e-7)
    assert abs(got.sum() - 1.0) < 1e-2  # input_subset_image_labels_test.py:41-43


@pytest.mark.parametrize("ds", ["cityscapes", "vistas"])
def test_replacevoids_matches_reference(ds):
    from utils.utils import _replacevoids
    assert _replacevoids(list(GOLD[f"replacevoids_{ds}_in"])) == list(GOLD[f"replacevoids_{ds}_out"])


@pytest.mark.parametrize("case", range(4))
def test_eval_metrics_match_reference(case):
    cm = GOLD[f"cm{case}"]
    glob, macc, miou, _, _ = eval_metrics(cm)
    np.testing.assert_allclose([glob, macc, miou], GOLD[f"cm{case}_metrics"], atol=0.0051)
    from utils.utils import metrics_from_confusion_matrix
    g2, m2, i2, _, _ = metrics_from_confusion_matrix(cm)
    np.testing.assert_allclose([g2, m2, i2], [glob, macc, miou], rtol=1e-12)


# ---------------------------------------------------------------- TF semantics known answers
def test_same_padding_and_maxpool_geometry():
    assert same_pads(512, 3, 2) == (0, 1)      # SAME max-pool: 0 before, 1 after (even size)
    assert same_pads(128, 3, 1, 4) == (4, 4)   # dilated SAME pad = rate
    x = torch.arange(2 * 1 * 6 * 6, dtype=torch.float64).reshape(2, 1, 6, 6)
    y = tfseg.maxpool_same_3x3s2(x)
    assert y.shape == (2, 1, 3, 3)
    assert float(y[0, 0, 0, 0]) == float(x[0, 0, 2, 2])   # window rows/cols 0..2 (no front pad)
    assert float(y[0, 0, 2, 2]) == float(x[0, 0, 5, 5])   # last window clipped by the back pad


def test_resize_align_corners_matches_torch():
    x = torch.randn(2, 5, 7, 9, dtype=torch.float64)
    ours = resize_bilinear_ac(x, 25, 33)
    ref = F.interpolate(x, size=(25, 33), mode="bilinear", align_corners=True)
    assert torch.allclose(ours, ref, atol=1e-5)
    lo, hi, lerp = resize_tables(16, 128)
    assert lo[0] == 0 and lerp[0] == 0 and hi[-1] == 15 and lo[-1] in (14, 15)


def test_xent_known_answers():
    logits = torch.zeros(3, 7, 2, 2, dtype=torch.float64, requires_grad=True)
    y = torch.zeros(3, 7, 2, 2, dtype=torch.float64)
    y[:, 2] = 1.0
    loss = xent(logits, y)
    assert torch.allclose(loss, torch.full_like(loss, math.log(7)))
    loss.sum().backward()
    exp = torch.full_like(logits, 1 / 7) - y           # backprop = softmax - labels
    assert torch.allclose(logits.grad, exp)


def test_weighted_loss_safe_division():
    raw = torch.rand(4, 5, dtype=torch.float64)
    val, n = weighted_loss(raw, torch.zeros_like(raw))
    assert float(val) == 0.0 and n == 0
    w = torch.zeros_like(raw)
    w[0, :2] = 1.0
    val, n = weighted_loss(raw, w)
    assert n == 2 and abs(float(val) - float(raw[0, :2].mean())) < 1e-12


def test_unit_schedule_output_stride_8():
    u = resnet_units(50, 8)
    assert len(u) == 16 and len(resnet_units(101, 8)) == 33
    # block1: stride on its last unit; block2 at rate 1; block3 rate 2; block4 rate 4
    assert [x[4] for x in u[:3]] == [1, 1, 2]
    assert all(x[4] == 1 for x in u[3:])
    assert [x[5] for x in u[3:7]] == [1, 1, 1, 1]
    assert all(x[5] == 2 for x in u[7:13]) and all(x[5] == 4 for x in u[13:])


def test_parameter_counts():
    tot50 = sum(s.co * s.k * s.k * s.ci for s in build_specs(SegConfig(depth=50, pyramid="none")))
    assert abs(tot50 - 26.15e6) < 0.01e6   # SURVEY §2b (encoder + heads)
    tot101 = sum(s.co * s.k * s.k * s.ci for s in build_specs(SegConfig(depth=101, pyramid="none")))
    assert abs(tot101 - 45.09e6) < 0.01e6


def test_all_void_labels_give_zero_l1_loss():
    cfg = SegConfig(height=32, width=32, nb_pp=1, pyramid="none")
    net = OracleNet(cfg, init_params(cfg, seed=1))
    low = net.forward(torch.zeros(1, 32, 32, 3, dtype=torch.float64))
    lab = np.full((1, 32, 32), 19, dtype=np.int64)       # cityscapes void
    L = net.losses(low, lab)
    assert float(L["l1_segmentation"]) == 0.0 and L["counts"][0] == 0
    assert float(L["l2_vehicle_segmentation"]) == 0.0 and L["counts"][1] == 0


def test_weak_weights_follow_l1_decision():
    """A weak pixel contributes to the vehicle loss iff l1 decides 'vehicle' (:233-237)."""
    cfg = SegConfig(height=32, width=32, nb_pp=0, nb_pb=1, pyramid="none")
    net = OracleNet(cfg, init_params(cfg, seed=2))
    low = net.forward(torch.zeros(1, 32, 32, 3, dtype=torch.float64))
    soft = np.zeros((1, 32, 32, 15))
    soft[..., 2] = 1.0                                    # 'car' box everywhere
    L = net.losses(low, np.zeros((0, 32, 32), np.int64), bbox_soft=soft)
    dec = L["decisions"]["l1_logits"].numpy()
    assert L["counts"][1] == int((dec == CITYSCAPES["cid_l1_vehicle"]).sum())
    assert L["counts"][2] == 0                            # car boxes are void for the human head


def test_label_resize_geometry_known_answers():
    """resize_images_or_labels(preserve_aspect_ratio=True, mode='max') sizes and the TF 1.12
    nearest-neighbour source index (utils/utils.py:567-585; align_corners=False)."""
    from input_pipelines.weak_labels import aspect_preserving_size, nearest_index
    assert aspect_preserving_size(1024, 2048, 512, 1024) == (512, 1024)
    assert aspect_preserving_size(375, 500, 512, 1024) == (768, 1024)   # scale = 2.048
    assert aspect_preserving_size(600, 400, 512, 1024) == (1536, 1024)
    np.testing.assert_array_equal(nearest_index(7, 7), np.arange(7))
    np.testing.assert_array_equal(nearest_index(4, 8), [0, 0, 1, 1, 2, 2, 3, 3])
    np.testing.assert_array_equal(nearest_index(5, 3), [0, 1, 3])       # floor(d * 5/3)


def test_bbox_label_map_identity_equals_rasterisation():
    from input_pipelines.weak_labels import bbox_label_map, generate_bbox_rla
    cids = np.array([2, 7])
    coords = np.array([[0.1, 0.6, 0.2, 0.9], [0.5, 1.0, 0.0, 0.4]], np.float32)
    a = bbox_label_map(cids, coords, (20, 30), (20, 30), (0, 0), (20, 30))
    np.testing.assert_array_equal(a, generate_bbox_rla(cids, coords, (20, 30)))


def test_bbox_coordinates_truncate_the_float64_product():
    """The reference's int(coord * size) sees numpy's float64 product of a float32 coordinate
    and an integer size; a float32 product can round up across an integer and move a box
    edge by one pixel."""
    from input_pipelines.weak_labels import generate_bbox_rla
    c = np.float32(0.7)      # c * 10 = 6.99999988 in float64; the float32 product rounds to 7
    assert int(np.float32(c) * np.float32(10)) == 7 and int(float(c) * 10) == 6
    rla = generate_bbox_rla([4], np.array([[0.0, c, 0.0, 1.0]], np.float32), (2, 10))
    assert rla[0, 6, 4] == 1.0 and rla[0, 7, 14] == 1.0


def test_oracle_cross_replica_bn_duplicate_replicas():
    """train_step_replicas over two identical replicas is the single-replica step: the same
    normalisation, the same mean loss and gradient; only the moving-variance input differs
    (biased global variance instead of the fused op's Bessel-corrected one)."""
    import torch
    from input_pipelines.synthetic import batch
    from oracle.tfseg import OracleNet, SegConfig, init_params
    cfg = SegConfig(height=64, width=128, nb_pp=1, nb_pb=1, pyramid="psp")
    params = init_params(cfg, seed=2)
    b = batch(5, 1, 1, 0, 64, 128)
    L, _, g, newp, _, _, stats = OracleNet(cfg, params).train_step(b["images"], b["px"], b["bbox"])
    Ls, g2, newp2, _, stats2 = OracleNet(cfg, params).train_step_replicas([b, b])
    assert abs(float(Ls[0]["segmentation"]) - float(L["segmentation"])) < 1e-10
    for k in g:   # float64 summation order differs (2n-row reductions): relative 1e-7
        assert float((g2[k] - g[k]).norm()) <= 1e-7 * float(g[k].norm()) + 1e-15, k
    for name, (m, v) in stats.items():
        torch.testing.assert_close(stats2[name][0], m, rtol=1e-9, atol=1e-10)
        # biased global variance over 2n samples vs the Bessel-corrected one over n
        assert torch.all(stats2[name][1] <= v + 1e-12)


def test_nearest_align_corners_known_answers():
    """TF 1.12 ResizeNearestNeighbor(align_corners=True): in = min(roundf(o*(in-1)/(out-1)),
    in-1), half away from zero (used by _resize_predictions,
    define_estimator_hierarchical.py:566-570)."""
    from oracle.tfseg import nearest_ac_index
    assert nearest_ac_index(4, 4).tolist() == [0, 1, 2, 3]
    assert nearest_ac_index(5, 3).tolist() == [0, 2, 4]
    assert nearest_ac_index(3, 5).tolist() == [0, 1, 1, 2, 2]     # 0.5 -> 1, 1.5 -> 2
    assert nearest_ac_index(2, 4).tolist() == [0, 0, 1, 1]        # 1/3, 2/3
    assert nearest_ac_index(7, 1).tolist() == [0]


def test_oracle_eval_decisions_map_replace_resize():
    """eval_decisions on hand-built logits: the fused decision, the cid map (with -1 -> void),
    the _replace_voids rule (mapped decision == C1 - 1 -> l1 top-2 index, else l1 top-1) and
    the nearest-neighbour resize."""
    import torch
    from oracle.tfseg import OracleNet, SegConfig, init_params
    cfg = SegConfig(height=16, width=16, nb_pp=1, pyramid="none")
    net = OracleNet(cfg, init_params(cfg, seed=0))
    low = {"l1_logits": torch.zeros(1, 14, 2, 2), "l2_vehicle_logits": torch.zeros(1, 7, 2, 2),
           "l2_human_logits": torch.zeros(1, 3, 2, 2)}
    low["l1_logits"][:, 5] = 4.0           # l1 class 5 -> cid 5 everywhere
    low["l1_logits"][:, 2] = 3.0           # runner-up: 2
    ident = list(range(19)) + [-1]
    d = net.eval_decisions(low, ident, 16, 16)
    assert d.shape == (1, 16, 16) and (d == 5).all()
    m = list(ident)
    m[5] = -1                              # ignored -> void = 19
    assert (net.eval_decisions(low, m, 8, 8) == 19).all()
    m2 = list(ident)
    m2[5] = 13                             # mapped decision == C1 - 1 -> top-2 index
    assert (net.eval_decisions(low, m2, 4, 4, replace_voids=True) == 2).all()
    assert (net.eval_decisions(low, ident, 4, 4, replace_voids=True) == 5).all()
    # vehicle branch: l1 argmax 12 (vehicle) -> l2 vehicle decision through veh_to_common
    low["l1_logits"][:, 12] = 9.0
    low["l2_vehicle_logits"][:, 3] = 1.0
    d = net.eval_decisions(low, ident, 3, 3)
    from oracle.tfseg import CITYSCAPES
    assert (d == CITYSCAPES["veh_to_common"][3]).all()


def test_oracle_predict_decisions_resize_then_replace():
    """predict_decisions (PREDICT order, define_estimator_hierarchical.py:227-231): nearest
    resize of the fused decisions, bilinear align-corners resize of the l1 probabilities, then
    _replace_voids on the resized probabilities. Known answers on hand-built logits, and at the
    network size it equals eval_decisions with the identity map."""
    import torch
    from oracle.tfseg import OracleNet, SegConfig, init_params
    cfg = SegConfig(height=16, width=16, nb_pp=1, pyramid="none")
    net = OracleNet(cfg, init_params(cfg, seed=0))
    low = {"l1_logits": torch.zeros(1, 14, 2, 2), "l2_vehicle_logits": torch.zeros(1, 7, 2, 2),
           "l2_human_logits": torch.zeros(1, 3, 2, 2)}
    from oracle.tfseg import CITYSCAPES
    veh = CITYSCAPES["cid_l1_vehicle"]
    b = list(CITYSCAPES["veh_to_common"]).index(13)   # common cid 13 == C1 - 1 ("void" rule)
    low["l1_logits"][:, veh] = 4.0         # l1 argmax: the vehicle class ...
    low["l1_logits"][:, 2] = 3.0           # ... runner-up 2
    low["l2_vehicle_logits"][:, b] = 1.0   # ... and the vehicle head's class of cid 13
    ident = list(range(20))
    assert (net.predict_decisions(low, 7, 9) == 13).all()
    # void -> second of top-2 of the resized l1 probabilities
    assert (net.predict_decisions(low, 7, 9, replace_voids=True) == 2).all()
    low["l2_vehicle_logits"][:, (b + 1) % 7] = 2.0   # another vehicle class wins
    assert (net.predict_decisions(low, 7, 9) != 13).all()
    # elsewhere the first of top-2 (the l1 argmax index, not the fused decision)
    assert (net.predict_decisions(low, 7, 9, replace_voids=True) == veh).all()
    # left half class 4, right half class 7 at low resolution; the resized probabilities'
    # top-1 follows the bilinear blend of the two softmaxes, columns split at the midpoint
    low["l1_logits"].zero_()
    low["l1_logits"][0, 4, :, 0] = 5.0
    low["l1_logits"][0, 7, :, 1] = 5.0
    d = net.predict_decisions(low, 5, 31, replace_voids=True)[0]
    assert (d[:, :15] == 4).all() and (d[:, 16:] == 7).all()
    g = torch.Generator().manual_seed(0)
    low = {k: torch.randn(2, c, 3, 5, generator=g) for k, c in
           (("l1_logits", 14), ("l2_vehicle_logits", 7), ("l2_human_logits", 3))}
    for rv in (False, True):
        a = net.predict_decisions(low, 16, 16, replace_voids=rv)
        b = net.eval_decisions(low, ident, 16, 16, replace_voids=rv)
        assert torch.equal(a, b)


# ---------------------------------------------------------------- shifted-GEMM conv restatement
@pytest.mark.parametrize("case", [
    # N, H, W, Ci, Co, k, stride, rate, explicit_pad
    (2, 13, 17, 5, 6, 3, 1, 2, False),     # dilated 3x3, ragged
    (1, 11, 9, 7, 4, 1, 1, 1, False),      # 1x1
    (2, 18, 22, 3, 5, 3, 2, 1, True),      # conv2d_same stride 2
    (1, 19, 23, 3, 4, 7, 2, 1, True),      # stem 7x7/2
    (1, 9, 12, 4, 3, 3, 1, 18, False),     # rate larger than the map (ASPP 18 at small size)
    (1, 10, 11, 3, 2, 1, 2, 1, False),     # SAME stride 2 (shortcut-style)
])
def test_conv_props_match_conv_tf_and_autograd(case):
    """oracle/conv_props (the full-size GPU tests' float64 restatement) equals conv_tf and its
    autograd data / weight gradients."""
    from oracle.conv_props import conv_dgrad, conv_fwd, conv_wgrad, geometry
    N, H, W, Ci, Co, k, s, r, ep = case
    spec = tfseg.ConvSpec("t", Ci, Co, k, s, r, explicit_pad=ep)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, H, W, Ci, dtype=torch.float64, generator=g)
    w = torch.randn(Co, k, k, Ci, dtype=torch.float64, generator=g)
    xt = x.permute(0, 3, 1, 2).clone().requires_grad_(True)
    wt = w.clone().requires_grad_(True)
    y = tfseg.conv_tf(xt, wt, spec)
    Ho, Wo = geometry(H, W, spec)[:2]
    assert (Ho, Wo) == tuple(y.shape[2:])
    dy = torch.randn(y.shape, dtype=torch.float64, generator=g)
    y.backward(dy)
    dyn = dy.permute(0, 2, 3, 1).contiguous()
    torch.testing.assert_close(conv_fwd(x, w, spec), y.detach().permute(0, 2, 3, 1), rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(conv_dgrad(dyn, w, spec, H, W), xt.grad.permute(0, 2, 3, 1),
                               rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(conv_wgrad(x, dyn, spec), wt.grad, rtol=1e-12, atol=1e-12)


def test_increase_fov_spec_order_and_validation():
    """extension/increase_fov (resnet50_extended_feature_extractor.py:44-49) follows
    decrease_fdims in variable-creation order, fd -> fd channels, SAME, BN + ReLU; setting only
    one of the two flags is an error (hierarchical.py:272-274)."""
    import argparse
    from oracle.tfseg import build_specs
    from models.resnet50_extended_model_hierarchical import _validate_params
    specs = build_specs(SegConfig(pyramid="psp", fov_k=3, fov_rate=2))
    names = [s.name for s in specs]
    i = names.index("feature_extractor/extension/increase_fov")
    assert names[i - 1] == "feature_extractor/extension/decrease_fdims"
    s = specs[i]
    assert (s.ci, s.co, s.k, s.stride, s.rate, s.relu, s.explicit_pad) == (256, 256, 3, 1, 2, True, False)
    assert "feature_extractor/extension/increase_fov" not in [x.name for x in build_specs(SegConfig())]
    with pytest.raises(ValueError):
        _validate_params(argparse.Namespace(fov_expansion_kernel_size=3, fov_expansion_kernel_rate=0))
    _validate_params(argparse.Namespace(fov_expansion_kernel_size=3, fov_expansion_kernel_rate=2))


def test_hybrid_deconv_matches_tf_conv2d_transpose_definition():
    """The oracle's hybrid upsampler (F.conv_transpose2d on D[in][kh][kw][out]) equals TF's
    conv2d_transpose definition written out: y[p][o] = b[o] + sum_{kh,kw,i}
    x[p + 1 - (kh, kw)][i] * W[kh][kw][o][i] (SAME, stride 1, zero outside the map)."""
    rng = np.random.default_rng(3)
    c, h, w = 5, 6, 7
    x = rng.standard_normal((1, c, h, w))
    W = rng.standard_normal((3, 3, c, c))            # TF filter [kh][kw][out][in]
    b = rng.standard_normal(c)
    D = W.transpose(3, 0, 1, 2)                      # [in][kh][kw][out]
    got = F.conv_transpose2d(torch.tensor(x), torch.tensor(D).permute(0, 3, 1, 2),
                             torch.tensor(b), padding=1).numpy()
    ref = np.tile(b[None, :, None, None], (1, 1, h, w))
    for py in range(h):
        for px in range(w):
            for kh in range(3):
                for kw in range(3):
                    qy, qx = py + 1 - kh, px + 1 - kw
                    if 0 <= qy < h and 0 <= qx < w:
                        ref[0, :, py, px] += W[kh, kw] @ x[0, :, qy, qx]
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-12)
    cfg = SegConfig(height=64, width=128, pyramid="none", upsampling="hybrid")
    p = tfseg.init_params(cfg, seed=1)
    assert p["softmax_classifier/upsampling/Conv2d_transpose_2/weights"].shape == (3, 3, 3, 3)
    assert np.all(p["softmax_classifier/upsampling/Conv2d_transpose/biases"] == 0)
    net = OracleNet(cfg, p)
    low = net.forward(torch.zeros(1, 64, 128, 3, dtype=torch.float64))
    assert low["l1_logits"].shape == (1, 14, 8, 16)


def test_group_norm_restatement_matches_torch_group_norm():
    """The oracle's group norm (tf.contrib.layers.group_norm semantics: per image, moments
    over H x W x C/G, biased variance, epsilon 1e-5) equals torch.nn.functional.group_norm;
    the logits use one group (softmax_classifier arg scope, hierarchical.py:78); no moving
    statistics are created (names under GroupNorm/)."""
    cfg = SegConfig(height=64, width=128, pyramid="none", norm="group")
    p = tfseg.init_params(cfg, seed=2)
    assert not any("moving" in k or "BatchNorm" in k for k in p)
    rng = np.random.default_rng(0)
    for k in p:
        if k.endswith("/gamma") or k.endswith("/beta"):
            p[k] = rng.standard_normal(p[k].shape)
    net = OracleNet(cfg, p)
    x = torch.tensor(rng.standard_normal((2, 256, 8, 16)))
    name = "adaptation_module/l1_features/conv1"
    got = net.conv_bn(x, name, relu=False)
    y = tfseg.conv_tf(x, net.p[name + "/weights"], net.spec_by_name[name])
    ref = F.group_norm(y, 32, net.p[name + "/GroupNorm/gamma"], net.p[name + "/GroupNorm/beta"], eps=1e-5)
    assert torch.allclose(got, ref, rtol=1e-10, atol=1e-10)
    lg = "softmax_classifier/l1_logits"
    got = net.conv_bn(x, lg, relu=False)
    y = tfseg.conv_tf(x, net.p[lg + "/weights"], net.spec_by_name[lg])
    ref = F.group_norm(y, 1, net.p[lg + "/GroupNorm/gamma"], net.p[lg + "/GroupNorm/beta"], eps=1e-5)
    assert torch.allclose(got, ref, rtol=1e-10, atol=1e-10)
