"""EVAL / PREDICT path through the C ABI against the oracle.

* moving-statistics batch norm (is_training = batch_norm_accumulate_statistics = False,
  models/resnet50_extended_model_hierarchical.py:40-49,306-307): low-res logits of an
  inference-mode forward vs the oracle's, 1e-3 relative (or 4x the fp32 oracle's own gap);
  the moving statistics are the oracle's batch statistics of another batch, so activations
  stay in the range real checkpoints give;
* seg_predict (define_estimator_hierarchical.py:161-232): decisions mapped to evaluation cids,
  optionally void-replaced, nearest-neighbour resized to the label size. The oracle is fed the
  NATIVE low-res logits so the decision logic is checked by itself: equal up to fp32 near-ties
  of the softmax argmax (at most 0.1 % of the pixels; 0 expected);
* the streaming confusion matrix of the EVAL spec, and SemanticSegmentation.evaluate /
  .predict end to end on synthetic input.
"""
import os

import numpy as np
import pytest
import torch

from oracle.tfseg import OracleNet, SegConfig, confusion_matrix, init_params

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBLEM = os.path.join(REPO, "iv2019-boosting-semantic-segmentation-with-weak-labels_amd",
                       "problem_definitions", "cityscapes", "problem01.json")


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _params_with_moving_stats(cfg, seed=3):
    """init_params + moving statistics = the oracle's batch statistics of another batch."""
    from input_pipelines.synthetic import batch
    params = init_params(cfg, seed=seed)
    other = batch(99, cfg.nb, 0, 0, cfg.height, cfg.width)
    net = OracleNet(cfg, params, dtype=torch.float64)
    net.forward(torch.as_tensor(other["images"]))
    for name, (m, v) in net.batch_stats.items():
        params[f"{name}/BatchNorm/moving_mean"] = m.numpy()
        params[f"{name}/BatchNorm/moving_variance"] = v.numpy()
    # non-trivial affine parameters too
    rng = np.random.default_rng(5)
    for k in params:
        if k.endswith("/gamma"):
            params[k] = 1.0 + 0.1 * rng.standard_normal(params[k].shape)
        elif k.endswith("/beta"):
            params[k] = 0.1 * rng.standard_normal(params[k].shape)
    return {k: np.asarray(v, np.float32) for k, v in params.items()}


def _ctx(cfg, dtype="fp32"):
    from seg_hip import SegContext
    return SegContext(depth=cfg.depth, pyramid=cfg.pyramid, height=cfg.height, width=cfg.width,
                      nb_pp=cfg.nb_pp, nb_pb=cfg.nb_pb, nb_pi=cfg.nb_pi, dtype=dtype)


CFGS = [SegConfig(height=64, width=128, nb_pp=2, pyramid="psp"),
        SegConfig(height=48, width=64, nb_pp=1, pyramid="aspp")]


@pytest.mark.parametrize("cfg", CFGS, ids=lambda c: f"{c.height}x{c.width}-{c.pyramid}")
def test_inference_bn_forward_fp32(cuda, cfg):
    from input_pipelines.synthetic import batch
    params = _params_with_moving_stats(cfg)
    data = batch(11, cfg.nb, 0, 0, cfg.height, cfg.width)
    ctx = _ctx(cfg)
    ctx.load_params(params)
    ctx.set_bn_inference(True)
    ctx.forward(torch.as_tensor(data["images"]).to(cuda))
    _, _, lg = ctx.outputs()
    lg = lg.cpu().numpy().copy()
    outs = {}
    for dt in (torch.float64, torch.float32):
        net = OracleNet(cfg, params, dtype=dt)
        net.bn_inference = True
        outs[dt] = {k: v.detach() for k, v in net.forward(torch.as_tensor(data["images"])).items()}
    c1, c2, c3 = 14, 7, 3
    for key, a, b in (("l1_logits", 0, c1), ("l2_vehicle_logits", c1, c1 + c2),
                      ("l2_human_logits", c1 + c2, c1 + c2 + c3)):
        ref = outs[torch.float64][key].permute(0, 2, 3, 1).numpy()
        gap = _rel(outs[torch.float32][key].permute(0, 2, 3, 1).numpy(), ref)
        assert _rel(lg[..., a:b], ref) < max(1e-3, 4 * gap), (key, gap)
    # the training-mode forward of the same context differs (batch statistics)
    ctx.set_bn_inference(False)
    ctx.forward(torch.as_tensor(data["images"]).to(cuda))
    _, _, lg_train = ctx.outputs()
    assert _rel(lg_train.cpu().numpy()[..., :c1], lg[..., :c1]) > 1e-2
    ctx.close()


MAPS = {
    "identity": list(range(19)) + [-1],
    # merge some classes, ignore others (-1 -> void = max + 1)
    "merge": [0, 0, 1, 1, 2, -1, 3, 3, 4, 5, 6, 7, 7, 8, 8, 8, 9, 9, 9, -1],
}


@pytest.mark.parametrize("replace_voids", [False, True])
@pytest.mark.parametrize("out_hw", [(64, 128), (32, 64), (128, 256), (45, 77)])
@pytest.mark.parametrize("mapname", sorted(MAPS))
def test_predict_decisions(cuda, mapname, out_hw, replace_voids):
    from input_pipelines.synthetic import batch
    cfg = CFGS[0]
    params = _params_with_moving_stats(cfg)
    data = batch(12, cfg.nb, 0, 0, cfg.height, cfg.width)
    ctx = _ctx(cfg)
    ctx.load_params(params)
    ctx.set_bn_inference(True)
    ctx.forward(torch.as_tensor(data["images"]).to(cuda))
    _, _, lg = ctx.outputs()
    out = torch.full((cfg.nb,) + out_hw, -7, dtype=torch.int32, device=cuda)
    ctx.predict(MAPS[mapname], out, replace_voids=replace_voids)
    nat = out.cpu().numpy()
    low = lg.cpu().permute(0, 3, 1, 2).contiguous()
    c1, c2 = 14, 7
    net = OracleNet(cfg, params, dtype=torch.float32)
    lowd = {"l1_logits": low[:, :c1], "l2_vehicle_logits": low[:, c1:c1 + c2],
            "l2_human_logits": low[:, c1 + c2:c1 + c2 + 3]}
    ref = net.eval_decisions(lowd, MAPS[mapname], out_hw[0], out_hw[1],
                             replace_voids=replace_voids).numpy()
    assert nat.shape == ref.shape and (nat >= 0).all()
    mism = float(np.mean(nat != ref))
    assert mism <= 1e-3, mism
    ctx.close()


@pytest.mark.parametrize("out_hw", [(64, 128), (32, 64), (128, 256), (45, 77), (97, 301)])
def test_predict_order_resize_then_replace_voids(cuda, out_hw):
    """the PREDICT branch resizes first -- decisions nearest, l1
    probabilities bilinear (align_corners) -- and replaces voids on the RESIZED probabilities
    (define_estimator_hierarchical.py:227-231, :530-630), against
    OracleNet.predict_decisions on the native low-res logits. At the network size it equals
    the EVAL order (same launch, mode 1). Only fp32-vs-fp32 rounding near-ties of the top-2
    may differ (<= 1e-3 of the pixels)."""
    from input_pipelines.synthetic import batch
    cfg = CFGS[0]
    params = _params_with_moving_stats(cfg)
    data = batch(12, cfg.nb, 0, 0, cfg.height, cfg.width)
    ctx = _ctx(cfg)
    ctx.load_params(params)
    ctx.set_bn_inference(True)
    ctx.forward(torch.as_tensor(data["images"]).to(cuda))
    _, _, lg = ctx.outputs()
    low = lg.cpu().permute(0, 3, 1, 2).contiguous()
    c1, c2 = 14, 7
    net = OracleNet(cfg, params, dtype=torch.float32)
    lowd = {"l1_logits": low[:, :c1], "l2_vehicle_logits": low[:, c1:c1 + c2],
            "l2_human_logits": low[:, c1 + c2:c1 + c2 + 3]}
    ident = list(range(20))   # PREDICT keeps training cids
    got = {}
    for rv in (False, True):
        out = torch.full((cfg.nb,) + out_hw, -7, dtype=torch.int32, device=cuda)
        ctx.predict(ident, out, replace_voids=rv, order="predict")
        nat = out.cpu().numpy()
        ref = net.predict_decisions(lowd, out_hw[0], out_hw[1], replace_voids=rv).numpy()
        assert nat.shape == ref.shape and (nat >= 0).all()
        assert float(np.mean(nat != ref)) <= 1e-3, (rv, float(np.mean(nat != ref)))
        got[rv] = nat
    if out_hw == (cfg.height, cfg.width):
        out = torch.empty((cfg.nb,) + out_hw, dtype=torch.int32, device=cuda)
        ctx.predict(ident, out, replace_voids=True, order="eval")
        np.testing.assert_array_equal(out.cpu().numpy(), got[True])
    ctx.close()


def test_predict_spec_replace_voids_resized(cuda, tmp_path, init_ckpt):
    """define_estimator(PREDICT) with --replace_voids and a system size different from the
    network size (was NotImplementedError in round 4): the facade's decisions equal
    OracleNet.predict_decisions on the same forward's logits."""
    from estimator.define_estimator_hierarchical import define_estimator
    from estimator.mode_keys import ModeKeys
    from models.resnet50_extended_model_hierarchical import add_model_arguments, model
    from system_factory import RunConfig
    from utils.utils import SemanticSegmentationArguments
    from input_pipelines.synthetic import batch
    a = SemanticSegmentationArguments(mode=ModeKeys.PREDICT)
    add_model_arguments(a.argparser)
    s = a.parse_args([str(tmp_path), PROBLEM, str(tmp_path / "pred"), "--Nb", "1",
                      "--height_feature_extractor", "48", "--width_feature_extractor", "64",
                      "--compute_dtype", "fp32", "--replace_voids"])
    s.per_pixel_dataset_name = "cityscapes"
    from input_pipelines.synthetic import predict_input
    from system_factory import SemanticSegmentation
    s = SemanticSegmentation({"predict": predict_input}, model, s).settings   # output_Nclasses etc.
    s.height_system, s.width_system = 100, 150
    params = init_ckpt(tmp_path, pyramid="none", height=48, width=64, nb_pp=1, dtype="fp32")
    data = batch(5, 1, 0, 0, 48, 64)
    feats = {"proimages": torch.as_tensor(data["images"]).to(cuda)}
    spec = define_estimator(ModeKeys.PREDICT, feats, None, model, RunConfig(), s)
    d = spec.predictions["decisions"].cpu().numpy()
    assert d.shape == (1, 100, 150)
    ctx = spec.predictions["_context"]
    _, _, lg = ctx.outputs()
    low = lg.cpu().permute(0, 3, 1, 2).contiguous()
    cfg = SegConfig(height=48, width=64, nb_pp=1, pyramid="none")
    net = OracleNet(cfg, {k: v.numpy() for k, v in params.items()}, dtype=torch.float32)
    lowd = {"l1_logits": low[:, :14], "l2_vehicle_logits": low[:, 14:21],
            "l2_human_logits": low[:, 21:24]}
    ref = net.predict_decisions(lowd, 100, 150, replace_voids=True).numpy()
    assert float(np.mean(d != ref)) <= 1e-3


def test_predict_rejects_bad_map(cuda):
    cfg = CFGS[0]
    ctx = _ctx(cfg)
    out = torch.zeros((cfg.nb, 8, 8), dtype=torch.int32, device=cuda)
    with pytest.raises(RuntimeError):
        ctx.predict(list(range(10)), out)
    with pytest.raises(ValueError):
        ctx.predict(MAPS["identity"], torch.zeros((cfg.nb + 1, 8, 8), dtype=torch.int32,
                                                  device=cuda))
    ctx.close()


def _eval_settings(tmp_path, nb=2, h=64, w=128, neval=4):
    from models.resnet50_extended_model_hierarchical import add_model_arguments
    from utils.utils import SemanticSegmentationArguments
    from estimator.mode_keys import ModeKeys
    a = SemanticSegmentationArguments(mode=ModeKeys.EVAL)
    add_model_arguments(a.argparser)
    s = a.parse_args([str(tmp_path), str(neval), PROBLEM, "--Nb", str(nb), "--psp_module",
                      "--height_feature_extractor", str(h), "--width_feature_extractor", str(w),
                      "--compute_dtype", "fp32"])
    s.per_pixel_dataset_name = "cityscapes"
    return s


def test_evaluate_end_to_end(cuda, tmp_path, init_ckpt):
    """SemanticSegmentation.evaluate(): per-batch EVAL specs, device confusion matrices summed
    over the pass, void row/column dropped (system_factory.py:395-405)."""
    from input_pipelines.synthetic import evaluate_input
    from models.resnet50_extended_model_hierarchical import model
    from system_factory import SemanticSegmentation
    init_ckpt(tmp_path, pyramid="psp", height=64, width=128, nb_pp=2, dtype="fp32")
    s = _eval_settings(tmp_path)
    system = SemanticSegmentation({"eval": evaluate_input}, model, s)
    res = system.evaluate()
    assert len(res) == 1
    cm = res[0]["confusion_matrix"]
    assert cm.shape == (19, 19) and cm.dtype == np.int32
    # the same batches through the oracle-side confusion of the native decisions
    st = system.settings
    from estimator.define_estimator_hierarchical import define_estimator
    from system_factory import RunConfig
    from estimator.mode_keys import ModeKeys
    total = np.zeros((20, 20), np.int64)
    data = evaluate_input(RunConfig(), st)
    for _ in range(st.num_eval_steps):
        f, l = next(data)
        spec = define_estimator(ModeKeys.EVAL, f, l, model, RunConfig(), st)
        total += confusion_matrix(l["prolabels"].cpu().numpy(),
                                  spec.predictions["decisions"].cpu().numpy(), 20)
        assert float(spec.loss) == 0.0
    np.testing.assert_array_equal(cm, total[:-1, :-1])
    assert st.num_eval_steps == 2


def test_predict_end_to_end(cuda, tmp_path, init_ckpt):
    from input_pipelines.synthetic import predict_input
    from models.resnet50_extended_model_hierarchical import model
    from system_factory import SemanticSegmentation
    from utils.utils import SemanticSegmentationArguments
    from estimator.mode_keys import ModeKeys
    from models.resnet50_extended_model_hierarchical import add_model_arguments
    a = SemanticSegmentationArguments(mode=ModeKeys.PREDICT)
    add_model_arguments(a.argparser)
    s = a.parse_args([str(tmp_path), PROBLEM, str(tmp_path / "pred"), "--Nb", "1",
                      "--height_feature_extractor", "48", "--width_feature_extractor", "64",
                      "--compute_dtype", "fp32"])
    s.per_pixel_dataset_name = "cityscapes"
    init_ckpt(tmp_path, pyramid="none", height=48, width=64, nb_pp=1, dtype="fp32")
    system = SemanticSegmentation({"predict": predict_input}, model, s)
    preds = list(system.predict(max_steps=2))
    assert len(preds) == 2
    for p in preds:
        d = p["decisions"].cpu().numpy()
        assert d.shape == (1, 48, 64) and d.min() >= 0 and d.max() <= 19


def test_evaluate_script_main(cuda, tmp_path, init_ckpt):
    """evaluate.py main: the reference's command line, metrics written to <log_dir>/eval."""
    import importlib.util
    path = os.path.join(REPO, "iv2019-boosting-semantic-segmentation-with-weak-labels_amd",
                        "evaluate.py")
    spec = importlib.util.spec_from_file_location("seg_evaluate_main", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    init_ckpt(tmp_path, pyramid="none", height=48, width=64, nb_pp=1, dtype="fp32")
    res = mod.main([str(tmp_path), "2", PROBLEM, "cityscapes", "--Nb", "1",
                    "--height_feature_extractor", "48", "--width_feature_extractor", "64",
                    "--compute_dtype", "fp32"])
    # Neval 2 at Nb 1: two batches; the void row / column are dropped from the counts
    assert len(res) == 1 and 0 < int(res[0]["confusion_matrix"].sum()) <= 2 * 48 * 64
    txt = open(tmp_path / "eval" / "all_metrics.txt").read()
    assert txt.startswith("00000 ") and len(txt.split()) > 3   # step, global acc, mean acc, mIoU, ...
    z = np.load(tmp_path / "eval" / "all_metrics.npz")
    assert z["confusion_matrix"].shape == (1, 19, 19)



def test_confusion_more_than_64_classes(cuda):
    """Vistas evaluates 66 classes: the confusion matrix takes the global-atomic path."""
    cfg = CFGS[0]
    ctx = _ctx(cfg)
    rng = np.random.default_rng(4)
    lab = rng.integers(-1, 67, 100000).astype(np.int32)
    dec = rng.integers(0, 66, 100000).astype(np.int32)
    for nc in (20, 66):
        cm = torch.empty((nc, nc), dtype=torch.int32, device=cuda)
        ctx.confusion(torch.from_numpy(lab).to(cuda), torch.from_numpy(dec).to(cuda), nc, cm)
        ok = (lab >= 0) & (lab < nc) & (dec < nc)
        np.testing.assert_array_equal(cm.cpu().numpy(), confusion_matrix(lab[ok], dec[ok], nc))
    ctx.close()


def test_predict_script_exports(cuda, tmp_path, init_ckpt):
    """predict.py: images of predict_dir -> device preprocessing -> PREDICT -> decisions at the
    raw image size exported as label-id / colour / overlapped PNGs (predict.py:112-135)."""
    import importlib.util
    from PIL import Image
    pdir = tmp_path / "in"
    rdir = tmp_path / "out"
    pdir.mkdir()
    rdir.mkdir()
    rng = np.random.default_rng(6)
    for i in range(3):
        Image.fromarray(rng.integers(0, 256, (50, 90, 3), dtype=np.uint8)).save(pdir / f"img{i}.png")
    init_ckpt(tmp_path, pyramid="none", height=48, width=64, nb_pp=2, dtype="fp32")
    path = os.path.join(REPO, "iv2019-boosting-semantic-segmentation-with-weak-labels_amd",
                        "predict.py")
    spec = importlib.util.spec_from_file_location("seg_predict_main", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    # 3 images at Nb 2: the short last batch is padded, every image is exported
    n = mod.main([str(tmp_path), PROBLEM, str(pdir), "cityscapes", "--Nb", "2",
                  "--height_feature_extractor", "48", "--width_feature_extractor", "64",
                  "--compute_dtype", "fp32", "--results_dir", str(rdir), "--export_lids_images",
                  "--export_color_decisions", "--export_overlapped_color_decisions"])
    assert n == 3
    for i in range(3):
        lids = np.asarray(Image.open(rdir / f"img{i}_result_lids.png"))
        col = np.asarray(Image.open(rdir / f"img{i}_result_color.png"))
        assert lids.shape == (50, 90) and col.shape == (50, 90, 3)
        assert (rdir / f"img{i}_result_overlapped_color.png").exists()


@pytest.mark.parametrize("dataset", ["cityscapes", "vistas"])
def test_model_predictions_full_resolution(cuda, dataset):
    """model()'s predictions carry the reference's ten keys (hierarchical.py:121-130) at full
    network resolution: upsampled logits, per-head softmax and argmax, fused decisions. The
    oracle's head_predictions is fed the NATIVE low-res logits so the upsample / softmax /
    argmax / fusion is checked by itself: logits and probabilities 1e-5 relative, decisions
    equal up to fp32 near-ties (<= 0.1 % of the pixels)."""
    import argparse
    from input_pipelines.synthetic import batch
    from models.resnet50_extended_model_hierarchical import (LAZY_KEYS, model,
                                                             release_contexts)
    from estimator.mode_keys import ModeKeys
    h, w, nb = 48, 64, 2
    s = argparse.Namespace(Nb=nb, height_feature_extractor=h, width_feature_extractor=w,
                           per_pixel_dataset_name=dataset, compute_dtype="fp32",
                           pyramid="none", name_feature_extractor="resnet_v1_50")
    data = batch(21, nb, 0, 0, h, w)
    release_contexts()
    _, _, pred = model(ModeKeys.EVAL, torch.as_tensor(data["images"]).to(cuda), None, None, s)
    assert set(LAZY_KEYS) | {"decisions"} <= set(pred.keys())
    assert "l1_logits" not in pred.materialised()          # lazy until asked for
    c = (53, 12, 5) if dataset == "vistas" else (14, 7, 3)
    low_nat = {k: pred[f"{k}_lowres"].cpu().permute(0, 3, 1, 2).contiguous()
               for k in ("l1_logits", "l2_vehicle_logits", "l2_human_logits")}
    cfg = SegConfig(height=h, width=w, nb_pp=nb, pyramid="none", dataset=dataset)
    net = OracleNet(cfg, init_params(cfg, seed=0), dtype=torch.float32)
    up, probs, decs, fused = net.head_predictions(low_nat)
    for head, ci in zip(("l1", "l2_vehicle", "l2_human"), c):
        lg = pred[f"{head}_logits"]
        assert tuple(lg.shape) == (nb, h, w, ci)
        assert _rel(lg.cpu().numpy(), up[f"{head}_logits"].permute(0, 2, 3, 1).numpy()) < 1e-5
        pr = pred[f"{head}_probabilities"].cpu().numpy()
        assert _rel(pr, probs[f"{head}_logits"].permute(0, 2, 3, 1).numpy()) < 1e-5
        np.testing.assert_allclose(pr.sum(-1), 1.0, atol=1e-5)
        d = pred[f"{head}_decisions"].cpu().numpy()
        assert d.dtype == np.int32 and d.shape == (nb, h, w)
        assert float(np.mean(d != decs[f"{head}_logits"].numpy())) <= 1e-3
    # fused decisions (common cids) through the C ABI's optional decisions output
    fd = torch.full((nb, h, w), -1, dtype=torch.int32, device=cuda)
    pred["_context"].full_predictions(decisions=fd)
    assert float(np.mean(fd.cpu().numpy() != fused.numpy())) <= 1e-3
    # a newer forward invalidates the lazy entries not yet materialised
    _, _, pred2 = model(ModeKeys.EVAL, torch.as_tensor(data["images"]).to(cuda), None, None, s)
    model(ModeKeys.EVAL, torch.as_tensor(data["images"]).to(cuda), None, None, s)
    with pytest.raises(RuntimeError):
        pred2["l1_probabilities"]
    release_contexts()
