"""The TRAIN plumbing of the drop-in surface end to end: ``train.main`` (code/train.py:24-40)
-> ``SemanticSegmentation.train`` (system_factory.py:189-302: settings, LR boundaries in
epochs -> steps, the step loop, checkpoints) -> ``define_estimator(TRAIN)``
(define_estimator_hierarchical.py:77-129: model_fn, define_losses, create_train_op with the
EMA of the model variables in UPDATE_OPS, MomentumOptimizer) for three steps, against the
oracle's own three chained steps (OracleNet.train_step fed its own previous parameters,
momentum and EMA shadows, never the native state).

Configuration: fp32 (the reference's arithmetic), 64 x 128, no pyramid, a strong-only and a
2 : 1 : 1 strong : bbox : tag batch; EMA decay 0.9 with num_updates = global step, i.e.
min(0.9, (1+k)/(10+k)) at step k. The learning rate is the schedule's first segment in all
three steps: train.py sets Ntrain = 2975 for cityscapes whatever --Ntrain says (as the
reference's train.py:42-68 does), so the first piecewise boundary is >= 1487 steps away; the
schedule arithmetic (epochs -> steps, decayed values, tf.train.piecewise_constant's
x <= boundary rule) is pinned on the CPU by tests/test_host.py (test_learning_rate_schedule_
piecewise_constant, test_facade_lr_boundaries_in_epochs).

lr0 = 1e-5 (flag --learning_rate_initial), not the default 0.01, and no PSP: a random-init
ResNet at a test-sized input is chaotic under SGD, so no fp32 implementation can follow the
fp64 chain there. Measured on the oracle alone (its float32 chain against its float64 chain,
same seeds): at lr 0.01 the step-2 losses differ by 1-40 % even at 128 x 256 without a
pyramid; with PSP (BN of the 1 x 1 grid branch over 2 samples) by up to 1.8 % even at lr 1e-5;
without PSP at lr 1e-5 by < 1e-3. In that linear regime the losses check the data order and
each step's forward, and a wrong learning rate / momentum / EMA decay still shows at tens of
percent in the parameter deltas.

Weak batches: the l2 weights of weak pixels are gated by the l1 argmax
(define_losses_hierarchical.py:169-177), so a near-tied pixel can flip in or out between any
two implementations. Both oracle chains are therefore run under the NATIVE run's weight mask
(OracleNet.losses(weak_l1_decisions=...), the decisions captured from each native step's
predictions), which makes every loss term comparable at the north star's 1e-3; the l2 counts
under that mask must equal the native counts exactly (proof that the captured decisions are
the loss head's own), and the oracle's own gate may differ from the native one on at most
0.1 % of a weak image's pixels per head (the flip count, asserted separately).

Tolerances: the losses are read from the device after each step's train_op (fp32 scalars, not
the 4-decimal log line), all four terms, with no absolute slack: step 0 (both sides from the same
weights and inputs) at rtol 1e-3; steps 1-2 follow updated weights, whose gradients carry the
ill-conditioned early-layer error of every fp32 implementation (test_gpu_step.py's docstring),
so each term there is held to max(1e-3, 3 x the fp32 oracle's own relative gap on that term)
(measured: the fp32 oracle's l2h at step 2 of the strong-bbox-tag run is 6.5e-4 off fp64);
the parameter, momentum and EMA changes over the three steps (w3 - w0, v3, e3 - w0, all
trainable tensors flattened, L2-relative) max(1e-2, 3 x the fp32 oracle's own gap on the same
quantity); BN moving statistics max(1e-3, 4 x that gap).
"""
import re

import numpy as np
import pytest
import torch

from oracle.tfseg import OracleNet, SegConfig, init_params

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _capture_weak_decisions(monkeypatch, captured):
    """Wrap the estimator's define_losses: after each TRAIN loss head, record the native
    l1 decisions of the weak images (the Predictions' full-resolution l1 argmax of the same
    forward) and the loss head's non-zero-weight counts (n1, n2v, n2h)."""
    import estimator.define_estimator_hierarchical as deh
    orig = deh.define_losses

    def wrapped(mode, predictions, labels, config, params):
        L = orig(mode, predictions, labels, config, params)
        ctx = predictions['_context']
        npp = ctx.cfg.nb_pp
        d1 = predictions['l1_decisions'][npp:].cpu().numpy().astype(np.int64)
        captured.append((d1, L.counts()))
        return L
    monkeypatch.setattr(deh, "define_losses", wrapped)


def _check_losses(logged, ref_losses, l32):
    """Device loss terms vs the fp64 oracle chain: step 0 at rtol 1e-3; later steps at
    max(1e-3, 3 x the fp32 oracle chain's own relative gap), per term (module docstring)."""
    for k, (got, ref, r32) in enumerate(zip(logged, ref_losses, l32)):
        got, ref, r32 = np.array(got), np.array(ref), np.array(r32)
        scale = np.maximum(np.abs(ref), 1e-30)
        tol = 1e-3 if k == 0 else np.maximum(1e-3, 3 * np.abs(r32 - ref) / scale)
        assert np.all(np.abs(got - ref) <= tol * scale), (k, got, ref, r32)


def _capture_device_losses(monkeypatch, out):
    """Wrap the facade's define_estimator so that, right after each TRAIN step's train_op
    (define_estimator_hierarchical.py:120-129: the regulariser -- and so 'total' -- is written
    by the fused update), the four logged loss terms are read from the device as fp32 scalars
    (the same values the log line prints to 4 decimals)."""
    import system_factory as sf
    orig = sf.define_estimator

    def wrapped(mode, features, labels, model_fn, config, params):
        spec = orig(mode, features, labels, model_fn, config, params)
        if spec.train_op is None:
            return spec

        def train_op():
            L = spec.train_op()
            out.append(tuple(float(L[n]) for n in ("total", "l1_segmentation",
                                                   "l2_vehicle_segmentation",
                                                   "l2_human_segmentation")))
            return L
        return spec._replace(train_op=train_op)
    monkeypatch.setattr(sf, "define_estimator", wrapped)


def _gate_flips(net, low, weak, native_d1, npp):
    """Per weak image and l2 head: pixels whose weak-weight gate (not void, l1 decision ==
    the head's l1 class, max non-void soft label >= 0.01; define_losses_hierarchical.py:
    154-185) differs between the oracle's own l1 argmax and the native one."""
    from oracle.tfseg import TABLES
    t = TABLES[net.cfg.dataset]
    _, _, decs, _ = net.head_predictions(low)
    own = decs["l1_logits"][npp:].numpy()
    flips = []
    for table, cid in ((t["pb2veh"], t["cid_l1_vehicle"]), (t["pb2hum"], t["cid_l1_human"])):
        nseg = max(table) + 1
        y = np.zeros(weak.shape[:3] + (nseg,))
        for c, sid in enumerate(table):
            y[..., sid] += weak[..., c]
        ok = ((1.0 - y[..., -1]) > 0.01) & (y[..., :-1].max(-1) >= 0.01)
        flips.append((((own == cid) & ok) != ((native_d1 == cid) & ok)).reshape(len(own), -1).sum(1))
    return np.stack(flips)      # [2 heads, n weak]


@pytest.mark.parametrize("mix,nesterov", [((2, 0, 0), False), ((2, 1, 1), False), ((2, 0, 0), True)],
                         ids=["strong", "strong-bbox-tag", "strong-nesterov"])
def test_train_main_matches_oracle_trajectory(cuda, tmp_path, capsys, monkeypatch, mix, nesterov):
    import train
    from estimator.define_estimator_hierarchical import get_or_create_global_step
    from input_pipelines.synthetic import batch
    from models import resnet50_extended_model_hierarchical as mh
    mh.release_contexts()
    get_or_create_global_step().value = 0
    H, W = 64, 128
    npp, npb, npi = mix
    argv = [str(tmp_path / "logs"), "cityscapes", "--max_steps", "3", "--compute_dtype", "fp32",
            "--height_feature_extractor", str(H), "--width_feature_extractor", str(W),
            "--Nb_per_pixel", str(npp), "--Nb_per_bbox", str(npb), "--Nb_per_image", str(npi),
            "--learning_rate_initial", "1e-5",
            "--save_summaries_steps", "1", "--save_checkpoints_steps", "100"]
    if nesterov:   # MomentumOptimizer(use_nesterov=True), define_optimizer.py:17-20
        argv.append("--use_nesterov")
    native, logged = [], []
    _capture_weak_decisions(monkeypatch, native)
    _capture_device_losses(monkeypatch, logged)
    assert train.main(argv) == 3 and len(native) == 3
    out = capsys.readouterr().out
    printed = re.findall(r"step \d+: total ([-\d.]+) l1 ([-\d.]+) l2v ([-\d.]+) l2h ([-\d.]+)", out)
    assert len(logged) == 3 and len(printed) == 3, out
    # the log line is the device value rounded to 4 decimals
    assert all(abs(float(p[0]) - g[0]) <= 5.1e-5 for p, g in zip(printed, logged)), (printed, logged)
    ctx = next(iter(mh._CONTEXTS.values()))
    assert ctx.ema is not None   # ema_decay defaults to 0.9 (utils/utils.py:112)

    # the oracle's trajectory from the same seeded initialisation and the same batches
    cfg = SegConfig(height=H, width=W, nb_pp=npp, nb_pb=npb, nb_pi=npi, pyramid="none")
    p0 = {k: v.astype(np.float32) for k, v in init_params(cfg, seed=0).items()}
    native_init = mh.init_params(ctx.param_info, seed=0)
    assert all(np.array_equal(native_init[k].reshape(-1), p0[k].reshape(-1)) for k in p0)
    nweak = npb + npi

    def chain(dtype):
        params = {k: v.astype(np.float64) for k, v in p0.items()}
        mom = ema = None
        losses, flips = [], []
        for k, lr in enumerate((1e-5, 1e-5, 1e-5)):
            d = batch(k, npp, npb, npi, H, W)   # train.synthetic_train_input's seeds on rank 0
            net = OracleNet(cfg, params, dtype=dtype)
            d1 = native[k][0] if nweak else None   # the native run's weight mask
            L, low, _, new_p, mom, ema, _ = net.train_step(d["images"], d["px"], d["bbox"], d["tag"],
                                                           lr=lr, mom_state=mom, ema_state=ema,
                                                           ema_decay=0.9, step=k,
                                                           nesterov=nesterov, weak_l1_decisions=d1)
            losses.append(tuple(float(L[n].detach()) for n in (
                "total", "l1_segmentation", "l2_vehicle_segmentation", "l2_human_segmentation")))
            assert tuple(int(c) for c in L["counts"]) == native[k][1], (k, L["counts"], native[k][1])
            if nweak:
                weak = np.concatenate([x for x in (d["bbox"], d["tag"]) if x is not None and len(x)])
                flips.append(_gate_flips(net, {q: v.detach() for q, v in low.items()}, weak, d1, npp))
            params = {n: v.detach().numpy() for n, v in new_p.items()}
        return losses, params, {n: v.numpy() for n, v in mom.items()}, \
            {n: v.detach().numpy() for n, v in ema.items()}, flips

    ref_losses, ref_p, ref_m, ref_e, flips = chain(torch.float64)
    l32, p32, m32, e32, _ = chain(torch.float32)
    # every term at 1e-3: with weak images both chains use the native weak-weight mask
    _check_losses(logged, ref_losses, l32)
    # the gate itself, counted separately: the oracle's own argmax moves at most 0.1 % of a
    # weak image's pixels in or out of a head's weights (measured: <= 1 px at step 0, where
    # both start from the same weights; <= 4 of 8192 px at steps 1-2, where the trajectories
    # differ by the fp32-vs-fp64 gap)
    assert all(int(f.max()) <= max(2, H * W // 1000) for f in flips), flips

    nat_p, nat_m, nat_e = ctx.named("params"), ctx.named("momentum"), ctx.named("ema")
    keys = list(ref_m)
    flat = lambda d, ks: np.concatenate([np.asarray(d[k], np.float64).reshape(-1) for k in ks])
    w0 = flat(p0, keys)
    rows = []
    for what, nat, ref, r32, base in (("momentum", nat_m, ref_m, m32, 0), ("w3 - w0", nat_p, ref_p, p32, w0),
                                      ("ema - w0", nat_e, ref_e, e32, w0)):
        gap = _rel(flat(r32, keys) - base, flat(ref, keys) - base)
        err = _rel(flat(nat, keys) - base, flat(ref, keys) - base)
        rows.append((what, err, gap))
    assert all(err < max(1e-2, 3 * gap) for _, err, gap in rows), rows
    moving = [k for k in ref_p if "moving" in k]
    gap = _rel(flat(p32, moving), flat(ref_p, moving))
    assert _rel(flat(nat_p, moving), flat(ref_p, moving)) < max(1e-3, 4 * gap)
    # the final checkpoint carries the step, the weights and the EMA shadows
    state = torch.load(tmp_path / "logs" / "model.ckpt-3.pt", weights_only=True)
    assert state["global_step"] == 3 and "ema" in state
    mh.release_contexts()


def test_train_resumes_from_checkpoint(cuda, tmp_path):
    """A second train() in the same log_dir continues from model.ckpt-<step>.pt (loaded with
    torch.load(weights_only=True)) with the weights, BN moving statistics, momentum and EMA
    shadows of the first run (system_factory.py:279-302: the estimator's warm restart)."""
    import os
    import train
    from estimator.define_estimator_hierarchical import get_or_create_global_step
    from models import resnet50_extended_model_hierarchical as mh
    argv = [str(tmp_path / "logs"), "cityscapes", "--max_steps", "2", "--compute_dtype", "fp32",
            "--height_feature_extractor", "64", "--width_feature_extractor", "128",
            "--Nb_per_pixel", "2", "--Nb_per_bbox", "0", "--Nb_per_image", "0",
            "--save_summaries_steps", "100"]
    mh.release_contexts()
    get_or_create_global_step().value = 0
    assert train.main(argv) == 2
    ctx = next(iter(mh._CONTEXTS.values()))
    saved = {b: ctx.named(b) for b in ("params", "momentum", "ema")}
    assert any(np.any(v != 0) for v in saved["momentum"].values())
    mh.release_contexts()
    os.remove(tmp_path / "logs" / "settings.txt")   # train() refuses to overwrite it
    get_or_create_global_step().value = 0
    assert train.main(argv) == 2                      # restored at step 2: nothing left to run
    ctx = next(iter(mh._CONTEXTS.values()))
    for b, ref in saved.items():
        got = ctx.named(b)
        assert all(np.array_equal(got[k], ref[k]) for k in ref), b
    mh.release_contexts()


def test_train_main_real_data_matches_oracle(cuda, tmp_path, capsys, monkeypatch):
    """``train.main`` on the committed tiny real-data set
    (tests/golden/tiny_train: a per-pixel TFRecord + OpenImages-style box / tag indices and
    JPEGs) trains 2 steps through host decode (a pool of 3 threads, 2 batches ahead) ->
    device preprocessing (seg_prepare_images /
    _labels / _images_crop) -> device bbox rasterisation; every batch it consumed is captured
    and the oracle's own 2-step chain on those decoded batches (weak maps restated on the host
    by weak_labels.bbox_label_map / generate_tag_rla) matches the logged losses and the
    parameter / momentum / EMA changes, with the tolerances of the synthetic test above.
    The device image crop path is pinned bit-exactly to oracle.prepare_images_np on the first
    bbox image of each batch."""
    import json
    import os
    import train
    from estimator.define_estimator_hierarchical import get_or_create_global_step
    from input_pipelines import train_inputs
    from input_pipelines.weak_labels import bbox_label_map, generate_tag_rla
    from models import resnet50_extended_model_hierarchical as mh
    from oracle.tfseg import prepare_images_np
    tiny = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "tiny_train")
    mh.release_contexts()
    get_or_create_global_step().value = 0
    H, W = 64, 128
    from input_pipelines import tfrecords
    captured, crops = [], []
    orig = train_inputs.heterogeneous_train_input
    orig_crop = tfrecords.prepare_images_crop

    def crop(raw, resized, offset, h, w, stream=None):   # the decoded weak images, in order
        crops.append(raw.cpu().numpy()[0].copy())
        return orig_crop(raw, resized, offset, h, w, stream)

    def capture(config, params):
        for feats, labels in orig(config, params):
            captured.append((feats["proimages"].cpu().numpy().copy(),
                             labels["prolabels_per_pixel"].cpu().numpy().copy(),
                             list(labels["prolabels_per_bbox"]), list(labels["prolabels_per_image"])))
            yield feats, labels
    monkeypatch.setattr(train_inputs, "heterogeneous_train_input", capture)
    monkeypatch.setattr(tfrecords, "prepare_images_crop", crop)
    native, logged = [], []
    _capture_weak_decisions(monkeypatch, native)
    _capture_device_losses(monkeypatch, logged)
    argv = [str(tmp_path / "logs"), "cityscapes", "--max_steps", "2", "--compute_dtype", "fp32",
            "--height_feature_extractor", str(H), "--width_feature_extractor", str(W),
            "--Nb_per_pixel", "2", "--Nb_per_bbox", "1", "--Nb_per_image", "1",
            "--learning_rate_initial", "1e-5", "--save_summaries_steps", "1",
            "--save_checkpoints_steps", "100",
            "--tfrecords_path_per_pixel", os.path.join(tiny, "cityscapes.tfrecord"),
            "--bboxes_index_path", os.path.join(tiny, "bboxes.json"),
            "--bboxes_images_dir", os.path.join(tiny, "images"),
            "--image_labels_index_path", os.path.join(tiny, "tags.json"),
            "--image_labels_images_dir", os.path.join(tiny, "images"),
            "--input_workers", "3", "--input_prefetch", "2"]
    assert train.main(argv) == 2
    out = capsys.readouterr().out
    assert len(logged) == 2 and len(captured) >= 2, out
    ctx = next(iter(mh._CONTEXTS.values()))
    # the per-pixel labels are training cids (void = 19) and the crop path is bit-exact
    for k in range(2):
        _, px, boxes, _ = captured[k]
        assert px.min() >= 0 and px.max() <= 19
        cids, coords, src, rs, off = boxes[0]
        ref = prepare_images_np(crops[2 * k][None], H, W, resized=rs, offset=off)[0]
        assert np.array_equal(captured[k][0][2], ref)
    cfg = SegConfig(height=H, width=W, nb_pp=2, nb_pb=1, nb_pi=1, pyramid="none")
    p0 = {k: v.astype(np.float32) for k, v in init_params(cfg, seed=0).items()}

    def chain(dtype):
        params = {k: v.astype(np.float64) for k, v in p0.items()}
        mom = ema = None
        losses, flips = [], []
        for k in range(2):
            im, px, boxes, tags = captured[k]
            bb = np.stack([bbox_label_map(c, co, s, r, o, (H, W)) for c, co, s, r, o in boxes])
            tg = np.stack([np.broadcast_to(generate_tag_rla(list(t)), (H, W, 15)) for t in tags])
            net = OracleNet(cfg, params, dtype=dtype)
            d1 = native[k][0]   # the native run's weak-weight mask
            L, low, _, new_p, mom, ema, _ = net.train_step(im, px, bb.astype(np.float32),
                                                           tg.astype(np.float32), lr=1e-5,
                                                           mom_state=mom, ema_state=ema,
                                                           ema_decay=0.9, step=k,
                                                           weak_l1_decisions=d1)
            losses.append(tuple(float(L[n].detach()) for n in (
                "total", "l1_segmentation", "l2_vehicle_segmentation", "l2_human_segmentation")))
            assert tuple(int(c) for c in L["counts"]) == native[k][1], (k, L["counts"], native[k][1])
            flips.append(_gate_flips(net, {q: v.detach() for q, v in low.items()},
                                     np.concatenate([bb, tg]), d1, 2))
            params = {n: v.detach().numpy() for n, v in new_p.items()}
        return losses, params, {n: v.numpy() for n, v in mom.items()}, \
            {n: v.detach().numpy() for n, v in ema.items()}, flips

    ref_losses, ref_p, ref_m, ref_e, flips = chain(torch.float64)
    l32, p32, m32, e32, _ = chain(torch.float32)
    _check_losses(logged, ref_losses, l32)
    assert all(int(f.max()) <= max(2, H * W // 1000) for f in flips), flips
    nat_p, nat_m, nat_e = ctx.named("params"), ctx.named("momentum"), ctx.named("ema")
    keys = list(ref_m)
    flat = lambda d, ks: np.concatenate([np.asarray(d[k], np.float64).reshape(-1) for k in ks])
    w0 = flat(p0, keys)
    rows = []
    for what, nat, ref, r32, base in (("momentum", nat_m, ref_m, m32, 0), ("w2 - w0", nat_p, ref_p, p32, w0),
                                      ("ema - w0", nat_e, ref_e, e32, w0)):
        gap = _rel(flat(r32, keys) - base, flat(ref, keys) - base)
        err = _rel(flat(nat, keys) - base, flat(ref, keys) - base)
        rows.append((what, err, gap))
    assert all(err < max(1e-2, 3 * gap) for _, err, gap in rows), rows
    assert json.load(open(os.path.join(tiny, "tags.json")))
    mh.release_contexts()


@pytest.mark.timeout(600)
def test_train_main_c1_reference_default_shape(cuda, tmp_path, monkeypatch):
    """BASELINE config C1 -- the reference train.py's own Cityscapes default
    (code/train.py:55-64: ResNet-50, no pyramid module, 512 x 1024, batch 2 per-pixel images,
    Nb_per_bbox = Nb_per_image = 0), fp32 (the reference's arithmetic), through ``train.main``
    for one step at the default learning rate 0.01 and EMA 0.9, against OracleNet.train_step in
    float64 on the same seeded batch (train.synthetic_train_input's seed for rank 0, step 0).

    Tolerances: loss terms at rtol 1e-3 (device fp32 values, no absolute slack) and the
    non-zero-weight counts exact; the low-resolution logits (64 x 128) L2-relative max(1e-3,
    4 x the fp32 oracle's own gap); the parameter change w1 - w0, the momentum and the EMA change
    max(1e-2, 3 x that gap) (the trajectory tests' bound); BN moving statistics max(1e-3, 4 x gap).
    At 512 x 1024 every BN channel of the encoder averages >= 16k samples, so the conditioning
    problem of the small step tests (module docstring of test_gpu_step.py) is much weaker here."""
    import train
    from estimator.define_estimator_hierarchical import get_or_create_global_step
    from input_pipelines.synthetic import batch
    from models import resnet50_extended_model_hierarchical as mh
    mh.release_contexts()
    get_or_create_global_step().value = 0
    H, W, NPP = 512, 1024, 2
    argv = [str(tmp_path / "logs"), "cityscapes", "--max_steps", "1", "--compute_dtype", "fp32",
            "--height_feature_extractor", str(H), "--width_feature_extractor", str(W),
            "--Nb_per_pixel", str(NPP), "--Nb_per_bbox", "0", "--Nb_per_image", "0",
            "--synthetic_pool", "1", "--save_summaries_steps", "1", "--save_checkpoints_steps", "100"]
    import estimator.define_estimator_hierarchical as deh
    orig = deh.define_losses
    seen, logged = [], []

    def wrapped(mode, predictions, labels, config, params):
        L = orig(mode, predictions, labels, config, params)
        ctx = predictions['_context']
        seen.append((ctx.outputs()[2].cpu().numpy().copy(), L.counts(),
                     float(params.learning_rate_initial)))
        return L
    monkeypatch.setattr(deh, "define_losses", wrapped)
    _capture_device_losses(monkeypatch, logged)
    assert train.main(argv) == 1 and len(seen) == 1 and len(logged) == 1
    ctx = next(iter(mh._CONTEXTS.values()))
    assert (ctx.cfg.depth, ctx.cfg.height, ctx.cfg.width, ctx.cfg.nb_pp) == (50, H, W, NPP)
    assert ctx.cfg.pyramid in (0, "none")   # seg_cfg.pyramid: 0 = no pyramid module
    logits, counts, lr = seen[0]
    assert lr == 0.01
    nat_p, nat_m, nat_e = ctx.named("params"), ctx.named("momentum"), ctx.named("ema")

    cfg = SegConfig(height=H, width=W, nb_pp=NPP, pyramid="none")
    p0 = {k: v.astype(np.float32) for k, v in init_params(cfg, seed=0).items()}
    d = batch(0, NPP, 0, 0, H, W)

    def step(dtype):
        net = OracleNet(cfg, {k: v.astype(np.float64) for k, v in p0.items()}, dtype=dtype)
        L, low, _, new_p, mom, ema, _ = net.train_step(d["images"], d["px"], lr=lr, ema_decay=0.9,
                                                       step=0)
        out = (tuple(float(L[n].detach()) for n in ("total", "l1_segmentation",
                                                   "l2_vehicle_segmentation", "l2_human_segmentation")),
               tuple(int(c) for c in L["counts"]),
               {q: v.detach().permute(0, 2, 3, 1).numpy() for q, v in low.items()},
               {n: v.detach().numpy() for n, v in new_p.items()},
               {n: v.numpy() for n, v in mom.items()}, {n: v.detach().numpy() for n, v in ema.items()})
        del net, L, low
        return out

    ref_l, ref_c, ref_low, ref_p, ref_m, ref_e = step(torch.float64)
    l32, _, low32, p32, m32, e32 = step(torch.float32)
    got = np.array(logged[0])
    assert np.all(np.abs(got - np.array(ref_l)) <= 1e-3 * np.abs(np.array(ref_l))), (got, ref_l, l32)
    assert counts == ref_c, (counts, ref_c)
    c1, c2 = 14, 7
    for key, a, b in (("l1_logits", 0, c1), ("l2_vehicle_logits", c1, c1 + c2),
                      ("l2_human_logits", c1 + c2, c1 + c2 + 3)):
        gap = _rel(low32[key], ref_low[key])
        err = _rel(logits[..., a:b], ref_low[key])
        assert err < max(1e-3, 4 * gap), (key, err, gap)
    keys = list(ref_m)
    flat = lambda dd, ks: np.concatenate([np.asarray(dd[k], np.float64).reshape(-1) for k in ks])
    w0 = flat(p0, keys)
    rows = []
    for what, nat, ref, r32, base in (("momentum", nat_m, ref_m, m32, 0), ("w1 - w0", nat_p, ref_p, p32, w0),
                                      ("ema - w0", nat_e, ref_e, e32, w0)):
        gap = _rel(flat(r32, keys) - base, flat(ref, keys) - base)
        err = _rel(flat(nat, keys) - base, flat(ref, keys) - base)
        rows.append((what, err, gap))
    assert all(err < max(1e-2, 3 * gap) for _, err, gap in rows), rows
    moving = [k for k in ref_p if "moving" in k]
    gap = _rel(flat(p32, moving), flat(ref_p, moving))
    assert _rel(flat(nat_p, moving), flat(ref_p, moving)) < max(1e-3, 4 * gap)
    print("C1 parity:", rows, "losses", got.tolist(), ref_l)
    mh.release_contexts()


@pytest.mark.timeout(900)
def test_train_main_c1_trajectory_needs_the_fp32_gap(cuda, tmp_path, monkeypatch, capsys):
    """is the relaxed trajectory bound of the 64 x 128 tests (steps 1-2 at
    max(1e-3, 3 x the fp32 oracle's own gap)) needed at a realistic shape? Three chained
    ``train.main`` steps at BASELINE config C1 (R50, no pyramid, 512 x 1024, 2 per-pixel images,
    fp32, the default learning rate 0.01, EMA 0.9; train.synthetic_train_input's batches 0-2 on
    rank 0) against OracleNet.train_step chained in float64 from the same initialisation (the
    oracle fed its own previous parameters, momentum and EMA shadows), and the same chain in
    float32 beside it.

    Answer (first run, profiles/r06_c1_trajectory.txt): yes. At lr 0.01 the float32 ORACLE
    itself is 0.4-1.3e-2 off float64 on the step-1 / step-2 loss terms (l2 heads worst), while
    step 0 agrees to 2e-6; the parameter change w3 - w0 differs by 0.67 (L2-relative) for the
    float32 oracle and the native chain alike. The native chain tracks float64 as closely as the
    float32 restatement does (per term at most 1.3x its gap; 0.26-1.0x on 7 of the 8). So no
    fp32 implementation meets a bare 1e-3 after the first update at this learning rate; the
    1.30e-3 vs 6.5e-4 of the 64 x 128 run is that same fp32 divergence, not a native defect.

    Asserted: step 0 at a bare rtol 1e-3 on all four device-read loss terms, counts exact every
    step; steps 1-2 per term at max(1e-3, 2 x the float32 oracle's own gap) (tighter than the
    small tests' 3x); the float32 oracle's own gap above 1e-3 on some step-1/2 term (the fact
    that makes the bare bound unreachable); the parameter change and momentum within 1.5x the
    float32 oracle's own distance from float64."""
    import train
    from estimator.define_estimator_hierarchical import get_or_create_global_step
    from input_pipelines.synthetic import batch
    from models import resnet50_extended_model_hierarchical as mh
    mh.release_contexts()
    get_or_create_global_step().value = 0
    H, W, NPP, STEPS = 512, 1024, 2, 3
    argv = [str(tmp_path / "logs"), "cityscapes", "--max_steps", str(STEPS), "--compute_dtype", "fp32",
            "--height_feature_extractor", str(H), "--width_feature_extractor", str(W),
            "--Nb_per_pixel", str(NPP), "--Nb_per_bbox", "0", "--Nb_per_image", "0",
            "--save_summaries_steps", "1", "--save_checkpoints_steps", "100"]
    import estimator.define_estimator_hierarchical as deh
    orig = deh.define_losses
    counts, logged = [], []

    def wrapped(mode, predictions, labels, config, params):
        L = orig(mode, predictions, labels, config, params)
        counts.append(L.counts())
        return L
    monkeypatch.setattr(deh, "define_losses", wrapped)
    _capture_device_losses(monkeypatch, logged)
    assert train.main(argv) == STEPS and len(logged) == STEPS
    ctx = next(iter(mh._CONTEXTS.values()))
    nat_p, nat_m = ctx.named("params"), ctx.named("momentum")
    mh.release_contexts()

    cfg = SegConfig(height=H, width=W, nb_pp=NPP, pyramid="none")
    p0 = {k: v.astype(np.float32) for k, v in init_params(cfg, seed=0).items()}

    def chain(dtype):
        params = {k: v.astype(np.float64) for k, v in p0.items()}
        mom = ema = None
        losses, cnts = [], []
        for k in range(STEPS):
            d = batch(k, NPP, 0, 0, H, W)
            net = OracleNet(cfg, params, dtype=dtype)
            L, low, _, new_p, mom, ema, _ = net.train_step(d["images"], d["px"], lr=0.01, mom_state=mom,
                                                           ema_state=ema, ema_decay=0.9, step=k)
            losses.append(tuple(float(L[n].detach()) for n in (
                "total", "l1_segmentation", "l2_vehicle_segmentation", "l2_human_segmentation")))
            cnts.append(tuple(int(c) for c in L["counts"]))
            params = {n: v.detach().numpy() for n, v in new_p.items()}
            del net, L, low
        return losses, cnts, params, {n: v.numpy() for n, v in mom.items()}

    ref_l, ref_c, ref_p, ref_m = chain(torch.float64)
    l32, _, p32, m32 = chain(torch.float32)
    got = np.array(logged)
    ref = np.array(ref_l)
    err = np.abs(got - ref) / np.abs(ref)
    gap32 = np.abs(np.array(l32) - ref) / np.abs(ref)
    keys = list(ref_m)
    flat = lambda dd, ks: np.concatenate([np.asarray(dd[k], np.float64).reshape(-1) for k in ks])
    w0 = flat(p0, keys)
    dw = (_rel(flat(nat_p, keys) - w0, flat(ref_p, keys) - w0), _rel(flat(p32, keys) - w0, flat(ref_p, keys) - w0))
    dm = (_rel(flat(nat_m, keys), flat(ref_m, keys)), _rel(flat(m32, keys), flat(ref_m, keys)))
    print("C1 trajectory: native rel err per step / term", err.tolist())
    print("C1 trajectory: fp32 oracle rel gap per step / term", gap32.tolist())
    print("C1 trajectory: w3 - w0 rel err native / fp32 oracle", dw, "momentum", dm)
    assert [tuple(c) for c in counts] == ref_c, (counts, ref_c)
    assert np.all(err[0] <= 1e-3), err[0]
    assert np.all(err[1:] <= np.maximum(1e-3, 2 * gap32[1:])), (err.tolist(), gap32.tolist())
    assert gap32[1:].max() > 1e-3, gap32.tolist()
    assert dw[0] <= 1.5 * dw[1] and dm[0] <= 1.5 * dm[1], (dw, dm)
