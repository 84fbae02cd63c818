"""Vistas label hierarchy (53 / 12 / 5 logits, 66 per-pixel classes) through the C ABI against
the oracle, whose VISTAS tables are transcribed from define_losses_hierarchical.py:38-74 and
resnet50_extended_model_hierarchical.py:95-106: one fp32 training step's losses, counts and
low-res logits (north-star 1e-3), the fused decisions of the loss head, and the EVAL
decisions of seg_predict (66 classes)."""
import numpy as np
import pytest
import torch

from oracle.tfseg import OracleNet, SegConfig, init_params

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def test_vistas_step_and_decisions(cuda):
    from input_pipelines.synthetic import bbox_labels, images, pixel_labels
    from seg_hip import SegContext
    cfg = SegConfig(height=64, width=128, nb_pp=1, nb_pb=1, pyramid="psp", dataset="vistas")
    params = {k: v.astype(np.float32) for k, v in init_params(cfg, seed=3).items()}
    rng = np.random.default_rng(21)
    img = images(rng, cfg.nb, cfg.height, cfg.width)
    px = pixel_labels(rng, cfg.nb_pp, cfg.height, cfg.width, n_classes=66)
    bb = bbox_labels(rng, cfg.nb_pb, cfg.height, cfg.width)
    ctx = SegContext(depth=50, pyramid="psp", height=cfg.height, width=cfg.width, nb_pp=1,
                     nb_pb=1, nb_pi=0, dtype="fp32", dataset="vistas")
    ctx.load_params(params)
    dec = torch.zeros((cfg.nb, cfg.height, cfg.width), dtype=torch.int32, device=cuda)
    ctx.forward(torch.as_tensor(img).to(cuda))
    ctx.loss(torch.as_tensor(px).to(cuda), torch.as_tensor(bb).to(cuda), None, dec)
    losses, _, lg = ctx.outputs()
    nat_l = losses.cpu().numpy().copy()
    lg = lg.cpu().numpy().copy()
    net = OracleNet(cfg, params, dtype=torch.float64)
    L, low, _, _, _, _, _ = net.train_step(img, px, bb, None, lr=0.01)
    ref = [float(L["segmentation"]), float(L["l1_segmentation"]),
           float(L["l2_vehicle_segmentation"]), float(L["l2_human_segmentation"])]
    np.testing.assert_allclose(nat_l[:4], ref, rtol=1e-3, atol=1e-6)
    for a, b in zip(nat_l[4:7], L["counts"]):   # weak weights follow the l1 argmax
        assert abs(int(a) - b) <= max(2, 1e-3 * b)
    c1, c2, c3 = 53, 12, 5
    net32 = OracleNet(cfg, params, dtype=torch.float32)
    _, low32, _, _, _, _, _ = net32.train_step(img, px, bb, None, lr=0.01)
    for key, a, b in (("l1_logits", 0, c1), ("l2_vehicle_logits", c1, c1 + c2),
                      ("l2_human_logits", c1 + c2, c1 + c2 + c3)):
        r = low[key].detach().permute(0, 2, 3, 1).numpy()
        gap = _rel(low32[key].detach().permute(0, 2, 3, 1).numpy(), r)
        assert _rel(lg[..., a:b], r) < max(1e-3, 4 * gap), (key, gap)
    # fused decisions: the oracle's rule on the NATIVE logits (decision logic by itself)
    lowt = torch.as_tensor(lg).permute(0, 3, 1, 2).contiguous()
    lowd = {"l1_logits": lowt[:, :c1], "l2_vehicle_logits": lowt[:, c1:c1 + c2],
            "l2_human_logits": lowt[:, c1 + c2:c1 + c2 + c3]}
    _, _, _, fused = net32.head_predictions(lowd)
    assert float(np.mean(dec.cpu().numpy() != fused.numpy())) <= 1e-3
    # EVAL decisions with a 66-class identity map (void = 65 -> -1 -> 65)
    cmap = list(range(65)) + [-1]
    out = torch.empty((cfg.nb, 40, 70), dtype=torch.int32, device=cuda)
    ctx.predict(cmap, out)
    refd = net32.eval_decisions(lowd, cmap, 40, 70).numpy()
    assert float(np.mean(out.cpu().numpy() != refd)) <= 1e-3
    ctx.close()
