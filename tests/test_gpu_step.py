"""End-to-end parity of one training step (forward, fused loss head, backward, SGDM, BN
moving statistics) through the C ABI against the oracle (TF 1.12 semantics, float64 CPU).

fp32 mode is held to the north-star 1e-3 relative tolerance (per tensor, L2-norm relative);
bf16 mode to 5e-2 on losses/logits (bf16 storage, fp32 accumulation)."""
import numpy as np
import pytest
import torch

from oracle.tfseg import OracleNet, SegConfig, init_params

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _native_step(cuda, cfg, params, data, dtype, lr=0.01, steps=1):
    from input_pipelines import synthetic  # noqa: F401  (path check)
    from seg_hip import SegContext
    ctx = SegContext(depth=cfg.depth, pyramid=cfg.pyramid, height=cfg.height, width=cfg.width,
                     nb_pp=cfg.nb_pp, nb_pb=cfg.nb_pb, nb_pi=cfg.nb_pi, dtype=dtype,
                     weight_decay=cfg.weight_decay, bn_decay=cfg.bn_decay)
    ctx.load_params(params)
    img = torch.as_tensor(data["images"]).to(cuda)
    px = torch.as_tensor(data["px"]).to(cuda) if cfg.nb_pp else None
    bb = torch.as_tensor(data["bbox"]).to(cuda) if cfg.nb_pb else None
    tg = torch.as_tensor(data["tag"]).to(cuda) if cfg.nb_pi else None
    dec = torch.zeros((cfg.nb, cfg.height, cfg.width), dtype=torch.int32, device=cuda)
    out = {}
    for _ in range(steps):
        ctx.forward(img)
        ctx.loss(px, bb, tg, dec)
        losses, reg, logits = ctx.outputs()
        out["losses"] = losses.cpu().numpy().copy()
        out["logits"] = logits.cpu().numpy().copy()
        ctx.backward()
        out["grads"] = ctx.named("grads")
        ctx.apply_update(lr, 0.9)
        torch.cuda.synchronize()
        out["reg"] = float(reg.cpu().numpy()[0])
    out["params"] = ctx.named("params")
    out["decisions"] = dec.cpu().numpy()
    ctx.close()
    return out


def _oracle_step(cfg, params, data, lr=0.01):
    net = OracleNet(cfg, params)
    L, low, g, newp, _, _, _ = net.train_step(data["images"], data["px"], data.get("bbox"),
                                              data.get("tag"), lr=lr)
    return L, low, g, newp


CONFIGS = [
    SegConfig(height=64, width=128, nb_pp=2, pyramid="psp"),
    SegConfig(height=64, width=96, nb_pp=1, nb_pb=1, nb_pi=1, pyramid="psp"),
    SegConfig(height=48, width=64, nb_pp=1, pyramid="none"),
]


@pytest.mark.parametrize("cfg", CONFIGS, ids=lambda c: f"{c.height}x{c.width}-{c.nb_pp}{c.nb_pb}{c.nb_pi}-{c.pyramid}")
def test_train_step_fp32(cuda, cfg):
    from input_pipelines.synthetic import batch
    params = {k: v.astype(np.float32) for k, v in init_params(cfg, seed=3).items()}
    data = batch(11, cfg.nb_pp, cfg.nb_pb, cfg.nb_pi, cfg.height, cfg.width)
    nat = _native_step(cuda, cfg, params, data, "fp32")
    L, low, g, newp = _oracle_step(cfg, params, data)
    # losses: {seg, l1, l2v, l2h, n1, n2v, n2h}
    ref = [float(L["segmentation"]), float(L["l1_segmentation"]),
           float(L["l2_vehicle_segmentation"]), float(L["l2_human_segmentation"])]
    np.testing.assert_allclose(nat["losses"][:4], ref, rtol=1e-3, atol=1e-6)
    assert tuple(int(v) for v in nat["losses"][4:7]) == tuple(L["counts"])
    assert abs(nat["reg"] - float(L["regularization"])) <= 1e-3 * float(L["regularization"])
    # low-res logits
    c1, c2, c3 = 14, 7, 3
    lg = nat["logits"]
    for key, a, b in (("l1_logits", 0, c1), ("l2_vehicle_logits", c1, c1 + c2),
                      ("l2_human_logits", c1 + c2, c1 + c2 + c3)):
        refl = low[key].detach().permute(0, 2, 3, 1).numpy()
        assert _rel(lg[..., a:b], refl) < 1e-3, key
    # gradients of every trainable tensor
    worst = max((_rel(nat["grads"][k], g[k].numpy().reshape(-1)), k) for k in g)
    assert worst[0] < 1e-3, worst
    # updated parameters and moving statistics
    for k, v in newp.items():
        assert _rel(nat["params"][k], v.detach().numpy().reshape(-1)) < 1e-4, k


def test_train_step_bf16(cuda):
    from input_pipelines.synthetic import batch
    cfg = SegConfig(height=64, width=128, nb_pp=1, nb_pb=1, pyramid="psp")
    params = {k: v.astype(np.float32) for k, v in init_params(cfg, seed=5).items()}
    data = batch(12, cfg.nb_pp, cfg.nb_pb, cfg.nb_pi, cfg.height, cfg.width)
    nat = _native_step(cuda, cfg, params, data, "bf16")
    L, low, g, newp = _oracle_step(cfg, params, data)
    np.testing.assert_allclose(nat["losses"][1], float(L["l1_segmentation"]), rtol=5e-2)
    refl = low["l1_logits"].detach().permute(0, 2, 3, 1).numpy()
    assert _rel(nat["logits"][..., :14], refl) < 5e-2
    gk = "feature_extractor/pyramid_module/Conv_4/weights"
    assert _rel(nat["grads"][gk], g[gk].numpy().reshape(-1)) < 0.1
