"""Diagnostic: loss-head gradient (grad_un * dzscale) and head tensors vs the oracle."""
import os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "iv2019-boosting-semantic-segmentation-with-weak-labels_amd")]
from oracle.tfseg import SegConfig, init_params, OracleNet
from input_pipelines.synthetic import batch
from seg_hip import SegContext

def rel(a, b):
    return float(np.linalg.norm(np.float64(a) - np.float64(b)) / max(np.linalg.norm(np.float64(b)), 1e-30))

cfg = SegConfig(height=64, width=128, nb_pp=2, pyramid="psp")
params = {k: v.astype(np.float32) for k, v in init_params(cfg, seed=3).items()}
data = batch(11, cfg.nb_pp, cfg.nb_pb, cfg.nb_pi, cfg.height, cfg.width)
dev = torch.device("cuda", 0)
ctx = SegContext(pyramid="psp", height=64, width=128, nb_pp=2, dtype="fp32")
ctx.load_params(params)
ctx.forward(torch.as_tensor(data["images"]).to(dev))
ctx.loss(torch.as_tensor(data["px"]).to(dev))
ctx.backward()
torch.cuda.synchronize()
gu = ctx.debug_tensor("grad_un")
sc = ctx.debug_tensor("dzscale").reshape(-1)
dl = gu * sc[None, None, None, :gu.shape[-1]]
net = OracleNet(cfg, params)
trainable = [k for k in net.p if not k.endswith("moving_mean") and not k.endswith("moving_variance")]
for k in trainable: net.p[k].requires_grad_(True)
rec = {}
low = net.forward(torch.as_tensor(data["images"]), record=rec)
for k in ("l1_logits", "l2_vehicle_logits", "l2_human_logits"):
    low[k].retain_grad()
L = net.losses(low, data["px"])
L["segmentation"].backward()
off = 0
for k, c in (("l1_logits", 14), ("l2_vehicle_logits", 7), ("l2_human_logits", 3)):
    ref = low[k].grad.permute(0, 2, 3, 1).numpy()
    print("dlogits", k, rel(dl[..., off:off + c], ref))
    d = np.abs(dl[..., off:off + c] - ref).max(axis=-1)
    idx = np.unravel_index(np.argmax(d), d.shape)
    print("   worst pixel", idx, d[idx], np.abs(ref).max())
    off += c
for h, nm in enumerate(("l1", "l2_vehicle", "l2_human")):
    print("head out", nm, ctx.debug_tensor(f"head{h}_out").shape)
# per-conv forward outputs and gradients for every conv after the encoder
from oracle.tfseg import build_specs
specs = build_specs(cfg)
net2 = OracleNet(cfg, params)
for k in trainable: net2.p[k].requires_grad_(True)
rec = {}
low = net2.forward(torch.as_tensor(data["images"]), record=rec)
for v in rec.values(): v.retain_grad()
L = net2.losses(low, data["px"])
L["segmentation"].backward()
for i, s in enumerate(specs):
    if not (s.name.startswith("adaptation") or s.name.startswith("softmax") or "pyramid" in s.name or "decrease" in s.name or "block4/unit_3" in s.name):
        continue
    y = ctx.debug_tensor(f"conv{i}_y")
    dy = ctx.debug_tensor(f"conv{i}_dy")
    ry = rec[s.name].detach().permute(0, 2, 3, 1).numpy()
    rdy = rec[s.name].grad.permute(0, 2, 3, 1).numpy()
    print("%-60s y %.2e dy %.2e |dy| %.2e" % (s.name, rel(y, ry), rel(dy, rdy), np.linalg.norm(rdy)))
