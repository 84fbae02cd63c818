"""Numerics of the linear BN-backward fold (csrc/lbf.h) at the bench shape (GPU box): for the
folded conv3 layers, the native weight gradient against float64 references built from the
step's own tensors -- with the exact conv output (z3 = y2 W3^T), with the stored 16-bit z3, and
through the materialised 16-bit dz3 (what tests/test_gpu_fullsize.py compares against)."""
import math, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "iv2019-boosting-semantic-segmentation-with-weak-labels_amd")]
import numpy as np
import torch
from input_pipelines.synthetic import batch
from oracle.tfseg import SegConfig, build_specs, init_params
from seg_hip import SegContext

H, W = 1024, 2048
cfg = SegConfig(depth=50, height=H, width=W, nb_pp=4, pyramid="aspp")
params = {k: v.astype(np.float32) for k, v in init_params(cfg, seed=2).items()}
data = batch(17, 4, 0, 0, H, W)
ctx = SegContext(depth=50, pyramid="aspp", height=H, width=W, nb_pp=4, dtype="bf16")
ctx.load_params(params)
dev = torch.device("cuda")
ctx.forward(torch.as_tensor(data["images"]).to(dev))
ctx.loss(torch.as_tensor(data["px"]).to(dev), None, None)
ctx.backward()
torch.cuda.synchronize()
print("lbf layers", ctx.counter("lbf_layers"))
specs = build_specs(cfg)
info = {p.name: p for p in ctx.param_info}


def rel(a, b):
    return float((a - b).norm() / b.norm())


for i, s in enumerate(specs):
    if not s.name.endswith("conv3") or "block" not in s.name:
        continue
    try:
        coef = ctx.debug_device(f"conv{i}_lbfcoef").double().reshape(3, -1)
    except Exception:
        continue
    y2 = ctx.debug_device(f"conv{i}_x").double().reshape(-1, s.ci)
    z3s = ctx.debug_device(f"conv{i}_y").double().reshape(-1, s.co)
    dyh = ctx.debug_device(f"conv{i}_dyhat").double().reshape(-1, s.co)
    w3 = torch.as_tensor(params[s.name + "/weights"]).to(dev).to(torch.bfloat16).double().reshape(s.co, s.ci)
    A, B, D = coef[0], coef[1], coef[2]
    z3e = y2 @ w3.t()
    dze = A * dyh + B + D * z3e
    dzs = A * dyh + B + D * z3s
    p = info[s.name + "/weights"]
    nat = ctx.grads[p.offset:p.offset + p.numel].view(s.co, s.ci).double()
    ref_e = dze.t() @ y2
    ref_s = dzs.t() @ y2
    dzm = ctx.debug_device(f"conv{i}_dy").double().reshape(-1, s.co)   # materialised (16-bit)
    ref_m = dzm.t() @ y2
    absref = dzm.abs().t() @ y2.abs()
    n = y2.shape[0]
    bound = 1e-3 * ref_m.abs() + 1e-4 * ref_m.pow(2).mean().sqrt() + 2.0 ** -24 * math.sqrt(n) * absref
    ex = ((nat - ref_m).abs() / bound)
    ex_e = ((ref_e - ref_m).abs() / bound)
    ratio = float((D.abs() * z3e.abs().mean(0)).mean() / dze.abs().mean())
    print(f"{s.name.split('resnet_v1_50/')[1]}: native vs exact-z3 {rel(nat, ref_e):.2e}, vs stored-z3 {rel(nat, ref_s):.2e}, "
          f"vs 16-bit dz3 {rel(nat, ref_m):.2e}; exact vs 16-bit dz3 {rel(ref_e, ref_m):.2e}; "
          f"test bound excess native {float(ex.max()):.2f} ({int((ex > 1).sum())} bad), exact-ref {float(ex_e.max()):.2f} "
          f"({int((ex_e > 1).sum())} bad); |D z3| / |dz3| {ratio:.2f}", flush=True)
    del y2, z3s, dyh, z3e, dze, dzs, ref_e, ref_s, dzm, ref_m, absref, bound, ex, ex_e
    torch.cuda.empty_cache()
