"""Diagnostic (GPU box): head-side gradient errors of the fp32 step for the hybrid-upsampling
config of test_gpu_step.py, next to the same mix with bilinear upsampling. Per tensor: native vs
fp64 oracle, native vs fp32 oracle, fp32-vs-fp64 oracle gap, norm; and the weak-gate count
differences (native vs oracle l1 decisions on the bbox image)."""
import os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "iv2019-boosting-semantic-segmentation-with-weak-labels_amd"), os.path.join(REPO, "tests")]
from test_gpu_step import _native_step, _oracle_step, _rel
from oracle.tfseg import SegConfig, init_params
from input_pipelines.synthetic import batch

dev = torch.device("cuda", 0)
for ups in ("hybrid", "bilinear"):
    cfg = SegConfig(height=48, width=64, nb_pp=1, nb_pb=1, pyramid="none", upsampling=ups)
    params = {k: v.astype(np.float32) for k, v in init_params(cfg, seed=3).items()}
    data = batch(11, cfg.nb_pp, cfg.nb_pb, cfg.nb_pi, cfg.height, cfg.width)
    nat = _native_step(dev, cfg, params, data, "fp32")
    L, _, g, _ = _oracle_step(cfg, params, data)
    L32, _, g32, _ = _oracle_step(cfg, params, data, dtype=torch.float32)
    print(f"== {ups}: native counts {[int(v) for v in nat['losses'][4:7]]} oracle64 {list(L['counts'])} "
          f"oracle32 {list(L32['counts'])}", flush=True)
    rows = []
    for k in g:
        if "adaptation_module" not in k and "logits" not in k and "upsampl" not in k and "decrease" not in k:
            continue
        ref = g[k].numpy().reshape(-1)
        rows.append((_rel(nat["grads"][k], ref), _rel(nat["grads"][k], g32[k].numpy().reshape(-1)),
                     _rel(g32[k].numpy().reshape(-1), ref), float(np.linalg.norm(ref)), k))
    for r in sorted(rows, reverse=True)[:14]:
        print("  err64 %.2e err32 %.2e gap %.2e |g| %.3e %s" % r, flush=True)
