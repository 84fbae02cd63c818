"""Diagnostic (GPU box): how much of test_gpu_step.py's gradient tolerance each fp32 step
configuration uses. Per config: well-conditioned tensors (fp32-oracle gap < 1e-3) -> max of
err / max(1e-3, 4 gap); ill-conditioned ones -> max err, max err / gap, and the largest
err / max(floor, 2 gap) for a few candidate floors."""
import os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "iv2019-boosting-semantic-segmentation-with-weak-labels_amd"), os.path.join(REPO, "tests")]
from test_gpu_step import CONFIGS, _native_step, _oracle_step, _rel
from oracle.tfseg import init_params
from input_pipelines.synthetic import batch

dev = torch.device("cuda", 0)
floors = (5e-2, 3e-2, 2e-2, 1e-2)
for cfg in CONFIGS:
    params = {k: v.astype(np.float32) for k, v in init_params(cfg, seed=3).items()}
    data = batch(11, cfg.nb_pp, cfg.nb_pb, cfg.nb_pi, cfg.height, cfg.width)
    nat = _native_step(dev, cfg, params, data, "fp32")
    _, _, g, _ = _oracle_step(cfg, params, data)
    _, _, g32, _ = _oracle_step(cfg, params, data, dtype=torch.float32)
    well, ill = [], []
    for k in g:
        e = _rel(nat["grads"][k], g[k].numpy().reshape(-1))
        c = _rel(g32[k].numpy().reshape(-1), g[k].numpy().reshape(-1))
        (well if c < 1e-3 else ill).append((e, c, k))
    name = f"r{cfg.depth}-{cfg.height}x{cfg.width}-{cfg.nb_pp}{cfg.nb_pb}{cfg.nb_pi}-{cfg.pyramid}-fov{cfg.fov_k}-{cfg.upsampling}-{cfg.norm}"
    wu = max((e / max(1e-3, 4 * c) for e, c, _ in well), default=0.0)
    line = f"{name}: {len(well)} well (max use {wu:.2f})"
    if ill:
        me = max(e for e, _, _ in ill)
        mr = max(e / c for e, c, _ in ill)
        uses = " ".join(f"floor {f:g}: {max(e / max(f, 2 * c) for e, c, _ in ill):.2f}" for f in floors)
        worst = max(ill)
        line += f"; {len(ill)} ill (max err {me:.2e}, max err/gap {mr:.2f}; {uses}; worst {worst[2]} err {worst[0]:.2e} gap {worst[1]:.2e})"
    print(line, flush=True)
