"""One C2 bf16 training step's gradient buffer from the working-tree library and from an A/B
build (SEG_HIP_LIB), each in its own child process: max relative difference per tensor class.
    python tools/ab_grads.py ab/<variant>/libseg_hip.so"""
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import os, sys
sys.path[:0] = [%r, %r]
import numpy as np, torch
from input_pipelines.synthetic import batch
from models.initializers import init_params
from seg_hip import SegContext
ctx = SegContext(depth=50, pyramid="aspp", height=1024, width=2048, nb_pp=4, dtype="bf16")
ctx.load_params(init_params(ctx.param_info, seed=0))
d = batch(1000, 4, 0, 0, 1024, 2048)
img = torch.as_tensor(d["images"]).cuda(); px = torch.as_tensor(d["px"]).cuda()
ctx.forward(img); ctx.loss(px); ctx.backward(); torch.cuda.synchronize()
np.save(sys.argv[1], ctx.grads.cpu().numpy())
print("losses", ctx.outputs()[0].cpu().numpy()[:4])
"""


def run(lib, out):
    env = dict(os.environ)
    env.pop("SEG_HIP_LIB", None)
    if lib:
        env["SEG_HIP_LIB"] = lib
    src = CHILD % (REPO, os.path.join(REPO, "iv2019-boosting-semantic-segmentation-with-weak-labels_amd"))
    r = subprocess.run([sys.executable, "-c", src, out], env=env, capture_output=True, text=True, timeout=300)
    print(r.stdout.strip(), r.stderr.strip()[-300:])
    r.check_returncode()
    return np.load(out)


a = run(None, "/tmp/ab_grads_a.npy")
b = run(os.path.abspath(sys.argv[1]), "/tmp/ab_grads_b.npy")
d = np.abs(a.astype(np.float64) - b)
print(f"grads: max |a-b| {d.max():.3e}, rel L2 {np.linalg.norm(d) / np.linalg.norm(a):.3e}, "
      f"bitwise equal {np.array_equal(a, b)}")
