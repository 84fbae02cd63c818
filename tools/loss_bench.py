"""Loss-head timing at the C2 shape (GPU box): python tools/loss_bench.py [reps]."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "iv2019-boosting-semantic-segmentation-with-weak-labels_amd")]
import torch
from input_pipelines.synthetic import batch
from models.initializers import init_params
from seg_hip import SegContext
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
ctx = SegContext(depth=50, pyramid="aspp", height=1024, width=2048, nb_pp=4, dtype="bf16")
ctx.load_params(init_params(ctx.param_info, seed=0))
d = batch(1000, 4, 0, 0, 1024, 2048)
img = torch.as_tensor(d["images"]).cuda(); px = torch.as_tensor(d["px"]).cuda()
ctx.forward(img); ctx.loss(px); torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    ctx.loss(px)
e1.record(); torch.cuda.synchronize()
print("loss head + finalize: %.1f us" % (e0.elapsed_time(e1) / reps * 1e3), ctx.outputs()[0][:4].tolist())
