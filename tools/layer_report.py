"""Per-layer conv kernel timing of one bench-shaped step (GPU box): TFLOP/s per launch."""
import os, sys, collections
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "iv2019-boosting-semantic-segmentation-with-weak-labels_amd")]
import torch
from input_pipelines.synthetic import batch
from models.initializers import init_params
from seg_hip import SegContext
H, W, NB = 1024, 2048, 4
ctx = SegContext(depth=50, pyramid="psp", height=H, width=W, nb_pp=NB, dtype="bf16")
ctx.load_params(init_params(ctx.param_info, seed=0))
d = batch(1000, NB, 0, 0, H, W)
img = torch.as_tensor(d["images"]).cuda(); px = torch.as_tensor(d["px"]).cuda()
def step():
    ctx.forward(img); ctx.loss(px); ctx.backward(); ctx.apply_update(0.01, 0.9)
for _ in range(2): step()
torch.cuda.synchronize()
ctx.profile(True)
step()
torch.cuda.synchronize()
rows = ctx.profile_dump()
tot = collections.defaultdict(float)
for r in rows:
    tot[r["cls"]] += r["ms"]
print("class totals ms:", dict(tot))
rows.sort(key=lambda r: -r["ms"])
for r in rows[:45]:
    print("%d %-62s ci=%4d co=%4d k=%d r=%d %4dx%-4d %7.2f GF %7.3f ms %6.0f TF/s" % (
        r["cls"], r["name"][-62:], r["ci"], r["co"], r["k"], r["rate"], r["ho"], r["wo"], r["gflop"], r["ms"], r["gflop"] / r["ms"]))
