"""Per-layer kernel timing of one bench-shaped step (GPU box): conv classes 0-2 in TFLOP/s,
BN streaming classes 3-5 (apply / bwd reduce / bwd apply) in TB/s of algorithmic traffic."""
import os, sys, collections
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "iv2019-boosting-semantic-segmentation-with-weak-labels_amd")]
import torch
from input_pipelines.synthetic import batch
from models.initializers import init_params
from seg_hip import SegContext
H, W, NB = 1024, 2048, 4
PYR = os.environ.get("PYRAMID", "aspp")
ctx = SegContext(depth=50, pyramid=PYR, height=H, width=W, nb_pp=NB, dtype="bf16")
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
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
with open(os.path.join(REPO, "gpurun_out", "layers.csv"), "w") as f:
    f.write("cls,name,ci,co,k,rate,ho,wo,gflop,ms\n")
    for r in rows:
        f.write("%d,%s,%d,%d,%d,%d,%d,%d,%.4f,%.5f\n" % (r["cls"], r["name"], r["ci"], r["co"], r["k"], r["rate"], r["ho"], r["wo"], r["gflop"], r["ms"]))
rows.sort(key=lambda r: -r["ms"])
bn = [r for r in rows if r["cls"] >= 3]
for k in (3, 4, 5):
    g = sum(r["gflop"] for r in bn if r["cls"] == k); t = sum(r["ms"] for r in bn if r["cls"] == k)
    print("BN class %d: %.2f GB in %.3f ms = %.2f TB/s" % (k, g, t, g / max(t, 1e-9)))
for r in bn[:25]:
    print("%d %-62s co=%4d %4dx%-4d %7.3f GB %7.3f ms %5.2f TB/s" % (
        r["cls"], r["name"][-62:], r["co"], r["ho"], r["wo"], r["gflop"], r["ms"], r["gflop"] / r["ms"]))
rows = [r for r in rows if r["cls"] < 3]
for r in rows[:45]:
    print("%d %-62s ci=%4d co=%4d k=%d r=%d %4dx%-4d %7.2f GF %7.3f ms %6.0f TF/s" % (
        r["cls"], r["name"][-62:], r["ci"], r["co"], r["k"], r["rate"], r["ho"], r["wo"], r["gflop"], r["ms"], r["gflop"] / r["ms"]))
