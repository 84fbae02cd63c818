"""Eager vs hipGraph-replayed step timing (GPU box): the forward + loss + backward launches
captured once through torch.cuda.graph (our C ABI launches on torch's current stream)."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "iv2019-boosting-semantic-segmentation-with-weak-labels_amd")]
import torch
from input_pipelines.synthetic import batch
from models.initializers import init_params
from seg_hip import SegContext
H, W, NB = 1024, 2048, 4
ctx = SegContext(depth=50, pyramid="aspp", height=H, width=W, nb_pp=NB, dtype="bf16")
ctx.load_params(init_params(ctx.param_info, seed=0))
d = batch(1000, NB, 0, 0, H, W)
img = torch.as_tensor(d["images"]).cuda(); px = torch.as_tensor(d["px"]).cuda()
def fwdbwd():
    ctx.forward(img); ctx.loss(px); ctx.backward()
def step():
    fwdbwd(); ctx.apply_update(0.0, 0.9)
for _ in range(3): step()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(10): step()
torch.cuda.synchronize()
te = (time.perf_counter() - t) / 10
l_eager = ctx.outputs()[0].cpu().clone()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
g = torch.cuda.CUDAGraph()
with torch.cuda.stream(s):
    fwdbwd()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        fwdbwd()
torch.cuda.synchronize()
def gstep():
    g.replay(); ctx.apply_update(0.0, 0.9)
for _ in range(3): gstep()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(10): gstep()
torch.cuda.synchronize()
tg = (time.perf_counter() - t) / 10
l_graph = ctx.outputs()[0].cpu().clone()
print(f"eager {te*1e3:.2f} ms/step ({NB/te:.1f} img/s), graph {tg*1e3:.2f} ms/step ({NB/tg:.1f} img/s)")
print("losses eager", l_eager[:4].tolist(), "graph", l_graph[:4].tolist())
