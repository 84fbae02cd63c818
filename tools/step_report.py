"""Per-layer time budget of one bench-shaped training step (GPU box), from the context's own
HIP-event profile (single-stream backward): every conv launch (TFLOP/s vs the bf16 MFMA peak)
and BN streaming launch (algorithmic TB/s vs the 8 TB/s HBM peak), sorted by the time above a
reference rate (1.5 PFLOP/s for convs, 6 TB/s for streaming), with class totals.

    python tools/step_report.py [C2|C3|C5] > gpurun_out/step_report.txt"""
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "iv2019-boosting-semantic-segmentation-with-weak-labels_amd")]
import torch  # noqa: E402
from input_pipelines.synthetic import batch  # noqa: E402
from models.initializers import init_params  # noqa: E402
from seg_hip import SegContext  # noqa: E402

CFG = {"C2": (50, (4, 0, 0), "bf16"), "C3": (101, (4, 0, 0), "bf16"), "C5": (101, (1, 2, 1), "fp16")}
name = sys.argv[1] if len(sys.argv) > 1 else "C2"
depth, (npp, npb, npi), dt = CFG[name]
H, W = 1024, 2048
ctx = SegContext(depth=depth, pyramid="aspp", height=H, width=W, nb_pp=npp, nb_pb=npb, nb_pi=npi,
                 dtype=dt, ema=True)
ctx.load_params(init_params(ctx.param_info, seed=0))
if dt == "fp16":
    ctx.set_loss_scale(8192.0)
d = batch(1000, npp, npb, npi, H, W)
dev = lambda a: None if a is None else torch.as_tensor(a).cuda()
img, px, bb, tg = dev(d["images"]), dev(d["px"]), dev(d["bbox"]), dev(d["tag"])


def step():
    ctx.forward(img)
    ctx.loss(px, bb, tg)
    ctx.backward()
    ctx.apply_update(0.01, 0.9, 0.5, 1.0)


for _ in range(3):
    step()
torch.cuda.synchronize()
ctx.profile(True)
step()
torch.cuda.synchronize()
rows = ctx.profile_dump()
CLS = ["fwd", "dgrad", "wgrad", "bn_apply", "bn_bwd_reduce", "bn_bwd_apply"]
tot = collections.defaultdict(lambda: [0.0, 0.0, 0])
att = collections.defaultdict(float)
fam_att = collections.defaultdict(float)
out = []
for r in rows:
    c = r["cls"]
    t = tot[CLS[c]]
    t[0] += r["ms"]; t[1] += r["gflop"]; t[2] += 1
    if c < 3:
        rate = r["gflop"] / r["ms"]            # TFLOP/s
        ideal = r["gflop"] / 1500.0             # ms at 1.5 PFLOP/s
        unit = "TF/s"
    else:
        rate = r["gflop"] / r["ms"]            # TB/s (gflop field = GB for BN classes)
        ideal = r["gflop"] / 6.0
        unit = "TB/s"
    if c < 3:   # attainable: max(flops / 2.5 PF, compulsory bytes / 6.3 TB/s achievable)
        att[CLS[c]] += max(r["gflop"] / 2500.0, r.get("gbytes", 0.0) / 6.3)
        fam_att[(CLS[c], r["ci"], r["co"], r["k"], r["ho"])] += max(r["gflop"] / 2500.0, r.get("gbytes", 0.0) / 6.3)
    out.append((r["ms"] - ideal, CLS[c], r["name"], r["ci"], r["co"], r["k"], r["rate"], r["ho"], r["wo"], r["ms"], rate, unit,
                r.get("gbytes", 0.0) / r["ms"] if c < 3 else rate))
print(f"{name}: class totals")
for k in CLS:
    ms, gf, n = tot[k]
    u = "TF/s" if k in ("fwd", "dgrad", "wgrad") else "TB/s"
    extra = f"  attainable {att[k]:7.3f} ms ({att[k] / max(ms, 1e-9):.2f})" if k in att else ""
    print(f"  {k:14s} {n:4d} launches {ms:8.3f} ms  {gf / max(ms, 1e-9):8.1f} {u}{extra}")
fam = collections.defaultdict(lambda: [0.0, 0.0, 0])
for lost, c, nm, ci, co, k, rt, ho, wo, ms, rate, unit, tbs in out:
    key = (c, ci, co, k, ho)
    fam[key][0] += ms; fam[key][1] += lost; fam[key][2] += 1
print("\nfamilies (class ci co k Ho): launches, ms, ms above the reference rate")
for key, (ms, lost, n) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
    a = fam_att.get(key)
    at = f"  attainable {a:7.3f} ms ({a / ms:.2f})" if a else ""
    print(f"  {key[0]:13s} {key[1]:5d} {key[2]:5d} k{key[3]} {key[4]:4d}  {n:3d}  {ms:7.3f} ms  {lost:7.3f} ms{at}")
print("\nlaunches by time above the reference rate (ms lost, class, layer, ci co k rate HoxWo, ms, rate, compulsory TB/s)")
for lost, c, nm, ci, co, k, rt, ho, wo, ms, rate, unit, tbs in sorted(out, reverse=True)[:70]:
    print(f"{lost:7.3f} {c:13s} {nm[-58:]:58s} {ci:5d} {co:5d} {k} r{rt:<2d} {ho}x{wo} {ms:7.3f} ms {rate:7.1f} {unit} {tbs:5.2f} TB/s")
