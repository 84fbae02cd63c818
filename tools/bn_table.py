"""Per-layer table of the BN streaming classes: for every BN apply (3),
BN-backward reduce (4) and BN-backward apply (5) launch of a profiled C2 step (layers.csv from
tools/layer_report.py), grouped by channel count and rows: launches, algorithmic GB, kernel-alone
ms, TB/s, fraction of the 8 TB/s HBM peak and of the 6.29 TB/s measured copy ceiling
(MI355X_MICROARCH.md). Class 5 rows of the folded conv3 layers also carry the linear
BN-backward fold's prep / H / combine launches, which are not streaming work.
    python tools/bn_table.py profiles/r06_s7_layers.csv"""
import collections
import csv
import sys

NAMES = {3: "bn_apply8 (fwd BN + ReLU [+ residual])", 4: "bn_bwd_reduce8", 5: "bn_bwd_apply8 (+ fold ops)"}
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
for r in rows:
    c = int(r["cls"])
    if c < 3:
        continue
    m = int(r["ho"]) * int(r["wo"])
    k = (c, int(r["co"]), m)
    agg[k][0] += 1
    agg[k][1] += float(r["gflop"])   # BN classes: the gflop field holds algorithmic GB
    agg[k][2] += float(r["ms"])
for c in (3, 4, 5):
    tot_ms = sum(v[2] for k, v in agg.items() if k[0] == c)
    print(f"== class {c} {NAMES[c]}: {tot_ms:.3f} ms per step")
    print(f"{'C':>6} {'rows/img':>9} {'launches':>8} {'GB':>8} {'ms':>8} {'us/launch':>9} {'TB/s':>6} {'/8TB/s':>7} {'/copy':>6}")
    for (cc, co, m), (n, gb, ms) in sorted(agg.items()):
        if cc != c or ms <= 0:
            continue
        tbs = gb / ms
        print(f"{co:>6} {m:>9} {n:>8} {gb:>8.3f} {ms:>8.3f} {1e3 * ms / n:>9.1f} {tbs:>6.2f} {tbs / 8:>7.3f} {tbs / 6.29:>6.3f}")
