"""Which co-running pair costs the backward: per compute-stream kernel of
one training step, its duration beside the weight-gradient stream (two-stream trace) against
its duration alone (single-stream trace, SEG_SIDE_STREAM=0, same kernel order once the
weight-gradient kernels are removed), and what ran beside it on the side stream.

    python tools/corun.py two_stream.db single_stream.db

Per compute-kernel class: launches, time alone, time beside the side stream, the slow-down,
and the slow-down split over the side-stream classes by overlap time (conv_wgrad, splitk
reduce, nothing). A step is delimited like tools/timeline.py (the image cast kernels)."""
import sqlite3
import sys
from collections import defaultdict

SIDE = ("conv_wgrad", "splitk_reduce")


def cls(n):
    for k in ("conv_wgrad", "splitk_reduce", "conv_nt", "bn_apply8", "bn_bwd_reduce", "bn_bwd_apply",
              "bn_stats_final", "bn_bwd_final", "sgdm", "loss_head", "maxpool", "skinny", "grid_",
              "resize", "psp_", "weight_flip"):
        if k in n:
            return k
    return n.split("(")[0][-30:]


def step_rows(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, stream_id, start, end from kernels order by start").fetchall()
    rows = [r for r in rows if "at::native" not in r[0]]   # host-side torch ops (train.py loss sums)
    starts = [r[2] for r in rows if "cast_s2d_kernel" in r[0] or "cast_pad8_kernel" in r[0]]
    t0, t1 = starts[-3], starts[-2]
    step = [r for r in rows if t0 <= r[2] < t1]
    lh = [r for r in step if "loss_head_kernel" in r[0]][0]
    return step, lh[3]


def main():
    two, t_b2 = step_rows(sys.argv[1])
    one, t_b1 = step_rows(sys.argv[2])
    streams = defaultdict(int)
    for r in two:
        if r[2] >= t_b2:
            streams[r[1]] += 1
    side_ids = {r[1] for r in two if cls(r[0]) in SIDE}
    comp2 = [r for r in two if r[2] >= t_b2 and r[1] not in side_ids]
    side2 = [r for r in two if r[1] in side_ids]
    comp1 = [r for r in one if r[2] >= t_b1 and cls(r[0]) not in SIDE]
    if [cls(r[0]) for r in comp1] != [cls(r[0]) for r in comp2]:
        # sgdm / flips may sit differently; align on the common prefix of identical classes
        n = 0
        while n < min(len(comp1), len(comp2)) and cls(comp1[n][0]) == cls(comp2[n][0]):
            n += 1
        print(f"warning: kernel sequences differ after {n} of {len(comp1)} / {len(comp2)}")
        comp1, comp2 = comp1[:n], comp2[:n]
    agg = defaultdict(lambda: defaultdict(float))
    for a, b in zip(comp1, comp2):
        c = cls(b[0])
        d1, d2 = (a[3] - a[2]) / 1e3, (b[3] - b[2]) / 1e3
        ov = defaultdict(float)
        for s in side2:
            lo, hi = max(b[2], s[2]), min(b[3], s[3])
            if hi > lo:
                ov[cls(s[0])] += (hi - lo) / 1e3
        none = max(0.0, d2 - sum(ov.values()))
        tot = max(d2, 1e-9)
        g = agg[c]
        g["n"] += 1
        g["alone_us"] += d1
        g["beside_us"] += d2
        slow = d2 - d1
        for k, v in list(ov.items()) + [("nothing", none)]:
            g[f"ov_{k}_us"] += v
            g[f"slow_{k}_us"] += slow * v / tot
    print(f"backward compute-stream kernels: {len(comp2)} (side stream: {len(side2)} kernels)")
    print(f"{'class':16s} {'n':>4s} {'alone ms':>9s} {'beside ms':>9s} {'slow ms':>8s}  "
          "slow-down by co-runner (ms) [overlap ms]")
    tot = defaultdict(float)
    for c, g in sorted(agg.items(), key=lambda kv: -kv[1]["beside_us"]):
        parts = []
        for k in SIDE + ("nothing",):
            if g.get(f"ov_{k}_us", 0) > 0:
                parts.append(f"{k} {g[f'slow_{k}_us'] / 1e3:+.2f} [{g[f'ov_{k}_us'] / 1e3:.2f}]")
                tot[k] += g[f"slow_{k}_us"]
        print(f"{c:16s} {int(g['n']):4d} {g['alone_us'] / 1e3:9.2f} {g['beside_us'] / 1e3:9.2f} "
              f"{(g['beside_us'] - g['alone_us']) / 1e3:+8.2f}  " + ", ".join(parts))
    print("total slow-down by co-runner: " + ", ".join(f"{k} {v / 1e3:+.2f} ms" for k, v in tot.items()))


if __name__ == "__main__":
    main()
