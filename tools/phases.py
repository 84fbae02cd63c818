"""Forward / backward phase split of one two-stream training step from a rocprofv3 kernel
trace (python tools/phases.py run_results.db): per phase, wall time, per-stream busy time and
the kernel classes on each stream (sum of kernel durations), to see where the side stream
(weight gradients) overlaps the compute stream and what each phase costs."""
import sqlite3
import sys
from collections import defaultdict

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, stream_id, queue_id, start, end from kernels order by start").fetchall()
starts = [r[3] for r in rows if "cast_s2d_kernel" in r[0] or "cast_pad8_kernel" in r[0]]
t0, t1 = starts[-3], starts[-2]
step = [r for r in rows if t0 <= r[3] < t1]
lh = [r for r in step if "loss_head_kernel" in r[0]][0]
t_b = lh[4]


def cls(n):
    for k in ("conv_wgrad", "splitk_reduce", "conv_nt", "bn_apply8", "bn_bwd_reduce", "bn_bwd_apply",
              "bn_stats_final", "bn_bwd_final", "sgdm", "loss_head", "maxpool", "skinny", "grid_", "resize",
              "psp_", "weight_flip"):
        if k in n:
            return k
    return n.split("(")[0][-30:]


def busy(ks):
    tot, last = 0, None
    for a, b in sorted(ks):
        if last is None or a >= last:
            tot += b - a
            last = b
        elif b > last:
            tot += b - last
            last = b
    return tot


print(f"step {(t1 - t0) / 1e6:.2f} ms: forward {(t_b - t0) / 1e6:.2f} ms, backward+update {(t1 - t_b) / 1e6:.2f} ms")
for name, lo, hi in (("forward", t0, t_b), ("backward", t_b, t1)):
    ph = [r for r in step if lo <= r[3] < hi]
    streams = defaultdict(list)
    for r in ph:
        streams[r[1]].append(r)
    for s, ks in sorted(streams.items(), key=lambda kv: -len(kv[1])):
        by = defaultdict(float)
        for r in ks:
            by[cls(r[0])] += (r[4] - r[3]) / 1e6
        top = sorted(by.items(), key=lambda kv: -kv[1])[:8]
        print(f"  {name} stream {s}: {len(ks)} kernels, busy {busy([(r[3], r[4]) for r in ks]) / 1e6:.2f} ms; "
              + ", ".join(f"{k} {v:.2f}" for k, v in top))
