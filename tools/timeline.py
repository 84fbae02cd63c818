"""Per-stream busy / idle time of one training step from a rocprofv3 kernel trace
(normal two-stream run): python tools/timeline.py gpurun_out/prof2/run_results.db
A step is delimited by the forward's stem conv (the first conv after the cast_pad8 kernel)."""
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
c = sqlite3.connect(db)
rows = c.execute("select name, stream_id, queue_id, start, end from kernels order by start").fetchall()
starts = [r[3] for r in rows if "cast_s2d_kernel" in r[0] or "cast_pad8_kernel" in r[0]]
if len(starts) < 3:
    sys.exit("need >= 3 steps")
# the second-to-last complete step (the last one is the bench's extra mIoU forward)
t0, t1 = starts[-3], starts[-2]
step = [r for r in rows if t0 <= r[3] < t1]
print(f"step: {(t1 - t0) / 1e6:.2f} ms, {len(step)} kernels")
by = defaultdict(list)
for n, s, q, a, b in step:
    by[(s, q)].append((a, b, n))
for key, ks in sorted(by.items(), key=lambda kv: -len(kv[1])):
    busy, last = 0, None
    gaps = []
    for a, b, n in ks:
        if last is not None and a > last:
            gaps.append((a - last, n))
        busy += b - max(a, last) if last is not None and a < last else b - a
        last = max(last or 0, b)
    gaps.sort(reverse=True)
    print(f"stream {key}: {len(ks)} kernels, busy {busy / 1e6:.2f} ms, idle {sum(g for g, _ in gaps) / 1e6:.2f} ms "
          f"in {len(gaps)} gaps; largest: " + ", ".join(f"{g / 1e3:.0f} us before {n[:40]}" for g, n in gaps[:6]))
# union busy (any stream)
iv = sorted((a, b) for _, _, _, a, b in step)
tot, cur_a, cur_b = 0, None, None
for a, b in iv:
    if cur_b is None or a > cur_b:
        if cur_b is not None:
            tot += cur_b - cur_a
        cur_a, cur_b = a, b
    else:
        cur_b = max(cur_b, b)
tot += cur_b - cur_a
print(f"GPU busy (any stream): {tot / 1e6:.2f} ms of {(t1 - t0) / 1e6:.2f}")

# optional: the last N kernels of the step per stream (start offset, duration, name)
if len(sys.argv) > 2:
    n_tail = int(sys.argv[2])
    print(f"last {n_tail} kernels of the step (offset ms from step start, duration us):")
    for n, s, q, a, b in step[-n_tail:]:
        print(f"  s{s}/q{q}  {(a - t0) / 1e6:8.3f}  {(b - a) / 1e3:8.1f}  {n[:90]}")
