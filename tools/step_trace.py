"""Dump one training step's kernels (stream, start/end relative to the step, duration, name) from
a rocprofv3 kernel-trace database as CSV: python tools/step_trace.py run_results.db out.csv
(the second-to-last complete step, delimited like tools/timeline.py)."""
import csv
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, stream_id, start, end from kernels order by start").fetchall()
starts = [r[2] for r in rows if "cast_s2d_kernel" in r[0] or "cast_pad8_kernel" in r[0]]
t0, t1 = starts[-3], starts[-2]
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["stream", "start_us", "end_us", "dur_us", "name"])
    for n, s, a, b in rows:
        if t0 <= a < t1:
            w.writerow([s, round((a - t0) / 1e3, 2), round((b - t0) / 1e3, 2), round((b - a) / 1e3, 2), n[:90]])
