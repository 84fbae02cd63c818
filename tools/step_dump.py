"""Every kernel of one two-stream training step from a rocprofv3 kernel trace, as CSV
(start offset us, duration us, stream, name): python tools/step_dump.py run_results.db out.csv"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, stream_id, queue_id, start, end from kernels order by start").fetchall()
starts = [r[3] for r in rows if "cast_s2d_kernel" in r[0] or "cast_pad8_kernel" in r[0]]
t0, t1 = starts[-3], starts[-2]
with open(sys.argv[2], "w") as f:
    f.write("start_us,dur_us,stream,name\n")
    for n, s, q, a, b in rows:
        if t0 <= a < t1:
            short = n.replace("void ", "", 1).replace("(anonymous namespace)::", "").split("(")[0]
            f.write("%.2f,%.2f,%d,%s\n" % ((a - t0) / 1e3, (b - a) / 1e3, s, short.replace(",", ";")))
