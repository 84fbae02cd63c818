"""Summarise a rocprofv3 kernel-trace database (rocpd SQLite, ROCm 7 default output) into the
classic --stats CSV (Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs) plus
per-class totals matching bench.py's profile classes.

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db [out.csv] [--skip-steps S]

Classes: fwd/dgrad share conv_nt*_kernel (split by bench's own HIP events, not separable
here); wgrad = conv_wgrad*_kernel.
"""
import csv
import sqlite3
import sys


def main():
    db = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else None
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), "
                     "max(duration) from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows)
    table = [[n, k, s, round(a, 1), round(100.0 * s / total, 3), mn, mx] for n, k, s, a, mn, mx in rows]
    hdr = ["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"]
    if out:
        with open(out, "w", newline="") as f:
            w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
            w.writerow(hdr)
            w.writerows(table)
    for r in table[:25]:
        print(f"{r[4]:6.2f}%  {r[1]:6d}  avg {r[3] / 1e3:9.3f} us  {r[0][:110]}")
    cls = {"conv_nt (fwd+dgrad)": ("conv_nt_kernel", "conv_nt_v2_kernel", "conv_nt_pp_kernel", "conv_nt_patch_kernel", "conv_nt_patch_s2d_kernel"),
           "conv_wgrad": ("conv_wgrad_kernel", "conv_wgrad_v2_kernel", "conv_wgrad_pp_kernel")}
    for k, pats in cls.items():
        sel = [r for r in rows if any(f"::{p}<" in r[0] for p in pats)]
        n = sum(r[1] for r in sel)
        s = sum(r[2] for r in sel)
        print(f"class {k}: {n} launches, total {s / 1e6:.3f} ms, avg {s / max(n, 1) / 1e3:.3f} us")
    print(f"all kernels: {total / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
