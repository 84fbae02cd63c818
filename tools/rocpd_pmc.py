"""Print per-kernel PMC counter values (averaged over dispatches) from rocprofv3 rocpd
databases: python tools/rocpd_pmc.py DIR [name-substring]"""
import glob
import sqlite3
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    vals = defaultdict(lambda: defaultdict(list))
    for db in sorted(glob.glob(f"{d}/p*/run_results.db")):
        c = sqlite3.connect(db)
        # rows are per hardware instance: sum per (dispatch, counter), then average dispatches
        q = ("select kernel_name, counter_name, dispatch_id, sum(value) from counters_collection "
             "group by kernel_name, counter_name, dispatch_id")
        for name, cn, _, v in c.execute(q):
            if sub in name:
                vals[name][cn].append(v)
    for k, cv in vals.items():
        print(k[:100])
        for cn, v in sorted(cv.items()):
            print(f"   {cn:28s} {sum(v) / len(v):16.4g}  (n={len(v)})")


if __name__ == "__main__":
    main()
