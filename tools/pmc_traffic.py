"""Per-kernel-class HBM traffic from the two PMC passes of tools/pmc_traffic.sh.

FETCH_SIZE and WRITE_SIZE are reported in KiB per dispatch. On gfx950 FETCH_SIZE counts half
the bytes of wide coalesced streaming reads (MI355X_MICROARCH.md, HBM section), so reads are
taken as 2 x FETCH_SIZE; WRITE_SIZE is exact for 16-B-per-lane stores.

    python tools/pmc_traffic.py OUTDIR profiles/r01_pmc_traffic.json
"""
import json
import sqlite3
import sys
from collections import defaultdict

CLASSES = {"conv_wgrad": ("conv_wgrad_pp_kernel", "conv_wgrad_v2_kernel", "conv_wgrad_kernel"),
           "conv_nt": ("conv_nt_pp_kernel", "conv_nt_v2_kernel", "conv_nt_kernel")}


def per_dispatch(db, counter):
    c = sqlite3.connect(db)
    q = ("select kernel_name, dispatch_id, sum(value) from counters_collection "
         "where counter_name = ? group by kernel_name, dispatch_id")
    return [(n, d, v) for n, d, v in c.execute(q, (counter,))]


def main():
    out, dst = sys.argv[1], sys.argv[2]
    fetch = per_dispatch(f"{out}/fetch/run_results.db", "FETCH_SIZE")
    write = per_dispatch(f"{out}/write/run_results.db", "WRITE_SIZE")
    res = {}
    for cls, pats in CLASSES.items():
        f = [v for n, _, v in fetch if any(f"::{p}<" in n for p in pats)]
        w = [v for n, _, v in write if any(f"::{p}<" in n for p in pats)]
        if not f or not w:
            continue
        rd = 2.0 * 1024.0 * sum(f) / len(f)
        wr = 1024.0 * sum(w) / len(w)
        res[cls] = {"launches_sampled": len(f), "read_bytes_per_launch": rd,
                    "write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr}
    res["method"] = ("rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE (separate passes) on "
                     "bench.py --steps 3 --warmup 1; reads = 2 x FETCH_SIZE (gfx950 correction)")
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
