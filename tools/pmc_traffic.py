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
         "where counter_name = ? group by kernel_name, dispatch_id order by dispatch_id")
    return [(n, d, v) for n, d, v in c.execute(q, (counter,))]


def step_class(n):
    for k in ("conv_wgrad", "splitk_reduce", "conv_nt", "bn_apply8", "bn_bwd_reduce", "bn_bwd_apply",
              "bn_stats_final", "bn_bwd_final", "sgdm", "loss_head", "maxpool", "skinny", "grid_",
              "resize", "psp_", "weight_flip", "bn_relu_maxpool", "cast_"):
        if k in n:
            return k
    return "other"


def step_ledger(fetch, write):
    """HBM-side bytes of ONE training step (the last complete one: the dispatches from the
    second-to-last image cast to the last, which starts the bench's extra mIoU forward), per
    kernel class: reads 2 x FETCH_SIZE, writes WRITE_SIZE (Infinity-Cache hits included)."""
    casts = [i for i, (n, _, _) in enumerate(fetch) if "cast_s2d_kernel" in n or "cast_pad8_kernel" in n]
    lo, hi = casts[-3], casts[-2]
    wmap = {d: v for _, d, v in write}
    by = {}
    for n, d, v in fetch[lo:hi]:
        c = step_class(n)
        e = by.setdefault(c, {"launches": 0, "read_bytes": 0.0, "write_bytes": 0.0})
        e["launches"] += 1
        e["read_bytes"] += 2.0 * 1024.0 * v
        e["write_bytes"] += 1024.0 * wmap.get(d, 0.0)
    tot_r = sum(e["read_bytes"] for e in by.values())
    tot_w = sum(e["write_bytes"] for e in by.values())
    return {"dispatches": hi - lo, "read_bytes": tot_r, "write_bytes": tot_w,
            "hbm_bytes": tot_r + tot_w,
            "classes": dict(sorted(by.items(), key=lambda kv: -(kv[1]["read_bytes"] + kv[1]["write_bytes"])))}


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
    try:
        res["step"] = step_ledger(fetch, write)
    except (IndexError, ValueError) as e:
        res["step"] = {"error": repr(e)}
    res["method"] = ("rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE (separate passes) on "
                     "bench.py --steps 3 --warmup 1; reads = 2 x FETCH_SIZE (gfx950 correction)")
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
