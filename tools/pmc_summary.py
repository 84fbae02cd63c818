"""Derived per-kernel counter metrics from the tools/pmc_passes.sh summaries (rocpd_pmc.py
text) of one measurement round: python tools/pmc_summary.py DIR OUT.json

For every pmc_<op>_<layer>.txt: MFMA busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
kernel cycles), kernel cycles = GRBM_GUI_ACTIVE / 8 (the GRBM counter sums the 8 XCDs); LDS bank
conflicts per LDS instruction; L2 (TCC) hit rate; HBM-side bytes (2 x FETCH_SIZE + WRITE_SIZE,
KiB counters, gfx950 FETCH correction of MI355X_MICROARCH.md) against the layer's compulsory
bytes; wave-cycle split (SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over
SQ_WAVE_CYCLES)."""
import glob
import json
import os
import re
import sys

SHAPES = {  # tools/op_bench.py: N, H, W, Ci, Co, k
    "b4c2": (4, 128, 256, 512, 512, 3), "b4c3": (4, 128, 256, 512, 2048, 1),
    "b4c1": (4, 128, 256, 2048, 512, 1), "b3c2": (4, 128, 256, 256, 256, 3),
    "b3c1": (4, 128, 256, 1024, 256, 1), "b3c3": (4, 128, 256, 256, 1024, 1),
}


def parse(path):
    out, name = {}, None
    for line in open(path):
        if not line.startswith(" "):
            name = line.strip()
            out[name] = {}
            continue
        m = re.match(r"\s+(\S+)\s+([-\d.e+]+)", line)
        if m and name:
            out[name][m.group(1)] = float(m.group(2))
    return out


def main():
    d, dst = sys.argv[1], sys.argv[2]
    res = {}
    for f in sorted(glob.glob(os.path.join(d, "pmc_*_*.txt"))):
        op, layer = os.path.basename(f)[4:-4].split("_", 1)
        for kname, c in parse(f).items():
            if "conv" not in kname or "GRBM_GUI_ACTIVE" not in c:
                continue
            cyc = c["GRBM_GUI_ACTIVE"] / 8.0
            N, H, W, Ci, Co, k = SHAPES[layer]
            P = N * H * W
            alg = {"fwd": (P * Ci + Co * k * k * Ci + P * Co) * 2,
                   "dgrad": (P * Co + Co * k * k * Ci + P * Ci) * 2,
                   "wgrad": (P * Co + P * Ci) * 2 + Co * k * k * Ci * 4}[op]
            hbm = (2 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024
            wc = c.get("SQ_WAVE_CYCLES", 0) or 1
            res[f"{op}_{layer}"] = {
                "kernel": kname.split("::")[-1][:80],
                "kernel_cycles": round(cyc),
                "mfma_busy_frac": round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc), 4),
                "mfma_insts": c.get("SQ_INSTS_MFMA"),
                "lds_bank_conflicts_per_lds_inst": round(c.get("SQ_LDS_BANK_CONFLICT", 0) /
                                                         max(c.get("SQ_INSTS_LDS", 1), 1), 4),
                "l2_hit_rate": round(c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4),
                "hbm_bytes": round(hbm), "algorithmic_bytes": alg,
                "traffic_ratio": round(hbm / alg, 3),
                "wave_cycles_waiting": round(c.get("SQ_WAIT_ANY", 0) / wc, 3),
                "wave_cycles_issue_stalled": round(c.get("SQ_WAIT_INST_ANY", 0) / wc, 3),
                "wave_cycles_issuing": round(c.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3),
            }
    res["method"] = ("rocprofv3 --kernel-trace --pmc, 5 separate passes per op (tools/pmc_passes.sh) "
                     "on tools/op_bench.py at the C2 layer shape (REPS=3, averaged dispatches)")
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
