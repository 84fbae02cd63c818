"""Per-tile phase timing of the persistent NT ping-pong kernel (A/B diagnostic, GPU box):
    SEG_HIP_LIB=.../build/tim/libseg_hip.so python tools/pp_timing.py fwd b3c3
(build: make VARIANT=tim EXTRA=-DPP_DBG_TIMING). Prints, in s_memtime cycles, the median per
tile of: main loop, fused statistics, staged epilogue + stores, and the gap to the next tile."""
import ctypes, os, runpy, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("REPS", "1")
runpy.run_path(os.path.join(REPO, "tools", "op_bench.py"), run_name="__main__")
from seg_hip import LIB
buf = (ctypes.c_ulonglong * (256 * 16 * 16))()
assert LIB.seg_dbg_pp_timing(buf) == 0
t = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(256, 16, 16)
valid = t[:, :, 0] > 0
n = valid.sum(axis=1)
print("tiles per block: min %d max %d" % (n.min(), n.max()))
ph = {"main": [], "stats": [], "epi": [], "gap": []}
# the epilogue's pieces (stamps 4-11): per column half the staging writes (from the previous
# stamp), statistics, staging barrier, staging reads + stores
sub = {f"q{q}_{n}": [] for q in (0, 1) for n in ("stage", "stats", "bar", "store")}
# RQ=1 (the one-tile residual epilogue, in place per 128-column half): stamps 4 + 3h after the
# residual wait and barrier, 5 + 3h after the in-place sums and barrier, 6 + 3h after the stores
RQ = os.environ.get("RQ") == "1"
if RQ:
    sub = {f"h{q}_{n}": [] for q in range(2) for n in ("wait", "add", "store")}
for b in range(256):
    for i in range(n[b]):
        r = t[b, i]
        ph["main"].append(r[1] - r[0]); ph["stats"].append(r[2] - r[1]); ph["epi"].append(r[3] - r[2])
        if i + 1 < n[b]:
            ph["gap"].append(t[b, i + 1, 0] - r[3])
        if r[4] > 0 and RQ:
            prev = r[2]
            for q in range(2):
                for j, nm in enumerate(("wait", "add", "store")):
                    sub[f"h{q}_{nm}"].append(r[4 + 3 * q + j] - prev)
                    prev = r[4 + 3 * q + j]
        elif r[4] > 0:
            prev = r[2]
            for q in (0, 1):
                for j, nm in enumerate(("stage", "stats", "bar", "store")):
                    sub[f"q{q}_{nm}"].append(r[4 + 4 * q + j] - prev)
                    prev = r[4 + 4 * q + j]
span = (t[:, :, 3][valid].max() - t[:, 0, 0].min())
print("kernel span %d cycles" % span)
for k, v in list(ph.items()) + list(sub.items()):
    if v:
        v = np.array(v)
        print("%-6s median %8d  p10 %8d  p90 %8d  (sum/block %8d)" % (k, np.median(v), np.percentile(v, 10), np.percentile(v, 90), v.sum() / 256))
