"""Segment timing of the short-K double-buffered NT kernel (conv_db.hip; A/B diagnostic, GPU box):
    SEG_HIP_LIB=ab/dbtim/libseg_hip.so python tools/db_timing.py fwd b4c3
(build: make VARIANT=dbtim EXTRA=-DDB_DBG_TIMING). Per stagger group, median s_memtime cycles of
the load segment's parts (epilogue work, DMA issue, fragment reads, group 1's vmcnt wait), barrier
A, the MFMA segment, group 0's vmcnt wait, barrier B, and the whole item (ideal: 1024 cycles of
MFMA issue per SIMD at two waves)."""
import ctypes, os, runpy
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("REPS", "1")
runpy.run_path(os.path.join(REPO, "tools", "op_bench.py"), run_name="__main__")
from seg_hip import LIB
buf = (ctypes.c_ulonglong * (8 * 8 * 8 * 10))()
assert LIB.seg_dbg_db_timing(buf) == 0
t = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(8, 8, 8, 10)  # block, wave, item, stamp
names = ["epi", "dma", "frag", "vm1", "barA", "mfma", "vm0", "barB"]
for grp in (0, 1):
    w = t[:, grp * 4:(grp + 1) * 4, :, :9]
    d = np.diff(w, axis=-1)
    it = w[:, :, 1:, 0] - w[:, :, :-1, 0]
    med = [int(np.median(d[..., i])) for i in range(8)]
    print(f"group {grp}: " + "  ".join(f"{n} {v}" for n, v in zip(names, med)) +
          f"  | item {int(np.median(it))} (ideal MFMA 1024)")
