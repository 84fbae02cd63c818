"""Segment timing of the NT ping-pong main loop (A/B diagnostic, GPU box):
    SEG_HIP_LIB=ab/nttim/libseg_hip.so python tools/nt_timing.py fwd b4c2
(build: make VARIANT=nttim EXTRA=-DNT_DBG_TIMING). Per wave row, median s_memtime cycles of:
L0 (loop top -> before barrier A: phase-0 fragment reads, DMA issue, waits), barA wait, M0 (first
MFMA segment issue + row 0's vmcnt wait), barB, L1, barC, M1, and the whole K-tile (ideal: 2048
cycles of MFMA issue per SIMD at two waves)."""
import ctypes, os, runpy
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("REPS", "1")
runpy.run_path(os.path.join(REPO, "tools", "op_bench.py"), run_name="__main__")
from seg_hip import LIB
buf = (ctypes.c_ulonglong * (8 * 8 * 8 * 8))()
assert LIB.seg_dbg_nt_timing(buf) == 0
t = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(8, 8, 8, 8)  # block, wave, kt, stamp
names = ["L0", "barA", "M0", "barB", "L1", "barC", "M1"]
for row in (0, 1):
    w = t[:, row * 4:(row + 1) * 4]
    d = np.diff(w, axis=-1)
    kt = w[:, :, 1:, 0] - w[:, :, :-1, 0]
    med = [int(np.median(d[..., i])) for i in range(7)]
    print(f"row {row}: " + "  ".join(f"{n} {v}" for n, v in zip(names, med)) +
          f"  | K-tile {int(np.median(kt))} (ideal MFMA 2048)")
