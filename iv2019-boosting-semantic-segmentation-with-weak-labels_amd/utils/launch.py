"""One process per GPU, started by the program itself (the reference's ``--distribute`` takes
every visible GPU in one launch: ``tf.contrib.distribute.MirroredStrategy()``,
code/system_factory.py:276-283).

``spawn_ranks`` starts N child processes of a script with the ``torch.distributed`` rendezvous
variables set (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, a free
MASTER_PORT), before the parent touches the GPU (the parent only counts devices, which does not
initialise one). Children are plain ``subprocess`` processes -- never an exec of the parent --
in the parent's process group, so a ``timeout`` or a terminal's group signal reaches them too;
the parent also forwards SIGTERM / SIGINT / SIGHUP to every live child and stops the others as
soon as one rank fails. Returns 0 only when every rank exited 0.

``rank_device`` maps LOCAL_RANK to the device a rank uses: one rank per GPU under RCCL; the
gloo backend (``SEG_*_BACKEND=gloo``: rehearsing N ranks on one GPU, RCCL cannot share a
device) wraps around the visible devices.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import List, Optional, Sequence


def visible_gpus() -> int:
    """Visible devices, counted without initialising one (torch.cuda.device_count on ROCm)."""
    import torch
    return torch.cuda.device_count()


def free_port() -> int:
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def rank_device(local_rank: int, backend: str, ndev: int) -> int:
    if ndev <= 0:
        raise RuntimeError(f"LOCAL_RANK {local_rank}: no visible GPU")
    if local_rank >= ndev:
        if backend == "nccl":
            raise RuntimeError(f"LOCAL_RANK {local_rank} but only {ndev} visible GPU(s): one rank "
                               "per GPU under RCCL (the gloo backend rehearses N ranks on fewer GPUs)")
        return local_rank % ndev
    return local_rank


def spawn_ranks(n: int, cmd: Sequence[str], outs: Optional[List] = None, deadline_s: Optional[float] = None,
                name: str = "launch", poll_s: float = 0.2) -> int:
    """Run ``cmd`` as N ranks (module docstring). ``outs[r]``: rank r's stdout file object, or
    None to inherit the parent's. ``deadline_s``: wall-clock limit of the whole run (every rank
    is stopped when it passes; returns 124). A rank that fails stops the others; its exit
    code (or 1 for a signal) is returned."""
    if n < 1:
        raise ValueError(f"{name}: need at least one rank, got {n}")
    port = free_port()
    procs: List[subprocess.Popen] = []
    stop = {"sig": None}

    def _forward(sig, _frame):
        stop["sig"] = sig
        for p in procs:
            if p.poll() is None:
                try:
                    p.send_signal(sig)
                except OSError:
                    pass

    handled = (signal.SIGTERM, signal.SIGINT, signal.SIGHUP)
    previous = {s: signal.signal(s, _forward) for s in handled}
    rc = 0
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                       LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            out = outs[r] if outs is not None else None
            procs.append(subprocess.Popen(list(cmd), env=env, stdout=out))
        t0 = time.monotonic()
        live = set(range(n))
        while live:
            for r in sorted(live):
                c = procs[r].poll()
                if c is None:
                    continue
                live.discard(r)
                if c != 0:
                    print(f"{name}: rank {r} exited with {c}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    rc = rc or (c if c > 0 else 1)
            if rc or stop["sig"] is not None:
                break
            if deadline_s is not None and time.monotonic() - t0 > deadline_s:
                print(f"{name}: deadline of {deadline_s:.0f} s passed; stopping every rank",
                      file=sys.stderr, flush=True)
                rc = 124
                break
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        for s, h in previous.items():
            signal.signal(s, h)
    if stop["sig"] is not None:
        return 128 + int(stop["sig"])
    return rc
