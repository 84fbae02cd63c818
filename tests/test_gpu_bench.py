"""bench.py's own launch paths on the GPU box (subprocesses, so the test process's GPU state is
not shared with the ranks):

* `--config C1` -- the reference train.py's Cityscapes default (R50, no pyramid module,
  512 x 1024, batch 2; BASELINE.json configs[0]) runs through the bench's training step and
  prints one JSON line with finite losses and the roofline object (the C1 config
  was never run by a test);
* `--gpus 2` without WORLD_SIZE -- bench.py starts its two rank processes itself (VERDICT r4
  item 2); on a one-GPU box the ranks share the device over gloo (SEG_BENCH_BACKEND=gloo), so
  the line must say n_gpus 2, a two-rank process group, and flag the roofline as invalid.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env_extra=None, timeout=400):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env,
                       capture_output=True, text=True, timeout=timeout, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.timeout(600)
def test_bench_config_c1(cuda):
    d = _bench(["--config", "C1", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                "--no-train-py", "--no-eval"])
    assert d["n_gpus"] == 1 and d["config"]["image"] == [512, 1024]
    assert d["config"]["per_gpu_batch"] == 2 and "C1" in d["config"]["workload"]
    assert "NONE" in d["config"]["workload"]          # no pyramid module (train.py's default)
    assert all(v == v and abs(v) < 1e3 for v in d["losses_last_step"])
    assert d["value"] > 0 and d["roofline"]["frac"] > 0


@pytest.mark.timeout(900)
def test_bench_self_launches_two_ranks(cuda):
    d = _bench(["--gpus", "2", "--config", "C1", "--steps", "2", "--warmup", "1", "--no-eval",
                "--no-train-py", "--no-cpu-baseline"], {"SEG_BENCH_BACKEND": "gloo"})
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["comm"]["world_size"] == 2 and d["comm"]["backend"] == "gloo"
    assert d["comm"]["allreduce_bytes_per_step"] > 0 and d["comm"]["buckets"] >= 1
    assert d["roofline"]["frac"] is None and "share" in d["roofline"]["invalid"]
    assert all(v == v for v in d["losses_last_step"])
