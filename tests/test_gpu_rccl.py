"""The production collective path on real RCCL. A one-GPU box cannot host
two RCCL ranks, but a one-rank `nccl` process group is legal and runs every piece the 8-GPU
bench uses: the communicator, the bucketed all-reduce on the comm stream waiting on the
backward's bucket events (define_estimator_hierarchical.allreduce_grads, forced at n = 1), and
the cross-replica BN hook (seg_set_bn_sync) issuing RCCL all-reduces ordered on the step's
stream. Reference: code/system_factory.py:279-295 (MirroredStrategy / NCCL),
code/utils/cross_replica_batch_normalization.py:398-424 (merge_call sum).

A SUM over one rank is the identity, so:
* a bf16 step through the RCCL bucketed all-reduce is bitwise the collective-free step
  (gradients, parameters, momentum, moving statistics);
* a cross-replica-BN step whose hook runs on RCCL is bitwise the same step whose hook runs on
  gloo (same arithmetic, only the transport differs).
Each case runs in a fresh spawned process (no GPU state inherited from the test runner)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

H, W = 128, 256


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _step(ctx, d, dev, collective):
    import torch
    from estimator.define_estimator_hierarchical import allreduce_grads
    ctx.forward(torch.as_tensor(d["images"]).to(dev))
    ctx.loss(torch.as_tensor(d["px"]).to(dev), torch.as_tensor(d["bbox"]).to(dev))
    ctx.backward()
    if collective:
        scale = allreduce_grads(ctx, always=True)
        assert scale == 1.0
    else:
        scale = 1.0
    ctx.apply_update(0.01, 0.9, 0.0, scale)
    torch.cuda.synchronize()
    losses, _, _ = ctx.outputs()
    return {"losses": losses.cpu().numpy().copy(), "grads": ctx.grads.cpu().numpy().copy(),
            "params": ctx.params.cpu().numpy().copy(), "momentum": ctx.momentum.cpu().numpy().copy(),
            "moving": ctx.moving.cpu().numpy().copy()}


def _rccl_worker(port, q):
    try:
        import torch
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="1", RANK="0")
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        assert dist.get_backend() == "nccl"
        gloo = dist.new_group(backend="gloo")
        from input_pipelines.synthetic import batch
        from models.initializers import init_params
        from seg_hip import SegContext
        d = batch(31, 1, 1, 0, H, W)
        out = {}
        for name, dtype, collective, sync in (("plain", "bf16", False, None),
                                              ("rccl", "bf16", True, None),
                                              ("sync_rccl", "fp32", True, "nccl"),
                                              ("sync_gloo", "fp32", True, "gloo")):
            ctx = SegContext(pyramid="psp", height=H, width=W, nb_pp=1, nb_pb=1, dtype=dtype, device=0)
            ctx.load_params(init_params(ctx.param_info, seed=4))
            if sync is not None:
                ctx.set_bn_sync(group=None if sync == "nccl" else gloo, always=True)
            buckets = len(ctx.grad_buckets())
            out[name] = _step(ctx, d, dev, collective)
            out[name]["buckets"] = buckets
            if sync is not None:
                ctx.set_bn_sync(1)
            ctx.close()
        # the comm stream the bucketed path created really issued RCCL work: one more
        # all-reduce on a device tensor must succeed on the same communicator
        t = torch.ones(4, device=dev)
        dist.all_reduce(t)
        torch.cuda.synchronize()
        out["check"] = float(t.sum())
        dist.destroy_process_group()
        q.put((out, None))
    except Exception as e:
        import traceback
        q.put((None, traceback.format_exc() + repr(e)))


def test_rccl_one_rank_bucketed_allreduce_and_sync_bn():
    import torch.multiprocessing as mp
    mctx = mp.get_context("spawn")
    q = mctx.Queue()
    p = mctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    out, err = q.get(timeout=240)
    p.join(timeout=60)
    assert err is None, err
    assert out["check"] == 4.0
    assert out["rccl"]["buckets"] >= 2
    for k in ("losses", "grads", "params", "momentum", "moving"):
        np.testing.assert_array_equal(out["rccl"][k], out["plain"][k], err_msg=k)
    for k in ("losses", "grads", "params", "momentum", "moving"):
        np.testing.assert_array_equal(out["sync_rccl"][k], out["sync_gloo"][k], err_msg=k)
    assert np.all(np.isfinite(out["sync_rccl"]["losses"]))
