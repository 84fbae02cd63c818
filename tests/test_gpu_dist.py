"""Two ranks on one GPU (gloo over CUDA tensors: one card cannot host two RCCL ranks): the
bucketed all-reduce path of allreduce_grads (per-bucket events, side stream) produces the
exact mean of the two ranks' gradients, and both ranks apply the same update."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, q):
    try:
        import torch
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2",
                          RANK=str(rank))
        dist.init_process_group("gloo", rank=rank, world_size=2)
        from estimator.define_estimator_hierarchical import allreduce_grads
        from input_pipelines.synthetic import batch
        from models.initializers import init_params
        from seg_hip import SegContext
        dev = torch.device("cuda", 0)
        H, W = 64, 128
        ctx = SegContext(pyramid="psp", height=H, width=W, nb_pp=1, nb_pb=1, dtype="bf16", device=0)
        ctx.load_params(init_params(ctx.param_info, seed=1))
        d = batch(20 + rank, 1, 1, 0, H, W)
        ctx.forward(torch.as_tensor(d["images"]).to(dev))
        ctx.loss(torch.as_tensor(d["px"]).to(dev), torch.as_tensor(d["bbox"]).to(dev))
        ctx.backward()
        torch.cuda.synchronize()
        local = ctx.grads.cpu().clone()
        scale = allreduce_grads(ctx)
        ctx.apply_update(0.01, 0.9, 0.0, scale)
        torch.cuda.synchronize()
        gathered = [torch.empty_like(local) for _ in range(2)]
        dist.all_gather(gathered, local)
        exp = (gathered[0] + gathered[1]) * 0.5
        got = ctx.grads.cpu()   # the update scaled the summed buffer in place
        params = ctx.params.cpu()
        q.put((rank, float((got - exp).abs().max()), params.numpy(), len(ctx.grad_buckets())))
        ctx.close()
        dist.destroy_process_group()
    except Exception as e:  # surface worker failures in the test
        q.put((rank, repr(e), None, 0))


def test_bucketed_allreduce_two_ranks_one_gpu():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for rank, err, params, nb in res:
        assert params is not None, err
        assert nb >= 2
        assert err == 0.0, f"rank {rank}: bucketed mean differs by {err}"
    np.testing.assert_array_equal(res[0][2], res[1][2])
