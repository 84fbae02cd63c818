"""Gradient all-reduce buckets (seg_grad_buckets / seg_stream_wait_bucket): the ranges tile
the flat buffer exactly once, follow the backward's write order, and each bucket's event
fires only after its gradients are final (a side stream that waits on it copies the final
values while the rest of the backward is still running)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_buckets_tile_the_buffer_and_fire_after_their_gradients(cuda):
    from input_pipelines.synthetic import batch
    from models.initializers import init_params
    from seg_hip import SegContext
    H, W = 128, 256
    ctx = SegContext(pyramid="aspp", height=H, width=W, nb_pp=2, dtype="bf16")
    ctx.load_params(init_params(ctx.param_info, seed=3))
    d = batch(9, 2, 0, 0, H, W)
    img, px = torch.as_tensor(d["images"]).to(cuda), torch.as_tensor(d["px"]).to(cuda)
    buckets = ctx.grad_buckets()
    n = ctx.grads.numel()
    cover = np.zeros(n, np.int32)
    for lo, hi in buckets:
        assert 0 <= lo < hi <= n
        cover[lo:hi] += 1
    assert np.all(cover == 1)
    assert len(buckets) >= 2
    # weight buckets come top-down (the backward visits the last layers first)
    wl = [lo for lo, _ in buckets[:-1]]
    assert wl == sorted(wl, reverse=True)
    side = torch.cuda.Stream(cuda)
    for trial in range(2):
        ctx.grads.fill_(float("nan"))
        ctx.forward(img)
        ctx.loss(px)
        ctx.backward()
        copies = []
        for i, (lo, hi) in enumerate(buckets):
            ctx.wait_bucket(i, side)
            with torch.cuda.stream(side):
                copies.append(ctx.grads[lo:hi].clone())
        torch.cuda.synchronize()
        for (lo, hi), c in zip(buckets, copies):
            assert torch.equal(c, ctx.grads[lo:hi]), f"bucket [{lo},{hi}) copied before its event"
        assert torch.isfinite(ctx.grads).all()
    ctx.close()
