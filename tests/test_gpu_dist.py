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


SYNC_H, SYNC_W = 64, 128


def _sync_worker(rank, port, q):
    """One replica of a cross-replica-BN step (fp32): forward / loss / backward with the BN
    moments and gradient means exchanged through seg_set_bn_sync (gloo on the device
    tensors), then the averaged gradient and the update."""
    try:
        import torch
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2",
                          RANK=str(rank))
        dist.init_process_group("gloo", rank=rank, world_size=2)
        from estimator.define_estimator_hierarchical import allreduce_grads
        from input_pipelines.synthetic import batch
        from oracle.tfseg import SegConfig, init_params
        from seg_hip import SegContext
        dev = torch.device("cuda", 0)
        cfg = SegConfig(height=SYNC_H, width=SYNC_W, nb_pp=1, nb_pb=1, pyramid="psp")
        params = {k: v.astype(np.float32) for k, v in init_params(cfg, seed=3).items()}
        ctx = SegContext(pyramid="psp", height=SYNC_H, width=SYNC_W, nb_pp=1, nb_pb=1,
                         dtype="fp32", device=0)
        ctx.load_params(params)
        ctx.set_bn_sync()
        d = batch(40 + rank, 1, 1, 0, SYNC_H, SYNC_W)
        ctx.forward(torch.as_tensor(d["images"]).to(dev))
        ctx.loss(torch.as_tensor(d["px"]).to(dev), torch.as_tensor(d["bbox"]).to(dev))
        ctx.backward()
        losses, _, _ = ctx.outputs()
        lv = losses.cpu().numpy()[:4].copy()
        scale = allreduce_grads(ctx)
        ctx.apply_update(0.01, 0.9, 0.0, scale)
        torch.cuda.synchronize()
        q.put((rank, lv, ctx.named("grads"), ctx.named("params"), None))
        ctx.set_bn_sync(1)
        ctx.close()
        dist.destroy_process_group()
    except Exception as e:
        import traceback
        q.put((rank, None, None, None, traceback.format_exc() + repr(e)))


def test_cross_replica_bn_two_ranks_matches_oracle():
    """--cross_replica_norm over two replicas (one GPU, gloo) against the oracle's
    train_step_replicas (BN over both sub-batches, per-replica loss normalisation, gradient of
    the replica mean): per-replica losses 1e-3, averaged gradients with the conditioning-aware
    bound of test_gpu_step.test_train_step_fp32, moving statistics 1e-3."""
    import torch
    import torch.multiprocessing as mp
    from input_pipelines.synthetic import batch
    from oracle.tfseg import OracleNet, SegConfig, init_params
    mctx = mp.get_context("spawn")
    q = mctx.Queue()
    port = _free_port()
    procs = [mctx.Process(target=_sync_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[4] is None, r[4]
    cfg = SegConfig(height=SYNC_H, width=SYNC_W, nb_pp=1, nb_pb=1, pyramid="psp")
    params = {k: v.astype(np.float32) for k, v in init_params(cfg, seed=3).items()}
    batches = [batch(40 + r, 1, 1, 0, SYNC_H, SYNC_W) for r in range(2)]
    Ls, g, newp, _, _ = OracleNet(cfg, params).train_step_replicas(batches)
    _, g32, _, _, _ = OracleNet(cfg, params, dtype=torch.float32).train_step_replicas(batches)

    def rel(a, b):
        a, b = np.asarray(a, np.float64).reshape(-1), np.asarray(b, np.float64).reshape(-1)
        return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
    for r in range(2):
        ref = [float(Ls[r][k]) for k in ("segmentation", "l1_segmentation",
                                         "l2_vehicle_segmentation", "l2_human_segmentation")]
        np.testing.assert_allclose(res[r][1], ref, rtol=1e-3, atol=1e-6)
    # both replicas hold the same averaged gradient and the same parameters
    for k in g:
        np.testing.assert_array_equal(res[0][2][k], res[1][2][k])
    for k in res[0][3]:
        np.testing.assert_array_equal(res[0][3][k], res[1][3][k])
    errs = {k: rel(res[0][2][k], g[k].numpy()) for k in g}
    cond = {k: rel(g32[k].numpy(), g[k].numpy()) for k in g}
    bad = [(errs[k], cond[k], k) for k in g
           if errs[k] > (max(1e-3, 4 * cond[k]) if cond[k] < 1e-3 else max(5e-2, 2 * cond[k]))]
    nrm = {k: (float(np.linalg.norm(res[0][2][k])), float(g[k].norm()), float(g32[k].norm()))
           for _, _, k in bad}
    assert not bad, (sorted(bad, reverse=True)[:10], nrm)
    for k, v in newp.items():
        if "moving" in k:
            assert rel(res[0][3][k], v.detach().numpy()) < 1e-3, k


DP4_H, DP4_W, DP4_WORLD = 64, 128, 4


def _dp4_worker(rank, port, tmp, q):
    """One rank of `train.py --distribute` at world size 4 (gloo over CUDA tensors: one GPU
    cannot host four RCCL ranks) with the reference's global 4 : 8 : 4 pixel : bbox : tag batch
    (train.py:62-64), one fp32 step at 64 x 128: records this rank's sub-batch, loss terms and
    counts, weak l1 decisions, and the state after the update."""
    try:
        import torch
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                          WORLD_SIZE=str(DP4_WORLD), RANK=str(rank), LOCAL_RANK="0")
        dist.init_process_group("gloo", rank=rank, world_size=DP4_WORLD)
        import train
        import estimator.define_estimator_hierarchical as deh
        from models import resnet50_extended_model_hierarchical as mh
        seen = []
        orig = deh.define_losses

        def wrapped(mode, predictions, labels, config, params):
            L = orig(mode, predictions, labels, config, params)
            ctx = predictions['_context']
            lv = ctx.outputs()[0].cpu().numpy()[:4].copy()
            d1 = predictions['l1_decisions'][ctx.cfg.nb_pp:].cpu().numpy().astype(np.int64)
            seen.append(((ctx.cfg.nb_pp, ctx.cfg.nb_pb, ctx.cfg.nb_pi), lv, L.counts(), d1,
                         int(config.train_distribute.num_towers)))
            return L
        deh.define_losses = wrapped
        argv = [os.path.join(tmp, "logs"), "cityscapes", "--max_steps", "1", "--compute_dtype", "fp32",
                "--height_feature_extractor", str(DP4_H), "--width_feature_extractor", str(DP4_W),
                "--Nb_per_pixel", "4", "--Nb_per_bbox", "8", "--Nb_per_image", "4",
                "--learning_rate_initial", "1e-3", "--save_summaries_steps", "1",
                "--save_checkpoints_steps", "100", "--distribute"]
        assert train.main(argv) == 1
        ctx = next(iter(mh._CONTEXTS.values()))
        torch.cuda.synchronize()
        tail = ctx.grads[ctx.n_train:].cpu().numpy().copy()   # averaged BN batch statistics
        q.put((rank, seen, ctx.named("params"), tail, None))
        mh.release_contexts()
        dist.destroy_process_group()
    except Exception as e:
        import traceback
        q.put((rank, None, None, None, traceback.format_exc() + repr(e)))


def test_four_ranks_mixed_batch_matches_oracle(tmp_path):
    """MirroredStrategy semantics at world size 4 with the reference's
    mixed batch, through the drop-in trainer. Each rank must take Nb/4 of EVERY sub-batch
    (get_temp_Nb per stream, input_pipelines/utils.py:118-125: 1 strong + 2 bbox + 1 tag),
    normalise its losses by its own non-zero-weight counts (define_losses per tower), and
    the step must apply the MEAN of the four per-rank gradients and of the four per-rank BN
    batch statistics (the moving averages' input). Checked against the oracle run with the
    identical sharding: each rank's shard through OracleNet (same seeds as
    train.synthetic_train_input, same weak-weight mask as the native rank), then the mean.
    Tolerances: per-rank losses 1e-3 and counts exact; the parameter change and the averaged
    statistics tail L2-relative max(1e-2, 3x) / max(1e-3, 4x) the fp32 oracle's own gap."""
    import torch
    import torch.multiprocessing as mp
    from input_pipelines.synthetic import batch
    from oracle.tfseg import OracleNet, SegConfig, init_params
    mctx = mp.get_context("spawn")
    q = mctx.Queue()
    port = _free_port()
    procs = [mctx.Process(target=_dp4_worker, args=(r, port, str(tmp_path / f"r{r}"), q))
             for r in range(DP4_WORLD)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[4] is None, r[4]
    for rank, seen, _, _, _ in res:
        assert len(seen) == 1 and seen[0][0] == (1, 2, 1) and seen[0][4] == DP4_WORLD, (rank, seen)
    # every rank applied the same averaged update
    for k in res[0][2]:
        for r in range(1, DP4_WORLD):
            np.testing.assert_array_equal(res[0][2][k], res[r][2][k])
    np.testing.assert_array_equal(res[0][3], res[1][3])

    cfg = SegConfig(height=DP4_H, width=DP4_W, nb_pp=1, nb_pb=2, nb_pi=1, pyramid="none")
    p0 = {k: v.astype(np.float32) for k, v in init_params(cfg, seed=0).items()}

    from test_gpu_train import _gate_flips   # tests/ is on sys.path (pytest's prepend mode)
    flips = []

    def oracle(dtype):
        losses, counts, grads, stats = [], [], [], []
        for r in range(DP4_WORLD):
            d = batch(1000003 * r, 1, 2, 1, DP4_H, DP4_W)   # train.synthetic_train_input, rank r
            net = OracleNet(cfg, {k: v.astype(np.float64) for k, v in p0.items()}, dtype=dtype)
            L, low, g, _, _, _, st = net.train_step(d["images"], d["px"], d["bbox"], d["tag"],
                                                    lr=1e-3, weak_l1_decisions=res[r][1][0][3])
            if dtype == torch.float64:   # the oracle's own l1 gate vs the native rank's
                flips.append(_gate_flips(net, {q_: v.detach() for q_, v in low.items()},
                                         np.concatenate([d["bbox"], d["tag"]]), res[r][1][0][3], 1))
            losses.append([float(L[n]) for n in ("segmentation", "l1_segmentation",
                                                  "l2_vehicle_segmentation", "l2_human_segmentation")])
            counts.append(tuple(int(c) for c in L["counts"]))
            grads.append({k: v.detach().numpy() for k, v in g.items()})
            stats.append({k: (m.detach().numpy(), v.detach().numpy()) for k, (m, v) in st.items()})
        g = {k: sum(gr[k] for gr in grads) / DP4_WORLD for k in grads[0]}
        st = {k: (sum(s[k][0] for s in stats) / DP4_WORLD, sum(s[k][1] for s in stats) / DP4_WORLD)
              for k in stats[0]}
        # step 0 of MomentumOptimizer: accum = g + wd * w; w -= lr * accum
        new_p = {k: p0[k] - 1e-3 * (g[k] + (cfg.weight_decay * p0[k] if k.endswith("/weights") else 0.0))
                 for k in g}
        return losses, counts, new_p, st

    ref_l, ref_c, ref_p, ref_s = oracle(torch.float64)
    _, _, p32, s32 = oracle(torch.float32)
    for r in range(DP4_WORLD):
        np.testing.assert_allclose(res[r][1][0][1], ref_l[r], rtol=1e-3, atol=1e-6, err_msg=f"rank {r}")
        assert tuple(res[r][1][0][2]) == ref_c[r], (r, res[r][1][0][2], ref_c[r])
    # the weak-weight gate itself (as test_gpu_train): the oracle's own l1 argmax moves at most
    # 0.1 % of a weak image's pixels in or out of a head's weights on every rank
    assert len(flips) == DP4_WORLD
    assert all(int(f.max()) <= max(2, DP4_H * DP4_W // 1000) for f in flips), flips
    # per-rank normalisation is not the global one: the ranks' counts differ
    assert len(set(ref_c)) > 1

    def rel(a, b):
        a, b = np.asarray(a, np.float64).reshape(-1), np.asarray(b, np.float64).reshape(-1)
        return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
    keys = sorted(ref_p)
    flat = lambda d: np.concatenate([np.asarray(d[k], np.float64).reshape(-1) for k in keys])
    w0 = flat(p0)
    err = rel(flat(res[0][2]) - w0, flat(ref_p) - w0)
    gap = rel(flat(p32) - w0, flat(ref_p) - w0)
    assert err < max(1e-2, 3 * gap), (err, gap)
    # the statistics tail (moving-buffer layout): rank-mean of the batch means / variances
    info = {}
    for k, (m, v) in ref_s.items():
        info[f"{k}/BatchNorm/moving_mean"] = m
        info[f"{k}/BatchNorm/moving_variance"] = v
    info32 = {}
    for k, (m, v) in s32.items():
        info32[f"{k}/BatchNorm/moving_mean"] = m
        info32[f"{k}/BatchNorm/moving_variance"] = v
    tail = res[0][3]
    offs = _moving_offsets(cfg)
    got = np.concatenate([tail[offs[k][0]:offs[k][0] + offs[k][1]] for k in sorted(info)])
    exp = np.concatenate([np.asarray(info[k]).reshape(-1) for k in sorted(info)])
    e32 = np.concatenate([np.asarray(info32[k]).reshape(-1) for k in sorted(info)])
    assert rel(got, exp) < max(1e-3, 4 * rel(e32, exp)), (rel(got, exp), rel(e32, exp))


def _moving_offsets(cfg):
    """name -> (offset, numel) of the moving statistics in the context's moving buffer (the
    layout of the gradient buffer's statistics tail), from a throw-away context."""
    from seg_hip import SegContext
    ctx = SegContext(pyramid="none", height=cfg.height, width=cfg.width, nb_pp=cfg.nb_pp,
                     nb_pb=cfg.nb_pb, nb_pi=cfg.nb_pi, dtype="fp32")
    out = {p.name: (p.offset, p.numel) for p in ctx.param_info
           if p.kind in ("moving_mean", "moving_variance")}
    ctx.close()
    return out


def test_train_distribute_launches_its_own_ranks(tmp_path):
    """`train.py ... --distribute` with no launcher starts its ranks itself
    (utils/launch.spawn_ranks, as the reference's MirroredStrategy takes every visible GPU in one
    launch, system_factory.py:276-283). Two ranks share this box's one GPU over gloo
    (SEG_TRAIN_RANKS=2, SEG_TRAIN_BACKEND=gloo; one card cannot host two RCCL ranks), one fp32
    step at 64 x 128 with the global batch of 4 per-pixel images (2 per rank). Checked: the run
    exits 0; rank 0's console log and rank 1's <log_dir>/rank1.log carry each rank's own loss
    terms, equal to the oracle on that rank's shard (train.synthetic_train_input's seeds) at
    1e-3 (4-decimal log values); rank 0's checkpoint holds the mean of the two ranks' updates
    (step 0 of MomentumOptimizer and the BN moving averages are linear in the gradient and the
    batch statistics, so the expected state is the mean of the per-rank oracle updates) at
    max(1e-2, 3 x the fp32 oracle's gap) for the parameter change and max(1e-3, 4 x) for the
    moving statistics. A failing rank fails the run: test_host.py covers that on the CPU."""
    import re
    import subprocess
    import sys
    import torch
    from input_pipelines.synthetic import batch
    from oracle.tfseg import OracleNet, SegConfig, init_params
    H, W, NPP, LR = 64, 128, 4, 1e-3
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    train_py = os.path.join(repo, "iv2019-boosting-semantic-segmentation-with-weak-labels_amd", "train.py")
    log_dir = str(tmp_path / "logs")
    env = dict(os.environ, SEG_TRAIN_RANKS="2", SEG_TRAIN_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, train_py, log_dir, "cityscapes", "--max_steps", "1",
                        "--compute_dtype", "fp32", "--height_feature_extractor", str(H),
                        "--width_feature_extractor", str(W), "--Nb_per_pixel", str(NPP),
                        "--Nb_per_bbox", "0", "--Nb_per_image", "0", "--learning_rate_initial", str(LR),
                        "--save_summaries_steps", "1", "--save_checkpoints_steps", "100", "--distribute"],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    pat = r"step 1: total ([-\d.]+) l1 ([-\d.]+) l2v ([-\d.]+) l2h ([-\d.]+)"
    logs = [r.stdout, open(os.path.join(log_dir, "rank1.log")).read()]
    assert "training 1 steps on 2 GPU(s)" in r.stdout, r.stdout
    got = [np.array([float(v) for v in re.findall(pat, t)[0]]) for t in logs]
    state = torch.load(os.path.join(log_dir, "model.ckpt-1.pt"), weights_only=True)
    assert state["global_step"] == 1 and "ema" not in state   # --distribute drops the EMA
    nat = {k: v.numpy() for k, v in state["params"].items()}

    cfg = SegConfig(height=H, width=W, nb_pp=NPP // 2, pyramid="none")
    p0 = {k: v.astype(np.float32) for k, v in init_params(cfg, seed=0).items()}

    def oracle(dtype):
        losses, news = [], []
        for rank in range(2):
            d = batch(1000003 * rank, NPP // 2, 0, 0, H, W)   # train.synthetic_seed(rank, 0)
            net = OracleNet(cfg, {k: v.astype(np.float64) for k, v in p0.items()}, dtype=dtype)
            L, _, _, new_p, _, _, _ = net.train_step(d["images"], d["px"], lr=LR)
            losses.append(np.array([float(L[n]) for n in ("total", "l1_segmentation",
                                                           "l2_vehicle_segmentation", "l2_human_segmentation")]))
            news.append({k: v.detach().numpy() for k, v in new_p.items()})
        return losses, {k: (news[0][k] + news[1][k]) / 2 for k in news[0]}

    ref_l, ref_p = oracle(torch.float64)
    _, p32 = oracle(torch.float32)
    for rank in range(2):
        np.testing.assert_allclose(got[rank], ref_l[rank], rtol=1e-3, atol=1e-4, err_msg=f"rank {rank}")
    assert not np.allclose(ref_l[0], ref_l[1])   # the ranks trained on different shards

    def rel(a, b):
        return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
    trained = sorted(k for k in ref_p if "moving" not in k)
    moving = sorted(k for k in ref_p if "moving" in k)
    flat = lambda d, ks: np.concatenate([np.asarray(d[k], np.float64).reshape(-1) for k in ks])
    w0 = flat(p0, trained)
    err = rel(flat(nat, trained) - w0, flat(ref_p, trained) - w0)
    gap = rel(flat(p32, trained) - w0, flat(ref_p, trained) - w0)
    assert err < max(1e-2, 3 * gap), (err, gap)
    err_m = rel(flat(nat, moving), flat(ref_p, moving))
    gap_m = rel(flat(p32, moving), flat(ref_p, moving))
    assert err_m < max(1e-3, 4 * gap_m), (err_m, gap_m)
