"""Parity of the implicit-GEMM conv kernels (fwd / dgrad / wgrad, fp32, bf16 and fp16) against
the oracle's TF-semantics conv (torch CPU, float64). Tolerances: fp32 rel 1e-4 (exact-fp32
MFMA with a different summation order), bf16 rel 2e-2 and fp16 rel 3e-3 against a reference
fed the same rounded operands (fp32 accumulation on both sides; the output is rounded once)."""
import numpy as np
import pytest
import torch

from oracle.tfseg import ConvSpec, conv_tf

pytestmark = pytest.mark.gpu

CASES = [
    # N, H, W, Ci, Co, k, stride, rate, explicit_pad
    (2, 13, 17, 64, 64, 3, 1, 2, False),      # dilated 3x3, ragged tiles
    (2, 16, 20, 128, 256, 3, 1, 4, False),    # rate 4
    (1, 11, 9, 256, 128, 1, 1, 1, False),     # 1x1
    (2, 18, 22, 64, 64, 3, 2, 1, True),       # conv2d_same stride 2
    (1, 37, 45, 3, 64, 7, 2, 1, True),        # stem (generic small-C path)
    (2, 9, 10, 256, 14, 1, 1, 1, False),      # logits (Co=14): skinny narrow-N / narrow-K
    (1, 37, 45, 256, 7, 1, 1, 1, False),      # l2 vehicle logits, ragged 128-row stats tiles
    (2, 9, 10, 256, 3, 1, 1, 1, False),       # l2 human logits
    (1, 6, 6, 1280, 256, 1, 1, 1, False),     # PSP final (C=1280)
    (2, 15, 21, 256, 512, 1, 1, 1, False),    # short K, wide N: 128-row tiles, 2 per CU
    (1, 20, 20, 128, 256, 1, 1, 1, False),    # ping-pong tile whose second wave row is ragged (16 rows)
    # small-channel 3x3 patch kernel (8 x 32 pixel tiles, input patch staged once per chunk)
    (2, 16, 64, 64, 64, 3, 1, 1, False),      # one 64-channel chunk, Co 64
    (1, 24, 96, 128, 128, 3, 1, 1, False),    # two chunks (second patch streamed), Co 128
    (1, 8, 32, 128, 64, 3, 1, 1, False),      # two chunks, Co 64 (its dgrad: one chunk, Co 128)
    # short-K dense 1x1 on the persistent ping-pong loop (several tiles per workgroup: the next
    # tile's prologue in flight during the epilogue); the dgrad of the same case is a short-K
    # problem too where Ci > 128
    (2, 16, 32, 256, 512, 1, 1, 1, False),    # K 256 -> 512: 4 x 2 tiles, one per workgroup
    (1, 16, 16, 64, 256, 1, 1, 1, False),     # K 64: one K-tile per tile
    (1, 128, 128, 256, 1024, 1, 1, 1, False), # 256 tiles
    (1, 96, 128, 128, 768, 1, 1, 1, False),  # 288 tiles: 2 or 1 per workgroup, K 128
    (2, 64, 128, 512, 1024, 1, 1, 1, False),  # K 512, 512 tiles; its dgrad K 1024 (ping-pong)
]


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _tensors(case, seed=0):
    N, H, W, Ci, Co, k, s, r, ep = case
    g = np.random.default_rng(seed)
    x = g.standard_normal((N, H, W, Ci)).astype(np.float32)
    w = (g.standard_normal((Co, k, k, Ci)) * np.sqrt(2.0 / (k * k * Ci))).astype(np.float32)
    return x, w


def _bf16_round(a):
    return torch.as_tensor(a).to(torch.bfloat16).to(torch.float32).numpy()


TDT = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}
ABI = {"fp32": 0, "bf16": 1, "fp16": 2}
TOL = {"fp32": 1e-4, "bf16": 2e-2, "fp16": 3e-3}


def _round(a, dtype):
    return torch.as_tensor(a).to(TDT[dtype]).to(torch.float32).numpy()


def _geom(case):
    N, H, W, Ci, Co, k, s, r, ep = case
    spec = ConvSpec("t", Ci, Co, k, s, r, explicit_pad=ep)
    y = conv_tf(torch.zeros(1, Ci, H, W, dtype=torch.float64),
                torch.zeros(Co, k, k, Ci, dtype=torch.float64), spec)
    return spec, y.shape[2], y.shape[3]


def _ref_conv(x, w, spec):
    xt = torch.as_tensor(x, dtype=torch.float64).permute(0, 3, 1, 2)
    return conv_tf(xt, torch.as_tensor(w, dtype=torch.float64), spec).permute(0, 2, 3, 1).numpy()


@pytest.mark.parametrize("dtype", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("case", CASES)
def test_conv_fwd(cuda, dtype, case):
    from seg_hip import LIB, check
    N, H, W, Ci, Co, k, s, r, ep = case
    x, w = _tensors(case)
    spec, Ho, Wo = _geom(case)
    tdt = TDT[dtype]
    if dtype != "fp32":
        x, w = _round(x, dtype), _round(w, dtype)
    ref = _ref_conv(x, w, spec)
    xd = torch.as_tensor(x).to(cuda, tdt).contiguous()
    wd = torch.as_tensor(w).to(cuda, tdt).contiguous()
    # narrow outputs (the logits) live in 16-channel pixels, as the runtime lays them out
    ldy = Co if Co % 8 == 0 else (Co + 15) // 16 * 16
    yd = torch.zeros((N, Ho, Wo, ldy), dtype=tdt, device=cuda)
    M = N * Ho * Wo
    # BN partials: one per stat-rows block of the kernel the dispatcher picks (64 / 128 / 256)
    tr = LIB.seg_op_conv_stat_rows(ABI[dtype], N, H, W, Ci, Ci, Co, Co, k, s, r, int(ep))
    stats = torch.zeros(((M + tr - 1) // tr, Co, 2), dtype=torch.float32, device=cuda)
    s_ = torch.cuda.current_stream().cuda_stream
    check(LIB.seg_op_conv_fwd(ABI[dtype], xd.data_ptr(), N, H, W, Ci, Ci,
                              wd.data_ptr(), Co, k, s, r, int(ep), yd.data_ptr(), ldy,
                              stats.data_ptr(), s_))
    torch.cuda.synchronize()
    y = yd[..., :Co].float().cpu().numpy()
    tol = TOL[dtype]
    assert _rel(y, ref) < tol
    # BN partial statistics: merge (sum, M2 about the tile mean) and compare
    nt = (M + tr - 1) // tr
    st = stats.cpu().numpy().astype(np.float64)[:nt]
    cnt = np.minimum(tr, M - np.arange(nt) * tr).astype(np.float64)
    mean = st[:, :, 0].sum(0) / M
    tile_mean = st[:, :, 0] / cnt[:, None]
    m2 = st[:, :, 1].sum(0) + (cnt[:, None] * (tile_mean - mean) ** 2).sum(0)
    # fp32: against the stored output; bf16: the statistics are taken from the fp32
    # accumulators (before the bf16 rounding of the stored y), so against the fp64 reference
    # (mean error measured in units of the channel's standard deviation: means are ~0 here)
    yr = (y if dtype == "fp32" else ref).reshape(-1, Co).astype(np.float64)
    sd = np.sqrt(yr.var(0))
    assert np.linalg.norm(mean - yr.mean(0)) / np.linalg.norm(sd) < (1e-5 if dtype == "fp32" else 1e-3)
    assert _rel(m2 / M, yr.var(0)) < 1e-3


@pytest.mark.parametrize("dtype", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("case", [c for c in CASES if c[3] != 3])
def test_conv_dgrad(cuda, dtype, case):
    from seg_hip import LIB, check
    N, H, W, Ci, Co, k, s, r, ep = case
    x, w = _tensors(case)
    spec, Ho, Wo = _geom(case)
    g = np.random.default_rng(1).standard_normal((N, Ho, Wo, Co)).astype(np.float32)
    tdt = TDT[dtype]
    if dtype != "fp32":
        w, g = _round(w, dtype), _round(g, dtype)
    xt = torch.as_tensor(x, dtype=torch.float64).permute(0, 3, 1, 2).requires_grad_(True)
    y = conv_tf(xt, torch.as_tensor(w, dtype=torch.float64), spec)
    y.backward(torch.as_tensor(g, dtype=torch.float64).permute(0, 3, 1, 2))
    ref = xt.grad.permute(0, 2, 3, 1).numpy()
    wt = np.ascontiguousarray(np.flip(w, (1, 2)).transpose(3, 1, 2, 0))  # [Ci][k][k][Co] flipped
    # narrow gradients (of the logits) come in 16-channel pixels, as the runtime lays them out
    lddy = Co if Co % 8 == 0 else (Co + 15) // 16 * 16
    gp = np.zeros(g.shape[:3] + (lddy,), np.float32)
    gp[..., :Co] = g
    gd = torch.as_tensor(gp).to(cuda, tdt).contiguous()
    wtd = torch.as_tensor(wt).to(cuda, tdt).contiguous()
    dx = torch.zeros((N, H, W, Ci), dtype=tdt, device=cuda)
    check(LIB.seg_op_conv_dgrad(ABI[dtype], gd.data_ptr(), N, Ho, Wo, Co, lddy,
                                wtd.data_ptr(), Ci, k, s, r, int(ep), H, W, dx.data_ptr(), Ci,
                                torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert _rel(dx.float().cpu().numpy(), ref) < TOL[dtype]


# the identity units' data-gradient epilogue (seg_op_conv_dgrad_res): N, H, W, Co (= the
# forward conv's output channels: dy's), Ci (dx's), with residual, with the consumer's ReLU bits
RES_CASES = [
    (2, 16, 32, 256, 512, True, True),     # persistent residual launch (RQP): residual + mask (4 x 2 tiles)
    (2, 16, 32, 256, 512, True, False),    # residual only
    (1, 20, 20, 128, 256, True, True),     # ragged rows (400 pixels), K 128
    (1, 16, 16, 64, 256, False, True),     # mask only (the premasked dgrad without residual), K 64
    (2, 8, 16, 512, 2048, True, True),     # the block4 shape class: K 512 -> N 2048
    (1, 12, 20, 256, 128, True, False),    # Ci <= 128: the v2 kernel's residual epilogue
    # RQP with more tiles than CUs (506 tiles: blocks run two, the next tile's mask bytes and
    # K-tile 0 issued inside the epilogue), a ragged last row tile; K 192 = 3 K-tiles (odd: the
    # starting buffer alternates tile to tile) and K 256 (even)
    (4, 63, 257, 192, 512, True, True),
    (4, 63, 257, 256, 512, True, True),
    # ragged columns: Ci = 384 / 320 leave the last column tile half / three-quarters empty
    # (RQP reads past the row end into the next row or past the buffer, never stores there),
    # with ragged rows (640 pixels) and 3 K-tiles
    (2, 16, 32, 256, 384, True, True),
    (1, 16, 40, 192, 320, True, True),
    # the consumer's ReLU bits without a residual (one-tile launches), 506 tiles, ragged, K 192
    (4, 63, 257, 192, 512, False, True),
]


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
@pytest.mark.parametrize("case", RES_CASES)
def test_conv_dgrad_residual_masked(cuda, dtype, case):
    """dx = round(dgrad(dy) + r) (RQP: one rounding; the v2 kernel's epilogue rounds the data
    gradient first), stored with the outputs whose ReLU bit is 0 set to zero (pre-masked identity-unit gradients, staged residuals -- the identity units'
    conv1 data gradient), against a float64 restatement on the same 16-bit operands: kept
    elements at the 16-bit bound of the other op tests (L2-relative), masked-off elements exactly
    zero, the residual read in place (r aliasing dx) bitwise the same as from another buffer."""
    from seg_hip import LIB, check
    N, H, W, Co, Ci, with_r, with_m = case
    g = np.random.default_rng(7)
    dy = _round(g.standard_normal((N, H, W, Co)).astype(np.float32), dtype)
    w = _round((g.standard_normal((Co, Ci)) * np.sqrt(2.0 / Ci)).astype(np.float32), dtype)
    res = _round(g.standard_normal((N, H, W, Ci)).astype(np.float32), dtype) if with_r else None
    bits = g.integers(0, 256, size=(N, H, W, Ci // 8), dtype=np.uint8) if with_m else None
    dg = (dy.reshape(-1, Co).astype(np.float64) @ w.astype(np.float64)).reshape(N, H, W, Ci)
    tdt = TDT[dtype]
    ref = dg
    if with_r:   # the exact sum: one rounding (RQP) and two (v2) are both within the bound
        ref = dg + res
    keep = np.ones((N, H, W, Ci), bool)
    if with_m:
        keep = ((bits[..., :, None] >> np.arange(8)) & 1).astype(bool).reshape(N, H, W, Ci)
    st = torch.cuda.current_stream().cuda_stream
    dyd = torch.as_tensor(dy).to(cuda, tdt).contiguous()
    wtd = torch.as_tensor(np.ascontiguousarray(w.T)).to(cuda, tdt).contiguous()   # [Ci][Co]
    md = torch.as_tensor(bits).to(cuda).contiguous() if with_m else None
    outs = []
    for alias in ((False, True) if with_r else (False,)):
        if alias:
            dx = torch.as_tensor(res).to(cuda, tdt).contiguous()
            rd = dx
        else:
            dx = torch.full((N, H, W, Ci), 7.0, dtype=tdt, device=cuda)
            rd = torch.as_tensor(res).to(cuda, tdt).contiguous() if with_r else None
        check(LIB.seg_op_conv_dgrad_res(ABI[dtype], dyd.data_ptr(), N, H, W, Co, Co, wtd.data_ptr(), Ci,
                                        dx.data_ptr(), Ci, rd.data_ptr() if rd is not None else None, Ci,
                                        md.data_ptr() if md is not None else None, st))
        torch.cuda.synchronize()
        outs.append(dx.float().cpu().numpy())
    for got in outs:
        assert np.all(got[~keep] == 0.0)
        assert _rel(got[keep], ref[keep]) < TOL[dtype]
    if len(outs) == 2:
        assert np.array_equal(outs[0], outs[1])


@pytest.mark.parametrize("dtype", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("case", CASES)
def test_conv_wgrad(cuda, dtype, case):
    from seg_hip import LIB, check
    N, H, W, Ci, Co, k, s, r, ep = case
    # Co % 8 != 0 (the logits convs: 14 / 7 / 3 classes): the runtime pads the gradient's
    # channels and the weight-gradient rows to a multiple of 16 with zeros (net.cpp conv_wgrad,
    # co_pad); the padded rows must come out zero
    co_pad = Co if Co % 8 == 0 else (Co + 15) // 16 * 16
    x, w = _tensors(case)
    spec, Ho, Wo = _geom(case)
    g = np.random.default_rng(2).standard_normal((N, Ho, Wo, Co)).astype(np.float32)
    tdt = TDT[dtype]
    if dtype != "fp32":
        x, g = _round(x, dtype), _round(g, dtype)
    wt = torch.as_tensor(w, dtype=torch.float64).requires_grad_(True)
    y = conv_tf(torch.as_tensor(x, dtype=torch.float64).permute(0, 3, 1, 2), wt, spec)
    y.backward(torch.as_tensor(g, dtype=torch.float64).permute(0, 3, 1, 2))
    ref = wt.grad.numpy()
    xd = torch.as_tensor(x).to(cuda, tdt).contiguous()
    gp = np.zeros((N, Ho, Wo, co_pad), np.float32)
    gp[..., :Co] = g
    gd = torch.as_tensor(gp).to(cuda, tdt).contiguous()
    dw = torch.full((co_pad, k, k, Ci), float("nan"), dtype=torch.float32, device=cuda)
    ws = torch.zeros(64 << 20, dtype=torch.uint8, device=cuda)
    check(LIB.seg_op_conv_wgrad(ABI[dtype], gd.data_ptr(), N, Ho, Wo, co_pad, co_pad,
                                xd.data_ptr(), H, W, Ci, Ci, k, s, r, int(ep), dw.data_ptr(),
                                ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    dwh = dw.cpu().numpy()
    assert _rel(dwh[:Co], ref) < TOL[dtype]
    assert np.all(dwh[Co:] == 0.0)


# small-channel 3x3 stride-1 weight gradient on input patches (wgrad_patch.hip): 64-pixel row
# strips, 64-channel co / ci blocks, dilation <= 4, padding rows and columns at every border
WGRAD_PATCH_CASES = [
    (1, 8, 128, 128, 128, 3, 1, 1, False),    # 2 x 2 channel blocks, two strips per row
    (2, 6, 64, 64, 128, 3, 1, 2, False),      # rate 2, Co 128 / Ci 64
    (1, 5, 64, 128, 64, 3, 1, 4, False),      # rate 4 (widest patch), Ci 128 / Co 64
    (3, 1, 192, 64, 64, 3, 1, 1, False),      # one output row per image (all taps padded)
]


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
@pytest.mark.parametrize("case", WGRAD_PATCH_CASES)
def test_conv_wgrad_patch(cuda, dtype, case):
    from seg_hip import LIB, check
    N, H, W, Ci, Co, k, s, r, ep = case
    x, w = _tensors(case)
    spec, Ho, Wo = _geom(case)
    assert (Ho, Wo) == (H, W) and Wo % 64 == 0
    g = _round(np.random.default_rng(5).standard_normal((N, Ho, Wo, Co)).astype(np.float32), dtype)
    x = _round(x, dtype)
    wt = torch.as_tensor(w, dtype=torch.float64).requires_grad_(True)
    y = conv_tf(torch.as_tensor(x, dtype=torch.float64).permute(0, 3, 1, 2), wt, spec)
    y.backward(torch.as_tensor(g, dtype=torch.float64).permute(0, 3, 1, 2))
    ref = wt.grad.numpy()
    xd = torch.as_tensor(x).to(cuda, TDT[dtype]).contiguous()
    gd = torch.as_tensor(g).to(cuda, TDT[dtype]).contiguous()
    dw = torch.zeros((Co, k, k, Ci), dtype=torch.float32, device=cuda)
    ws = torch.zeros(64 << 20, dtype=torch.uint8, device=cuda)
    check(LIB.seg_op_conv_wgrad(ABI[dtype], gd.data_ptr(), N, Ho, Wo, Co, Co,
                                xd.data_ptr(), H, W, Ci, Ci, k, s, r, int(ep), dw.data_ptr(),
                                ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert _rel(dw.cpu().numpy(), ref) < TOL[dtype]


WGRAD_CFG_CASES = [
    # case (N, H, W, Ci, Co, k, stride, rate, explicit_pad), bm, bn, splits
    ((1, 8, 72, 256, 256, 3, 1, 2, False), 256, 256, 3),   # ping-pong, Wo >= 64 (row carries)
    ((2, 13, 17, 128, 256, 3, 1, 2, False), 256, 256, 2),  # ping-pong, Wo < 64, ragged columns
    ((1, 9, 70, 64, 320, 1, 1, 1, False), 256, 256, 4),    # ragged co tile, Ncol < 256
    ((2, 18, 132, 64, 256, 3, 2, 1, True), 256, 256, 5),   # stride-2 conv2d_same gather
    ((1, 6, 66, 256, 256, 3, 1, 4, False), 256, 256, 64),  # splits with no pixels (zero slabs)
    ((2, 13, 17, 128, 256, 3, 1, 2, False), 128, 256, 3),  # v2 configurations
    ((1, 8, 72, 256, 256, 1, 1, 1, False), 64, 128, 2),
]


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
@pytest.mark.parametrize("case,bm,bn,splits", WGRAD_CFG_CASES)
def test_conv_wgrad_cfg(cuda, case, bm, bn, splits, dtype):
    """bf16 weight gradient at an explicit tile / split configuration (every kernel the
    runtime can pick, reached at test sizes), vs float64 on the same bf16 operands."""
    from seg_hip import LIB, check
    N, H, W, Ci, Co, k, s, r, ep = case
    x, w = _tensors(case)
    spec, Ho, Wo = _geom(case)
    g = _round(np.random.default_rng(3).standard_normal((N, Ho, Wo, Co)).astype(np.float32), dtype)
    x = _round(x, dtype)
    wt = torch.as_tensor(w, dtype=torch.float64).requires_grad_(True)
    y = conv_tf(torch.as_tensor(x, dtype=torch.float64).permute(0, 3, 1, 2), wt, spec)
    y.backward(torch.as_tensor(g, dtype=torch.float64).permute(0, 3, 1, 2))
    ref = wt.grad.numpy()
    xd = torch.as_tensor(x).to(cuda, TDT[dtype]).contiguous()
    gd = torch.as_tensor(g).to(cuda, TDT[dtype]).contiguous()
    dw = torch.zeros((Co, k, k, Ci), dtype=torch.float32, device=cuda)
    ws = torch.full((splits * Co * k * k * Ci,), float("nan"), dtype=torch.float32, device=cuda)
    check(LIB.seg_op_conv_wgrad_cfg(ABI[dtype], gd.data_ptr(), N, Ho, Wo, Co, Co, xd.data_ptr(), H, W, Ci,
                                    Ci, k, s, r, int(ep), dw.data_ptr(), ws.data_ptr(),
                                    ws.numel() * 4, bm, bn, splits,
                                    torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert _rel(dw.cpu().numpy(), ref) < TOL[dtype]
