"""Parity at the benchmark's shapes (BASELINE config C2: R50 + ASPP, 1024 x 2048, 4 images per
GPU, bf16 storage / fp32 accumulation), through the production dispatch.

At these sizes every conv runs the kernels the bench times: the persistent ping-pong NT loop
(more 256 x 256 tiles than CUs, so each workgroup walks several tiles with the next tile's
DMA in flight during the epilogue), the non-persistent residual dgrad launches, the split-K
weight gradient with large pixel counts (op entry: ~2 waves of workgroups; in the step: the
side-stream sizing beside the dgrad -> BN chain), the v2 kernels for Co <= 128, the tap8
stem and the transposed-stride dgrad.

* ``test_conv_c2_layer`` — single layers through ``seg_op_conv_fwd / _dgrad / _wgrad``,
  every output element against the oracle's ``conv_tf`` on the CPU (float32 accumulation of
  the same bf16 / fp16 operands; the convolution of ``resnet50_extended_feature_extractor.py:
  25-30`` / ``hierarchical.py:59-64`` at the C2 layer shapes).
* ``test_step_layerwise_fullsize`` — one full training step (C2, C4, C5) of the native context, then every
  conv's forward output and weight gradient, and the whole backward chain of the data
  gradients (dgrad -> ReLU mask -> BN backward, residual and strided-subsample shortcuts,
  the ASPP transposes, the stem max-pool), against a float64 restatement fed the tensors the
  native step itself consumed (``oracle/conv_props.py``, pinned to ``conv_tf`` and autograd by
  ``tests/test_oracle.py``); plus the loss terms and fused decisions of the loss head against
  ``OracleNet.losses`` / ``head_predictions`` on the native low-resolution logits.

Tolerances (written per check below):
* 16-bit outputs (forward y, data gradients of the op tests): per element
  |got - ref| <= 2u |ref| + 1e-3 rms(ref), u = 2^-8 (bf16) / 2^-11 (fp16) — one rounding of
  the fp32 accumulator plus summation-order noise; any missing tap, K-chunk or tile breaks it.
* fp32 weight gradients: per element |got - ref| <= 1e-3 |ref| + 1e-4 rms(ref), plus in the
  step 2^-24 sqrt(P) sum_p |dy x| (an fp32 sum over P pixels is off by ~sqrt(P) ulps of the
  absolute sum where the signed sum cancels; a missing 64-pixel K-step is ~20x that).
* BN-backward outputs of the step (dy of every conv): L2-relative 2e-2 over the tensor and
  5e-2 over every 256-pixel tile (bf16 dgrad outputs feed a cancelling formula: dh minus its
  mean and its x-hat projection).
"""
import math

import numpy as np
import pytest
import torch

from oracle.conv_props import conv_dgrad, conv_fwd, conv_wgrad
from oracle.tfseg import BN_EPS, ConvSpec, OracleNet, SegConfig, build_specs, conv_tf, init_params, resnet_units

pytestmark = pytest.mark.gpu

TDT = {"bf16": torch.bfloat16, "fp16": torch.float16}
ABI = {"bf16": 1, "fp16": 2}
ULP = {"bf16": 2.0 ** -8, "fp16": 2.0 ** -11}


def _elementwise(got, ref, rtol, atol_rms, what, absref=None, n_sum=0):
    """|got - ref| <= rtol |ref| + atol_rms rms(ref) [+ 2^-24 sqrt(n_sum) absref]: absref =
    the same sum over |terms| (an fp32 sum of n_sum terms in any order is off by ~sqrt(n) ulps
    of the absolute sum, which matters where the signed sum cancels)."""
    got = got.double()
    ref = ref.double().to(got.device)
    rms = float(ref.pow(2).mean().sqrt())
    bound = rtol * ref.abs() + atol_rms * rms
    if absref is not None:
        bound = bound + 2.0 ** -24 * math.sqrt(n_sum) * absref
    excess = (got - ref).abs() / bound
    nbad = int((excess > 1).sum())
    assert nbad == 0, f"{what}: {nbad} of {ref.numel()} elements out of tolerance " \
                      f"(worst {float(excess.max()):.3g}x the bound)"


def _tiles(got, ref, tol, tile_tol, what, rows=256):
    """L2-relative over the tensor and over every `rows`-pixel tile of the NHWC pixel order."""
    C = ref.shape[-1]
    g = got.double().reshape(-1, C)
    r = ref.double().reshape(-1, C).to(g.device)
    rel = float((g - r).norm() / r.norm().clamp_min(1e-300))
    assert rel < tol, f"{what}: rel {rel:.3g}"
    M = r.shape[0]
    pad = (-M) % rows
    e2 = torch.nn.functional.pad((g - r).pow(2).sum(1), (0, pad)).reshape(-1, rows).sum(1)
    r2 = torch.nn.functional.pad(r.pow(2).sum(1), (0, pad)).reshape(-1, rows).sum(1)
    floor = 1e-2 * float(r2.mean())   # tiles the ReLU mask zeroed almost entirely
    trel = (e2 / r2.clamp_min(floor)).sqrt()
    worst = int(trel.argmax())
    assert float(trel[worst]) < tile_tol, f"{what}: tile {worst} of {len(trel)} rel {float(trel[worst]):.3g}"


# ------------------------------------------------------------------------- single layers
C2_LAYERS = [
    # name, N, H, W, Ci, Co, k, stride, rate, explicit_pad
    ("block4_conv2_r4", 4, 128, 256, 512, 512, 3, 1, 4, False),
    ("block3_conv2_r2", 4, 128, 256, 256, 256, 3, 1, 2, False),
    ("block4_conv3_1x1_co2048", 4, 128, 256, 512, 2048, 1, 1, 1, False),
    ("block4_conv1_1x1_ci2048", 4, 128, 256, 2048, 512, 1, 1, 1, False),
    ("aspp_conv_r18", 4, 128, 256, 256, 256, 3, 1, 18, False),
    ("block1_conv2_s2", 4, 256, 512, 64, 64, 3, 2, 1, True),
    ("block2_conv1_co128", 4, 128, 256, 256, 128, 1, 1, 1, False),
    # the small-channel 3x3 patch kernel (conv_v2.hip conv_nt_patch_kernel): forward and the
    # stride-1 data gradient of block1 / block2 conv2
    ("block1_conv2_c64", 4, 256, 512, 64, 64, 3, 1, 1, False),
    ("block2_conv2_c128", 4, 128, 256, 128, 128, 3, 1, 1, False),
    ("l1_logits_co14", 4, 128, 256, 256, 14, 1, 1, 1, False),
]
LAYER_DTYPES = [(c, "bf16") for c in C2_LAYERS] + [(C2_LAYERS[0], "fp16"), (C2_LAYERS[2], "fp16"),
                                                    (C2_LAYERS[9], "fp16")]


def _operands(case, dtype, seed):
    _, N, H, W, Ci, Co, k, s, r, ep = case
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, H, W, Ci, generator=g).to(TDT[dtype])
    w = (torch.randn(Co, k, k, Ci, generator=g) * math.sqrt(2.0 / (k * k * Ci))).to(TDT[dtype])
    return x, w


def _cpu_conv(x, w, spec):
    """oracle conv_tf in float32 on the CPU (NHWC in / out)."""
    return conv_tf(x.float().permute(0, 3, 1, 2), w.float(), spec).permute(0, 2, 3, 1)


@pytest.mark.parametrize("case,dtype", LAYER_DTYPES, ids=lambda v: v[0] if isinstance(v, tuple) else v)
def test_conv_c2_layer(cuda, case, dtype):
    from seg_hip import LIB, check
    name, N, H, W, Ci, Co, k, s, r, ep = case
    spec = ConvSpec(name, Ci, Co, k, s, r, explicit_pad=ep)
    x, w = _operands(case, dtype, 0)
    st = torch.cuda.current_stream().cuda_stream
    # ---- forward (+ the epilogue's BN partial statistics)
    ref = _cpu_conv(x, w, spec)
    Ho, Wo = ref.shape[1], ref.shape[2]
    M = N * Ho * Wo
    xd, wd = x.to(cuda), w.to(cuda)
    yd = torch.empty((N, Ho, Wo, Co), dtype=TDT[dtype], device=cuda)
    # BN partials: one per stat-rows block of the kernel the dispatcher picks (64 / 128 / 256)
    tr = LIB.seg_op_conv_stat_rows(ABI[dtype], N, H, W, Ci, Ci, Co, Co, k, s, r, int(ep))
    stats = torch.zeros(((M + tr - 1) // tr, Co, 2), dtype=torch.float32, device=cuda)
    check(LIB.seg_op_conv_fwd(ABI[dtype], xd.data_ptr(), N, H, W, Ci, Ci, wd.data_ptr(), Co, k, s, r,
                              int(ep), yd.data_ptr(), Co, stats.data_ptr(), st))
    torch.cuda.synchronize()
    refd = ref.to(cuda)
    _elementwise(yd, refd, 2 * ULP[dtype], 1e-3, f"{name} fwd")
    nt = (M + tr - 1) // tr
    sp = stats[:nt].double()
    cnt = torch.clamp(M - torch.arange(nt, device=cuda) * tr, max=tr).double()
    mean = sp[:, :, 0].sum(0) / M
    m2 = sp[:, :, 1].sum(0) + (cnt[:, None] * (sp[:, :, 0] / cnt[:, None] - mean) ** 2).sum(0)
    r64 = refd.double().reshape(-1, Co)
    sd = r64.std(0, unbiased=False)
    assert float(((mean - r64.mean(0)).abs() / sd).max()) < 1e-3, f"{name} BN mean"
    assert float(((m2 / M) / r64.var(0, unbiased=False) - 1).abs().max()) < 1e-3, f"{name} BN var"
    del yd, refd, r64, stats
    # ---- data gradient (the runtime passes the spatially flipped, transposed weights)
    g = torch.Generator().manual_seed(1)
    dy = torch.randn(N, Ho, Wo, Co, generator=g).to(TDT[dtype])
    xt = torch.zeros(N, Ci, H, W, requires_grad=True)
    conv_tf(xt, w.float(), spec).backward(dy.float().permute(0, 3, 1, 2))
    ref = xt.grad.permute(0, 2, 3, 1)
    wt = torch.flip(w, (1, 2)).permute(3, 1, 2, 0).contiguous()   # [Ci][k][k][Co]
    dyd, wtd = dy.to(cuda), wt.to(cuda)
    dx = torch.empty((N, H, W, Ci), dtype=TDT[dtype], device=cuda)
    check(LIB.seg_op_conv_dgrad(ABI[dtype], dyd.data_ptr(), N, Ho, Wo, Co, Co, wtd.data_ptr(), Ci, k,
                                s, r, int(ep), H, W, dx.data_ptr(), Ci, st))
    torch.cuda.synchronize()
    _elementwise(dx, ref.to(cuda), 2 * ULP[dtype], 1e-3, f"{name} dgrad")
    del dx, wtd
    # ---- weight gradient (split-K over the 131 k - 524 k pixels, fp32 slabs + reduce); the
    # runtime pads Co % 8 != 0 rows (the logits) itself: that one is covered by the step test
    if Co % 8:
        return
    wg = torch.zeros(Co, k, k, Ci, requires_grad=True)
    conv_tf(x.float().permute(0, 3, 1, 2), wg, spec).backward(dy.float().permute(0, 3, 1, 2))
    dw = torch.zeros((Co, k, k, Ci), dtype=torch.float32, device=cuda)
    ws = torch.empty(768 << 20, dtype=torch.uint8, device=cuda)
    check(LIB.seg_op_conv_wgrad(ABI[dtype], dyd.data_ptr(), N, Ho, Wo, Co, Co, xd.data_ptr(), H, W, Ci,
                                Ci, k, s, r, int(ep), dw.data_ptr(), ws.data_ptr(), ws.numel(), st))
    torch.cuda.synchronize()
    _elementwise(dw, wg.grad.to(cuda), 1e-3, 1e-4, f"{name} wgrad")


# ------------------------------------------------------------------------- one full C2 step
def _bn_bwd(dz, y, z, gamma, y_exact):
    """TF fused-BN training backward of [relu](bn(y)) (z = the ReLU output whose positives
    pass the gradient, None = no ReLU), float64: dy = g * invstd * (dh - mean dh - xh mean(dh xh)).
    The batch moments come from y_exact (the unrounded conv output: the native statistics are
    reduced from the fp32 accumulators in the conv epilogue), x-hat from the stored y the
    native BN backward reads. With 4 nearly equal samples (the ASPP image-pool branch: means of
    random images) moments of the 16-bit y would be off by more than the batch spread."""
    C = y.shape[-1]
    ye = y_exact.double().reshape(-1, C)
    dh = dz.double() if z is None else dz.double() * (z > 0)
    dh = dh.reshape(-1, C)
    mu = ye.mean(0)
    inv = torch.rsqrt(ye.var(0, unbiased=False) + BN_EPS)
    xh = (y.double().reshape(-1, C) - mu) * inv
    out = gamma * inv * (dh - dh.mean(0) - xh * (dh * xh).mean(0))
    return out.reshape(y.shape)


def _maxpool_bwd(z0, g):
    """3x3 / 2 SAME max-pool backward: the gradient goes to the first maximum of each window
    in row-major scan order (TF MaxPoolGrad), padding never selected."""
    N, H, W, C = z0.shape
    Ho, Wo = g.shape[1], g.shape[2]
    ph = max((Ho - 1) * 2 + 3 - H, 0) // 2
    pw = max((Wo - 1) * 2 + 3 - W, 0) // 2
    zp = torch.full((N, H + 2, W + 2, C), -math.inf, dtype=torch.float64, device=z0.device)
    zp[:, ph:ph + H, pw:pw + W] = z0
    taps = [zp[:, i:i + 2 * (Ho - 1) + 1:2, j:j + 2 * (Wo - 1) + 1:2] for i in range(3) for j in range(3)]
    am = torch.stack(taps, 0).argmax(0)     # first maximum
    del taps
    acc = torch.zeros_like(zp)
    for t in range(9):
        i, j = divmod(t, 3)
        acc[:, i:i + 2 * (Ho - 1) + 1:2, j:j + 2 * (Wo - 1) + 1:2] += g * (am == t)
    return acc[:, ph:ph + H, pw:pw + W]


# BASELINE configs at their per-GPU shape (1024 x 2048, 4 images): C2 as the bench runs it;
# C4 = R101 + pyramid with the 1:2:1 strong : bbox : tag mix in bf16 (covers C3's kernels and
# adds the weak-label loss head); C5 = the same mix in fp16 with fp32 master gradients under a
# loss scale of 4096 (the dynamic scaler settles at 8192 on these weights)
# C2-PSP = C2 with the reference's live pyramid module (_create_psp_module, hierarchical.py:
# 186-207; the shipped checkpoint uses it, README.md:31): at 1024 x 2048 the 3- and 6-grids pool
# 42 x 85 and 21 x 42 windows of the 128 x 256 map and drop the remainder rows and columns
FULL_CONFIGS = [
    ("C2", 50, "bf16", (4, 0, 0), "aspp"),
    ("C2-PSP", 50, "bf16", (4, 0, 0), "psp"),
    ("C4", 101, "bf16", (1, 2, 1), "aspp"),
    ("C5", 101, "fp16", (1, 2, 1), "aspp"),
]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name,depth,dtype,mix,pyramid", FULL_CONFIGS, ids=[c[0] for c in FULL_CONFIGS])
def test_step_layerwise_fullsize(cuda, name, depth, dtype, mix, pyramid):
    from input_pipelines.synthetic import batch
    from seg_hip import SegContext
    H, W = 1024, 2048
    npp, npb, npi = mix
    NB = npp + npb + npi
    cfg = SegConfig(depth=depth, height=H, width=W, nb_pp=npp, nb_pb=npb, nb_pi=npi, pyramid=pyramid)
    params = {k: v.astype(np.float32) for k, v in init_params(cfg, seed=2).items()}
    data = batch(17, npp, npb, npi, H, W)
    ctx = SegContext(depth=depth, pyramid=pyramid, height=H, width=W, nb_pp=npp, nb_pb=npb,
                     nb_pi=npi, dtype=dtype)
    ctx.load_params(params)
    if dtype == "fp16":
        ctx.set_loss_scale(4096.0)
    dec = torch.zeros((NB, H, W), dtype=torch.int32, device=cuda)
    ctx.forward(torch.as_tensor(data["images"]).to(cuda))
    dev = lambda a: None if a is None else torch.as_tensor(a).to(cuda)
    ctx.loss(dev(data["px"]), dev(data["bbox"]), dev(data["tag"]), dec)
    losses, _, logits = ctx.outputs()
    ctx.backward()
    torch.cuda.synchronize()
    assert bool(torch.isfinite(ctx.grads).all()), "non-finite gradients"
    u = ULP[dtype]
    specs = build_specs(cfg)
    idx = {s.name: i for i, s in enumerate(specs)}
    info = {p.name: p for p in ctx.param_info}

    def X(i):
        return ctx.debug_device(f"conv{i}_x").double()

    def Y(i):
        return ctx.debug_device(f"conv{i}_y").double()

    def DY(i):
        return ctx.debug_device(f"conv{i}_dy").double()

    def Wt(i):   # the weights the step ran with (16-bit copies of the fp32 masters)
        return torch.as_tensor(params[specs[i].name + "/weights"]).to(cuda).to(TDT[dtype]).double()

    def gamma(i):
        return torch.as_tensor(params[specs[i].name + "/BatchNorm/gamma"], dtype=torch.float64, device=cuda)

    def native_grad(i):
        p = info[specs[i].name + "/weights"]
        return ctx.grads[p.offset:p.offset + p.numel].view(p.shape)

    # conv3 layers the linear BN-backward fold took (csrc/lbf.h): their weight gradient was
    # formed from the affine dz3 = A dyhat + B + D z3 without rounding dz3 to 16 bits (so the
    # 16-bit dz3 the apply would have stored is no reference for it: its rounding errors follow
    # z3 wherever the gate is closed and do not average out, 2.4-2.8e-3 of the gradient on
    # these layers, profiles/r05_lbf_diag.txt); the reference is that affine form in float64
    # from the step's coefficients and gated gradient with the exact conv output. The
    # coefficients themselves are checked through dz3 (chk below: the apply on the same inputs
    # against the float64 BN backward)
    folded = set()
    if ctx.counter("lbf_layers") > 0:
        for i, s in enumerate(specs):
            try:
                ctx.debug_device(f"conv{i}_lbfcoef")
                folded.add(i)
            except Exception:
                pass

    # ---- every conv: forward output and weight gradient (the stem's 3 real channels of tap8)
    for i, s in enumerate(specs):
        x = X(i)
        _elementwise(Y(i), conv_fwd(x, Wt(i), s), 2 * u, 1e-3, f"fwd {s.name}")
        if i in folded:
            coef = ctx.debug_device(f"conv{i}_lbfcoef").double().reshape(3, -1)
            dy = coef[0] * ctx.debug_device(f"conv{i}_dyhat").double() + coef[1] + \
                coef[2] * conv_fwd(x, Wt(i), s)
        else:
            dy = DY(i)
        _elementwise(native_grad(i), conv_wgrad(x, dy, s), 1e-3, 1e-4, f"wgrad {s.name}",
                     absref=conv_wgrad(x.abs(), dy.abs(), s), n_sum=dy[..., 0].numel())
        del dy
        del x

    def chk(i, dz, z, what):
        ye = conv_fwd(X(i), Wt(i), specs[i])
        _tiles(DY(i), _bn_bwd(dz, Y(i), z, gamma(i), ye), 2e-2, 5e-2, f"{what} -> dy {specs[i].name}")

    def dgrad(i, like):
        return conv_dgrad(DY(i), Wt(i), specs[i], like.shape[1], like.shape[2])

    def unit_chain(scope, g_out, out):
        """conv3 (+ projection shortcut) from the unit-output gradient, then conv3 -> conv2 ->
        conv1 inside the unit; returns the gradient w.r.t. the unit input."""
        i1, i2, i3 = idx[f"{scope}/conv1"], idx[f"{scope}/conv2"], idx[f"{scope}/conv3"]
        chk(i3, g_out, out, f"{scope} out")
        isc = idx.get(f"{scope}/shortcut")
        if isc is not None:
            chk(isc, g_out, out, f"{scope} out")
        chk(i2, dgrad(i3, X(i3)), X(i3), f"{scope} conv3 dgrad")
        chk(i1, dgrad(i2, X(i2)), X(i2), f"{scope} conv2 dgrad")
        xin = X(i1)
        g_in = dgrad(i1, xin)
        m = g_out * (out > 0)
        if isc is not None:
            g_in += dgrad(isc, xin)
        elif m.shape[1] == xin.shape[1]:
            g_in += m
        else:   # resnet_utils.subsample: identity shortcut read at stride 2
            g_in[:, ::2, ::2] += m
        return g_in

    # ---- heads: logits dgrad -> head unit; dfeat = sum over heads (identity shortcuts)
    dfeat = None
    for h in ("l1", "l2_vehicle", "l2_human"):
        il = idx[f"softmax_classifier/{h}_logits"]
        out = X(il)
        g = unit_chain(f"adaptation_module/{h}_features", dgrad(il, out), out)
        dfeat = g if dfeat is None else dfeat + g
    pm = "feature_extractor/pyramid_module"
    fd = cfg.feature_dims_decreased
    idfd = idx["feature_extractor/extension/decrease_fdims"]
    if pyramid == "aspp":
        # ---- ASPP: final 1x1 over the 1280-channel concat, four conv branches, image pool
        ifin = idx[f"{pm}/Conv_5"]
        concat = X(ifin)
        chk(ifin, dfeat, X(idx["adaptation_module/l1_features/conv1"]), "dfeat")
        dconcat = dgrad(ifin, concat)
        dz_dfd = 0
        for b in range(1, 5):
            ib = idx[f"{pm}/Conv_{b}"]
            chk(ib, dconcat[..., b * fd:(b + 1) * fd], concat[..., b * fd:(b + 1) * fd], "ASPP concat")
            dz_dfd = dz_dfd + dgrad(ib, X(ib))
        ip = idx[f"{pm}/Conv"]
        chk(ip, dconcat[..., :fd].sum((1, 2), keepdim=True), concat[:, :1, :1, :fd], "ASPP image pool")
        dz_dfd = dz_dfd + dgrad(ip, X(ip)) / (X(ifin).shape[1] * X(ifin).shape[2])
        chk(idfd, dz_dfd, X(idx[f"{pm}/Conv_1"]), "ASPP inputs")
    else:
        # ---- PSP (hierarchical.py:186-207): concat = [z | resize(relu(bn(conv(avgpool_k(z)))))
        # for the grids k = 1, 2, 3, 6], the 1280 -> 256 Conv_4 over it. Forward: the pooled
        # inputs (VALID windows of (hf/8, wf/8) // k, remainder rows / columns dropped) and the
        # align-corners resizes into the concat; backward: the resize transposes, the branch BN
        # backward gated by the branch's own ReLU output, the branch data gradients and the
        # average-pool transposes summed with the identity slice into decrease_fdims' output
        # gradient. float64 references; pooling and resizing by torch on the device
        import torch.nn.functional as F
        from oracle.tfseg import psp_grids
        ifin = idx[f"{pm}/Conv_4"]
        concat = X(ifin)
        z = concat[..., :fd].permute(0, 3, 1, 2)                       # NCHW, decrease_fdims output
        hf, wf = z.shape[2], z.shape[3]
        chk(ifin, dfeat, X(idx["adaptation_module/l1_features/conv1"]), "dfeat")
        dconcat = dgrad(ifin, concat)
        dz_dfd = dconcat[..., :fd].clone()
        grids = psp_grids(H, W)
        assert grids[2] == (42, 85) and grids[3] == (21, 42)          # the dropped remainders
        for b, nm in enumerate(["Conv", "Conv_1", "Conv_2", "Conv_3"]):
            ib = idx[f"{pm}/{nm}"]
            kh, kw = grids[b]
            pooled = F.avg_pool2d(z, (kh, kw), stride=(kh, kw)).permute(0, 2, 3, 1)
            _elementwise(X(ib), pooled, 2 * u, 1e-3, f"PSP pool {nm} ({kh}x{kw})")
            zb = ctx.debug_device(f"pyr{b}_z").double()
            up = F.interpolate(zb.permute(0, 3, 1, 2), size=(hf, wf), mode="bilinear",
                               align_corners=True).permute(0, 2, 3, 1)
            _elementwise(concat[..., (b + 1) * fd:(b + 2) * fd], up, 2 * u, 1e-3, f"PSP resize {nm}")
            src = torch.zeros_like(zb.permute(0, 3, 1, 2), requires_grad=True)
            F.interpolate(src, size=(hf, wf), mode="bilinear", align_corners=True).backward(
                dconcat[..., (b + 1) * fd:(b + 2) * fd].permute(0, 3, 1, 2))
            dzb = src.grad.permute(0, 2, 3, 1)
            chk(ib, dzb, zb, f"PSP resize transpose {nm}")
            dpool = dgrad(ib, X(ib))
            zin = torch.zeros_like(z, requires_grad=True)
            F.avg_pool2d(zin, (kh, kw), stride=(kh, kw)).backward(dpool.permute(0, 3, 1, 2))
            dz_dfd += zin.grad.permute(0, 2, 3, 1)
            del zb, up, src, dzb, dpool, zin
        chk(idfd, dz_dfd, concat[..., :fd], "PSP inputs")
    # ---- encoder units, top down, through residual / subsample / projection shortcuts
    rn = f"feature_extractor/base/resnet_v1_{depth}"
    scopes = [f"{rn}/{unit[0]}" for unit in resnet_units(depth, 8)]
    g_out, out = dgrad(idfd, X(idfd)), X(idfd)
    for k in reversed(range(len(scopes))):
        g_out = unit_chain(scopes[k], g_out, out)
        out = X(idx[f"{scopes[k]}/conv1"])
    # ---- stem: max-pool backward -> ReLU mask -> BN backward
    z0 = ctx.debug_device("z0").double()
    chk(0, _maxpool_bwd(z0, g_out), z0, "max-pool")
    del z0, g_out, out, dfeat, dconcat, concat, dz_dfd

    # ---- loss head on the native low-resolution logits (define_losses_hierarchical.py:98-210)
    net = OracleNet(cfg, params)
    lg = logits.double().cpu()
    low = {}
    c0 = 0
    for key, c in (("l1_logits", 14), ("l2_vehicle_logits", 7), ("l2_human_logits", 3)):
        low[key] = lg[..., c0:c0 + c].permute(0, 3, 1, 2).contiguous()
        c0 += c
    L = net.losses(low, data["px"], data["bbox"], data["tag"])
    ref = [float(L[k]) for k in ("segmentation", "l1_segmentation", "l2_vehicle_segmentation",
                                  "l2_human_segmentation")]
    lv = losses.cpu().numpy()
    np.testing.assert_allclose(lv[:4], ref, rtol=1e-4)
    for a, b in zip(lv[4:7], L["counts"]):   # weak weights follow the l1 argmax (near-ties)
        assert abs(int(a) - int(b)) <= (0 if npb + npi == 0 else max(2, 1e-5 * int(b)))
    _, _, _, fused = net.head_predictions(low)
    mism = float((dec.cpu().long() != fused).double().mean())
    assert mism < 1e-5, f"fused decisions differ on {mism:.2e} of the pixels"
    ctx.close()
