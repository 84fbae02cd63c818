"""ctypes binding of ``libseg_hip.so`` (C ABI in ``include/seg_hip.h``).

This is the only way the host code reaches the GPU path. There is no fallback: if the
library is missing or does not load, importing this module raises ``RuntimeError``.
PyTorch is used only for device memory (flat parameter buffers, inputs) and the stream
handle; every kernel of the training step is in the HIP library.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# SEG_HIP_LIB: development override (kernel A/B variants built by `make VARIANT=...`)
LIB_PATH = os.environ.get("SEG_HIP_LIB") or os.path.join(_HERE, "libseg_hip.so")

EXPORTED_SYMBOLS = [
    "seg_create", "seg_destroy", "seg_last_error", "seg_sizes", "seg_bind_buffers",
    "seg_param_count", "seg_param_info", "seg_param_shape", "seg_params_updated", "seg_forward", "seg_loss",
    "seg_backward", "seg_apply_update", "seg_outputs", "seg_confusion", "seg_debug_tensor",
    "seg_profile", "seg_profile_dump",
    "seg_profile_read", "seg_op_conv_fwd", "seg_op_conv_stat_rows", "seg_op_conv_dgrad",
    "seg_op_conv_dgrad_res",
    "seg_op_conv_wgrad", "seg_op_conv_wgrad_cfg", "seg_bbox_labels", "seg_tag_labels",
    "seg_grad_buckets", "seg_stream_wait_bucket", "seg_set_loss_scale", "seg_found_inf",
    "seg_set_bn_sync", "seg_set_bn_inference", "seg_predict", "seg_full_predictions",
    "seg_set_nesterov", "seg_set_defer_stem", "seg_flush_grads", "seg_set_premask", "seg_set_lbf",
    "seg_counter",
    "seg_crc32c", "seg_prepare_images", "seg_prepare_labels", "seg_prepare_images_crop",
]

# int (*seg_allreduce_fn)(void* user, float* buf, int64_t n, void* stream)
SEG_ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                    ctypes.c_void_p)

PYRAMID = {"none": 0, "psp": 1, "aspp": 2}
DTYPE = {"fp32": 0, "bf16": 1, "fp16": 2}
DATASET = {"cityscapes": 0, "vistas": 1}
PARAM_KIND = {0: "weights", 1: "gamma", 2: "beta", 3: "moving_mean", 4: "moving_variance",
              5: "biases"}
UPSAMPLING = {"bilinear": 0, "hybrid": 1}
NORM = {"batch": 0, "group": 1}


class SegCfg(ctypes.Structure):
    _fields_ = [
        ("depth", ctypes.c_int), ("pyramid", ctypes.c_int), ("height", ctypes.c_int),
        ("width", ctypes.c_int), ("nb_pp", ctypes.c_int), ("nb_pb", ctypes.c_int),
        ("nb_pi", ctypes.c_int), ("dtype", ctypes.c_int), ("dataset", ctypes.c_int),
        ("output_stride", ctypes.c_int), ("feature_dims", ctypes.c_int),
        ("bn_decay", ctypes.c_float), ("train_bn", ctypes.c_int),
        ("weight_decay", ctypes.c_float), ("fov_k", ctypes.c_int), ("fov_rate", ctypes.c_int),
        ("upsampling", ctypes.c_int), ("norm", ctypes.c_int), ("groups", ctypes.c_int),
    ]


def _load():
    # torch first: its HIP runtime must be the process's one before libseg_hip.so resolves
    # libamdhip64 (loading the library first left torch's later device init with
    # "no ROCm-capable device" on the box)
    import torch  # noqa: F401
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"libseg_hip.so not found at {LIB_PATH}: build it with __graft_entry__.build() "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover
        raise RuntimeError(f"failed to load {LIB_PATH}: {e}") from e
    vp, ip, i64, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float
    sig = {
        "seg_create": (ip, [ip, ctypes.POINTER(SegCfg), ctypes.POINTER(vp)]),
        "seg_destroy": (ip, [vp]),
        "seg_last_error": (ctypes.c_char_p, [vp]),
        "seg_sizes": (ip, [vp] + [ctypes.POINTER(i64)] * 4),
        "seg_bind_buffers": (ip, [vp, vp, vp, vp, vp, vp]),
        "seg_param_count": (i64, [vp]),
        "seg_param_info": (ip, [vp, i64, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(i64),
                                ctypes.POINTER(i64), ctypes.POINTER(ip)]),
        "seg_param_shape": (ip, [vp, i64, ctypes.POINTER(i64)]),
        "seg_params_updated": (ip, [vp, vp]),
        "seg_forward": (ip, [vp, vp, vp]),
        "seg_loss": (ip, [vp, vp, vp, vp, vp, vp]),
        "seg_backward": (ip, [vp, vp]),
        "seg_apply_update": (ip, [vp, f, f, f, f, vp]),
        "seg_outputs": (ip, [vp, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp),
                             ctypes.POINTER(ip), ctypes.POINTER(ip), ctypes.POINTER(ip)]),
        "seg_confusion": (ip, [vp, vp, vp, i64, ip, vp, vp]),
        "seg_debug_tensor": (ip, [vp, ctypes.c_char_p, ctypes.POINTER(vp), ctypes.POINTER(ip),
                                  ctypes.POINTER(ip), ctypes.POINTER(ip)]),
        "seg_profile": (ip, [vp, ip]),
        "seg_profile_dump": (ip, [vp, ctypes.c_char_p, ip]),
        "seg_profile_read": (ip, [vp, ip, ctypes.POINTER(ctypes.c_double),
                                  ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i64),
                                  ctypes.POINTER(ctypes.c_double), ctypes.c_char_p, ip]),
        "seg_op_conv_fwd": (ip, [ip, vp, ip, ip, ip, ip, ip, vp, ip, ip, ip, ip, ip, vp, ip, vp, vp]),
        "seg_op_conv_stat_rows": (ip, [ip] * 12),
        "seg_op_conv_dgrad": (ip, [ip, vp, ip, ip, ip, ip, ip, vp, ip, ip, ip, ip, ip, ip, ip, vp,
                                   ip, vp]),
        "seg_op_conv_dgrad_res": (ip, [ip, vp, ip, ip, ip, ip, ip, vp, ip, vp, ip, vp, ip, vp, vp]),
        "seg_op_conv_wgrad": (ip, [ip, vp, ip, ip, ip, ip, ip, vp, ip, ip, ip, ip, ip, ip, ip, ip,
                                   vp, vp, i64, vp]),
        "seg_op_conv_wgrad_cfg": (ip, [ip, vp, ip, ip, ip, ip, ip, vp, ip, ip, ip, ip, ip, ip, ip,
                                       ip, vp, vp, i64, ip, ip, ip, vp]),
        "seg_bbox_labels": (ip, [vp, vp, vp, vp, ip, ip, ip, ip, vp, vp]),
        "seg_grad_buckets": (ip, [vp, ip, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
        "seg_stream_wait_bucket": (ip, [vp, ip, vp]),
        "seg_set_loss_scale": (ip, [vp, ctypes.c_float]),
        "seg_found_inf": (ip, [vp, ctypes.POINTER(ctypes.c_void_p)]),
        "seg_set_bn_sync": (ip, [vp, SEG_ALLREDUCE_FN, vp, ip]),
        "seg_tag_labels": (ip, [vp, ip, ip, ip, vp, vp]),
        "seg_set_bn_inference": (ip, [vp, ip]),
        "seg_prepare_images": (ip, [vp, ip, ip, ip, ip, ip, vp, vp]),
        "seg_prepare_images_crop": (ip, [vp, ip, ip, ip, ip, ip, ip, ip, ip, ip, vp, vp]),
        "seg_prepare_labels": (ip, [vp, ip, ip, ip, ip, ip, ctypes.POINTER(ctypes.c_int32), ip,
                                    vp, vp]),
        "seg_crc32c": (ctypes.c_uint32, [ctypes.c_uint32, vp, ctypes.c_size_t]),
        "seg_predict": (ip, [vp, ctypes.POINTER(ctypes.c_int32), ip, ip, ip, ip, vp, vp]),
        "seg_full_predictions": (ip, [vp, vp, vp, vp, vp, vp]),
        "seg_set_nesterov": (ip, [vp, ip]),
        "seg_set_defer_stem": (ip, [vp, ip]),
        "seg_flush_grads": (ip, [vp, vp]),
        "seg_set_premask": (ip, [vp, ip]),
        "seg_set_lbf": (ip, [vp, ip]),
        "seg_counter": (ip, [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64)]),
    }
    override = "SEG_HIP_LIB" in os.environ   # A/B builds of older commits may lack new entries
    for name, (res, args) in sig.items():
        if override and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


LIB = _load()


def check(rc: int, ctx=None):
    if rc != 0:
        msg = LIB.seg_last_error(ctx)
        raise RuntimeError(f"libseg_hip error {rc}: {msg.decode() if msg else ''}")


def _ptr(t) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _stream(stream=None) -> int:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


@dataclass
class ParamInfo:
    name: str
    offset: int
    numel: int
    kind: str
    shape: tuple


class SegContext:
    """One device context of the native training path (one per GPU per process).

    Owns the flat fp32 buffers (as torch tensors on the context's device): ``params``,
    ``grads`` (+ BN batch-statistics tail), ``momentum``, optional ``ema`` and ``moving``.
    """

    def __init__(self, *, depth=50, pyramid="psp", height=512, width=1024, nb_pp=2, nb_pb=0,
                 nb_pi=0, dtype="bf16", dataset="cityscapes", output_stride=8,
                 feature_dims=256, bn_decay=0.9, train_bn=True, weight_decay=0.00017,
                 ema=False, device=None, fov_k=0, fov_rate=0, upsampling="bilinear",
                 norm="batch", groups=0):
        import torch
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self.cfg = SegCfg(depth, PYRAMID[pyramid], height, width, nb_pp, nb_pb, nb_pi,
                          DTYPE[dtype], DATASET[dataset], output_stride, feature_dims,
                          bn_decay, int(bool(train_bn)), weight_decay, fov_k, fov_rate,
                          UPSAMPLING[upsampling], NORM[norm], groups)
        self.dtype = dtype
        h = ctypes.c_void_p()
        check(LIB.seg_create(self.device.index, ctypes.byref(self.cfg), ctypes.byref(h)))
        self.h = h
        vals = [ctypes.c_int64() for _ in range(4)]
        check(LIB.seg_sizes(self.h, *[ctypes.byref(v) for v in vals]), self.h)
        self.n_train, self.n_decay, self.n_moving, self.n_stats = [v.value for v in vals]
        f32 = dict(dtype=torch.float32, device=self.device)
        self.params = torch.zeros(self.n_train, **f32)
        self.grads = torch.zeros(self.n_train + self.n_stats, **f32)
        self.momentum = torch.zeros(self.n_train, **f32)
        self.ema = torch.zeros(self.n_train, **f32) if ema else None
        self.moving = torch.zeros(self.n_moving, **f32)
        check(LIB.seg_bind_buffers(self.h, _ptr(self.params), _ptr(self.grads),
                                   _ptr(self.momentum), _ptr(self.ema), _ptr(self.moving)), self.h)
        self.param_info = self._param_info()

    # ---- parameters -----------------------------------------------------------------
    def _param_info(self) -> List[ParamInfo]:
        out = []
        for i in range(LIB.seg_param_count(self.h)):
            nm, off, n, k = ctypes.c_char_p(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int()
            check(LIB.seg_param_info(self.h, i, ctypes.byref(nm), ctypes.byref(off),
                                     ctypes.byref(n), ctypes.byref(k)), self.h)
            dims = (ctypes.c_int64 * 4)()
            check(LIB.seg_param_shape(self.h, i, dims), self.h)
            kind = PARAM_KIND[k.value]
            shape = tuple(dims) if kind == "weights" else (dims[0],)
            out.append(ParamInfo(nm.value.decode(), off.value, n.value, kind, shape))
        return out

    def _buffer_for(self, p: ParamInfo):
        return self.moving if p.kind in ("moving_mean", "moving_variance") else self.params

    def load_params(self, values: Dict[str, np.ndarray], stream=None):
        """Write named parameters (weights [Co][KH][KW][Ci]) and refresh compute copies."""
        import torch
        for p in self.param_info:
            if p.name in values:
                v = torch.as_tensor(np.asarray(values[p.name], dtype=np.float32).reshape(-1))
                if v.numel() != p.numel:
                    raise ValueError(f"{p.name}: expected {p.numel} values, got {v.numel()}")
                self._buffer_for(p)[p.offset:p.offset + p.numel].copy_(v.to(self.device))
        if self.ema is not None:
            self.ema.copy_(self.params)
        check(LIB.seg_params_updated(self.h, _stream(stream)), self.h)

    def named(self, buffer: str = "params") -> Dict[str, np.ndarray]:
        """Host copies of named tensors of params/grads/momentum/ema."""
        buf = {"params": self.params, "grads": self.grads, "momentum": self.momentum,
               "ema": self.ema}[buffer]
        if buffer == "grads":   # a deferred stem weight gradient (seg_set_defer_stem) finishes first
            self.flush_grads()
        out = {}
        for p in self.param_info:
            if p.kind in ("moving_mean", "moving_variance"):
                src = self.moving if buffer == "params" else None
            else:
                src = buf
            if src is not None:
                out[p.name] = src[p.offset:p.offset + p.numel].detach().cpu().numpy()
        return out

    def flush_grads(self, stream=None):
        """Join a still-running deferred stem weight gradient (seg_set_defer_stem) on ``stream``
        so the gradient buffer is complete; a no-op otherwise."""
        check(LIB.seg_flush_grads(self.h, _stream(stream)), self.h)

    # ---- step -----------------------------------------------------------------------
    def forward(self, images, stream=None):
        check(LIB.seg_forward(self.h, _ptr(images), _stream(stream)), self.h)
        self.forward_count = getattr(self, "forward_count", 0) + 1

    def loss(self, px_labels=None, bbox_soft=None, tag_soft=None, decisions=None, stream=None):
        check(LIB.seg_loss(self.h, _ptr(px_labels), _ptr(bbox_soft), _ptr(tag_soft),
                           _ptr(decisions), _stream(stream)), self.h)

    def set_bn_inference(self, on: bool):
        """BN normalises with the moving statistics in later forwards (is_training=False,
        the reference's default unless --batch_norm_accumulate_statistics)."""
        check(LIB.seg_set_bn_inference(self.h, 1 if on else 0), self.h)
        self.bn_inference = bool(on)

    def predict(self, cid_map, out, replace_voids=False, stream=None, order="eval"):
        """Decisions of the last forward mapped through ``cid_map`` (training -> eval/inference
        cids, -1 = void), optionally void-replaced, nearest-neighbour resized to out's
        [N, Ho, Wo] (device int32). ``order``: "eval" replaces voids at network resolution
        before the resize (the EVAL branch); "predict" resizes first -- l1 probabilities
        bilinearly (align_corners) -- and replaces voids on the resized probabilities (the
        PREDICT branch, define_estimator_hierarchical.py:227-231)."""
        if order not in ("eval", "predict"):
            raise ValueError(f"order must be 'eval' or 'predict', got {order!r}")
        m = (ctypes.c_int32 * len(cid_map))(*[int(v) for v in cid_map])
        import torch
        n = self.cfg.nb_pp + self.cfg.nb_pb + self.cfg.nb_pi
        if not (out.dtype == torch.int32 and out.dim() == 3 and out.is_contiguous()
                and out.shape[0] == n and out.is_cuda):
            raise ValueError(f"decisions buffer must be a contiguous device int32 [{n}, Ho, Wo]")
        rv = (2 if order == "predict" else 1) if replace_voids else 0
        check(LIB.seg_predict(self.h, m, len(cid_map), rv,
                              int(out.shape[1]), int(out.shape[2]), _ptr(out), _stream(stream)),
              self.h)

    def full_predictions(self, logits=None, probs=None, head_decisions=None, decisions=None,
                         stream=None):
        """The model's full-resolution predictions of the last forward at network resolution
        (hierarchical.py:84-130) written into the given device buffers (any may be None):
        logits / probs f32 [N, H, W, C] (C = c1 + c2 + c3, heads l1 | l2v | l2h),
        head_decisions int32 [N, H, W, 3], decisions int32 [N, H, W] (fused, common cids)."""
        import torch
        n = self.cfg.nb_pp + self.cfg.nb_pb + self.cfg.nb_pi
        hw = (self.cfg.height, self.cfg.width)
        for t, dt, tail in ((logits, torch.float32, None), (probs, torch.float32, None),
                            (head_decisions, torch.int32, (3,)), (decisions, torch.int32, ())):
            if t is None:
                continue
            if tail is None:
                tail = (sum((53, 12, 5) if self.cfg.dataset == DATASET["vistas"] else (14, 7, 3)),)
            ok = (t.dtype == dt and t.is_cuda and t.is_contiguous() and tuple(t.shape[:3]) == (n,) + hw
                  and tuple(t.shape[3:]) == tail)
            if not ok:
                raise ValueError(f"prediction buffer {tuple(t.shape)} {t.dtype}: expected a "
                                 f"contiguous device tensor [{n}, {hw[0]}, {hw[1]}, ...]")
        check(LIB.seg_full_predictions(self.h, _ptr(logits), _ptr(probs), _ptr(head_decisions),
                                       _ptr(decisions), _stream(stream)), self.h)

    def backward(self, stream=None):
        check(LIB.seg_backward(self.h, _stream(stream)), self.h)

    def set_loss_scale(self, scale: float):
        """Gradient-seed multiplier (fp16 dynamic loss scaling; see seg_set_loss_scale)."""
        check(LIB.seg_set_loss_scale(self.h, float(scale)), self.h)
        self.loss_scale = float(scale)

    def found_inf(self):
        """Device int32 view of the last update's overflow flag (None unless loss scaling)."""
        p = ctypes.c_void_p()
        check(LIB.seg_found_inf(self.h, ctypes.byref(p)), self.h)
        return None if not p.value else _wrap_i32(p.value, (1,), self.device)

    def set_bn_sync(self, world=None, group=None, always=False):
        """Cross-replica batch norm (the reference's --cross_replica_norm, see seg_set_bn_sync):
        each BN layer's moments (forward) and gradient means (backward) are summed over
        `group` by torch.distributed.all_reduce (RCCL or gloo) ordered on the step's stream.
        world=None takes the group's size; a world of 1 turns synchronisation off unless
        `always` (then the one-replica group still runs every exchange: tests of the
        collective path on one GPU)."""
        import torch
        import torch.distributed as dist
        if world is None:
            world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        if world <= 1 and not always:
            check(LIB.seg_set_bn_sync(self.h, SEG_ALLREDUCE_FN(), None, 1), self.h)
            self._sync_cb = None
            return
        dev = self.device

        def _exchange(user, buf, n, stream):   # called from inside seg_forward / seg_backward
            try:
                t = _wrap(buf, (int(n),), dev)
                s = (torch.cuda.ExternalStream(stream, device=dev) if stream
                     else torch.cuda.default_stream(dev))
                with torch.cuda.stream(s):
                    dist.all_reduce(t, group=group)
                return 0
            except Exception as e:  # reported through the failing seg_* call
                self.sync_error = e
                return 1
        cb = SEG_ALLREDUCE_FN(_exchange)
        check(LIB.seg_set_bn_sync(self.h, cb, None, int(world)), self.h)
        self._sync_cb = cb   # the C side holds the raw pointer: keep the thunk alive

    def grad_buckets(self):
        """[(lo, hi)] ranges of self.grads in the order the backward completes them."""
        n = LIB.seg_grad_buckets(self.h, 0, None, None)
        if n < 0:
            check(n, self.h)
        lo, hi = (ctypes.c_int64 * n)(), (ctypes.c_int64 * n)()
        check(LIB.seg_grad_buckets(self.h, n, lo, hi) - n, self.h)
        return [(int(lo[i]), int(hi[i])) for i in range(n)]

    def wait_bucket(self, i, stream):
        """Make `stream` wait until the last seg_backward has written bucket i."""
        check(LIB.seg_stream_wait_bucket(self.h, i, _stream(stream)), self.h)

    def set_nesterov(self, on: bool):
        """MomentumOptimizer(use_nesterov=on) for the following updates."""
        check(LIB.seg_set_nesterov(self.h, 1 if on else 0), self.h)
        self.nesterov = bool(on)

    def set_defer_stem(self, on: bool):
        """Single-process training loops: update every other parameter beside the stem's weight
        gradient (the step's last kernel); gradients must not be read between backward() and
        apply_update() while this is on."""
        check(LIB.seg_set_defer_stem(self.h, 1 if on else 0), self.h)

    def set_premask(self, on):
        """seg_set_premask: pre-masked identity-unit gradients (default on; results unchanged)."""
        check(LIB.seg_set_premask(self.h, 1 if on else 0), self.h)

    def set_lbf(self, on):
        """seg_set_lbf: the linear BN-backward fold of the bottleneck conv3 layers (default on;
        off = the separate BN-backward apply pass, the fold's reference path in tests)."""
        check(LIB.seg_set_lbf(self.h, 1 if on else 0), self.h)

    def counter(self, name: str) -> int:
        """seg_counter: a runtime counter since creation (e.g. "premask_launches")."""
        v = ctypes.c_int64()
        check(LIB.seg_counter(self.h, name.encode(), ctypes.byref(v)), self.h)
        return v.value

    def apply_update(self, lr, momentum=0.9, ema_decay_eff=0.0, grad_scale=1.0, stream=None):
        check(LIB.seg_apply_update(self.h, lr, momentum, ema_decay_eff, grad_scale,
                                   _stream(stream)), self.h)

    def outputs(self):
        """(losses[10], reg[1], low-res logits [N,Hl,Wl,ldl]) as torch views (device)."""
        import torch
        l, r, lg = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        ld, hl, wl = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(LIB.seg_outputs(self.h, ctypes.byref(l), ctypes.byref(r), ctypes.byref(lg),
                              ctypes.byref(ld), ctypes.byref(hl), ctypes.byref(wl)), self.h)
        n = self.cfg.nb_pp + self.cfg.nb_pb + self.cfg.nb_pi
        return (_wrap(l.value, (10,), self.device), _wrap(r.value, (1,), self.device),
                _wrap(lg.value, (n, hl.value, wl.value, ld.value), self.device))

    def confusion(self, labels, decisions, num_classes, out, stream=None):
        check(LIB.seg_confusion(self.h, _ptr(labels), _ptr(decisions), labels.numel(),
                                num_classes, _ptr(out), _stream(stream)), self.h)

    def debug_tensor(self, name: str):
        """Host copy (float32, [N,H,W,C]) of an internal tensor (parity tests only)."""
        import torch
        ptr = ctypes.c_void_p()
        dims = (ctypes.c_int * 4)()
        ld, dt = ctypes.c_int(), ctypes.c_int()
        check(LIB.seg_debug_tensor(self.h, name.encode(), ctypes.byref(ptr), dims, ctypes.byref(ld),
                                   ctypes.byref(dt)), self.h)
        n, hh, ww, c = list(dims)
        torch.cuda.synchronize()
        if dt.value == 0:
            t = _wrap(ptr.value, (n * hh * ww, ld.value), self.device)
        else:
            t = _wrap_u16(ptr.value, (n * hh * ww, ld.value), self.device, half=dt.value == 2)
        return t[:, :c].float().cpu().numpy().reshape(n, hh, ww, c)

    def debug_device(self, name: str):
        """Zero-copy device view [N,H,W,C] (storage dtype, pixel stride ld) of an internal
        tensor: the full-size parity tests read 1024 x 2048 activations without a host copy."""
        import torch
        ptr = ctypes.c_void_p()
        dims = (ctypes.c_int * 4)()
        ld, dt = ctypes.c_int(), ctypes.c_int()
        check(LIB.seg_debug_tensor(self.h, name.encode(), ctypes.byref(ptr), dims, ctypes.byref(ld),
                                   ctypes.byref(dt)), self.h)
        n, hh, ww, c = list(dims)
        if dt.value == 0:
            t = _wrap(ptr.value, (n * hh * ww, ld.value), self.device)
        else:
            t = _wrap_u16(ptr.value, (n * hh * ww, ld.value), self.device, half=dt.value == 2)
        return t[:, :c].unflatten(0, (n, hh, ww))

    def profile(self, enable: bool):
        check(LIB.seg_profile(self.h, int(enable)), self.h)

    def profile_read(self, cls: int):
        ms, gf, mx = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        n = ctypes.c_int64()
        name = ctypes.create_string_buffer(256)
        check(LIB.seg_profile_read(self.h, cls, ctypes.byref(ms), ctypes.byref(gf), ctypes.byref(n),
                                   ctypes.byref(mx), name, 256), self.h)
        return dict(ms=ms.value, gflop=gf.value, launches=n.value, ms_max_layer=mx.value,
                    max_layer=name.value.decode())

    def profile_dump(self):
        """Per-launch records of the conv kernels: list of dicts."""
        buf = ctypes.create_string_buffer(1 << 22)
        check(LIB.seg_profile_dump(self.h, buf, len(buf)), self.h)
        rows = []
        for line in buf.value.decode().splitlines():
            f = line.split()
            rows.append(dict(cls=int(f[0]), name=f[1], ci=int(f[2]), co=int(f[3]), k=int(f[4]),
                             rate=int(f[5]), ho=int(f[6]), wo=int(f[7]), gflop=float(f[8]),
                             ms=float(f[9]), gbytes=float(f[10]) if len(f) > 10 else 0.0))
        return rows

    def close(self):
        if getattr(self, "h", None):
            LIB.seg_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _wrap_u16(ptr: int, shape: Tuple[int, ...], device, half=False):
    """Zero-copy view of a bf16 (or fp16) device buffer (reinterpreted from int16)."""
    import torch

    class _CAI:
        pass
    o = _CAI()
    o.__cuda_array_interface__ = {"shape": shape, "typestr": "<i2", "data": (ptr, False),
                                  "version": 3, "strides": None}
    return torch.as_tensor(o, device=device).view(torch.float16 if half else torch.bfloat16)


def _wrap_i32(ptr: int, shape: Tuple[int, ...], device):
    import torch

    class _CAI:
        pass
    o = _CAI()
    o.__cuda_array_interface__ = {"shape": shape, "typestr": "<i4", "data": (ptr, False),
                                  "version": 3, "strides": None}
    return torch.as_tensor(o, device=device)


def _wrap(ptr: int, shape: Tuple[int, ...], device):
    """Zero-copy torch view of a context-owned fp32 device buffer."""
    import torch

    class _CAI:
        pass
    o = _CAI()
    o.__cuda_array_interface__ = {"shape": shape, "typestr": "<f4", "data": (ptr, False),
                                  "version": 3, "strides": None}
    return torch.as_tensor(o, device=device)
