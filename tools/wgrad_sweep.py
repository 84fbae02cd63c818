"""Tile / split sweep of the v2 weight-gradient kernel on the small-channel C2 layers (GPU box):
    python tools/wgrad_sweep.py [layer ...]   (layers from tools/op_bench.py SHAPES)
For every (bm, bn, splits) it times kernel + fixed-order split-K reduce (HIP events, 10 reps)
and prints the default choice (conv_wgrad_v2_tile + wgrad_splits' full-chip target) beside the
best one."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "iv2019-boosting-semantic-segmentation-with-weak-labels_amd")]
import torch  # noqa: E402
from seg_hip import LIB, check  # noqa: E402

SHAPES = {  # N, H, W, Ci, Co, k, stride, rate
    "b1c2": (4, 256, 512, 64, 64, 3, 1, 1),
    "b1c3": (4, 256, 512, 64, 256, 1, 1, 1),
    "b1c1": (4, 256, 512, 256, 64, 1, 1, 1),
    "b2c2": (4, 128, 256, 128, 128, 3, 1, 1),
    "b2c1": (4, 128, 256, 512, 128, 1, 1, 1),
    "b2c3": (4, 128, 256, 128, 512, 1, 1, 1),
    "b3c2": (4, 128, 256, 256, 256, 3, 1, 2),
    "b3c3": (4, 128, 256, 256, 1024, 1, 1, 1),
    "b3c1": (4, 128, 256, 1024, 256, 1, 1, 1),
    "b4c1": (4, 128, 256, 2048, 512, 1, 1, 1),
    "b4c3": (4, 128, 256, 512, 2048, 1, 1, 1),
    "b4c2": (4, 128, 256, 512, 512, 3, 1, 4),
    "head1": (4, 128, 256, 256, 256, 1, 1, 1),
}
PP_ONLY = os.environ.get("PP_ONLY") == "1"   # 256 x 256 tiles (the ping-pong kernel) only
vp, ip, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
LIB.seg_op_conv_wgrad_cfg.argtypes = [ip, vp, ip, ip, ip, ip, ip, vp, ip, ip, ip, ip, ip, ip, ip,
                                      ip, vp, vp, i64, ip, ip, ip, vp]
layers = sys.argv[1:] or ["b1c2", "b2c2", "b1c3", "b1c1", "b2c1", "b2c3"]
dev = torch.device("cuda")
ws = torch.empty(768 << 20, device=dev, dtype=torch.uint8)
stream = torch.cuda.current_stream().cuda_stream
for name in layers:
    N, H, W, Ci, Co, k, s, r = SHAPES[name]
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(N, H, W, Ci, generator=g).to(dev, torch.bfloat16)
    dy = torch.randn(N, H, W, Co, generator=g).to(dev, torch.bfloat16)
    dw = torch.empty(Co * k * k * Ci, device=dev, dtype=torch.float32)
    P, ncol = N * H * W, k * k * Ci
    fl = 2.0 * P * Co * ncol
    res = []
    for bm in ((256,) if PP_ONLY else (64, 128, 256)):
        if bm > 64 and Co <= bm // 2:
            continue
        for bn in ((256,) if PP_ONLY else (64, 128, 256)):
            if bn > 64 and ncol <= bn // 2:
                continue
            for sp in ((4, 8, 16, 24, 32, 48, 64, 96, 128) if PP_ONLY else (32, 64, 128, 256, 512)):
                if sp > max(1, P // 1024) or sp * Co * ncol * 4 > ws.numel():
                    continue
                def run():
                    check(LIB.seg_op_conv_wgrad_cfg(1, dy.data_ptr(), N, H, W, Co, Co, x.data_ptr(), H, W,
                                                    Ci, Ci, k, s, r, 0, dw.data_ptr(), ws.data_ptr(),
                                                    ws.numel(), bm, bn, sp, stream))
                run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    run()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / 10
                res.append((ms, bm, bn, sp))
    res.sort()
    print(f"{name} (Co {Co}, Ncol {ncol}, P {P}): best " +
          ", ".join(f"{bm}x{bn}/s{sp} {ms*1e3:.1f}us {fl/ms/1e9:.0f}TF/s" for ms, bm, bn, sp in res[:4]))
    if PP_ONLY:
        print("   all: " + ", ".join(f"s{sp} {ms*1e3:.0f}" for ms, bm, bn, sp in sorted(res, key=lambda t: t[3])))
    sys.stdout.flush()
