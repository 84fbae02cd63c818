"""Single-op timing of the conv kernels at C2 layer shapes (GPU box):
    python tools/op_bench.py [fwd|dgrad|dgradres|wgrad] [layer]   (layer: b4c2, b4c3, b3c2, b4c1)
Used under rocprofv3 --pmc for counter passes on one kernel class."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "iv2019-boosting-semantic-segmentation-with-weak-labels_amd")]
import torch
from seg_hip import LIB, check

SHAPES = {  # N, H, W, Ci, Co, k, stride, rate
    "b4c2": (4, 128, 256, 512, 512, 3, 1, 4),
    "b4c3": (4, 128, 256, 512, 2048, 1, 1, 1),
    "b4c1": (4, 128, 256, 2048, 512, 1, 1, 1),
    "b3c2": (4, 128, 256, 256, 256, 3, 1, 2),
    "b3c1": (4, 128, 256, 1024, 256, 1, 1, 1),
    "b3c3": (4, 128, 256, 256, 1024, 1, 1, 1),
    "head1": (4, 128, 256, 256, 256, 1, 1, 1),
    "b1c2": (4, 256, 512, 64, 64, 3, 1, 1),
    "b1c3": (4, 256, 512, 64, 256, 1, 1, 1),
    "b2c2": (4, 128, 256, 128, 128, 3, 1, 1),
    "b2c1": (4, 128, 256, 512, 128, 1, 1, 1),
    "b2c3": (4, 128, 256, 128, 512, 1, 1, 1),
}
op = sys.argv[1] if len(sys.argv) > 1 else "wgrad"
N, H, W, Ci, Co, k, s, r = SHAPES[sys.argv[2] if len(sys.argv) > 2 else "b4c2"]
reps = int(os.environ.get("REPS", "20"))
dev = torch.device("cuda")
g = torch.Generator(device="cpu").manual_seed(0)
x = torch.randn(N, H, W, Ci, generator=g).to(dev, torch.bfloat16)
w = (torch.randn(Co, k, k, Ci, generator=g) * 0.02).to(dev, torch.bfloat16)
dy = torch.randn(N, H, W, Co, generator=g).to(dev, torch.bfloat16)
y = torch.empty(N, H, W, Co, device=dev, dtype=torch.bfloat16)
dx = torch.empty(N, H, W, Ci, device=dev, dtype=torch.bfloat16)
st = torch.empty((N * H * W + 63) // 64 * Co * 2, device=dev, dtype=torch.float32)   # 64-row partials at most
dw = torch.empty(Co * k * k * Ci, device=dev, dtype=torch.float32)
ws = torch.empty(512 << 20, device=dev, dtype=torch.uint8)
wt = w.flip(1, 2).permute(3, 1, 2, 0).contiguous()
if op == "dgradres":
    assert k == 1 and s == 1
    res = torch.randn(N, H, W, Ci, generator=g).to(dev, torch.bfloat16)
    bits = torch.randint(0, 256, (N, H, W, Ci // 8), generator=g, dtype=torch.uint8).to(dev)
stream = torch.cuda.current_stream().cuda_stream
def run():
    if op == "fwd":
        check(LIB.seg_op_conv_fwd(1, x.data_ptr(), N, H, W, Ci, Ci, w.data_ptr(), Co, k, s, r, 0,
                                  y.data_ptr(), Co, 0 if os.environ.get("NOSTATS") else st.data_ptr(), stream))
    elif op == "dgradres":   # the identity units' conv1 data gradient: + residual, premasked
        check(LIB.seg_op_conv_dgrad_res(1, dy.data_ptr(), N, H, W, Co, Co, wt.data_ptr(), Ci,
                                        dx.data_ptr(), Ci, res.data_ptr(), Ci, bits.data_ptr(), stream))
    elif op == "dgrad":
        check(LIB.seg_op_conv_dgrad(1, dy.data_ptr(), N, H, W, Co, Co, wt.data_ptr(), Ci, k, s, r, 0,
                                    H, W, dx.data_ptr(), Ci, stream))
    elif os.environ.get("SPLITS"):   # the 256 x 256 kernel at an explicit split count (side-stream sizing)
        check(LIB.seg_op_conv_wgrad_cfg(1, dy.data_ptr(), N, H, W, Co, Co, x.data_ptr(), H, W, Ci, Ci,
                                        k, s, r, 0, dw.data_ptr(), ws.data_ptr(), ws.numel(), 256, 256,
                                        int(os.environ["SPLITS"]), stream))
    else:
        check(LIB.seg_op_conv_wgrad(1, dy.data_ptr(), N, H, W, Co, Co, x.data_ptr(), H, W, Ci, Ci,
                                    k, s, r, 0, dw.data_ptr(), ws.data_ptr(), ws.numel(), stream))
run(); torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps): run()
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
fl = 2.0 * N * H * W * Co * k * k * Ci
print(f"{op} {sys.argv[2] if len(sys.argv) > 2 else 'b4c2'}: {ms*1e3:.1f} us/launch (incl. split-K reduce for wgrad), {fl/ms/1e9:.0f} TF/s")
