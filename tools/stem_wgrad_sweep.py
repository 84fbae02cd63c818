"""Tile / split sweep of the space-to-depth stem's weight gradient (GPU box):
    python tools/stem_wgrad_sweep.py
The stem (7 x 7 stride 2 over 3 channels) runs as a 4 x 4 VALID conv over the 16-channel
space-to-depth image: dy [4, 512, 1024, 64], x [4, 515, 1027, 16]. The op entry has no VALID
4 x 4 geometry, so the sweep runs the SAME-padded one (x [4, 512, 1024, 16]: the same gather per
output pixel, a one-pixel border of out-of-range taps); the library's own choice is
the v2 kernel at 64 x 256 with 256 splits (conv_wgrad_v2_tile, wgrad_splits). Prints us per
launch (weight-gradient kernel + split-K reduce) for each (bm, bn, splits)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "iv2019-boosting-semantic-segmentation-with-weak-labels_amd")]
import torch
from seg_hip import LIB, check

N, Ho, Wo, Co, C, k = 4, 512, 1024, 64, 16, 4
H, W = Ho, Wo
dev = torch.device("cuda")
g = torch.Generator(device="cpu").manual_seed(0)
dy = torch.randn(N, Ho, Wo, Co, generator=g).to(dev, torch.bfloat16)
x = torch.randn(N, H, W, C, generator=g).to(dev, torch.bfloat16)
dw = torch.empty(Co * k * k * C, device=dev, dtype=torch.float32)
ws = torch.empty(1 << 30, device=dev, dtype=torch.uint8)
st = torch.cuda.current_stream().cuda_stream
reps = int(os.environ.get("REPS", "20"))
ref = None
for bm, bn in ((64, 256), (64, 128), (64, 64)):
    for splits in (128, 256, 512, 1024):
        def run():
            check(LIB.seg_op_conv_wgrad_cfg(1, dy.data_ptr(), N, Ho, Wo, Co, Co, x.data_ptr(), H, W, C, C,
                                            k, 1, 1, 0, dw.data_ptr(), ws.data_ptr(), ws.numel(), bm, bn,
                                            splits, st))
        run(); torch.cuda.synchronize()
        if ref is None:
            ref = dw.clone()
        err = ((dw - ref).norm() / ref.norm()).item()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run()
        e1.record(); torch.cuda.synchronize()
        print(f"bm {bm:3d} bn {bn:3d} splits {splits:4d}: {e0.elapsed_time(e1) / reps * 1e3:7.1f} us  (rel diff {err:.1e})", flush=True)
