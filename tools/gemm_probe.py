"""Reference rates of the vendor GEMM (torch.mm -> hipBLASLt/rocBLAS) at the 1x1-conv GEMM
shapes of C2, to size the hand-written implicit-GEMM kernels against."""
import torch
def t(a, b, name, reps=10):
    c = a @ b; torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): c = a @ b
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    fl = 2.0 * a.shape[0] * a.shape[1] * b.shape[1]
    print(f"{name:34s} {ms*1e3:8.1f} us {fl/ms/1e9:7.0f} TF/s")
M = 131072
bf = torch.bfloat16
for (k, n, nm) in ((512, 2048, "b4c3 fwd  M x 512 x 2048"), (2048, 512, "b4c1 fwd  M x 2048 x 512"),
                   (1024, 2048, "b4sc fwd  M x 1024 x 2048"), (256, 1024, "b3c3 fwd  M x 256 x 1024")):
    a = torch.randn(M, k, device="cuda", dtype=bf); b = torch.randn(k, n, device="cuda", dtype=bf)
    t(a, b, nm)
    # wgrad: dY^T (n x M) @ X (M x k)
    dy = torch.randn(M, n, device="cuda", dtype=bf)
    t(dy.t(), a, nm.replace("fwd", "wgr"))
# 3x3 as a big GEMM (im2col-equivalent flops): M x 4608 x 512
a = torch.randn(M, 4608, device="cuda", dtype=bf); b = torch.randn(4608, 512, device="cuda", dtype=bf)
t(a, b, "im2col b4c2 M x 4608 x 512")
