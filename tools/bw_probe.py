"""HBM streaming reference rates on this GPU (torch's own elementwise kernels), to size the
BN streaming kernels against: 1R+1W copy, 2R+1W add, 3R-ish reductions, bf16, 268M elems."""
import torch
n = 131072 * 2048
a = torch.randn(n, dtype=torch.bfloat16, device="cuda")
b = torch.randn(n, dtype=torch.bfloat16, device="cuda")
c = torch.empty_like(a)
def t(f, nbytes, name, reps=10):
    f(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): f()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"{name:28s} {ms*1e3:8.1f} us  {nbytes/ms/1e9:6.2f} TB/s")
t(lambda: c.copy_(a), 4 * n, "copy 1R1W")
t(lambda: torch.add(a, b, out=c), 6 * n, "add 2R1W")
t(lambda: a.view(-1, 2048).sum(0, dtype=torch.float32), 2 * n, "colsum 1R")
t(lambda: c.zero_(), 2 * n, "fill 1W")
# the C2 BN layer sizes (67 MB / 268 MB per operand): short streams pay launch ramp and tail
for m in (131072 * 256, 131072 * 1024):
    x = torch.randn(m, dtype=torch.bfloat16, device="cuda")
    y = torch.empty_like(x)
    t(lambda: y.copy_(x), 4 * m, f"copy 1R1W {m * 2 >> 20} MB")
