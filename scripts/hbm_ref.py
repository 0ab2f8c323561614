# Reference data-movement rates on this box (torch kernels): copy, write-only, read-only.
import torch, time
def t(fn, n=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e-3
N = 4 << 30
a = torch.empty(N // 4, dtype=torch.int32, device='cuda'); a.fill_(1)
b = torch.empty_like(a)
s = t(lambda: b.copy_(a)); print(f"copy  {2 * N / s / 1e9:8.1f} GB/s")
s = t(lambda: b.fill_(3)); print(f"write {N / s / 1e9:8.1f} GB/s")
s = t(lambda: a.sum(dtype=torch.int64)); print(f"read  {N / s / 1e9:8.1f} GB/s")
c = a[: int(N * 0.6) // 4]
s = t(lambda: b[: c.numel()].copy_(c) if False else (b.fill_(0), c.sum(dtype=torch.int64))); print(f"fill+sum(0.6) {(N + 0.6 * N) / s / 1e9:8.1f} GB/s")
