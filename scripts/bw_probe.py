"""HBM bandwidth probe: read+write (copy), write-only (fill) and read-only (sum) on 2 GiB tensors."""
import torch

dev = torch.device("cuda:0")
n = 512 * 1024 * 1024  # 2 GiB fp32
x = torch.rand(n, device=dev)
y = torch.empty_like(x)


def t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[reps // 2]


gb = n * 4 / 1e9
print(f"copy  {2 * gb / t(lambda: y.copy_(x)) :.2f} TB/s (read+write)")
print(f"fill  {gb / t(lambda: y.fill_(1.0)):.2f} TB/s (write)")
print(f"sum   {gb / t(lambda: x.sum()):.2f} TB/s (read)")
