"""Debug: achievable HBM write / read+write bandwidth on this GPU (torch fill_ / copy_)."""
import time
import torch
x = torch.empty(256 * 1024 * 1024, dtype=torch.float32, device="cuda")  # 1 GiB
y = torch.empty_like(x)
for name, fn, nbytes in (("fill (write only)", lambda: x.fill_(1.0), x.numel() * 4),
                         ("copy (read + write)", lambda: y.copy_(x), 2 * x.numel() * 4),
                         ("sum (read only)", lambda: x.sum(), x.numel() * 4)):
    fn(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 20
    print(f"{name}: {nbytes / dt / 1e12:.2f} TB/s", flush=True)
