"""Calibration: device-to-device copy and read-only bandwidth on this GPU
(the practical ceiling for the scatter/local kernels' read+write streams)."""
import time
import torch

n = 2 * 10**9  # 16 GB of int64
a = torch.empty(n, dtype=torch.int64, device="cuda").random_()
b = torch.empty_like(a)
for name, fn, nbytes in (("copy_ (torch)", lambda: b.copy_(a), 2 * 8 * n),
                         ("hipMemcpyDtoD", lambda: b.copy_(a, non_blocking=True), 2 * 8 * n),
                         ("sum (read)", lambda: a.sum(), 8 * n)):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 5
    print(f"{name:16s} {dt * 1e3:8.2f} ms  {nbytes / dt / 1e12:6.2f} TB/s")
