"""Calibration: does the 256 MB Infinity Cache absorb an intermediate buffer
that is written, read back and overwritten (a ring), so that its bytes never
reach HBM? Streams X -> R -> Y slice by slice; R either reused (ring) or a
fresh slice each time. Same kernel work either way."""
import time
import torch

total = 2 * 10**9  # int64 elements streamed (16 GB)
X = torch.empty(total, dtype=torch.int64, device="cuda").random_()
Y = torch.empty_like(X)
Rbig = torch.empty_like(X)
for slice_mb in (16, 32, 64, 128):
    m = slice_mb * 2**20 // 8
    ns = total // m
    for mode in ("fresh", "ring"):
        def run():
            for i in range(ns):
                R = Rbig[:m] if mode == "ring" else Rbig[i * m:(i + 1) * m]
                R.copy_(X[i * m:(i + 1) * m])
                Y[i * m:(i + 1) * m].copy_(R)
        run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"slice {slice_mb:4d} MB {mode:5s}: {dt * 1e3:8.2f} ms  "
              f"(2 copies of 16 GB; {4 * 8 * ns * m / dt / 1e12:5.2f} TB/s apparent)", flush=True)
