"""PCIe-inclusive rate of the host-pointer drop-in (srs_sort_soa on host
arrays: H2D, device sort, D2H), with raw pageable/pinned copy rates beside it.
usage: python tools/host_rate.py [n]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "simd-radix-sort_amd", "python"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import srs_amd  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 2 * 10**8
# C1 workload generated on the device, copied to host arrays
dk = torch.empty(n, dtype=torch.int64, device="cuda")
dp = torch.empty(n, dtype=torch.int64, device="cuda")
srs_amd.fill_synthetic_device(dk, dp, seed=42 << 32, key_kind=srs_amd.KEY_U64)
k0 = dk.cpu().numpy().view(np.uint64)
p0 = dp.cpu().numpy().view(np.uint64)
nbytes = n * 16

t = torch.empty(n, dtype=torch.int64)
pin = torch.empty(n, dtype=torch.int64).pin_memory()
for name, src, dst in (("H2D pageable", t, dk), ("H2D pinned", pin, dk)):
    dst.copy_(src)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dst.copy_(src)
    torch.cuda.synchronize()
    print(f"{name:14s} {n * 8 / (time.perf_counter() - t0) / 1e9:6.1f} GB/s", flush=True)
for name, dst in (("D2H pageable", t), ("D2H pinned", pin)):
    dst.copy_(dk)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dst.copy_(dk)
    torch.cuda.synchronize()
    print(f"{name:14s} {n * 8 / (time.perf_counter() - t0) / 1e9:6.1f} GB/s", flush=True)
del dk, dp

for rep in range(2):
    k, p = k0.copy(), p0.copy()
    t0 = time.perf_counter()
    srs_amd.sort(k, p)
    dt = time.perf_counter() - t0
    print(f"host drop-in sort n={n}: {dt * 1e3:.1f} ms = {n / dt / 1e9:.3f} Gkeys/s "
          f"({2 * nbytes / dt / 1e9:.1f} GB/s over PCIe both ways)", flush=True)
ok = bool(np.all(k[1:] >= k[:-1]))
print("sorted", ok)
