"""PCIe-inclusive rate of the host-pointer drop-in (srs_sort_soa on host
arrays: staged H2D, device sort, staged D2H), against its bound: the 2*n*s
bytes that must cross PCIe at 57 GB/s (the link measured at 57 GB/s each way
and not duplex).
usage: python tools/host_rate.py [n] [devices, e.g. 0,1,2,3]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "simd-radix-sort_amd", "python"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import srs_amd  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 2 * 10**8
devs = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else []
srs_amd.set_host_devices(devs)
# C1 workload generated on the device, copied to host arrays
dk = torch.empty(n, dtype=torch.int64, device="cuda")
dp = torch.empty(n, dtype=torch.int64, device="cuda")
srs_amd.fill_synthetic_device(dk, dp, seed=42 << 32, key_kind=srs_amd.KEY_U64)
k0 = dk.cpu().numpy().view(np.uint64)
p0 = dp.cpu().numpy().view(np.uint64)
del dk, dp
torch.cuda.empty_cache()
nbytes = n * 16
bound = 2 * nbytes / 57e9
res = []
for rep in range(3):
    k, p = k0.copy(), p0.copy()
    t0 = time.perf_counter()
    srs_amd.sort(k, p)
    dt = time.perf_counter() - t0
    res.append(dt)
    print(f"host drop-in sort n={n} devices={devs or 'current'}: {dt * 1e3:.1f} ms = "
          f"{n / dt / 1e9:.3f} Gkeys/s ({2 * nbytes / dt / 1e9:.1f} GB/s over PCIe both ways; "
          f"{dt / bound:.3f} x the 57 GB/s bound {bound * 1e3:.1f} ms)", flush=True)
ok = bool(np.all(k[1:] >= k[:-1]))
print("sorted", ok)
print(json.dumps({"n": n, "devices": devs, "best_ms": round(min(res) * 1e3, 1),
                  "bound_ms": round(bound * 1e3, 1), "ratio": round(min(res) / bound, 3),
                  "sorted": ok}))
