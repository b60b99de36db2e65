"""Distribution of per-call times of mid-size device sorts (int64 keys +
int64 payload, the reference's Uniform; perf_dat's call shape), to find
outliers that a mean shows and a median hides.
usage: python tools/mid_outliers.py [n ...]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "simd-radix-sort_amd", "python"))
import srs_amd  # noqa: E402


def main():
    rng = np.random.default_rng(5)
    for n in [int(float(x)) for x in sys.argv[1:]] or [8192, 16384, 65536, 262144]:
        k = rng.integers(-(1 << 63), (1 << 63) - 1, n, dtype=np.int64)
        p = rng.integers(-(1 << 63), (1 << 63) - 1, n, dtype=np.int64)
        src, psrc = torch.from_numpy(k).cuda(), torch.from_numpy(p).cuda()
        dk, dp = torch.empty_like(src), torch.empty_like(psrc)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev, wall = [], []
        for r in range(216):
            dk.copy_(src)
            dp.copy_(psrc)
            t0 = time.perf_counter()
            a.record()
            srs_amd.sort_device(dk, dp, key_kind=srs_amd.KEY_I64)
            b.record()
            t1 = time.perf_counter()
            b.synchronize()
            if r >= 16:
                ev.append(a.elapsed_time(b) * 1e3)
                wall.append((t1 - t0) * 1e6)
        ev = np.array(ev)
        wall = np.array(wall)
        print(f"n={n}: event us median {np.median(ev):.1f} mean {ev.mean():.1f} p99 "
              f"{np.percentile(ev, 99):.1f} max {ev.max():.1f}; call (host) us median "
              f"{np.median(wall):.1f} max {wall.max():.1f}; >1 ms: {int((ev > 1000).sum())}",
              flush=True)


if __name__ == "__main__":
    main()
