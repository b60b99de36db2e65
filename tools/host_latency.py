"""Per-call time of the host-pointer drop-in (radix_sort::sort on host
arrays, radixSort.hpp:1780 -> srs_sort_soa) at medium sizes, u64 keys + one
u64 payload, against the PCIe bound (2 * n * 16 bytes at 57 GB/s, DESIGN.md
§6). Median of the calls; each call sorts a fresh copy of the input.
usage: python tools/host_latency.py [n ...]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "simd-radix-sort_amd", "python"))
import srs_amd  # noqa: E402


def main():
    sizes = [int(float(x)) for x in sys.argv[1:]] or [1 << 18, 1 << 20, 1 << 21, 1 << 22,
                                                      1 << 23, 1 << 24]
    rng = np.random.default_rng(1)
    for n in sizes:
        k0 = rng.integers(0, 2**64 - 1, n, dtype=np.uint64)
        p0 = rng.integers(0, 2**64 - 1, n, dtype=np.uint64)
        k, p = np.empty_like(k0), np.empty_like(p0)
        reps = max(5, min(50, (1 << 26) // n))
        ts = []
        for r in range(2 + reps):
            np.copyto(k, k0)
            np.copyto(p, p0)
            t0 = time.perf_counter()
            srs_amd.sort(k, p)
            t1 = time.perf_counter()
            if r >= 2:
                ts.append((t1 - t0) * 1e3)
        ts.sort()
        ok = bool((k[1:] >= k[:-1]).all())
        bound = 2 * n * 16 / 57e9 * 1e3
        print(f"n={n:>9} ms median={ts[len(ts) // 2]:8.3f} min={ts[0]:8.3f} "
              f"pcie_bound_ms={bound:7.3f} ratio={ts[len(ts) // 2] / bound:5.2f} sorted={ok}",
              flush=True)


if __name__ == "__main__":
    main()
