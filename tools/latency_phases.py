"""Per-family kernel time (HIP events around each launch family) of a device
sort at small / medium n, u64 keys + u64 payload: where a call's GPU time
goes (the mid-size launch, the first level, the LDS pass and its fallbacks).
The events add their own gaps; tools/latency.py gives the call's latency.
usage: python tools/latency_phases.py [n ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "simd-radix-sort_amd", "python"))
import srs_amd  # noqa: E402

FAMILIES = ["mid", "mid_level", "plan", "count", "scan", "scatter", "local", "local_fast",
            "local_stable", "local_lsd", "copy"]


def main():
    sizes = [int(float(x)) for x in sys.argv[1:]] or [1 << 20, (1 << 20) + 1, 1 << 21, 3_000_000,
                                                    3_900_000, 1 << 22]
    dev = torch.device("cuda:0")
    for n in sizes:
        keys = torch.empty(n, dtype=torch.int64, device=dev)
        pays = torch.empty(n, dtype=torch.int64, device=dev)
        srs_amd.fill_synthetic_device(keys, pays, key_kind=srs_amd.KEY_U64)
        outs = (torch.empty_like(keys), torch.empty_like(pays))
        reps = 20
        srs_amd.sort_device(keys, pays, key_kind=srs_amd.KEY_U64, out=outs)
        torch.cuda.synchronize()
        srs_amd.reset_kernel_stats()
        srs_amd.set_kernel_timing(True)
        try:
            for _ in range(reps):
                srs_amd.sort_device(keys, pays, key_kind=srs_amd.KEY_U64, out=outs)
            torch.cuda.synchronize()
        finally:
            srs_amd.set_kernel_timing(False)
        parts = []
        for f in FAMILIES:
            try:
                c, ms, _ = srs_amd.kernel_stats(f)
            except Exception:  # (a family that never ran)
                continue
            if c:
                parts.append(f"{f}={ms * 1e3 / reps:.1f}us/{c // reps}")
        print(f"n={n:>9} " + " ".join(parts), flush=True)


if __name__ == "__main__":
    main()
