"""Kernel time of the single-workgroup small sort by path (run under
rocprofv3 --kernel-trace): 50 device sorts per case, u64 key + u64 payload,
in the order printed. usage: python tools/small_paths.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "simd-radix-sort_amd", "python"))
import srs_amd  # noqa: E402

CASES = [
    ("n16_full", 16, 64), ("n4096_equal", 4096, 0), ("n4096_bits40", 4096, 40),
    ("n4096_full", 4096, 64), ("n8192_bits40", 8192, 40), ("n8192_full", 8192, 64),
    ("n2048_bits40", 2048, 40), ("n1024_bits40", 1024, 40),
]


def main():
    rng = np.random.default_rng(1)
    for name, n, bits in CASES:
        if bits == 0:
            k = np.full(n, 12345, dtype=np.uint64)
        else:
            k = rng.integers(0, 1 << bits if bits < 64 else 1 << 64, n, dtype=np.uint64)
        kd = torch.from_numpy(k.view(np.int64)).cuda()
        pd = torch.arange(n, dtype=torch.int64, device="cuda")
        k0, p0 = kd.clone(), pd.clone()
        for _ in range(50):
            kd.copy_(k0)
            pd.copy_(p0)
            srs_amd.sort_device(kd, pd, key_kind=srs_amd.KEY_U64)
        torch.cuda.synchronize()
        print(name, flush=True)


if __name__ == "__main__":
    main()
