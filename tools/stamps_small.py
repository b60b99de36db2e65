"""Per-phase cycles of the small sort's fast body (stamp build, one
workgroup): u64 key + u64 payload, keys of 40 random bits, in place.
usage: SRS_AMD_LIB=.../variants/stamps/libsrs_amd.so python tools/stamps_small.py [n ...]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "simd-radix-sort_amd", "python"))
import srs_amd  # noqa: E402

NAMES = ["keys loaded", "or reduced", "barrier passed", "var", "direct decided", "atomics issued", "barrier", "scanned",
         "bucket hist done", "bucket scatter", "rank", "col0 moved", "col1 moved"]


def main():
    L = srs_amd.lib()
    L.srs_debug_set_stamp_buffer.argtypes = [ctypes.c_void_p]
    acc = torch.zeros(64, dtype=torch.int64, device="cuda")
    rng = np.random.default_rng(1)
    for n in [int(x) for x in sys.argv[1:]] or [1024, 4096, 8192]:
        k = rng.integers(0, 1 << 40, n, dtype=np.uint64)
        kd = torch.from_numpy(k.view(np.int64)).cuda()
        pd = torch.arange(n, dtype=torch.int64, device="cuda")
        k0, p0 = kd.clone(), pd.clone()
        srs_amd.sort_device(kd, pd, key_kind=srs_amd.KEY_U64)  # warm-up
        reps = 20
        acc.zero_()
        torch.cuda.synchronize()
        L.srs_debug_set_stamp_buffer(acc.data_ptr())
        for _ in range(reps):
            kd.copy_(k0)
            pd.copy_(p0)
            srs_amd.sort_device(kd, pd, key_kind=srs_amd.KEY_U64)
        torch.cuda.synchronize()
        L.srs_debug_set_stamp_buffer(None)
        a = acc.cpu().tolist()
        wg = max(a[16], 1)
        print(f"n={n}: {a[16]} workgroups (stamped)")
        for i, nm in enumerate(NAMES):
            print(f"   {nm:20s} {a[17 + i] / wg:10.0f} cyc")


if __name__ == "__main__":
    main()
