"""Device mid-size sorts (16384 int64 keys + int64 payload) before and after
host-array sorts of the given sizes (perf_dat's order of calls): the median
event time of 40 calls each time.
usage: python tools/mid_after_host.py [host sizes ...]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "simd-radix-sort_amd", "python"))
import srs_amd  # noqa: E402

rng = np.random.default_rng(1)
n = 16384
k = rng.integers(-(1 << 63), (1 << 63) - 1, n, dtype=np.int64)
p = rng.integers(-(1 << 63), (1 << 63) - 1, n, dtype=np.int64)
src, psrc = torch.from_numpy(k).cuda(), torch.from_numpy(p).cuda()
dk, dp = torch.empty_like(src), torch.empty_like(psrc)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def dev_median():
    ts = []
    for r in range(40):
        dk.copy_(src)
        dp.copy_(psrc)
        a.record()
        srs_amd.sort_device(dk, dp, key_kind=srs_amd.KEY_I64)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return sorted(ts)[20]


print("before any host sort: %.1f us" % dev_median(), flush=True)
for hs in [int(x) for x in sys.argv[1:]] or [1, 2, 16, 1024, 8192]:
    for _ in range(3):
        kk = rng.integers(-(1 << 63), (1 << 63) - 1, hs, dtype=np.int64)
        pp = kk.copy()
        srs_amd.sort(kk, pp)
    print("after host sorts of %d: %.1f us" % (hs, dev_median()), flush=True)

# perf_dat's exact order at one size: 80 reference sorts (one core), 80 host
# sorts of the previous size, then the device sorts
if os.environ.get("WITH_REF"):
    import ctypes
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
    from srs_testlib import ref_sort_soa_timed
    for _ in range(80):
        kk, pp = k.copy(), p.copy()
        ref_sort_soa_timed(srs_amd.KEY_I64, True, kk, [pp])
    print("after 80 reference sorts: %.1f us" % dev_median(), flush=True)
    for _ in range(80):
        kk = rng.integers(-(1 << 63), (1 << 63) - 1, 8192, dtype=np.int64)
        pp = kk.copy()
        srs_amd.sort(kk, pp)
    print("after 80 host sorts of 8192: %.1f us" % dev_median(), flush=True)

# many host sorts (perf_dat runs ~1800 of them below 16K keys)
if os.environ.get("MANY_HOST"):
    for i in range(int(os.environ["MANY_HOST"])):
        kk = rng.integers(-(1 << 63), (1 << 63) - 1, 16, dtype=np.int64)
        pp = kk.copy()
        srs_amd.sort(kk, pp)
    print("after %s host sorts of 16: %.1f us" % (os.environ["MANY_HOST"], dev_median()), flush=True)
    src2, psrc2 = torch.from_numpy(k).cuda(), torch.from_numpy(p).cuda()
    dk, dp = torch.empty_like(src2), torch.empty_like(psrc2)
    print("  ... with new device tensors: %.1f us" % dev_median(), flush=True)
