"""Randomised parity sweep over the entry points and the size classes the
round-5/6 paths split on (single-workgroup small sorts on 128-1024 threads,
the mid-size single launch up to 2^20 keys, the general levels; host arrays through
coherent pinned memory, the packed DMA or the staged copies; device arrays
in place or out of place): 600 seeded cases of random key kind, direction,
size (log-uniform 1 .. 1.2M), key distribution and payload columns, each
equal to a stable sort bit for bit (the GPU sort is stable; with n <=
cmp_sort_threshold floats compare -0.0 == +0.0, as the reference's leaf).
NaN keys are outside the contract and not generated."""
import numpy as np
import pytest

from srs_testlib import KIND_DTYPES, KIND_NAMES, KIND_UINT, stable_reference
from test_gpu_sort import bytes_equal

pytestmark = pytest.mark.gpu

srs_amd = pytest.importorskip("srs_amd")

N_CASES = 600


def _torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _keys(kind, n, dist, rng):
    dt = np.dtype(KIND_DTYPES[kind])
    ut = np.dtype(KIND_UINT[kind])
    bits = 8 * dt.itemsize
    if KIND_NAMES[kind].startswith("f"):
        if dist == "full":
            return rng.uniform(-1e6, 1e6, n).astype(dt)
        if dist == "narrow":
            return (rng.integers(-50, 50, n) * 0.25).astype(dt)  # dups, +-0.0
        if dist == "const":
            return np.full(n, -0.0, dt)
        v = rng.uniform(-1, 1, n).astype(dt)
        v[rng.random(n) < 0.5] = 0.0
        return v
    if dist == "full":
        u = rng.integers(0, 1 << bits, n, dtype=np.uint64) if bits < 64 else \
            rng.integers(0, 1 << 63, n, dtype=np.uint64) * np.uint64(2) + \
            rng.integers(0, 2, n, dtype=np.uint64)
    elif dist == "narrow":
        u = rng.integers(0, 1 << min(bits, 12), n, dtype=np.uint64)
    elif dist == "const":
        u = np.full(n, 7, np.uint64)
    else:  # "skew": most keys in one narrow band, the rest spread
        u = rng.integers(0, 1 << (bits - 1), n, dtype=np.uint64)
        m = rng.random(n) < 0.8
        u[m] = rng.integers(0, 1 << min(bits - 1, 20), int(m.sum()), dtype=np.uint64)
    return u.astype(ut).view(dt)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    _torch()
    srs_amd.lib()


@pytest.mark.parametrize("case", range(N_CASES))
def test_fuzz_case(case):
    torch = _torch()
    rng = np.random.default_rng(1_000_003 * case + 17)
    kind = int(rng.integers(0, 10))
    up = bool(rng.integers(0, 2))
    n = int(np.exp(rng.uniform(0, np.log(1_200_000))))
    dist = ["full", "narrow", "const", "skew"][int(rng.integers(0, 4))]
    keys = _keys(kind, n, dist, rng)
    widths = [int(w) for w in rng.choice([1, 2, 4, 8], int(rng.integers(0, 3)))]
    pays = [rng.integers(0, 1 << (8 * w), n, dtype=np.uint64).astype(f"u{w}") for w in widths]
    pays.append(np.arange(n, dtype=np.uint32))  # input order: stability is checked
    thresh = int(rng.choice([16, 16, 64, 1 << 20]))
    want = stable_reference(kind, up, [keys] + pays, thresh)
    api = ["host", "device_inplace", "device_out"][int(rng.integers(0, 3))]
    if api == "host":
        cols = [keys.copy()] + [p.copy() for p in pays]
        srs_amd.sort_thresh(thresh, cols[0], *cols[1:], up=up)
        got = cols
    else:
        dev = [torch.from_numpy(c.view(f"u{c.dtype.itemsize}").view(
            {1: np.uint8, 2: np.int16, 4: np.int32, 8: np.int64}[c.dtype.itemsize])).cuda()
            for c in [keys] + pays]
        out = None if api == "device_inplace" else tuple(torch.empty_like(t) for t in dev)
        srs_amd.sort_device(dev[0], *dev[1:], up=up, key_kind=kind, cmp_sort_threshold=thresh,
                            out=out)
        torch.cuda.synchronize()
        res = dev if out is None else out
        got = [t.cpu().numpy() for t in res]
        for t, c in zip(dev, [keys] + pays):  # out of place: the inputs stay as they were
            if out is not None:
                assert bytes_equal(t.cpu().numpy(), c), (case, "input changed")
    for i, (g, w) in enumerate(zip(got, want)):
        assert bytes_equal(g, w), (case, KIND_NAMES[kind], up, n, dist, widths, thresh, api, i)
