"""Narrow key ranges against the reference itself (key offset).

The reference's Gaussian distribution (src/data.hpp:379-386: round(N(0, 100)),
used by its test matrix, src/test.cpp:85-90) puts ~1000 distinct values
around 0, so signed keys straddle the sign bit and every transformed bit from
the top down varies. The sort then starts its digits at the highest bit of
u - min(u) (one exact min/max pass) instead of the top of the key. These
tests sort such inputs at >= 2^25 records (the hot path: global levels, then
single-valued buckets written straight home) on the GPU and with the
reference's own AVX-512 sort on the host (oracle/_ref), and compare every
byte. Payload = f(key), so the sorted output is unique and the comparison is
exact although the reference is unstable. Also: keys that share their top
bits (the first level starts below them), two values (ZeroOne), one value
(Zero: the input is the output), float and AoS variants.
"""
import numpy as np
import pytest

from srs_testlib import ref_lib, ref_sort_aos, ref_sort_soa

pytestmark = pytest.mark.gpu

srs_amd = pytest.importorskip("srs_amd")

N = (1 << 25) + 1234


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if ref_lib() is None:
        pytest.fail("oracle/_ref/libsrs_ref.so missing or host lacks AVX-512 VBMI2")
    return torch


def _f(bits):
    """payload = splitmix64(key bits): a function of the key"""
    x = bits.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def _keys(dist, dtype, seed=5):
    rng = np.random.default_rng(seed)
    if dist == "gaussian":
        k = np.round(rng.normal(0.0, 100.0, N))
    elif dist == "zeroone":
        k = rng.integers(0, 2, N)
    elif dist == "zero":
        k = np.zeros(N)
    elif dist == "shared_top":  # 2^20 values above a common 44-bit prefix
        return (np.uint64(0x123456789AB) << np.uint64(20)) + rng.integers(
            0, 1 << 20, N, dtype=np.uint64)
    elif dist == "straddle_mid":  # u64 keys around 2^63 (the top bit flips)
        return np.uint64(1 << 63) - np.uint64(5000) + rng.integers(0, 10000, N, dtype=np.uint64)
    else:
        raise ValueError(dist)
    return k.astype(dtype)


def _sort_soa_both(torch, kind, k, up=True, inplace=False):
    bits = k.view({8: np.uint64, 4: np.uint32}[k.dtype.itemsize])
    p = _f(bits)
    kd = torch.from_numpy(k.copy()).cuda()
    pd = torch.from_numpy(p.view(np.int64).copy()).cuda()
    if inplace:
        srs_amd.sort_device(kd, pd, key_kind=kind, up=up)
        ko, po = kd, pd
    else:
        ko, po = torch.empty_like(kd), torch.empty_like(pd)
        srs_amd.sort_device(kd, pd, key_kind=kind, up=up, out=(ko, po))
    k_ref, p_ref = k.copy(), p.copy()
    ref_sort_soa(kind, up, k_ref, [p_ref])
    torch.cuda.synchronize()
    assert np.array_equal(ko.cpu().numpy().view(k.dtype), k_ref), "keys differ from the reference"
    assert np.array_equal(po.cpu().numpy().view(np.uint64), p_ref), "payloads differ"
    if not inplace:  # the input is untouched
        assert np.array_equal(kd.cpu().numpy().view(k.dtype), k)


@pytest.mark.parametrize("up", [True, False], ids=["up", "down"])
def test_gaussian_i64_vs_reference(torch, up):
    _sort_soa_both(torch, srs_amd.KEY_I64, _keys("gaussian", np.int64), up=up)


def test_gaussian_i64_inplace_vs_reference(torch):
    _sort_soa_both(torch, srs_amd.KEY_I64, _keys("gaussian", np.int64, seed=6), inplace=True)


def test_gaussian_f64_vs_reference(torch):
    """float keys around 0: negative floats map to the low half, reversed"""
    _sort_soa_both(torch, srs_amd.KEY_F64, _keys("gaussian", np.float64, seed=7))


def test_gaussian_i32_vs_reference(torch):
    _sort_soa_both(torch, srs_amd.KEY_I32, _keys("gaussian", np.int32, seed=8))


@pytest.mark.parametrize("dist", ["zeroone", "zero"])
def test_few_values_i64_vs_reference(torch, dist):
    _sort_soa_both(torch, srs_amd.KEY_I64, _keys(dist, np.int64))


@pytest.mark.parametrize("dist", ["shared_top", "straddle_mid"])
def test_narrow_u64_vs_reference(torch, dist):
    _sort_soa_both(torch, srs_amd.KEY_U64, _keys(dist, np.uint64))


def test_gaussian_aos16_vs_reference(torch):
    k = _keys("gaussian", np.int64, seed=9)
    rec = np.empty((N, 16), np.uint8)
    rec[:, :8] = k.view(np.uint8).reshape(N, 8)
    rec[:, 8:] = _f(k.view(np.uint64)).view(np.uint8).reshape(N, 8)
    rd = torch.from_numpy(rec.copy()).cuda()
    out = torch.empty_like(rd)
    srs_amd.sort_combined_device(rd, srs_amd.KEY_I64, out=out)
    ref_sort_aos(srs_amd.KEY_I64, True, rec)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), rec)


# ---- several key clusters, outliers, stability -----------------
def _clustered(seed, n, centers, width, outliers=()):
    """u64 keys in narrow clusters around `centers` (+- width), plus a few
    outlier keys placed where a sample of the input is unlikely to see them
    (single keys at fixed positions): they widen the exact min / max the range
    level computes beyond the sampled clusters."""
    rng = np.random.default_rng(seed)
    which = rng.integers(0, len(centers), n)
    c = np.array(centers, dtype=np.uint64)[which]
    k = c - np.uint64(width) + rng.integers(0, 2 * width, n, dtype=np.uint64)
    for i, v in enumerate(outliers):
        k[(i * 7919 + 13) % n] = np.uint64(v)
    return k


@pytest.mark.parametrize("case", ["3_clusters", "4_clusters_both_ends", "outliers",
                                  "empty_middle"])
def test_range_level_clusters_vs_reference(torch, case):
    """The range level with 2-4 key clusters, unsigned keys at both ends of
    the range, empty ranges between clusters, and unsampled outliers that
    widen the exact min / max: bit-equal to the reference at 2^25 + 1234."""
    top = (1 << 64) - 1
    if case == "3_clusters":
        k = _clustered(21, N, [1 << 40, 1 << 50, 1 << 60], 3000)
    elif case == "4_clusters_both_ends":
        k = _clustered(22, N, [4000, 1 << 62, 3 << 62, top - 4000], 3000)
    elif case == "outliers":
        k = _clustered(23, N, [1 << 41, 5 << 59], 2000,
                       outliers=[0, 1, top, top - 1, 1 << 63, (1 << 52) + 17])
    else:  # two clusters with nothing between them but one outlier
        k = _clustered(24, N, [1000, top - 1000], 900, outliers=[1 << 63])
    _sort_soa_both(torch, srs_amd.KEY_U64, k)


@pytest.mark.parametrize("case", ["gaussian", "3_clusters", "outliers"])
def test_range_level_is_stable(torch, case):
    """Index payloads and many duplicate keys: the GPU output equals a stable
    CPU argsort (the home-write path of the range level keeps input order)."""
    from srs_testlib import transformed_keys
    if case == "gaussian":
        k = _keys("gaussian", np.int64, seed=31)
        kind = srs_amd.KEY_I64
    else:
        k = _clustered(32, N, [1 << 40, 1 << 50, 1 << 60], 300,
                       outliers=[0, (1 << 64) - 1] if case == "outliers" else ())
        kind = srs_amd.KEY_U64
    idx = np.arange(N, dtype=np.int64)
    kd = torch.from_numpy(k.view(np.int64).copy()).cuda()
    pd = torch.from_numpy(idx.copy()).cuda()
    srs_amd.sort_device(kd, pd, key_kind=kind)
    order = np.argsort(transformed_keys(kind, True, k), kind="stable")
    torch.cuda.synchronize()
    assert np.array_equal(kd.cpu().numpy().view(k.dtype), k[order])
    assert np.array_equal(pd.cpu().numpy(), idx[order])
