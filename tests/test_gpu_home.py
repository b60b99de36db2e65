"""The home-write path (round 6): when a large SoA sort's output
columns are not srs_alloc_device memory -- the reference's in-place contract
on the caller's own array (radixSort.hpp:1780), or outputs from the caller's
allocator -- the scatters stay in the placed workspace (IN -> TMP -> TMP2)
and only the LDS local pass writes OUT. Every shape the path takes (one to
three payload columns of any width, keys only, every key kind, both
directions, in place and out of place) must equal a stable sort bit for bit,
and the same sort into srs_alloc_device outputs (the other path) must equal
it too."""
import numpy as np
import pytest

from srs_testlib import stable_reference

pytestmark = pytest.mark.gpu

srs_amd = pytest.importorskip("srs_amd")

N = (1 << 24) + 4097  # (the path starts at 2^24 records)


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _cols(torch, kind, psizes, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    kdt = {srs_amd.KEY_U64: torch.int64, srs_amd.KEY_I64: torch.int64,
           srs_amd.KEY_U32: torch.int32, srs_amd.KEY_F64: torch.float64,
           srs_amd.KEY_F32: torch.float32, srs_amd.KEY_U16: torch.int16}[kind]
    if kdt.is_floating_point:
        keys = torch.randn(N, dtype=kdt, device="cuda", generator=g)
    else:
        info = torch.iinfo(kdt)
        keys = torch.randint(info.min, info.max, (N,), dtype=kdt, device="cuda", generator=g)
    pdt = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}
    pays = [torch.randint(0, 100, (N,), dtype=pdt[s], device="cuda", generator=g) for s in psizes]
    return keys, pays


def _np(t):
    return t.cpu().numpy().copy()


@pytest.mark.parametrize("kind,psizes,up,inplace", [
    ("U64", [8], True, True), ("U64", [8], False, False), ("I64", [8], True, True),
    ("U64", [], True, True), ("U32", [8], True, False), ("F64", [8], True, True),
    ("U64", [8, 8], True, True), ("U32", [4], False, True), ("U64", [2, 1, 8], True, False),
    ("F32", [8], True, True), ("U16", [8], True, False)])
def test_home_write_equals_stable_sort(torch, kind, psizes, up, inplace):
    k = getattr(srs_amd, "KEY_" + kind)
    keys, pays = _cols(torch, k, psizes, seed=len(psizes) * 7 + k)
    ref = stable_reference(k, up, [_np(keys)] + [_np(p) for p in pays])
    if inplace:
        srs_amd.sort_device(keys, *pays, key_kind=k, up=up)
        outs = [keys] + pays
    else:
        outs = [torch.empty_like(keys)] + [torch.empty_like(p) for p in pays]
        srs_amd.sort_device(keys, *pays, key_kind=k, up=up, out=tuple(outs))
    torch.cuda.synchronize()
    for a, b in zip(outs, ref):
        assert np.array_equal(_np(a).view(np.uint8), b.view(np.uint8))


def test_home_write_matches_placed_outputs(torch):
    """The same C1-shaped input into torch outputs (home-write path) and into
    srs_alloc_device outputs (scatter into OUT): identical bytes."""
    keys = torch.empty(N, dtype=torch.int64, device="cuda")
    pays = torch.empty(N, dtype=torch.int64, device="cuda")
    srs_amd.fill_synthetic_device(keys, pays, seed=99 << 32, key_kind=srs_amd.KEY_U64)
    a = (torch.empty_like(keys), torch.empty_like(pays))
    b = (srs_amd.empty_device(N, torch.int64), srs_amd.empty_device(N, torch.int64))
    srs_amd.sort_device(keys, pays, key_kind=srs_amd.KEY_U64, out=a)
    srs_amd.sort_device(keys, pays, key_kind=srs_amd.KEY_U64, out=b)
    torch.cuda.synchronize()
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    ks = a[0].cpu().numpy().view(np.uint64)
    assert (ks[1:] >= ks[:-1]).all()


@pytest.mark.parametrize("n,kind,psizes", [((1 << 21) + 77, "U64", [8]), ((1 << 21) + 123, "U32", [4, 4]),
                                           ((1 << 21) + 5, "F32", [8, 2]), (3_000_017, "U64", [])])
def test_medium_sort_both_local_classes(torch, n, kind, psizes):
    """Round 6: medium sorts (<= 2^24 records) run the two LDS classes on two
    streams. Both classes hold segments here (srs_debug_last_local_classes)
    and the result equals a stable sort bit for bit."""
    k = getattr(srs_amd, "KEY_" + kind)
    g = torch.Generator(device="cuda")
    g.manual_seed(n)
    kdt = {srs_amd.KEY_U64: torch.int64, srs_amd.KEY_U32: torch.int32,
           srs_amd.KEY_F32: torch.float32}[k]
    if kdt.is_floating_point:
        keys = torch.randn(n, dtype=kdt, device="cuda", generator=g)
    else:
        info = torch.iinfo(kdt)
        keys = torch.randint(info.min, info.max, (n,), dtype=kdt, device="cuda", generator=g)
    pdt = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}
    pays = [torch.randint(0, 1000, (n,), dtype=pdt[s], device="cuda", generator=g)
            for s in psizes]
    ref = stable_reference(k, True, [_np(keys)] + [_np(p) for p in pays])
    outs = [torch.empty_like(keys)] + [torch.empty_like(p) for p in pays]
    srs_amd.sort_device(keys, *pays, key_kind=k, out=tuple(outs))
    torch.cuda.synchronize()
    small, large = srs_amd.last_local_classes()[:2]
    if kind != "F32" and n < 3_000_000:  # (uniform keys, ~4096 per bucket: both classes)
        assert small > 0 and large > 0, (small, large)
    for a, b in zip(outs, ref):
        assert np.array_equal(_np(a).view(np.uint8), b.view(np.uint8))


def _confined(torch, n, kind, top3, seed):
    """keys whose top 3 transformed bits are `top3` (the span one of 8 shard
    ranks receives), as the key kind's storage"""
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    if kind == srs_amd.KEY_U64:
        k = torch.randint(0, 2**61, (n,), dtype=torch.int64, device="cuda", generator=g)
        return k | (top3 << 61)
    if kind == srs_amd.KEY_I64:  # transformed = bits ^ sign bit
        k = torch.randint(0, 2**61, (n,), dtype=torch.int64, device="cuda", generator=g)
        return (k | (top3 << 61)) ^ (-2**63)
    assert top3 < 4  # (U32 in int32 storage)
    k = torch.randint(0, 2**29, (n,), dtype=torch.int32, device="cuda", generator=g)
    return k | (top3 << 29)


@pytest.mark.parametrize("n,kind,psizes,top3", [
    ((1 << 25) + 1234, "U64", [8], 1), ((1 << 25) + 77, "I64", [8], 6),
    ((1 << 25) + 5, "U32", [4, 4], 2), (3_000_017, "U64", [8], 5), (700_001, "U64", [8], 3)])
def test_whole_range_segment_known_bits(torch, n, kind, psizes, top3):
    """srs_sort_segments_device with ONE segment over the whole range and
    known top bits (the multi-GPU shard's rounds), at sizes that take two
    levels or one: equal to a stable sort bit for bit. (Round 6 measured
    routing such a segment through the whole-array levels -- stripe first
    level, known bits skipped: no faster)"""
    k = getattr(srs_amd, "KEY_" + kind)
    keys = _confined(torch, n, k, top3, seed=n + top3)
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    pdt = {4: torch.int32, 8: torch.int64}
    pays = [torch.randint(-2**31, 2**31 - 1, (n,), dtype=pdt[s], device="cuda", generator=g)
            for s in psizes]
    ref = stable_reference(k, True, [_np(keys)] + [_np(p) for p in pays])
    srs_amd.sort_segments_device(keys, *pays, bounds=[0, n], key_kind=k, known_top_bits=3)
    torch.cuda.synchronize()
    for a, b in zip([keys] + pays, ref):
        assert np.array_equal(_np(a).view(np.uint8), b.view(np.uint8))


def test_whole_range_segment_skewed_below_known_bits(torch):
    """Known top bits over keys that are also skewed below them (90 % share
    the next 20 bits): exact."""
    n = (1 << 25) + 99
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    low = torch.randint(0, 2**40, (n,), dtype=torch.int64, device="cuda", generator=g)
    mid = torch.where(torch.rand(n, device="cuda", generator=g) < 0.9, 12345,
                      torch.randint(0, 2**20, (n,), device="cuda", generator=g))
    keys = (1 << 61) | (mid.to(torch.int64) << 40) | low
    pay = torch.arange(n, dtype=torch.int64, device="cuda")
    ref = stable_reference(srs_amd.KEY_U64, True, [_np(keys), _np(pay)])
    srs_amd.sort_segments_device(keys, pay, bounds=[0, n], key_kind=srs_amd.KEY_U64,
                                 known_top_bits=3)
    torch.cuda.synchronize()
    assert np.array_equal(_np(keys), ref[0]) and np.array_equal(_np(pay), ref[1])
