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
