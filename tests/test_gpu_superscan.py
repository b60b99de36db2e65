"""The super-group column scan (round 6). A level over ONE
large segment -- a shard's partition chunk or round sort, the first level of
a sort without stripes -- used to scan its tile counts on one workgroup, one
CU walking every scan group (0.17-0.47 ms per 250 M-key chunk). Above 256
groups (33.5 M keys) it now scans sums of 64 groups and spreads the offsets
back over the groups grid-wide. srs_debug_set_super_scan lowers the
threshold so that the path runs at test sizes (one to several super rows, a
partial last row, both directions): the result must equal a stable sort bit
for bit, and the same sort with the path off."""
import numpy as np
import pytest

from srs_testlib import stable_reference

pytestmark = pytest.mark.gpu

srs_amd = pytest.importorskip("srs_amd")


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    yield torch
    srs_amd.debug_set_super_scan(0)  # (the product threshold again)


def _cols(torch, n, seed, narrow=False):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    hi = (1 << 30) if narrow else 2**63 - 1
    lo = 0 if narrow else -2**63
    keys = torch.randint(lo, hi, (n,), dtype=torch.int64, device="cuda", generator=g)
    pays = torch.arange(n, dtype=torch.int64, device="cuda") * 7 + seed
    return keys, pays


@pytest.mark.parametrize("n,up", [(300_000, True), (9_000_017, True), (9_000_017, False),
                                  (20_000_000, True)])
def test_one_segment_super_scan(torch, n, up):
    keys, pays = _cols(torch, n, seed=n % 1000 + up)
    k0, p0 = keys.cpu().numpy(), pays.cpu().numpy()
    ref = stable_reference(srs_amd.KEY_U64, up, [k0.view(np.uint64), p0])
    outs = []
    for min_groups in (2, 1 << 40):  # the super scan, then the one-workgroup scan
        srs_amd.debug_set_super_scan(min_groups)
        k, p = keys.clone(), pays.clone()
        srs_amd.sort_segments_device(k, p, bounds=[0, n], up=up, key_kind=srs_amd.KEY_U64)
        torch.cuda.synchronize()
        outs.append((k.cpu().numpy(), p.cpu().numpy()))
    srs_amd.debug_set_super_scan(0)
    for k, p in outs:
        assert np.array_equal(k.view(np.uint64), ref[0])
        assert np.array_equal(p, ref[1])


def test_narrow_keys_whole_sort(torch):
    # keys below 2^30: the planner's levels over one segment (no stripes)
    n = 12_000_003
    keys, pays = _cols(torch, n, seed=5, narrow=True)
    k0, p0 = keys.cpu().numpy(), pays.cpu().numpy()
    ref = stable_reference(srs_amd.KEY_I64, True, [k0, p0])
    srs_amd.debug_set_super_scan(2)
    try:
        srs_amd.sort_device(keys, pays, key_kind=srs_amd.KEY_I64)
        torch.cuda.synchronize()
    finally:
        srs_amd.debug_set_super_scan(0)
    assert np.array_equal(keys.cpu().numpy(), ref[0])
    assert np.array_equal(pays.cpu().numpy(), ref[1])
