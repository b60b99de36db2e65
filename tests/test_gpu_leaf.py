"""CmpSorterNoSort (src/cmp_sorters.hpp:66-78; thesis:3113-3124) on the GPU.

The reference's recursion stops at leaves of <= cmpSortThreshold elements
(radixSort.hpp:1743) and, with CmpSorterNoSort, leaves them in partition
order. The guarantee checked here, on the GPU path (SRS_LEAF_UNSORTED):

  * the output splits into consecutive leaves of <= T elements, each holding
    exactly the keys a full sort puts there (cut j is a leaf boundary when
    every key before it orders <= every key after it);
  * hence every element ends within T - 1 places of its sorted slot;
  * payloads stay with their keys (payload = original index);
  * num <= T leaves the input untouched (the whole input is one leaf);
  * and the mode really skips work: uniform keys come back unsorted.
"""
import numpy as np
import pytest

from srs_testlib import KIND_DTYPES, stable_reference, transformed_keys

pytestmark = pytest.mark.gpu

srs_amd = pytest.importorskip("srs_amd")


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def check_leaves(kind, up, keys_in, keys_out, pay_out, T):
    """The NoSort guarantee for keys_out / pay_out (payload = input index)."""
    n = len(keys_in)
    assert np.array_equal(np.sort(pay_out), np.arange(n)), "payloads are not a permutation"
    assert np.array_equal(keys_in[pay_out].view(np.uint8), keys_out.view(np.uint8)), \
        "a payload left its key"
    u = transformed_keys(kind, up, keys_out)
    su = np.sort(u)
    assert np.array_equal(np.sort(u), su)
    # leaf boundaries: prefix max <= suffix min (in the reference's key order)
    pmax = np.maximum.accumulate(u)
    smin = np.minimum.accumulate(u[::-1])[::-1]
    cuts = np.concatenate([[0], np.flatnonzero(pmax[:-1] <= smin[1:]) + 1, [n]])
    gaps = np.diff(cuts)
    assert gaps.max() <= T, f"a leaf of {gaps.max()} elements > cmpSortThreshold {T}"
    # within T - 1 of the sorted slot range of its key
    lo = np.searchsorted(su, u, "left")
    hi = np.searchsorted(su, u, "right") - 1
    i = np.arange(n)
    assert np.all(i >= lo - (T - 1)) and np.all(i <= hi + (T - 1))
    return bool(np.all(u[1:] >= u[:-1]))


def _keys(torch, n, kind, seed, dist="uniform"):
    g = np.random.default_rng(seed)
    dt = KIND_DTYPES[kind]
    if dist == "uniform":
        if np.dtype(dt).kind == "f":
            k = g.uniform(-1, 1, n).astype(dt)
        else:
            k = g.integers(0, 2**64, n, dtype=np.uint64).astype(dt)
    else:  # "clustered": the global level's 7-bit digit (bits 57-63) makes
        # local segments of ~2300 keys that vary in bits 0-3 and 20-23 only:
        # the local bucket digit (top 11 varying bits) sees 16 values, so the
        # buckets hold ~150 keys
        k = ((g.integers(0, 128, n, dtype=np.uint64) << np.uint64(57)) |
             (g.integers(0, 16, n, dtype=np.uint64) << np.uint64(20)) |
             g.integers(0, 16, n, dtype=np.uint64)).astype(dt)
    return k


@pytest.mark.parametrize("n", [100, 5000, 300_000, (1 << 25) + 99],
                         ids=["tiny", "one-launch", "levels", "stripes"])
@pytest.mark.parametrize("T", [16, 64])
def test_nosort_soa_u64(torch, n, T):
    kind = srs_amd.KEY_U64
    k = _keys(torch, n, kind, seed=n + T)
    keys = torch.from_numpy(k.view(np.int64)).cuda()
    pay = torch.arange(n, dtype=torch.int64, device="cuda")
    srs_amd.sort_device(keys, pay, key_kind=kind, cmp_sort_threshold=T, cmp_sorter="nosort")
    ko = keys.cpu().numpy().view(np.uint64)
    po = pay.cpu().numpy()
    fully_sorted = check_leaves(kind, True, k, ko, po, T)
    if n >= 5000:
        assert not fully_sorted, "NoSort mode sorted every leaf (the rank step ran)"


@pytest.mark.parametrize("kind", [srs_amd.KEY_I32, srs_amd.KEY_F32, srs_amd.KEY_F64],
                         ids=["i32", "f32", "f64"])
@pytest.mark.parametrize("up", [True, False], ids=["up", "down"])
def test_nosort_key_kinds(torch, kind, up):
    n, T = 200_000, 16
    k = _keys(torch, n, kind, seed=kind)
    keys = torch.from_numpy(k.copy()).cuda()
    pay = torch.arange(n, dtype=torch.int64, device="cuda")
    ko_t, po_t = torch.empty_like(keys), torch.empty_like(pay)
    srs_amd.sort_device(keys, pay, up=up, cmp_sort_threshold=T, cmp_sorter="nosort",
                        out=(ko_t, po_t))
    assert np.array_equal(keys.cpu().numpy(), k), "out of place: the input changed"
    check_leaves(kind, up, k, ko_t.cpu().numpy(), po_t.cpu().numpy(), T)


def test_nosort_large_threshold_buckets(torch):
    """T = 256 > the fast kernel's 64-key rank limit: buckets of 65..256 keys
    are leaves too and must not go to the stable (fully sorting) fallback."""
    n, T = 300_000, 256
    kind = srs_amd.KEY_U64
    k = _keys(torch, n, kind, seed=5, dist="clustered")
    keys = torch.from_numpy(k.view(np.int64)).cuda()
    pay = torch.arange(n, dtype=torch.int64, device="cuda")
    srs_amd.sort_device(keys, pay, key_kind=kind, cmp_sort_threshold=T, cmp_sorter="nosort")
    assert not check_leaves(kind, True, k, keys.cpu().numpy().view(np.uint64),
                            pay.cpu().numpy(), T), "the buckets were sorted (stable fallback?)"


def test_nosort_whole_input_is_one_leaf(torch):
    """num <= cmpSortThreshold: radixSort.hpp:1743 calls the leaf sorter on
    the whole input, and CmpSorterNoSort does nothing."""
    k = np.array([5, 3, 9, 1, 1, 7], np.uint64)
    p = np.arange(6, dtype=np.uint64)
    srs_amd.sort_thresh(16, k, p, cmp_sorter="nosort")
    assert k.tolist() == [5, 3, 9, 1, 1, 7] and p.tolist() == list(range(6))
    srs_amd.sort_thresh(6, k, p, cmp_sorter="nosort")
    assert k.tolist() == [5, 3, 9, 1, 1, 7]
    srs_amd.sort_thresh(5, k, p, cmp_sorter="nosort")  # 6 > 5: partitioned
    check_leaves(srs_amd.KEY_U64, True, np.array([5, 3, 9, 1, 1, 7], np.uint64), k,
                 p.astype(np.int64), 5)
    kk = torch.tensor([4, 2, 3], dtype=torch.int64, device="cuda")
    out = torch.empty_like(kk)
    srs_amd.sort_device(kk, cmp_sort_threshold=16, cmp_sorter="nosort", out=(out,))
    assert out.tolist() == [4, 2, 3]


@pytest.mark.parametrize("n", [6000, 3_000_000])
def test_nosort_host_and_combined(torch, n):
    """The host drop-in and the DataElement entry point in NoSort mode."""
    T = 16
    k = _keys(torch, n, srs_amd.KEY_U64, seed=n)
    kh, ph = k.copy(), np.arange(n, dtype=np.int64)
    srs_amd.sort_thresh(T, kh, ph, cmp_sorter="nosort")
    check_leaves(srs_amd.KEY_U64, True, k, kh, ph, T)
    rec = np.empty((n, 2), np.uint64)
    rec[:, 0] = k
    rec[:, 1] = np.arange(n, dtype=np.uint64)
    srs_amd.sort_combined(rec, srs_amd.KEY_U64, cmp_sort_threshold=T, cmp_sorter="nosort")
    check_leaves(srs_amd.KEY_U64, True, k, rec[:, 0].copy(), rec[:, 1].astype(np.int64), T)


def test_insertion_sort_is_still_full(torch):
    """The default leaf sorter still sorts completely (same inputs)."""
    n = 300_000
    k = _keys(torch, n, srs_amd.KEY_U64, seed=1)
    keys = torch.from_numpy(k.view(np.int64)).cuda()
    pay = torch.arange(n, dtype=torch.int64, device="cuda")
    srs_amd.sort_device(keys, pay, key_kind=srs_amd.KEY_U64, cmp_sort_threshold=16)
    ref_k, ref_p = stable_reference(srs_amd.KEY_U64, True, [k, np.arange(n)])
    assert np.array_equal(keys.cpu().numpy().view(np.uint64), ref_k)
    assert np.array_equal(pay.cpu().numpy(), ref_p)
