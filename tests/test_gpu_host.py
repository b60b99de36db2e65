"""The host-pointer drop-in (the reference's calling convention,
radixSort.hpp:1780: host arrays sorted in place) at full hot-path sizes,
against the reference's own sort (oracle/_ref).

Covers the staged PCIe path on one device and the split of one host array
over several devices (srs_set_host_devices): the same device listed 2 or 3
times exercises the whole protocol (chunked H2D, top-bits histograms, the
partition into key ranges, the gather, per-range sorts, D2H into place) on
a one-GPU box. Inputs use payload = f(key), so the comparison with the
(unstable) reference is exact.
"""
import numpy as np
import pytest

from srs_testlib import ref_lib, ref_sort_aos, ref_sort_soa, stable_reference

pytestmark = pytest.mark.gpu

srs_amd = pytest.importorskip("srs_amd")


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if ref_lib() is None:
        pytest.fail("the reference library (oracle/_ref) cannot run on this host")
    yield torch
    srs_amd.set_host_devices(())


def _host_workload(torch, n, kind, psizes, first_index=0):
    dt = {srs_amd.KEY_U64: torch.int64, srs_amd.KEY_F32: torch.float32}[kind]
    keys = torch.empty(n, dtype=dt, device="cuda")
    pays = [torch.empty(n, dtype={4: torch.int32, 8: torch.int64}[s], device="cuda")
            for s in psizes]
    srs_amd.fill_synthetic_device(keys, *pays, seed=42 << 32, first_index=first_index,
                                  key_kind=kind)
    npk = {srs_amd.KEY_U64: np.uint64, srs_amd.KEY_F32: np.float32}[kind]
    k = keys.cpu().numpy().view(npk).copy()
    p = [t.cpu().numpy().view({4: np.uint32, 8: np.uint64}[t.element_size()]).copy()
         for t in pays]
    return k, p


@pytest.mark.parametrize("devices", [(), (0, 0), (0, 0, 0)], ids=["one", "split2", "split3"])
def test_host_c1_vs_reference(torch, devices):
    n = (1 << 25) + 77
    srs_amd.set_host_devices(devices)
    k, p = _host_workload(torch, n, srs_amd.KEY_U64, [8], first_index=len(devices) << 32)
    k_ref, p_ref = k.copy(), p[0].copy()
    srs_amd.sort(k, p[0])
    ref_sort_soa(srs_amd.KEY_U64, True, k_ref, [p_ref])
    assert np.array_equal(k, k_ref), "keys differ from the reference"
    assert np.array_equal(p[0], p_ref), "payloads differ from the reference"


def test_host_split_c2_shape_down_vs_reference(torch):
    n = (1 << 23) + 5
    srs_amd.set_host_devices((0, 0))
    k, p = _host_workload(torch, n, srs_amd.KEY_F32, [4, 4])
    k_ref, p_ref = k.copy(), [c.copy() for c in p]
    srs_amd.sort(k, *p, up=False)
    ref_sort_soa(srs_amd.KEY_F32, False, k_ref, p_ref)
    assert np.array_equal(k.view(np.uint32), k_ref.view(np.uint32))
    for a, b in zip(p, p_ref):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("case", ["equal", "two_values", "sorted"])
def test_host_split_skewed_vs_stable(torch, case):
    """Key ranges that cannot be balanced: every key in one histogram bin
    (one shard receives everything), two values, already sorted input."""
    n = (1 << 22) + 3
    srs_amd.set_host_devices((0, 0, 0))
    g = np.random.default_rng(3)
    if case == "equal":
        k = np.full(n, 12345, np.int64)
    elif case == "two_values":
        k = g.integers(0, 2, n).astype(np.int64) << 40
    else:
        k = np.sort(g.integers(-2**62, 2**62, n, dtype=np.int64))
    p = np.arange(n, dtype=np.int64)
    ref_k, ref_p = stable_reference(srs_amd.KEY_I64, True, [k.copy(), p.copy()])
    srs_amd.sort(k, p)
    assert np.array_equal(k, ref_k) and np.array_equal(p, ref_p)


def test_host_split_nosort_leaves(torch):
    from test_gpu_leaf import check_leaves
    n = (1 << 22) + 11
    srs_amd.set_host_devices((0, 0))
    g = np.random.default_rng(9)
    k = g.integers(0, 2**64, n, dtype=np.uint64)
    k0 = k.copy()
    p = np.arange(n, dtype=np.int64)
    srs_amd.sort_thresh(16, k, p, cmp_sorter="nosort")
    check_leaves(srs_amd.KEY_U64, True, k0, k, p, 16)


def test_host_aos_c3_vs_reference(torch):
    n = (1 << 24) + 9
    srs_amd.set_host_devices(())
    k, p = _host_workload(torch, n, srs_amd.KEY_U64, [8], first_index=99)
    rec = np.empty((n, 2), np.uint64)
    rec[:, 0], rec[:, 1] = k, p[0]
    rec = rec.view(np.uint8).reshape(n, 16)
    r_ref = rec.copy()
    srs_amd.sort_combined(rec, srs_amd.KEY_U64)
    ref_sort_aos(srs_amd.KEY_U64, True, r_ref)
    assert np.array_equal(rec, r_ref)


def test_host_devices_are_validated(torch):
    import torch as t
    with pytest.raises(srs_amd.SrsError):
        srs_amd.set_host_devices((t.cuda.device_count(),))
    with pytest.raises(srs_amd.SrsError):
        srs_amd.set_host_devices((-1,))
    srs_amd.set_host_devices(())
