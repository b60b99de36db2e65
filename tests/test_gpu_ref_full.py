"""Full-path parity against the reference itself.

Inputs of >= 2^25 records take the sort's real hot path (the stripe first
level, the gathered second level, the LDS local pass). These tests sort the
benchmark workloads' own inputs (device splitmix64 generator, payload =
f(key)) at n = 2^25 + 1234 on the GPU and with the REFERENCE's own AVX-512
sort (oracle/_ref/libsrs_ref.so, radixSort.hpp:1761-1783 compiled from
/root/reference by oracle/Makefile) on the host, and compare every key and
payload byte. With payload = f(key) the sorted output is unique, so the
comparison is exact even though the reference is unstable.

C1: u64 key + u64 payload (both directions); C2: f32 key + two u32 payload
columns (duplicate-heavy: ~2^24 distinct float values); C3:
DataElement<u64,u64> records (AoS entry point, radixSort.hpp:1770-1778).
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
        pytest.fail("oracle/_ref/libsrs_ref.so missing or host lacks AVX-512 VBMI2: "
                    "the reference cannot run here")
    return torch


def _workload(torch, kind, psizes, first_index=0):
    dt = {srs_amd.KEY_U64: torch.int64, srs_amd.KEY_F32: torch.float32,
          srs_amd.KEY_I64: torch.int64}[kind]
    keys = torch.empty(N, dtype=dt, device="cuda")
    pays = [torch.empty(N, dtype={4: torch.int32, 8: torch.int64}[s], device="cuda")
            for s in psizes]
    srs_amd.fill_synthetic_device(keys, *pays, seed=42 << 32, first_index=first_index,
                                  key_kind=kind)
    return keys, pays


def _np(t, dtype):
    return t.cpu().numpy().view(dtype).copy()


@pytest.mark.parametrize("up", [True, False], ids=["up", "down"])
def test_c1_u64_u64_vs_reference(torch, up):
    keys, pays = _workload(torch, srs_amd.KEY_U64, [8], first_index=7 << 30)
    k_ref, p_ref = _np(keys, np.uint64), _np(pays[0], np.uint64)
    ko, po = torch.empty_like(keys), torch.empty_like(pays[0])
    srs_amd.sort_device(keys, pays[0], key_kind=srs_amd.KEY_U64, up=up, out=(ko, po))
    ref_sort_soa(srs_amd.KEY_U64, up, k_ref, [p_ref])
    torch.cuda.synchronize()
    assert np.array_equal(_np(ko, np.uint64), k_ref), "keys differ from the reference"
    assert np.array_equal(_np(po, np.uint64), p_ref), "payloads differ from the reference"


def test_c1_i64_inplace_vs_reference(torch):
    """Signed keys (sign-bit direction of bitDirUp, radixSort.hpp:1568-1581),
    in place, through the same hot path."""
    keys, pays = _workload(torch, srs_amd.KEY_I64, [8], first_index=3 << 33)
    k_ref, p_ref = _np(keys, np.int64), _np(pays[0], np.uint64)
    srs_amd.sort_device(keys, pays[0], key_kind=srs_amd.KEY_I64)
    ref_sort_soa(srs_amd.KEY_I64, True, k_ref, [p_ref])
    torch.cuda.synchronize()
    assert np.array_equal(_np(keys, np.int64), k_ref)
    assert np.array_equal(_np(pays[0], np.uint64), p_ref)


def test_c2_f32_two_u32_vs_reference(torch):
    keys, pays = _workload(torch, srs_amd.KEY_F32, [4, 4])
    k_ref = _np(keys, np.float32)
    p_ref = [_np(p, np.uint32) for p in pays]
    outs = [torch.empty_like(keys)] + [torch.empty_like(p) for p in pays]
    srs_amd.sort_device(keys, *pays, key_kind=srs_amd.KEY_F32, out=tuple(outs))
    ref_sort_soa(srs_amd.KEY_F32, True, k_ref, p_ref)
    torch.cuda.synchronize()
    assert np.array_equal(_np(outs[0], np.uint32), k_ref.view(np.uint32)), "keys differ"
    for c in range(2):
        assert np.array_equal(_np(outs[1 + c], np.uint32), p_ref[c]), f"payload {c} differs"


@pytest.mark.parametrize("up", [True, False], ids=["up", "down"])
def test_c3_aos16_vs_reference(torch, up):
    keys, pays = _workload(torch, srs_amd.KEY_U64, [8], first_index=11 << 30)
    rec = torch.stack([keys, pays[0]], dim=1).contiguous()
    del keys, pays
    r_ref = rec.cpu().numpy().view(np.uint8).reshape(N, 16).copy()
    out = torch.empty_like(rec)
    srs_amd.sort_combined_device(rec, srs_amd.KEY_U64, up=up, out=out)
    ref_sort_aos(srs_amd.KEY_U64, up, r_ref)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint8).reshape(N, 16), r_ref)


def test_c0_u32_keys_only_vs_reference(torch):
    """C0 (BASELINE configs[0]): 1e6 uint32 keys, no payload, ascending, through
    the host-array entry point (radixSort.hpp:1780 with no payload), against
    the reference's own sort and the oracle restatement."""
    from srs_testlib import oracle_sort_soa
    n = 10**6
    rng = np.random.default_rng(2024)
    keys = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    k = keys.copy()
    srs_amd.sort(k)
    k_ref = keys.copy()
    ref_sort_soa(srs_amd.KEY_U32, True, k_ref, [])
    assert np.array_equal(k, k_ref), "keys differ from the reference"
    k_or = keys.copy()
    oracle_sort_soa(srs_amd.KEY_U32, True, k_or, [])
    assert np.array_equal(k, k_or), "keys differ from the oracle"
