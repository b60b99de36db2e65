"""GPU parity tests: the HIP path (through the C ABI) against the golden
vectors made by the reference, the CPU oracle, and a stable numpy reference.

Parity contract:
  * keys: bit-identical to the reference;
  * payloads: bit-identical whenever payload = f(key) (the reference's own
    test convention, src/data.hpp:393-406); otherwise the multiset of payload
    tuples per run of equal keys is identical, and the GPU output equals a
    STABLE sort bit for bit (the GPU sort is stable, the reference is not);
  * n <= cmpSortThreshold: bit-identical including payload order (the
    reference sorts such inputs with its stable insertion sort).
"""
import numpy as np
import pytest

from srs_testlib import (KIND_DTYPES, KIND_NAMES, KIND_UINT, golden_arrays,
                         golden_manifest, key_size, oracle_sort_aos, oracle_sort_soa,
                         runs_multiset_equal, stable_reference, transformed_keys)

pytestmark = pytest.mark.gpu

srs_amd = pytest.importorskip("srs_amd")


def _torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    _torch()
    srs_amd.lib()


def bytes_equal(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint8),
                          np.ascontiguousarray(b).view(np.uint8))


def stable_aos(kind, up, elems, thresh=16):
    ks = key_size(kind)
    keys = np.ascontiguousarray(elems[:, :ks]).view(KIND_DTYPES[kind]).reshape(-1)
    (rec,) = stable_reference(kind, up, [keys, np.arange(len(keys))], thresh)[1:]
    return elems[rec]


# ---------------------------------------------------------------------------
# golden vectors (reference output)
# ---------------------------------------------------------------------------
def test_golden_all_cases():
    m = golden_manifest()
    fails = []
    for c in m["cases"]:
        ins, outs = golden_arrays(c)
        cols = [a.copy() for a in ins]
        if c["layout"] == "aos":
            srs_amd.sort_combined(cols[0], c["key_kind"], up=bool(c["up"]),
                                  cmp_sort_threshold=c["thresh"])
        else:
            srs_amd.sort_thresh(c["thresh"], cols[0], *cols[1:], up=bool(c["up"]))
        f_of_key = c["family"] in ("soa", "aos", "large")
        small = c["n"] <= c["thresh"]
        if c["layout"] == "aos":
            ks = key_size(c["key_kind"])
            ok = bytes_equal(cols[0][:, :ks], outs[0][:, :ks])
            if f_of_key or small:
                ok &= bytes_equal(cols[0], outs[0])
            else:
                ok &= bytes_equal(cols[0], stable_aos(c["key_kind"], c["up"], ins[0], c["thresh"]))
        else:
            ok = bytes_equal(cols[0], outs[0])
            if f_of_key or small:
                ok &= all(bytes_equal(a, b) for a, b in zip(cols[1:], outs[1:]))
            else:
                ok &= runs_multiset_equal(cols[0], outs[0], cols[1:], outs[1:])
                st = stable_reference(c["key_kind"], c["up"], ins, c["thresh"])
                ok &= all(bytes_equal(a, b) for a, b in zip(cols, st))
        if not ok:
            fails.append((c["family"], KIND_NAMES[c["key_kind"]], c["dist"], c["n"], c["up"]))
    assert not fails, f"{len(fails)} golden cases differ, e.g. {fails[:5]}"


# ---------------------------------------------------------------------------
# synthetic distributions at sizes that take the multi-level paths
# ---------------------------------------------------------------------------
def splitmix64(x):
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(0xFFFFFFFFFFFFFFFF)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def make_keys(kind, dist, n, seed):
    rng = np.random.default_rng(seed)
    dt = KIND_DTYPES[kind]
    ut = KIND_UINT[kind]
    nb = 8 * key_size(kind)
    if dist == "uniform":
        if KIND_NAMES[kind].startswith("f"):
            return rng.uniform(-1, 1, n).astype(dt)
        return rng.integers(0, 2**nb, n, dtype=np.uint64).astype(ut).view(dt)
    if dist == "gaussian":
        if KIND_NAMES[kind].startswith("f"):
            return rng.normal(0, 1, n).astype(dt)
        v = np.round(rng.normal(0, 100, n)).astype(np.int64)
        return v.astype(dt) if KIND_NAMES[kind].startswith("i") else v.astype(ut).view(dt)
    if dist == "zero":
        return np.zeros(n, dt)
    if dist == "zeroone":
        return rng.integers(0, 2, n).astype(dt)
    if dist == "sorted":
        return np.sort(make_keys(kind, "uniform", n, seed))
    if dist == "reverse":
        return np.sort(make_keys(kind, "uniform", n, seed))[::-1].copy()
    if dist == "fewdistinct":
        vals = make_keys(kind, "uniform", 37, seed + 1)
        return vals[rng.integers(0, 37, n)]
    if dist == "highbits":  # only the top byte varies: deep recursion
        u = rng.integers(0, 256, n, dtype=np.uint64) << np.uint64(nb - 8)
        return u.astype(ut).view(dt)
    if dist == "lowbits":  # only the low byte varies: skipped empty levels
        return rng.integers(0, 256, n, dtype=np.uint64).astype(ut).view(dt)
    raise ValueError(dist)


def payload_of(keys, size, salt=0):
    bits = keys.view(KIND_UINT[list(map(np.dtype, KIND_DTYPES)).index(keys.dtype)]).astype(np.uint64)
    h = splitmix64(bits ^ np.uint64(salt * 0x9E37))
    return h.astype({1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[size])


DISTS = ["uniform", "gaussian", "zero", "zeroone", "sorted", "reverse", "fewdistinct",
         "highbits", "lowbits"]


@pytest.mark.parametrize("kind", range(10), ids=KIND_NAMES)
@pytest.mark.parametrize("up", [True, False], ids=["up", "down"])
def test_distributions_vs_stable_and_oracle(kind, up):
    for di, dist in enumerate(DISTS):
        for n in (9000, 70001):
            keys = make_keys(kind, dist, n, 1000 * kind + 10 * di + n % 7)
            p64 = payload_of(keys, 8)
            idx = np.arange(n, dtype=np.uint32)  # NOT a function of the key
            k, a, b = keys.copy(), p64.copy(), idx.copy()
            srs_amd.sort(k, a, b, up=up)
            st = stable_reference(kind, up, [keys, p64, idx])
            assert bytes_equal(k, st[0]), (dist, n, "keys")
            assert bytes_equal(a, st[1]), (dist, n, "f(key) payload")
            assert bytes_equal(b, st[2]), (dist, n, "index payload (stability)")
            if n == 9000:  # the oracle restates the reference's own algorithm
                ok, op = keys.copy(), p64.copy()
                oracle_sort_soa(kind, up, ok, [op])
                assert bytes_equal(k, ok) and bytes_equal(a, op), (dist, n, "oracle")


def test_unaligned_host_arrays():
    """The reference takes unaligned arrays (loadu, src/simd.hpp); the host
    drop-in stages them through HBM, so byte-offset views sort like aligned
    ones. (Device arrays must be word-aligned: test_capi checks the error.)"""
    n = 100003
    keys = make_keys(6, "uniform", n, 7)
    pay = payload_of(keys, 4)
    kb = np.zeros(n * 8 + 3, np.uint8)
    pb = np.zeros(n * 4 + 1, np.uint8)
    k = kb[3:].view(np.uint64)
    p = pb[1:].view(np.uint32)
    assert k.ctypes.data % 8 and p.ctypes.data % 4
    k[:] = keys
    p[:] = pay
    srs_amd.sort(k, p)
    ok, op = keys.copy(), pay.copy()
    oracle_sort_soa(6, True, ok, [op])
    assert bytes_equal(k, ok) and bytes_equal(p, op)
    rec = np.zeros(n * 16 + 1, np.uint8)[1:].reshape(n, 16)
    rec[:, :8] = keys.view(np.uint8).reshape(n, 8)
    rec[:, 8:] = payload_of(keys, 8).view(np.uint8).reshape(n, 8)
    want = stable_aos(6, True, rec.copy())
    srs_amd.sort_combined(rec, 6)
    assert bytes_equal(rec, want)


@pytest.mark.parametrize("n", [0, 1, 2, 3, 15, 16, 17, 63, 64, 65, 4095, 4096, 8191, 8192,
                               8193, 12287, 16384, 16385, 24577, 100003, 1 << 20])
def test_sizes_u64_vs_oracle(n):
    keys = make_keys(6, "uniform", n, n)
    pay = payload_of(keys, 8)
    k, p = keys.copy(), pay.copy()
    srs_amd.sort(k, p)
    ok, op = keys.copy(), pay.copy()
    oracle_sort_soa(6, True, ok, [op])
    assert bytes_equal(k, ok) and bytes_equal(p, op)


def _fallback_keys(case, n, rng):
    if case in ("random64", "mid64"):
        # random64 (one small sort): the full 64-bit range fits the small sort's
        # below-digit words (12 / 13-bit bucket digit) -> no fallback. mid64:
        # after one global level the segments' ranges fit the fast kernel's
        # wide mode -> no fallback
        return rng.integers(0, 1 << 64, n, dtype=np.uint64)
    if case == "wide_dups":
        # wide keys and 200 copies of one value: the fast kernel hands
        # the segment over (a bucket > 64 records), the stable kernel ranks
        # key-only words (too wide for (key, index)) and keeps the equal
        # bucket as it is
        # (the copies alone in their top-10-bit bucket: the others < 2^63)
        k = rng.integers(0, 1 << 63, n, dtype=np.uint64)
        k[rng.choice(n, 200, replace=False)] = np.uint64(0xFFE0_1234_5678_9ABC)
        return k
    if case == "dups":      # big all-equal buckets: fast kernel -> stable kernel
        k = np.full(n, 0x1234_5678_9ABC, dtype=np.uint64)
        m = rng.random(n) < 0.1
        k[m] = rng.integers(1 << 62, 1 << 63, int(m.sum()), dtype=np.uint64)  # never in its bucket
    elif case == "wide":    # a big mixed bucket and a 61-bit varying range: -> stable -> LSD
        k = rng.integers(0, 1 << 20, n, dtype=np.uint64)
        k[rng.choice(n, 5, replace=False)] = rng.integers(1 << 59, 1 << 61, 5, dtype=np.uint64)
    else:                   # "groups": the same inside every top-6-bit group, many segments
        k = rng.integers(0, 1 << 16, n, dtype=np.uint64) | (
            (np.arange(n, dtype=np.uint64) % np.uint64(64)) << np.uint64(58))
        m = rng.random(n) < 0.002
        k[m] |= rng.integers(1 << 40, 1 << 57, int(m.sum()), dtype=np.uint64)
    return k


@pytest.mark.parametrize("case,n", [("random64", 16), ("random64", 3000), ("random64", 8000),
                                    ("wide_dups", 3000), ("wide_dups", 8000),
                                    ("mid64", 1 << 20), ("mid64", 100_003),
                                    ("dups", 3000), ("dups", 8000), ("wide", 3000),
                                    ("wide", 8000), ("groups", 300_000)])
def test_local_fallback_paths(case, n):
    """The stable and LSD local kernels run only when the fast kernel hands
    segments over (srs_debug_last_fallbacks reads the hand-over counts): these inputs
    force each path; the result must equal a stable sort bit for bit."""
    rng = np.random.default_rng(7)
    keys = _fallback_keys(case, n, rng)
    idx = np.arange(n, dtype=np.uint64)
    k, p = keys.copy(), idx.copy()
    srs_amd.sort(k, p)
    stable_n, lsd_n = srs_amd.last_fallbacks()
    order = np.argsort(keys, kind="stable")
    assert bytes_equal(k, keys[order]) and bytes_equal(p, idx[order])
    if case in ("mid64", "random64"):
        assert stable_n == 0 and lsd_n == 0, "the fast kernel should have sorted every segment"
        return
    assert stable_n > 0, "stable fallback not exercised"
    if case in ("wide", "groups"):
        assert lsd_n > 0, "LSD fallback not exercised"
    else:
        assert lsd_n == 0, "the stable kernel should have finished these segments"


@pytest.mark.parametrize("shape", ["u64+u64", "u32+u64", "i64+u64-down",
                                   "f32+2xu32", "f32+2xu32-dups", "i32+2xu32-down",
                                   "rec16-u64", "rec16-f64-down", "u64+u64-exact",
                                   "u64+u64-equal", "u64+u64-wide", "u64+u64-nosort",
                                   "u64+u64-large", "u32+u64-large", "i32+2xu32-large",
                                   "i32+2xu32-dups-large", "rec16-u64-large",
                                   "u64+u64-down-large"])
def test_direct_local_kernel(shape):
    """The direct local kernel (4 workgroups of 256 x 16 per CU)
    takes every local segment of the common shapes -- a 4/8-byte key with one
    8-byte payload (C1), a key with two 4-byte payloads (C2, exact segments
    included: '-dups' puts ~60 copies on each key value), 16-byte records of
    an 8-byte key (C3) -- and hands the rest to the fast kernel: segments of
    <= 11 varying bits in the C1 shape ('-exact'). srs_debug_last_local_counts
    proves which kernel ran; the result equals a stable sort bit for bit
    ('-nosort': CmpSorterNoSort leaves, checked against their guarantee).
    8-byte keys span 50 bits here: at this size one global level leaves up
    to 55 varying bits of full-range keys, and (key bits, index) words of
    more than 52 key bits go to the fast kernel's wide mode ('-wide').
    Segments of few varying bits ('-exact', '-equal': 3000 copies of each
    value) go to the fast kernel's exact pass, except in the pair mode.
    '-large': ~5.9K records per local segment (uniform integer keys: float
    keys spread unevenly over the first level's buckets), the large LDS class
    (512 x 16 per workgroup, two per CU); srs_debug_last_local_classes proves
    that class took them."""
    import os
    os.environ["SRS_DIRECT_MIN_SEGS"] = "1"  # (by default only sorts of >= 8192 local segments)
    try:
        _direct_local_case(shape)
    finally:
        del os.environ["SRS_DIRECT_MIN_SEGS"]


def _check_local_class(large):
    """-large: the large class took most segments, and its direct kernel
    handed (almost) none of them to the fast kernel."""
    if not large:
        return
    small, big, redo_small, redo_big = srs_amd.last_local_classes()
    assert big > small and redo_big * 100 <= big, (small, big, redo_small, redo_big)


def _direct_local_case(shape):
    rng = np.random.default_rng(sum(map(ord, shape)))
    large = shape.endswith("-large")
    shape = shape[:-len("-large")] if large else shape
    # (-large: one global level of 512 buckets leaves ~5.9K keys per bucket)
    n = 3_000_077 if large else (1 << 21) + 77
    up = not shape.endswith("-down")
    idx = np.arange(n, dtype=np.uint64)
    if shape.startswith("rec16"):
        kind = 9 if "f64" in shape else 6
        if kind == 9:  # integers < 2^40 as doubles, both signs: trailing zero mantissa bits
            keys = (rng.integers(0, 1 << 40, n) * rng.choice([-1, 1], n)).astype(np.float64)
        else:
            keys = make_keys(kind, "uniform", n, 5) >> np.uint64(14)
        elems = np.empty((n, 16), dtype=np.uint8)
        elems[:, :8] = keys.view(np.uint8).reshape(n, 8)
        elems[:, 8:] = idx.view(np.uint8).reshape(n, 8)
        e = elems.copy()
        srs_amd.sort_combined(e, kind, up=up)
        nloc, redo = srs_amd.last_local_counts()
        _check_local_class(large)
        assert bytes_equal(e, stable_aos(kind, up, elems))
        assert nloc > 0 and redo * 100 <= nloc, (nloc, redo)
        return
    if "2xu32" in shape:
        kind = 5 if shape.startswith("i32") else 8
        if shape.endswith("-dups") and kind == 5:  # 2^16 values, ~46 copies each (-large)
            keys = (rng.integers(-(1 << 15), 1 << 15, n) << 16).astype(np.int32)
        elif shape.endswith("-dups"):
            keys = (rng.integers(-(1 << 15), 1 << 15, n) / 32768.0).astype(np.float32)
        else:
            keys = make_keys(kind, "uniform", n, 9)
        p0 = payload_of(keys, 4)
        p1 = np.arange(n, dtype=np.uint32)
        k, a, b = keys.copy(), p0.copy(), p1.copy()
        srs_amd.sort(k, a, b, up=up)
        nloc, redo = srs_amd.last_local_counts()
        _check_local_class(large)
        st = stable_reference(kind, up, [keys, p0, p1])
        assert bytes_equal(k, st[0]) and bytes_equal(a, st[1]) and bytes_equal(b, st[2])
        # (a few segments may never have left the input arrays, where the
        # pair layout does not hold: those go to the fast kernel)
        assert nloc > 0 and redo * 100 <= nloc, (nloc, redo)
        return
    kind = {"u64": 6, "u32": 4, "i64": 7}[shape.split("+")[0]]
    if shape.endswith("-exact"):  # 2^20 distinct values: ~2 per value, <= 11 bits per segment
        keys = (rng.integers(0, 1 << 20, n, dtype=np.uint64) << np.uint64(30)).astype(np.uint64)
    elif shape.endswith("-equal"):  # 3000 copies of each value
        keys = ((np.arange(n, dtype=np.uint64) // np.uint64(3000)) << np.uint64(40))
        keys = keys[rng.permutation(n)]
    else:
        keys = make_keys(kind, "uniform", n, 3)
        if kind != 4 and not shape.endswith("-wide"):
            keys = keys >> keys.dtype.type(14)
    k, p = keys.copy(), idx.copy()
    nosort = shape.endswith("-nosort")
    if nosort:
        srs_amd.sort_thresh(16, k, p, cmp_sorter="nosort")
    else:
        srs_amd.sort(k, p, up=up)
    nloc, redo = srs_amd.last_local_counts()
    _check_local_class(large)
    assert nloc > 0
    if shape.endswith("-equal") or shape.endswith("-exact"):
        pass  # (few values per segment, or one: either kernel may take them)
    elif shape.endswith("-wide"):
        # (the balanced first level's key-range groups need not align with
        # powers of two, so only part of the segments lands in the class)
        assert redo > 0, (nloc, redo)
    else:
        assert redo == 0, (nloc, redo)
    if nosort:
        assert bytes_equal(keys[p.astype(np.int64)], k)
        srt = np.sort(keys)
        lo = np.searchsorted(srt, k, "left")
        hi = np.searchsorted(srt, k, "right") - 1
        i = np.arange(n)
        assert np.all(i >= lo - 15) and np.all(i <= hi + 15)
        assert not bytes_equal(k, srt)
        return
    st = stable_reference(kind, up, [keys, idx])
    assert bytes_equal(k, st[0]) and bytes_equal(p, st[1])


@pytest.mark.parametrize("n", [5000, 50000], ids=["one-launch", "levels"])
@pytest.mark.parametrize("sizes", [[1], [2], [4], [8], [8, 1], [4, 4], [8, 8, 8], [1] * 63,
                                   [2, 8, 1, 4]])
def test_payload_packs(sizes, n):
    # n = 5000: the single-launch small sort, whose descriptor (up to 65
    # columns) travels as a kernel argument
    keys = make_keys(5, "gaussian", n, 7)
    pays = [payload_of(keys, s, salt=i) for i, s in enumerate(sizes)]
    idx = np.arange(n, dtype=np.uint64)
    cols = [keys.copy()] + [p.copy() for p in pays] + [idx.copy()]
    srs_amd.sort(*cols)
    st = stable_reference(5, True, [keys] + pays + [idx])
    assert all(bytes_equal(a, b) for a, b in zip(cols, st))


@pytest.mark.parametrize("kind", [0, 3, 4, 6, 8, 9], ids=lambda k: KIND_NAMES[k])
@pytest.mark.parametrize("esz_mult", [1, 2, 4, 8])
@pytest.mark.parametrize("up", [True, False], ids=["up", "down"])
def test_combined_records(kind, esz_mult, up):
    ks = key_size(kind)
    esz = ks * esz_mult
    if esz > 64:
        pytest.skip("DataElement larger than 64 bytes")
    n = 30011
    keys = make_keys(kind, "gaussian" if kind in (3, 8) else "uniform", n, esz)
    rng = np.random.default_rng(esz)
    elems = rng.integers(0, 256, (n, esz), dtype=np.uint8)
    elems[:, :ks] = keys.view(np.uint8).reshape(n, ks)
    e = elems.copy()
    srs_amd.sort_combined(e, kind, up=up)
    assert bytes_equal(e, stable_aos(kind, up, elems))
    if n < 40000:
        o = elems.copy()
        oracle_sort_aos(kind, up, o)
        assert bytes_equal(e[:, :ks], o[:, :ks])


@pytest.mark.parametrize("esz,n,case", [(16, 4_000_003, "uniform"), (32, 3_500_000, "uniform"),
                                        (64, 3_300_001, "gaussian"), (16, 200_000, "dupblock"),
                                        (32, 150_000, "dupblock")])
def test_combined_records_slice_columns(esz, n, case):
    """Records of 16+ bytes travel as SoA slice columns through TMP / TMP2
    between the first scatter and the local pass (SortDesc::tmp2): two
    global levels (n > 3.1M) use both workspace buffers; 'dupblock' puts 40 %
    of the records on one key, a finished segment larger than the local
    capacity that is copied home column by column (copy_home_kernel)."""
    kind = 7  # int64 keys
    rng = np.random.default_rng(n + esz)
    if case == "dupblock":
        keys = rng.integers(-2**62, 2**62, n, dtype=np.int64)
        keys[rng.random(n) < 0.4] = 123456789
    else:
        keys = make_keys(kind, case, n, esz)
    elems = rng.integers(0, 256, (n, esz), dtype=np.uint8)
    elems[:, :8] = keys.view(np.uint8).reshape(n, 8)
    e = elems.copy()
    srs_amd.sort_combined(e, kind)
    assert bytes_equal(e, stable_aos(kind, True, elems))


# ---------------------------------------------------------------------------
# device API (torch tensors in HBM)
# ---------------------------------------------------------------------------
def test_device_inplace_and_out_of_place():
    torch = _torch()
    n = 3_000_000
    dev = torch.device("cuda:0")
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    p0 = torch.empty(n, dtype=torch.int32, device=dev)
    p1 = torch.empty(n, dtype=torch.int32, device=dev)
    srs_amd.fill_synthetic_device(keys, p0, p1, key_kind=srs_amd.KEY_U64)
    k_in = keys.clone()
    p0_in, p1_in = p0.clone(), p1.clone()
    ko, o0, o1 = torch.empty_like(keys), torch.empty_like(p0), torch.empty_like(p1)
    srs_amd.sort_device(keys, p0, p1, key_kind=srs_amd.KEY_U64, out=(ko, o0, o1))
    torch.cuda.synchronize()
    assert torch.equal(keys, k_in) and torch.equal(p0, p0_in) and torch.equal(p1, p1_in)
    srs_amd.sort_device(keys, p0, p1, key_kind=srs_amd.KEY_U64)
    torch.cuda.synchronize()
    assert torch.equal(keys, ko) and torch.equal(p0, o0) and torch.equal(p1, o1)
    kh = k_in.cpu().numpy().view(np.uint64)
    st = stable_reference(6, True, [kh, p0_in.cpu().numpy(), p1_in.cpu().numpy()])
    assert bytes_equal(ko.cpu().numpy(), st[0])
    assert bytes_equal(o0.cpu().numpy(), st[1]) and bytes_equal(o1.cpu().numpy(), st[2])


def test_two_streams_share_the_workspace():
    """Sorts queued back to back on two non-blocking streams share the
    device's cached workspace (descriptor, lists, TMP): the second call must
    wait on the device for the first one's kernels (srs_api.hip WsUse).
    Three rounds of alternating streams, each result against a stable sort."""
    torch = _torch()
    dev = torch.device("cuda:0")
    streams = [torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)]
    sizes = [3_000_000, 2_500_001]
    ins, outs = [], []
    for i, n in enumerate(sizes):
        k = torch.empty(n, dtype=torch.int64, device=dev)
        p = torch.empty(n, dtype=torch.int64, device=dev)
        srs_amd.fill_synthetic_device(k, p, seed=1000 + i, key_kind=srs_amd.KEY_U64)
        ins.append((k, p))
        outs.append((torch.empty_like(k), torch.empty_like(p)))
    torch.cuda.synchronize()
    for _ in range(3):
        for s, (k, p), (ko, po) in zip(streams, ins, outs):
            s.wait_stream(torch.cuda.current_stream(dev))  # inputs are ready
            srs_amd.sort_device(k, p, key_kind=srs_amd.KEY_U64, out=(ko, po), stream=s)
    torch.cuda.synchronize()
    for (k, p), (ko, po) in zip(ins, outs):
        kh, ph = k.cpu().numpy().view(np.uint64), p.cpu().numpy()
        st = stable_reference(6, True, [kh, ph])
        assert bytes_equal(ko.cpu().numpy(), st[0]) and bytes_equal(po.cpu().numpy(), st[1])


def test_device_api_rejects_mismatched_tensors():
    torch = _torch()
    dev = torch.device("cuda:0")
    k = torch.zeros(100, dtype=torch.int64, device=dev)
    with pytest.raises(ValueError):
        srs_amd.sort_device(k, torch.zeros(100, dtype=torch.int64))  # payload on the host
    with pytest.raises(ValueError):
        srs_amd.sort_device(k, out=(torch.zeros(99, dtype=torch.int64, device=dev),))
    with pytest.raises(ValueError):
        srs_amd.sort_device(k, out=(torch.zeros(100, dtype=torch.int32, device=dev),))


@pytest.mark.parametrize("kind", [0, 3, 4, 7, 8, 9], ids=lambda k: KIND_NAMES[k])
@pytest.mark.parametrize("up", [True, False], ids=["up", "down"])
def test_two_u32_payloads_travel_as_words(kind, up):
    """A key and two 4-byte payloads (C2's shape) move through the workspace
    as one interleaved 8-byte word per record (SortDesc::pair): joined by the
    first scatter, split by the local pass, copied home apart by the copy
    list; a payload of input indices checks stability bit for bit."""
    for di, dist in enumerate(["uniform", "gaussian", "zero", "fewdistinct", "highbits"]):
        n = 70001 if di else 600_011
        keys = make_keys(kind, dist, n, 31 * kind + di)
        p0 = payload_of(keys, 4)
        p1 = np.arange(n, dtype=np.uint32)
        k, a, b = keys.copy(), p0.copy(), p1.copy()
        srs_amd.sort(k, a, b, up=up)
        st = stable_reference(kind, up, [keys, p0, p1])
        assert bytes_equal(k, st[0]) and bytes_equal(a, st[1]) and bytes_equal(b, st[2]), dist


def test_device_float_keys_two_payloads():
    """C2 shape: f32 keys in [-1, 1) + two u32 payload columns."""
    torch = _torch()
    n = 2_000_003
    dev = torch.device("cuda:0")
    keys = torch.empty(n, dtype=torch.float32, device=dev)
    p0 = torch.empty(n, dtype=torch.int32, device=dev)
    p1 = torch.empty(n, dtype=torch.int32, device=dev)
    srs_amd.fill_synthetic_device(keys, p0, p1)
    kh, ah, bh = keys.cpu().numpy(), p0.cpu().numpy(), p1.cpu().numpy()
    srs_amd.sort_device(keys, p0, p1)
    torch.cuda.synchronize()
    st = stable_reference(8, True, [kh, ah, bh])
    assert bytes_equal(keys.cpu().numpy(), st[0])
    assert bytes_equal(p0.cpu().numpy(), st[1]) and bytes_equal(p1.cpu().numpy(), st[2])


def test_device_combined_records():
    """C3 shape: DataElement<uint64, uint64> records."""
    torch = _torch()
    n = 2_000_000
    dev = torch.device("cuda:0")
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    pays = torch.empty(n, dtype=torch.int64, device=dev)
    srs_amd.fill_synthetic_device(keys, pays, key_kind=srs_amd.KEY_U64)
    rec = torch.stack([keys, pays], dim=1).contiguous()
    host = rec.cpu().numpy().view(np.uint8).reshape(n, 16).copy()
    srs_amd.sort_combined_device(rec, srs_amd.KEY_U64)
    torch.cuda.synchronize()
    assert bytes_equal(rec.cpu().numpy().view(np.uint8).reshape(n, 16), stable_aos(6, True, host))


def test_errors_are_loud():
    with pytest.raises(srs_amd.SrsError):
        srs_amd.sort_combined(np.zeros((10, 12), np.uint8), srs_amd.KEY_U32)  # not a power of two
    with pytest.raises(TypeError):
        srs_amd.sort(np.zeros(10, np.complex64))


# ---------------------------------------------------------------------------
# multi-GPU shard primitives on one GPU
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("kind", [4, 6, 7, 8, 9], ids=lambda k: KIND_NAMES[k])
def test_key_histogram_and_partition(kind):
    torch = _torch()

    def balanced_split(h, parts):  # bins -> parts, non-decreasing (the shard plan's rule)
        hv = h.cpu().numpy().astype(np.float64)
        mid = np.cumsum(hv) - hv + 0.5 * hv
        p = np.maximum.accumulate(np.clip(np.floor(mid * parts / hv.sum()), 0, parts - 1))
        return torch.from_numpy(p.astype(np.int32)).cuda()
    n = 1_000_003
    keys_h = make_keys(kind, "gaussian" if kind in (7, 9) else "uniform", n, kind)
    pay_h = np.arange(n, dtype=np.int64)
    tdt = {4: torch.int32, 6: torch.int64, 7: torch.int64, 8: torch.float32, 9: torch.float64}
    keys = torch.from_numpy(keys_h.view(np.int32 if kind == 4 else np.int64)
                            if kind in (4, 6) else keys_h).cuda()
    pay = torch.from_numpy(pay_h).cuda()
    bits = 10
    hist = torch.zeros(1 << bits, dtype=torch.int64, device="cuda")
    srs_amd.key_histogram_device(keys, hist, bits, key_kind=kind)
    u = transformed_keys(kind, True, keys_h)
    top = (u >> np.uint64(8 * key_size(kind) - bits)).astype(np.int64)
    assert np.array_equal(hist.cpu().numpy(), np.bincount(top, minlength=1 << bits))
    aligned = {8: torch.arange(1 << bits, dtype=torch.int32, device="cuda") >> (bits - 3),
               512: torch.arange(1 << bits, dtype=torch.int32, device="cuda") >> (bits - 9)}
    for world in (1, 3, 8, "a8", "a512"):
        if isinstance(world, str):  # groups = top-bit ranges: the plain-digit partition
            world = int(world[1:])
            pob = aligned[world]
        else:
            pob = balanced_split(hist, world)
        ko, po = torch.empty_like(keys), torch.empty_like(pay)
        counts = srs_amd.partition_device(keys, [pay], bits, pob, world, (ko, po), key_kind=kind)
        dest = pob.cpu().numpy()[top]
        assert counts == np.bincount(dest, minlength=world).tolist()
        order = np.argsort(dest, kind="stable")  # stable partition
        assert bytes_equal(ko.cpu().numpy(), keys.cpu().numpy()[order])
        assert bytes_equal(po.cpu().numpy(), pay_h[order])


@pytest.mark.parametrize("kind", [6, 8, 3], ids=lambda k: KIND_NAMES[k])
def test_sort_segments_device(kind):
    """srs_sort_segments_device: every segment sorted on its own (stable),
    bytes outside the segments untouched; sizes span the local and global
    paths."""
    torch = _torch()
    rng = np.random.default_rng(5)
    lens = [0, 1, 2, 17, 4096, 4097, 8192, 8193, 50_000, 300_001, 3]
    gaps = [5, 0, 3, 0, 0, 1, 0, 7, 0, 2, 0]
    pos, segs = 0, []
    for ln, gp in zip(lens, gaps):
        pos += gp
        segs.append((pos, pos + ln))
        pos += ln
    n = pos + 11
    keys_h = make_keys(kind, "uniform", n, kind)
    pay_h = np.arange(n, dtype=np.int64)
    keys = torch.from_numpy(keys_h.view(np.int64) if kind == 6 else keys_h).cuda()
    pay = torch.from_numpy(pay_h).cuda()
    # bounds list every segment's ends; the stretches between listed
    # segments are segments too, and [0, 5) and the last 11 are outside all
    flat = []
    for a, b in segs:
        flat += [a, b]
    srs_amd.sort_segments_device(keys, pay, bounds=flat, key_kind=kind)
    ko = keys.cpu().numpy().view(keys_h.dtype)
    po = pay.cpu().numpy()
    exp_k, exp_p = keys_h.copy(), pay_h.copy()
    edges = list(zip(flat[:-1], flat[1:]))  # every consecutive pair is a segment
    for a, b in edges:
        if b - a < 2:
            continue
        u = transformed_keys(kind, True, keys_h[a:b])
        o = np.argsort(u, kind="stable")
        exp_k[a:b] = keys_h[a:b][o]
        exp_p[a:b] = pay_h[a:b][o]
    assert bytes_equal(ko, exp_k) and np.array_equal(po, exp_p)


# ---------------------------------------------------------------------------
# scale: adversarial distributions at 5e7 against torch's stable sort, and
# more than 2^32 keys (64-bit positions everywhere)
# ---------------------------------------------------------------------------
def _device_keys(torch, dist, n, g):
    i64 = torch.int64
    if dist == "uniform":
        return torch.randint(-2**63, 2**63 - 1, (n,), dtype=i64, device="cuda", generator=g)
    if dist == "equal":
        return torch.full((n,), 12345, dtype=i64, device="cuda")
    if dist == "zeroone":
        return torch.randint(0, 2, (n,), dtype=i64, device="cuda", generator=g)
    if dist == "fewdistinct":
        vals = torch.randint(-2**63, 2**63 - 1, (37,), dtype=i64, device="cuda", generator=g)
        return vals[torch.randint(0, 37, (n,), device="cuda", generator=g)]
    if dist == "dup64":  # every value ~64 times (duplicate-heavy local segments)
        return torch.randint(0, n // 64, (n,), dtype=i64, device="cuda", generator=g) * 7919
    if dist == "sorted":
        return torch.sort(torch.randint(0, 2**62, (n,), dtype=i64, device="cuda", generator=g))[0]
    if dist == "reverse":
        return torch.sort(torch.randint(0, 2**62, (n,), dtype=i64, device="cuda",
                                        generator=g))[0].flip(0)
    if dist == "highbits":
        return torch.randint(0, 256, (n,), dtype=i64, device="cuda", generator=g) << 56
    if dist == "lowbits":
        return torch.randint(0, 256, (n,), dtype=i64, device="cuda", generator=g)
    if dist == "gaussian":
        return (torch.randn(n, device="cuda", generator=g) * 1e6).round().to(i64)
    raise ValueError(dist)


@pytest.mark.parametrize("dist", ["uniform", "equal", "zeroone", "fewdistinct", "dup64",
                                  "sorted", "reverse", "highbits", "lowbits", "gaussian"])
def test_scale_distributions_vs_torch_stable(dist):
    """5e7 u64 keys + their input index as payload: keys and payloads must
    equal torch's stable sort (signed view of the unsigned order) exactly."""
    torch = _torch()
    n = 50_000_017
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    keys = _device_keys(torch, dist, n, g)
    pay = torch.arange(n, dtype=torch.int64, device="cuda")
    ko, po = torch.empty_like(keys), torch.empty_like(pay)
    srs_amd.sort_device(keys, pay, key_kind=srs_amd.KEY_U64, out=(ko, po))
    ref_k, ref_i = torch.sort(keys ^ torch.iinfo(torch.int64).min, stable=True)
    assert torch.equal(ko, ref_k ^ torch.iinfo(torch.int64).min)
    assert torch.equal(po, ref_i)


@pytest.mark.parametrize("case", ["u32_pays_down_inplace", "i64_keys_only", "u64_fewbuckets",
                                  "u32_equal", "u64_tiny_pieces"])
def test_stripe_first_level(case):
    """n >= 2^25 plain SoA sorts take the stripe first level (each stripe
    partitioned on its own, the second level reading every bucket's pieces
    through gathered tiles): keys and every payload column against torch's
    stable sort, including pieces far from their average size (few buckets
    used, all-equal keys, buckets that most stripes leave nearly empty)."""
    torch = _torch()
    n = (1 << 25) + 4099
    g = torch.Generator(device="cuda")
    g.manual_seed(17)
    idx = torch.arange(n, dtype=torch.int64, device="cuda")
    up = True
    if case == "u32_pays_down_inplace":
        keys = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device="cuda", generator=g)
        kind, up = srs_amd.KEY_U32, False
    elif case == "i64_keys_only":
        keys = torch.randint(-2**63, 2**63 - 1, (n,), dtype=torch.int64, device="cuda", generator=g)
        kind = srs_amd.KEY_I64
    elif case == "u64_fewbuckets":  # every other top-digit bucket empty, uniform below
        keys = (torch.randint(0, 256, (n,), dtype=torch.int64, device="cuda", generator=g) << 56) | \
            torch.randint(0, 2**40, (n,), dtype=torch.int64, device="cuda", generator=g)
        kind = srs_amd.KEY_U64
    elif case == "u32_equal":  # the key sample declines the stripe level: plain path
        keys = torch.full((n,), 77, dtype=torch.int32, device="cuda")
        kind = srs_amd.KEY_U32
    else:  # sorted keys: a stripe holds one or two buckets, every other piece is empty
        keys = torch.sort(torch.randint(0, 2**62, (n,), dtype=torch.int64, device="cuda",
                                        generator=g))[0]
        kind = srs_amd.KEY_U64
    if keys.dtype == torch.int32:
        order_view = keys ^ torch.iinfo(torch.int32).min if kind == srs_amd.KEY_U32 else keys
    else:
        order_view = keys ^ torch.iinfo(torch.int64).min if kind == srs_amd.KEY_U64 else keys
    if not up:
        order_view = ~order_view
    ref_v, ref_i = torch.sort(order_view, stable=True)
    ref_k = keys[ref_i]
    if case == "u32_pays_down_inplace":
        p8 = (idx & 0xFF).to(torch.uint8)
        p16 = (idx & 0x7FFF).to(torch.int16)
        p64 = idx.clone()
        k = keys.clone()
        srs_amd.sort_device(k, p8, p16, p64, key_kind=kind, up=up)
        assert torch.equal(k, ref_k)
        assert torch.equal(p64, ref_i)
        assert torch.equal(p8, (ref_i & 0xFF).to(torch.uint8))
        assert torch.equal(p16, (ref_i & 0x7FFF).to(torch.int16))
    elif case == "i64_keys_only":
        ko = torch.empty_like(keys)
        srs_amd.sort_device(keys, key_kind=kind, out=(ko,))
        assert torch.equal(ko, ref_k)
        # the workspace (stripe tables included) is freed and grown again
        srs_amd.release_workspace()
        ko.zero_()
        srs_amd.sort_device(keys, key_kind=kind, out=(ko,))
        assert torch.equal(ko, ref_k)
    else:
        ko, po = torch.empty_like(keys), torch.empty_like(idx)
        srs_amd.sort_device(keys, idx, key_kind=kind, out=(ko, po))
        assert torch.equal(ko, ref_k)
        assert torch.equal(po, ref_i)


@pytest.mark.parametrize("kind", ["u32", "i32", "f32", "u64", "i64", "f64"])
@pytest.mark.parametrize("up", [True, False])
def test_stripe_first_level_key_kinds(kind, up):
    """Every 4- and 8-byte key kind, both directions, through the stripe first
    level (uniform keys: the key sample lets it run; floats in [-1e6, 1e6),
    no -0.0 or NaN), with the input index as payload: keys and payloads equal
    torch's stable sort in the reference's order."""
    torch = _torch()
    n = (1 << 25) + 1234
    g = torch.Generator(device="cuda")
    g.manual_seed(29)
    idx = torch.arange(n, dtype=torch.int64, device="cuda")
    if kind in ("u32", "i32"):
        keys = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device="cuda", generator=g)
        ov = keys ^ torch.iinfo(torch.int32).min if kind == "u32" else keys
    elif kind in ("u64", "i64"):
        keys = torch.randint(-2**63, 2**63 - 1, (n,), dtype=torch.int64, device="cuda", generator=g)
        ov = keys ^ torch.iinfo(torch.int64).min if kind == "u64" else keys
    else:
        dt = torch.float32 if kind == "f32" else torch.float64
        keys = (torch.rand(n, device="cuda", generator=g, dtype=dt) * 2 - 1) * 1e6
        keys = torch.where(keys == 0, torch.ones_like(keys), keys)
        ov = keys
    ref_v, ref_i = torch.sort(ov if up else (-ov if kind in ("f32", "f64") else ~ov), stable=True)
    kk = {"u32": srs_amd.KEY_U32, "i32": srs_amd.KEY_I32, "f32": srs_amd.KEY_F32,
          "u64": srs_amd.KEY_U64, "i64": srs_amd.KEY_I64, "f64": srs_amd.KEY_F64}[kind]
    ko, po = torch.empty_like(keys), torch.empty_like(idx)
    srs_amd.sort_device(keys, idx, key_kind=kk, up=up, out=(ko, po))
    assert torch.equal(po, ref_i)
    assert torch.equal(ko, keys[ref_i])


@pytest.mark.parametrize("case", ["aos16", "aos32_down", "aos16_inplace", "aos8",
                                  "f32_two_u32_grid", "f32_two_u32_uniform", "u64_six_payloads"])
def test_stripe_first_level_layouts(case):
    """The stripe first level under the other column layouts: AoS records as
    slice columns (16 and 32 bytes), C2's key + two 4-byte payloads as word
    pairs, with the balanced digit-table first level (skewed grid floats) and
    without it (uniform floats); against torch's stable sort."""
    torch = _torch()
    n = (1 << 25) + 777
    g = torch.Generator(device="cuda")
    g.manual_seed(23)
    idx = torch.arange(n, dtype=torch.int64, device="cuda")
    if case == "aos8":  # DataElement<int32, int32>: one 8-byte column
        keys = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device="cuda",
                             generator=g) & ~0xFF  # duplicates, top bits spread
        rec = torch.stack([keys, idx.to(torch.int32)], dim=1).contiguous()
        out = torch.empty_like(rec)
        srs_amd.sort_combined_device(rec, srs_amd.KEY_I32, out=out)
        _, ref_i = torch.sort(keys, stable=True)
        assert torch.equal(out, rec[ref_i])
        return
    if case.startswith("aos"):
        words = 4 if case == "aos32_down" else 2
        up = case != "aos32_down"
        keys = torch.randint(-2**63, 2**63 - 1, (n,), dtype=torch.int64, device="cuda", generator=g)
        keys = keys & ~((1 << 40) - 1)  # duplicates (equal keys keep input order), top bits spread
        rec = torch.stack([keys] + [idx * (w + 1) for w in range(words - 1)], dim=1).contiguous()
        ov = keys if up else ~keys
        _, ref_i = torch.sort(ov, stable=True)
        exp = rec[ref_i]
        if case == "aos16_inplace":
            srs_amd.sort_combined_device(rec, srs_amd.KEY_I64, up=up)
            assert torch.equal(rec, exp)
        else:
            out = torch.empty_like(rec)
            srs_amd.sort_combined_device(rec, srs_amd.KEY_I64, up=up, out=out)
            assert torch.equal(out, exp)
        return
    if case == "u64_six_payloads":
        keys = torch.randint(-2**63, 2**63 - 1, (n,), dtype=torch.int64, device="cuda", generator=g)
        pays = [(idx * (c + 1)).to(dt) for c, dt in
                enumerate([torch.int64, torch.int32, torch.int16, torch.uint8, torch.int64,
                           torch.int32])]
        outs = [torch.empty_like(p) for p in pays]
        ko = torch.empty_like(keys)
        srs_amd.sort_device(keys, *pays, key_kind=srs_amd.KEY_U64, out=(ko, *outs))
        _, ref_i = torch.sort(keys ^ torch.iinfo(torch.int64).min, stable=True)
        assert torch.equal(ko, keys[ref_i])
        for p, o in zip(pays, outs):
            assert torch.equal(o, p[ref_i])
        return
    if case == "f32_two_u32_grid":
        keys = (torch.randint(0, 1 << 24, (n,), device="cuda", generator=g).to(torch.float32)
                * (1.0 / (1 << 23)) - 1.0)
    else:
        keys = torch.rand(n, device="cuda", generator=g) * 2 - 1
    keys = torch.where(keys == 0, torch.zeros_like(keys), keys)
    p0 = idx.to(torch.int32)
    p1 = (idx * 3).to(torch.int32)
    ko, o0, o1 = torch.empty_like(keys), torch.empty_like(p0), torch.empty_like(p1)
    srs_amd.sort_device(keys, p0, p1, key_kind=srs_amd.KEY_F32, out=(ko, o0, o1))
    ref_k, ref_i = torch.sort(keys, stable=True)
    assert torch.equal(ko.view(torch.int32), ref_k.view(torch.int32))
    assert torch.equal(o0, ref_i.to(torch.int32))
    assert torch.equal(o1, (ref_i * 3).to(torch.int32))


def test_more_than_2_pow_32_keys():
    """n > 2^32: positions, tile indices and offsets are 64-bit throughout.
    u32 keys (17 GB), in place; checked by order and by two multiset sums."""
    torch = _torch()
    n = (1 << 32) + 1027
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    keys = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device="cuda", generator=g)
    wide = keys.to(torch.int64) & 0xFFFFFFFF
    s1, s2 = int(wide.sum().item()), int((wide * wide).sum().item())
    del wide
    srs_amd.sort_device(keys, key_kind=srs_amd.KEY_U32)
    wide = keys.to(torch.int64) & 0xFFFFFFFF
    assert bool((wide[1:] >= wide[:-1]).all().item())
    assert int(wide.sum().item()) == s1 and int((wide * wide).sum().item()) == s2


@pytest.mark.parametrize("dist", ["f32grid", "f32normal", "f64normal", "f64uniform"])
def test_scale_float_keys_vs_torch_stable(dist):
    """5e7 float keys (C2's grid distribution included: heavy duplicates and
    a quarter of the keys under one exponent -> the balanced first level) +
    input index payload, against torch's stable sort (no -0.0 and no NaN in
    the inputs, so float order equals the reference's bit order)."""
    torch = _torch()
    n = 50_000_021
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    if dist == "f32grid":
        keys = (torch.randint(0, 1 << 24, (n,), device="cuda", generator=g).to(torch.float32)
                * (1.0 / (1 << 23)) - 1.0)
    elif dist == "f32normal":
        keys = torch.randn(n, device="cuda", generator=g)
    elif dist == "f64normal":
        keys = torch.randn(n, device="cuda", generator=g, dtype=torch.float64)
    else:
        keys = torch.rand(n, device="cuda", generator=g, dtype=torch.float64) * 2 - 1
    keys = torch.where(keys == 0, torch.zeros_like(keys), keys)  # no -0.0
    kind = srs_amd.KEY_F32 if keys.dtype == torch.float32 else srs_amd.KEY_F64
    pay = torch.arange(n, dtype=torch.int64, device="cuda")
    ko, po = torch.empty_like(keys), torch.empty_like(pay)
    srs_amd.sort_device(keys, pay, key_kind=kind, out=(ko, po))
    ref_k, ref_i = torch.sort(keys, stable=True)
    assert torch.equal(ko.view(torch.int32 if kind == srs_amd.KEY_F32 else torch.int64),
                       ref_k.view(torch.int32 if kind == srs_amd.KEY_F32 else torch.int64))
    assert torch.equal(po, ref_i)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("n", [3000, 70000])
@pytest.mark.parametrize("up", [True, False])
def test_float_zero_canon_large_threshold(dtype, n, up):
    """n <= cmpSortThreshold with many -0.0/+0.0 keys: the reference's leaf
    compares by value (-0.0 == +0.0, input order kept), radixSort.hpp:1743 +
    :159-178. With a threshold >= n the GPU runs the canon-zero kernel
    instantiations (SRS_KS_CANON) through the local (n=3000) and the global
    levels (n=70000); a threshold of 16 must keep -0.0 before +0.0."""
    rng = np.random.default_rng(n + (dtype == np.float64))
    keys = rng.choice(np.array([-0.0, 0.0, 1.5, -2.25, 0.5, -0.0, 0.0], dtype=dtype), n)
    mix = rng.random(n) < 0.3
    keys[mix] = rng.standard_normal(int(mix.sum())).astype(dtype)
    pay = np.arange(n, dtype=np.uint32)
    kind = srs_amd.key_kind_of(keys.dtype)
    for thresh in (n, 16):
        k, p = keys.copy(), pay.copy()
        srs_amd.sort_thresh(thresh, k, p, up=up)
        ek, ep = stable_reference(kind, up, [keys, pay], thresh)
        assert bytes_equal(k, ek), (thresh, "keys")
        assert bytes_equal(p, ep), (thresh, "payload order")


def test_copy_list_long_and_many_short_segments():
    """Finished segments that are not in OUT go home through the copy list:
    here one segment of 2^23 equal keys beside ~800 segments of 10000 equal
    keys each (the chunked copy grid gives the long one the
    whole grid), keys + two payload columns against torch's stable sort."""
    torch = _torch()
    n_long, n_short, reps = 1 << 23, 800, 10000
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    short = torch.arange(1, n_short + 1, dtype=torch.int64, device="cuda").repeat_interleave(reps)
    keys = torch.cat([torch.full((n_long,), 10**9, dtype=torch.int64, device="cuda"), short])
    keys = keys[torch.randperm(keys.numel(), device="cuda", generator=g)]
    n = keys.numel()
    p1 = torch.arange(n, dtype=torch.int64, device="cuda")
    p2 = (p1 & 0xFFFF).to(torch.int16)
    outs = (torch.empty_like(keys), torch.empty_like(p1), torch.empty_like(p2))
    srs_amd.sort_device(keys, p1, p2, out=outs)
    ref_k, ref_i = torch.sort(keys, stable=True)
    assert torch.equal(outs[0], ref_k)
    assert torch.equal(outs[1], ref_i)
    assert torch.equal(outs[2], (ref_i & 0xFFFF).to(torch.int16))


def test_placed_device_memory():
    """srs_alloc_device (empty_device): the tensor views the placed block,
    sorts into it match a sort into torch memory, the probe answers."""
    torch = _torch()
    n = (1 << 22) + 77
    keys = torch.empty(n, dtype=torch.int64, device="cuda")
    pays = torch.empty(n, dtype=torch.int64, device="cuda")
    srs_amd.fill_synthetic_device(keys, pays, seed=5 << 32, key_kind=srs_amd.KEY_U64)
    ko, po = srs_amd.empty_device(n, torch.int64), srs_amd.empty_device(n, torch.int64)
    assert ko.is_cuda and ko.numel() == n and ko.dtype == torch.int64
    ko2, po2 = torch.empty_like(keys), torch.empty_like(pays)
    srs_amd.sort_device(keys, pays, key_kind=srs_amd.KEY_U64, out=(ko, po))
    srs_amd.sort_device(keys, pays, key_kind=srs_amd.KEY_U64, out=(ko2, po2))
    torch.cuda.synchronize()
    assert torch.equal(ko, ko2) and torch.equal(po, po2)
    big = srs_amd.empty_device(1 << 28, torch.int64)  # 2 GB: probed placement
    assert srs_amd.debug_probe_write(big.data_ptr(), 8 << 28) > 0
    del big, ko, po
    torch.cuda.synchronize()


@pytest.mark.parametrize("mode", ["1", "3"])
@pytest.mark.parametrize("shape", ["u64_u64", "u32_u32", "u32_keys", "f64_u64", "aos16",
                                   "aos8_f32"])
def test_tile_pair_scatter_all_shapes(shape, mode, monkeypatch):
    """The tile-pair scatter (two count tiles per workgroup)
    forced onto every shape it accepts (SRS_PAIR_TILES=1 / 3: the key plus one
    column of 4- and 8-byte keys, AoS slices): stable, bit for bit, over
    sizes whose levels have pairs that straddle two segments."""
    torch = _torch()
    monkeypatch.setenv("SRS_PAIR_TILES", mode)
    for n in (70_001, 1_234_567):
        for dist in ("uniform", "gaussian"):
            if shape == "aos8_f32":  # DataElement<float, uint32>: record wider than its key
                keys = make_keys(8, dist, n, n % 83)
                rec = np.empty((n, 8), np.uint8)
                rec[:, :4] = keys.view(np.uint8).reshape(n, 4)
                rec[:, 4:] = np.arange(n, dtype=np.uint32).view(np.uint8).reshape(n, 4)
                d = torch.from_numpy(rec.copy()).cuda()
                srs_amd.sort_combined_device(d, 8)
                torch.cuda.synchronize()
                assert bytes_equal(d.cpu().numpy(), stable_aos(8, True, rec)), (shape, n, dist)
                continue
            if shape == "aos16":
                keys = make_keys(6, dist, n, n % 97)
                rec = np.empty((n, 16), np.uint8)
                rec[:, :8] = keys.view(np.uint8).reshape(n, 8)
                rec[:, 8:] = np.arange(n, dtype=np.uint64).view(np.uint8).reshape(n, 8)
                d = torch.from_numpy(rec.copy()).cuda()
                srs_amd.sort_combined_device(d, 6)
                torch.cuda.synchronize()
                assert bytes_equal(d.cpu().numpy(), stable_aos(6, True, rec)), (shape, n, dist)
                continue
            kind = {"u64_u64": 6, "u32_u32": 4, "u32_keys": 4, "f64_u64": 9}[shape]
            keys = make_keys(kind, dist, n, n % 89)
            cols = [keys]
            if shape != "u32_keys":
                cols.append(np.arange(n, dtype=np.uint64 if kind in (6, 9) else np.uint32))
            host = [c.copy() for c in cols]
            srs_amd.sort(*host)
            st = stable_reference(kind, True, cols)
            for a, b in zip(host, st):
                assert bytes_equal(a, b), (shape, n, dist)


def test_tile_pair_scatter_on_the_digit_table_level(monkeypatch):
    """C2's shape at 2^24 + 4321 keys (a balanced digit-table first level)
    with the tile-pair scatter on every level (SRS_PAIR_TILES=3), index
    payloads: stable, bit for bit."""
    torch = _torch()
    monkeypatch.setenv("SRS_PAIR_TILES", "3")
    n = (1 << 24) + 4321
    keys = torch.empty(n, dtype=torch.float32, device="cuda")
    p0 = torch.empty(n, dtype=torch.int32, device="cuda")
    srs_amd.fill_synthetic_device(keys, p0)
    p1 = torch.arange(n, dtype=torch.int32, device="cuda")
    kh, ah, bh = keys.cpu().numpy(), p0.cpu().numpy(), p1.cpu().numpy()
    srs_amd.sort_device(keys, p0, p1)
    torch.cuda.synchronize()
    st = stable_reference(8, True, [kh, ah, bh])
    assert bytes_equal(keys.cpu().numpy(), st[0])
    assert bytes_equal(p0.cpu().numpy(), st[1]) and bytes_equal(p1.cpu().numpy(), st[2])
