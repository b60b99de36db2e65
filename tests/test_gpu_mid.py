"""GPU parity tests for the mid-size single launch (kLocalCap < n <= 2^20:
one launch with grid barriers does the first level and every bucket's local
sort, DESIGN.md §6 "Mid-size sorts"; above 2^18 keys with the count
matrix's column scans spread over the grid). The result must equal a stable sort bit for
bit in every shape the general path takes at these sizes: separate and in
place device columns, key + two 4-byte payloads (the general path's pair
layout is off here), 16-byte records (no slice columns), float keys with
canonicalised zeros (n <= cmp_sort_threshold), all-equal keys (the launch
copies the input through), skewed keys whose one bucket overflows an LDS sort
(the launch hands it to the general levels), and both ends of the range.
"""
import numpy as np
import pytest

from srs_testlib import KIND_DTYPES, stable_reference
from test_gpu_sort import bytes_equal, make_keys, payload_of, stable_aos

pytestmark = pytest.mark.gpu

srs_amd = pytest.importorskip("srs_amd")

MID_SIZES = [8193, 12289, 40000, 131072, 262143, 262144, 262145, 600001, 1048575, 1048576]


def _torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    _torch()
    srs_amd.lib()


def _dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("n", MID_SIZES)
@pytest.mark.parametrize("kind", [4, 6, 7, 8, 9], ids=["u32", "u64", "i64", "f32", "f64"])
def test_mid_device_out_of_place(kind, n):
    """Separate output tensors (IN stays untouched), one 8-byte payload."""
    torch = _torch()
    keys = make_keys(kind, "uniform", n, 17 * n + kind)
    pay = np.arange(n, dtype=np.uint64)
    dk, dp = _dev(torch, keys), _dev(torch, pay)
    ok, op = torch.empty_like(dk), torch.empty_like(dp)
    srs_amd.sort_device(dk, dp, key_kind=kind, out=(ok, op))
    torch.cuda.synchronize()
    st = stable_reference(kind, True, [keys, pay])
    assert bytes_equal(ok.cpu().numpy(), st[0]) and bytes_equal(op.cpu().numpy(), st[1])
    assert bytes_equal(dk.cpu().numpy(), keys), "the input columns must stay untouched"


@pytest.mark.parametrize("n", [8193, 65536, 262144])
@pytest.mark.parametrize("up", [True, False], ids=["up", "down"])
def test_mid_in_place_pair_shape(n, up):
    """A 4-byte key and two 4-byte payloads, sorted in place on the device."""
    torch = _torch()
    keys = make_keys(5, "uniform", n, n)
    a = payload_of(keys, 4)
    b = np.arange(n, dtype=np.uint32)
    dk, da, db = _dev(torch, keys), _dev(torch, a), _dev(torch, b)
    srs_amd.sort_device(dk, da, db, up=up, key_kind=5)
    torch.cuda.synchronize()
    st = stable_reference(5, up, [keys, a, b])
    for got, want in zip((dk, da, db), st):
        assert bytes_equal(got.cpu().numpy(), want)


@pytest.mark.parametrize("n", [9000, 100003, 262144])
@pytest.mark.parametrize("esz", [8, 16, 32])
def test_mid_records(n, esz):
    """DataElement records (key at offset 0, whole records move)."""
    rng = np.random.default_rng(esz * n)
    keys = make_keys(6, "uniform", n, esz)
    elems = rng.integers(0, 256, (n, esz), dtype=np.uint8)
    elems[:, :8] = keys.view(np.uint8).reshape(n, 8)
    e = elems.copy()
    srs_amd.sort_combined(e, 6)
    assert bytes_equal(e, stable_aos(6, True, elems))


@pytest.mark.parametrize("kind", [8, 9], ids=["f32", "f64"])
def test_mid_canonical_zero(kind):
    """n <= cmp_sort_threshold: -0.0 and +0.0 compare equal (the reference's
    insertion sort), so they keep their input order."""
    n = 50000
    rng = np.random.default_rng(kind)
    keys = rng.choice(np.array([-0.0, 0.0, -1.5, 2.25, 1e-30], dtype=KIND_DTYPES[kind]), n)
    idx = np.arange(n, dtype=np.uint32)
    k, p = keys.copy(), idx.copy()
    srs_amd.sort_thresh(n, k, p)
    st = stable_reference(kind, True, [keys, idx], n)
    assert bytes_equal(k, st[0]) and bytes_equal(p, st[1])


@pytest.mark.parametrize("inplace", [True, False], ids=["inplace", "out"])
def test_mid_all_equal(inplace):
    """No varying bit: the launch copies the input through (stable)."""
    torch = _torch()
    n = 70001
    keys = np.full(n, 0x0123_4567_89AB_CDEF, dtype=np.uint64)
    pay = np.arange(n, dtype=np.uint64)
    dk, dp = _dev(torch, keys), _dev(torch, pay)
    if inplace:
        srs_amd.sort_device(dk, dp, key_kind=6)
        ok, op = dk, dp
    else:
        ok, op = torch.zeros_like(dk), torch.zeros_like(dp)
        srs_amd.sort_device(dk, dp, key_kind=6, out=(ok, op))
    torch.cuda.synchronize()
    assert bytes_equal(ok.cpu().numpy(), keys) and bytes_equal(op.cpu().numpy(), pay)


@pytest.mark.parametrize("n", [20000, 262144, 1048576])
def test_mid_skewed_bucket_continues(n):
    """80 % of the keys share the first digit's bucket (> kLocalCap records):
    that bucket goes back to the host's general levels, the rest are sorted
    inside the launch; the stable and LSD fallbacks stay reachable."""
    rng = np.random.default_rng(n)
    keys = rng.integers(0, 1 << 64, n, dtype=np.uint64)
    m = rng.random(n) < 0.8
    keys[m] = rng.integers(0, 1 << 40, int(m.sum()), dtype=np.uint64)
    idx = np.arange(n, dtype=np.uint64)
    k, p = keys.copy(), idx.copy()
    srs_amd.sort(k, p)
    order = np.argsort(keys, kind="stable")
    assert bytes_equal(k, keys[order]) and bytes_equal(p, idx[order])


@pytest.mark.parametrize("dist", ["gaussian", "fewdistinct", "highbits", "lowbits", "zeroone"])
def test_mid_distributions(dist):
    for n in (8200, 33333, 250000):
        keys = make_keys(7, dist, n, n)
        idx = np.arange(n, dtype=np.uint32)
        k, p = keys.copy(), idx.copy()
        srs_amd.sort(k, p, up=False)
        st = stable_reference(7, False, [keys, idx])
        assert bytes_equal(k, st[0]) and bytes_equal(p, st[1]), (dist, n)


def test_mid_nosort_leaves():
    """CmpSorterNoSort: leaves stay unsorted, everything above them is."""
    n = 100000
    keys = make_keys(6, "uniform", n, 5)
    idx = np.arange(n, dtype=np.uint64)
    k, p = keys.copy(), idx.copy()
    srs_amd.sort_thresh(16, k, p, cmp_sorter="nosort")
    assert bytes_equal(keys[p.astype(np.int64)], k)
    assert np.array_equal(np.sort(k), np.sort(keys))


def test_mid_fallback_counters():
    """srs_debug_last_fallbacks reports the launch's own bodies: full-range
    keys of one small bucket take the stable body."""
    n = 9000
    rng = np.random.default_rng(3)
    keys = rng.integers(0, 1 << 64, n, dtype=np.uint64)
    keys[: n - 8] = rng.integers(0, 1 << 20, n - 8, dtype=np.uint64)
    idx = np.arange(n, dtype=np.uint64)
    k, p = keys.copy(), idx.copy()
    srs_amd.sort(k, p)
    order = np.argsort(keys, kind="stable")
    assert bytes_equal(k, keys[order]) and bytes_equal(p, idx[order])
    stable_n, lsd_n = srs_amd.last_fallbacks()
    assert stable_n >= 0 and lsd_n >= 0


def test_mid_two_streams_and_threads():
    """Mid-size sorts queued on two non-blocking streams, interleaved with a
    small and a general-path sort, and from two host threads at once: the
    launches share the workspace (its TMP, counters and the host-memory
    flag), so each call must wait for the previous one's kernels and read
    its own flag only. Every result against a stable sort."""
    import threading
    torch = _torch()
    dev = torch.device("cuda:0")
    streams = [torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)]
    sizes = [100_000, 5_000, 200_003, 3_000_000]
    ins, outs = [], []
    for i, n in enumerate(sizes):
        k = torch.empty(n, dtype=torch.int64, device=dev)
        p = torch.empty(n, dtype=torch.int64, device=dev)
        srs_amd.fill_synthetic_device(k, p, seed=77 + i, key_kind=srs_amd.KEY_U64)
        ins.append((k, p))
        outs.append((torch.empty_like(k), torch.empty_like(p)))
    torch.cuda.synchronize()
    for _ in range(3):
        for j, ((k, p), (ko, po)) in enumerate(zip(ins, outs)):
            s = streams[j % 2]
            s.wait_stream(torch.cuda.current_stream(dev))
            srs_amd.sort_device(k, p, key_kind=srs_amd.KEY_U64, out=(ko, po), stream=s)
    torch.cuda.synchronize()
    for (k, p), (ko, po) in zip(ins, outs):
        st = stable_reference(6, True, [k.cpu().numpy().view(np.uint64), p.cpu().numpy()])
        assert bytes_equal(ko.cpu().numpy(), st[0]) and bytes_equal(po.cpu().numpy(), st[1])

    errors = []

    def worker(t):
        try:
            s = torch.cuda.Stream(device=dev)
            rng = np.random.default_rng(t)
            for it in range(10):
                n = int(rng.integers(8193, 262145))
                keys = rng.integers(0, 1 << 64, n, dtype=np.uint64)
                idx = np.arange(n, dtype=np.uint64)
                with torch.cuda.stream(s):
                    dk = torch.from_numpy(keys.view(np.int64)).to(dev, non_blocking=False)
                    dp = torch.from_numpy(idx.view(np.int64)).to(dev, non_blocking=False)
                    s.synchronize()
                    srs_amd.sort_device(dk, dp, key_kind=srs_amd.KEY_U64, stream=s)
                    s.synchronize()
                order = np.argsort(keys, kind="stable")
                if not (bytes_equal(dk.cpu().numpy(), keys[order]) and
                        bytes_equal(dp.cpu().numpy(), idx[order])):
                    errors.append((t, it, n))
        except Exception as e:  # (reported below)
            errors.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors


def test_many_streams_bound_the_flag_slots():
    """Single-launch sorts on 70 fresh streams (small and mid-size): the
    per-stream fallback-flag slots are recycled past 64 streams; every result
    stays correct and srs_debug_last_fallbacks keeps answering."""
    torch = _torch()
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(70)
    for i in range(70):
        n = 5000 if i % 2 else 20000
        keys = rng.integers(0, 1 << 64, n, dtype=np.uint64)
        idx = np.arange(n, dtype=np.uint64)
        s = torch.cuda.Stream(device=dev)
        dk = torch.from_numpy(keys.view(np.int64)).to(dev)
        dp = torch.from_numpy(idx.view(np.int64)).to(dev)
        torch.cuda.synchronize()
        srs_amd.sort_device(dk, dp, key_kind=srs_amd.KEY_U64, stream=s)
        s.synchronize()
        order = np.argsort(keys, kind="stable")
        assert bytes_equal(dk.cpu().numpy(), keys[order]), i
        assert bytes_equal(dp.cpu().numpy(), idx[order]), i
        stable_n, lsd_n = srs_amd.last_fallbacks()
        assert stable_n >= 0 and lsd_n >= 0


@pytest.mark.parametrize("n", [262145, 1 << 20])
def test_mid_launch_takes_large_sizes(n):
    """Round 6: 2^18 < n <= 2^20 keys take the one launch (the kernel timing
    counts one "mid" launch and no count pass), not the general path."""
    torch = _torch()
    g = torch.Generator(device="cuda")
    g.manual_seed(n)
    keys = torch.randint(-2**63, 2**63 - 1, (n,), dtype=torch.int64, device="cuda", generator=g)
    pays = torch.arange(n, dtype=torch.int64, device="cuda")
    ref = stable_reference(7, True, [keys.cpu().numpy(), pays.cpu().numpy()])
    srs_amd.reset_kernel_stats()
    srs_amd.set_kernel_timing(True)
    try:
        srs_amd.sort_device(keys, pays, key_kind=7)
        torch.cuda.synchronize()
    finally:
        srs_amd.set_kernel_timing(False)
    def launches(name):
        try:
            return srs_amd.kernel_stats(name)[0]
        except Exception:  # (a family that never ran)
            return 0
    assert launches("mid") == 1 and launches("count") == 0
    assert bytes_equal(keys.cpu().numpy(), ref[0]) and bytes_equal(pays.cpu().numpy(), ref[1])
