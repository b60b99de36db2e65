"""GPU parity tests for the mid-level launch (2^20 < n <= 2^22: the first
level -- count, column scans and scatter into TMP -- in one launch with grid
barriers, each workgroup looping over several tiles; the buckets go to the
work lists and their lengths to the host before the scatter ends, DESIGN.md
§4). Every shape must equal a stable sort bit for bit: every key kind, in
place and out of place, a key with two 4-byte payloads, records (16/32-byte
records as slice columns), keys sharing their top bits (the launch counts
again below them), all-equal keys (copied through), skewed keys whose big
bucket continues on the general levels, 1- and 2-byte keys whose buckets
are final (the copy list past the LDS capacity), and both ends of the range.
"""
import numpy as np
import pytest

from srs_testlib import stable_reference
from test_gpu_sort import bytes_equal, make_keys, payload_of, stable_aos

pytestmark = pytest.mark.gpu

srs_amd = pytest.importorskip("srs_amd")

SIZES = [(1 << 20) + 1, 1_500_001, 1 << 21, (1 << 21) + 3, 3_000_017, (1 << 22) - 1, 1 << 22]


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


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("kind", [4, 6, 7, 8, 9], ids=["u32", "u64", "i64", "f32", "f64"])
def test_mid_level_out_of_place(kind, n):
    torch = _torch()
    keys = make_keys(kind, "uniform", n, 31 * n + kind)
    pay = np.arange(n, dtype=np.uint64)
    dk, dp = _dev(torch, keys), _dev(torch, pay)
    ok, op = torch.empty_like(dk), torch.empty_like(dp)
    srs_amd.sort_device(dk, dp, key_kind=kind, out=(ok, op))
    torch.cuda.synchronize()
    st = stable_reference(kind, True, [keys, pay])
    assert bytes_equal(ok.cpu().numpy(), st[0]) and bytes_equal(op.cpu().numpy(), st[1])
    assert bytes_equal(dk.cpu().numpy(), keys), "the input columns must stay untouched"


@pytest.mark.parametrize("n", [(1 << 20) + 7, 1 << 21, 1 << 22])
@pytest.mark.parametrize("up", [True, False], ids=["up", "down"])
def test_mid_level_in_place_pair_shape(n, up):
    """A 4-byte key and two 4-byte payloads, in place (no pair words here)."""
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


@pytest.mark.parametrize("n", [1_100_000, 2_500_001])
@pytest.mark.parametrize("esz", [8, 16, 32])
def test_mid_level_records(n, esz):
    rng = np.random.default_rng(esz + n)
    keys = make_keys(6, "uniform", n, esz)
    elems = rng.integers(0, 256, (n, esz), dtype=np.uint8)
    elems[:, :8] = keys.view(np.uint8).reshape(n, 8)
    e = elems.copy()
    srs_amd.sort_combined(e, 6)
    assert bytes_equal(e, stable_aos(6, True, elems))


@pytest.mark.parametrize("kind", [0, 1, 2, 3], ids=["u8", "i8", "u16", "i16"])
@pytest.mark.parametrize("dist", ["uniform", "fewdistinct"])
def test_mid_level_short_keys(kind, dist):
    """1- and 2-byte keys: the digit reaches the last bit, every bucket is
    final (LDS pass or, above its capacity, the copy list)."""
    n = 2_000_003
    keys = make_keys(kind, dist, n, kind + 11)
    idx = np.arange(n, dtype=np.uint32)
    k, p = keys.copy(), idx.copy()
    srs_amd.sort(k, p)
    st = stable_reference(kind, True, [keys, idx])
    assert bytes_equal(k, st[0]) and bytes_equal(p, st[1])


@pytest.mark.parametrize("shared", [8, 24, 40, 60])
def test_mid_level_shared_top_bits(shared):
    """Keys whose top `shared` bits are equal: the first count's digit puts
    every key in one bucket and the launch counts again below them."""
    n = 2_100_000
    rng = np.random.default_rng(shared)
    keys = rng.integers(0, 1 << (64 - shared), n, dtype=np.uint64) | np.uint64(0x5A << 56 if shared >= 8 else 0)
    idx = np.arange(n, dtype=np.uint64)
    k, p = keys.copy(), idx.copy()
    srs_amd.sort(k, p)
    order = np.argsort(keys, kind="stable")
    assert bytes_equal(k, keys[order]) and bytes_equal(p, idx[order])


@pytest.mark.parametrize("inplace", [True, False], ids=["inplace", "out"])
def test_mid_level_all_equal(inplace):
    torch = _torch()
    n = 3_000_001
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


@pytest.mark.parametrize("n", [1_200_000, 4_000_000])
def test_mid_level_skewed_bucket_continues(n):
    """80 % of the keys in one first-level bucket: it continues on the
    general levels (the big list), the rest go straight to the LDS pass."""
    rng = np.random.default_rng(n)
    keys = rng.integers(0, 1 << 64, n, dtype=np.uint64)
    m = rng.random(n) < 0.8
    keys[m] = rng.integers(0, 1 << 40, int(m.sum()), dtype=np.uint64)
    idx = np.arange(n, dtype=np.uint64)
    k, p = keys.copy(), idx.copy()
    srs_amd.sort(k, p)
    order = np.argsort(keys, kind="stable")
    assert bytes_equal(k, keys[order]) and bytes_equal(p, idx[order])


@pytest.mark.parametrize("dist", ["gaussian", "fewdistinct", "highbits", "lowbits", "zeroone",
                                  "sorted", "reverse"])
def test_mid_level_distributions(dist):
    for n in (1_048_600, 2_900_000):
        keys = make_keys(7, dist, n, n)
        idx = np.arange(n, dtype=np.uint32)
        k, p = keys.copy(), idx.copy()
        srs_amd.sort(k, p, up=False)
        st = stable_reference(7, False, [keys, idx])
        assert bytes_equal(k, st[0]) and bytes_equal(p, st[1]), (dist, n)


@pytest.mark.parametrize("n", [(1 << 20) + 1, 3_900_000])
def test_mid_level_launch_taken(n):
    """Up to 512 x 7808 keys the first level (the one launch) is the only
    one: no count pass."""
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
    assert launches("mid_level") == 1 and launches("count") == 0
    assert bytes_equal(keys.cpu().numpy(), ref[0]) and bytes_equal(pays.cpu().numpy(), ref[1])


def test_mid_level_streams():
    """Mid-level sorts on two streams interleaved with mid-size and general
    sorts (shared workspace, flag and barrier words): every result exact."""
    torch = _torch()
    dev = torch.device("cuda:0")
    streams = [torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)]
    sizes = [2_000_000, 100_000, 3_500_000, 6_000_000]
    ins, outs = [], []
    for i, n in enumerate(sizes):
        k = torch.empty(n, dtype=torch.int64, device=dev)
        p = torch.empty(n, dtype=torch.int64, device=dev)
        srs_amd.fill_synthetic_device(k, p, seed=99 + i, key_kind=srs_amd.KEY_U64)
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
