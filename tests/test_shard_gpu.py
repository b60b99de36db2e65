"""The multi-GPU shard sort through its C ABI (csrc/srs_shard.hip) with the
REAL HIP kernels at world 1-8 on the test box's one GPU. RCCL puts no two
ranks on one device, so world > 1 runs on the host-staged transport
(srs_shard_comm_init_staged: the ranks are threads of this process and only
the collectives and peer messages travel through host memory); world 1 also
runs over RCCL. Everything else is the product path: the chunk histograms,
the header/status collectives, the 512-group partition, the message plan,
the own-piece copies, the round sorts with known prefix bits on the side
stream. The union of the ranks' outputs must equal a stable sort of the
inputs in (rank, index) order, keys and payloads bit for bit, and at
2^25 + 1234 records the reference's own sort (oracle/_ref, radixSort.hpp)."""
import os
import sys
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "simd-radix-sort_amd", "python"))

torch = pytest.importorskip("torch")


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _inputs(world, dist_kind, kind, n_base):
    import srs_amd
    out = []
    for rank in range(world):
        n = n_base + 3_001 * rank  # ragged shards
        g = torch.Generator(device="cuda")
        g.manual_seed(1000 + rank)
        pay = torch.arange(n, dtype=torch.int64, device="cuda") + rank * 10**7
        if dist_kind == "c4":  # BASELINE C4's generator: global indices [r * n, (r + 1) * n)
            keys = torch.empty(n, dtype=torch.int64, device="cuda")
            srs_amd.fill_synthetic_device(keys, pay, seed=42 << 32, first_index=rank * n_base,
                                          key_kind=kind)
        elif dist_kind == "uniform":
            keys = torch.randint(-2**63, 2**63 - 1, (n,), dtype=torch.int64, device="cuda",
                                 generator=g)
        elif dist_kind == "skewed":  # a few top buckets + duplicates
            keys = (torch.randint(0, 3, (n,), dtype=torch.int64, device="cuda", generator=g) << 61
                    | torch.randint(0, 5000, (n,), dtype=torch.int64, device="cuda", generator=g))
        elif dist_kind == "equal":
            keys = torch.full((n,), 77, dtype=torch.int64, device="cuda")
        elif dist_kind == "empty1":  # rank 1 holds nothing
            keys = torch.randint(-2**63, 2**63 - 1, (0 if rank == 1 else n,), dtype=torch.int64,
                                 device="cuda", generator=g)
            pay = pay[:keys.numel()].contiguous()
        else:  # floats
            keys = torch.randn(n, device="cuda", generator=g)
        out.append((keys, [pay]))
    torch.cuda.synchronize()
    return out


def _check_union(inputs, outs, kind):
    from srs_testlib import transformed_keys
    ink = np.concatenate([k.cpu().numpy() for k, _ in inputs])
    inp = np.concatenate([p[0].cpu().numpy() for _, p in inputs])
    order = np.argsort(transformed_keys(kind, True, ink), kind="stable")
    outk = np.concatenate([k.cpu().numpy() for k, _ in outs])
    outp = np.concatenate([p[0].cpu().numpy() for _, p in outs])
    assert np.array_equal(outk.view(np.uint8), ink[order].view(np.uint8))
    assert np.array_equal(outp, inp[order])


@pytest.mark.parametrize("world,dist_kind,kind,n_base,rounds,chunks", [
    (2, "uniform", 7, 200_000, 0, 0), (3, "skewed", 7, 200_000, 0, 0),
    (4, "uniform", 7, 200_000, 0, 0), (3, "equal", 7, 200_000, 0, 0),
    (2, "float", 8, 200_000, 0, 0), (3, "empty1", 7, 100_000, 0, 0),
    (4, "uniform", 6, 300_000, 16, 8), (3, "skewed", 6, 200_000, 1, 1),
    (2, "uniform", 7, 50_000, 64, 16),
    # C4's shape (u64 key + f(key) payload from global indices) at 8 ranks
    (8, "c4", 6, 1_000_000, 0, 0)])
def test_shard_staged_multi_rank(world, dist_kind, kind, n_base, rounds, chunks):
    _need_gpu()
    from srs_amd import shard
    comms = shard.staged(world)
    for c in comms:
        c.set_options(rounds, chunks)
    inputs = _inputs(world, dist_kind, kind, n_base)
    for _ in range(2):  # twice: buffers are reused
        outs = shard.sort_multi(comms, inputs, key_kind=kind)
    _check_union(inputs, outs, kind)
    # the inputs are untouched
    again = _inputs(world, dist_kind, kind, n_base)
    for (a, _), (b, _) in zip(inputs, again):
        assert torch.equal(a, b)
    for r, c in enumerate(comms):
        rep = c.report()
        assert rep["transport"] == "staged" and rep["world"] == world and rep["rank"] == r
        assert rep["records_out"] == outs[r][0].numel()
        st = rep["stamps_ms"]
        R = rep["rounds"]
        need = ["start", "hist", "plan", "end"] + [f"partition{i}" for i in range(rep["chunks"])] \
            + [f"round{i}_{x}" for i in range(R) for x in ("recv", "sort_start", "sort_end")]
        assert all(k in st for k in need), (need, st)
        assert len(rep["bytes_to_peer_per_round"]) == R
        assert all(b[r] == 0 for b in rep["bytes_to_peer_per_round"])
        lf = shard.link_figures(rep)
        assert set(lf["model"]) == {"T_ms_at_50GBs", "T_ms_at_64GBs", "T_ms_at_77GBs"}
    del outs
    for c in comms:
        c.close()


def test_shard_staged_matches_reference():
    """C1's shape (u64 key + f(key) u64 payload) spread over 3 ragged ranks,
    2^25 + 1234 records in all: the union of the shard outputs equals the
    REFERENCE's own sort of the concatenated input (oracle/_ref)."""
    _need_gpu()
    import srs_amd
    from srs_amd import shard
    from srs_testlib import ref_lib, ref_sort_soa
    if ref_lib() is None:
        pytest.fail("oracle/_ref/libsrs_ref.so missing or host lacks AVX-512 VBMI2")
    total = (1 << 25) + 1234
    cuts = [0, total // 5, total // 5 + total // 2, total]
    keys = torch.empty(total, dtype=torch.int64, device="cuda")
    pays = torch.empty(total, dtype=torch.int64, device="cuda")
    srs_amd.fill_synthetic_device(keys, pays, seed=7 << 32, key_kind=srs_amd.KEY_U64)
    inputs = [(keys[a:b], [pays[a:b]]) for a, b in zip(cuts[:-1], cuts[1:])]
    comms = shard.staged(3)
    outs = shard.sort_multi(comms, inputs, key_kind=srs_amd.KEY_U64)
    k = keys.cpu().numpy().view(np.uint64).copy()
    p = pays.cpu().numpy().view(np.uint64).copy()
    ref_sort_soa(srs_amd.KEY_U64, True, k, [p])
    outk = np.concatenate([o[0].cpu().numpy() for o in outs]).view(np.uint64)
    outp = np.concatenate([o[1][0].cpu().numpy() for o in outs]).view(np.uint64)
    assert np.array_equal(outk, k)
    assert np.array_equal(outp, p)
    del outs
    for c in comms:
        c.close()


@pytest.mark.parametrize("rounds,chunks", [(0, 0), (8, 4), (16, 8)])
def test_shard_rccl_world1_equals_plain_sort(rounds, chunks):
    """One rank over RCCL (srs_shard_comm_init): one chunk sorts the rounds
    in the partition buffer (alias); several chunks take the receive-buffer
    path with own-piece copies. Both equal the one-GPU sort bit for bit."""
    _need_gpu()
    import srs_amd
    from srs_amd import shard
    n = 3_000_017
    keys = torch.empty(n, dtype=torch.int64, device="cuda")
    pays = torch.empty(n, dtype=torch.int64, device="cuda")
    srs_amd.fill_synthetic_device(keys, pays, seed=11 << 32, key_kind=srs_amd.KEY_U64)
    ko, po = torch.empty_like(keys), torch.empty_like(pays)
    srs_amd.sort_device(keys, pays, key_kind=srs_amd.KEY_U64, out=(ko, po))
    comm = shard.ShardComm.rccl(1, 0, shard.unique_id())
    comm.set_options(rounds, chunks)
    k, (p,) = comm.sort(keys, pays, key_kind=srs_amd.KEY_U64)
    torch.cuda.synchronize()
    assert torch.equal(k, ko) and torch.equal(p, po)
    rep = comm.report()
    assert rep["transport"] == "rccl" and rep["chunks"] == (chunks or 1)
    del k, p
    comm.close()


@pytest.mark.parametrize("rounds,chunks,cap", [(16, 8, 64 << 10), (8, 1, 0), (3, 2, 4096)])
def test_shard_rccl_self_messages(rounds, chunks, cap):
    """the RCCL point-to-point path on hardware. With self
    messages a single rank posts every piece as an ncclSend / ncclRecv to
    itself inside the wavefront's grouped posts (no device copies), with a
    small message cap forcing the split of each piece into several messages;
    the receive events on the communication stream and the bounded polling
    beside in-flight RCCL kernels all run. Equal to the one-GPU sort bit for
    bit; the report shows the messages and their bytes."""
    _need_gpu()
    import srs_amd
    from srs_amd import shard
    n = 3_000_017
    keys = torch.empty(n, dtype=torch.int64, device="cuda")
    pays = torch.empty(n, dtype=torch.int64, device="cuda")
    srs_amd.fill_synthetic_device(keys, pays, seed=13 << 32, key_kind=srs_amd.KEY_U64)
    ko, po = torch.empty_like(keys), torch.empty_like(pays)
    srs_amd.sort_device(keys, pays, key_kind=srs_amd.KEY_U64, out=(ko, po))
    comm = shard.ShardComm.rccl(1, 0, shard.unique_id())
    comm.set_options(rounds, chunks)
    comm.set_message_options(True, cap)
    for _ in range(2):  # (buffers reused)
        k, (p,) = comm.sort(keys, pays, key_kind=srs_amd.KEY_U64)
        torch.cuda.synchronize()
        assert torch.equal(k, ko) and torch.equal(p, po)
    rep = comm.report()
    assert rep["transport"] == "rccl" and rep["self_messages"] == 1
    assert rep["max_message_bytes"] == (cap or 256 << 20)
    pieces = rounds * chunks  # (uniform keys: every (round, chunk) piece is non-empty)
    assert rep["sends"] == rep["recvs"] >= 2 * pieces
    if cap and cap < 8 * n // pieces:
        assert rep["sends"] > 2 * pieces  # (pieces split into several messages)
    sent = sum(b[0] for b in rep["bytes_to_peer_per_round"])
    assert sent == 16 * n
    lf = shard.link_figures(rep)
    assert lf["busiest_link_bytes"] == 16 * n and lf.get("link_gbs", 0) > 0
    del k, p
    comm.close()


def test_shard_rccl_self_messages_match_reference():
    """C1's shape at 2^25 + 1234 records through one rank's RCCL self
    messages (8 chunks, 16 rounds, 1 MiB messages: each ~2 MB piece of a
    column split in several): equal to the REFERENCE's own sort
    (oracle/_ref, radixSort.hpp)."""
    _need_gpu()
    import srs_amd
    from srs_amd import shard
    from srs_testlib import ref_lib, ref_sort_soa
    if ref_lib() is None:
        pytest.fail("oracle/_ref/libsrs_ref.so missing or host lacks AVX-512 VBMI2")
    n = (1 << 25) + 1234
    keys = torch.empty(n, dtype=torch.int64, device="cuda")
    pays = torch.empty(n, dtype=torch.int64, device="cuda")
    srs_amd.fill_synthetic_device(keys, pays, seed=17 << 32, key_kind=srs_amd.KEY_U64)
    comm = shard.ShardComm.rccl(1, 0, shard.unique_id())
    comm.set_options(16, 8)
    comm.set_message_options(True, 1 << 20)
    k, (p,) = comm.sort(keys, pays, key_kind=srs_amd.KEY_U64)
    torch.cuda.synchronize()
    kr = keys.cpu().numpy().view(np.uint64).copy()
    pr = pays.cpu().numpy().view(np.uint64).copy()
    ref_sort_soa(srs_amd.KEY_U64, True, kr, [pr])
    assert np.array_equal(k.cpu().numpy().view(np.uint64), kr)
    assert np.array_equal(p.cpu().numpy().view(np.uint64), pr)
    rep = comm.report()
    assert rep["sends"] > 2 * 16 * 8 and rep["deferred_frees"] >= 0
    del k, p
    comm.close()


def test_shard_staged_self_messages():
    """Self messages over the host-staged transport at world 3 (the FIFO of a
    rank to itself), with a message cap that splits pieces: the union equals a
    stable sort."""
    _need_gpu()
    from srs_amd import shard
    comms = shard.staged(3)
    for c in comms:
        c.set_options(4, 2)
        c.set_message_options(True, 8192)
    inputs = _inputs(3, "skewed", 7, 100_000)
    outs = shard.sort_multi(comms, inputs, key_kind=7)
    _check_union(inputs, outs, 7)
    for r, c in enumerate(comms):
        rep = c.report()
        assert rep["self_messages"] == 1
        assert sum(b[r] for b in rep["bytes_to_peer_per_round"]) > 0
    del outs
    for c in comms:
        c.close()


def test_shard_message_cap_must_agree():
    """Ranks with different message caps would split pieces differently:
    the header collective fails every rank."""
    _need_gpu()
    from srs_amd import shard
    comms = shard.staged(2)
    comms[1].set_message_options(False, 4096)
    inputs = _inputs(2, "uniform", 7, 50_000)
    with pytest.raises(Exception, match="disagree on the message cap"):
        shard.sort_multi(comms, inputs, key_kind=7)
    for c in comms:
        c.close()


def _two_gpus():
    if not torch.cuda.is_available() or torch.cuda.device_count() < 2:
        pytest.skip("needs 2 GPUs (RCCL puts no two ranks on one device)")


def test_shard_rccl_two_ranks():
    """two ranks over RCCL (srs_shard_comm_init_all, one thread
    per rank): the union equals a stable sort of the inputs. Skipped on a
    one-GPU box (the driver's 8-GPU node runs it)."""
    _two_gpus()
    from srs_amd import shard
    comms = shard.init_all([0, 1])
    inputs = []
    for r in range(2):
        with torch.cuda.device(r):
            n = 400_000 + 1001 * r
            g = torch.Generator(device=f"cuda:{r}")
            g.manual_seed(5 + r)
            k = torch.randint(-2**63, 2**63 - 1, (n,), dtype=torch.int64, device=f"cuda:{r}",
                              generator=g)
            p = torch.arange(n, dtype=torch.int64, device=f"cuda:{r}") + r * 10**7
            inputs.append((k, [p]))
    for c in comms:
        c.set_options(4, 2)
    outs = shard.sort_multi(comms, inputs, key_kind=7)
    _check_union(inputs, outs, 7)
    del outs
    for c in comms:
        c.close()


@pytest.mark.parametrize("point", [3, 4, 5])
def test_shard_rccl_two_ranks_failures(point):
    """failure injection over RCCL at two ranks: a late partition
    or round-sort failure fails both ranks with the communicators usable; a
    transport failure aborts both."""
    _two_gpus()
    from srs_amd import shard
    comms = shard.init_all([0, 1])
    inputs = []
    for r in range(2):
        with torch.cuda.device(r):
            k = torch.randint(-2**63, 2**63 - 1, (200_000,), dtype=torch.int64, device=f"cuda:{r}")
            inputs.append((k, [torch.arange(200_000, dtype=torch.int64, device=f"cuda:{r}")]))
    comms[1].inject(point)
    with pytest.raises(Exception):
        shard.sort_multi(comms, inputs, key_kind=7)
    if point == 5:
        with pytest.raises(Exception, match="aborted"):
            shard.sort_multi(comms, inputs, key_kind=7)
    else:
        outs = shard.sort_multi(comms, inputs, key_kind=7)
        _check_union(inputs, outs, 7)
        del outs
    for c in comms:
        c.close()


def _per_rank_threads(comms, inputs, kind, ranks_opts=None):
    """Each rank's srs_shard_sort_device from its own host thread; returns
    [(ok, error text, seconds)] per rank."""
    res = [None] * len(comms)

    def run(i):
        t0 = time.time()
        try:
            with torch.cuda.device(comms[i].device):
                s = torch.cuda.Stream()
                k, ps = inputs[i]
                comms[i].sort(k, *ps, key_kind=kind, stream=s)
            res[i] = (True, "", time.time() - t0)
        except Exception as e:
            res[i] = (False, str(e), time.time() - t0)
    th = [threading.Thread(target=run, args=(i,)) for i in range(len(comms))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a rank hung"
    return res


@pytest.mark.parametrize("point", [1, 2, 3, 4])
def test_shard_one_rank_fails_every_rank_fails(point):
    """VERDICT r04 / ADVICE r04: one rank's failure (a bad argument, an
    allocation before the exchange, its partition after the first messages,
    its last round's sort) makes every rank return an error within seconds,
    none hangs, and the communicators stay usable: the next sort is right."""
    _need_gpu()
    from srs_amd import shard
    comms = shard.staged(3)
    inputs = _inputs(3, "uniform", 7, 200_000)
    comms[1].inject(point)
    res = _per_rank_threads(comms, inputs, 7)
    assert all(not ok for ok, _, _ in res), res
    assert all(dt < 60 for _, _, dt in res), res
    assert "injected" in res[1][1], res
    assert all("rank(s) 1" in e for i, (_, e, _) in enumerate(res) if i != 1), res
    outs = shard.sort_multi(comms, inputs, key_kind=7)  # still usable
    _check_union(inputs, outs, 7)
    del outs
    for c in comms:
        c.close()


def test_shard_transport_failure_aborts_every_rank():
    """A transport failure after the first messages (injected abort on rank
    2) ends every rank's sort with an error; the communicators are dead."""
    _need_gpu()
    from srs_amd import shard
    comms = shard.staged(3)
    inputs = _inputs(3, "uniform", 7, 100_000)
    comms[2].inject(5)
    res = _per_rank_threads(comms, inputs, 7)
    assert all(not ok for ok, _, _ in res), res
    assert all(dt < 60 for _, _, dt in res), res
    with pytest.raises(Exception, match="aborted"):
        shard.sort_multi(comms, inputs, key_kind=7)
    for c in comms:
        c.close()


@pytest.mark.parametrize("what", ["rounds", "kind"])
def test_shard_ranks_disagree_every_rank_fails(what):
    """Ranks that disagree on the options or the key kind all fail (no rank
    sizes a collective differently from another)."""
    _need_gpu()
    from srs_amd import shard
    comms = shard.staged(3)
    inputs = _inputs(3, "uniform", 7, 50_000)
    kinds = [7, 7, 7]
    if what == "rounds":
        comms[1].set_options(2, 0)
    else:
        kinds[2] = 6
    res = [None] * 3

    def run(i):
        try:
            k, ps = inputs[i]
            comms[i].sort(k, *ps, key_kind=kinds[i], stream=torch.cuda.Stream())
            res[i] = "ok"
        except Exception as e:
            res[i] = str(e)
    th = [threading.Thread(target=run, args=(i,)) for i in range(3)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert all(r != "ok" and r is not None and "disagree" in r for r in res), res
    for c in comms:
        c.close()
