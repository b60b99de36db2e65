"""Multi-process tests of the top-radix-bits shard protocol (srs_amd.dist)
on CPU with the gloo backend, world_size 2 and 3. The device kernels are
replaced by a numpy backend that follows the same contracts (stable
partition by a bucket -> rank table; stable sort in the reference key order);
the GPU kernels themselves are covered by the -m gpu tests."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from srs_testlib import KIND_UINT, key_size, transformed_keys


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class NumpyShardOps:
    """CPU stand-in for HipShardOps with the same contracts."""

    def __init__(self, kind):
        self.kind = kind

    def _u(self, keys):
        return transformed_keys(self.kind, True, keys.numpy())

    def histogram(self, keys, bits):
        top = self._u(keys) >> np.uint64(8 * key_size(self.kind) - bits)
        return torch.from_numpy(np.bincount(top.astype(np.int64), minlength=1 << bits)
                                .astype(np.int64))

    def partition(self, keys, pays, bits, part_of_bucket, nparts, out):
        top = (self._u(keys) >> np.uint64(8 * key_size(self.kind) - bits)).astype(np.int64)
        dest = part_of_bucket.numpy()[top]
        order = np.argsort(dest, kind="stable")
        out[0][:len(order)] = keys[torch.from_numpy(order)]
        for o, p in zip(out[1:], pays):
            o[:len(order)] = p[torch.from_numpy(order)]
        return np.bincount(dest, minlength=nparts).tolist()

    def sort(self, keys, pays):
        order = torch.from_numpy(np.argsort(self._u(keys), kind="stable"))
        keys.copy_(keys[order])
        for p in pays:
            p.copy_(p[order])

    def sort_segments(self, keys, pays, bounds, known_top_bits=0, stamp=None):
        if stamp:
            stamp("sort_start", None)
        # the known prefix must really be shared inside every segment
        for a, b in zip(bounds[:-1], bounds[1:]):
            if b > a and known_top_bits:
                top = self._u(keys[a:b]) >> np.uint64(8 * key_size(self.kind) - known_top_bits)
                assert (top == top[0]).all()
        for a, b in zip(bounds[:-1], bounds[1:]):
            self.sort(keys[a:b], [p[a:b] for p in pays])
        if stamp:
            stamp("sort_end", None)

    def finish(self, device):
        pass


def _worker(rank, world, port, kind, n_per, dist_kind, q, bits=8, chunks=4):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "simd-radix-sort_amd",
                                    "python"))
    from srs_amd.dist import ShardSorter
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _run(rank, world, kind, n_per, dist_kind, q, bits, chunks)
    except Exception as e:  # report instead of hanging the parent
        q.put(("error", repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _run(rank, world, kind, n_per, dist_kind, q, bits=8, chunks=4):
    from srs_amd.dist import ShardSorter
    if True:
        rng = np.random.default_rng(100 + rank)
        ut = KIND_UINT[kind]
        n = n_per + rank * 17  # ragged shard sizes
        if dist_kind == "uniform":
            k = rng.integers(0, 2**63, n, dtype=np.uint64).astype(ut)
        elif dist_kind == "skewed":  # everything in a few top buckets
            k = (rng.integers(0, 3, n, dtype=np.uint64) << np.uint64(8 * key_size(kind) - 3)
                 | rng.integers(0, 1000, n, dtype=np.uint64)).astype(ut)
        else:  # all equal
            k = np.full(n, 7, dtype=ut)
        keys = torch.from_numpy(k.copy())
        pay = torch.from_numpy(np.arange(n, dtype=np.int64) + rank * 10**9)
        sorter = ShardSorter(NumpyShardOps(kind), n, [torch.int64], keys.dtype, "cpu", bits=bits,
                             chunk_bytes=1024, chunks=chunks)  # many exchange rounds
        # never more groups than histogram bins of the (clamped) key width
        assert sorter.groups <= 1 << sorter.bits
        ok, (op,) = sorter.sort(keys, [pay])
        _check_phases(sorter, world, rank, n)
        mine = ok.numpy().copy()
        u = transformed_keys(kind, True, mine)
        sorted_ok = bool(np.all(u[1:] >= u[:-1]))
        # boundary check with the next rank, and a multiset check on rank 0
        lohi = torch.tensor([int(u[0]) if len(u) else -1, int(u[-1]) if len(u) else -1],
                            dtype=torch.float64)
        allb = [torch.zeros(2, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(allb, lohi)
        gathered_k = [None] * world
        gathered_p = [None] * world
        dist.all_gather_object(gathered_k, mine.tolist())
        dist.all_gather_object(gathered_p, op.numpy().tolist())
        inputs = [None] * world
        dist.all_gather_object(inputs, (k.tolist(), pay.numpy().tolist()))
        if rank == 0:
            outk = np.concatenate([np.array(g, dtype=ut) for g in gathered_k])
            outp = np.concatenate([np.array(g, dtype=np.int64) for g in gathered_p])
            ink = np.concatenate([np.array(i[0], dtype=ut) for i in inputs])
            inp = np.concatenate([np.array(i[1], dtype=np.int64) for i in inputs])
            ref = np.argsort(transformed_keys(kind, True, ink), kind="stable")
            q.put((sorted_ok, np.array_equal(outk, ink[ref]),
                   sorted(zip(outk.tolist(), outp.tolist())) ==
                   sorted(zip(ink.tolist(), inp.tolist())),
                   [b.tolist() for b in allb]))
        else:
            q.put((sorted_ok, True, True, None))


def _check_phases(sorter, world, rank, n):
    """bench.py's N > 1 line carries ShardSorter.phases() of every rank: the
    stamps of each phase, the bytes sent to each peer per round, the implied
    link rate and the DESIGN.md §7 model's prediction (JSON-serializable)."""
    import json
    ph = sorter.phases()
    json.dumps(ph)
    st = ph["stamps_ms"]
    R = sorter.rounds
    C = sorter.chunks
    need = ["start", "hist", "plan", "end"] + [f"partition{c}" for c in range(C)] + \
        [f"round{r}_recv" for r in range(R)]
    assert all(k in st for k in need), (need, st)
    assert st["start"] == 0 and all(v >= 0 for v in st.values())
    assert st["plan"] >= st["hist"] and st["end"] >= st[f"round{R - 1}_recv"]
    b = ph["bytes_to_peer_per_round"]
    assert len(b) == R and all(len(x) == world and x[rank] == 0 for x in b)
    tot = sum(sum(x) for x in b)
    assert tot <= n * sorter.rec_bytes
    assert ph["busiest_link_bytes"] == max(sum(x[d] for x in b) for d in range(world))
    assert set(ph["model"]) == {"T_ms_at_50GBs", "T_ms_at_77GBs"}
    assert ph["measured_T_ms"] == st["end"]


def _run_world(world, kind, dist_kind, bits=8, chunks=4):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, 3000, dist_kind, q, bits,
                                               chunks))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert not [r for r in res if r[0] == "error"], res
    for sorted_ok, keys_ok, multiset_ok, bounds in res:
        assert sorted_ok and keys_ok and multiset_ok
    b = [r[3] for r in res if r[3] is not None][0]
    nonempty = [x for x in b if x[0] >= 0]
    for a, c in zip(nonempty, nonempty[1:]):
        assert a[1] <= c[0]  # last key of rank r <= first key of rank r+1


@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("dist_kind", ["uniform", "skewed", "equal"])
def test_shard_sort_gloo(world, dist_kind):
    _run_world(world, 6, dist_kind)


@pytest.mark.parametrize("chunks", [1, 3])
def test_shard_sort_gloo_partition_chunks(chunks):
    """the partition in 1 or 3 input chunks (the first round's messages of a
    chunk overlap the next chunk's partition): same result, stable"""
    _run_world(3, 6, "skewed", chunks=chunks)


@pytest.mark.parametrize("kind", [0, 3])  # u8, i16: keys narrower than the default 12 bits
@pytest.mark.parametrize("dist_kind", ["uniform", "skewed"])
def test_shard_sort_gloo_narrow_keys(kind, dist_kind):
    _run_world(2, kind, dist_kind, bits=12)


def test_balanced_split_is_monotone_and_balanced():
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "simd-radix-sort_amd",
                                    "python"))
    from srs_amd.dist import balanced_split
    h = torch.tensor([5, 0, 100, 3, 3, 3, 50, 0, 0, 36], dtype=torch.int64)
    for w in (1, 2, 3, 8):
        p = balanced_split(h, w)
        assert p.dtype == torch.int32 and len(p) == len(h)
        assert bool((p[1:] >= p[:-1]).all()) and int(p.min()) >= 0 and int(p.max()) < w
    u = balanced_split(torch.full((256,), 10, dtype=torch.int64), 8)
    assert torch.bincount(u.long(), minlength=8).tolist() == [32] * 8


class _BadCountOps(NumpyShardOps):
    """Reports wrong group sizes for the second partition chunk (after the
    first chunk's messages are posted)."""

    def __init__(self, kind):
        super().__init__(kind)
        self.calls = 0

    def partition(self, *a, **k):
        got = super().partition(*a, **k)
        self.calls += 1
        if self.calls == 2:
            got = list(got)
            got[0] += 1
        return got


def _bad_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "simd-radix-sort_amd",
                                    "python"))
    from srs_amd.dist import ShardSorter
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(rank)
    n = 4000
    keys = torch.from_numpy(rng.integers(0, 2**63, n, dtype=np.uint64))
    pay = torch.arange(n, dtype=torch.int64)
    ops = _BadCountOps(6) if rank == 0 else NumpyShardOps(6)
    sorter = ShardSorter(ops, n, [torch.int64], keys.dtype, "cpu", bits=8, chunk_bytes=1024,
                         chunks=3)
    try:
        sorter.sort(keys, [pay])
        q.put((rank, "finished"))
    except Exception as e:
        q.put((rank, type(e).__name__ + ": " + str(e)[:200]))
    dist.destroy_process_group()


def test_shard_sort_failure_does_not_hang_peers():
    """a rank that finds its partition sizes wrong after posting
    messages keeps to the agreed message plan, so its peers are not left
    waiting on receives, and every rank raises at the end."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bad_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert "partition sizes differ" in res[0], res
    assert "partition sizes differ" in res[1] and "another rank" in res[1], res
    for p in procs:
        assert p.exitcode == 0
