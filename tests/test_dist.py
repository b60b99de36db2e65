"""The multi-GPU shard protocol's plan on CPU: the library's own planner
(srs_debug_shard_plan: the host code srs_shard.hip runs on every rank, no
GPU needed) drives a gloo world of 2-4 processes. Each rank histograms and
partitions its keys with numpy (stable, by the plan's bin -> group table),
executes the plan's message groups in its posting order with gloo
send/recv, sorts each round's segments with numpy after checking the top
key bits the plan says they share, and the union must equal a stable sort of
every rank's input in (rank, index) order. The device side of the same
protocol (histogram, partition and round-sort kernels, both transports) runs
in tests/test_shard_gpu.py. The reference has no multi-device path."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from srs_testlib import KIND_UINT, key_size, transformed_keys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard():
    sys.path.insert(0, os.path.join(REPO, "simd-radix-sort_amd", "python"))
    from srs_amd import shard
    return shard


def _top(kind, keys, bits):
    return (transformed_keys(kind, True, keys) >> np.uint64(8 * key_size(kind) - bits)).astype(
        np.int64)


def _chunk_bound(n, c, chunks):
    """The library's chunk bounds (srs_shard.hip chunk_bound): the first
    chunk weighs 1, every other 4."""
    if c <= 0:
        return 0
    if c >= chunks:
        return n
    return n * (4 * c - 3) // (4 * chunks - 3)


def _chunk_hists(kind, keys, chunks, bits):
    n = len(keys)
    out = np.zeros((chunks, 1 << bits), np.uint64)
    top = _top(kind, keys, bits)
    for c in range(chunks):
        a, b = _chunk_bound(n, c, chunks), _chunk_bound(n, c + 1, chunks)
        out[c] = np.bincount(top[a:b], minlength=1 << bits)
    return out


def _make_keys(kind, dist_kind, n, rng):
    ut = KIND_UINT[kind]
    kb = 8 * key_size(kind)
    if dist_kind == "uniform":
        return rng.integers(0, 2**63, n, dtype=np.uint64).astype(ut)
    if dist_kind == "skewed":  # a few top buckets + duplicates
        return (rng.integers(0, 3, n, dtype=np.uint64) << np.uint64(kb - 3)
                | rng.integers(0, 1000, n, dtype=np.uint64)).astype(ut)
    return np.full(n, 7, dtype=ut)  # all equal


def _run_rank(rank, world, kind, dist_kind, n_per, chunks, rounds, self_msgs=False):
    shard = _shard()
    rng = np.random.default_rng(100 + rank)
    n = n_per + rank * 17  # ragged shards
    keys = _make_keys(kind, dist_kind, n, rng)
    pay = np.arange(n, dtype=np.int64) + rank * 10**9
    kbits = 8 * key_size(kind)
    bits = min(12, kbits)
    ch = _chunk_hists(kind, keys, chunks, bits)
    allh = [torch.zeros(ch.shape, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(allh, torch.from_numpy(ch.view(np.int64)))
    allh = np.stack([h.numpy().view(np.uint64) for h in allh])
    plan = shard.debug_plan(world, rank, chunks, rounds, kbits, allh, n, self_messages=self_msgs)
    assert not (self_msgs and plan["alias"])
    gob = np.array(plan["group_of_bin"], np.int64)
    # the partition (the device's srs_partition_device): per chunk, stable by group
    top = _top(kind, keys, bits)
    kcol = keys.view(KIND_UINT[kind]).astype(np.int64)  # bits, widened for gloo
    part_k, part_p = np.empty_like(kcol), np.empty_like(pay)
    cbnd = plan["chunk_bounds"]
    assert cbnd == [_chunk_bound(n, c, chunks) for c in range(chunks + 1)]
    for c in range(chunks):
        a, b = cbnd[c], cbnd[c + 1]
        order = a + np.argsort(gob[top[a:b]], kind="stable")
        part_k[a:b], part_p[a:b] = kcol[order], pay[order]
    total = plan["total"]
    if plan["alias"]:
        recv_k, recv_p = part_k, part_p
    else:
        recv_k, recv_p = np.zeros(total, np.int64), np.zeros(total, np.int64)
    cols = [(part_k, recv_k), (part_p, recv_p)]
    own = []  # self messages in posting order (gloo has no send to self)
    for post in plan["posts"]:
        ops, landings = [], []
        for op, peer, src, dst, cnt in post["msgs"]:
            assert cnt > 0 and (peer != rank or self_msgs) or op == 2
            assert not (self_msgs and op == 2)
            for sbuf, rbuf in cols:
                if op == 0 and peer == rank:
                    own.append(sbuf[src:src + cnt].copy())
                elif op == 1 and peer == rank:
                    m = own.pop(0)
                    assert len(m) == cnt
                    rbuf[dst:dst + cnt] = m
                elif op == 0:
                    ops.append(dist.P2POp(dist.isend, torch.from_numpy(sbuf[src:src + cnt].copy()),
                                          peer))
                elif op == 1:
                    t = torch.zeros(cnt, dtype=torch.int64)
                    ops.append(dist.P2POp(dist.irecv, t, peer))
                    landings.append((rbuf, dst, t))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        for rbuf, dst, t in landings:
            rbuf[dst:dst + len(t)] = t.numpy()
        for op, peer, src, dst, cnt in post["msgs"]:
            if op == 2:
                for sbuf, rbuf in cols:
                    rbuf[dst:dst + cnt] = sbuf[src:src + cnt]
    # the rounds: each a contiguous key range, sorted as the plan's segments
    assert plan["rounds"][0]["start"] == 0 and plan["rounds"][-1]["end"] == total
    ut = KIND_UINT[kind]
    rk = recv_k.astype(ut)
    for rd in plan["rounds"]:
        a = rd["start"]
        bnd = rd["bounds"]
        kn = rd["known_bits"]
        for s0, s1 in zip(bnd[:-1], bnd[1:]):
            seg = rk[a + s0:a + s1].view(keys.dtype)
            if kn and len(seg):
                t = transformed_keys(kind, True, seg) >> np.uint64(kbits - kn)
                assert (t == t[0]).all(), ("known bits not shared", rd)
            order = a + s0 + np.argsort(transformed_keys(kind, True, seg), kind="stable")
            rk[a + s0:a + s1] = rk[order]
            recv_p[a + s0:a + s1] = recv_p[order]
    return keys, pay, rk.view(keys.dtype), recv_p


def _worker(rank, world, port, kind, dist_kind, n_per, chunks, rounds, self_msgs, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        keys, pay, ok, op = _run_rank(rank, world, kind, dist_kind, n_per, chunks, rounds,
                                      self_msgs)
        outs = [None] * world
        dist.all_gather_object(outs, (keys, pay, ok, op))
        if rank == 0:
            ink = np.concatenate([o[0] for o in outs])
            inp = np.concatenate([o[1] for o in outs])
            outk = np.concatenate([o[2] for o in outs])
            outp = np.concatenate([o[3] for o in outs])
            ref = np.argsort(transformed_keys(kind, True, ink), kind="stable")
            q.put(("ok", bool(np.array_equal(outk.view(np.uint8), ink[ref].view(np.uint8))),
                   bool(np.array_equal(outp, inp[ref]))))
    except Exception as e:  # report instead of hanging the parent
        q.put(("error", repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _run_world(world, kind, dist_kind, chunks=4, rounds=3, n_per=3000, self_msgs=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, dist_kind, n_per, chunks,
                                               rounds, self_msgs, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
    assert res[0] == "ok", res
    assert res[1] and res[2], res
    for p in procs:
        assert p.exitcode == 0


@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("dist_kind", ["uniform", "skewed", "equal"])
def test_shard_plan_gloo(world, dist_kind):
    _run_world(world, 6, dist_kind)


@pytest.mark.parametrize("chunks,rounds", [(1, 1), (3, 8), (8, 16)])
def test_shard_plan_gloo_chunks_rounds(chunks, rounds):
    """partition chunks (each chunk's round-0 messages posted after its
    partition) and exchange rounds: same result, stable"""
    _run_world(3, 6, "skewed", chunks=chunks, rounds=rounds)


@pytest.mark.parametrize("kind", [0, 3, 8])  # u8, i16 (narrower than 12 bits), f32
@pytest.mark.parametrize("dist_kind", ["uniform", "skewed"])
def test_shard_plan_gloo_key_kinds(kind, dist_kind):
    _run_world(2, kind, dist_kind)


@pytest.mark.parametrize("chunks,rounds", [(1, 4), (4, 4)])
def test_shard_plan_one_rank(chunks, rounds):
    """world 1: one chunk = the partitioned buffer is the receive buffer
    (alias, each group its own segment); several chunks = own-piece copies"""
    _run_world(1, 6, "uniform", chunks=chunks, rounds=rounds)


@pytest.mark.parametrize("world,chunks,rounds", [(1, 1, 4), (1, 8, 16), (3, 4, 8)])
def test_shard_plan_self_messages(world, chunks, rounds):
    """srs_shard_set_message_options(self_messages=1): own pieces travel as
    messages to the rank itself (matched in posting order, as RCCL matches
    them), never as copies; one chunk at world 1 then no longer aliases the
    partition buffer. Same result, stable."""
    _run_world(world, 6, "skewed", chunks=chunks, rounds=rounds, self_msgs=True)


# ---- the plan itself, every rank in one process ------------------------------
@pytest.mark.parametrize("self_msgs", [False, True])
@pytest.mark.parametrize("world,chunks,rounds,kind", [
    (2, 8, 8, 6), (3, 4, 16, 6), (8, 8, 8, 6), (8, 16, 64, 6), (5, 2, 3, 0), (4, 8, 8, 2),
    (1, 8, 16, 6)])
def test_shard_plan_messages_pair_up(world, chunks, rounds, kind, self_msgs):
    """For every pair of ranks the sends of one match the receives of the
    other in posting order and size; every rank's receives and own copies
    tile its receive buffer exactly once; every partitioned record is sent
    or copied exactly once; rounds are contiguous and in key order."""
    shard = _shard()
    rng = np.random.default_rng(world * 100 + chunks)
    kbits = 8 * key_size(kind)
    bits = min(12, kbits)
    nb = 1 << bits
    ns = [int(x) for x in rng.integers(0, 5000, world)]
    hs = np.zeros((world, chunks, nb), np.uint64)
    for s in range(world):
        top = np.minimum(rng.geometric(0.002, ns[s]) - 1, nb - 1)  # skewed bins
        for c in range(chunks):
            a, b = _chunk_bound(ns[s], c, chunks), _chunk_bound(ns[s], c + 1, chunks)
            hs[s, c] = np.bincount(top[a:b], minlength=nb)
    plans = [shard.debug_plan(world, r, chunks, rounds, kbits, hs, ns[r], self_messages=self_msgs)
             for r in range(world)]
    assert all(p["group_of_bin"] == plans[0]["group_of_bin"] for p in plans)
    assert all(p["rank_of_group"] == plans[0]["rank_of_group"] for p in plans)
    assert sum(p["total"] for p in plans) == sum(ns)
    rog = plans[0]["rank_of_group"]
    assert rog == sorted(rog)
    nposts = len(plans[0]["posts"])
    assert all(len(p["posts"]) == nposts for p in plans)
    for i in range(nposts):
        for s in range(world):
            for d in range(world):
                if s == d and not self_msgs:
                    assert not [m for m in plans[s]["posts"][i]["msgs"] if m[1] == s and m[0] < 2]
                    continue
                sends = [m[4] for m in plans[s]["posts"][i]["msgs"] if m[0] == 0 and m[1] == d]
                recvs = [m[4] for m in plans[d]["posts"][i]["msgs"] if m[0] == 1 and m[1] == s]
                assert sends == recvs, (i, s, d)
    for r, p in enumerate(plans):
        cover = np.zeros(p["total"], np.int64)
        used = np.zeros(ns[r], np.int64)
        for post in p["posts"]:
            for op, peer, src, dst, cnt in post["msgs"]:
                if op in (1, 2):
                    cover[dst:dst + cnt] += 1
                if op in (0, 2):
                    used[src:src + cnt] += 1
        if not p["alias"]:
            assert (cover == 1).all() and (used == 1).all(), r
        if self_msgs:
            assert not p["alias"]
            assert not [m for post in p["posts"] for m in post["msgs"] if m[0] == 2]
        rd = p["rounds"]
        assert [x["start"] for x in rd[1:]] == [x["end"] for x in rd[:-1]]
        for x in rd:
            assert x["bounds"][0] == 0 and x["bounds"][-1] == x["end"] - x["start"] or \
                x["end"] == x["start"]
            assert 0 <= x["known_bits"] < kbits


def test_shard_plan_small_first_chunk_and_last_round():
    """The head and tail of the exchange: with uniform keys the
    first partition chunk and the last round are the short ones (weight 1
    against 4)."""
    shard = _shard()
    world, chunks, rounds, n = 8, 8, 16, 1 << 20
    rng = np.random.default_rng(3)
    keys = rng.integers(0, 2**63, n, dtype=np.uint64) << np.uint64(1)
    hs = np.stack([_chunk_hists(6, keys, chunks, 12)] * world)
    p = shard.debug_plan(world, 0, chunks, rounds, 64, hs, n)
    cb = p["chunk_bounds"]
    sizes = [b - a for a, b in zip(cb[:-1], cb[1:])]
    assert sizes[0] * 3 < min(sizes[1:]), sizes
    rs = [x["end"] - x["start"] for x in p["rounds"]]
    assert rs[-1] < 0.6 * min(rs[:-1]), rs  # (whole groups: 2 of rank 0's 64 against 4-5)
