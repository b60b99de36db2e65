"""The multi-GPU shard protocol with the REAL HIP kernels and several ranks:
world 2-4 gloo processes share the one GPU of the test box (RCCL cannot put
two ranks on one device), so ShardSorter runs with stage_host=True (its
peer-to-peer messages travel through host memory). Everything else is the
product path: srs_key_histogram_device, the 512-group LUT partition,
srs_sort_segments_device with known prefix bits on a side stream, the
exchange rounds. The union sorted across ranks must equal a stable sort of
the inputs in (rank, index) order, keys and payloads bit for bit."""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, dist_kind, kind, q, n_base=200_000):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        sys.path.insert(0, os.path.join(REPO, "simd-radix-sort_amd", "python"))
        import torch
        import torch.distributed as dist
        import srs_amd
        from srs_amd.dist import HipShardOps, ShardSorter
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
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
        else:  # floats
            keys = torch.randn(n, device="cuda", generator=g)
        sorter = ShardSorter(HipShardOps(kind), n, [torch.int64], keys.dtype, "cuda",
                             chunk_bytes=64 << 10, stage_host=True)
        for _ in range(2):  # twice: buffers are reused
            rk, (rp,) = sorter.sort(keys, [pay])
        torch.cuda.synchronize()
        outs = [None] * world
        dist.all_gather_object(outs, (rk.cpu().numpy(), rp.cpu().numpy()))
        ins = [None] * world
        dist.all_gather_object(ins, (keys.cpu().numpy(), pay.cpu().numpy()))
        if rank == 0:
            q.put(("ok", outs, ins))
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        q.put(("error", repr(e)))
        raise


def _transformed(k, kind):
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from srs_testlib import transformed_keys
    return transformed_keys(kind, True, k)


@pytest.mark.parametrize("world,dist_kind,kind,n_base", [
    (2, "uniform", 7, 200_000), (3, "skewed", 7, 200_000), (4, "uniform", 7, 200_000),
    (3, "equal", 7, 200_000), (2, "float", 8, 200_000),
    # C4's shape (u64 key + f(key) payload from global indices) at 8 ranks
    (8, "c4", 6, 1_000_000)])
def test_shard_sorter_multi_rank_on_gpu(world, dist_kind, kind, n_base):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, dist_kind, kind, q, n_base))
             for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
    assert res[0] == "ok", res
    _, outs, ins = res
    for p in procs:
        assert p.exitcode == 0
    ink = np.concatenate([i[0] for i in ins])
    inp = np.concatenate([i[1] for i in ins])
    order = np.argsort(_transformed(ink, kind), kind="stable")
    outk = np.concatenate([o[0] for o in outs])
    outp = np.concatenate([o[1] for o in outs])
    assert np.array_equal(outk.view(np.uint8), ink[order].view(np.uint8))
    assert np.array_equal(outp, inp[order])
