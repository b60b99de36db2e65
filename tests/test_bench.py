"""bench.py's launcher contract (CPU): `--gpus N` starts N ranks through
torch.distributed.run before anything touches the GPU, and a WORLD_SIZE that
disagrees with --gpus is an error. The GPU case (--gpus 2 on a 1-GPU box
fails with a message) is a -m gpu test."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(kw)
    return env


def test_launcher_argv_and_env():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--steps", "7", "--warmup", "2",
                        "--dry-run-launch"], capture_output=True, text=True, env=_env(),
                       timeout=60)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    argv = d["argv"]
    assert argv[0] == sys.executable and argv[1:3] == ["-m", "torch.distributed.run"]
    assert "--nnodes=1" in argv and "--nproc-per-node=4" in argv
    assert "--master-addr=127.0.0.1" in argv
    assert any(a.startswith("--master-port=") and int(a.split("=")[1]) > 0 for a in argv)
    i = argv.index(os.path.abspath(BENCH))
    assert argv[i + 1:] == ["--", "--gpus", "4", "--steps", "7", "--warmup", "2"]
    assert d["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert d["env"]["MASTER_ADDR"] == "127.0.0.1"


def test_launcher_parent_never_imports_torch():
    """The parent must not initialise the GPU: it may not even import torch
    (a process that touched the GPU must never exec another)."""
    code = ("import sys, runpy\n"
            f"sys.argv = [{BENCH!r}, '--gpus', '2', '--dry-run-launch']\n"
            "try:\n"
            f"    runpy.run_path({BENCH!r}, run_name='__main__')\n"
            "except SystemExit as e:\n"
            "    assert e.code in (0, None), e.code\n"
            "assert 'torch' not in sys.modules, 'parent imported torch'\n"
            "print('ok')\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=_env(),
                       timeout=60)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


def test_launched_ranks_parse_every_bench_option():
    """The ranks get bench's own options intact (torchrun would reject --n as
    an abbreviation of its own options without the separator); on a host
    without GPUs every rank then stops at the device check."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--n", "1e6", "--cpu-sample", "0", "--config", "c2"],
                       capture_output=True, text=True, env=_env(CUDA_VISIBLE_DEVICES="",
                                                                HIP_VISIBLE_DEVICES=""),
                       timeout=300)
    assert r.returncode != 0
    assert "--gpus 2 needs 2 GPUs on this node, 0 visible" in r.stderr, r.stderr[-3000:]


def test_world_size_must_match_gpus():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--steps", "1"],
                       capture_output=True, text=True,
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), timeout=60)
    assert r.returncode != 0
    assert "WORLD_SIZE=2 but --gpus 4" in r.stderr


@pytest.mark.gpu
def test_more_gpus_than_visible_fails_loudly():
    import torch
    ndev = torch.cuda.device_count()
    n = ndev + 1
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--steps", "1", "--warmup", "0",
                        "--n", "1e6", "--cpu-sample", "0"], capture_output=True, text=True,
                       env=_env(), timeout=300)
    assert r.returncode != 0
    assert f"--gpus {n} needs {n} GPUs on this node, {ndev} visible" in r.stderr
    assert '"metric"' not in r.stdout


def _verify_worker(rank, world, port, q):
    import os as _os
    import sys as _sys
    import torch
    import torch.distributed as dist
    _sys.path.insert(0, REPO)
    _os.environ["MASTER_ADDR"] = "127.0.0.1"
    _os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        g = torch.Generator()
        g.manual_seed(5)
        n = 40_000
        allk = torch.randint(-2**63, 2**63 - 1, (world * n,), dtype=torch.int64, generator=g)
        allp = bench._splitmix64(bench._u64_bits(allk, torch), torch)  # payload = f(key)
        mine = slice(rank * n, (rank + 1) * n)
        ink, inp = allk[mine].clone(), allp[mine].clone()
        # the shard contract: rank r holds the r-th key range, sorted (u64 order)
        order = torch.argsort(allk ^ torch.iinfo(torch.int64).min, stable=True)
        sk, sp = allk[order], allp[order]
        cut = [0, world * n // 3, world * n]  # ragged output ranks
        outk, outp = sk[cut[rank]:cut[rank + 1]], sp[cut[rank]:cut[rank + 1]]
        good = bench.verify_shards(ink, [inp], (outk, [outp]), "u64", [8], torch, dist, "cpu")
        # a broken output: rank 1 drops its last record and repeats its first
        if rank == 1:
            outk = torch.cat([outk[:1], outk[:-1]])
            outp = torch.cat([outp[:1], outp[:-1]])
        bad = bench.verify_shards(ink, [inp], (outk, [outp]), "u64", [8], torch, dist, "cpu")
        if rank == 0:
            q.put(("ok", good, bad))
    except Exception as e:  # report instead of hanging the parent
        q.put(("error", repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


def test_verify_shards_over_gloo():
    """The N > 1 bench line's full-size check (bench.verify_shards: every rank
    sorted with payload = f(key), rank boundaries ordered, the multiset hash
    and count over all ranks unchanged) on two gloo ranks: a correct shard
    output passes every check, a rank that lost a record fails the hash."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_verify_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = q.get(timeout=180)
    for p in ps:
        p.join(timeout=60)
    assert res[0] == "ok", res
    good, bad = res[1], res[2]
    assert all(good.values()), good
    assert not bad["multiset_hash_equal"], bad
