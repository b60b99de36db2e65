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
