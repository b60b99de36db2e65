"""Reproducer: does a single large RCCL message come back intact?

DESIGN.md §7 caps every shard message at 256 MB because one 8 GB
all_to_all_single (world 1, 1e9 int64 keys) came back corrupted. This runs
world-1 collectives (RCCL over the one local GPU) with messages straddling
2^31 and 2^32 bytes, in the three forms the shard protocol could use, and
checks every element against a known pattern:
  all_to_all_single (one peer: the whole buffer is one message),
  batch_isend_irecv to self (the p2p form dist.py uses),
  broadcast (a plain collective of the same size).
usage: python tools/rccl_msg_size.py [sizes in MiB, comma separated]
Prints one line per (form, size): OK, or the first bad index and count."""
import os
import sys
import time

import torch
import torch.distributed as dist


def pattern(n, dev):
    # element i = i * 0x9E3779B97F4A7C15 + 7 (wrapping): no two equal, no zero runs
    i = torch.arange(n, dtype=torch.int64, device=dev)
    return i * (0x9E3779B97F4A7C15 - (1 << 64)) + 7


def check(name, mib, out, ref):
    bad = (out != ref)
    nbad = int(bad.sum().item())
    if nbad == 0:
        print(f"{name:22s} {mib:7d} MiB ({mib * 2**20:>11d} B): OK", flush=True)
        return True
    first = int(torch.nonzero(bad)[0].item())
    print(f"{name:22s} {mib:7d} MiB ({mib * 2**20:>11d} B): {nbad} bad int64, first at element "
          f"{first} (byte {first * 8}, {first * 8 / 2**31:.4f} x 2^31)", flush=True)
    return False


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    sizes = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else \
        [256, 2047, 2048, 2049, 4095, 4096, 4097, 8192]
    ok = True
    for mib in sizes:
        n = mib * 2**20 // 8
        src = pattern(n, dev)
        out = torch.zeros_like(src)
        t0 = time.perf_counter()
        dist.all_to_all_single(out, src)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ok &= check("all_to_all_single", mib, out, src)
        out.zero_()
        reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, src, 0), dist.P2POp(dist.irecv, out, 0)])
        for r in reqs:
            r.wait()
        torch.cuda.synchronize()
        ok &= check("batch_isend_irecv self", mib, out, src)
        b = src.clone()
        dist.broadcast(b, 0)
        torch.cuda.synchronize()
        ok &= check("broadcast", mib, b, src)
        print(f"   (all_to_all_single took {dt * 1e3:.1f} ms)", flush=True)
        del src, out, b
        torch.cuda.empty_cache()
    dist.destroy_process_group()
    print("ALL OK" if ok else "SOME MESSAGES CORRUPTED", flush=True)


if __name__ == "__main__":
    main()
