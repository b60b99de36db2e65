"""In-process A/B of output buffers (placement): one resident C1
input, several output sets — placed (srs_alloc_device, probed) and plain
(torch.empty, i.e. hipMalloc) — sorted into in turn, arms alternated step by
step, so that only the written buffers differ. Per arm: the median step time
(HIP-event markers around every launch), the median second-level scatter and
local times (the kernels that write the outputs), and the placement probe's
ms per GB of each output column (srs_debug_probe_write), to see whether the
probe ranks the buffers the way the sort does.

"inplace" arms sort a torch array in place (restored from the input before
each step, untimed): the reference's in-place contract.

usage: python tools/ab_outputs.py [--sets placed,plain,inplace,placed] [--rounds 7]
"""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "simd-radix-sort_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", default="placed,plain,placed,plain")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--n", type=float, default=1e9)
    a = ap.parse_args()
    import torch

    import srs_amd
    n = int(a.n)
    dev = torch.device("cuda", 0)
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    pays = torch.empty(n, dtype=torch.int64, device=dev)
    srs_amd.fill_synthetic_device(keys, pays, seed=42 << 32, key_kind=srs_amd.KEY_U64)
    torch.cuda.synchronize()
    arms = []
    for i, kind in enumerate(a.sets.split(",")):
        if kind == "placed":
            outs = [srs_amd.empty_device(n, torch.int64, dev) for _ in range(2)]
        elif kind == "inplace":  # (the caller's own arrays, restored before each step)
            outs = [torch.empty(n, dtype=torch.int64, device=dev) for _ in range(2)]
        else:
            outs = [torch.empty(n, dtype=torch.int64, device=dev) for _ in range(2)]
        torch.cuda.synchronize()
        probe = [round(srs_amd.debug_probe_write(o.data_ptr(), o.numel() * 8) / (o.numel() * 8 / 1e9), 4)
                 for o in outs]
        arms.append({"name": f"{i}:{kind}", "outs": outs, "probe_ms_per_gb": probe,
                     "inplace": kind == "inplace", "step_ms": [], "scatter.L2": [], "local": [],
                     "scatter.L1": [], "count": [], "scan": []})
    def run(arm):
        if arm["inplace"]:
            srs_amd.sort_device(*arm["outs"], key_kind=srs_amd.KEY_U64)
        else:
            srs_amd.sort_device(keys, pays, key_kind=srs_amd.KEY_U64, out=tuple(arm["outs"]))

    def restore(arm):
        if arm["inplace"]:
            arm["outs"][0].copy_(keys)
            arm["outs"][1].copy_(pays)

    for arm in arms:  # warmup
        restore(arm)
        run(arm)
    torch.cuda.synchronize()
    srs_amd.set_kernel_timing(True)
    for _ in range(a.rounds):
        for arm in arms:
            restore(arm)
            srs_amd.reset_kernel_stats()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(arm)
            torch.cuda.synchronize()
            arm["step_ms"].append((time.perf_counter() - t0) * 1e3)
            for k in ("scatter.L1", "scatter.L2", "local", "count", "scan"):
                l, ms, _ = srs_amd.kernel_stats(k)
                if l:
                    arm[k].append(ms / l)
    srs_amd.set_kernel_timing(False)
    print(json.dumps({"n": n, "rounds": a.rounds, "arms": [
        {"arm": arm["name"], "probe_ms_per_gb": arm["probe_ms_per_gb"],
         **{k: round(statistics.median(arm[k]), 4) for k in ("step_ms", "scatter.L1", "scatter.L2",
                                                              "local", "count", "scan") if arm[k]}}
        for arm in arms]}))


if __name__ == "__main__":
    main()
