"""In-process A/B of a library setting read at every sort (an environment
variable such as SRS_PAIR_TILES): one resident input, one set of placed
outputs, the arms alternated step by step, so that the buffers' placement
and the box are the same for every arm (process-to-process placement moves a
scatter by 10-15 %). Per arm: the median step time (HIP-event
markers around every launch, the same cost in every arm) and the median
per-level kernel times.

usage: python tools/ab_inproc.py --config c1 --env SRS_PAIR_TILES --values 0,1 [--rounds 7]
"""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "simd-radix-sort_amd", "python"))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c1", choices=sorted(bench.CONFIGS))
    ap.add_argument("--env", required=True)
    ap.add_argument("--values", required=True)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--n", type=float, default=1e9)
    a = ap.parse_args()
    import torch

    import srs_amd
    kname, psizes, layout, _ = bench.CONFIGS[a.config]
    kind = bench.kind_id(kname)
    n = int(a.n)
    dev = torch.device("cuda", 0)
    tdt = {8: torch.int64, 4: torch.int32}
    key_dt = {"u64": torch.int64, "f32": torch.float32, "u32": torch.int32}[kname]
    keys = torch.empty(n, dtype=key_dt, device=dev)
    pays = [torch.empty(n, dtype=tdt[s], device=dev) for s in psizes]
    srs_amd.fill_synthetic_device(keys, *pays, seed=42 << 32, key_kind=kind)
    if layout == "aos":
        rec = torch.stack([keys, pays[0]], dim=1).contiguous()
        out = srs_amd.empty_device(rec.numel(), rec.dtype, dev).view(rec.shape)
        del keys, pays

        def step():
            srs_amd.sort_combined_device(rec, kind, out=out)
    else:
        outs = [srs_amd.empty_device(t.numel(), t.dtype, dev) for t in [keys] + pays]

        def step():
            srs_amd.sort_device(keys, *pays, key_kind=kind, out=tuple(outs))
    names = ["count", "scatter", "local"] + [f"{k}.L{i}" for i in (1, 2, 3) for k in
                                             ("count", "scatter")]
    values = a.values.split(",")
    res = {v: {"step_ms": [], **{k: [] for k in names}} for v in values}
    for v in values:  # warmup of every arm
        os.environ[a.env] = v
        step()
    torch.cuda.synchronize()
    srs_amd.set_kernel_timing(True)
    for _ in range(a.rounds):
        for v in values:
            os.environ[a.env] = v
            srs_amd.reset_kernel_stats()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            step()
            torch.cuda.synchronize()
            res[v]["step_ms"].append((time.perf_counter() - t0) * 1e3)
            for k in names:
                l, ms, _ = srs_amd.kernel_stats(k)
                if l:
                    res[v][k].append(ms / l)
    srs_amd.set_kernel_timing(False)
    summary = {v: {k: round(statistics.median(x), 4) for k, x in r.items() if x}
               for v, r in res.items()}
    print(json.dumps({"config": a.config, "n": n, "env": a.env, "rounds": a.rounds,
                      "median": summary,
                      "step_ms_all": {v: [round(x, 3) for x in r["step_ms"]]
                                      for v, r in res.items()}}))


if __name__ == "__main__":
    main()
