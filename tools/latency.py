"""Per-call latency of the device sort at small and medium n (u64 keys +
u64 payload, uniform): host wall time per call (call + synchronize) and the
HIP-event time around the call, as tools/perf_dat.py measures it.
usage: python tools/latency.py [n ...]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "simd-radix-sort_amd", "python"))
import srs_amd  # noqa: E402


def main():
    sizes = [int(float(x)) for x in sys.argv[1:]] or [
        16, 1024, 4096, 8192, 16384, 32768, 65536, 262144, 524288, 1 << 20, 1 << 21, 1 << 22]
    dev = torch.device("cuda:0")
    for n in sizes:
        keys = torch.empty(n, dtype=torch.int64, device=dev)
        pays = torch.empty(n, dtype=torch.int64, device=dev)
        srs_amd.fill_synthetic_device(keys, pays, key_kind=srs_amd.KEY_U64)
        k0, p0 = keys.clone(), pays.clone()
        reps = max(5, min(200, (1 << 22) // max(n, 1)))
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        wall, ev = [], []
        for r in range(3 + reps):
            keys.copy_(k0)
            pays.copy_(p0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            a.record()
            srs_amd.sort_device(keys, pays, key_kind=srs_amd.KEY_U64)
            b.record()
            b.synchronize()
            t1 = time.perf_counter()
            if r >= 3:
                wall.append((t1 - t0) * 1e6)
                ev.append(a.elapsed_time(b) * 1e3)
        wall.sort()
        ev.sort()
        kh = keys.cpu().numpy().view(np.uint64)
        ok = bool((kh[1:] >= kh[:-1]).all())
        print(f"n={n:>9} wall_us median={wall[len(wall) // 2]:9.1f} min={wall[0]:9.1f} "
              f"event_us median={ev[len(ev) // 2]:9.1f}  sorted={ok}", flush=True)


if __name__ == "__main__":
    main()
