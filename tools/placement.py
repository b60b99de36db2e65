"""Placement probe: does the C1 sort's speed depend on where its buffers sit?

One process, one resident C1 input (1e9 u64 + u64, the bench generator).
The same sort runs against several output buffers (torch allocations,
hipMalloc, a physically contiguous allocation, a VMM mapping at 1 GiB
alignment) and several workspace placements (SRS_WS_ALLOC), and every run
reports its per-level kernel times (HIP events) and the buffer addresses.
Also times a streaming fill (pure writes) into each output buffer.
Prints one JSON object per measurement. Diagnostic.
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "simd-radix-sort_amd", "python"))

import torch  # noqa: E402

import srs_amd  # noqa: E402

NAMES = ("count.L1", "count.L2", "scatter.L1", "scatter.L2", "local", "scan", "plan", "copy")


def sort_ptrs(L, n, kin, pin, kout, pout, stream):
    vp = ctypes.c_void_p
    pays = (vp * 1)(pin)
    sizes = (ctypes.c_uint32 * 1)(8)
    pouts = (vp * 1)(pout)
    rc = L.srs_sort_soa_device_leaf(n, srs_amd.KEY_U64, 1, 16, 0, kin, 1, pays, sizes, kout,
                                    pouts, stream)
    if rc:
        raise RuntimeError(L.srs_last_error().decode())


def fill_ptrs(L, n, k, p, stream):
    vp = ctypes.c_void_p
    pays = (vp * 1)(p)
    sizes = (ctypes.c_uint32 * 1)(8)
    rc = L.srs_fill_synthetic_device(n, srs_amd.KEY_U64, 7 << 32, 0, k, 1, pays, sizes, stream)
    if rc:
        raise RuntimeError(L.srs_last_error().decode())


def measure(L, n, kin, pin, kout, pout, steps, stream):
    sort_ptrs(L, n, kin, pin, kout, pout, stream)
    torch.cuda.synchronize()
    srs_amd.reset_kernel_stats()
    srs_amd.set_kernel_timing(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        sort_ptrs(L, n, kin, pin, kout, pout, stream)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps * 1e3
    srs_amd.set_kernel_timing(False)
    out = {"ms_per_step": round(wall, 3)}
    for nm in NAMES:
        l, ms, _ = srs_amd.kernel_stats(nm)
        if l:
            out[nm] = round(ms / l, 4)
    # no event markers: the plain step time
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        sort_ptrs(L, n, kin, pin, kout, pout, stream)
    torch.cuda.synchronize()
    out["ms_plain"] = round((time.perf_counter() - t0) / steps * 1e3, 3)
    return out


def fill_rate(L, n, k, p, stream):
    fill_ptrs(L, n, k, p, stream)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        fill_ptrs(L, n, k, p, stream)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 3
    return round(16 * n / ms / 1e6, 1)  # GB/s written


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=1e9)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--tag", default="")
    ap.add_argument("--out-modes", default="torch,torch,0,1,2")
    ap.add_argument("--ws-modes", default="malloc,contig,vmm")
    ap.add_argument("--rot-modes", default="",
                    help="SRS_XCD_ROT values: measure every output buffer and the contiguous "
                         "workspace with each (instead of the plain output/workspace sweep)")
    args = ap.parse_args()
    n = int(args.n)
    L = srs_amd.lib()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    pays = torch.empty(n, dtype=torch.int64, device=dev)
    srs_amd.fill_synthetic_device(keys, pays, seed=42 << 32, key_kind=srs_amd.KEY_U64)
    torch.cuda.synchronize()
    base = {"tag": args.tag, "pid": os.getpid(), "keys": hex(keys.data_ptr()),
            "pays": hex(pays.data_ptr())}
    print(json.dumps(dict(base, what="start", version=srs_amd.version())), flush=True)

    # output candidates
    outs, hold = [], []
    for i, m in enumerate(args.out_modes.split(",")):
        if m == "torch":
            ko = torch.empty_like(keys)
            po = torch.empty_like(pays)
            hold += [ko, po]
            outs.append((f"torch{i}", ko.data_ptr(), po.data_ptr(), None))
        else:
            ko = srs_amd.debug_alloc(8 * n, int(m))
            po = srs_amd.debug_alloc(8 * n, int(m))
            outs.append((f"alloc{m}_{i}", ko, po, (ko, po)))
    if args.rot_modes:
        for wm in ("malloc", "contig"):
            srs_amd.release_workspace()
            os.environ["SRS_WS_ALLOC"] = wm
            for name, ko, po, _ in outs:
                for rm in args.rot_modes.split(","):
                    os.environ["SRS_XCD_ROT"] = rm
                    r = measure(L, n, keys.data_ptr(), pays.data_ptr(), ko, po, args.steps, stream)
                    print(json.dumps(dict(base, what="rot", rot=int(rm), ws=wm, out=name,
                                          tmp=hex(srs_amd.debug_workspace()[0]), **r)), flush=True)
        os.environ["SRS_XCD_ROT"] = "0"
        srs_amd.release_workspace()
        for _, _, _, raw in outs:
            if raw:
                for p in raw:
                    srs_amd.debug_free(p)
        return
    os.environ["SRS_WS_ALLOC"] = "malloc"
    for name, ko, po, _ in outs:
        r = measure(L, n, keys.data_ptr(), pays.data_ptr(), ko, po, args.steps, stream)
        tmp = srs_amd.debug_workspace()
        print(json.dumps(dict(base, what="out", out=name, kout=hex(ko), pout=hex(po),
                              tmp=hex(tmp[0]), fill_gbs=fill_rate(L, n, ko, po, stream),
                              probe_k=srs_amd.debug_probe_write(ko, 8 * n),
                              probe_p=srs_amd.debug_probe_write(po, 8 * n), **r)),
              flush=True)
    # workspace placements, with the first output fixed
    name, ko, po, _ = outs[0]
    for wm in args.ws_modes.split(","):
        srs_amd.release_workspace()
        os.environ["SRS_WS_ALLOC"] = wm
        r = measure(L, n, keys.data_ptr(), pays.data_ptr(), ko, po, args.steps, stream)
        tmp = srs_amd.debug_workspace()
        print(json.dumps(dict(base, what="ws", ws=wm, out=name, tmp=hex(tmp[0]),
                              probe_t0=srs_amd.debug_probe_write(tmp[0], 8 * n),
                              probe_t1=srs_amd.debug_probe_write(tmp[0] + 8 * n, 8 * n), **r)),
              flush=True)
    # the first configuration again (drift check)
    srs_amd.release_workspace()
    os.environ["SRS_WS_ALLOC"] = "malloc"
    r = measure(L, n, keys.data_ptr(), pays.data_ptr(), ko, po, args.steps, stream)
    print(json.dumps(dict(base, what="again", out=name, tmp=hex(srs_amd.debug_workspace()[0]),
                          **r)), flush=True)
    srs_amd.release_workspace()
    for _, _, _, raw in outs:
        if raw:
            for p in raw:
                srs_amd.debug_free(p)


if __name__ == "__main__":
    main()
