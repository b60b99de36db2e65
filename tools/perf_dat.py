"""Benchmark harness in the reference's own .dat formats (src/perf.hpp), so
that GPU numbers sit beside the thesis curves (bachelors-thesis/data/):

  tpe-<K>[-<P>]-<Dist>.dat       "number_of_elements <method>..." rows for
                                 n = 1, 2, 4, ... (perf.hpp:366-410)
  <K>[-<P>]-<Dist>-262144.dat    "sort_method nanoseconds_per_element"
                                 (perf.hpp:412-447)
  cmpThresh-<K>[-<P>]-<Method>-<Dist>.dat  (--thresh) "cmpThresh 262144"
                                 then "threshold ns_per_element" rows,
                                 thresholds 2..512 for the insertion-sort
                                 leaf and 1..262144 for the leaves left
                                 unsorted (perf.hpp:159-212)

Methods (columns):
  RadixSIMD    the reference itself (oracle/_ref/libsrs_ref.so, AVX-512,
               one core, CPU time around the sort call: perf.hpp:33-46)
  GPURadix     this library, device-resident arrays (HIP events around
               srs_sort_soa_device; the input is restored between runs)
  GPURadixHost this library through the host-pointer drop-in (srs_sort_soa:
               PCIe both ways included; wall clock)
  In cmpThresh files the reference's SortMethodRadixSort names
  (sort_methods.hpp:26-52) are used: RadixSIMD / RadixSIMDNoCmp (the
  reference with CmpSorterInsertionSort / CmpSorterNoSort) and GPURadix /
  GPURadixNoCmp (this library, SRS_LEAF_SORTED / SRS_LEAF_UNSORTED).

Repetitions follow perf.hpp:68-69 (max(1, 2^22/n) timed runs after
max(1, 2^18/n) warm-ups, each on a fresh copy), capped at --max-reps per
point so that small n stay affordable on the GPU (a launch costs ~10 us).
Input distributions restate src/data.hpp's generators in numpy (seeded).

usage (GPU box): python tools/perf_dat.py --out gpurun_out/perf_dat
       [--types int64,double] [--payload int64] [--dists Uniform,Zero]
       [--max-log2 22]
"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simd-radix-sort_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

TYPES = {  # perf.hpp type_name -> (numpy dtype, srs key kind)
    "int8": (np.int8, 1), "int16": (np.int16, 3), "int32": (np.int32, 5),
    "int64": (np.int64, 7), "uint8": (np.uint8, 0), "uint16": (np.uint16, 2),
    "uint32": (np.uint32, 4), "uint64": (np.uint64, 6), "float": (np.float32, 8),
    "double": (np.float64, 9),
}
DISTS = ["Uniform", "Gaussian", "Zero", "ZeroOne", "Sorted", "ReverseSorted", "AlmostSorted",
         "AlmostReverseSorted"]


def make(dtype, dist, n, rng):
    """src/data.hpp:105-170 in numpy: uniform over the type's range (floats
    in [-1, 1)), gaussian, constant, {0, 1}, sorted / reverse sorted, and
    almost sorted (sqrt(n) random swaps)."""
    dt = np.dtype(dtype)
    if dist in ("Uniform", "Sorted", "ReverseSorted", "AlmostSorted", "AlmostReverseSorted"):
        if dt.kind == "f":
            a = rng.uniform(-1, 1, n).astype(dt)
        else:
            info = np.iinfo(dt)
            a = rng.integers(info.min, info.max, n, dtype=dt, endpoint=True)
        if dist != "Uniform":
            a = np.sort(a)
            if "Reverse" in dist:
                a = a[::-1].copy()
            if dist.startswith("Almost") and n > 1:
                k = max(1, int(np.sqrt(n)))
                i, j = rng.integers(0, n, k), rng.integers(0, n, k)
                a[i], a[j] = a[j], a[i].copy()
        return a
    if dist == "Gaussian":
        v = rng.normal(0, 1, n) if dt.kind == "f" else rng.normal(0, 100, n).round()
        if dt.kind != "f":
            info = np.iinfo(dt)
            v = np.clip(v, info.min, info.max)
        return v.astype(dt)
    if dist == "Zero":
        return np.zeros(n, dt)
    if dist == "ZeroOne":
        return rng.integers(0, 2, n).astype(dt)
    raise ValueError(dist)


def reps(n, cap):
    return min(cap, max(1, (1 << 22) // n)), min(cap, max(1, (1 << 18) // n))


class Methods:
    def __init__(self, kind, pdtype, max_reps, with_host):
        import torch
        import srs_amd
        from srs_testlib import ref_lib
        self.torch, self.srs, self.kind = torch, srs_amd, kind
        self.ref = ref_lib()
        self.ref.srs_ref_sort_soa_timed.argtypes = [
            ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p,
            ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
        self.pdtype = pdtype
        self.max_reps = max_reps
        self.names = ["RadixSIMD", "GPURadix"] + (["GPURadixHost"] if with_host else [])

        self.ref.srs_ref_sort_soa_leaf_timed.argtypes = [
            ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int,
            ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.POINTER(ctypes.c_double)]

    def _ref_once(self, k, p, thresh=16, leaf=0):
        k = k.copy()
        pays = [] if p is None else [p.copy()]
        arr = (ctypes.c_void_p * 1)(*(x.ctypes.data for x in pays)) if pays else None
        sz = (ctypes.c_uint32 * 1)(*(x.itemsize for x in pays)) if pays else None
        ns = ctypes.c_double()
        rc = self.ref.srs_ref_sort_soa_leaf_timed(len(k), self.kind, 1, int(thresh), int(leaf),
                                                  k.ctypes.data, len(pays), arr, sz,
                                                  ctypes.byref(ns))
        if rc != 0:
            raise RuntimeError(f"reference sort failed ({rc})")
        if leaf == 0 and np.any(k[1:] < k[:-1]):  # perf.hpp:118-126 checks the same
            raise RuntimeError("reference output not sorted")
        return ns.value

    def measure(self, name, k, p, thresh=16):
        """ns per element, averaged like measureTimePerElementWithRepsAndWarmup
        (and measureTimePerElementThreshWithRepsAndWarmup, perf.hpp:131-157)."""
        n = len(k)
        timed, warm = reps(n, self.max_reps)
        torch = self.torch
        if name in ("RadixSIMD", "RadixSIMDNoCmp"):
            leaf = 1 if name.endswith("NoCmp") else 0
            for _ in range(warm):
                self._ref_once(k, p, thresh, leaf)
            return sum(self._ref_once(k, p, thresh, leaf) for _ in range(timed)) / timed / n
        if name == "GPURadixHost":
            def once():
                kk = k.copy()
                pp = [] if p is None else [p.copy()]
                t0 = time.perf_counter()
                self.srs.sort(kk, *pp)
                return (time.perf_counter() - t0) * 1e9
            for _ in range(warm):
                once()
            return sum(once() for _ in range(timed)) / timed / n
        # device-resident: input restored from a pristine copy between runs
        self.last_gpu = []  # (per-call event times in us, for the progress line)
        src = torch.from_numpy(k.view(np.uint8)).cuda()
        dk = torch.empty_like(src)
        psrc = None if p is None else torch.from_numpy(p.view(np.uint8)).cuda()
        dp = None if p is None else torch.empty_like(psrc)
        ks, ps = k.itemsize, (None if p is None else p.itemsize)
        kt = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        tot = 0.0
        for r in range(warm + timed):
            dk.copy_(src)
            if dp is not None:
                dp.copy_(psrc)
            keys = dk.view(kt[ks])
            pays = [] if dp is None else [dp.view(kt[ps])]
            a.record()
            self.srs.sort_device(keys, *pays, key_kind=self.kind, cmp_sort_threshold=thresh,
                                 cmp_sorter="nosort" if name.endswith("NoCmp") else "insertion")
            b.record()
            b.synchronize()
            if r >= warm:
                tot += a.elapsed_time(b) * 1e6
                self.last_gpu.append(a.elapsed_time(b) * 1e3)
        if not name.endswith("NoCmp"):
            out = dk.view(kt[ks]).cpu().numpy().view(k.dtype)
            if np.any(out[1:] < out[:-1]):
                raise RuntimeError(f"{name}: output not sorted")
        return tot / timed / n


def thresh_files(m, tname, args, pdt, rng):
    """perfTestThresh (perf.hpp:159-212): n = 2^18, thresholds doubling from
    2 to 512 (insertion-sort leaf) or from 1 to n (leaves unsorted), one file
    per sort method and distribution."""
    n = 1 << 18
    dtype = TYPES[tname][0]
    for dist in args.dists.split(","):
        k = make(dtype, dist, n, rng)
        p = None if pdt is None else make(pdt, "Uniform", n, rng)
        for name in ("RadixSIMD", "RadixSIMDNoCmp", "GPURadix", "GPURadixNoCmp"):
            lo, hi = (1, n) if name.endswith("NoCmp") else (2, 512)
            desc = (f"cmpThresh-{tname}" + (f"-{args.payload}" if args.payload else "")
                    + f"-{name}-{dist}")
            rows, t = [], lo
            while t <= hi:
                rows.append((t, m.measure(name, k, p, thresh=t)))
                print(desc, t, f"{rows[-1][1]:.3f}", flush=True)
                t *= 2
            with open(os.path.join(args.out, desc + ".dat"), "w") as f:
                f.write(f"cmpThresh {n}\n")
                for t, v in rows:
                    f.write(f"{t} {v:.6f}\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "perf_dat"))
    ap.add_argument("--types", default="int64,double")
    ap.add_argument("--payload", default="", help="payload type name (one column) or empty")
    ap.add_argument("--dists", default="Uniform")
    ap.add_argument("--max-log2", type=int, default=22)
    ap.add_argument("--max-reps", type=int, default=64)
    ap.add_argument("--no-host", action="store_true")
    ap.add_argument("--thresh", action="store_true",
                    help="write the cmpThresh-* files (perf.hpp:159-212) instead")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    rng = np.random.default_rng(42)
    pdt = TYPES[args.payload][0] if args.payload else None
    for tname in args.types.split(","):
        dtype, kind = TYPES[tname]
        m = Methods(kind, pdt, args.max_reps, not args.no_host)
        if args.thresh:
            thresh_files(m, tname, args, pdt, rng)
            continue
        for dist in args.dists.split(","):
            desc = tname + (f"-{args.payload}" if args.payload else "") + f"-{dist}"
            # one pass over the sizes per method (the same inputs in every
            # pass): with the host-array calls interleaved between sizes, the
            # device calls of 16K-128K keys measured ~45 us slower per call
            # (kernels unchanged), which no isolated sequence
            # reproduced
            inputs = []
            for lg in range(0, args.max_log2 + 1):
                n = 1 << lg
                k = make(dtype, dist, n, rng)
                p = None if pdt is None else make(pdt, "Uniform", n, rng)
                inputs.append((n, k, p))
            cols = {}
            for name in m.names:
                cols[name] = []
                for n, k, p in inputs:
                    cols[name].append(m.measure(name, k, p))
                    extra = ""
                    if name.startswith("GPURadix") and name != "GPURadixHost":
                        g = sorted(getattr(m, "last_gpu", []) or [0.0])
                        extra = f" (device calls: median {g[len(g) // 2]:.1f} us, max {g[-1]:.1f} us)"
                    print(desc, name, n, f"{cols[name][-1]:.3f}" + extra, flush=True)
            rows = [(n, [cols[name][i] for name in m.names]) for i, (n, _, _) in enumerate(inputs)]
            with open(os.path.join(args.out, f"tpe-{desc}.dat"), "w") as f:
                f.write("number_of_elements " + " ".join(m.names) + "\n")
                for n, vals in rows:
                    f.write(f"{n} " + " ".join(f"{v:.6f}" for v in vals) + "\n")
            at = dict(rows).get(1 << 18)
            if at is not None:
                with open(os.path.join(args.out, f"{desc}-262144.dat"), "w") as f:
                    f.write("sort_method nanoseconds_per_element\n")
                    for name, v in sorted(zip(m.names, at), key=lambda x: -x[1]):
                        f.write(f"{name} {v:.6f}\n")


if __name__ == "__main__":
    main()
