"""Shared test helpers: golden-vector loader and ctypes bindings of the oracle.

TEST INFRASTRUCTURE. The oracle libraries (oracle/_build/libsrs_oracle.so =
C restatement, oracle/_ref/libsrs_ref.so = the reference's own radixSort.hpp
behind a C shim) are used here ONLY as checkers, never as the thing tested.
"""
from __future__ import annotations

import ctypes
import json
import os
from functools import lru_cache

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN_DIR = os.path.join(REPO, "tests", "golden")
ORACLE_SO = os.path.join(REPO, "oracle", "_build", "libsrs_oracle.so")
REF_SO = os.path.join(REPO, "oracle", "_ref", "libsrs_ref.so")

# srs_key_kind numbering (include/srs_c_api.h)
KIND_NAMES = ["u8", "i8", "u16", "i16", "u32", "i32", "u64", "i64", "f32", "f64"]
KIND_DTYPES = [np.uint8, np.int8, np.uint16, np.int16, np.uint32, np.int32,
               np.uint64, np.int64, np.float32, np.float64]
KIND_UINT = [np.uint8, np.uint8, np.uint16, np.uint16, np.uint32, np.uint32,
             np.uint64, np.uint64, np.uint32, np.uint64]
UINT_OF_SIZE = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}


def key_size(kind: int) -> int:
    return np.dtype(KIND_DTYPES[kind]).itemsize


# --------------------------------------------------------------------------
# golden vectors
# --------------------------------------------------------------------------
@lru_cache(maxsize=1)
def golden_manifest():
    with open(os.path.join(GOLDEN_DIR, "manifest.json")) as f:
        return json.load(f)


@lru_cache(maxsize=1)
def golden_blob() -> bytes:
    with open(os.path.join(GOLDEN_DIR, "golden.bin"), "rb") as f:
        return f.read()


def golden_arrays(case):
    """Returns (inputs, outputs): lists of numpy arrays (copies).

    SoA: [keys(dtype of kind), payload columns (uint of size)...]
    AoS: [elements as uint8 matrix (n, elem_size)]
    """
    blob = golden_blob()
    n = case["n"]

    def arr(off, dtype, count):
        return np.frombuffer(blob, dtype=dtype, count=count, offset=off).copy()

    def unpack(offs):
        if case["layout"] == "aos":
            es = case["elem_size"]
            return [arr(offs[0], np.uint8, n * es).reshape(n, es)]
        out = [arr(offs[0], KIND_DTYPES[case["key_kind"]], n)]
        for off, sz in zip(offs[1:], case["payload_sizes"]):
            out.append(arr(off, UINT_OF_SIZE[sz], n))
        return out

    return unpack(case["in"]), unpack(case["out"])


# --------------------------------------------------------------------------
# oracle bindings
# --------------------------------------------------------------------------
def _ptrs(arrs):
    return (ctypes.c_void_p * max(1, len(arrs)))(*[a.ctypes.data for a in arrs])


def _sizes(arrs):
    return (ctypes.c_uint32 * max(1, len(arrs)))(*[a.dtype.itemsize for a in arrs])


@lru_cache(maxsize=1)
def oracle_lib():
    lib = ctypes.CDLL(ORACLE_SO)
    lib.srs_oracle_sort_soa.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    lib.srs_oracle_sort_aos.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int64, ctypes.c_void_p, ctypes.c_uint32,
                                        ctypes.c_int]
    return lib


def oracle_sort_soa(kind, up, keys, payloads=(), thresh=16, bit_sorter=0):
    """In-place CPU restatement of radix_sort::sort on numpy arrays."""
    assert keys.flags.c_contiguous and all(p.flags.c_contiguous for p in payloads)
    rc = oracle_lib().srs_oracle_sort_soa(len(keys), kind, int(up), thresh,
                                          keys.ctypes.data, len(payloads),
                                          _ptrs(payloads), _sizes(payloads), bit_sorter)
    assert rc == 0, rc


def oracle_sort_aos(kind, up, elems, thresh=16, bit_sorter=0):
    assert elems.flags.c_contiguous and elems.ndim == 2
    rc = oracle_lib().srs_oracle_sort_aos(elems.shape[0], kind, int(up), thresh,
                                          elems.ctypes.data, elems.shape[1], bit_sorter)
    assert rc == 0, rc


def host_has_avx512_vbmi2() -> bool:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("flags"):
                    fl = set(line.split(":", 1)[1].split())
                    need = {"avx512f", "avx512bw", "avx512dq", "avx512vl",
                            "avx512vbmi", "avx512_vbmi2"}
                    return need <= fl
    except OSError:
        pass
    return False


@lru_cache(maxsize=1)
def ref_lib():
    """The reference's own sort (oracle/_ref), or None if unavailable/unsafe."""
    if not os.path.exists(REF_SO) or not host_has_avx512_vbmi2():
        return None
    lib = ctypes.CDLL(REF_SO)
    lib.srs_ref_sort_soa.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32,
                                     ctypes.c_void_p, ctypes.c_void_p]
    lib.srs_ref_sort_aos.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int64, ctypes.c_void_p, ctypes.c_uint32]
    lib.srs_ref_sort_soa_timed.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32,
                                           ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.POINTER(ctypes.c_double)]
    lib.srs_ref_sort_soa_leaf_timed.argtypes = [
        ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int,
        ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.POINTER(ctypes.c_double)]
    return lib


def ref_sort_soa(kind, up, keys, payloads=(), thresh=16):
    rc = ref_lib().srs_ref_sort_soa(len(keys), kind, int(up), thresh, keys.ctypes.data,
                                    len(payloads), _ptrs(payloads), _sizes(payloads))
    assert rc == 0, rc


def ref_sort_soa_timed(kind, up, keys, payloads=(), thresh=16):
    """ref_sort_soa timed inside the library with CLOCK_PROCESS_CPUTIME_ID
    around the sort call only (the reference's src/perf.hpp:33-46); returns
    the CPU nanoseconds."""
    ns = ctypes.c_double(0)
    rc = ref_lib().srs_ref_sort_soa_timed(len(keys), kind, int(up), thresh, keys.ctypes.data,
                                          len(payloads), _ptrs(payloads), _sizes(payloads),
                                          ctypes.byref(ns))
    assert rc == 0, rc
    return ns.value


def ref_sort_aos(kind, up, elems, thresh=16):
    rc = ref_lib().srs_ref_sort_aos(elems.shape[0], kind, int(up), thresh,
                                    elems.ctypes.data, elems.shape[1])
    assert rc == 0, rc


# --------------------------------------------------------------------------
# key order helpers (numpy) used by the parity checks
# --------------------------------------------------------------------------
def transformed_keys(kind, up, keys):
    """The unsigned sort key the reference's per-bit directions induce
    (bitDirUp, radixSort.hpp:1568-1581): unsigned as is; signed: flip sign
    bit; float: negative -> ~bits, else bits ^ signbit; descending: ~u."""
    ut = KIND_UINT[kind]
    bits = keys.view(ut).astype(np.uint64)
    nb = 8 * key_size(kind)
    mask = np.uint64((1 << nb) - 1)
    sb = np.uint64(1 << (nb - 1))
    name = KIND_NAMES[kind]
    if name.startswith("i"):
        u = bits ^ sb
    elif name.startswith("f"):
        neg = (bits & sb) != 0
        u = np.where(neg, ~bits & mask, bits ^ sb)
    else:
        u = bits
    if not up:
        u = ~u & mask
    return u.astype(np.uint64)


def stable_reference(kind, up, cols, thresh=16):
    """Stable sort by the reference key order (used to check the GPU path,
    which is stable, bit for bit, including payload order). For n <= thresh
    floats compare by value (-0.0 == +0.0), as the reference's leaf does."""
    keys = cols[0]
    u = transformed_keys(kind, up, keys)
    if len(keys) <= thresh and KIND_NAMES[kind].startswith("f"):
        zero = keys == 0
        u = np.where(zero, transformed_keys(kind, up, np.zeros(1, keys.dtype))[0], u)
    order = np.argsort(u, kind="stable")
    return [c[order] for c in cols]


def runs_multiset_equal(keys_a, keys_b, pays_a, pays_b) -> bool:
    """Per maximal run of equal keys, the multiset of payload tuples match
    (the parity contract for an unstable reference)."""
    if not np.array_equal(keys_a.view(np.uint8), keys_b.view(np.uint8)):
        return False
    n = len(keys_a)
    if n == 0 or not pays_a:
        return True
    kb = keys_a.view(KIND_UINT_FOR_DTYPE[keys_a.dtype.itemsize])
    brk = np.flatnonzero(kb[1:] != kb[:-1]) + 1
    starts = np.concatenate([[0], brk])
    run_id = np.repeat(np.arange(len(starts)), np.diff(np.concatenate([starts, [n]])))
    # sort each side by (run, payload bytes) and compare
    def canon(pays):
        rows = np.concatenate([p.view(np.uint8).reshape(n, -1) for p in pays], axis=1)
        order = np.lexsort(tuple(rows[:, ::-1].T) + (run_id,))
        return rows[order]
    return np.array_equal(canon(pays_a), canon(pays_b))


KIND_UINT_FOR_DTYPE = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}
