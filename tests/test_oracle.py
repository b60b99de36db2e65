"""CPU tests of the parity oracle (no GPU).

The oracle (oracle/srs_oracle.c) restates the reference's BitSorterSIMD +
radixRecursion + CmpSorterInsertionSort. It is pinned here against golden
vectors produced by the reference itself (tests/golden/, oracle/gen_golden.cpp)
and, where this host can run AVX-512 VBMI2, against the reference's own sort
built from /root/reference (oracle/_ref/libsrs_ref.so)."""
import os

import numpy as np
import pytest

from srs_testlib import (KIND_DTYPES, KIND_NAMES, KIND_UINT, golden_arrays, golden_manifest,
                         key_size, oracle_sort_aos, oracle_sort_soa, ref_lib, ref_sort_aos,
                         ref_sort_soa, runs_multiset_equal, stable_reference)


def beq(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint8),
                          np.ascontiguousarray(b).view(np.uint8))


def test_manifest_covers_reference_test_matrix():
    m = golden_manifest()
    cases = m["cases"]
    assert len(cases) > 1000
    assert {c["key_kind"] for c in cases} == set(range(10))
    assert {c["dist"] for c in cases} >= {"Uniform", "Gaussian", "Zero", "ZeroOne", "Sorted",
                                          "ReverseSorted", "AlmostSorted", "AlmostReverseSorted"}
    assert {c["layout"] for c in cases} == {"soa", "aos"}
    assert {c["up"] for c in cases} == {0, 1}


@pytest.mark.parametrize("family", ["soa", "aos", "large", "index", "zeros"])
def test_oracle_matches_golden_bitwise(family):
    """Bit for bit, payload order included: the restatement reproduces the
    reference's exact (unstable) permutation."""
    bad = []
    for c in golden_manifest()["cases"]:
        if c["family"] != family:
            continue
        ins, outs = golden_arrays(c)
        cols = [a.copy() for a in ins]
        if c["layout"] == "aos":
            oracle_sort_aos(c["key_kind"], c["up"], cols[0], c["thresh"])
        else:
            oracle_sort_soa(c["key_kind"], c["up"], cols[0], cols[1:], c["thresh"])
        if not all(beq(a, b) for a, b in zip(cols, outs)):
            bad.append((KIND_NAMES[c["key_kind"]], c["dist"], c["n"], c["up"]))
    assert not bad, bad[:5]


def test_sequential_bitsorter_same_keys_and_runs():
    """BitSorterSequential (src/radix_sort.hpp:66-92) permutes equal keys
    differently but must give the same keys and per-run payload multisets."""
    for c in golden_manifest()["cases"]:
        if c["layout"] != "soa" or c["family"] not in ("index", "large"):
            continue
        ins, outs = golden_arrays(c)
        cols = [a.copy() for a in ins]
        oracle_sort_soa(c["key_kind"], c["up"], cols[0], cols[1:], c["thresh"], bit_sorter=1)
        assert runs_multiset_equal(cols[0], outs[0], cols[1:], outs[1:])


def test_golden_key_order_is_transformed_unsigned_order():
    """The reference's key order equals the unsigned order of the key
    transform used by the GPU kernels (bitDirUp, radixSort.hpp:1568-1581)."""
    for c in golden_manifest()["cases"]:
        if c["layout"] != "soa":
            continue
        ins, outs = golden_arrays(c)
        st = stable_reference(c["key_kind"], c["up"], ins, c["thresh"])
        assert beq(st[0], outs[0]), (c["family"], c["key_kind"], c["dist"], c["n"])
        assert runs_multiset_equal(st[0], outs[0], st[1:], outs[1:])


needs_ref = pytest.mark.skipif(ref_lib() is None,
                               reason="reference build (oracle/_ref) or AVX-512 VBMI2 host missing")


@needs_ref
@pytest.mark.parametrize("kind", range(10), ids=KIND_NAMES)
def test_oracle_vs_reference_random(kind):
    rng = np.random.default_rng(kind)
    for n in (1, 2, 16, 17, 100, 5000, 40000):
        for up in (True, False):
            nb = 8 * key_size(kind)
            bits = rng.integers(0, 2**nb, n, dtype=np.uint64) >> np.uint64(rng.integers(0, nb))
            keys = bits.astype(KIND_UINT[kind]).view(KIND_DTYPES[kind])
            if KIND_NAMES[kind].startswith("f"):
                keys = np.where(np.isnan(keys), KIND_DTYPES[kind](0.5), keys)
            p = np.arange(n, dtype=np.uint64)
            a_k, a_p = keys.copy(), p.copy()
            b_k, b_p = keys.copy(), p.copy()
            oracle_sort_soa(kind, up, a_k, [a_p])
            ref_sort_soa(kind, up, b_k, [b_p])
            assert beq(a_k, b_k) and beq(a_p, b_p), (n, up)


@needs_ref
@pytest.mark.parametrize("esz", [8, 16, 32, 64])
def test_oracle_vs_reference_combined(esz):
    rng = np.random.default_rng(esz)
    n = 20000
    e = rng.integers(0, 256, (n, esz), dtype=np.uint8)
    e[:, :4] = (rng.integers(0, 50, n).astype(np.uint32)).view(np.uint8).reshape(n, 4)
    a, b = e.copy(), e.copy()
    oracle_sort_aos(4, True, a)
    ref_sort_aos(4, True, b)
    assert beq(a, b)


@needs_ref
@pytest.mark.parametrize("thresh", [1, 16, 64, 1024])
def test_reference_leaves_unsorted_guarantee(thresh):
    """The reference with its no-op leaf sorter (CmpSorterNoSort,
    src/cmp_sorters.hpp:66-78; oracle/_ref's leaf = 1) keeps the contract
    tests/test_gpu_leaf.py holds the GPU's SRS_LEAF_UNSORTED mode to: the
    multiset is kept and every key ends within thresh - 1 places of its
    sorted slot (thesis 3113-3124). Sorted leaves (leaf = 0) give the
    insertion sort's fully sorted output."""
    import ctypes
    lib = ref_lib()
    rng = np.random.default_rng(thresh)
    n = 1 << 16
    keys = rng.integers(0, 1 << 20, n, dtype=np.uint64)  # duplicates in every leaf size
    srt = np.sort(keys)
    for leaf in (0, 1):
        k = keys.copy()
        p = np.arange(n, dtype=np.uint64)
        arr = (ctypes.c_void_p * 1)(p.ctypes.data)
        sz = (ctypes.c_uint32 * 1)(8)
        ns = ctypes.c_double()
        assert lib.srs_ref_sort_soa_leaf_timed(n, 6, 1, thresh, leaf, k.ctypes.data, 1, arr, sz,
                                               ctypes.byref(ns)) == 0
        assert np.array_equal(keys[p.astype(np.int64)], k)  # payloads travel with their keys
        if leaf == 0 or thresh == 1:
            assert np.array_equal(k, srt)
            continue
        assert np.array_equal(np.sort(k), srt)
        assert not np.array_equal(k, srt)  # leaves really stay unsorted
        # each key's slot lies inside its value's sorted run widened by thresh - 1
        lo = np.searchsorted(srt, k, "left")
        hi = np.searchsorted(srt, k, "right") - 1
        i = np.arange(n)
        assert np.all(i >= lo - (thresh - 1)) and np.all(i <= hi + (thresh - 1))


def test_oracle_under_address_and_ub_sanitizers():
    """The C restatement built with -fsanitize=address,undefined (oracle/Makefile
    `asan`) sorts every key kind, both directions, SoA payload
    packs and AoS records of 2-64 bytes around the leaf threshold and the
    emulated vector widths; the reference's invariants must hold and no
    sanitizer may fire."""
    import subprocess
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-C", os.path.join(repo, "oracle"), "asan"], check=True,
                   capture_output=True)
    r = subprocess.run([os.path.join(repo, "oracle", "_build", "asan_check")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout and "ERROR" not in r.stderr
