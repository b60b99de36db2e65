"""CPU tests of the C-ABI library: it loads without a GPU, exports every
symbol include/srs_c_api.h declares, and validates arguments (no compute)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "srs_c_api.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(srs_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_entry_points():
    fns = declared_functions()
    for f in ["srs_sort_soa", "srs_sort_aos", "srs_sort_soa_device", "srs_sort_aos_device",
              "srs_last_error", "srs_version"]:
        assert f in fns


def test_library_exports_every_declared_symbol():
    import srs_amd
    lib = srs_amd.lib()
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", srs_amd.LIB_PATH],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (srs_[a-z_0-9]+)", out))
    assert set(declared_functions()) <= exported


def test_library_is_gfx950_code_object():
    import srs_amd
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list",
                          "--type=o", f"--input={srs_amd.LIB_PATH}"],
                         capture_output=True, text=True)
    blob = open(srs_amd.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_header_compiles_as_c():
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-fsyntax-only", "-x", "c", HEADER],
                   check=True)


def test_argument_validation_without_gpu():
    import srs_amd
    lib = srs_amd.lib()
    k = np.zeros(4, np.uint32)
    rc = lib.srs_sort_soa(4, 42, 1, 16, k.ctypes.data, 0, None, None)
    assert rc == -1
    assert b"key_kind" in lib.srs_last_error()
    sz = (ctypes.c_uint32 * 1)(3)
    p = (ctypes.c_void_p * 1)(k.ctypes.data)
    assert lib.srs_sort_soa(4, 4, 1, 16, k.ctypes.data, 1, p, sz) == -2
    e = np.zeros((4, 12), np.uint8)
    assert lib.srs_sort_aos(4, 4, 1, 16, e.ctypes.data, 12) == -2
    assert b"power of two" in lib.srs_last_error()
    # num <= 1 is a no-op, as in the reference (radixSort.hpp:1740)
    assert lib.srs_sort_soa(1, 4, 1, 16, k.ctypes.data, 0, None, None) == 0
    assert lib.srs_sort_soa(-5, 4, 1, 16, k.ctypes.data, 0, None, None) == 0
    assert srs_amd.version().startswith("srs_amd")
    # device arrays must be word-aligned (rejected before any device access;
    # the addresses below are never dereferenced)
    fn = lib.srs_sort_soa_device
    fn.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p,
                   ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                   ctypes.c_void_p, ctypes.c_void_p]
    assert fn(4, 6, 1, 16, 0x10004, 0, None, None, None, None, None) == -1  # u64 at +4
    assert b"aligned" in lib.srs_last_error()
    p8 = (ctypes.c_void_p * 1)(0x20002)
    s8 = (ctypes.c_uint32 * 1)(8)
    assert fn(4, 4, 1, 16, 0x10000, 1, p8, s8, None, None, None) == -1  # u64 payload at +2
    fa = lib.srs_sort_aos_device
    fa.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p,
                   ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    assert fa(4, 4, 1, 16, 0x10004, 16, None, None) == -1  # 16-byte records at +4
    assert b"aligned" in lib.srs_last_error()


def _kernel_resources():
    """Per-kernel VGPRs / scratch / occupancy from the build's compiler
    remarks (simd-radix-sort_amd/build/srs_kernels.remarks)."""
    path = os.path.join(REPO, "simd-radix-sort_amd", "build", "srs_kernels.remarks")
    if not os.path.exists(path):
        pytest.skip("no resource remarks (library built elsewhere)")
    res, cur = {}, None
    for line in open(path):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            res[cur] = {}
            continue
        m = re.search(r"(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                      r"LDS Size \[bytes/block\]): (\d+)", line)
        if m and cur:
            res[cur][m.group(1).split()[0]] = int(m.group(2))
    return res


def test_hot_kernels_keep_their_occupancy():
    """The occupancy the tuning relies on: two 16-wave scatter
    workgroups per CU need <= 64 VGPRs (8 waves/SIMD), with or without the
    24 KB digit table; count 8 waves/SIMD (6 for digit-table passes);
    the small local class 6 waves/SIMD (3 workgroups of 8 waves); the
    tile-pair scatter two 8-wave workgroups per CU (4 waves/SIMD, <= 80 KB of
    LDS each); nothing on the hot path spills to scratch."""
    res = _kernel_resources()
    need = {"scatter_kernel": 8, "count_kernel": 8, "local_kernelI": None,
            "scatter_pair_kernel": 4}
    seen = set()
    for name, r in res.items():
        for key, occ in need.items():
            if key not in name:
                continue
            seen.add(key)
            assert r.get("ScratchSize", 0) == 0, (name, r)
            if key == "local_kernelI":
                occ = 6 if "Li512ELi8ELi6E" in name else 4
            if key == "count_kernel" and "Li1E" in name:
                occ = 6  # passes with the big digit table stage up to 26 KB in LDS
                #          (the small-table kind, Li2E, keeps 8 waves per SIMD)
            if key == "count_kernel" and "ImmLi2E" in name:
                occ = 6  # the 8-byte range level: 7 or 8 waves spill VGPRs to scratch
            assert r["Occupancy"] >= occ, (name, r)
            if key == "scatter_pair_kernel":
                assert r["LDS"] * 2 <= 160 * 1024, (name, r)
    assert seen == set(need)


def test_library_matches_the_sources():
    """srs_version() carries the hash of the sources the library was built
    from (simd-radix-sort_amd/Makefile SRC_HASH): a stale libsrs_amd.so
    shipped with the tree fails here, on CPU and on the GPU box alike."""
    import hashlib

    import srs_amd
    pkg = os.path.join(REPO, "simd-radix-sort_amd")
    files = [os.path.join(pkg, "csrc", f) for f in ("srs_kernels.hip", "srs_api.hip",
                                                    "srs_shard.hip", "srs_common.h",
                                                    "srs_kernels.h")]
    files.append(HEADER)
    h = hashlib.sha256(b"".join(open(f, "rb").read() for f in files)).hexdigest()[:16]
    v = srs_amd.version()
    assert v.endswith("src:" + h), (v, h)
