"""The reference's correctness matrix (src/test.cpp) re-expressed in C++
against the drop-in header include/simd_sort/radix_sort.hpp (tests/cpp/
test_dropin.cpp): {Separate, Combined} x {Up, Down} x 10 key types x 14
payload packs x 8 distributions x n in {1, 10, 100, 1000, 10000}."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(REPO, "tests", "cpp")
BIN = os.path.join(CPP, "_build", "test_dropin")


def test_dropin_header_compiles_without_avx512():
    """The drop-in header needs no AVX-512 (unlike the reference's)."""
    src = ('#include "simd_sort/radix_sort.hpp"\n'
           "int main(){ unsigned long long k[4]={3,1,2,0}; float p[4]={0,1,2,3};\n"
           " simd_sort::radix_sort::sort(4, k, p);\n"
           " simd_sort::DataElement<unsigned, unsigned> e[2]{};\n"
           " simd_sort::radix_sort::sort<false>(2, e);\n"
           " return 0; }\n")
    subprocess.run(["g++", "-std=c++17", "-mno-avx512f", "-fsyntax-only", "-x", "c++",
                    "-I", os.path.join(REPO, "include"), "-"], input=src.encode(), check=True)


def test_dropin_rejects_non_power_of_two_element_at_compile_time():
    src = ('#include "simd_sort/radix_sort.hpp"\n'
           "int main(){ simd_sort::DataElement<float, unsigned, unsigned> e[2]{};\n"
           " simd_sort::radix_sort::sort(2, e); return 0; }\n")
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-x", "c++",
                        "-I", os.path.join(REPO, "include"), "-"], input=src.encode(),
                       capture_output=True)
    assert r.returncode != 0 and b"power of two" in r.stderr


def _compile(src):
    return subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-x", "c++",
                           "-I", os.path.join(REPO, "include"), "-"], input=src.encode(),
                          capture_output=True)


def test_dropin_accepts_every_reference_sorter_tag():
    """src/cmp_sorters.hpp's three leaf sorters and both bit sorters."""
    src = ('#include "simd_sort/radix_sort.hpp"\n'
           "using namespace simd_sort;\n"
           "int main(){ double k[4]={3,1,2,0}; double p[4]={0,1,2,3}; int i[4]={4,3,2,1};\n"
           " radix_sort::sort<true, radix_sort::BitSorterSIMD, CmpSorterNoSort>(16, 4, k, p);\n"
           " radix_sort::sort<true, radix_sort::BitSorterSequential, CmpSorterInsertionSort>(16, 4, k);\n"
           " radix_sort::sort<true, radix_sort::BitSorterSIMD, CmpSorterBramasSmallSort>(16, 4, k, p);\n"
           " radix_sort::sort<true, radix_sort::BitSorterSIMD, CmpSorterBramasSmallSort>(16, 4, i);\n"
           " DataElement<unsigned, unsigned> e[2]{};\n"
           " radix_sort::sort<false, radix_sort::BitSorterSIMD, CmpSorterNoSort>(16, 2, e);\n"
           " return 0; }\n")
    r = _compile(src)
    assert r.returncode == 0, r.stderr.decode()[-2000:]


def _compile_with(src, *extra):
    return subprocess.run(["g++", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-fsyntax-only",
                           "-x", "c++", "-I", os.path.join(REPO, "include"), "-I", CPP, *extra,
                           "-"], input=src.encode(), capture_output=True)


def test_dropin_accepts_the_reference_call_forms():
    """Every call spelling the reference accepts:
    the defaulted thresholded form (radixSort.hpp:1761-1763), the plain
    `BitSorterSIMD` of radixSort.hpp:1583 and the class template
    `BitSorterSIMD<OneReg>` of src/radix_sort.hpp:109, and the harness
    adapter's shapes (src/sort_methods.hpp:24-98, re-expressed in
    tests/cpp/sort_method.hpp) for every bit/leaf sorter it names."""
    src = ('#include "simd_sort/radix_sort.hpp"\n'
           '#include "sort_method.hpp"\n'
           "using namespace simd_sort; namespace rs = simd_sort::radix_sort;\n"
           "using srs_test::RadixMethod;\n"
           "int main(){ unsigned long long k[4]={3,1,2,0}; unsigned long long p[4]={0,1,2,3};\n"
           " int i[4]={4,3,2,1}; double d[4]={1,2,3,4}; float f[4]={1,2,3,4};\n"
           " rs::sort(16, 4, k, p); rs::sort<false>(16, 4, k); rs::sort(16, 4, f, p, i);\n"
           " rs::sort<true, rs::BitSorterSIMD, CmpSorterInsertionSort>(16, 4, k, p);\n"
           " rs::sort<true, rs::BitSorterSIMD<>, CmpSorterInsertionSort>(16, 4, k, p);\n"
           " rs::sort<false, rs::BitSorterSIMD<true>, CmpSorterNoSort>(16, 4, k, p);\n"
           " rs::sort<true, rs::BitSorterSequential>(64, 4, k, p);\n"
           " rs::sort(4, k, p); rs::sort<false>(4, k);\n"
           " DataElement<unsigned long long, unsigned long long> e[2]{};\n"
           " rs::sort(16, 2, e); rs::sort(2, e); rs::sort<false>(2, e);\n"
           " rs::sort<false, rs::BitSorterSIMD, CmpSorterNoSort>(16, 2, e);\n"
           " rs::sort<true, rs::BitSorterSIMD<true>, CmpSorterInsertionSort>(16, 2, e);\n"
           " static_assert(std::is_same_v<rs::BitSorterSIMD<>, rs::BitSorterSIMD<false>>);\n"
           " (void)rs::BitSorterSIMD<true>::name(); (void)rs::BitSorterSequential::name();\n"
           " RadixMethod<rs::BitSorterSIMD<false>, CmpSorterInsertionSort>::sort(4, k, p);\n"
           " RadixMethod<rs::BitSorterSIMD<true>, CmpSorterInsertionSort>::sort<false>(4, k, p);\n"
           " RadixMethod<rs::BitSorterSequential, CmpSorterInsertionSort>::sort(4, d);\n"
           " RadixMethod<rs::BitSorterSIMD<false>, CmpSorterNoSort>::sortThresh(64, 4, k, p);\n"
           " RadixMethod<rs::BitSorterSIMD<false>, CmpSorterBramasSmallSort>::sort(4, i, i);\n"
           " RadixMethod<rs::BitSorterSIMD<true>, CmpSorterBramasSmallSort>::sort(4, d);\n"
           " RadixMethod<rs::BitSorterSIMD<false>, CmpSorterInsertionSort, true>::sort(2, e);\n"
           " return RadixMethod<rs::BitSorterSIMD<true>, CmpSorterNoSort, true>::name().size()"
           " == 0; }\n")
    r = _compile_with(src)
    assert r.returncode == 0, r.stderr.decode()[-3000:]


@pytest.mark.parametrize("call,msg", [
    ("radix_sort::sort<true, radix_sort::BitSorterSIMD, CmpSorterBramasSmallSort>(16, 4, f)",
     "only supports int and double"),
    ("radix_sort::sort<false, radix_sort::BitSorterSIMD, CmpSorterBramasSmallSort>(16, 4, k)",
     "only supports sorting up"),
    ("radix_sort::sort<true, radix_sort::BitSorterSIMD, CmpSorterBramasSmallSort>(16, 4, k, f)",
     "same type"),
    ("radix_sort::sort<true, radix_sort::BitSorterSIMD, MySorter>(16, 4, k)",
     "user-defined leaf sorter"),
])
def test_dropin_rejects_what_the_reference_rejects(call, msg):
    src = ('#include "simd_sort/radix_sort.hpp"\n'
           "using namespace simd_sort; struct MySorter {};\n"
           "int main(){ double k[4]={3,1,2,0}; float f[4]={0,1,2,3};\n "
           + call + "; return 0; }\n")
    r = _compile(src)
    assert r.returncode != 0 and msg.encode() in r.stderr, r.stderr.decode()[-1500:]


@pytest.mark.gpu
def test_dropin_matrix_on_gpu():
    subprocess.run(["make", "-C", CPP, "_build/test_dropin"], check=True)  # (incremental)
    r = subprocess.run([BIN, "10000", "42"], capture_output=True, text=True, timeout=900)
    tail = "\n".join(r.stdout.splitlines()[-12:])
    assert r.returncode == 0 and "All tests passed" in r.stdout, tail + r.stderr[-2000:]


@pytest.mark.gpu
def test_shard_sort_cabi_over_rccl_matches_reference(tmp_path):
    """The multi-GPU shard sort through the C ABI, driven from C++ without
    torch (tests/cpp/test_shard.cpp): both RCCL communicator kinds at world 1
    and three ranks over the host-staged transport equal the one-GPU sort bit
    for bit, and (here) the output equals
    the REFERENCE's own sort of the same input (oracle/_ref, radixSort.hpp)
    at 2^25 + 1234 records: the shard path's partition level, segmented
    round sorts and stripe/gathered levels all run."""
    import numpy as np

    from srs_testlib import ref_lib, ref_sort_soa
    if ref_lib() is None:
        pytest.fail("oracle/_ref/libsrs_ref.so missing or host lacks AVX-512 VBMI2")
    binp = os.path.join(CPP, "_build", "test_shard")
    subprocess.run(["make", "-C", CPP, "_build/test_shard"], check=True)  # (incremental)
    n = (1 << 25) + 1234
    prefix = str(tmp_path / "shard")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([binp, str(n), prefix], capture_output=True, text=True, timeout=600,
                       env=env)
    assert r.returncode == 0 and "shard ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
    k = np.fromfile(prefix + "_in_k.bin", dtype=np.uint64)
    p = np.fromfile(prefix + "_in_p.bin", dtype=np.uint64)
    ref_sort_soa(6, True, k, [p])
    assert np.array_equal(np.fromfile(prefix + "_out_k.bin", dtype=np.uint64), k)
    assert np.array_equal(np.fromfile(prefix + "_out_p.bin", dtype=np.uint64), p)
