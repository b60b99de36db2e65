// ref_driver.cpp — extern "C" shim around the REFERENCE's own AVX-512 sort.
//
// TEST / BASELINE INFRASTRUCTURE ONLY. Built by oracle/Makefile directly from
// the reference's single header where it lies
// (/root/reference/radixSort.hpp, included by absolute path; nothing is
// copied into this repo) into oracle/_ref/libsrs_ref.so. Used to
//   * time the reference on the host cores (bench.py cpu_baseline,
//     kind "reference"), and
//   * cross-check the C restatement (oracle/srs_oracle.c) in tests.
// The product library never links it.
//
// Entry points mirror include/srs_c_api.h's srs_sort_soa / srs_sort_aos.
// Because the reference is a template library, each (key type, payload
// pack) needs an instantiation; payload types only matter through their
// sizes, so payloads are instantiated as unsigned integers of the given
// size, and DataElement payload bytes as one std::array<uint8_t, N>.
#include <time.h>
#include <array>
#include <cstdint>
#include <cstring>
#include <type_traits>
#include <utility>

#include REF_HEADER  // "/root/reference/radixSort.hpp"

using simd_sort::DataElement;
using simd_sort::SortIndex;
namespace rs = simd_sort::radix_sort;

namespace {

template <std::size_t N>
struct UIntOf;
template <> struct UIntOf<1> { using type = uint8_t; };
template <> struct UIntOf<2> { using type = uint16_t; };
template <> struct UIntOf<4> { using type = uint32_t; };
template <> struct UIntOf<8> { using type = uint64_t; };

// The reference's CmpSorterNoSort (src/cmp_sorters.hpp:66-78) lives outside
// the single header; a leaf sorter is only a type with a static
// sort<Up>(left, right, keys, payloads...) that radixRecursion calls on each
// range of <= cmpSortThreshold elements (radixSort.hpp:1743). This one leaves
// the range as the partitions left it, as the reference's does.
struct LeafUnsorted {
  template <bool Up, typename K, typename... Ps>
  static inline void sort(const SortIndex, const SortIndex, K* const, Ps* const...) {}
};

// leaf: 0 = CmpSorterInsertionSort, 1 = the no-op leaf (SRS_LEAF_UNSORTED)
thread_local int g_leaf = 0;

template <typename K, bool Up, std::size_t... Sz, std::size_t... I>
int sort_soa_seq(int64_t thresh, int64_t num, void* keys, void* const* pays,
                 std::index_sequence<I...>) {
  // radix_sort::sort<Up, BitSorterSIMD, CmpSorterInsertionSort>(thresh, ...)
  // radixSort.hpp:1761-1768 (the two-argument sort() uses thresh = 16).
  if (g_leaf == 1)
    rs::sort<Up, rs::BitSorterSIMD, LeafUnsorted>((SortIndex)thresh, (SortIndex)num, (K*)keys,
                                                  ((typename UIntOf<Sz>::type*)pays[I])...);
  else
    rs::sort<Up, rs::BitSorterSIMD, simd_sort::CmpSorterInsertionSort>(
        (SortIndex)thresh, (SortIndex)num, (K*)keys,
        ((typename UIntOf<Sz>::type*)pays[I])...);
  return 0;
}

template <typename K, bool Up, std::size_t... Sz>
int sort_soa_pack(int64_t thresh, int64_t num, void* keys, void* const* pays) {
  return sort_soa_seq<K, Up, Sz...>(thresh, num, keys, pays,
                                    std::make_index_sequence<sizeof...(Sz)>{});
}

template <typename K, bool Up>
int sort_soa_k(int64_t thresh, int64_t num, void* keys, int32_t np,
               void* const* pays, const uint32_t* sz) {
  auto is = [&](std::initializer_list<uint32_t> l) {
    if ((int32_t)l.size() != np) return false;
    int32_t j = 0;
    for (uint32_t v : l)
      if (sz[j++] != v) return false;
    return true;
  };
  if (np == 0) return sort_soa_pack<K, Up>(thresh, num, keys, pays);
  if (is({1})) return sort_soa_pack<K, Up, 1>(thresh, num, keys, pays);
  if (is({2})) return sort_soa_pack<K, Up, 2>(thresh, num, keys, pays);
  if (is({4})) return sort_soa_pack<K, Up, 4>(thresh, num, keys, pays);
  if (is({8})) return sort_soa_pack<K, Up, 8>(thresh, num, keys, pays);
  if (is({8, 1})) return sort_soa_pack<K, Up, 8, 1>(thresh, num, keys, pays);
  if (is({8, 8})) return sort_soa_pack<K, Up, 8, 8>(thresh, num, keys, pays);
  if (is({4, 4})) return sort_soa_pack<K, Up, 4, 4>(thresh, num, keys, pays);
  if (is({8, 8, 8})) return sort_soa_pack<K, Up, 8, 8, 8>(thresh, num, keys, pays);
  return -2;
}

template <typename K, bool Up, std::size_t E>
int sort_aos_e(int64_t thresh, int64_t num, void* elems) {
  if constexpr (E == sizeof(K)) {
    using D = DataElement<K>;
    static_assert(sizeof(D) == E);
    rs::sort<Up, rs::BitSorterSIMD, simd_sort::CmpSorterInsertionSort>(
        (SortIndex)thresh, (SortIndex)num, (D*)elems);
    return 0;
  } else if constexpr (E > sizeof(K)) {
    using D = DataElement<K, std::array<uint8_t, E - sizeof(K)>>;
    static_assert(sizeof(D) == E, "DataElement size");
    rs::sort<Up, rs::BitSorterSIMD, simd_sort::CmpSorterInsertionSort>(
        (SortIndex)thresh, (SortIndex)num, (D*)elems);
    return 0;
  } else {
    return -2;
  }
}

template <typename K, bool Up>
int sort_aos_k(int64_t thresh, int64_t num, void* elems, uint32_t esz) {
  switch (esz) {
    case 1: return sort_aos_e<K, Up, 1>(thresh, num, elems);
    case 2: return sort_aos_e<K, Up, 2>(thresh, num, elems);
    case 4: return sort_aos_e<K, Up, 4>(thresh, num, elems);
    case 8: return sort_aos_e<K, Up, 8>(thresh, num, elems);
    case 16: return sort_aos_e<K, Up, 16>(thresh, num, elems);
    case 32: return sort_aos_e<K, Up, 32>(thresh, num, elems);
    case 64: return sort_aos_e<K, Up, 64>(thresh, num, elems);
    default: return -2;
  }
}

#define SRS_KIND_SWITCH(CALL)                      \
  switch (kind) {                                  \
    case 0: return up ? CALL(uint8_t, true) : CALL(uint8_t, false);   \
    case 1: return up ? CALL(int8_t, true) : CALL(int8_t, false);     \
    case 2: return up ? CALL(uint16_t, true) : CALL(uint16_t, false); \
    case 3: return up ? CALL(int16_t, true) : CALL(int16_t, false);   \
    case 4: return up ? CALL(uint32_t, true) : CALL(uint32_t, false); \
    case 5: return up ? CALL(int32_t, true) : CALL(int32_t, false);   \
    case 6: return up ? CALL(uint64_t, true) : CALL(uint64_t, false); \
    case 7: return up ? CALL(int64_t, true) : CALL(int64_t, false);   \
    case 8: return up ? CALL(float, true) : CALL(float, false);       \
    case 9: return up ? CALL(double, true) : CALL(double, false);     \
    default: return -1;                            \
  }

}  // namespace

extern "C" {

// Same argument meaning as srs_sort_soa (include/srs_c_api.h). Returns 0,
// -1 (bad kind) or -2 (payload pack not instantiated here).
int srs_ref_sort_soa(int64_t num, int kind, int up, int64_t thresh, void* keys,
                     int32_t np, void* const* pays, const uint32_t* sz) {
#define CALL(K, U) sort_soa_k<K, U>(thresh, num, keys, np, pays, sz)
  SRS_KIND_SWITCH(CALL)
#undef CALL
}

int srs_ref_sort_aos(int64_t num, int kind, int up, int64_t thresh, void* elems,
                     uint32_t esz) {
#define CALL(K, U) sort_aos_k<K, U>(thresh, num, elems, esz)
  SRS_KIND_SWITCH(CALL)
#undef CALL
}

// srs_ref_sort_soa timed the way the reference's perf harness times it
// (src/perf.hpp:33-46): CLOCK_PROCESS_CPUTIME_ID around the sort call only;
// the elapsed nanoseconds go to *cpu_ns.
int srs_ref_sort_soa_timed(int64_t num, int kind, int up, int64_t thresh, void* keys,
                           int32_t np, void* const* pays, const uint32_t* sz,
                           double* cpu_ns) {
  struct timespec a, b;
  clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &a);
  const int rc = srs_ref_sort_soa(num, kind, up, thresh, keys, np, pays, sz);
  clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &b);
  if (cpu_ns) *cpu_ns = (b.tv_sec - a.tv_sec) * 1e9 + (double)(b.tv_nsec - a.tv_nsec);
  return rc;
}

// srs_ref_sort_soa_timed with the leaf sorter chosen at run time (leaf as
// srs_sort_soa_leaf's: 0 insertion sort, 1 leaves unsorted, the reference's
// CmpSorterNoSort); used by tools/perf_dat.py's cmpThresh files
// (src/perf.hpp:159-212).
int srs_ref_sort_soa_leaf_timed(int64_t num, int kind, int up, int64_t thresh, int leaf,
                                void* keys, int32_t np, void* const* pays, const uint32_t* sz,
                                double* cpu_ns) {
  if (leaf != 0 && leaf != 1) return -3;
  g_leaf = leaf;
  const int rc = srs_ref_sort_soa_timed(num, kind, up, thresh, keys, np, pays, sz, cpu_ns);
  g_leaf = 0;
  return rc;
}

const char* srs_ref_build_info(void) {
  return "jonicho/simd-radix-sort radixSort.hpp (BitSorterSIMD + "
         "CmpSorterInsertionSort), g++ -O3 -mavx512f/bw/dq/vl/vbmi/vbmi2";
}

}  // extern "C"
