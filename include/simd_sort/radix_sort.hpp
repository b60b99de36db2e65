// simd_sort/radix_sort.hpp — drop-in replacement for jonicho/simd-radix-sort's
// radixSort.hpp on AMD Instinct MI355X.
//
// Same namespace, same overloads, same semantics as the reference
// (radixSort.hpp:1761-1783, src/radix_sort.hpp:297-337):
//
//   simd_sort::radix_sort::sort(num, keyArray, payloadArrays...);
//   simd_sort::radix_sort::sort<false>(num, keyArray, payloadArrays...);
//   simd_sort::radix_sort::sort(num, (simd_sort::DataElement<K, Ps...>*) combined);
//   simd_sort::radix_sort::sort<Up, BitSorter, CmpSorter>(cmpSortThreshold, num, ...);
//   simd_sort::radix_sort::sort(cmpSortThreshold, num, ...);   // defaulted, :1761-1763
//
// BitSorter may be spelled as in radixSort.hpp (`BitSorterSIMD`, a plain
// name) or as in src/radix_sort.hpp:109 (`BitSorterSIMD<>`,
// `BitSorterSIMD<false>`, `BitSorterSIMD<true>` = OneReg).
//
// The arrays are sorted in place. Instead of the AVX-512 partition the work
// runs as HIP kernels on the GPU through the C ABI in srs_c_api.h
// (link with -lsrs_amd). Unlike the reference this header needs no AVX-512
// and compiles with any C++17 compiler.
//
// Error behaviour: the reference returns void and cannot fail at run time;
// unsupported type combinations fail at compile time (static_assert), as
// there. A run-time failure of the GPU path (no device, out of memory)
// prints the library's message and calls std::abort(): there is no silent
// CPU fallback.
#pragma once

#include <sys/types.h>

#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <tuple>
#include <type_traits>

#include "../srs_c_api.h"

namespace simd_sort {

// src/common.hpp:14
using SortIndex = ssize_t;

// src/common.hpp:105-106
template <std::size_t X>
inline constexpr bool is_power_of_two = X > 0 && (X & (X - 1)) == 0;

// Combined key + payload element, layout-identical to the reference's
// (radixSort.hpp:180-195): the key at offset 0, payloads in a std::tuple.
template <typename K, typename... Ps>
struct DataElement {
  K key;
  std::tuple<Ps...> payloads;
  bool operator<(const DataElement& other) const { return key < other.key; }
  bool operator>(const DataElement& other) const { return key > other.key; }
};

template <typename K>
struct DataElement<K> {
  K key;
  bool operator<(const DataElement& other) const { return key < other.key; }
  bool operator>(const DataElement& other) const { return key > other.key; }
};

// Leaf sorter selectors. The reference's CmpSorterInsertionSort
// (radixSort.hpp:159-178) becomes the GPU's LDS-resident leaf; the name is
// kept so that existing call sites compile unchanged.
struct CmpSorterInsertionSort {};
// src/cmp_sorters.hpp:66-78: the recursion stops at leaves of <=
// cmpSortThreshold elements and leaves them in partition order, so each
// element ends within cmpSortThreshold of its sorted position (thesis
// 3113-3124). On the GPU the local pass skips its in-bucket rank when every
// bucket holds <= cmpSortThreshold keys (SRS_LEAF_UNSORTED); every leaf holds
// exactly the elements a full sort puts there. The order inside a leaf is
// unspecified and may differ between runs.
struct CmpSorterNoSort {};
// src/cmp_sorters.hpp:40-63 (needs the vendored bramas sorters there): the
// leaves are sorted (as here); the reference's type restrictions are kept
// as compile-time errors below.
struct CmpSorterBramasSmallSort {};

namespace radix_sort {

// Bit-sorter selectors. src/radix_sort.hpp:109 declares
// `template <bool OneReg = false> struct BitSorterSIMD` (OneReg: one
// register per payload vector, :119-121); radixSort.hpp:1583 has the plain
// `struct BitSorterSIMD`. Here it is the class template, and the sort()
// overloads below also take the template itself as a template-template
// argument, so both spellings compile. BitSorterSequential is
// src/radix_sort.hpp:66. All produce the same key order; on the GPU all run
// the same multi-bit digit passes.
template <bool OneReg = false>
struct BitSorterSIMD {
  static std::string name() { return OneReg ? "BitSorterSIMD<OneReg>" : "BitSorterSIMD"; }
};
struct BitSorterSequential {
  static std::string name() { return "BitSorterSequential"; }
};

namespace detail {

template <typename K>
constexpr int key_kind() {
  if constexpr (std::is_same_v<K, uint8_t>) return SRS_KEY_U8;
  else if constexpr (std::is_same_v<K, int8_t>) return SRS_KEY_I8;
  else if constexpr (std::is_same_v<K, uint16_t>) return SRS_KEY_U16;
  else if constexpr (std::is_same_v<K, int16_t>) return SRS_KEY_I16;
  else if constexpr (std::is_same_v<K, uint32_t>) return SRS_KEY_U32;
  else if constexpr (std::is_same_v<K, int32_t>) return SRS_KEY_I32;
  else if constexpr (std::is_same_v<K, uint64_t>) return SRS_KEY_U64;
  else if constexpr (std::is_same_v<K, int64_t>) return SRS_KEY_I64;
  else if constexpr (std::is_same_v<K, float>) return SRS_KEY_F32;
  else if constexpr (std::is_same_v<K, double>) return SRS_KEY_F64;
  else if constexpr (std::is_same_v<K, char> && std::is_signed_v<char>) return SRS_KEY_I8;
  else if constexpr (std::is_same_v<K, char>) return SRS_KEY_U8;
  else if constexpr (std::is_same_v<K, long> && sizeof(long) == 8) return SRS_KEY_I64;
  else if constexpr (std::is_same_v<K, unsigned long> && sizeof(long) == 8) return SRS_KEY_U64;
  else if constexpr (std::is_same_v<K, long long>) return SRS_KEY_I64;
  else if constexpr (std::is_same_v<K, unsigned long long>) return SRS_KEY_U64;
  else return -1;
}

template <typename CmpSorter>
inline constexpr bool known_cmp_sorter = std::is_same_v<CmpSorter, CmpSorterInsertionSort> ||
                                         std::is_same_v<CmpSorter, CmpSorterNoSort> ||
                                         std::is_same_v<CmpSorter, CmpSorterBramasSmallSort>;

template <typename CmpSorter>
inline constexpr int leaf_mode =
    std::is_same_v<CmpSorter, CmpSorterNoSort> ? SRS_LEAF_UNSORTED : SRS_LEAF_SORTED;

template <typename BitSorter>
inline constexpr bool known_bit_sorter = std::is_same_v<BitSorter, BitSorterSIMD<false>> ||
                                         std::is_same_v<BitSorter, BitSorterSIMD<true>> ||
                                         std::is_same_v<BitSorter, BitSorterSequential>;

// src/cmp_sorters.hpp:47-61
template <bool Up, typename CmpSorter, typename K, typename... Ps>
constexpr void check_cmp_sorter() {
  static_assert(known_cmp_sorter<CmpSorter>,
                "CmpSorter must be CmpSorterInsertionSort, CmpSorterNoSort or "
                "CmpSorterBramasSmallSort (a user-defined leaf sorter cannot run on the GPU)");
  if constexpr (std::is_same_v<CmpSorter, CmpSorterBramasSmallSort>) {
    static_assert(std::is_same_v<K, double> || std::is_same_v<K, int>,
                  "BramasSmallSort only supports int and double");
    static_assert(Up, "BramasSmallSort only supports sorting up");
    static_assert(sizeof...(Ps) <= 1, "BramasSmallSort only supports one or zero payloads");
    static_assert(((std::is_same_v<K, Ps>) && ...), "key and payload must have the same type");
  }
}

template <typename T>
inline constexpr bool valid_payload =
    std::is_trivially_copyable_v<T> &&
    (sizeof(T) == 1 || sizeof(T) == 2 || sizeof(T) == 4 || sizeof(T) == 8);

inline void check(int rc, const char* what) {
  if (rc != SRS_OK) {
    std::fprintf(stderr, "simd_sort::radix_sort::%s failed (%d): %s\n", what, rc,
                 srs_last_error());
    std::abort();
  }
}

}  // namespace detail

// sort(cmpSortThreshold, num, keys, payloads...) — radixSort.hpp:1761-1768
// (defaults as there: Up = true, BitSorterSIMD, CmpSorterInsertionSort)
template <bool Up = true, typename BitSorter = BitSorterSIMD<>,
          typename CmpSorter = CmpSorterInsertionSort, typename K, typename... Ps>
void sort(SortIndex cmpSortThreshold, const SortIndex num, K* const keys,
          Ps* const... payloads) {
  static_assert(detail::known_bit_sorter<BitSorter>,
                "BitSorter must be BitSorterSIMD or BitSorterSequential");
  detail::check_cmp_sorter<Up, CmpSorter, K, Ps...>();
  static_assert(detail::key_kind<K>() >= 0,
                "key type must be one of u8/i8/u16/i16/u32/i32/u64/i64/float/double");
  static_assert((detail::valid_payload<Ps> && ...),
                "payload element sizes must be 1, 2, 4 or 8 bytes");
  static_assert(sizeof...(Ps) <= SRS_MAX_PAYLOADS, "too many payload arrays");
  void* pays[sizeof...(Ps) + 1] = {(void*)payloads..., nullptr};
  uint32_t sizes[sizeof...(Ps) + 1] = {(uint32_t)sizeof(Ps)..., 0};
  detail::check(srs_sort_soa_leaf((int64_t)num, detail::key_kind<K>(), Up ? 1 : 0,
                                  (int64_t)cmpSortThreshold, detail::leaf_mode<CmpSorter>,
                                  (void*)keys, (int32_t)sizeof...(Ps), pays, sizes),
                "sort");
}

// sort(cmpSortThreshold, num, DataElement<K, Ps...>*) — radixSort.hpp:1770-1778
// (the reference also reaches it through the defaulted SoA form with
// K = DataElement; partial ordering picks this overload for both)
template <bool Up = true, typename BitSorter = BitSorterSIMD<>,
          typename CmpSorter = CmpSorterInsertionSort, typename K, typename... Ps>
void sort(SortIndex cmpSortThreshold, const SortIndex num,
          DataElement<K, Ps...>* const elements) {
  static_assert(detail::known_bit_sorter<BitSorter>,
                "BitSorter must be BitSorterSIMD or BitSorterSequential");
  static_assert(detail::known_cmp_sorter<CmpSorter>,
                "CmpSorter must be CmpSorterInsertionSort, CmpSorterNoSort or "
                "CmpSorterBramasSmallSort (a user-defined leaf sorter cannot run on the GPU)");
  static_assert(is_power_of_two<sizeof(DataElement<K, Ps...>)>,
                "size of DataElement<K, Ps...> must be a power of two");
  static_assert(sizeof(DataElement<K, Ps...>) <= 64, "DataElement larger than 64 bytes");
  static_assert(detail::key_kind<K>() >= 0,
                "key type must be one of u8/i8/u16/i16/u32/i32/u64/i64/float/double");
  detail::check(srs_sort_aos_leaf((int64_t)num, detail::key_kind<K>(), Up ? 1 : 0,
                                  (int64_t)cmpSortThreshold, detail::leaf_mode<CmpSorter>,
                                  (void*)elements, (uint32_t)sizeof(DataElement<K, Ps...>)),
                "sort");
}

// The radixSort.hpp spelling sort<Up, BitSorterSIMD, CmpSorter>(...): the
// bit sorter named without template arguments (radixSort.hpp:1583, 1764).
template <bool Up, template <bool> class BitSorter, typename CmpSorter = CmpSorterInsertionSort,
          typename K, typename... Ps>
void sort(SortIndex cmpSortThreshold, const SortIndex num, K* const keys,
          Ps* const... payloads) {
  sort<Up, BitSorter<false>, CmpSorter>(cmpSortThreshold, num, keys, payloads...);
}

template <bool Up, template <bool> class BitSorter, typename CmpSorter = CmpSorterInsertionSort,
          typename K, typename... Ps>
void sort(SortIndex cmpSortThreshold, const SortIndex num,
          DataElement<K, Ps...>* const elements) {
  sort<Up, BitSorter<false>, CmpSorter>(cmpSortThreshold, num, elements);
}

// sort<Up>(num, keys, payloads...) — radixSort.hpp:1780-1783 (threshold 16)
template <bool Up = true, typename K, typename... Ps>
void sort(const SortIndex num, K* const keys, Ps* const... payloads) {
  sort<Up, BitSorterSIMD<>, CmpSorterInsertionSort>(16, num, keys, payloads...);
}

// ---- device-resident extension (no reference counterpart) ----------------
// Same semantics on arrays already in HBM, enqueued on `stream` (a
// hipStream_t, nullptr = default stream).
namespace device {

template <bool Up = true, typename K, typename... Ps>
void sort(void* stream, const SortIndex num, K* const keys, Ps* const... payloads) {
  static_assert(detail::key_kind<K>() >= 0, "unsupported key type");
  static_assert((detail::valid_payload<Ps> && ...), "payload sizes must be 1, 2, 4 or 8");
  void* pays[sizeof...(Ps) + 1] = {(void*)payloads..., nullptr};
  uint32_t sizes[sizeof...(Ps) + 1] = {(uint32_t)sizeof(Ps)..., 0};
  detail::check(srs_sort_soa_device((int64_t)num, detail::key_kind<K>(), Up ? 1 : 0, 16,
                                    (void*)keys, (int32_t)sizeof...(Ps), pays, sizes, nullptr,
                                    nullptr, stream),
                "device::sort");
}

template <bool Up = true, typename K, typename... Ps>
void sort(void* stream, const SortIndex num, DataElement<K, Ps...>* const elements) {
  static_assert(is_power_of_two<sizeof(DataElement<K, Ps...>)>,
                "size of DataElement<K, Ps...> must be a power of two");
  detail::check(srs_sort_aos_device((int64_t)num, detail::key_kind<K>(), Up ? 1 : 0, 16,
                                    (void*)elements, (uint32_t)sizeof(DataElement<K, Ps...>),
                                    nullptr, stream),
                "device::sort");
}

}  // namespace device
}  // namespace radix_sort
}  // namespace simd_sort
