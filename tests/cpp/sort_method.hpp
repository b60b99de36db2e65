// sort_method.hpp — the call shapes of the reference's harness adapter
// SortMethodRadixSort<BitSorter, CmpSorter, Combined>
// (src/sort_methods.hpp:24-98), written against the drop-in header.
//
// It is the §8(b) "Callers" row: code written for the reference names
// radix_sort::BitSorterSIMD<false> / <true> / BitSorterSequential as types,
// compares them with std::is_same_v, picks a default threshold per bit
// sorter (16 / 64 / 16*64/sizeof(K), :77-89) and forwards to
// radix_sort::sort<Up, BitSorter, CmpSorter>(thresh, num, keys, payloads...)
// (:91-97). None of it may need changes to compile and run on the GPU.
#pragma once

#include <string>
#include <type_traits>

#include "simd_sort/radix_sort.hpp"

namespace srs_test {

template <typename>
inline constexpr bool always_false = false;

template <typename BitSorter, typename CmpSorter, bool Combined = false>
struct RadixMethod {
  static std::string name() {
    namespace rs = simd_sort::radix_sort;
    std::string n = "Radix";
    if constexpr (std::is_same_v<BitSorter, rs::BitSorterSequential>) n += "Seq";
    else if constexpr (std::is_same_v<BitSorter, rs::BitSorterSIMD<false>>) n += "SIMD";
    else if constexpr (std::is_same_v<BitSorter, rs::BitSorterSIMD<true>>) n += "SIMDOneReg";
    else static_assert(always_false<BitSorter>, "unknown bit sorter");
    if constexpr (std::is_same_v<CmpSorter, simd_sort::CmpSorterNoSort>) n += "NoCmp";
    else if constexpr (std::is_same_v<CmpSorter, simd_sort::CmpSorterBramasSmallSort>)
      n += "BramSmall";
    if constexpr (Combined) n += "Combined";
    return n;
  }

  template <bool Up = true, typename K, typename... Ps>
  static void sort(const simd_sort::SortIndex num, K* const keys, Ps* const... payloads) {
    if constexpr (std::is_same_v<CmpSorter, simd_sort::CmpSorterBramasSmallSort>)
      sortThresh<Up>(16 * 64 / sizeof(K), num, keys, payloads...);
    else if constexpr (std::is_same_v<BitSorter, simd_sort::radix_sort::BitSorterSequential>)
      sortThresh<Up>(64, num, keys, payloads...);
    else
      sortThresh<Up>(16, num, keys, payloads...);
  }

  template <bool Up = true, typename K, typename... Ps>
  static void sortThresh(const simd_sort::SortIndex thresh, const simd_sort::SortIndex num,
                         K* const keys, Ps* const... payloads) {
    simd_sort::radix_sort::sort<Up, BitSorter, CmpSorter>(thresh, num, keys, payloads...);
  }
};

}  // namespace srs_test
