// test_dropin.cpp — the reference's correctness matrix (src/test.cpp:20-224),
// re-expressed against the MI355X drop-in header.
//
// Cartesian product: {Separate, Combined} x {Up, Down} x 10 key types x
// payload packs x 8 input distributions x num in {1, 10, 100, ...}. Each case
// generates data, sorts it with simd_sort::radix_sort::sort (the GPU path),
// and checks the same invariants as the reference's Data::checkData
// (src/data.hpp:272-310): keys sorted in the requested direction, every
// payload equal to the function of its key it was generated from, and the
// multiset of keys unchanged (the reference checks presence both ways).
//
// Usage: test_dropin [maxNum=100000] [seed=42]; exit code 0 iff all pass.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <tuple>
#include <vector>

#include "simd_sort/radix_sort.hpp"
#include "sort_method.hpp"  // own rewrite of the harness adapter's call shapes

using namespace simd_sort;

enum class Dist { Uniform, Gaussian, Zero, ZeroOne, Sorted, ReverseSorted, AlmostSorted,
                  AlmostReverseSorted };
static const char* dist_name(Dist d) {
  static const char* n[] = {"Uniform", "Gaussian", "Zero", "ZeroOne", "Sorted",
                            "ReverseSorted", "AlmostSorted", "AlmostReverseSorted"};
  return n[(int)d];
}
template <typename T> const char* tname();
#define TN(T, S) template <> const char* tname<T>() { return S; }
TN(uint8_t, "uint8") TN(int8_t, "int8") TN(uint16_t, "uint16") TN(int16_t, "int16")
TN(uint32_t, "uint32") TN(int32_t, "int32") TN(uint64_t, "uint64") TN(int64_t, "int64")
TN(float, "float") TN(double, "double")

// payload p of key k: a hash of the key's bytes (payload = f(key) makes the
// output of an unstable sort checkable, as src/data.hpp:393-406 does)
template <typename K, typename P>
static P payload_of(const K& k, int column) {
  uint64_t b = 0;
  std::memcpy(&b, &k, sizeof(K));
  uint64_t x = b + 0x9E3779B97F4A7C15ull * (uint64_t)(column + 1);
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  P p;
  std::memcpy(&p, &x, sizeof(P));
  return p;
}

template <typename K>
static std::vector<K> make_keys(std::size_t n, Dist d, std::mt19937& gen) {
  std::vector<K> k(n);
  auto uniform = [&] {
    if constexpr (std::is_integral_v<K>) {
      std::uniform_int_distribution<K> u(std::numeric_limits<K>::lowest(),
                                         std::numeric_limits<K>::max());
      for (auto& x : k) x = u(gen);
    } else {
      std::uniform_real_distribution<K> u(K(-1), K(1));
      for (auto& x : k) x = u(gen);
    }
  };
  auto gaussian = [&] {
    if constexpr (std::is_integral_v<K>) {
      std::normal_distribution<double> g(0, 100);
      for (auto& x : k) x = (K)std::llround(g(gen));
    } else {
      std::normal_distribution<K> g(0, 1);
      for (auto& x : k) x = g(gen);
    }
  };
  auto base = [&] { if constexpr (std::is_integral_v<K>) uniform(); else gaussian(); };
  auto displace = [&] {
    const std::size_t m = (std::size_t)std::exp2(std::log10((double)n));
    std::uniform_int_distribution<std::size_t> u(0, n - 1);
    for (std::size_t i = 0; i < m; i++) std::swap(k[u(gen)], k[u(gen)]);
  };
  switch (d) {
    case Dist::Uniform: uniform(); break;
    case Dist::Gaussian: gaussian(); break;
    case Dist::Zero: std::fill(k.begin(), k.end(), K(0)); break;
    case Dist::ZeroOne: for (auto& x : k) x = K(gen() % 2); break;
    case Dist::Sorted: base(); std::sort(k.begin(), k.end()); break;
    case Dist::ReverseSorted: base(); std::sort(k.rbegin(), k.rend()); break;
    case Dist::AlmostSorted: base(); std::sort(k.begin(), k.end()); displace(); break;
    case Dist::AlmostReverseSorted: base(); std::sort(k.rbegin(), k.rend()); displace(); break;
  }
  return k;
}

template <typename K>
static bool same_key_multiset(std::vector<K> a, std::vector<K> b) {
  auto bits = [](const K& x) { uint64_t v = 0; std::memcpy(&v, &x, sizeof(K)); return v; };
  auto lt = [&](const K& x, const K& y) { return bits(x) < bits(y); };
  std::sort(a.begin(), a.end(), lt);
  std::sort(b.begin(), b.end(), lt);
  return std::equal(a.begin(), a.end(), b.begin(), [&](const K& x, const K& y) {
    return bits(x) == bits(y);
  });
}

template <bool Up, typename K>
static bool is_sorted_dir(const std::vector<K>& k) {
  for (std::size_t i = 1; i < k.size(); i++)
    if (Up ? (k[i - 1] > k[i]) : (k[i - 1] < k[i])) return false;
  return true;
}

static long g_cases = 0, g_failed = 0;

template <bool Combined, bool Up, typename K, typename... Ps>
static void test_case(Dist d, std::size_t n, unsigned seed) {
  std::mt19937 gen(seed);
  const std::vector<K> orig = make_keys<K>(n, d, gen);
  std::vector<K> keys = orig;
  std::tuple<std::vector<Ps>...> pays{std::vector<Ps>(n)...};
  {
    int c = 0;
    std::apply([&](auto&... p) {
      ((std::transform(orig.begin(), orig.end(), p.begin(), [&](const K& k) {
         return payload_of<K, typename std::decay_t<decltype(p)>::value_type>(k, c); }), c++), ...);
    }, pays);
  }
  if constexpr (Combined) {
    std::vector<DataElement<K, Ps...>> e(n);
    for (std::size_t i = 0; i < n; i++) {
      e[i].key = keys[i];
      if constexpr (sizeof...(Ps) > 0)
        e[i].payloads = std::apply([&](auto&... p) { return std::make_tuple(p[i]...); }, pays);
    }
    radix_sort::sort<Up, radix_sort::BitSorterSIMD, CmpSorterInsertionSort>(16, (SortIndex)n,
                                                                           e.data());
    for (std::size_t i = 0; i < n; i++) {
      keys[i] = e[i].key;
      if constexpr (sizeof...(Ps) > 0)
        std::apply([&](auto&... p) { std::tie(p[i]...) = e[i].payloads; }, pays);
    }
  } else if (seed % 3 == 0) {
    // the radixSort.hpp spelling (plain BitSorterSIMD), :1761-1768
    std::apply([&](auto&... p) {
      radix_sort::sort<Up, radix_sort::BitSorterSIMD, CmpSorterInsertionSort>(
          16, (SortIndex)n, keys.data(), p.data()...);
    }, pays);
  } else if (seed % 3 == 1) {
    // the harness adapter's shape (src/sort_methods.hpp:77-97) with the
    // src/radix_sort.hpp:109 spelling BitSorterSIMD<false>
    std::apply([&](auto&... p) {
      srs_test::RadixMethod<radix_sort::BitSorterSIMD<false>, CmpSorterInsertionSort>::
          template sort<Up>((SortIndex)n, keys.data(), p.data()...);
    }, pays);
  } else {
    // the defaulted thresholded form, radixSort.hpp:1761-1763
    std::apply([&](auto&... p) {
      radix_sort::sort<Up>(16, (SortIndex)n, keys.data(), p.data()...);
    }, pays);
  }
  std::string err;
  if (!is_sorted_dir<Up>(keys)) err += "not sorted; ";
  bool pay_ok = true;
  {
    int c = 0;
    std::apply([&](auto&... p) {
      ((pay_ok &= [&] {
          using P = typename std::decay_t<decltype(p)>::value_type;
          for (std::size_t i = 0; i < n; i++) {
            const P want = payload_of<K, P>(keys[i], c);
            if (std::memcmp(&want, &p[i], sizeof(P)) != 0) return false;
          }
          return true;
        }(), c++), ...);
    }, pays);
  }
  if (!pay_ok) err += "payloads are not ok; ";
  if (!same_key_multiset(keys, orig)) err += "key multiset changed; ";
  g_cases++;
  if (!err.empty()) {
    g_failed++;
    std::printf("Testing: %s", tname<K>());
    ((std::printf("-%s", tname<Ps>())), ...);
    std::printf(", %s, Distribution: %s, Up: %d, n=%zu: FAILED: %s\n",
                Combined ? "Combined" : "Separate", dist_name(d), (int)Up, n, err.c_str());
  }
}

template <bool Combined, bool Up, typename K, typename... Ps>
static void all_dists(std::size_t n, unsigned seed) {
  if constexpr (Combined && !is_power_of_two<sizeof(DataElement<K, Ps...>)>) {
    return;  // src/test.cpp:81-82
  } else if constexpr (Combined && sizeof(DataElement<K, Ps...>) > 64) {
    return;
  } else {
    for (int d = 0; d < 8; d++) test_case<Combined, Up, K, Ps...>((Dist)d, n, seed + d);
  }
}

using u8 = uint8_t;
template <bool Combined, bool Up, typename K>
static void all_payloads(std::size_t n, unsigned seed) {  // src/test.cpp:100-153
  all_dists<Combined, Up, K>(n, seed);
  all_dists<Combined, Up, K, uint8_t>(n, seed);
  all_dists<Combined, Up, K, uint16_t>(n, seed);
  all_dists<Combined, Up, K, uint32_t>(n, seed);
  all_dists<Combined, Up, K, uint64_t>(n, seed);
  all_dists<Combined, Up, K, uint64_t, uint8_t>(n, seed);
  all_dists<Combined, Up, K, uint64_t, uint64_t>(n, seed);
  all_dists<Combined, Up, K, uint64_t, uint64_t, uint64_t>(n, seed);
  all_dists<Combined, Up, K, uint64_t, uint64_t, uint64_t, uint64_t, uint64_t, uint64_t,
            uint64_t>(n, seed);
  all_dists<Combined, Up, K, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8,
            u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8,
            u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8,
            u8, u8, u8, u8>(n, seed);
  all_dists<Combined, Up, K, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8,
            u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8>(n, seed);
  all_dists<Combined, Up, K, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8, u8>(n, seed);
  all_dists<Combined, Up, K, u8, u8, u8, u8, u8, u8, u8>(n, seed);
  all_dists<Combined, Up, K, u8, u8, u8>(n, seed);
}

template <bool Combined, bool Up>
static void all_types(std::size_t n, unsigned seed) {  // src/test.cpp:155-169
  all_payloads<Combined, Up, uint8_t>(n, seed);
  all_payloads<Combined, Up, int8_t>(n, seed);
  all_payloads<Combined, Up, uint16_t>(n, seed);
  all_payloads<Combined, Up, int16_t>(n, seed);
  all_payloads<Combined, Up, uint32_t>(n, seed);
  all_payloads<Combined, Up, int32_t>(n, seed);
  all_payloads<Combined, Up, uint64_t>(n, seed);
  all_payloads<Combined, Up, int64_t>(n, seed);
  all_payloads<Combined, Up, float>(n, seed);
  all_payloads<Combined, Up, double>(n, seed);
}

// CmpSorterNoSort through the header (src/cmp_sorters.hpp:66-78): leaves of
// <= thresh elements stay in partition order, so the output splits into
// consecutive runs of <= thresh elements, each holding exactly the keys a
// full sort puts there, and the payloads stay with their keys.
template <typename K>
static bool nosort_case(std::size_t n, SortIndex thresh, unsigned seed) {
  std::mt19937 gen(seed);
  std::vector<K> keys = make_keys<K>(n, Dist::Uniform, gen);
  const std::vector<K> orig = keys;
  std::vector<uint64_t> pay(n);
  for (std::size_t i = 0; i < n; i++) pay[i] = payload_of<K, uint64_t>(keys[i], 0);
  srs_test::RadixMethod<radix_sort::BitSorterSIMD<false>, CmpSorterNoSort>::sortThresh(
      thresh, (SortIndex)n, keys.data(), pay.data());
  std::vector<K> sorted = orig;
  std::sort(sorted.begin(), sorted.end());
  // leaf boundaries: every key before a cut is <= every key after it
  std::vector<K> suffix_min(n + 1);
  for (std::size_t i = n; i-- > 0;) suffix_min[i] = i + 1 < n ? std::min(keys[i], suffix_min[i + 1]) : keys[i];
  K prefix_max = keys[0];
  std::size_t last_cut = 0;
  bool ok = same_key_multiset(keys, orig), unsorted = false;
  for (std::size_t i = 1; i <= n && ok; i++) {
    if (i < n) unsorted |= keys[i] < keys[i - 1];
    if (i == n || !(suffix_min[i] < prefix_max)) {  // a cut before i
      ok &= (SortIndex)(i - last_cut) <= thresh;
      last_cut = i;
    }
    if (i < n) prefix_max = std::max(prefix_max, keys[i]);
  }
  for (std::size_t i = 0; i < n && ok; i++) ok &= pay[i] == payload_of<K, uint64_t>(keys[i], 0);
  // (n > thresh and uniform integer keys: some leaf must be left unsorted;
  // uniform floats put half a segment under one exponent, a bucket the local
  // pass must rank, so their leaves may all come back sorted, which also
  // meets the guarantee)
  if constexpr (std::is_integral_v<K>) ok &= unsorted || n <= (std::size_t)thresh;
  g_cases++;
  if (!ok) {
    g_failed++;
    std::printf("Testing: %s, CmpSorterNoSort, thresh %ld, n=%zu: FAILED\n", tname<K>(),
                (long)thresh, n);
  }
  return ok;
}

int main(int argc, char** argv) {
  const std::size_t max_num = argc > 1 ? std::stoul(argv[1]) : 100000;
  const unsigned seed = argc > 2 ? (unsigned)std::stoul(argv[2]) : 42u;
  {
    const long before = g_failed;
    for (std::size_t n : {10000ul, 300000ul})
      for (SortIndex t : {16, 64}) {
        nosort_case<uint64_t>(n, t, seed);
        nosort_case<int32_t>(n, t, seed + 1);
        nosort_case<double>(n, t, seed + 2);
      }
    std::printf("Testing CmpSorterNoSort leaves: %s\n", g_failed == before ? "passed" : "FAILED");
  }
  for (std::size_t n = 1; n <= max_num; n *= 10) {
    const long before = g_failed;
    // (a progress line per quarter: at n = 1e6 a quarter takes about a minute)
    all_types<false, true>(n, seed);
    std::printf("  n=%zu: separate, up done\n", n);
    std::fflush(stdout);
    all_types<false, false>(n, seed);
    std::printf("  n=%zu: separate, down done\n", n);
    std::fflush(stdout);
    all_types<true, true>(n, seed);
    std::printf("  n=%zu: combined, up done\n", n);
    std::fflush(stdout);
    all_types<true, false>(n, seed);
    std::printf("Testing %zu elements: %s\n", n, g_failed == before ? "passed" : "FAILED");
    std::fflush(stdout);
  }
  std::printf("%ld cases, %ld failed\n", g_cases, g_failed);
  if (g_failed == 0) {
    std::printf("All tests passed\n");
    return 0;
  }
  std::printf("Tests failed, see above for details\n");
  return 1;
}
