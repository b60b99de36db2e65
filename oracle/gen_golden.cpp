// gen_golden.cpp — produces tests/golden/{golden.bin,manifest.json}.
//
// TEST INFRASTRUCTURE ONLY. Compiled (oracle/Makefile target `golden`) against
// the reference's own sources where they lie: /root/reference/src/data.hpp
// (input generators Data<K,Ps...>, src/data.hpp:105-170,364-406, payload = f(key)
// via srand/rand) and /root/reference/src/radix_sort.hpp (the default
// BitSorterSIMD + CmpSorterInsertionSort path). For every case it writes the
// input arrays and the arrays as sorted BY THE REFERENCE. Nothing of the
// reference's source text is stored: only data.
//
// Case families (see tests/golden/README.md):
//   soa   - 10 key types x {up,down} x 8 distributions x packs {[], [u64,u8]}
//           x n in {16, 17, 300}            (the src/test.cpp:101-179 matrix, trimmed)
//   aos   - DataElement<K> for all K plus 5 DataElement<K,Ps...> layouts x
//           {up,down} x 8 distributions x n = 300
//   large - a few n = 12000 cases (multi-level paths)
//   index - payload = original index (NOT a function of the key): pins the
//           reference's exact unstable permutation inside equal-key runs
//   zeros - float/double keys mixing -0.0 and +0.0 around the leaf threshold
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <tuple>
#include <vector>

#include "data.hpp"
#include "radix_sort.hpp"

using namespace simd_sort;

static std::ofstream g_bin;
static uint64_t g_off = 0;
static std::ostringstream g_man;
static int g_cases = 0;

template <typename T> constexpr int kind_of();
template <> constexpr int kind_of<uint8_t>() { return 0; }
template <> constexpr int kind_of<int8_t>() { return 1; }
template <> constexpr int kind_of<uint16_t>() { return 2; }
template <> constexpr int kind_of<int16_t>() { return 3; }
template <> constexpr int kind_of<uint32_t>() { return 4; }
template <> constexpr int kind_of<int32_t>() { return 5; }
template <> constexpr int kind_of<uint64_t>() { return 6; }
template <> constexpr int kind_of<int64_t>() { return 7; }
template <> constexpr int kind_of<float>() { return 8; }
template <> constexpr int kind_of<double>() { return 9; }

static uint64_t put(const void* p, std::size_t bytes) {
  const uint64_t off = g_off;
  g_bin.write((const char*)p, (std::streamsize)bytes);
  g_off += bytes;
  // keep every array 8-byte aligned in the file
  static const char pad[8] = {0};
  const std::size_t r = bytes % 8;
  if (r) {
    g_bin.write(pad, (std::streamsize)(8 - r));
    g_off += 8 - r;
  }
  return off;
}

static void begin_case(const std::string& family, const char* layout, int kind,
                       bool up, const char* dist, std::size_t n, long seed,
                       int thresh) {
  if (g_cases++) g_man << ",\n";
  g_man << "  {\"family\": \"" << family << "\", \"layout\": \"" << layout
        << "\", \"key_kind\": " << kind << ", \"up\": " << (up ? 1 : 0)
        << ", \"dist\": \"" << dist << "\", \"n\": " << n << ", \"seed\": " << seed
        << ", \"thresh\": " << thresh;
}

// The reference's default path: BitSorterSIMD<> / CmpSorterInsertionSort
// (src/radix_sort.hpp:297-312, :334-337) with an explicit threshold.
template <bool Up, typename K, typename... Ps>
void ref_sort(SortIndex thresh, SortIndex num, K* keys, Ps*... payloads) {
  radix_sort::sort<Up, radix_sort::BitSorterSIMD<>, CmpSorterInsertionSort>(
      thresh, num, keys, payloads...);
}

// ---- SoA ------------------------------------------------------------------
template <bool Up, typename K, typename... Ps>
void soa_case(const std::string& family, InputDistribution dist, std::size_t n,
              long seed) {
  Data<K, Ps...> data(n, dist, seed);
  begin_case(family, "soa", kind_of<K>(), Up, inputDistributionToString(dist), n,
             seed, 16);
  g_man << ", \"payload_sizes\": [";
  {
    int i = 0;
    ((g_man << (i++ ? ", " : "") << sizeof(Ps)), ...);
  }
  g_man << "], \"in\": [" << put(data.keys, n * sizeof(K));
  std::apply([&](auto*... p) { ((g_man << ", " << put(p, n * sizeof(*p))), ...); },
             data.payloads);
  std::apply([&](auto*... p) { ref_sort<Up>(16, n, data.keys, p...); },
             data.payloads);
  g_man << "], \"out\": [" << put(data.keys, n * sizeof(K));
  std::apply([&](auto*... p) { ((g_man << ", " << put(p, n * sizeof(*p))), ...); },
             data.payloads);
  g_man << "]}";
}

// ---- AoS ------------------------------------------------------------------
template <bool Up, typename K, typename... Ps>
void aos_case(const std::string& family, InputDistribution dist, std::size_t n,
              long seed) {
  using D = DataElement<K, Ps...>;
  static_assert(is_power_of_two<sizeof(D)>);
  Data<K, Ps...> data(n, dist, seed);
  std::vector<D> elems(n);
  data.convertToSingleArray(elems.data());  // src/data.hpp:332-344
  begin_case(family, "aos", kind_of<K>(), Up, inputDistributionToString(dist), n,
             seed, 16);
  g_man << ", \"elem_size\": " << sizeof(D) << ", \"payload_sizes\": [";
  {
    int i = 0;
    ((g_man << (i++ ? ", " : "") << sizeof(Ps)), ...);
  }
  g_man << "], \"in\": [" << put(elems.data(), n * sizeof(D));
  radix_sort::sort<Up, radix_sort::BitSorterSIMD<>, CmpSorterInsertionSort>(
      16, n, elems.data());
  g_man << "], \"out\": [" << put(elems.data(), n * sizeof(D)) << "]}";
}

// ---- index payloads -------------------------------------------------------
template <bool Up, typename K>
void index_case(InputDistribution dist, std::size_t n, long seed) {
  Data<K> data(n, dist, seed);
  std::vector<uint32_t> idx(n);
  for (std::size_t i = 0; i < n; i++) idx[i] = (uint32_t)i;
  begin_case("index", "soa", kind_of<K>(), Up, inputDistributionToString(dist), n,
             seed, 16);
  g_man << ", \"payload_sizes\": [4], \"in\": [" << put(data.keys, n * sizeof(K))
        << ", " << put(idx.data(), n * 4);
  ref_sort<Up>(16, n, data.keys, idx.data());
  g_man << "], \"out\": [" << put(data.keys, n * sizeof(K)) << ", "
        << put(idx.data(), n * 4) << "]}";
}

template <bool Up>
void index_aos_case(InputDistribution dist, std::size_t n, long seed) {
  using D = DataElement<uint32_t, uint32_t>;
  Data<uint32_t> data(n, dist, seed);
  std::vector<D> elems(n);
  for (std::size_t i = 0; i < n; i++) {
    elems[i].key = data.keys[i];
    std::get<0>(elems[i].payloads) = (uint32_t)i;
  }
  begin_case("index", "aos", kind_of<uint32_t>(), Up,
             inputDistributionToString(dist), n, seed, 16);
  g_man << ", \"elem_size\": 8, \"payload_sizes\": [4], \"in\": ["
        << put(elems.data(), n * sizeof(D));
  radix_sort::sort<Up, radix_sort::BitSorterSIMD<>, CmpSorterInsertionSort>(
      16, n, elems.data());
  g_man << "], \"out\": [" << put(elems.data(), n * sizeof(D)) << "]}";
}

// ---- signed zeros ---------------------------------------------------------
template <bool Up, typename F>
void zeros_case(std::size_t n, long seed) {
  std::vector<F> keys(n);
  std::vector<uint32_t> idx(n);
  std::mt19937 gen(seed);
  for (std::size_t i = 0; i < n; i++) {
    const unsigned r = gen() % 4;
    keys[i] = r == 0 ? F(-0.0) : r == 1 ? F(0.0) : r == 2 ? F(-1.5) : F(2.25);
    idx[i] = (uint32_t)i;
  }
  begin_case("zeros", "soa", kind_of<F>(), Up, "SignedZeros", n, seed, 16);
  g_man << ", \"payload_sizes\": [4], \"in\": [" << put(keys.data(), n * sizeof(F))
        << ", " << put(idx.data(), n * 4);
  ref_sort<Up>(16, n, keys.data(), idx.data());
  g_man << "], \"out\": [" << put(keys.data(), n * sizeof(F)) << ", "
        << put(idx.data(), n * 4) << "]}";
}

static const InputDistribution kDists[] = {
    InputDistribution::Uniform,      InputDistribution::Gaussian,
    InputDistribution::Zero,         InputDistribution::ZeroOne,
    InputDistribution::Sorted,       InputDistribution::ReverseSorted,
    InputDistribution::AlmostSorted, InputDistribution::AlmostReverseSorted};

template <typename K>
void soa_type(long& seed) {
  for (const auto d : kDists)
    for (const std::size_t n : {16, 17, 300}) {
      soa_case<true, K>("soa", d, n, seed++);
      soa_case<false, K>("soa", d, n, seed++);
      soa_case<true, K, uint64_t, uint8_t>("soa", d, n, seed++);
      soa_case<false, K, uint64_t, uint8_t>("soa", d, n, seed++);
    }
}

template <typename K, typename... Ps>
void aos_type(long& seed) {
  for (const auto d : kDists) {
    aos_case<true, K, Ps...>("aos", d, 300, seed++);
    aos_case<false, K, Ps...>("aos", d, 300, seed++);
  }
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "tests/golden";
  g_bin.open(dir + "/golden.bin", std::ios::binary);
  if (!g_bin) {
    std::fprintf(stderr, "cannot open %s/golden.bin\n", dir.c_str());
    return 1;
  }
  long seed = 1000;
  soa_type<uint8_t>(seed);
  soa_type<int8_t>(seed);
  soa_type<uint16_t>(seed);
  soa_type<int16_t>(seed);
  soa_type<uint32_t>(seed);
  soa_type<int32_t>(seed);
  soa_type<uint64_t>(seed);
  soa_type<int64_t>(seed);
  soa_type<float>(seed);
  soa_type<double>(seed);

  aos_type<uint8_t>(seed);
  aos_type<int8_t>(seed);
  aos_type<uint16_t>(seed);
  aos_type<int16_t>(seed);
  aos_type<uint32_t>(seed);
  aos_type<int32_t>(seed);
  aos_type<uint64_t>(seed);
  aos_type<int64_t>(seed);
  aos_type<float>(seed);
  aos_type<double>(seed);
  aos_type<uint64_t, uint64_t>(seed);
  aos_type<uint32_t, uint32_t>(seed);
  aos_type<float, uint32_t>(seed);
  aos_type<int16_t, uint8_t, uint8_t>(seed);
  aos_type<double, uint64_t>(seed);

  soa_case<true, uint64_t, uint64_t>("large", InputDistribution::Uniform, 12000, seed++);
  soa_case<false, uint64_t, uint64_t>("large", InputDistribution::Uniform, 12000, seed++);
  soa_case<true, float, uint32_t, uint32_t>("large", InputDistribution::Uniform, 12000, seed++);
  soa_case<true, int32_t>("large", InputDistribution::Gaussian, 12000, seed++);
  soa_case<true, double, uint64_t>("large", InputDistribution::Gaussian, 12000, seed++);
  aos_case<true, uint64_t, uint64_t>("large", InputDistribution::Uniform, 12000, seed++);

  for (const auto d : {InputDistribution::ZeroOne, InputDistribution::Gaussian,
                       InputDistribution::Uniform})
    for (const std::size_t n : {100, 2000}) {
      index_case<true, uint8_t>(d, n, seed++);
      index_case<false, uint8_t>(d, n, seed++);
      index_case<true, int32_t>(d, n, seed++);
      index_case<false, int32_t>(d, n, seed++);
      index_case<true, uint64_t>(d, n, seed++);
      index_case<false, uint64_t>(d, n, seed++);
      index_case<true, float>(d, n, seed++);
      index_case<false, float>(d, n, seed++);
      index_case<true, double>(d, n, seed++);
      index_case<false, double>(d, n, seed++);
      index_aos_case<true>(d, n, seed++);
      index_aos_case<false>(d, n, seed++);
    }

  for (const std::size_t n : {12, 16, 17, 40}) {
    zeros_case<true, float>(n, seed++);
    zeros_case<false, float>(n, seed++);
    zeros_case<true, double>(n, seed++);
    zeros_case<false, double>(n, seed++);
  }

  g_bin.close();
  std::ofstream man(dir + "/manifest.json");
  man << "{\"generator\": \"oracle/gen_golden.cpp\", \"reference\": "
         "\"jonicho/simd-radix-sort src/radix_sort.hpp BitSorterSIMD<> + "
         "CmpSorterInsertionSort, thresh 16\", \"key_kinds\": [\"u8\", \"i8\", "
         "\"u16\", \"i16\", \"u32\", \"i32\", \"u64\", \"i64\", \"f32\", \"f64\"], "
         "\"bytes\": "
      << g_off << ", \"cases\": [\n"
      << g_man.str() << "\n]}\n";
  std::printf("wrote %d cases, %llu bytes\n", g_cases, (unsigned long long)g_off);
  return 0;
}
