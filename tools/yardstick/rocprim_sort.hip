// GPU yardstick: rocPRIM's device radix sort on the
// same C1 workload as bench.py (1e9 uint64 keys + uint64 payload,
// key = splitmix64(42*2^32 + i), payload = splitmix64(key)), timed with HIP
// events, double-buffer API (no extra copy), data resident in HBM.
// Not part of the product: a comparison point for DESIGN.md.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

__device__ inline unsigned long long sm64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ void fill(long long n, unsigned long long* k, unsigned long long* p) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned long long key = sm64((42ull << 32) + (unsigned long long)i);
  k[i] = key;
  p[i] = sm64(key);
}

int main(int argc, char** argv) {
  const long long n = argc > 1 ? (long long)std::atof(argv[1]) : 1000000000LL;
  const int steps = argc > 2 ? std::atoi(argv[2]) : 3;
  unsigned long long *k0, *p0, *k1, *p1;
  CHECK(hipMalloc(&k0, n * 8));
  CHECK(hipMalloc(&p0, n * 8));
  CHECK(hipMalloc(&k1, n * 8));
  CHECK(hipMalloc(&p1, n * 8));
  rocprim::double_buffer<unsigned long long> kb(k0, k1), pb(p0, p1);
  size_t tmp_bytes = 0;
  CHECK(rocprim::radix_sort_pairs(nullptr, tmp_bytes, kb, pb, n));
  void* tmp = nullptr;
  CHECK(hipMalloc(&tmp, tmp_bytes));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  float best = 1e30f, total = 0.f;
  for (int s = 0; s <= steps; s++) {  // step 0 = warmup
    fill<<<(unsigned)((n + 255) / 256), 256>>>(n, k0, p0);
    rocprim::double_buffer<unsigned long long> kk(k0, k1), pp(p0, p1);
    CHECK(hipEventRecord(a));
    CHECK(rocprim::radix_sort_pairs(tmp, tmp_bytes, kk, pp, n));
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (s > 0) {
      total += ms;
      best = ms < best ? ms : best;
    }
    if (s == steps) {  // verify the last run
      std::vector<unsigned long long> hk(1 << 20);
      CHECK(hipMemcpy(hk.data(), kk.current(), hk.size() * 8, hipMemcpyDeviceToHost));
      for (size_t i = 1; i < hk.size(); i++)
        if (hk[i - 1] > hk[i]) { std::printf("NOT SORTED\n"); return 1; }
    }
  }
  const double avg = total / steps;
  std::printf("{\"yardstick\": \"rocprim::radix_sort_pairs u64+u64\", \"n\": %lld, "
              "\"avg_ms\": %.3f, \"best_ms\": %.3f, \"gkeys_per_s\": %.3f, \"temp_bytes\": %zu}\n",
              n, avg, best, n / avg / 1e6, tmp_bytes);
  return 0;
}
