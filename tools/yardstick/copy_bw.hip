// Read+write ceiling on this GPU: copy 16 GB with different access widths
// and cache hints (calibration for DESIGN.md; not part of the product).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::printf("%s\n", hipGetErrorString(e_)); std::exit(1); } } while (0)

template <typename T, int UNROLL, bool NT>
__global__ __launch_bounds__(256) void copy_k(const T* __restrict__ a, T* __restrict__ b, long long n) {
  long long i = ((long long)blockIdx.x * 256 * UNROLL) + threadIdx.x;
  T v[UNROLL];
#pragma unroll
  for (int u = 0; u < UNROLL; u++) {
    long long j = i + (long long)u * 256;
    if (j < n) v[u] = NT ? __builtin_nontemporal_load(a + j) : a[j];
  }
#pragma unroll
  for (int u = 0; u < UNROLL; u++) {
    long long j = i + (long long)u * 256;
    if (j < n) {
      if (NT) __builtin_nontemporal_store(v[u], b + j); else b[j] = v[u];
    }
  }
}

template <typename T, int UNROLL, bool NT>
void run(const char* name, void* a, void* b, size_t bytes) {
  long long n = bytes / sizeof(T);
  unsigned grid = (unsigned)((n + 256LL * UNROLL - 1) / (256LL * UNROLL));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  copy_k<T, UNROLL, NT><<<grid, 256>>>((const T*)a, (T*)b, n);
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < 5; r++) copy_k<T, UNROLL, NT><<<grid, 256>>>((const T*)a, (T*)b, n);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  ms /= 5;
  std::printf("%-28s %7.3f ms  %5.2f TB/s (read+write)\n", name, ms, 2.0 * bytes / ms / 1e9);
}

int main() {
  size_t bytes = 16ull << 30;
  void *a, *b;
  CHECK(hipMalloc(&a, bytes)); CHECK(hipMalloc(&b, bytes));
  CHECK(hipMemset(a, 1, bytes)); CHECK(hipMemset(b, 0, bytes));
  run<unsigned long long, 4, false>("8B/lane x4", a, b, bytes);
  run<unsigned long long, 8, false>("8B/lane x8", a, b, bytes);
  run<v4u, 2, false>("16B/lane x2", a, b, bytes);
  run<v4u, 4, false>("16B/lane x4", a, b, bytes);
  run<v4u, 8, false>("16B/lane x8", a, b, bytes);
  run<unsigned long long, 4, true>("8B/lane x4 nontemporal", a, b, bytes);
  run<v4u, 4, true>("16B/lane x4 nontemporal", a, b, bytes);
  return 0;
}
