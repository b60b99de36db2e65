// host_copy.hip — PCIe copy options for the host-pointer drop-in path.
// Measures, for one GB-sized pageable host array:
//   1. hipMemcpy pageable H2D / D2H (the runtime's own staging);
//   2. hipHostRegister of the array (cost per GB), then H2D / D2H from it;
//   3. chunked staging through pinned bounce buffers, T host threads copying
//      each chunk into (out of) a pinned buffer while the DMA of the previous
//      chunk runs (T = 1, 2, 4, 8, 16).
// usage: host_copy [GB=4] [chunk MB=64]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s -> %s\n", #x, hipGetErrorString(e));                 \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

static void par_memcpy(char* dst, const char* src, size_t n, int T) {
  if (T <= 1) {
    std::memcpy(dst, src, n);
    return;
  }
  std::vector<std::thread> th;
  const size_t per = (n / T + 4095) / 4096 * 4096;
  for (int t = 0; t < T; t++) {
    const size_t a = std::min(n, per * t), b = std::min(n, per * (t + 1));
    if (a < b) th.emplace_back([=] { std::memcpy(dst + a, src + a, b - a); });
  }
  for (auto& x : th) x.join();
}

int main(int argc, char** argv) {
  const double gb = argc > 1 ? atof(argv[1]) : 4.0;
  const size_t chunk = (size_t)(argc > 2 ? atof(argv[2]) : 64.0) << 20;
  const size_t n = (size_t)(gb * (1ull << 30));
  char* host = (char*)aligned_alloc(4096, n);
  char* host2 = (char*)aligned_alloc(4096, n);
  std::memset(host, 1, n);
  std::memset(host2, 2, n);
  char* dev = nullptr;
  CK(hipMalloc(&dev, n));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));

  // 1. pageable
  for (int rep = 0; rep < 2; rep++) {
    double t0 = now();
    CK(hipMemcpy(dev, host, n, hipMemcpyHostToDevice));
    double t1 = now();
    CK(hipMemcpy(host2, dev, n, hipMemcpyDeviceToHost));
    double t2 = now();
    std::printf("pageable  H2D %6.1f GB/s  D2H %6.1f GB/s\n", n / (t1 - t0) / 1e9,
                n / (t2 - t1) / 1e9);
  }
  // 2. register
  {
    double t0 = now();
    CK(hipHostRegister(host, n, hipHostRegisterDefault));
    double t1 = now();
    CK(hipHostRegister(host2, n, hipHostRegisterDefault));
    double t2 = now();
    std::printf("hipHostRegister %.3f s + %.3f s for %.1f GB each (%.1f GB/s)\n", t1 - t0,
                t2 - t1, n / 1e9, 2 * n / (t2 - t0) / 1e9);
    for (int rep = 0; rep < 2; rep++) {
      double a = now();
      CK(hipMemcpyAsync(dev, host, n, hipMemcpyHostToDevice, st));
      CK(hipStreamSynchronize(st));
      double b = now();
      CK(hipMemcpyAsync(host2, dev, n, hipMemcpyDeviceToHost, st));
      CK(hipStreamSynchronize(st));
      double c = now();
      std::printf("registered H2D %6.1f GB/s  D2H %6.1f GB/s\n", n / (b - a) / 1e9,
                  n / (c - b) / 1e9);
    }
    double u0 = now();
    CK(hipHostUnregister(host));
    CK(hipHostUnregister(host2));
    std::printf("hipHostUnregister %.3f s\n", now() - u0);
  }
  // 3. pinned staging, NB bounce buffers
  const int NB = 3;
  char* pin[NB];
  hipEvent_t ev[NB];
  for (int i = 0; i < NB; i++) {
    CK(hipHostMalloc((void**)&pin[i], chunk, hipHostMallocDefault));
    CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
  }
  const size_t nch = (n + chunk - 1) / chunk;
  for (int T : {1, 2, 4, 8, 16}) {
    // H2D: memcpy chunk i into pin[i % NB] (after its previous DMA), DMA it
    double t0 = now();
    for (size_t i = 0; i < nch; i++) {
      const size_t a = i * chunk, len = std::min(chunk, n - a);
      const int b = (int)(i % NB);
      if (i >= NB) CK(hipEventSynchronize(ev[b]));
      par_memcpy(pin[b], host + a, len, T);
      CK(hipMemcpyAsync(dev + a, pin[b], len, hipMemcpyHostToDevice, st));
      CK(hipEventRecord(ev[b], st));
    }
    CK(hipStreamSynchronize(st));
    double t1 = now();
    // D2H: DMA chunk i into pin[i % NB]; memcpy out once it landed
    for (size_t i = 0; i < nch + NB; i++) {
      if (i >= NB) {  // drain chunk i - NB
        const size_t j = i - NB, a = j * chunk, len = std::min(chunk, n - a);
        const int b = (int)(j % NB);
        CK(hipEventSynchronize(ev[b]));
        par_memcpy(host2 + a, pin[b], len, T);
      }
      if (i < nch) {
        const size_t a = i * chunk, len = std::min(chunk, n - a);
        const int b = (int)(i % NB);
        CK(hipMemcpyAsync(pin[b], dev + a, len, hipMemcpyDeviceToHost, st));
        CK(hipEventRecord(ev[b], st));
      }
    }
    double t2 = now();
    std::printf("staged T=%2d H2D %6.1f GB/s  D2H %6.1f GB/s  (chunk %zu MB)\n", T,
                n / (t1 - t0) / 1e9, n / (t2 - t1) / 1e9, chunk >> 20);
  }
  // raw pinned DMA rate (the staging ceiling)
  {
    double t0 = now();
    for (size_t i = 0; i < nch; i++) {
      const size_t a = i * chunk, len = std::min(chunk, n - a);
      CK(hipMemcpyAsync(dev + a, pin[i % NB], len, hipMemcpyHostToDevice, st));
    }
    CK(hipStreamSynchronize(st));
    double t1 = now();
    for (size_t i = 0; i < nch; i++) {
      const size_t a = i * chunk, len = std::min(chunk, n - a);
      CK(hipMemcpyAsync(pin[i % NB], dev + a, len, hipMemcpyDeviceToHost, st));
    }
    CK(hipStreamSynchronize(st));
    double t2 = now();
    std::printf("pinned DMA only H2D %6.1f GB/s  D2H %6.1f GB/s\n", n / (t1 - t0) / 1e9,
                n / (t2 - t1) / 1e9);
  }
  std::printf("host threads available: %u\n", std::thread::hardware_concurrency());
  return 0;
}
