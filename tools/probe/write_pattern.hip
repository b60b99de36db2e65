// write_pattern.hip — how the placement of a buffer in HBM changes the rate
// of the radix scatter's write pattern (placement study).
//
// A tile (one 256-thread workgroup) writes 32 KB as R runs of 32 KB / R
// bytes; run r of tile i of window w lands at w * W + r * (W / R_BUCKETS)
// + i * run, i.e. R_BUCKETS buckets per window each receiving consecutive
// runs from consecutive tiles, as the scatter's per-digit runs do. Tiles go
// to XCDs in contiguous ranges (as xcd_remap). R = 1 is a sequential write.
// Buffers: 0 hipMalloc, 1 physically contiguous, 2 one VMM handle mapped at
// 1 GiB alignment, 3 VMM 2 MB handles mapped in shuffled order, 4 VMM 2 MB
// handles mapped in order. Prints one line per (mode, pattern): GB/s.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__device__ __forceinline__ int64_t xcd_remap(int64_t bid, int64_t nwg) {
  const int64_t q = nwg / 8, r = nwg % 8, x = bid % 8, l = bid / 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + l;
}

// 256 threads x 8 x 16 B = 32 KB per tile
// bstride: bucket spacing in bytes (0: window / buckets); boff: optional
// per-bucket start offsets (bytes, any 8-byte alignment), replacing r * bstride
__global__ __launch_bounds__(256) void pattern_kernel(char* dst, int64_t window, int runs,
                                                      int buckets, int64_t tiles_per_window,
                                                      int64_t bstride, const int64_t* boff) {
  const int64_t t = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t w = t / tiles_per_window, i = t % tiles_per_window;
  const int run = 32768 / runs;
  if (bstride == 0) bstride = window / buckets;
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = {(uint32_t)t, 1u, 2u, 3u};
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const int off = (k * 256 + (int)threadIdx.x) * 16;  // byte in the tile
    const int r = off / run, o = off % run;
    char* p = dst + w * window + (boff ? boff[r] : (int64_t)r * bstride) + i * run + o;
    if (((uintptr_t)p & 15) == 0) {
      *(u32x4*)p = v;
    } else {  // (8-byte aligned runs: two 8-byte stores)
      ((uint64_t*)p)[0] = v[0];
      ((uint64_t*)p)[1] = v[1];
    }
  }
}

struct Buf {
  char* p = nullptr;
  size_t bytes = 0;
  int mode = 0;
  std::vector<hipMemGenericAllocationHandle_t> h;
  size_t chunk = 0;
};

Buf alloc(size_t bytes, int mode) {
  Buf b;
  b.bytes = bytes;
  b.mode = mode;
  if (mode == 0) {
    CK(hipMalloc((void**)&b.p, bytes));
    return b;
  }
  if (mode == 1) {
    CK(hipExtMallocWithFlags((void**)&b.p, bytes, hipDeviceMallocContiguous));
    return b;
  }
  int dev = 0;
  CK(hipGetDevice(&dev));
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = dev;
  size_t gran = 0;
  CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
  b.chunk = mode == 2 ? bytes : std::max<size_t>(gran, size_t(2) << 20);
  const size_t n = (bytes + b.chunk - 1) / b.chunk;
  CK(hipMemAddressReserve((void**)&b.p, n * b.chunk, size_t(1) << 30, nullptr, 0));
  std::vector<size_t> slot(n);
  for (size_t k = 0; k < n; k++) slot[k] = k;
  if (mode == 3) std::shuffle(slot.begin(), slot.end(), std::mt19937_64(12345));
  b.h.resize(n);
  for (size_t k = 0; k < n; k++) {
    CK(hipMemCreate(&b.h[k], b.chunk, &prop, 0));
    CK(hipMemMap(b.p + slot[k] * b.chunk, b.chunk, 0, b.h[k], 0));
  }
  hipMemAccessDesc a = {};
  a.location = prop.location;
  a.flags = hipMemAccessFlagsProtReadWrite;
  CK(hipMemSetAccess(b.p, n * b.chunk, &a, 1));
  return b;
}

void release(Buf& b) {
  if (b.mode <= 1) {
    CK(hipFree(b.p));
    return;
  }
  const size_t n = b.h.size();
  CK(hipMemUnmap(b.p, n * b.chunk));
  for (auto& h : b.h) CK(hipMemRelease(h));
  CK(hipMemAddressFree(b.p, n * b.chunk));
}

int main(int argc, char** argv) {
  const size_t bytes = argc > 1 ? strtoull(argv[1], nullptr, 10) << 20 : size_t(8) << 30;
  const char* modes = argc > 2 ? argv[2] : "0,1,2,3,4";
  struct Pat {
    const char* name;
    int64_t window;
    int runs, buckets;
    int64_t bstride;  // 0: window / buckets; -1: random 8-byte-aligned bucket starts
  };
  // C1's levels: 16 MB windows (2 M keys x 8 B), 512 buckets, 64-byte runs
  const int64_t W = int64_t(32) << 20;  // (room for spacing 32 KB + delta)
  const Pat pats[] = {
      {"seq", W, 1, 1, 0},
      {"s32K_r64", W, 512, 512, 32768},
      {"s32K+8_r64", W, 512, 512, 32768 + 8},
      {"s32K+16_r64", W, 512, 512, 32768 + 16},
      {"s32K+32_r64", W, 512, 512, 32768 + 32},
      {"s32K+64_r64", W, 512, 512, 32768 + 64},
      {"s32K+128_r64", W, 512, 512, 32768 + 128},
      {"s32K+256_r64", W, 512, 512, 32768 + 256},
      {"s32K+8_r128", W, 256, 256, 65536 + 8},
      {"s32K+8_r256", W, 128, 128, 131072 + 8},
      {"rand8_r64", W, 512, 512, -1},
      {"rand64_r64", W, 512, 512, -64},
      {"rand128_r64", W, 512, 512, -128},
      {"s30.5K_r64", W, 512, 512, 31250},
  };
  int64_t* d_off = nullptr;
  CK(hipMalloc((void**)&d_off, 512 * 8));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (const char* m = modes; *m; m++) {
    if (*m < '0' || *m > '9') continue;
    const int mode = *m - '0';
    Buf buf = alloc(bytes, mode);
    for (const Pat& p : pats) {
      const int64_t windows = (int64_t)(bytes / p.window);
      // tiles per window: every bucket's runs stay inside the window
      const int64_t span = p.bstride > 0 ? p.bstride : p.window / p.buckets;
      int64_t tpw = std::min<int64_t>(p.window / 32768, span / (32768 / p.runs));
      if (p.bstride < 0) tpw /= 2;  // (random starts: half of each bucket's span is jitter)
      const int64_t tiles = windows * tpw;
      const int64_t* boff = nullptr;
      if (p.bstride < 0) {  // random starts, sorted, aligned to -bstride bytes
        std::mt19937_64 g(7);
        std::vector<int64_t> o(512);
        const int64_t al = -p.bstride;
        const int64_t room = span - tpw * (32768 / p.runs);  // (buckets never overlap)
        for (int r = 0; r < 512; r++) o[r] = r * span + (int64_t)(g() % (uint64_t)(room / al)) * al;
        CK(hipMemcpy(d_off, o.data(), 512 * 8, hipMemcpyHostToDevice));
        boff = d_off;
      }
      const int64_t bs = p.bstride > 0 ? p.bstride : 0;
      pattern_kernel<<<(unsigned)tiles, 256>>>(buf.p, p.window, p.runs, p.buckets, tpw, bs, boff);
      CK(hipDeviceSynchronize());
      float best = 1e30f, sum = 0;
      const int reps = 5;
      for (int k = 0; k < reps; k++) {
        CK(hipEventRecord(a));
        pattern_kernel<<<(unsigned)tiles, 256>>>(buf.p, p.window, p.runs, p.buckets, tpw, bs, boff);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        best = std::min(best, ms);
        sum += ms;
      }
      const double gb = (double)tiles * 32768 / 1e9;
      printf("mode %d %-18s %8.3f GB  best %7.3f ms  %7.1f GB/s  avg %7.3f ms  base %p\n", mode,
             p.name, gb, best, gb / (best * 1e-3), sum / reps, (void*)buf.p);
      fflush(stdout);
    }
    release(buf);
  }
  return 0;
}
