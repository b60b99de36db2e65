// count_probe.hip — what bounds the radix count pass ("count
// pass"): 1e9 keys read in 4096-key tiles, one tile per 256-thread workgroup
// (the product's shape), each tile's 512-bin LDS histogram flushed as a row
// of u16. Variants take one cost away or change one knob at a time:
//   read      the loads alone (xor-reduced)
//   count     loads + digit + LDS atomic + row flush (the product's inner loop)
//   count_s2  the same into two LDS sub-histograms (waves 0,1 / 2,3)
//   atom      the atomics and flush alone (keys hashed in registers, no loads)
//   persist   resident workgroups (8 per CU) looping over tiles, next tile's
//             loads in flight while the current one is counted
//   count_m   count with 2 dependent metadata loads in front of the key loads
//             (tile -> segment, segment -> plan), as the product's gathered level
// usage: ./count_probe [keys (default 1e9)]  -> one line per (key width, variant)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int NT = 256, TILE = 4096, ITEMS = TILE / NT, BINS = 512;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t sm64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ int64_t xcd_remap(int64_t bid, int64_t nwg) {
  const int64_t q = nwg / 8, r = nwg % 8, x = bid % 8, l = bid / 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + l;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

template <typename K>
__global__ void fill_kernel(K* k, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    k[i] = (K)sm64((uint64_t)i);
}

template <typename K>
__device__ __forceinline__ void load_tile(const K* keys, int64_t n, int64_t t, K (&raw)[ITEMS],
                                          int64_t shift = 0) {
  constexpr int PER = 16 / sizeof(K);
  const int64_t base = t * TILE + shift;
  const int64_t rem = n - base;
  const uint32_t bytes = rem >= TILE ? TILE * sizeof(K) : (uint32_t)(rem * sizeof(K));
  const __amdgpu_buffer_rsrc_t r = rsrc(keys + base, bytes);
  u32x4 c[ITEMS / PER];
#pragma unroll
  for (int j = 0; j < ITEMS / PER; j++)
    c[j] = __builtin_amdgcn_raw_buffer_load_b128(r, (threadIdx.x + (uint32_t)j * NT) * 16u, 0, 0);
#pragma unroll
  for (int k = 0; k < ITEMS; k++) {
    const u32x4 v = c[k / PER];
    if constexpr (sizeof(K) == 8)
      raw[k] = (K)((uint64_t)v[2 * (k % PER)] | ((uint64_t)v[2 * (k % PER) + 1] << 32));
    else
      raw[k] = (K)v[k % PER];
  }
}

__device__ const void* g_ptrs[2];

template <typename K>
__device__ __forceinline__ uint32_t digit(K k) {
  return (uint32_t)(k >> (sizeof(K) * 8 - 9)) & (BINS - 1);
}

template <typename K>
__global__ __launch_bounds__(NT) void read_kernel(const K* keys, int64_t n, uint32_t* sink) {
  const int64_t t = xcd_remap(blockIdx.x, gridDim.x);
  K raw[ITEMS];
  load_tile(keys, n, t, raw);
  K x = 0;
#pragma unroll
  for (int k = 0; k < ITEMS; k++) x ^= raw[k];
  if ((uint32_t)x == 0x12345678u) sink[threadIdx.x] = (uint32_t)x;
}

template <int NSUB, bool ZERO = false>
__device__ __forceinline__ void flush_row(uint32_t (*h)[BINS], uint16_t* hist, int64_t t) {
  uint32_t* row = (uint32_t*)(hist + t * BINS);
  for (uint32_t i = threadIdx.x; i < BINS / 2; i += NT) {
    uint32_t a = 0, b = 0;
#pragma unroll
    for (int s = 0; s < NSUB; s++) {
      a += h[s][2 * i];
      b += h[s][2 * i + 1];
      if (ZERO) h[s][2 * i] = h[s][2 * i + 1] = 0;
    }
    row[i] = a | (b << 16);
  }
}

// MODE 0: keys from memory; 1: keys hashed in registers (no loads);
// 2: two dependent metadata loads before the key loads
template <typename K, int NSUB, int MODE>
__global__ __launch_bounds__(NT) void count_kernel(const K* keys, int64_t n, uint16_t* hist,
                                                   const int32_t* tile_seg, const int64_t* seg_start) {
  __shared__ uint32_t h[NSUB][BINS];
  int64_t t = xcd_remap(blockIdx.x, gridDim.x);
  K raw[ITEMS];
  if constexpr (MODE == 1) {
#pragma unroll
    for (int k = 0; k < ITEMS; k++) raw[k] = (K)sm64((uint64_t)(t * TILE + k * NT + threadIdx.x));
  } else if constexpr (MODE == 2) {
    const int s = tile_seg[t];
    const int64_t tt = seg_start[s] + (t - (int64_t)s * 64);
    load_tile(keys, n, tt, raw);
  } else if constexpr (MODE == 6) {  // the gathered level's chain: order -> tile -> plan -> base, + a reference key
    const int64_t to = (int64_t)tile_seg[t];               // (identity order table)
    const int s = (int)(to / 64);
    const int64_t st = seg_start[s];                        // plan
    const K* kb = (const K*)g_ptrs[st & 1];                 // base pointer (a descriptor load)
    const int64_t tt = st + (to - (int64_t)s * 64);
    load_tile(kb, n, tt, raw);
    const K ref = kb[st * TILE];                            // segment's first key
    raw[0] ^= ref & (K)0;                                   // (used, changes nothing)
  } else if constexpr (MODE == 3) {
    load_tile(keys, n - 1, t, raw, 1);
  } else {
    load_tile(keys, n, t, raw);
  }
  __shared__ uint32_t tab[MODE == 5 ? BINS : 1];
  if constexpr (MODE == 5)
    for (uint32_t i = threadIdx.x; i < BINS; i += NT) tab[i] = (i * 37u) & (BINS - 1);
  for (uint32_t i = threadIdx.x; i < NSUB * BINS; i += NT) (&h[0][0])[i] = 0;
  __syncthreads();
  if constexpr (MODE == 4) {  // float keys: order-preserving flip, varying-bit OR, valid checks
    __shared__ unsigned long long sor;
    if (threadIdx.x == 0) sor = 0;
    __syncthreads();
    const int64_t rem = n - t * TILE;
    const K uref = raw[0] ^ (K)((raw[0] >> (sizeof(K) * 8 - 1)) ? ~(K)0 : (K)1 << (sizeof(K) * 8 - 1));
    K vor = 0;
#pragma unroll
    for (int k = 0; k < ITEMS; k++) {
      constexpr int PER = 16 / sizeof(K);
      const int e = ((k / PER) * NT + (int)threadIdx.x) * PER + k % PER;
      const bool ok = e < rem;
      const K u = raw[k] ^ (K)((raw[k] >> (sizeof(K) * 8 - 1)) ? ~(K)0 : (K)1 << (sizeof(K) * 8 - 1));
      if (ok) vor |= u ^ uref;
      if (ok) atomicAdd(&h[0][digit(u)], 1u);
    }
    if (vor) atomicOr(&sor, (unsigned long long)vor);
    __syncthreads();
    flush_row<NSUB>(h, hist, t);
    if (threadIdx.x == 0 && sor) {  // (the product publishes new varying bits per segment)
      unsigned long long* vo = (unsigned long long*)tile_seg;
      const unsigned long long known = __hip_atomic_load(vo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (sor & ~known) atomicOr(vo, sor);
    }
    return;
  }
  const int sub = NSUB > 1 ? (int)(threadIdx.x / 64) % NSUB : 0;
  const int64_t rem = n - t * TILE;
#pragma unroll
  for (int k = 0; k < ITEMS; k++) {
    const int e = k * NT + (int)threadIdx.x;  // (mapping does not matter for the histogram)
    if constexpr (MODE == 5) {
      if (e < rem) atomicAdd(&h[sub][tab[digit(raw[k])]], 1u);
    } else {
      if (e < rem) atomicAdd(&h[sub][digit(raw[k])], 1u);
    }
  }
  __syncthreads();
  flush_row<NSUB>(h, hist, t);
}

// resident workgroups, each over a contiguous run of tiles, next tile's keys
// loaded before the current one is counted; histograms double-buffered
template <typename K>
__global__ __launch_bounds__(NT) void persist_kernel(const K* keys, int64_t n, uint16_t* hist,
                                                     int64_t ntiles) {
  __shared__ uint32_t h[2][1][BINS];
  const int64_t per = (ntiles + gridDim.x - 1) / gridDim.x;
  const int64_t w = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t t0 = w * per, t1 = std::min<int64_t>(ntiles, t0 + per);
  for (uint32_t i = threadIdx.x; i < 2 * BINS; i += NT) (&h[0][0][0])[i] = 0;
  __syncthreads();
  K ra[ITEMS], rb[ITEMS];
  if (t0 < t1) load_tile(keys, n, t0, ra);
  int cur = 0;
  for (int64_t t = t0; t < t1; t++) {
    if (t + 1 < t1) load_tile(keys, n, t + 1, rb);
    const int64_t rem = n - t * TILE;
#pragma unroll
    for (int k = 0; k < ITEMS; k++) {
      const int e = k * NT + (int)threadIdx.x;
      if (e < rem) atomicAdd(&h[cur][0][digit(ra[k])], 1u);
    }
    __syncthreads();
    flush_row<1, true>(h[cur], hist, t);  // (h[cur] is next added to after the next barrier)
#pragma unroll
    for (int k = 0; k < ITEMS; k++) ra[k] = rb[k];
    cur ^= 1;
  }
}

template <typename K>
void run(const char* kname, int64_t n) {
  K* keys;
  CK(hipMalloc(&keys, n * sizeof(K)));
  const int64_t ntiles = (n + TILE - 1) / TILE;
  uint16_t* hist;
  CK(hipMalloc(&hist, ntiles * BINS * 2));
  uint32_t* sink;
  CK(hipMalloc(&sink, 4096));
  const int64_t nseg = (ntiles + 63) / 64;
  int32_t* tile_seg;
  int64_t* seg_start;
  CK(hipMalloc(&tile_seg, ntiles * 4));
  int32_t* tile_seg_id;
  CK(hipMalloc(&tile_seg_id, ntiles * 4));
  {
    int32_t* id = (int32_t*)malloc(ntiles * 4);
    for (int64_t t = 0; t < ntiles; t++) id[t] = (int32_t)t;
    CK(hipMemcpy(tile_seg_id, id, ntiles * 4, hipMemcpyHostToDevice));
    free(id);
  }
  CK(hipMalloc(&seg_start, nseg * 8));
  {
    int32_t* ts = (int32_t*)malloc(ntiles * 4);
    int64_t* ss = (int64_t*)malloc(nseg * 8);
    for (int64_t t = 0; t < ntiles; t++) ts[t] = (int32_t)(t / 64);
    for (int64_t s = 0; s < nseg; s++) ss[s] = s * 64;
    CK(hipMemcpy(tile_seg, ts, ntiles * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(seg_start, ss, nseg * 8, hipMemcpyHostToDevice));
    free(ts);
    free(ss);
  }
  {
    const void* p2[2] = {keys, keys};
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_ptrs), p2, sizeof p2));
  }
  fill_kernel<K><<<4096, 256>>>(keys, n);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  int cus = 256;
  {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    cus = p.multiProcessorCount;
  }
  const unsigned g = (unsigned)ntiles;
  struct V {
    const char* name;
    int id;
  } vs[] = {{"read", 0},    {"count", 1},   {"count_s2", 2}, {"count_s4", 3},
            {"atom", 4},    {"persist8", 5}, {"persist4", 6}, {"count_m", 7},
            {"count_mis", 8}, {"count_xf", 9}, {"count_tab", 10}, {"count_chain", 11}};
  for (const V& v : vs) {
    auto launch = [&]() {
      switch (v.id) {
        case 0: read_kernel<K><<<g, NT>>>(keys, n, sink); break;
        case 1: count_kernel<K, 1, 0><<<g, NT>>>(keys, n, hist, nullptr, nullptr); break;
        case 2: count_kernel<K, 2, 0><<<g, NT>>>(keys, n, hist, nullptr, nullptr); break;
        case 3: count_kernel<K, 4, 0><<<g, NT>>>(keys, n, hist, nullptr, nullptr); break;
        case 4: count_kernel<K, 1, 1><<<g, NT>>>(keys, n, hist, nullptr, nullptr); break;
        case 5: persist_kernel<K><<<cus * 8, NT>>>(keys, n, hist, ntiles); break;
        case 6: persist_kernel<K><<<cus * 4, NT>>>(keys, n, hist, ntiles); break;
        case 7: count_kernel<K, 1, 2><<<g, NT>>>(keys, n, hist, tile_seg, seg_start); break;
        case 8: count_kernel<K, 1, 3><<<g, NT>>>(keys, n, hist, nullptr, nullptr); break;
        case 9: count_kernel<K, 1, 4><<<g, NT>>>(keys, n, hist, tile_seg, nullptr); break;
        case 10: count_kernel<K, 1, 5><<<g, NT>>>(keys, n, hist, nullptr, nullptr); break;
        case 11: count_kernel<K, 1, 6><<<g, NT>>>(keys, n, hist, tile_seg_id, seg_start); break;
      }
    };
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0;
    const int reps = 6;
    for (int r = 0; r < reps; r++) {
      CK(hipEventRecord(a));
      launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      best = std::min(best, ms);
      sum += ms;
    }
    const double gb = n * (double)sizeof(K) / 1e9;
    printf("%s %-9s n=%lld  best %.3f ms  avg %.3f ms  %.0f GB/s  %.2f keys/clk/CU (2.4 GHz)\n",
           kname, v.name, (long long)n, best, sum / reps, gb / (best * 1e-3),
           n / (best * 1e-3) / 2.4e9 / cus);
    fflush(stdout);
  }
  CK(hipFree(keys));
  CK(hipFree(hist));
  CK(hipFree(sink));
  CK(hipFree(tile_seg));
  CK(hipFree(tile_seg_id));
  CK(hipFree(seg_start));
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? (int64_t)atof(argv[1]) : 1000000000;
  run<uint32_t>("u32", n);
  run<uint64_t>("u64", n);
  return 0;
}
