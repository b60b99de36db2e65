// Probe: do same-address LDS atomics of one wave instruction return their
// pre-op values in lane order? (a stable multisplit rank needs exactly that)
// usage: ./lds_atomic_order  -> prints violations per pattern
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

// mode 0: 32-bit counters, mode 1: 16-bit halves packed in 32-bit words
template <int MODE>
__global__ __launch_bounds__(1024) void probe(int nbins, int iters, uint32_t seed,
                                              unsigned long long* bad, unsigned long long* checks) {
  __shared__ uint32_t cnt[16][512];
  __shared__ uint32_t got[1024];
  __shared__ uint32_t dig[1024];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned long long nbad = 0, nchk = 0;
  for (int it = 0; it < iters; it++) {
    for (int i = threadIdx.x; i < 16 * 512; i += 1024) (&cnt[0][0])[i] = 0;
    __syncthreads();
    const uint32_t d = mix(seed ^ (blockIdx.x * 7919u) ^ (it * 104729u) ^ threadIdx.x * 2654435761u) % nbins;
    uint32_t r;
    if (MODE == 0) {
      r = atomicAdd(&cnt[wave][d], 1u);
    } else {
      const uint32_t sh = (d & 1) << 4;
      r = (atomicAdd(&cnt[wave][d >> 1], 1u << sh) >> sh) & 0xFFFFu;
    }
    got[threadIdx.x] = r;
    dig[threadIdx.x] = d;
    __syncthreads();
    // lane l: count lanes below with the same digit; must equal r
    uint32_t below = 0;
    for (int j = 0; j < lane; j++) below += dig[wave * 64 + j] == d;
    nbad += below != r;
    nchk++;
    __syncthreads();
  }
  atomicAdd(bad, nbad);
  atomicAdd(checks, nchk);
}

int main() {
  unsigned long long *bad, *chk;
  hipMalloc(&bad, 8); hipMalloc(&chk, 8);
  const int bins[] = {1, 2, 8, 64, 512};
  for (int mode = 0; mode < 2; mode++)
    for (int b : bins) {
      hipMemset(bad, 0, 8); hipMemset(chk, 0, 8);
      if (mode == 0) probe<0><<<2048, 1024>>>(b, 64, 12345u + b, bad, chk);
      else probe<1><<<2048, 1024>>>(b, 64, 777u + b, bad, chk);
      unsigned long long hb = 0, hc = 0;
      hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
      hipMemcpy(&hc, chk, 8, hipMemcpyDeviceToHost);
      printf("mode %d bins %3d: %llu of %llu ranks out of lane order\n", mode, b, hb, hc);
    }
  return 0;
}
