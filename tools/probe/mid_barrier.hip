// Cost of the mid-size launch's grid barrier (srs_kernels.hip
// mid_grid_barrier: sense reversal on a central counter) per barrier, for
// G = 64 / 128 / 256 resident workgroups (one per CU: 100 KB of LDS each):
//   mode 0: agent-scope fences around the arrival (the product)
//   mode 1: no fences (atomics only; not a valid barrier for data)
//   mode 2: mode 0, each workgroup first writes 64 KB (dirty L2 lines for the
//           release write-back, as after the launch's scatter phase)
// usage: mid_barrier   (prints one line per (mode, G))
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(1024) void bar_kernel(unsigned* bar, int iters, int mode,
                                                   unsigned long long* junk) {
  __shared__ unsigned pad[25600];  // (100 KB: one workgroup per CU)
  pad[threadIdx.x] = threadIdx.x;
  for (int it = 0; it < iters; it++) {
    if (mode == 2)
      for (int i = threadIdx.x; i < 8192; i += 1024)
        junk[(size_t)blockIdx.x * 8192 + i] = it + i + pad[threadIdx.x & 1023];
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned* cnt = bar;
      unsigned* gen = bar + 32;
      const unsigned g0 = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (mode != 1) __threadfence();
      else __builtin_amdgcn_s_waitcnt(0);
      const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == gridDim.x - 1) {
        __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (mode != 1) __threadfence();
        __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g0)
          __builtin_amdgcn_s_sleep(2);
      }
      if (mode != 1) __threadfence();
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && pad[5] == 12345) bar[64] = 1;
}

int main() {
  unsigned* bar;
  unsigned long long* junk;
  hipMalloc(&bar, 4096);
  hipMemset(bar, 0, 4096);
  hipMalloc(&junk, (size_t)256 * 8192 * 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 200;
  for (int mode = 0; mode < 3; mode++)
    for (int G : {8, 64, 128, 256}) {
      bar_kernel<<<G, 1024>>>(bar, 10, mode, junk);  // warm
      hipEventRecord(a);
      bar_kernel<<<G, 1024>>>(bar, iters, mode, junk);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms0 = 0;
      hipEventElapsedTime(&ms0, a, b);
      hipEventRecord(a);
      bar_kernel<<<G, 1024>>>(bar, 0, mode, junk);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms1 = 0;
      hipEventElapsedTime(&ms1, a, b);
      printf("mode %d G %3d: %.2f us per barrier (empty launch %.1f us)\n", mode, G,
             (ms0 - ms1) * 1e3 / iters, ms1 * 1e3);
    }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
