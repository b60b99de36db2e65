// Cost of a grid barrier on MI355X: one cooperative launch of G workgroups x
// 1024 threads doing K barriers (plus a store each, as the mid-size sort's
// phases do), timed with HIP events over 50 launches, K = 0 and K = 16:
// cooperative groups' grid.sync(), and the grouped barrier of the mid-size
// sort (srs_kernels.hip mid_grid_barrier, restated here).
// build: hipcc -O3 --offload-arch=gfx950 -o grid_sync grid_sync.hip
#include <hip/hip_runtime.h>
#include <hip/hip_cooperative_groups.h>
#include <stdio.h>

namespace cg = cooperative_groups;

__global__ __launch_bounds__(1024) void k_sync(int K, unsigned* buf) {
  cg::grid_group grid = cg::this_grid();
  for (int i = 0; i < K; i++) {
    if (threadIdx.x == 0) buf[blockIdx.x] = i;
    grid.sync();
  }
}

struct alignas(128) Ctr {
  unsigned n;
  unsigned pad[31];
};
struct Bar {
  Ctr group[8];
  Ctr top;
  alignas(128) unsigned long long gen;
};

__device__ void grouped_barrier(Bar* B, int G, unsigned long long target) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const int x = (int)(blockIdx.x & 7);
    const unsigned members = (unsigned)((G - x + 7) / 8);
    const unsigned groups = (unsigned)(G < 8 ? G : 8);
    bool last = false;
    if (__hip_atomic_fetch_add(&B->group[x].n, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
        members - 1) {
      __hip_atomic_store(&B->group[x].n, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_fetch_add(&B->top.n, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
          groups - 1) {
        __hip_atomic_store(&B->top.n, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = true;
      }
    }
    if (last) {
      __hip_atomic_store(&B->gen, target, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      for (uint32_t i = 0;
           __hip_atomic_load(&B->gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target; i++) {
        if (i > (1u << 24)) break;
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __threadfence();
  }
  __syncthreads();
}

__global__ __launch_bounds__(1024) void k_grouped(int K, unsigned* buf, Bar* B,
                                                   unsigned long long base) {
  for (int i = 0; i < K; i++) {
    if (threadIdx.x == 0) buf[blockIdx.x] = i;
    grouped_barrier(B, (int)gridDim.x, base + i + 1);
  }
}

int main() {
  unsigned* buf;
  if (hipMalloc(&buf, 4096 * 4) != hipSuccess) return 1;
  Bar* bar;
  if (hipMalloc(&bar, sizeof(Bar)) != hipSuccess) return 1;
  (void)hipMemset(bar, 0, sizeof(Bar));
  unsigned long long base = 0;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int which = 0; which < 2; which++)
  for (int G : {4, 16, 64, 128, 256}) {
    for (int K : {0, 16}) {
      void* args[] = {&K, &buf};
      void* args2[] = {&K, &buf, &bar, &base};
      float best = 1e9f, tot = 0;
      for (int r = 0; r < 55; r++) {
        (void)hipEventRecord(a, 0);
        const hipError_t e =
            which == 0 ? hipLaunchCooperativeKernel((const void*)k_sync, dim3(G), dim3(1024), args, 0, 0)
                       : hipLaunchCooperativeKernel((const void*)k_grouped, dim3(G), dim3(1024), args2, 0, 0);
        base += (unsigned long long)K;
        if (e != hipSuccess) {
          printf("G=%d: launch refused\n", G);
          return 1;
        }
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (r >= 5) {
          tot += ms;
          if (ms < best) best = ms;
        }
      }
      printf("%s G=%3d K=%2d: mean %.1f us, min %.1f us per launch\n",
             which == 0 ? "grid.sync" : "grouped  ", G, K, 1000 * tot / 50, 1000 * best);
    }
  }
  return 0;
}
