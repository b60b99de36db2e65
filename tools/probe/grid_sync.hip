// Cost of a cooperative-groups grid barrier on MI355X: one cooperative
// launch of G workgroups x 1024 threads doing K grid.sync() calls (plus a
// store each, as the mid-size sort's phases do), timed with HIP events over
// 50 launches, K = 0 and K = 16.
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

int main() {
  unsigned* buf;
  if (hipMalloc(&buf, 4096 * 4) != hipSuccess) return 1;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int G : {4, 16, 64, 128, 256}) {
    for (int K : {0, 16}) {
      void* args[] = {&K, &buf};
      float best = 1e9f, tot = 0;
      for (int r = 0; r < 55; r++) {
        (void)hipEventRecord(a, 0);
        if (hipLaunchCooperativeKernel((const void*)k_sync, dim3(G), dim3(1024), args, 0, 0) !=
            hipSuccess) {
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
      printf("G=%3d K=%2d: mean %.1f us, min %.1f us per launch\n", G, K, 1000 * tot / 50,
             1000 * best);
    }
  }
  return 0;
}
