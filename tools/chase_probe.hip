// Dependent random-load latency on MI355X: each lane chases a random
// permutation cycle through an array of N u32 (one load per step, the next
// index is the loaded value); 1..8 waves per CU.  Prints ns per step for
// array sizes from 4 MB to 1 GB.  hipcc --offload-arch=gfx950 -O3 chase_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>
#include <algorithm>

__global__ void chase(const uint32_t* __restrict__ a, uint32_t* out, int steps, uint32_t n) {
  uint32_t i = (uint32_t)((blockIdx.x * 2654435761u + threadIdx.x * 40503u) % n);
  for (int s = 0; s < steps; ++s) i = a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = i;
}

int main() {
  for (size_t mb : {4, 24, 193, 1024}) {
    const uint32_t n = (uint32_t)(mb * 1024 * 1024 / 4);
    std::vector<uint32_t> perm(n);
    for (uint32_t k = 0; k < n; ++k) perm[k] = k;
    std::mt19937 g(1);
    std::shuffle(perm.begin(), perm.end(), g);
    std::vector<uint32_t> h(n);
    for (uint32_t k = 0; k < n; ++k) h[perm[k]] = perm[(k + 1) % n];  // one big cycle
    uint32_t *d, *o;
    hipMalloc(&d, (size_t)n * 4);
    hipMalloc(&o, 1 << 24);
    hipMemcpy(d, h.data(), (size_t)n * 4, hipMemcpyHostToDevice);
    for (int waves_per_cu : {1, 4}) {
      const int blocks = 256 * waves_per_cu;
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      for (int steps : {16, 64}) {
        hipLaunchKernelGGL(chase, dim3(blocks), dim3(64), 0, 0, d, o, steps, n);
        hipEventRecord(e0);
        hipLaunchKernelGGL(chase, dim3(blocks), dim3(64), 0, 0, d, o, steps, n);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("array %5zu MB  waves/CU %d  steps %3d  kernel %8.1f us  %7.1f ns/step\n", mb, waves_per_cu, steps,
               ms * 1e3, ms * 1e6 / steps);
      }
    }
    hipFree(d);
    hipFree(o);
  }
  return 0;
}
