// Measures the GPU-side duration of idle launches (a counter read, then exit)
// for several grid shapes: what an empty expand / deferred pass costs.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_idle(const unsigned* ctr, unsigned* sink) {
  if (*ctr == 0) return;
  sink[blockIdx.x] = 1;
}
__global__ void k_idle_lds(const unsigned* ctr, unsigned* sink) {
  __shared__ int s[270];
  if (*ctr == 0) return;
  s[threadIdx.x % 270] = 1;
  __syncthreads();
  sink[blockIdx.x] = s[(threadIdx.x + 1) % 270];
}

int main() {
  unsigned *ctr, *sink;
  hipMalloc(&ctr, 4);
  hipMemset(ctr, 0, 4);
  hipMalloc(&sink, 1 << 20);
  hipStream_t st;
  hipStreamCreate(&st);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  struct Shape { int blocks, threads, lds; } shapes[] = {
      {1, 64, 0}, {256, 64, 0}, {256, 256, 0}, {1056, 64, 1}, {2048, 256, 1}, {2048, 256, 0}, {8192, 256, 0}};
  for (auto sh : shapes) {
    for (int rep = 0; rep < 2; ++rep) {
      const int N = 200;
      hipEventRecord(a, st);
      for (int k = 0; k < N; ++k) {
        if (sh.lds) hipLaunchKernelGGL(k_idle_lds, dim3(sh.blocks), dim3(sh.threads), 0, st, ctr, sink);
        else hipLaunchKernelGGL(k_idle, dim3(sh.blocks), dim3(sh.threads), 0, st, ctr, sink);
      }
      hipEventRecord(b, st);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      if (rep) printf("blocks %5d threads %4d lds %d: %.2f us per launch (back-to-back)\n", sh.blocks, sh.threads,
                      sh.lds, 1e3 * ms / N);
    }
  }
  return 0;
}
