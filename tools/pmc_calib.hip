// pmc_calib.hip -- calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE for the access
// widths of the explain/is_valid kernels (MI355X_MICROARCH.md: widths other
// than 16 B/lane are uncalibrated).  Each kernel moves a known byte count over
// buffers larger than the 256 MiB Infinity Cache.
//   k_read8   8 B/lane coalesced f64 loads (mass / thr inputs)
//   k_write1  1 B/lane coalesced stores    (status / is_valid results)
//   k_write8  8 B/lane coalesced stores    (count / offset)
// build: hipcc --offload-arch=gfx950 -O3 -o tools/pmc_calib tools/pmc_calib.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void k_read8(const double* __restrict__ x, int64_t n, double* __restrict__ out) {
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    s += x[i];
  if (s == 12345.678) out[0] = s;  // keeps the loads alive; never true for the zeroed input
}
__global__ void k_write1(int8_t* __restrict__ y, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = (int8_t)(i & 3);
}
__global__ void k_write8(uint64_t* __restrict__ y, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = (uint64_t)i;
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main() {
  const int64_t n = 1ll << 26;  // 64 Mi elements: 512 MB of f64, 64 MB of i8
  double *x, *out;
  int8_t* y1;
  uint64_t* y8;
  CK(hipMalloc(&x, n * 8));
  CK(hipMalloc(&out, 8));
  CK(hipMalloc(&y1, n));
  CK(hipMalloc(&y8, n * 8));
  CK(hipMemset(x, 0, n * 8));
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_read8, dim3(8192), dim3(256), 0, 0, x, n, out);
    hipLaunchKernelGGL(k_write1, dim3(8192), dim3(256), 0, 0, y1, n);
    hipLaunchKernelGGL(k_write8, dim3(8192), dim3(256), 0, 0, y8, n);
  }
  CK(hipDeviceSynchronize());
  printf("{\"k_read8\": %lld, \"k_write1\": %lld, \"k_write8\": %lld}\n", (long long)(n * 8), (long long)n,
         (long long)(n * 8));
  CK(hipFree(x));
  CK(hipFree(out));
  CK(hipFree(y1));
  CK(hipFree(y8));
  return 0;
}
