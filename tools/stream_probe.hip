// Streaming floor of the scan's input pattern (gfx950): two f64 arrays of n
// queries (mass, thr) read once, one status byte per query written, persistent
// grid of 1024-lane workgroups, 2 per CU.  Variants:
//   v8   : one query per lane, 8-B nontemporal loads, 1-B stores (the scan today)
//   v16  : two queries per lane, 16-B nontemporal loads, 2-B stores
//   v16p : as v16 with plain loads
//   v8p  : as v8 with plain loads
// Prints the average launch time (HIP events) per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef double dbl2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int8_t classify(double m, double t) {
  const double q = m * 1000.0, th = t * 1000.0;
  return (int8_t)((q - th) < (q + th) ? ((int)q & 3) : 0);
}

template <bool NT>
__global__ __launch_bounds__(1024, 8) void k_v8(const double* __restrict__ mass, const double* __restrict__ thr,
                                                 uint32_t n, int8_t* __restrict__ st) {
  const uint32_t nw = gridDim.x * 16, w = blockIdx.x * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t ntiles = (n + 63) >> 6;
  auto ld = [&](uint32_t tl, double& m, double& t) {
    const uint32_t j = min(tl * 64 + lane, n - 1);
    if (NT) {
      m = __builtin_nontemporal_load(mass + j);
      t = __builtin_nontemporal_load(thr + j);
    } else {
      m = mass[j];
      t = thr[j];
    }
  };
  double mA, tA, mB, tB;
  ld(w, mA, tA);
  ld(w + nw, mB, tB);
  for (uint32_t tile = w; tile < ntiles; tile += 2 * nw) {
    uint32_t i = tile * 64 + lane;
    if (i < n) st[i] = classify(mA, tA);
    ld(tile + 2 * nw, mA, tA);
    if (tile + nw >= ntiles) break;
    i += nw * 64;
    if (i < n) st[i] = classify(mB, tB);
    ld(tile + 3 * nw, mB, tB);
  }
}

template <bool NT>
__global__ __launch_bounds__(1024, 8) void k_v16(const double* __restrict__ mass, const double* __restrict__ thr,
                                                  uint32_t n, int8_t* __restrict__ st) {
  const uint32_t nw = gridDim.x * 16, w = blockIdx.x * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t ntiles = (n + 127) >> 7;  // 128 queries per tile (n even here)
  auto ld = [&](uint32_t tl, dbl2& m, dbl2& t) {
    const uint32_t j = min(tl * 64 + lane, n / 2 - 1);
    if (NT) {
      m = __builtin_nontemporal_load((const dbl2*)mass + j);
      t = __builtin_nontemporal_load((const dbl2*)thr + j);
    } else {
      m = ((const dbl2*)mass)[j];
      t = ((const dbl2*)thr)[j];
    }
  };
  dbl2 mA, tA;
  ld(w, mA, tA);
  for (uint32_t tile = w; tile < ntiles; tile += nw) {
    const uint32_t i = tile * 64 + lane;
    const int8_t s0 = classify(mA.x, tA.x), s1 = classify(mA.y, tA.y);
    if (i < n / 2) ((uint16_t*)st)[i] = (uint16_t)((uint8_t)s0 | ((uint16_t)(uint8_t)s1 << 8));
    ld(tile + nw, mA, tA);
  }
}

int main() {
  const uint32_t n = 10711326 & ~1u;
  std::vector<double> h(n);
  for (uint32_t i = 0; i < n; ++i) h[i] = 300.0 + (i % 7919) * 0.37;
  double *m, *t;
  int8_t* st;
  hipMalloc(&m, n * 8ull);
  hipMalloc(&t, n * 8ull);
  hipMalloc(&st, n);
  hipMemcpy(m, h.data(), n * 8ull, hipMemcpyHostToDevice);
  hipMemcpy(t, h.data(), n * 8ull, hipMemcpyHostToDevice);
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int grid = p.multiProcessorCount * 2;
  // flush buffer: evicts the inputs from the MALL between launches
  char* flush;
  const size_t fb = 1ull << 30;
  hipMalloc(&flush, fb);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"v8_nt", "v8_plain", "v16_nt", "v16_plain"};
  printf("{\"n\": %u", n);
  for (int v = 0; v < 4; ++v) {
    float tot = 0;
    for (int r = 0; r < 6; ++r) {
      hipMemsetAsync(flush, r, fb);
      hipEventRecord(e0);
      if (v == 0) hipLaunchKernelGGL(k_v8<true>, grid, 1024, 0, 0, m, t, n, st);
      if (v == 1) hipLaunchKernelGGL(k_v8<false>, grid, 1024, 0, 0, m, t, n, st);
      if (v == 2) hipLaunchKernelGGL(k_v16<true>, grid, 1024, 0, 0, m, t, n, st);
      if (v == 3) hipLaunchKernelGGL(k_v16<false>, grid, 1024, 0, 0, m, t, n, st);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (r) tot += ms;
    }
    printf(", \"%s_us\": %.1f", names[v], tot / 5 * 1e3);
  }
  printf("}\n");
  return 0;
}
