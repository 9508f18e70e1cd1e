// VALU issue cost of the instruction kinds the scan kernel's quantisation
// uses (gfx950): every thread runs 8 independent chains of one opcode in
// inline asm, 256 CUs x 8 waves/SIMD; reported as cycles per wave64
// instruction per SIMD (clock from s_memtime / s_memrealtime).
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 2048

#define KERNEL(NAME, ASM)                                                                                \
  __global__ __launch_bounds__(256) void NAME(double* out, double seed) {                               \
    double a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,      \
           a6 = a0 + 6, a7 = a0 + 7;                                                                     \
    for (int i = 0; i < ITERS; ++i) {                                                                    \
      asm volatile(ASM " %0, %0\n" ASM " %1, %1\n" ASM " %2, %2\n" ASM " %3, %3\n" ASM " %4, %4\n" ASM    \
                       " %5, %5\n" ASM " %6, %6\n" ASM " %7, %7\n"                                       \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));    \
    }                                                                                                    \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;                  \
  }

KERNEL(k_rndne, "v_rndne_f64")
KERNEL(k_ceil, "v_ceil_f64")
KERNEL(k_fract, "v_fract_f64")

#define KERNEL2(NAME, ASM)                                                                               \
  __global__ __launch_bounds__(256) void NAME(double* out, double seed) {                               \
    double a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,      \
           a6 = a0 + 6, a7 = a0 + 7;                                                                     \
    for (int i = 0; i < ITERS; ++i) {                                                                    \
      asm volatile(ASM " %0, %0, %0\n" ASM " %1, %1, %1\n" ASM " %2, %2, %2\n" ASM " %3, %3, %3\n" ASM    \
                       " %4, %4, %4\n" ASM " %5, %5, %5\n" ASM " %6, %6, %6\n" ASM " %7, %7, %7\n"        \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));    \
    }                                                                                                    \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;                  \
  }
KERNEL2(k_mul, "v_mul_f64")
KERNEL2(k_add, "v_add_f64")

__global__ __launch_bounds__(256) void k_u32(double* out, double seed) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
           a7 = a0 + 7;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_add_u32 %0, %0, %0\nv_add_u32 %1, %1, %1\nv_add_u32 %2, %2, %2\nv_add_u32 %3, %3, %3\n"
        "v_add_u32 %4, %4, %4\nv_add_u32 %5, %5, %5\nv_add_u32 %6, %6, %6\nv_add_u32 %7, %7, %7\n"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

__global__ __launch_bounds__(256) void k_cvt(double* out, double seed) {
  double a0 = seed + threadIdx.x;
  unsigned u0 = 0, u1 = 0, u2 = 0, u3 = 0, u4 = 0, u5 = 0, u6 = 0, u7 = 0;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_cvt_u32_f64 %0, %8\nv_cvt_u32_f64 %1, %8\nv_cvt_u32_f64 %2, %8\nv_cvt_u32_f64 %3, %8\n"
        "v_cvt_u32_f64 %4, %8\nv_cvt_u32_f64 %5, %8\nv_cvt_u32_f64 %6, %8\nv_cvt_u32_f64 %7, %8\n"
        : "=v"(u0), "=v"(u1), "=v"(u2), "=v"(u3), "=v"(u4), "=v"(u5), "=v"(u6), "=v"(u7)
        : "v"(a0));
    a0 += 1.0;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = u0 + u1 + u2 + u3 + u4 + u5 + u6 + u7;
}

__global__ void k_clock(long long* o) {
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  long long t = t0;
  while (__builtin_amdgcn_s_memrealtime() - r0 < 1000000) t = __builtin_amdgcn_s_memtime();
  o[0] = t - t0;
  o[1] = __builtin_amdgcn_s_memrealtime() - r0;
}

typedef void (*KFn)(double*, double);

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const int blocks = cus * 8;  // 256 threads = 4 waves/block -> 8 waves per SIMD
  double* out;
  hipMalloc(&out, (size_t)blocks * 256 * sizeof(double));
  long long* clk;
  hipMalloc(&clk, 16);
  hipLaunchKernelGGL(k_clock, 1, 1, 0, 0, clk);
  long long hc[2];
  hipMemcpy(hc, clk, 16, hipMemcpyDeviceToHost);
  const double ghz = (double)hc[0] / hc[1] * 0.1;  // memrealtime = 100 MHz
  printf("{\"cus\": %d, \"clock_ghz\": %.3f", cus, ghz);
  struct {
    const char* name;
    KFn fn;
  } ks[] = {{"v_mul_f64", k_mul}, {"v_add_f64", k_add},   {"v_rndne_f64", k_rndne}, {"v_ceil_f64", k_ceil},
            {"v_fract_f64", k_fract}, {"v_cvt_u32_f64", k_cvt}, {"v_add_u32", k_u32}};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.fn, blocks, 256, 0, 0, out, 1.5);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k.fn, blocks, 256, 0, 0, out, 1.5);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    // wave-instructions per SIMD per launch
    const double winst = (double)blocks * 4 * ITERS * 8 / (cus * 4);
    const double cyc = ms / 5 * 1e-3 * ghz * 1e9 / winst;
    printf(", \"%s\": %.2f", k.name, cyc);
  }
  printf("}\n");
  return 0;
}
