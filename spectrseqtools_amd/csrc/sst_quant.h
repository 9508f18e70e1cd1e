// sst_quant.h -- the reference's window quantisation on the device, shared by
// the kernel sources of libsstgpu.so (not part of the public ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sst {

// Reference quantisation, mass_explanation.py:107,110-114: target =
// rint(mass / prec) (Python round(x, 0): ties-to-even) and thr = ceil(t / prec)
// on the IEEE f64 quotient (no fast-math).  The quotient is taken as
// mass * (1/prec), within 2.5 ulp of the exact one; the correctly rounded
// division runs only when that product lies within 2^-50 (relative) of a
// point where rint / ceil change value, so the integers are exactly the
// reference's.
__device__ __forceinline__ double rint_quot(double num, double den, double rden) {
  const double q = num * rden;
  const double f = q - __builtin_floor(q);
  if (!(__builtin_fabs(q) < 0x1p40) || __builtin_fabs(f - 0.5) <= __builtin_fabs(q) * 0x1p-50)
    return __builtin_rint(num / den);
  return __builtin_rint(q);
}
__device__ __forceinline__ double ceil_quot(double num, double den, double rden) {
  if (num == 0.0) return 0.0;
  const double q = num * rden;
  if (!(__builtin_fabs(q) < 0x1p40) || __builtin_fabs(q - __builtin_rint(q)) <= __builtin_fabs(q) * 0x1p-50)
    return __builtin_ceil(num / den);
  return __builtin_ceil(q);
}
// window [lo, hi] as exact f64 integers (|values| < 2^53)
__device__ __forceinline__ void quantise_f(double mass, double thr_abs, bool thr_none, double tol, double prec,
                                           double rprec, double& lo, double& hi) {
  const double t = thr_none ? tol * mass : thr_abs;
  const double target = rint_quot(mass, prec, rprec);
  const double th = ceil_quot(t, prec, rprec);
  lo = target - th;
  hi = target + th;
}
__device__ __forceinline__ void quantise(double mass, double thr_abs, bool thr_none, double tol, double prec,
                                         double rprec, int64_t& lo, int64_t& hi) {
  const double t = thr_none ? tol * mass : thr_abs;
  const int64_t target = (int64_t)rint_quot(mass, prec, rprec);
  const int64_t th = (int64_t)ceil_quot(t, prec, rprec);
  lo = target - th;
  hi = target + th;
}

}  // namespace sst
