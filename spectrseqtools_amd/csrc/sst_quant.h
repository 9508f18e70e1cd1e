// sst_quant.h -- the reference's window quantisation and is_valid window test
// on the device, shared by the kernel sources of libsstgpu.so (not part of
// the public ABI).
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

// Window of one query as exact f64 integers: target = rint(mass / prec) and
// thr = ceil(thr_abs / prec) (mass_explanation.py:107,110-114).  Both
// quotients are taken as x * (1/prec), within 2.5 ulp of the exact one; the
// correctly rounded division runs only when a product lies within 2^-50
// (relative) of a point where rint / ceil change value, or is huge, so the
// integers are exactly the reference's.  Straight-line except for that rare
// fallback (the lean form of rint_quot / ceil_quot).
__device__ __forceinline__ void quantise_lean(double m, double t, double prec, double rprec, double& lof,
                                              double& hif) {
  const double qm = m * rprec, qt = t * rprec;
  double rm = __builtin_rint(qm), ct = __builtin_ceil(qt);
  const double dm = qm - rm, dt = qt - __builtin_rint(qt);  // exact
  const bool slow = !(__builtin_fabs(qm) < 0x1p40) | !(__builtin_fabs(qt) < 0x1p40) |
                    (0.5 - __builtin_fabs(dm) <= __builtin_fabs(qm) * 0x1p-50) |
                    (__builtin_fabs(dt) <= __builtin_fabs(qt) * 0x1p-50);
  if (__builtin_expect(slow, 0)) {
    rm = __builtin_rint(m / prec);
    ct = __builtin_ceil(t / prec);
  }
  lof = rm - ct;
  hif = rm + ct;
}

// any bit of valid in [a, b] (a <= b, both < limit)
__device__ __forceinline__ bool any_bits(const uint64_t* valid, int64_t a, int64_t b) {
  int64_t wa = a >> 6, wb = b >> 6;
  for (int64_t wi = wa; wi <= wb; ++wi) {
    uint64_t x = valid[wi];
    if (wi == wa) x &= ~0ull << (a & 63);
    if (wi == wb) x &= ~0ull >> (63 - (b & 63));
    if (x) return true;
  }
  return false;
}
__device__ __forceinline__ int count_bits(const uint64_t* valid, int64_t a, int64_t b) {
  int64_t wa = a >> 6, wb = b >> 6;
  int c = 0;
  for (int64_t wi = wa; wi <= wb; ++wi) {
    uint64_t x = valid[wi];
    if (wi == wa) x &= ~0ull << (a & 63);
    if (wi == wb) x &= ~0ull >> (63 - (b & 63));
    c += __builtin_popcountll(x);
  }
  return c;
}

// is_valid_mass semantics (mass_explanation.py:63-88): ascending scan, skip
// v <= 0, raise at the first v >= limit, True at the first reachable v.
__device__ __forceinline__ int8_t valid_window(const uint64_t* valid, int64_t limit, int64_t lo, int64_t hi,
                                               int64_t full_lo = 1, int64_t full_hi = 1, int64_t first_reach = 0) {
  if (hi < lo) return 0;
  int64_t a = lo < 1 ? 1 : lo;
  if (a > hi) return 0;
  int64_t b = hi < limit - 1 ? hi : limit - 1;
  if (a <= b && b >= full_lo && a < full_hi) return 1;  // meets the all-reachable run: no bitset load
  if (a <= b && b >= first_reach && any_bits(valid, a, b)) return 1;  // below first_reach: nothing reachable
  return hi >= limit ? (int8_t)-1 : (int8_t)0;
}

// block-wide exclusive prefix sum of one value per thread (blockDim a multiple of 64, <= 1024)
__device__ __forceinline__ uint32_t block_excl(uint32_t v, uint32_t* s_w, uint32_t& total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) s_w[wv] = incl;
  __syncthreads();
  uint32_t base = 0, tot = 0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
    const uint32_t x = s_w[w];
    if (w < wv) base += x;
    tot += x;
  }
  __syncthreads();
  total = tot;
  return base + incl - v;
}

}  // namespace sst
