// sst_reach.hip -- per-row reachability of reduced alphabets (gfx950), for
// compute_sequence_length_bound after the skeleton's alphabet reduction
// (skeleton_building.py:315-336, mass_table.py:343-487).
//
//   k_reach_rows   one workgroup per spectrum: for each kept row k (ascending
//                  full-table rows r_0 < r_1 < ...) the bitset R_k over masses
//                  [0, 32 W): m is a sum of kept rows r_0..r_k.  These are the
//                  rebuilt reduced table's pairs (pair(r_k, m) != 0 <=> m in
//                  R_k; bit0 <=> m in R_{k-1}; bit1 <=> m - w_k in R_k,
//                  mass_table.py:207-248) -- what the length bound's replay
//                  must see: on the full table with a row mask, a left branch
//                  into a mass that only dropped rows reach returns its default
//                  (-1 for "upper") and counts as 0, so the masked
//                  walk is exact for "lower" only.
//
// R_k = R_{k-1} closed under + w_k: R_k[x] = R_{k-1}[x] | R_k[x - w_k], a
// recurrence of distance w_k >= w_min (every alphabet keeps C).  Words are
// produced in segments of at most q = floor(w_k / 32) words, so a segment
// reads only words of earlier segments, kept in an LDS ring (2^15 words >=
// segment + q + 1 for every row mass < 2^20); R_{k-1} is read back from HBM
// (the row just written, L2-resident), R_k streamed out.  HBM-bound: 8 B
// per word and row (read the previous row, write this one).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sst_internal.h"

namespace sst {

namespace {
constexpr int kReachWG = 1024;
constexpr int kReachRing = 1 << 15;  // words (128 KB)
constexpr int kReachRingMask = kReachRing - 1;
constexpr int kReachILP = 4;  // words per thread whose loads are in flight together
}  // namespace

__global__ __launch_bounds__(kReachWG) void k_reach_rows(ReachArgs a) {
  __shared__ uint32_t ring[kReachRing];
  for (int64_t g = blockIdx.x; g < a.n_spec; g += gridDim.x) {
    const uint64_t m0 = a.alpha[2 * g], m1 = a.alpha[2 * g + 1];
    const int64_t W = a.words[g];
    uint32_t* out = a.bits + a.off[g];
    int k = 0;
    for (int r = 1; r < a.n_rows; ++r) {
      if (!(r < 64 ? (m0 >> r) & 1ull : (m1 >> (r - 64)) & 1ull)) continue;
      const int64_t w = a.w[r];
      const int64_t q = w >> 5;
      const int sh = (int)(w & 31);
      const int64_t seg = q < kReachRing - q - 1 ? q : kReachRing - q - 1;
      const uint32_t* prev = k ? out + (int64_t)(k - 1) * W : nullptr;
      uint32_t* cur = out + (int64_t)k * W;
      for (int64_t s = 0; s < W; s += seg) {
        const int64_t e = s + seg < W ? s + seg : W;
        // kReachILP words per thread per step, their R_{k-1} loads issued
        // together (a segment's words only read the ring's earlier segments,
        // so they are independent of each other)
        for (int64_t j0w = s + threadIdx.x; j0w < e; j0w += (int64_t)kReachILP * blockDim.x) {
          uint32_t pv[kReachILP];
#pragma unroll
          for (int u = 0; u < kReachILP; ++u) {
            const int64_t j = j0w + (int64_t)u * blockDim.x;
            // R_{-1} = {0}: the sentinel row; R_{k-1} was written by this
            // workgroup's previous pass: read at device scope (from L2)
            pv[u] = j < e ? (prev ? __hip_atomic_load(prev + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                  : (j == 0 ? 1u : 0u))
                          : 0u;
          }
#pragma unroll
          for (int u = 0; u < kReachILP; ++u) {
            const int64_t j = j0w + (int64_t)u * blockDim.x;
            if (j >= e) break;
            const int64_t j0 = j - q, j1 = j - q - 1;
            uint32_t sft = 0;
            if (j0 >= 0) sft = ring[j0 & kReachRingMask] << sh;
            if (sh && j1 >= 0) sft |= ring[j1 & kReachRingMask] >> (32 - sh);
            const uint32_t v = pv[u] | sft;
            ring[j & kReachRingMask] = v;
            cur[j] = v;
          }
        }
        __syncthreads();
      }
      ++k;
    }
    __syncthreads();
  }
}

hipError_t launch_reach_rows(const ReachArgs& a, int n_wg, hipStream_t st) {
  if (a.n_spec <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_reach_rows, dim3(n_wg), dim3(kReachWG), 0, st, a);
  return hipGetLastError();
}

}  // namespace sst
