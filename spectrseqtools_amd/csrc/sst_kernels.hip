// sst_kernels.hip -- HIP kernels of the MI355X mass-explanation engine (gfx950).
//
// Data layout in HBM (one set per table, see DESIGN.md "Data layout"):
//   packed[r][c]  the reference's packed 2-bit table (mass_table.py:207-248),
//                 kept only to hand DynamicProgrammingTable.table back.
//   index[m]      16-B record per integer mass m < M = n_cols*C:
//                   .x = L bits of rows 0..63, .y = rows 64..119 | lo << 56
//                 L bit r = pair(r, m) bit1 ("left": reachable with >= 1 copy
//                 of row r), lo = lowest row whose pair is non-zero (0xFF: none).
//                 For a table produced by the reference recurrence,
//                 pair(r, m) bit0 == (r > lo) for every r, so (L, lo) is the
//                 whole column of the packed table in one aligned load.
//   valid[m/64]   bitset of pair(N-1, m) != 0: what is_valid_mass reads
//                 (mass_explanation.py:62-88); 2.8 MB for the full alphabet,
//                 L2-resident.
//
// The explain DFS (mass_explanation.py:118-188) is run in its chain form:
// from (m, r) the reference walks up rows r, r-1, ... while bit0 is set, then
// takes the left branches of those rows in ascending row order.  With the
// memo keyed on (m, row) and budgets ignored by the key, a node's result is
// fixed by its first visit; every visited set of rows of one mass is the
// contiguous range [lo(m), hv(m)].  Three query classes:
//   SHALLOW/DEEP  budgets provably never bind (fast-path theorem):
//                 enumerate all multisets in the window directly from index.
//   EXACT         budgets may bind: phase 1 replays the memoised DFS over
//                 masses (per-mass high-water row hv, enabled-left mask en,
//                 lowest non-empty row ne, in a per-lane hash), phase 2
//                 enumerates the enabled DAG.
//   NOMEMO        with_memo=False: enumeration carrying (A, B) budgets.
// One lane per query ("64 peaks per wavefront"): the query working set is a
// handful of 16-B index loads, so lane-per-query issues 64x fewer memory
// instructions than wave-per-query; outputs are compacted with a wavefront
// prefix sum and one arena atomic per workgroup.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "sst_internal.h"
#include "sst_quant.h"

namespace sst {

// ---------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------
struct M128 {
  uint64_t a, b;  // rows 0..63, rows 64..119 (bits 56..63 never set here)
};
__device__ __forceinline__ M128 rows_upto(int r) {  // rows 0..r inclusive
  M128 m;
  if (r >= 63) {
    m.a = ~0ull;
    int k = r - 63;  // number of rows in b
    m.b = k >= 64 ? ~0ull : ((1ull << k) - 1ull);
  } else {
    m.a = r < 0 ? 0ull : ((2ull << r) - 1ull);
    m.b = 0;
  }
  return m;
}
__device__ __forceinline__ M128 rows_from(int r) {  // rows r..119
  M128 u = rows_upto(r - 1);
  M128 m;
  m.a = ~u.a;
  m.b = ~u.b & ((1ull << 56) - 1ull);
  return m;
}
__device__ __forceinline__ M128 mand(M128 x, M128 y) { return {x.a & y.a, x.b & y.b}; }
__device__ __forceinline__ bool mzero(M128 x) { return (x.a | x.b) == 0; }
__device__ __forceinline__ int mlow(M128 x) { return x.a ? __builtin_ctzll(x.a) : 64 + __builtin_ctzll(x.b); }
__device__ __forceinline__ M128 mclear(M128 x, int r) {
  if (r < 64) x.a &= ~(1ull << r);
  else x.b &= ~(1ull << (r - 64));
  return x;
}
__device__ __forceinline__ bool mtest(M128 x, int r) { return r < 64 ? (x.a >> r) & 1ull : (x.b >> (r - 64)) & 1ull; }

// tables of <= 64 rows (NW): every mask lives in .a; zeroing .b lets the
// compiler drop the second word from the DFS loop's mask arithmetic
template <bool NW>
__device__ __forceinline__ M128 nrm(M128 x) {
  if (NW) x.b = 0;
  return x;
}
template <bool NW>
__device__ __forceinline__ M128 rows_upto_nw(int r) {
  if (NW) return M128{r >= 63 ? ~0ull : ((2ull << r) - 1ull), 0};
  return rows_upto(r);
}

__device__ __forceinline__ int rec_lo(ulonglong2 rec) { return (int)(rec.y >> 56); }
__device__ __forceinline__ M128 rec_L(ulonglong2 rec) { return {rec.x, rec.y & ((1ull << 56) - 1ull)}; }

__device__ __forceinline__ ulonglong2 ld_index(const ulonglong2* idx, int64_t m) { return idx[m]; }

// ---------------------------------------------------------------------------
// table build: bitsets R_r over masses [0, M), R_r = R_{r-1} closed under +w_r
// ---------------------------------------------------------------------------
__global__ void k_bits_seed(uint64_t* R0, int64_t nwords) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nwords) R0[i] = (i == 0) ? 1ull : 0ull;
}

// dst = src | (src << k) over an nbits-long bitset (bits >= nbits dropped).
__global__ void k_bits_shift_or(uint64_t* __restrict__ dst, const uint64_t* __restrict__ src, int64_t k,
                                int64_t nwords, int64_t nbits) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nwords) return;
  int64_t q = k >> 6;
  int s = (int)(k & 63);
  uint64_t v = src[i];
  int64_t j = i - q;
  if (j >= 0) {
    uint64_t x = src[j] << s;
    if (s && j >= 1) x |= src[j - 1] >> (64 - s);
    v |= x;
  }
  if (i == nwords - 1 && (nbits & 63)) v &= (1ull << (nbits & 63)) - 1ull;
  dst[i] = v;
}

__device__ __forceinline__ uint64_t bits_at(const uint64_t* R, int64_t pos, int n) {
  // n <= 32 bits starting at bit pos (pos >= 0), bit i of result = bit pos+i
  int64_t wi = pos >> 6;
  int s = (int)(pos & 63);
  uint64_t x = R[wi] >> s;
  if (s + n > 64) x |= R[wi + 1] << (64 - s);
  return n == 64 ? x : (x & ((1ull << n) - 1ull));
}
__device__ __forceinline__ uint64_t spread32(uint64_t x) {  // bit i -> bit 2i (x < 2^32)
  x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
  x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
  x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
  x = (x | (x << 2)) & 0x3333333333333333ull;
  x = (x | (x << 1)) & 0x5555555555555555ull;
  return x;
}

template <int C>
__device__ __forceinline__ uint64_t pword_get(const void* p, int64_t o) {
  if (C == 32) return ((const uint64_t*)p)[o];
  if (C == 16) return ((const uint32_t*)p)[o];
  if (C == 8) return ((const uint16_t*)p)[o];
  return ((const uint8_t*)p)[o];
}
template <int C>
__device__ __forceinline__ void pword_set(void* p, int64_t o, uint64_t v) {
  if (C == 32) ((uint64_t*)p)[o] = v;
  else if (C == 16) ((uint32_t*)p)[o] = (uint32_t)v;
  else if (C == 8) ((uint16_t*)p)[o] = (uint16_t)v;
  else ((uint8_t*)p)[o] = (uint8_t)v;
}
template <int C>
__device__ __forceinline__ uint64_t wmask() {
  return C == 32 ? ~0ull : ((1ull << (2 * C)) - 1ull);
}

// Rows whose mass is below C (step == 0) are not a plain closure in the
// reference: its in-place sweep shifts each word once and spills from the
// just-updated word (mass_table.py:230-243).  Those rows are computed
// literally: k_row_init writes the row-init bits (:221-223), one thread runs
// the sweep, k_unpack_any recovers the row's reachability bitset.
template <int C>
__global__ void k_row_init(const uint64_t* __restrict__ Rprev, int64_t ncols, void* __restrict__ row) {
  int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncols) return;
  uint64_t b0 = bits_at(Rprev, c * C, C);
  uint64_t rb0 = (uint64_t)(__builtin_bitreverse32((uint32_t)b0) >> (32 - C));
  pword_set<C>(row, c, spread32(rb0));
}
template <int C>
__global__ void k_row_sweep_literal(void* __restrict__ row, int64_t ncols, int shift) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  uint64_t alt_first = 0;
  for (int k = 0; k < C; ++k) alt_first |= 2ull << (2 * k);
  const uint64_t full = wmask<C>();
  for (int64_t j = 0; j < ncols; ++j) {
    uint64_t x = pword_get<C>(row, j);
    uint64_t y = x >> (2 * shift);
    pword_set<C>(row, j, x | (alt_first & (((y << 1) & full) | y)));
    if (shift != 0 && j + 1 < ncols) {
      x = pword_get<C>(row, j);
      uint64_t z = (x << (2 * (C - shift))) & full;
      pword_set<C>(row, j + 1, pword_get<C>(row, j + 1) | (alt_first & (((z << 1) & full) | z)));
    }
  }
}
template <int C>
__global__ void k_unpack_any(const void* __restrict__ row, int64_t ncols, int64_t rw, uint64_t* __restrict__ R) {
  int64_t wi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // one bitset word = 64 masses
  if (wi >= rw) return;
  uint64_t out = 0;
  for (int k = 0; k < 64; ++k) {
    int64_t m = wi * 64 + k;
    int64_t c = m / C;
    if (c >= ncols) break;
    uint64_t pair = (pword_get<C>(row, c) >> (2 * (C - 1 - (int)(m % C)))) & 3ull;
    if (pair) out |= 1ull << k;
  }
  R[wi] = out;
}

// packed[r][c] from bitsets (row 0: pair(0,0) = 3, the init 0xC0.. word),
// last column masked with the reference's formula (mass_table.py:246).
// Rows flagged `literal` were written by k_row_sweep_literal: mask only.
template <int C>
__global__ void k_pack(const uint64_t* __restrict__ R, int64_t rw, int n_rows, const int64_t* __restrict__ w,
                       int64_t ncols, int64_t M, uint64_t last_mask, const uint8_t* __restrict__ literal,
                       void* __restrict__ out) {
  int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int r = blockIdx.y;
  if (c >= ncols) return;
  if (literal[r]) {
    if (c == ncols - 1) {
      int64_t o = (int64_t)r * ncols + c;
      pword_set<C>(out, o, pword_get<C>(out, o) & last_mask);
    }
    return;
  }
  int64_t m0 = c * C;
  uint64_t b0, b1;
  if (r == 0) {
    b0 = b1 = (m0 == 0) ? 1ull : 0ull;
  } else {
    const uint64_t* Rp = R + (int64_t)(r - 1) * rw;
    const uint64_t* Rr = R + (int64_t)r * rw;
    b0 = bits_at(Rp, m0, C);
    int64_t wr = w[r];
    // b1 bit k = R_r(m0 + k - w_r) for m0 + k >= w_r
    int64_t s = m0 - wr;
    if (s >= 0) {
      b1 = bits_at(Rr, s, C);
    } else if (s > -C) {
      b1 = bits_at(Rr, 0, C) << (-s);
      b1 &= (C == 64) ? ~0ull : ((1ull << C) - 1ull);
    } else {
      b1 = 0;
    }
  }
  // mass k of the word sits at bits 2*(C-1-k): reverse the C-bit fields
  uint64_t rb0 = (uint64_t)(__builtin_bitreverse32((uint32_t)b0) >> (32 - C));
  uint64_t rb1 = (uint64_t)(__builtin_bitreverse32((uint32_t)b1) >> (32 - C));
  uint64_t word = spread32(rb0) | (spread32(rb1) << 1);
  if (c == ncols - 1) word &= last_mask;
  int64_t o = (int64_t)r * ncols + c;
  if (C == 32) ((uint64_t*)out)[o] = word;
  else if (C == 16) ((uint32_t*)out)[o] = (uint32_t)word;
  else if (C == 8) ((uint16_t*)out)[o] = (uint16_t)word;
  else ((uint8_t*)out)[o] = (uint8_t)word;
}

// index + valid bitset from a packed table of any compression; flags tables
// that violate bit0(r, m) == (some row < r has pair != 0).
template <int C>
__global__ void k_index(const void* __restrict__ packed, int n_rows, int64_t ncols, int64_t M,
                        ulonglong2* __restrict__ index, uint64_t* __restrict__ valid, int* __restrict__ err) {
  int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool in = m < M;
  int64_t mm = in ? m : 0;
  int64_t c = mm / C;
  int sh = 2 * (C - 1 - (int)(mm % C));
  uint64_t L0 = 0, L1 = 0;
  int lo = 0xFF;
  bool bad = false;
  int pair = 0;
  for (int r = 0; r < n_rows; ++r) {
    int64_t o = (int64_t)r * ncols + c;
    uint64_t word;
    if (C == 32) word = ((const uint64_t*)packed)[o];
    else if (C == 16) word = ((const uint32_t*)packed)[o];
    else if (C == 8) word = ((const uint16_t*)packed)[o];
    else word = ((const uint8_t*)packed)[o];
    pair = (int)((word >> sh) & 3ull);
    if (r >= 1 && (pair & 1) != (lo != 0xFF ? 1 : 0)) bad = true;
    if (pair && lo == 0xFF) lo = r;
    if (pair & 2) {
      if (r < 64) L0 |= 1ull << r;
      else L1 |= 1ull << (r - 64);
    }
  }
  if (in) {
    index[m] = make_ulonglong2(L0, L1 | ((uint64_t)lo << 56));
    if (bad) atomicOr(err, 1);
  }
  // one wave = 64 consecutive masses = one valid word
  uint64_t bal = __ballot(in && pair != 0);
  if ((threadIdx.x & 63) == 0 && m < M) valid[m >> 6] = bal;
}

// ---------------------------------------------------------------------------
// is_valid batch
// ---------------------------------------------------------------------------
// is_valid_mass (mass_explanation.py:45-89), one query per lane.  Windows
// meeting the all-reachable run or lying wholly below the first reachable
// mass need no bitset word; most others are decided by their first word
// (the rest scan on with an early exit): about one scattered L2 load per
// query.  (Measured alternatives, all slower: a persistent grid with the next
// tile's inputs in flight -- with and without the bitset load ordered ahead
// of the prefetch --, and 4 queries per lane with independent word loads.
// The kernel is bound by its dependent load chain per wave, and a fresh wave
// per tile overlaps those chains best.)
template <bool THR>
__global__ __launch_bounds__(256) void k_is_valid(ValidArgs v) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= (uint32_t)v.n) return;
  const double m = v.mass[i];
  const double t = THR ? v.thr[i] : v.tol * m;
  double lof, hif;
  quantise_lean(m, t, v.prec, v.rprec, lof, hif);
  // ascending scan of the window (:63-88): skip v <= 0, True at the first
  // reachable v, raise at the first v >= limit
  const double af = __builtin_fmax(lof, 1.0);
  const bool act = lof <= hif && af <= hif;
  const double bf = __builtin_fmin(hif, (double)(v.limit - 1));
  const bool inr = act && af <= bf;  // the window meets [1, limit)
  const bool full = inr && bf >= (double)v.full_lo && af < (double)v.full_hi;
  bool hit = full;
  if (inr && !full && bf >= (double)v.first_reach) hit = any_bits(v.valid, (uint32_t)af, (uint32_t)bf);
  v.out[i] = hit ? (int8_t)1 : (act && hif >= (double)v.limit ? (int8_t)-1 : (int8_t)0);
}

// is_valid_mass over peaks x breakage weights, as classify_fragments issues
// it (fragment_classification.py:39-67): su = obs - shift[k] (shift[k] =
// breakage weight x precision, the host's f64 product), threshold = tolerance
// x obs; out[k * n + p], breakage-major like the reference's pl.concat.  One
// lane per peak: the peak's mass is read once (8 B instead of 16 B per
// query) and its NW windows are quantised together, so their bitset loads
// are in flight at once.
template <int NW>
__device__ __forceinline__ void is_valid_peak(const ValidArgs& v, const PeakShifts& sh, const uint32_t p) {
  if (p >= (uint32_t)v.n) return;
  const double obs = __builtin_nontemporal_load(v.mass + p);
  const double t = v.tol * obs;
  const double bmax = (double)(v.limit - 1);
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    double lof, hif;
    quantise_lean(obs - sh.shift[k], t, v.prec, v.rprec, lof, hif);
    const double af = __builtin_fmax(lof, 1.0);
    const bool act = lof <= hif && af <= hif;
    const double bf = __builtin_fmin(hif, bmax);
    const bool inr = act && af <= bf;
    const bool full = inr && bf >= (double)v.full_lo && af < (double)v.full_hi;
    bool hit = full;
    if (inr && !full && bf >= (double)v.first_reach) hit = any_bits(v.valid, (uint32_t)af, (uint32_t)bf);
    v.out[(size_t)k * v.n + p] = hit ? (int8_t)1 : (act && hif >= (double)v.limit ? (int8_t)-1 : (int8_t)0);
  }
}
template <int NW>
__global__ __launch_bounds__(256) void k_is_valid_peaks(ValidArgs v, PeakShifts sh) {
  is_valid_peak<NW>(v, sh, blockIdx.x * 256 + threadIdx.x);
}

// ---------------------------------------------------------------------------
// is_singleton (fragment_classification.py:104-119): some value of the
// quantised window equals one of `masses` (the caller's integer masses, the
// table's rows incl. the sentinel 0 in classify_fragments :73-80).  Sorted,
// de-duplicated masses in LDS; one binary search per window.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_is_singleton(const int64_t* __restrict__ masses, int n_masses,
                                                      const double* __restrict__ mass,
                                                      const double* __restrict__ thr, int64_t n, double tol,
                                                      double prec, double rprec, int8_t* __restrict__ out) {
  __shared__ int64_t sm[kMaxSingletonMasses];
  for (int k = threadIdx.x; k < n_masses; k += blockDim.x) sm[k] = masses[k];
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t lo, hi;
  quantise(mass[i], thr ? thr[i] : 0.0, thr == nullptr, tol, prec, rprec, lo, hi);
  int l = 0, r = n_masses;  // first index with sm[idx] >= lo
  while (l < r) {
    const int mid = (l + r) >> 1;
    if (sm[mid] < lo) l = mid + 1;
    else r = mid;
  }
  out[i] = (lo <= hi && l < n_masses && sm[l] <= hi) ? (int8_t)1 : (int8_t)0;
}

// ---------------------------------------------------------------------------
// explain: shared pieces
// ---------------------------------------------------------------------------
struct Lds {
  int w[kMaxRows];
  int cap[kMaxRows];
  uint8_t mod[kMaxRows];
  uint64_t capz0, capz1;  // rows with cap <= 0 (the table's, or the current query's)
};
__device__ __forceinline__ void stage_rows(Lds& s, const TableArgs& t) {
  for (int r = threadIdx.x; r < t.n_rows; r += blockDim.x) {
    s.w[r] = t.w[r];
    s.cap[r] = t.cap[r];
    s.mod[r] = t.mod[r];
  }
  if (threadIdx.x == 0) {
    s.capz0 = t.capz0;
    s.capz1 = t.capz1;
  }
  __syncthreads();
}

__device__ __forceinline__ int clamp_budget(int64_t a) {
  if (a < 0) return kInfBudget;  // np.inf
  return a > kInfBudget ? kInfBudget : (int)a;
}

// fast-path theorem: no budget check can fail for any window value
// <= hi when every mod row s has cap[s] >= hi / w_s and A >= hi / w_min_mod.
__device__ __forceinline__ bool budgets_never_bind(const TableArgs& t, int64_t hi, int A) {
  if (!t.any_mod) return true;
  if (hi > t.fast_limit_B) return false;
  if (A >= kInfBudget) return true;
  return hi < (int64_t)(A + 1) * t.w_min_mod;
}

// Candidate sinks.  A candidate is the path rows st.row(0..d), chosen top-down
// (descending rows); the payload record is [d+1][rows ascending] (the
// reference's solution list is ascending mass == ascending row).
struct CountSink {
  template <typename Stack>
  __device__ __forceinline__ void put(const Stack&, int, uint64_t) {}
};
struct MemSink {  // straight to the arena (deep / exact / overflowed shallow)
  uint8_t* dst;
  uint64_t cap_count;
  uint64_t written = 0;
  template <typename Stack>
  __device__ __forceinline__ void put(const Stack& st, int d, uint64_t pos) {
    if (written++ >= cap_count) return;
    dst[pos] = (uint8_t)(d + 1);
    for (int k = 0; k <= d; ++k) dst[pos + 1 + k] = st.row(d - k);
  }
};
// First 32 payload bytes of a deep-path lane kept in VGPRs during the
// counting DFS, so that a window whose candidates fit needs no second DFS to
// write them (config 1: one candidate of <= 9 bytes per query, 2x shorter
// dependent chains).
struct RegSinkDeep {
  uint64_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
  bool over = false;
  __device__ __forceinline__ void byte(int p, uint64_t b) {
    const uint64_t v = b << (8 * (p & 7));
    switch (p >> 3) {
      case 0: w0 |= v; break;
      case 1: w1 |= v; break;
      case 2: w2 |= v; break;
      default: w3 |= v; break;
    }
  }
  template <typename Stack>
  __device__ __forceinline__ void put(const Stack& st, int d, uint64_t pos) {
    if (over || pos + d + 2 > 32) {
      over = true;
      return;
    }
    byte((int)pos, (uint64_t)(d + 1));
    for (int k = 0; k <= d; ++k) byte((int)pos + 1 + k, st.row(d - k));
  }
  __device__ __forceinline__ void flush(uint8_t* dst, uint64_t nbytes) const {
    for (uint64_t p = 0; p < nbytes; ++p) {
      const uint64_t w = p < 8 ? w0 : (p < 16 ? w1 : (p < 24 ? w2 : w3));
      dst[p] = (uint8_t)(w >> (8 * (p & 7)));
    }
  }
};
// The first two candidates of a deep-path lane as their packed paths (rows
// of depths 0..7, PathView::p0) and depths, kept in VGPRs during the
// counting DFS: a leaf costs two register moves instead of assembling its
// payload record byte by byte inside the divergent DFS loop (config 1: one
// candidate of <= 8 items per query; the record bytes were 10 of its 51 us).
// A third candidate or a deeper one sets `over` (the lane enumerates again
// straight into the arena).
struct RegSinkPaths {
  uint64_t p0 = 0, p1 = 0;
  int d0 = 0, d1 = 0, n = 0;
  bool over = false;
  template <typename Path>
  __device__ __forceinline__ void put(const Path& path, int d, uint64_t) {
    if (n >= 2 || d >= 8) {
      over = true;
      return;
    }
    if (n == 0) {
      p0 = path.p0;
      d0 = d;
    } else {
      p1 = path.p0;
      d1 = d;
    }
    ++n;
  }
  // record [d + 1][rows ascending] = [d + 1][row(d) .. row(0)]
  __device__ __forceinline__ static void record(uint8_t* dst, uint64_t p, int d) {
    dst[0] = (uint8_t)(d + 1);
    for (int k = 0; k <= d; ++k) dst[1 + k] = (uint8_t)(p >> (8 * (d - k)));
  }
  __device__ __forceinline__ void flush(uint8_t* dst, uint64_t) const {
    if (n > 0) record(dst, p0, d0);
    if (n > 1) record(dst + d0 + 2, p1, d1);
  }
};

// Sinks of the shallow path receive the (<= 3) rows ascending as scalars.
struct CountSink3 {
  __device__ __forceinline__ void put(uint64_t, int, int, int, int) {}
};
struct MemSink3 {
  uint8_t* dst;
  __device__ __forceinline__ void put(uint64_t pos, int n, int r0, int r1, int r2) {
    dst[pos] = (uint8_t)n;
    dst[pos + 1] = (uint8_t)r0;
    if (n > 1) dst[pos + 2] = (uint8_t)r1;
    if (n > 2) dst[pos + 3] = (uint8_t)r2;
  }
};
struct RegSink {  // first 16 payload bytes of a lane kept in two VGPR pairs
  uint64_t lo = 0, hi = 0;
  bool over = false;
  __device__ __forceinline__ void byte(int p, uint64_t b) {
    uint64_t v = b << (8 * (p & 7));
    if (p < 8) lo |= v;
    else hi |= v;
  }
  __device__ __forceinline__ void put(uint64_t pos, int n, int r0, int r1, int r2) {
    if (pos + n + 1 > 16) {
      over = true;
      return;
    }
    int p = (int)pos;
    byte(p, (uint64_t)n);
    byte(p + 1, (uint64_t)r0);
    if (n > 1) byte(p + 2, (uint64_t)r1);
    if (n > 2) byte(p + 3, (uint64_t)r2);
  }
  __device__ __forceinline__ void flush(uint8_t* dst, uint64_t nbytes) const {
    for (uint64_t p = 0; p < nbytes; ++p) dst[p] = (uint8_t)((p < 8 ? lo : hi) >> (8 * (p & 7)));
  }
};

struct GlobFrame {
  uint64_t a, b;
  uint32_t m;
  int A, B;
  uint8_t r, top, pad0, pad1;
};
// A lane's DFS stack in global memory, interleaved over the role's lanes:
// frame d of lane g at f0[d * stride + g], so the lanes of a wave at equal
// depth touch consecutive frames (coalesced) instead of lines 3 KB apart.
struct GlobStack {
  GlobFrame* f;       // this lane's frame 0
  uint32_t stride;    // lanes of the role (frames per depth level)
  static constexpr int depth = kMaxDepth;
  __device__ __forceinline__ GlobFrame& at(int d) const { return f[(size_t)d * stride]; }
  __device__ __forceinline__ uint32_t m(int d) const { return at(d).m; }
  __device__ __forceinline__ M128 mask(int d) const { return {at(d).a, at(d).b}; }
  __device__ __forceinline__ uint8_t row(int d) const { return at(d).r; }
  __device__ __forceinline__ void set(int d, uint32_t m, M128 k) {
    at(d).m = m;
    at(d).a = k.a;
    at(d).b = k.b;
  }
  __device__ __forceinline__ void set_mask(int d, M128 k) {
    at(d).a = k.a;
    at(d).b = k.b;
  }
  __device__ __forceinline__ void set_row(int d, int r) { at(d).r = (uint8_t)r; }
  __device__ __forceinline__ void set_budget(int d, int A, int B, int top) {
    at(d).A = A;
    at(d).B = B;
    at(d).top = (uint8_t)top;
  }
  __device__ __forceinline__ int A(int d) const { return at(d).A; }
  __device__ __forceinline__ int B(int d) const { return at(d).B; }
  __device__ __forceinline__ int top(int d) const { return at(d).top; }
};

// ---------------------------------------------------------------------------
// exact path: per-lane open-addressing hash, one 32-B entry per visited mass
// ---------------------------------------------------------------------------
struct HEntry {
  uint64_t key;   // (epoch << 32) | m
  uint32_t meta;  // hv | ne << 8 (0xFF = none)
  uint32_t pad;
  uint64_t en0, en1;
};
// The reduced table's pairs from per-row reachability bitsets (sst_reach.hip,
// one query per wave): kept row k (k-th kept full-table row, ascending) has
// R_k = the masses its rows and the kept rows below reach.  Lane L holds kept
// rows L and L + 64 (full-table row, mass) and the ranks among the kept rows
// of full-table rows L and L + 64 (-1: dropped).
struct ReachView {
  const uint32_t* bits;  // R_k at bits + k * W
  int64_t W;             // words per row: masses [0, 32 W)
  int K;
  M128 kept;             // the kept rows (row 0 excluded)
  int row0, row1, w0, w1;
  int rank0, rank1;
};
__device__ __forceinline__ bool reach_bit(const ReachView& rv, int k, int64_t x) {
  if (x < 0 || (x >> 5) >= rv.W) return false;
  return (rv.bits[(int64_t)k * rv.W + (x >> 5)] >> (x & 31)) & 1u;
}

constexpr int kValSlots = 64;  // kept rows a fused replay holds (the caller checks K <= 64)
struct Hash {
  HEntry* e;
  uint32_t mask;  // capacity - 1
  uint64_t epoch;
  uint32_t used;
  uint32_t limit;
  uint64_t sink = 0;  // folds prefetch loads (see p1_visit)
  uint32_t last_meta = 0;  // meta written by the last first visit (p1_visit)
  bool reach = false;      // wave mode only: node records from rv, not the full table's index
  ReachView rv{};
  M128 last_L{0, 0};       // reach mode: the left bits of the last first visit's record (p1_classify)
  uint32_t last_rlo = 0;   // the rows [last_rlo, r] the last first visit covered (p1_visit)
  // fused values (length bounds, both directions): a frame's rows get their
  // lower / upper values when the frame completes -- every child is final by
  // then -- instead of in separate passes over the DAG
  int8_t* vals_lo = nullptr;
  int8_t* vals_hi = nullptr;
  int dflt_lo = 0;
  bool vals_bad = false;  // fused values: a visited child had no memo entry (reported as SST_ABORTED)
  bool dense = false;  // fused values: entry i's values at slot pad (its insertion order) x kValSlots + kept rank
  // the query's row caps and the rows with cap <= 0 (the table's in LDS, or
  // the query's own: per-query budgets), set by the caller before phase 1
  const int* cap = nullptr;
  uint64_t capz0 = 0, capz1 = 0;
  __device__ __forceinline__ uint32_t slot(uint32_t m) const { return (m * 0x9E3779B1u) & mask; }
  // returns entry pointer or nullptr if absent
  __device__ __forceinline__ HEntry* find(uint32_t m) const {
    uint64_t key = (epoch << 32) | m;
    uint32_t i = slot(m);
    while (true) {
      uint64_t k = e[i].key;
      if (k == key) return &e[i];
      if ((k >> 32) != epoch) return nullptr;
      i = (i + 1) & mask;
    }
  }
  // returns entry (inserting a fresh one) or nullptr when full
  __device__ __forceinline__ HEntry* get(uint32_t m) {
    uint64_t key = (epoch << 32) | m;
    uint32_t i = slot(m);
    while (true) {
      uint64_t k = e[i].key;
      if (k == key) return &e[i];
      if ((k >> 32) != epoch) {
        if (used >= limit) return nullptr;
        ++used;
        e[i].key = key;
        e[i].meta = 0xFFFFu;
        e[i].pad = dense ? used - 1 : 0;
        e[i].en0 = 0;
        e[i].en1 = 0;
        return &e[i];
      }
      i = (i + 1) & mask;
    }
  }
};

// ---------------------------------------------------------------------------
// enumeration over the (enabled) DAG from root v: counts candidates, adds
// their payload bytes, writes them when dst != nullptr.
//   MODE_FAST   enabled = L (budgets never bind)
//   MODE_NOMEMO budgets carried along the path (with_memo=False)
//   MODE_EXACT  enabled = en from the phase-1 hash, pruned by ne
// ---------------------------------------------------------------------------
enum { MODE_FAST = 0, MODE_NOMEMO = 1, MODE_EXACT = 2 };

struct EnumOut {
  uint64_t count;
  uint64_t bytes;
  uint64_t nodes;
  int fail;  // 1 depth, 2 node budget
  uint32_t iters = 0;  // loop iterations (timing builds)
};

// The candidate's rows as the sinks read them: depths below 8 from a packed
// register, deeper ones from the lane's stack.
template <typename Stack>
struct PathView {
  const Stack& st;
  uint64_t p0;  // row of depth d < 8 at bits 8d .. 8d+7
  __device__ __forceinline__ uint8_t row(int d) const { return d < 8 ? (uint8_t)(p0 >> (8 * d)) : st.row(d); }
};

// The current frame (mass, rows left, budgets) lives in registers; the stack
// holds only ancestors that still have rows left, and a 128-bit register
// bitmap marks their depths.  A finished frame therefore returns straight to
// the deepest such ancestor with one stack read (a single-candidate window:
// none at all), instead of reading back every level on the way up; each
// descent costs one dependent load (the child's index record).
template <int MODE, bool NW = false, typename Stack, typename Sink>
__device__ __forceinline__ void enumerate_root(const TableArgs& t, const Lds& s, Stack& st, const Hash* h, uint32_t v, int A0,
                               Sink& sink, uint64_t node_budget, EnumOut& o, M128 am) {
  const int top_row = t.n_rows - 1;
  M128 k;
  if (MODE == MODE_EXACT) {
    const HEntry* e = h->find(v);
    if (!e) return;
    k = mand(M128{e->en0, e->en1}, rows_upto(top_row));
  } else {
    ulonglong2 rec = ld_index(t.index, v);
    o.nodes++;
    k = nrm<NW>(mand(mand(rec_L(rec), rows_upto_nw<NW>(top_row)), am));
  }
  uint32_t m = v;
  int A = A0, B = s.cap[top_row], top = top_row;  // budgets: MODE_NOMEMO only
  int d = 0;
  uint64_t pend0 = 0, pend1 = 0;  // depths (0..63, 64..127) of saved frames with rows left
  PathView<Stack> path{st, 0};
  while (true) {
#ifdef SST_DIAG_TIME
    o.iters++;
#endif
    if (mzero(k)) {
      if ((pend0 | pend1) == 0) break;
      if (pend1) {  // deepest pending ancestor
        d = 127 - __builtin_clzll(pend1);
        pend1 &= ~(1ull << (d - 64));
      } else {
        d = 63 - __builtin_clzll(pend0);
        pend0 &= ~(1ull << d);
      }
      m = st.m(d);
      k = nrm<NW>(st.mask(d));
      if (MODE == MODE_NOMEMO) {
        A = st.A(d);
        B = st.B(d);
        top = st.top(d);
      }
      continue;
    }
    const int rr = mlow(k);
    k = mclear(k, rr);
    int Bv = 0;
    if (MODE == MODE_NOMEMO) {
      Bv = (rr == top) ? B : s.cap[rr];
      if (s.mod[rr] && !(A > 0 && Bv > 0)) continue;
    }
    const int64_t child = (int64_t)m - s.w[rr];
    if (d < 8)
      path.p0 = (path.p0 & ~(0xFFull << (8 * d))) | ((uint64_t)rr << (8 * d));
    else
      st.set_row(d, rr);
    if (child == 0) {
      sink.put(path, d, o.bytes);
      o.bytes += (uint64_t)(d + 2);
      o.count++;
      continue;
    }
    if (child < 0) continue;
    if (MODE == MODE_FAST && t.census && child < t.pair_hi && d + 3 <= Stack::depth) {
      // at most 2 items remain (child < 3 w_min): the pair list's entries of sum
      // == child are the subtree's leaves, sorted by (sum, top row) -- the
      // DFS's order here (first row ascending, the second then fixed) -- read
      // through L2 from the census instead of 2 random index-record fetches
      const uint32_t c0 = t.pair_base - 1u, cc = (uint32_t)child;
      const uint32_t lo_x = cc - 1u < c0 ? c0 : cc - 1u, hi_x = cc < c0 ? c0 : cc;
      const uint32_t e0 = t.census[lo_x - c0] & 0xFFFFu, e1 = t.census[hi_x - c0] & 0xFFFFu;
      const uint32_t* recs = t.pair_data + (t.n_pairs + 2);
      for (uint32_t e = e0; e < e1; ++e) {
        const uint32_t rec = recs[e];
        const int n = (int)(rec & 0xFFu);
        const int top = (int)((rec >> (n == 1 ? 8 : 16)) & 0xFFu), low = (int)((rec >> 8) & 0xFFu);
        if (top > rr) break;
        if (!mtest(am, top) || !mtest(am, low)) continue;  // a row outside the query's alphabet
        for (int j = 0; j < n; ++j) {
          const int dj = d + 1 + j, rj = j == 0 ? top : low;
          if (dj < 8)
            path.p0 = (path.p0 & ~(0xFFull << (8 * dj))) | ((uint64_t)rj << (8 * dj));
          else
            st.set_row(dj, rj);
        }
        sink.put(path, d + n, o.bytes);
        o.bytes += (uint64_t)(d + n + 2);
        o.count++;
      }
      continue;
    }
    if (o.nodes >= node_budget) {
      o.fail = 2;
      return;
    }
    M128 kc;
    if (MODE == MODE_EXACT) {
      const HEntry* e = h->find((uint32_t)child);
      if (!e) continue;
      int ne = (int)((e->meta >> 8) & 0xFF);
      if (ne == 0xFF || rr < ne) continue;
      kc = mand(M128{e->en0, e->en1}, rows_upto(rr));
      o.nodes++;
    } else {
      ulonglong2 rec = ld_index(t.index, child);
      o.nodes++;
      if (rec_lo(rec) > rr) continue;
      kc = nrm<NW>(mand(mand(rec_L(rec), rows_upto_nw<NW>(rr)), am));
    }
    if (d + 1 >= Stack::depth) {
      o.fail = 1;
      return;
    }
    if (!mzero(k)) {  // save this frame only if it has rows left
      st.set(d, m, k);
      if (MODE == MODE_NOMEMO) st.set_budget(d, A, B, top);
      if (d < 64)
        pend0 |= 1ull << d;
      else
        pend1 |= 1ull << (d - 64);
    }
    ++d;
    m = (uint32_t)child;
    k = kc;
    if (MODE == MODE_NOMEMO) {
      const int md = s.mod[rr];
      A -= md;
      B = Bv - md;
      top = rr;
    }
  }
}

// payload bytes/counts of a whole window [a, b] of roots
template <int MODE, bool NW = false, typename Stack, typename Sink>
__device__ __forceinline__ void enumerate_window(const TableArgs& t, const Lds& s, Stack& st, const Hash* h, int64_t a, int64_t b,
                                 int A0, Sink& sink, uint64_t node_budget, EnumOut& o,
                                 M128 am = M128{~0ull, ~0ull}) {
  if (a > b) return;
  int64_t wa = a >> 6, wb = b >> 6;
  for (int64_t wi = wa; wi <= wb; ++wi) {
    uint64_t x = t.valid[wi];
    if (wi == wa) x &= ~0ull << (a & 63);
    if (wi == wb) x &= ~0ull >> (63 - (b & 63));
    while (x) {
      int bit = __builtin_ctzll(x);
      x &= x - 1;
      uint32_t v = (uint32_t)((wi << 6) + bit);
      enumerate_root<MODE, NW>(t, s, st, h, v, A0, sink, node_budget, o, am);
      if (o.fail) return;
    }
  }
}

// SHALLOW fast path: budgets never bind and every window value is below
// 4 * w_min, so a candidate has at most 3 items.  The chain-form DFS
// (ascending rows at each level, as the reference's solution lists) becomes
// three explicit loops with all state in registers.
template <typename Sink>
__device__ __forceinline__ void shallow_window(const TableArgs& t, const Lds& s, int64_t a, int64_t b, Sink& sink,
                                               EnumOut& o) {
  if (a > b) return;
  const M128 top_mask = rows_upto(t.n_rows - 1);
  const int64_t wa = a >> 6, wb = b >> 6;
  const int64_t nw = wb - wa + 1;
  // the first 6 bitset words are loaded together (one round trip) and then
  // rotated through x0 so that no private array is indexed dynamically
  uint64_t x0 = t.valid[wa];
  uint64_t x1 = nw > 1 ? t.valid[wa + 1] : 0, x2 = nw > 2 ? t.valid[wa + 2] : 0;
  uint64_t x3 = nw > 3 ? t.valid[wa + 3] : 0, x4 = nw > 4 ? t.valid[wa + 4] : 0, x5 = nw > 5 ? t.valid[wa + 5] : 0;
  for (int64_t wi = wa; wi <= wb; ++wi) {
    uint64_t x = wi - wa < 6 ? x0 : t.valid[wi];
    x0 = x1;
    x1 = x2;
    x2 = x3;
    x3 = x4;
    x4 = x5;
    if (wi == wa) x &= ~0ull << (a & 63);
    if (wi == wb) x &= ~0ull >> (63 - (b & 63));
    while (x) {
      const int64_t v = (wi << 6) + __builtin_ctzll(x);
      x &= x - 1;
      M128 k1 = mand(rec_L(ld_index(t.index, v)), top_mask);
      o.nodes++;
      while (!mzero(k1)) {
        const int r1 = mlow(k1);
        k1 = mclear(k1, r1);
        const int64_t c1 = v - s.w[r1];
        if (c1 == 0) {
          sink.put(o.bytes, 1, r1, 0, 0);
          o.bytes += 2;
          o.count++;
          continue;
        }
        if (c1 < 0) continue;
        const ulonglong2 rec1 = ld_index(t.index, c1);
        o.nodes++;
        if (rec_lo(rec1) > r1) continue;
        M128 k2 = mand(rec_L(rec1), rows_upto(r1));
        while (!mzero(k2)) {
          const int r2 = mlow(k2);
          k2 = mclear(k2, r2);
          const int64_t c2 = c1 - s.w[r2];
          if (c2 == 0) {
            sink.put(o.bytes, 2, r2, r1, 0);
            o.bytes += 3;
            o.count++;
            continue;
          }
          if (c2 < 0) continue;
          const ulonglong2 rec2 = ld_index(t.index, c2);
          o.nodes++;
          if (rec_lo(rec2) > r2) continue;
          M128 k3 = mand(rec_L(rec2), rows_upto(r2));
          while (!mzero(k3)) {  // a 4th item cannot fit below 4 * w_min
            const int r3 = mlow(k3);
            k3 = mclear(k3, r3);
            if (c2 == s.w[r3]) {
              sink.put(o.bytes, 3, r3, r2, r1);
              o.bytes += 4;
              o.count++;
            }
          }
        }
      }
    }
  }
}

// min (dir 0) / max (dir 1) of the length bound's values, and its prefix over the 64 lanes
__device__ __forceinline__ int lb_combine(int dir, int x, int y) { return dir ? (x > y ? x : y) : (x < y ? x : y); }
__device__ __forceinline__ int lb_scan(int dir, int x) {  // inclusive prefix combine over the 64 lanes
  // DPP: row_shr 1, 2, 4, 8 inside each 16-lane row, then row_bcast 15 / 31
  // across rows; lanes whose source is out of range read the identity
  const int id = dir ? -128 : 127;
#define SST_SCAN_STEP(ctrl, rmask)                                                 \
  {                                                                                \
    const int t = __builtin_amdgcn_update_dpp(id, x, ctrl, rmask, 0xF, false);     \
    x = lb_combine(dir, x, t);                                                     \
  }
  SST_SCAN_STEP(0x111, 0xF)
  SST_SCAN_STEP(0x112, 0xF)
  SST_SCAN_STEP(0x114, 0xF)
  SST_SCAN_STEP(0x118, 0xF)
  SST_SCAN_STEP(0x142, 0xA)
  SST_SCAN_STEP(0x143, 0xC)
#undef SST_SCAN_STEP
  return x;
}

// ---------------------------------------------------------------------------
// exact path phase 1: replay the memoised DFS (first-visit budgets)
// ---------------------------------------------------------------------------
struct P1Frame {
  uint64_t en0, en1;  // rows newly enabled by this frame
  HEntry* e;
  uint32_t m;
  int A, B;
  uint8_t rtop, rnext, ne, pad1;  // ne: the frame's lowest non-empty row so far (wave mode)
  uint32_t meta;                  // the entry's meta as this frame wrote it (wave mode)
};

// the index record of mass m on the reduced table (wave-uniform m): left
// bits of the kept rows r with m - w_r in R_r, lo = the lowest kept row
// whose R holds m (255: unreachable), in the full-table index's packing
__device__ __forceinline__ ulonglong2 reach_rec(const ReachView& rv, uint32_t m) {
  const int lane = threadIdx.x & 63;
  bool in0 = false, in1 = false, b0 = false, b1 = false;
  if (lane < rv.K) {
    in0 = reach_bit(rv, lane, m);
    b0 = reach_bit(rv, lane, (int64_t)m - rv.w0);
  }
  if (lane + 64 < rv.K) {
    in1 = reach_bit(rv, lane + 64, m);
    b1 = reach_bit(rv, lane + 64, (int64_t)m - rv.w1);
  }
  const uint64_t M0 = __ballot(in0), M1 = __ballot(in1), L0 = __ballot(b0), L1 = __ballot(b1);
  int lo = 255;
  if (M0 | M1) {
    const int kk = M0 ? __builtin_ctzll(M0) : 64 + __builtin_ctzll(M1);
    const int ra = __shfl(rv.row0, kk & 63, 64), rb = __shfl(rv.row1, kk & 63, 64);
    lo = kk < 64 ? ra : rb;
  }
  auto lbit = [&](int rank) {
    return rank >= 0 && (rank < 64 ? ((L0 >> rank) & 1ull) : ((L1 >> (rank - 64)) & 1ull));
  };
  const uint64_t La = __ballot(lbit(rv.rank0)), Lb = __ballot(lbit(rv.rank1));
  return make_ulonglong2(La, (Lb & ((1ull << 56) - 1ull)) | ((uint64_t)lo << 56));
}

// visit (m, r, A, B): returns 1 if (m, r) is a first visit (its newly
// visited rows' enabled-left mask in *en, its memo entry in *ent: the caller
// makes it the current frame), 0 otherwise (memo hit or pair == 0; *nonempty
// = the child's "non-empty at row r" verdict), -1 on hash exhaustion.
// Memo entry meta: hv (bits 0-7), ne (8-15), lo (16-23).
template <bool WAVE>
__device__ __forceinline__ int p1_visit(const TableArgs& t, const Lds& s, Hash& h, uint32_t m, int r, int A, int B,
                                        bool& nonempty, uint64_t& nodes, M128& en_out, HEntry*& ent, M128 am) {
  // the index record and the memo's first probe slot (key, meta and the
  // enabled mask: the whole 32-B entry) are independent: issue them together
  // (both were prefetched by the parent frame)
  const uint32_t sl = h.slot(m);
  ulonglong2 rec;
  if (WAVE && h.reach) rec = reach_rec(h.rv, m);
  else rec = ld_index(t.index, m);
  const ulonglong2 kv = *(const ulonglong2*)&h.e[sl];
  const ulonglong2 ev = *(const ulonglong2*)&h.e[sl].en0;
  nodes++;
  int lo = rec_lo(rec);
  if (r < lo) {  // pair(r, m) == 0: [] without memo (mass_explanation.py:148-149)
    nonempty = false;
    return 0;
  }
  HEntry* e;
  uint32_t meta;
  uint64_t en_old0 = 0, en_old1 = 0;
  if (kv.x == ((h.epoch << 32) | m)) {  // found in the first slot
    e = &h.e[sl];
    meta = (uint32_t)kv.y;
    en_old0 = ev.x;
    en_old1 = ev.y;
  } else {
    e = h.get(m);  // inserts a fresh entry when the key is absent
    if (!e) return -1;
    meta = e->meta;
    en_old0 = e->en0;
    en_old1 = e->en1;
  }
  int hv = (int)(meta & 0xFF);
  hv = hv == 0xFF ? -1 : hv;
  if (r <= hv) {  // memo hit (mass_explanation.py:122-123)
    int ne = (int)((meta >> 8) & 0xFF);
    nonempty = ne != 0xFF && r >= ne;
    return 0;
  }
  int rlo = lo > hv + 1 ? lo : hv + 1;
  // newly visited rows [rlo, r]; left enabled iff bit1 and (not mod or A>0 && B>0),
  // with B = cap[row] for rows reached by the up chain and B for row r itself
  M128 rng = mand(rows_upto(r), rows_from(rlo));
  M128 en = mand(rec_L(rec), rng);
  if (t.any_mod) {
    M128 blocked;
    if (A > 0) blocked = M128{t.mod0 & h.capz0, t.mod1 & h.capz1};
    else blocked = M128{t.mod0, t.mod1};
    en.a &= ~blocked.a;
    en.b &= ~blocked.b;
    if (s.mod[r] && mtest(rec_L(rec), r)) {
      bool ok = A > 0 && B > 0;
      if (ok) {
        if (r < 64) en.a |= 1ull << r;
        else en.b |= 1ull << (r - 64);
      } else {
        en = mclear(en, r);
      }
    }
  }
  en = mand(en, am);  // a reduced alphabet: left branches on its rows only
  e->en0 = en_old0 | en.a;
  e->en1 = en_old1 | en.b;
  e->meta = (meta & 0xFF00u) | ((uint32_t)lo << 16) | (uint32_t)r;
  h.last_meta = e->meta;
  h.last_rlo = (uint32_t)rlo;
  if (WAVE && h.reach) h.last_L = rec_L(rec);
  // the frame will visit (m - w_rr, rr) for every enabled row: issue their
  // index-record and first-probe loads now, independently, so the visits
  // that follow hit the cache instead of paying dependent HBM round trips
  if (WAVE && h.reach) {
    // reduced-table records are assembled from the rows' bitsets: no prefetch
  } else if (WAVE) {
    // one query per wave: lane L takes rows L and L + 64 -- and, speculating
    // one level deeper, the children (c0 - w_s, s <= rr0) of the first enabled
    // row rr0, the frame the DFS enters next, whose own records are then
    // already in flight when it is expanded
    const int lane = threadIdx.x & 63;
    const int rr0 = mzero(en) ? -1 : mlow(en);
    const int64_t c0 = rr0 >= 0 ? (int64_t)m - s.w[rr0] : 0;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int rr = lane + 64 * half;
      if (rr < t.n_rows) {
        const int64_t c = (int64_t)m - s.w[rr];
        if (mtest(en, rr) && c > 0) h.sink ^= __builtin_nontemporal_load(&t.index[c].y) ^ h.e[h.slot((uint32_t)c)].key;
        const int64_t g = c0 - s.w[rr];
        if (rr >= 1 && rr <= rr0 && g > 0)
          h.sink ^= __builtin_nontemporal_load(&t.index[g].y) ^ h.e[h.slot((uint32_t)g)].key;
      }
    }
  } else {
    for (M128 k = en; !mzero(k);) {
      const int rr = mlow(k);
      k = mclear(k, rr);
      const int64_t c = (int64_t)m - s.w[rr];
      if (c > 0) h.sink ^= __builtin_nontemporal_load(&t.index[c].y) ^ h.e[h.slot((uint32_t)c)].key;
    }
  }
  en_out = en;
  ent = e;
  return 1;
}

__device__ __forceinline__ void p1_set_ne(HEntry* e, int rr) {  // lowest non-empty row (first found wins)
  if (((e->meta >> 8) & 0xFF) == 0xFF) e->meta = (e->meta & ~0xFF00u) | ((uint32_t)rr << 8);
}

// returns 0 ok, -1 hash full, -2 depth, -3 node budget.  The current frame
// lives in registers; fr[] holds only the saved ancestors (touched on push
// and pop, not per row).
template <bool WAVE>
__device__ int phase1_body(const TableArgs& t, const Lds& s, Hash& h, P1Frame* fr, int64_t a, int64_t b, int A0,
                           uint64_t node_budget, uint64_t& nodes, M128 am) {
  const int top = t.n_rows - 1;
  for (int64_t v = a; v <= b; ++v) {
    if (!((t.valid[v >> 6] >> (v & 63)) & 1ull)) continue;
    bool ne_dummy;
    M128 rest;
    HEntry* e;
    int pr = p1_visit<WAVE>(t, s, h, (uint32_t)v, top, A0, h.cap[top], ne_dummy, nodes, rest, e, am);
    if (pr < 0) return -1;
    if (pr == 0) continue;
    uint32_t m = (uint32_t)v;
    int A = A0, B = h.cap[top], rtop = top, d = 0;
    for (;;) {
      if (mzero(rest)) {  // frame done: report to the parent (its pending row)
        if (d == 0) break;
        HEntry* ce = e;
        const P1Frame f = fr[--d];
        rest = M128{f.en0, f.en1};
        e = f.e;
        m = f.m;
        A = f.A;
        B = f.B;
        rtop = f.rtop;
        const int rr = f.rnext - 1;
        const int ne = (int)((ce->meta >> 8) & 0xFF);
        if (ne != 0xFF && rr >= ne) p1_set_ne(e, rr);
        continue;
      }
      const int rr = mlow(rest);
      rest = mclear(rest, rr);
      const int md = s.mod[rr];
      const int Bv = (rr == rtop) ? B : h.cap[rr];
      const int64_t child = (int64_t)m - s.w[rr];
      bool nonempty = false;
      if (child == 0) {
        nonempty = true;
      } else if (child > 0) {
        if (nodes >= node_budget) return -3;
        if (d + 1 >= kMaxDepth) return -2;
        M128 cen;
        HEntry* cent;
        const int pushed =
            p1_visit<WAVE>(t, s, h, (uint32_t)child, rr, A - md, Bv - md, nonempty, nodes, cen, cent, am);
        if (pushed < 0) return -1;
        if (pushed) {  // descend: save this frame (its pending row is rr)
          fr[d++] = P1Frame{rest.a, rest.b, e, m, A, B, (uint8_t)rtop, (uint8_t)(rr + 1), 0, 0};
          rest = cen;
          e = cent;
          m = (uint32_t)child;
          A -= md;
          B = Bv - md;
          rtop = rr;
          continue;
        }
      }
      if (nonempty) p1_set_ne(e, rr);
    }
  }
  return 0;
}

// Classification of a fresh frame's children in one probe round (wave mode).
// For child (c = m - w_r, r) two of the three outcomes of its visit are
// settled now and cannot change before the replay reaches row r:
//   r < lo(c): pair(r, c) == 0, [] without memo (static);
//   hv(c) >= r: memo hit, non-empty iff ne(c) <= r (hv only grows, and an ne
//     <= hv is final: an ne set later lies above the hv of that time);
// and the third, hv(c) < r, stays a first visit: the nodes inside an earlier
// sibling's subtree have rows r' < r and raise hv(c) to at most r' < r.
// Only those children are descended (ascending rows, as the reference).  The
// frame's lowest non-empty row is the minimum over its rows (the sequential
// replay meets them in ascending order, so "first found" is the minimum).
__device__ __forceinline__ M128 p1_classify(const TableArgs& t, const Lds& s, Hash& h, uint32_t m, M128 rows,
                                            int& ne) {
  const int lane = threadIdx.x & 63;
  bool desc[2];
  int nrow = 0xFF;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int r = lane + 64 * half;
    desc[half] = false;
    if (r < t.n_rows && mtest(rows, r)) {
      const int64_t c = (int64_t)m - s.w[r];
      bool reach_c;
      if (c <= 0) reach_c = false;
      else if (h.reach) reach_c = mtest(h.last_L, r);  // c in R_r (r kept): the frame's record says so
      else reach_c = r >= rec_lo(ld_index(t.index, c));
      if (c == 0) {
        nrow = nrow < r ? nrow : r;
      } else if (reach_c) {
        const HEntry* ce = h.find((uint32_t)c);
        const uint32_t meta = ce ? ce->meta : 0xFFFFu;
        const int hv = (meta & 0xFF) == 0xFF ? -1 : (int)(meta & 0xFF);
        if (r <= hv) {
          const int nec = (int)((meta >> 8) & 0xFF);
          if (nec != 0xFF && r >= nec) nrow = nrow < r ? nrow : r;
          if (h.vals_lo) {  // fused values: this final child's values are read when the frame completes
            const int rk = half ? h.rv.rank1 : h.rv.rank0;
            const size_t at = (size_t)ce->pad * kValSlots + (rk < 0 ? 0 : rk);
            h.sink ^= (uint64_t)h.vals_lo[at] ^ ((uint64_t)h.vals_hi[at] << 8);
          }
        } else {
          desc[half] = true;
        }
      }
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const int o = __shfl_xor(nrow, off, 64);
    nrow = nrow < o ? nrow : o;
  }
  ne = ne < nrow ? ne : nrow;
  const M128 d{(uint64_t)__ballot(desc[0]), (uint64_t)__ballot(desc[1])};
  if (h.reach && !mzero(d)) {
    // the replay descends into the lowest such child next: issue its record's
    // reach words now (reach_rec reads them), behind this frame's probes
    const int64_t c0 = (int64_t)m - s.w[mlow(d)];
    const ReachView& rv = h.rv;
    uint32_t sink = 0;
    if (lane < rv.K) {
      const int64_t x0 = c0 >> 5, x1 = (c0 - rv.w0) >> 5;
      if (x0 >= 0 && x0 < rv.W) sink ^= rv.bits[(int64_t)lane * rv.W + x0];
      if (x1 >= 0 && x1 < rv.W) sink ^= rv.bits[(int64_t)lane * rv.W + x1];
    }
    if (lane + 64 < rv.K) {
      const int64_t x0 = c0 >> 5, x1 = (c0 - rv.w1) >> 5;
      if (x0 >= 0 && x0 < rv.W) sink ^= rv.bits[(int64_t)(lane + 64) * rv.W + x0];
      if (x1 >= 0 && x1 < rv.W) sink ^= rv.bits[(int64_t)(lane + 64) * rv.W + x1];
    }
    h.sink ^= sink;
  }
  return d;
}

// Both length-bound values of a completed frame's rows [rlo, rtop] of mass m
// (lb_values_wave's recurrence, one frame at a time): row r's value combines
// the default, the row below (the up chain; the entry's earlier rows are
// final) and, when its left branch was enabled at the first visit, the
// child's value at row r plus one.  Values are kept for the alphabet's rows
// only, at slot kept-rank (a dropped row's value is the nearest kept row's
// below it), per entry in insertion order: 2 x kValSlots bytes per mass.
__device__ __forceinline__ void p1_values(const TableArgs& t, const Lds& s, Hash& h, const HEntry* e, uint32_t m,
                                          int rlo, int rtop) {
  const int lane = threadIdx.x & 63;
  const int lo = (int)((e->meta >> 16) & 0xFF);
  const M128 en{e->en0, e->en1};
  int cl[2] = {127, 127}, ch[2] = {-128, -128};
  int rk[2] = {h.rv.rank0, h.rv.rank1};
  bool miss = false;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int r = lane + 64 * half;
    if (r < t.n_rows && r >= rlo && r <= rtop && mtest(en, r)) {  // enabled rows are kept rows
      const uint32_t c = m - (uint32_t)s.w[r];
      int vl = 0, vh = 0;  // total_mass == 0 -> 0 (mass_table.py:378-379)
      if (c != 0) {
        const HEntry* ce = h.find(c);
        if (ce) {
          const size_t at = (size_t)ce->pad * kValSlots + rk[half];
          vl = h.vals_lo[at];
          vh = h.vals_hi[at];
        } else {
          miss = true;  // phase 1 memoises every child it enters: reported, not guessed (lb_uncomputed's -3)
        }
      }
      cl[half] = vl + 1;
      ch[half] = vh + 1;
    }
  }
  if (__ballot(miss)) h.vals_bad = true;
  const size_t base = (size_t)e->pad * kValSlots;
  // the seed: the value at row rlo - 1, i.e. at the highest kept row below rlo (if >= lo)
  const uint64_t below0 = rlo >= 64 ? ~0ull : ((1ull << rlo) - 1ull);
  const uint64_t below1 = rlo <= 64 ? 0ull : (rlo >= 128 ? ~0ull : ((1ull << (rlo - 64)) - 1ull));
  const M128 keptm = h.rv.kept;
  const int nb = __builtin_popcountll(keptm.a & below0) + __builtin_popcountll(keptm.b & below1);
  const bool has_seed = rlo > lo && nb > 0;  // lo is a kept row: rows in [lo, rlo) hold a kept one
  const int seed_lo = has_seed ? h.vals_lo[base + nb - 1] : h.dflt_lo;
  const int seed_hi = has_seed ? h.vals_hi[base + nb - 1] : -1;
  const int l0 = lb_scan(0, cl[0]), l1 = lb_combine(0, lb_scan(0, cl[1]), __shfl(l0, 63, 64));
  const int u0 = lb_scan(1, ch[0]), u1 = lb_combine(1, lb_scan(1, ch[1]), __shfl(u0, 63, 64));
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int r = lane + 64 * half;
    if (r < t.n_rows && r >= rlo && r <= rtop && rk[half] >= 0) {
      h.vals_lo[base + rk[half]] = (int8_t)lb_combine(0, seed_lo, half ? l1 : l0);
      h.vals_hi[base + rk[half]] = (int8_t)lb_combine(1, seed_hi, half ? u1 : u0);
    }
  }
}

// phase1_body for one query per wave: the same replay, with the saved frames
// in LDS and the current frame's lowest non-empty row in a register (written
// to its memo entry once, when the frame completes -- no other node can read
// that entry earlier, since every node below it has a smaller mass).  That
// leaves one memory round trip per visited node: its index record and memo
// entry, loaded together (p1_visit).
__device__ int phase1_body_wave(const TableArgs& t, const Lds& s, Hash& h, P1Frame* fr, int64_t a, int64_t b, int A0,
                                uint64_t node_budget, uint64_t& nodes, M128 am) {
  const int top = t.n_rows - 1;
  for (int64_t v = a; v <= b; ++v) {
    if (h.reach ? !reach_bit(h.rv, h.rv.K - 1, v) : !((t.valid[v >> 6] >> (v & 63)) & 1ull)) continue;
    bool ne_dummy;
    M128 rest;
    HEntry* e;
    int pr = p1_visit<true>(t, s, h, (uint32_t)v, top, A0, s.cap[top], ne_dummy, nodes, rest, e, am);
    if (pr < 0) return -1;
    if (pr == 0) continue;
    uint32_t m = (uint32_t)v, meta = h.last_meta;
    int A = A0, B = s.cap[top], rtop = top, d = 0;
    int rlo = (int)h.last_rlo;
    int ne = (int)((meta >> 8) & 0xFF);
    rest = p1_classify(t, s, h, m, rest, ne);
    for (;;) {
      if (mzero(rest)) {  // frame done: publish its non-empty row, report to the parent
        e->meta = (meta & ~0xFF00u) | ((uint32_t)ne << 8);
        if (h.vals_lo) p1_values(t, s, h, e, m, rlo, rtop);
        if (d == 0) break;
        const int cne = ne;
        const P1Frame f = fr[--d];
        rest = M128{f.en0, f.en1};
        e = f.e;
        m = f.m;
        A = f.A;
        B = f.B;
        rtop = f.rtop;
        rlo = f.pad1;
        ne = f.ne;
        meta = f.meta;
        const int rr = f.rnext - 1;
        if (cne != 0xFF && rr >= cne) ne = ne < rr ? ne : rr;
        continue;
      }
      const int rr = mlow(rest);
      rest = mclear(rest, rr);
      const int md = s.mod[rr];
      const int Bv = (rr == rtop) ? B : s.cap[rr];
      const int64_t child = (int64_t)m - s.w[rr];
      bool nonempty = false;
      if (child == 0) {
        nonempty = true;
      } else if (child > 0) {
        if (nodes >= node_budget) return -3;
        if (d + 1 >= kMaxDepth) return -2;
        M128 cen;
        HEntry* cent;
        const int pushed =
            p1_visit<true>(t, s, h, (uint32_t)child, rr, A - md, Bv - md, nonempty, nodes, cen, cent, am);
        if (pushed < 0) return -1;
        if (pushed) {  // descend: save this frame (its pending row is rr)
          fr[d++] = P1Frame{rest.a, rest.b, e, m, A, B, (uint8_t)rtop, (uint8_t)(rr + 1), (uint8_t)ne, (uint8_t)rlo,
                            meta};
          rest = cen;
          e = cent;
          m = (uint32_t)child;
          A -= md;
          B = Bv - md;
          rtop = rr;
          rlo = (int)h.last_rlo;
          meta = h.last_meta;
          ne = (int)((meta >> 8) & 0xFF);
          rest = p1_classify(t, s, h, m, rest, ne);
          continue;
        }
      }
      if (nonempty) ne = ne < rr ? ne : rr;  // lowest non-empty row
    }
  }
  return 0;
}

// WAVE: one query per wave.  Every lane runs the same (uniform) replay --
// identical loads and stores to the same addresses cost one transaction --
// and the lanes split only the prefetch loads (p1_visit).
template <bool WAVE>
__device__ int phase1(const TableArgs& t, const Lds& s, Hash& h, P1Frame* fr, int64_t a, int64_t b, int A0,
                      uint64_t node_budget, uint64_t& nodes, M128 am = M128{~0ull, ~0ull}) {
  h.sink = 0;
  const int rc = WAVE ? phase1_body_wave(t, s, h, fr, a, b, A0, node_budget, nodes, am)
                      : phase1_body<WAVE>(t, s, h, fr, a, b, A0, node_budget, nodes, am);
  // (never true) keeps every lane's prefetch loads alive; a ballot keeps rc uniform
  return __ballot(h.sink == 0x5bd1e9955bd1e995ull) ? rc - 100 : rc;
}

// ---------------------------------------------------------------------------
// workgroup output allocation: exclusive scan of per-lane byte counts, one
// atomic per workgroup on the arena cursor.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    uint64_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  return x;
}

// Sum a per-lane counter over the workgroup and add it to stats[k] with one
// atomic (all threads of the workgroup must call it).
__device__ __forceinline__ void wg_stat(unsigned long long* stats, int k, uint64_t v) {
  __shared__ uint64_t red[1024 / 64];  // up to 1024-lane workgroups
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t tot = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) tot += red[i];
    if (tot) atomicAdd(&stats[k], (unsigned long long)tot);
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Explain, part 1 -- k_explain_scan (persistent grid, independent waves):
// every wave streams 64-query tiles in a grid stride (inputs prefetched one
// tile ahead), quantises the window and resolves it: from the LDS pair list
// (<= 2-item windows), or -- tables without the list -- from the valid
// bitset, queueing the rest to the wave's own worklist region (ballot +
// mbcnt: no atomics) or the deferred class lists.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t lane_mask_lt(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {  // set bits of m below this lane
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Append query i to deferred class list `cls` (kClassDeep / kClassExact /
// kClassNomemo; -1: none) with one atomic per class per wave instruction:
// per-lane atomics on one counter serialise in L2 (125 k routed windows cost
// the scan 1.4 ms that way).  Call with every lane that may append active.
__device__ __forceinline__ void route_append(const OutArgs& out, int64_t n, int cls, uint32_t i) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int c = kClassDeep; c <= kClassNomemo; ++c) {
    const uint64_t m = __ballot(cls == c);
    if (!m) continue;
    const int leader = __builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(&out.counters[c], (uint32_t)__builtin_popcountll(m));
    base = (uint32_t)__shfl((int)base, leader, 64);
    if (cls == c) out.lists[(int64_t)c * n + base + mbcnt(m)] = i;
  }
}

// One query's final result on the deferred paths: its status byte, and for a
// query with candidates one hit record appended to the deferred hit list
// (k_result_pack moves the list behind the scan's hits and rebases its
// payload offsets).  Appends are wavefront-aggregated: one atomic per wave
// instruction over its active lanes.
__device__ __forceinline__ void emit_result(const OutArgs& out, bool live, uint32_t i, int8_t status,
                                            uint64_t count, uint64_t off, bool lane_owns = true) {
  if (live) out.status[i] = status;
  const bool hit = live && lane_owns && (status == SST_SOME || status == SST_OVERFLOW || status == SST_ABORTED);
  const uint64_t b = __ballot(hit);
  if (!b) return;
  const int lane = threadIdx.x & 63;
  const int leader = __builtin_ctzll(b);
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(out.dhit_count, (uint32_t)__builtin_popcountll(b));
  base = (uint32_t)__shfl((int)base, leader, 64);
  if (hit) {
    const bool some = status == SST_SOME;
    const uint64_t word = some ? off : count;
    out.dhits[base + __builtin_popcountll(b & lane_mask_lt(lane))] =
        make_uint4(i | (some ? kHitOffsetFlag : 0u), count > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)count,
                   (uint32_t)word, (uint32_t)(word >> 32));
  }
}

// any reachable value in [a, b]: up to 6 bitset words loaded at once
__device__ __forceinline__ bool window_has_roots(const uint64_t* valid, int64_t a, int64_t b) {
  const int64_t wa = a >> 6, wb = b >> 6;
  const int64_t nw = wb - wa + 1;
  const uint64_t fm = ~0ull << (a & 63), lm = ~0ull >> (63 - (b & 63));
  if (nw <= 6) {
    uint64_t x0 = valid[wa];
    uint64_t x1 = nw > 1 ? valid[wa + 1] : 0, x2 = nw > 2 ? valid[wa + 2] : 0;
    uint64_t x3 = nw > 3 ? valid[wa + 3] : 0, x4 = nw > 4 ? valid[wa + 4] : 0, x5 = nw > 5 ? valid[wa + 5] : 0;
    x0 &= fm;
    if (nw == 1) x0 &= lm;
    if (nw == 2) x1 &= lm;
    if (nw == 3) x2 &= lm;
    if (nw == 4) x3 &= lm;
    if (nw == 5) x4 &= lm;
    if (nw == 6) x5 &= lm;
    return (x0 | x1 | x2 | x3 | x4 | x5) != 0;
  }
  return any_bits(valid, a, b);
}

// Inclusive wavefront prefix sum of a u32 on the DPP crossbar (no LDS
// round trips): 16-lane row scans, then rows 1/3 and 2/3 take the running
// totals of the rows before them through row_bcast:15 / row_bcast:31.
__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return x;
}

// Payload allocation of one 64-query chunk of the SHALLOW role: wavefront
// prefix sum of the per-lane byte counts, one atomic on the spill cursor.
struct TileOut {
  uint64_t off;
  uint64_t bytes;
  int8_t status;
};
__device__ __forceinline__ TileOut spill_alloc(const OutArgs& out, int lane, uint64_t bytes, int8_t status) {
  const uint64_t incl = wave_incl_scan(bytes);
  const uint64_t total = __shfl(incl, 63, 64);
  uint64_t base = 0;
  if (total) {
    unsigned long long sb = 0;
    if (lane == 0) sb = atomicAdd((unsigned long long*)out.cursor, (unsigned long long)total);
    base = out.spill_base + __shfl(sb, 0, 64);
  }
  TileOut r{base + incl - bytes, bytes, status};
  if (bytes && r.off + bytes > out.arena_bytes) {
    r.status = (int8_t)kStatusArenaRetry;
    r.bytes = 0;
  }
  return r;
}

// Workgroup-wide exclusive allocation on a shared counter: one returning
// atomic per workgroup instead of one per wave (all threads call it, the
// trip count around it is workgroup-uniform).  A single counter word serves
// only ≈88 returning atomics per µs (MI355X_MICROARCH.md, dequeue row), so
// the deep role's ≈1.6 k waves of a config-1 pass spent ≈20 µs queueing on
// the spill cursor and the hit counter; 4-wave workgroups cut that by 4.
template <typename T>
__device__ __forceinline__ uint64_t wg_alloc(T* ctr, uint64_t v) {
  __shared__ uint64_t part[kDefWG / 64 + 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t incl = wave_incl_scan(v);
  if (lane == 63) part[w] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t tot = 0;
    for (int k = 0; k < kDefWG / 64; ++k) tot += part[k];
    part[kDefWG / 64] = tot ? (uint64_t)atomicAdd(ctr, (T)tot) : 0;
  }
  __syncthreads();
  uint64_t base = part[kDefWG / 64];
  for (int k = 0; k < w; ++k) base += part[k];
  __syncthreads();  // part[] is rewritten by the next call
  return base + incl - v;
}

// spill_alloc / emit_result with workgroup-wide allocation (deep role)
__device__ __forceinline__ TileOut spill_alloc_wg(const OutArgs& out, uint64_t bytes, int8_t status) {
  TileOut r{out.spill_base + wg_alloc((unsigned long long*)out.cursor, bytes), bytes, status};
  if (bytes && r.off + bytes > out.arena_bytes) {
    r.status = (int8_t)kStatusArenaRetry;
    r.bytes = 0;
  }
  return r;
}
__device__ __forceinline__ void emit_result_wg(const OutArgs& out, bool live, uint32_t i, int8_t status,
                                               uint64_t count, uint64_t off, bool lane_owns = true) {
  if (live) out.status[i] = status;
  const bool hit = live && lane_owns && (status == SST_SOME || status == SST_OVERFLOW || status == SST_ABORTED);
  const uint32_t k = (uint32_t)wg_alloc(out.dhit_count, hit ? 1u : 0u);
  if (hit) {
    const bool some = status == SST_SOME;
    const uint64_t word = some ? off : count;
    out.dhits[k] = make_uint4(i | (some ? kHitOffsetFlag : 0u), count > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)count,
                              (uint32_t)word, (uint32_t)(word >> 32));
  }
}

// counters of the SHALLOW windows one wave ran (shallow_chunk)
struct ShallowStats {
  uint64_t q, nodes, payload;
};
// a scan wave's counters into its own wave_stats slot (no atomics)
__device__ __forceinline__ void wave_stats_flush(const OutArgs& out, int64_t wave, int lane, int q_stat, int p_stat,
                                                 uint64_t n_q, uint64_t payload) {
  for (int o = 32; o > 0; o >>= 1) {
    n_q += __shfl_down(n_q, o, 64);
    payload += __shfl_down(payload, o, 64);
  }
  if (lane == 0) {
    unsigned long long* ws = out.wave_stats + wave * kNumStats;
    for (int k = 0; k < kNumStats; ++k) ws[k] = 0;
    ws[q_stat] = n_q;
    ws[p_stat] = payload;
  }
}

// Element i of a per-query array through a 32-bit byte offset (batches are
// capped at SST_MAX_EXPLAIN_BATCH = 2^29 queries): the compiler then
// addresses it as SGPR base + 32-bit VGPR offset instead of 64-bit VALU math.
template <typename T>
__device__ __forceinline__ T* q_at(T* base, uint32_t i) {
  return (T*)((char*)base + (uint32_t)(i * (uint32_t)sizeof(T)));
}

// Candidates of a pair-class window [a, hi] from the LDS pair list (layout:
// TableArgs::pair_data): the entries with sums in the window, in list order
// (= the reference's order).  The window's bucket word holds the first sum at
// or after the bucket start, which settles most empty windows with that one
// 4-byte read; the rest walk the sums array two entries per LDS round trip up
// to the first sum above hi (the sentinels bound the walk).  Sums carry the
// record kind in bit 0, so the walk compares against 2a and 2hi+1 and reads no
// records.  Returns the count, the first entry and the payload bytes
// ([1][top] = 2 B, [2][low][top] = 3 B).
struct PairLds {
  const uint32_t* sums;
  const uint32_t* recs;
  const uint32_t* bk;
  uint32_t base;
  int shift;
};
__device__ __forceinline__ uint32_t pair_walk(const PairLds& p, uint32_t a, uint32_t hi, uint32_t& first,
                                              uint32_t& bytes) {
  const uint32_t rel = a > p.base ? a - p.base : 0u;
  const uint32_t bw = p.bk[rel >> p.shift];
  uint32_t k = bw & 0xFFFFu, cnt = 0, nb = 0;
  if (p.base + ((rel >> p.shift) << p.shift) + (bw >> 16) <= hi) {
    const uint32_t a2 = a << 1, h2 = (hi << 1) | 1u;
    for (;;) {
      const uint32_t e0 = p.sums[k], e1 = p.sums[k + 1];
      const bool s0 = e0 <= h2, s1 = s0 && e1 <= h2;  // sorted: still inside the walk
      const bool in0 = s0 && e0 >= a2, in1 = s1 && e1 >= a2;
      cnt += (in0 ? 1u : 0u) + (in1 ? 1u : 0u);
      nb += (in0 ? 2u + (e0 & 1u) : 0u) + (in1 ? 2u + (e1 & 1u) : 0u);
      k += (s0 ? 1u : 0u) + (s1 ? 1u : 0u);
      if (!s1) break;
    }
  }
  first = k - cnt;  // the in-window entries end the walk
  bytes = nb;
  return cnt;
}
// One (unaligned) dword store per record: the 1-2 bytes past a record are
// rewritten by the lane's next record, or land in the 2 pad bytes allocated
// after the query's last one (never referenced: offsets and counts delimit
// the candidates).  Two stores per record (short + byte): scan +1 us.
typedef uint32_t __attribute__((aligned(1))) u32_unaligned;
__device__ __forceinline__ void pair_store(const PairLds& p, uint32_t first, uint32_t cnt, uint8_t* dst) {
#pragma unroll 1
  for (uint32_t k = first; k < first + cnt; ++k) {
    const uint32_t rec = p.recs[k];  // [k][rows] in the low 2-3 bytes, zero above
    *(u32_unaligned*)dst = rec;
    dst += (rec & 0xFFu) + 1u;
  }
}

// One 64-item chunk of a worklist: route unclassified windows (no reachable
// value -> NONE / EMPTY; deeper than SHALLOW or budget-binding -> the deferred
// class lists, status pending), run the SHALLOW fast path on the rest (all
// DFS state and the first 16 payload bytes in VGPRs), allocate payload in the
// spill area and write the status byte and hit record.
// WG: workgroup-wide allocation (the caller's trip count is workgroup-uniform)
template <bool WG = false>
__device__ __forceinline__ void shallow_item(const TableArgs& t, const QueryArgs& q, const OutArgs& out, const Lds& s,
                                             bool live, uint32_t i, int64_t a, int64_t b, uint32_t flags, int lane,
                                             ShallowStats& st) {
  int8_t status = SST_NONE;
  bool deferred = false;
  RegSink sink;
  EnumOut eo{0, 0, 0, 0};
  int cls = -1;
  if (live) {
    bool run = true;
    if (flags & kItemUnclassified) {  // from the bitset scan: route it here
      if (!window_has_roots(t.valid, a, b)) {
        run = false;
      } else if (!(flags & kItemNever) || b >= t.shallow_hi) {
        cls = (flags & kItemNever) ? kClassDeep : (q.with_memo ? kClassExact : kClassNomemo);
        run = false;
        deferred = true;
      }
    }
    if (run) {
      shallow_window(t, s, a, b, sink, eo);
      st.q++;
      st.nodes += eo.nodes;
    }
    status = eo.count ? (eo.count > q.cap_count ? SST_OVERFLOW : SST_SOME)
                      : ((flags & kItemZero) ? SST_EMPTY : SST_NONE);
    if (deferred) status = (int8_t)kStatusPending;
  }
  route_append(out, q.n, cls, i);
  const uint64_t want = status == SST_SOME ? eo.bytes : 0;
  const TileOut to = WG ? spill_alloc_wg(out, want, status) : spill_alloc(out, lane, want, status);
  if (to.bytes) {
    if (!sink.over) {
      sink.flush(out.payload + to.off, to.bytes);
    } else {  // more than 16 bytes: enumerate again straight into the arena
      MemSink3 ms{out.payload + to.off};
      EnumOut e2{0, 0, 0, 0};
      shallow_window(t, s, a, b, ms, e2);
    }
  }
  // deferred queries: pending here, the deep / exact roles write their result
  if (WG)
    emit_result_wg(out, live, i, to.status, eo.count, to.off, !deferred);
  else
    emit_result(out, live, i, to.status, eo.count, to.off, !deferred);
  st.payload += to.bytes;
}
__device__ __forceinline__ void shallow_chunk(const TableArgs& t, const QueryArgs& q, const OutArgs& out, const Lds& s,
                                              const uint4* wl, uint32_t k0, uint32_t nw, int lane, ShallowStats& st) {
  const bool live = k0 + lane < nw;
  const uint4 item = live ? wl[k0 + lane] : make_uint4(0, 1, 0, 0);  // {query, first window value >= 1, last, kItem* flags}
  shallow_item(t, q, out, s, live, item.x, item.y, item.z, item.w, lane, st);
}

// 64 scan hit records -> dense records; returns the running payload offset
__device__ __forceinline__ uint64_t pack_hits(uint4* __restrict__ out, uint32_t k, uint32_t nh, uint2 rr, uint64_t run) {
  const bool live = k < nh;
  const uint32_t cnt = rr.y & 0xFFFFu, bytes = live ? rr.y >> 16 : 0u;
  const uint32_t incl = wave_incl_scan32(bytes);
  const uint64_t word = bytes ? run + (incl - bytes) : (uint64_t)cnt;  // offset, or OVERFLOW's count
  if (live) out[k] = make_uint4(rr.x, cnt, (uint32_t)word, (uint32_t)(word >> 32));
  return run + (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
}
__device__ __forceinline__ uint32_t wave_sum32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan32(x), 63);
}

// The result header (u64 words, include order kHdr*): HBM copy and the
// host-mapped copy the host polls (system-scope stores, one lane)
__device__ __forceinline__ void write_header(uint64_t* hdr, uint64_t* hdr_host, const uint64_t* h) {
  for (int k = 0; k < kHdrWords; ++k) hdr[k] = h[k];
  if (hdr_host)
    for (int k = 0; k < kHdrWords; ++k)
      __hip_atomic_store(hdr_host + k, h[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t ctl_read(uint64_t* ctl, int k) {  // counters other workgroups added to
  return __hip_atomic_fetch_add(ctl + k, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Raw buffer resource over [base, base + bytes): a lane whose offset is past
// the end is dropped by the hardware (no memory access), so a masked store is
// one unconditional instruction.  The scan's tiles issue a fixed number of
// vector-memory instructions this way, which lets the compiler's vmcnt waits
// for the next tile's inputs be exact: the in-order counter then never makes
// a tile wait for the stores of the tile just before it.
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
constexpr uint32_t kBufSkip = 0x80000000u;
constexpr int kPreChunks = 4;  // hit-record chunks a scan wave prepares before its look-back wait  // an offset past every buffer the scan addresses
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
// payload bytes of `cnt` pair-list records from entry `first` (LDS)
__device__ __forceinline__ uint32_t pair_bytes(const PairLds& p, uint32_t first, uint32_t cnt) {
  uint32_t b = 0;
#pragma unroll 1
  for (uint32_t k = first; k < first + cnt; ++k) b += (p.recs[k] & 0xFFu) + 1u;
  return b;
}

// 8 waves/SIMD: two 1024-lane workgroups per CU, each with its LDS copy of
// the pair list (<= 44 KB).  Tables built here carry the list: a window below
// 3 * w_min whose budgets cannot bind is answered from LDS; every other
// non-empty window is routed (bitset check, SHALLOW worklist or deferred class
// lists).  THR: per-query thresholds given (else tol * mass).  MODS: per-query
// budgets given (else the host folded the scalar budget into q.pair_hi_lim /
// q.never_hi_lim, fold_scan_limits).  The classification is branch-free on
// exact f64 integers, then u32 (a window inside the table lies in [0, limit)
// with limit < 2^31).
//
// A tile (64 queries) issues exactly its input loads and two masked stores:
// the status bytes and one 8-B hit record {query, first entry | count << 16}
// per SOME / OVERFLOW query, at the back of the wave's worklist region.  The
// candidates' bytes are not written in the loop: after its tiles each wave
// turns its hit records into the result (payload bytes from the LDS pair
// list): on the device path (fused) the dense hit list and the dense payload,
// placed by a decoupled look-back over the workgroups' totals (the last
// workgroup writes the header); otherwise its payload region and 8-B records
// {query, count | bytes << 16} for k_result_pack.
template <bool THR, bool MODS>
__device__ __forceinline__ void explain_scan_wg(const TableArgs& t, const QueryArgs& q, const OutArgs& out,
                                                const uint32_t bid, const uint32_t nbid) {
  extern __shared__ uint32_t lds_pair_img[];
  if (bid == 0) {
    if (threadIdx.x < (unsigned)out.ctl_words) out.ctl_next[threadIdx.x] = 0;
    for (uint32_t k = threadIdx.x; k < nbid; k += blockDim.x) out.agg_next[k] = 0;
  }
  const int n_img = 2 * (t.n_pairs + 2) + t.n_buckets;
  // 16-B copies (the image is padded to 16 B; 4-B copies: scan +2.5 us)
  for (int k = threadIdx.x; k < ((n_img + 3) >> 2); k += blockDim.x)
    ((uint4*)lds_pair_img)[k] = ((const uint4*)t.pair_data)[k];
  __syncthreads();
  const PairLds pl{lds_pair_img, lds_pair_img + t.n_pairs + 2, lds_pair_img + 2 * (t.n_pairs + 2), t.pair_base,
                   t.pair_shift};
  const int lane = threadIdx.x & 63;
  // wave-uniform in SGPRs (the buffer resources below must be scalar)
  const uint32_t w_in = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t wave = bid * (kScanWG / 64) + w_in;
  const uint32_t n_waves = nbid * (kScanWG / 64);
  const uint32_t n = (uint32_t)q.n;  // < 2^32 - 64 (host checks)
  const uint32_t ntiles = (n + 63) >> 6;
  const double limitf = (double)t.limit;
  uint32_t st_q = 0, st_payload = 0;  // per lane: pair-path queries, their payload bytes (+ 2 pad bytes each)
  uint4* wl = out.work + (uint64_t)wave * out.work_region;
  uint32_t n_work = 0;  // wave-uniform
  // hit records fill the wave's worklist region from its END (a query is
  // either queued or a hit, and 16 * items + 8 * hits <= the region)
  const uint32_t wl_bytes = (uint32_t)(out.work_region * 16);  // < 2^32 (host checks)
  const __amdgpu_buffer_rsrc_t wl_rsrc = buf_rsrc(wl, wl_bytes);
  const __amdgpu_buffer_rsrc_t st_rsrc = buf_rsrc(out.status, n);
  uint32_t n_hit = 0;  // wave-uniform
  // deferred-class windows (deep / exact / no-memo): staged in the wave's own
  // slots during the tiles, copied to the class lists after them with one
  // atomic per class per workgroup -- atomics of every wave on the shared
  // class counters serialise (config 1: scan 80 -> 44 us without them)
  uint32_t* const stage = out.stage + (uint64_t)wave * out.work_region;
  uint32_t n_staged = 0;  // wave-uniform (one SGPR in the tile loop: the per-class counts are taken after it)
  // Software pipeline, two tiles deep: a tile's inputs are loaded two tiles
  // ahead into one of two register sets that swap roles between the unrolled
  // steps (no copies), each load issued after the previous tile's two stores.
  // Loads are unconditional (index clamped to the last query), streamed once
  // (nontemporal).
  auto fetch = [&](uint32_t tl, double& m, double& tt, int64_t& mm) {
    const uint32_t j = tl < ntiles ? min(tl * 64 + lane, n - 1) : n - 1;
    m = __builtin_nontemporal_load(q_at(q.mass, j));
    if (THR) tt = __builtin_nontemporal_load(q_at(q.thr, j));
    if (MODS) mm = __builtin_nontemporal_load(q_at(q.max_mods, j));
  };
  auto step = [&](uint32_t tile, double m_in, double t_in, int64_t mm_cur) {
    const uint32_t i = tile * 64 + lane;
    const bool live = i < n;
    const double m_cur = m_in, t_cur = THR ? t_in : q.tol * m_in;
    double lof, hif;
    quantise_lean(m_cur, t_cur, q.prec, q.rprec, lof, hif);
    const bool nonempty = live && lof <= hif;
    const bool oot = nonempty && !(hif < limitf);  // mass_explanation.py:134-138 (NotImplementedError)
    const bool zero = nonempty && !oot && lof <= 0.0 && hif >= 0.0;  // v == 0 -> [[]] (:130-131)
    const double af = __builtin_fmax(lof, 1.0);
    const bool active = nonempty && !oot && af <= hif;
    const uint32_t a = active ? (uint32_t)af : 0u, hi = active ? (uint32_t)hif : 0u;
    bool pair, never;
    if (MODS) {  // fast-path theorem per lane (budgets_never_bind on u32 values)
      const int A0 = clamp_budget(mm_cur);
      const bool a0ok =
          !t.any_mod || A0 >= kInfBudget || (uint64_t)hi < (uint64_t)(A0 + 1) * (uint64_t)t.w_min_mod;
      pair = active && a0ok && hi < t.pair_lim;
      // per-query budgets: the fast-path limit of the query's caps
      const uint32_t nl = q.qlen ? q.never_len[q.qlen[live ? i : n - 1]] : t.never_lim;
      never = a0ok && hi < nl;
    } else {
      pair = active && hi < q.pair_hi_lim;
      never = hi < q.never_hi_lim;
    }
    const bool work = active && !pair;  // routed below (bitset, depth, budgets)
    uint32_t first = 0, cnt = 0, bytes = 0;
    if (pair) cnt = pair_walk(pl, a, hi, first, bytes);
    int8_t status = oot ? (int8_t)SST_OUT_OF_TABLE : (zero ? (int8_t)SST_EMPTY : (int8_t)SST_NONE);
    if (cnt) status = cnt > q.cap32 ? (int8_t)SST_OVERFLOW : (int8_t)SST_SOME;
    st_payload += status == SST_SOME ? bytes + 2u : 0u;  // + 2 pad bytes (pair_store)
    st_q += pair ? 1u : 0u;
    // the tile's two stores (masked lanes dropped): NONE / EMPTY / OUT_OF_TABLE /
    // SOME / OVERFLOW status bytes; the hit records (pair path only: cnt == 0 off it)
    const uint64_t hbal = __ballot(cnt != 0);
    const uint32_t hpos = n_hit + mbcnt(hbal);
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)status, st_rsrc, (live && !work) ? i : kBufSkip, 0, 0);
    const u32x2 rv = {i, first | (cnt << 16)};
    __builtin_amdgcn_raw_buffer_store_b64(rv, wl_rsrc, cnt ? wl_bytes - 8u * (hpos + 1u) : kBufSkip, 0, 0);
    n_hit += (uint32_t)__builtin_popcountll(hbal);
    if (__ballot(work)) {  // wave-uniform, rare here: route the window now, so that the deferred class lists
                           // are complete when the scan ends (one tail launch runs every class)
      // (the class's role reads the window's bitset words itself: a window
      // without reachable values costs it one look; none here keeps the
      // tile loop free of scattered loads)
      int cls = -1;
      if (work) {
        if (never && hi < t.shallow_hi) {
          cls = kClassShallow;  // <= 3 items, budgets cannot bind: the SHALLOW role writes the result
        } else {
          cls = never ? kClassDeep : (q.with_memo ? kClassExact : kClassNomemo);
          out.status[i] = (int8_t)kStatusPending;
        }
      }
      const uint64_t cb = __ballot(cls >= 0);
      if (cls >= 0) stage[n_staged + mbcnt(cb)] = i | ((uint32_t)cls << 30);
      n_staged += (uint32_t)__builtin_popcountll(cb);
    }
  };
  double mA = 0.0, tA = 0.0, mB = 0.0, tB = 0.0;
  int64_t mmA = q.max_mods_scalar, mmB = q.max_mods_scalar;
  // tile order: pairs of waves of every workgroup first, so that the last,
  // partial round of tiles is spread over all CUs (not over the first few
  // workgroups) while tiles 2j, 2j+1 -- one 128-B line of status bytes --
  // stay in one workgroup, i.e. one XCD's L2 (A/B: -0.8 us)
  const uint32_t vw = (((w_in >> 1) * nbid + bid) << 1) | (w_in & 1u);
  fetch(vw, mA, tA, mmA);
  // two dropped stores where a tile's stores would be: the loop entry then has
  // the same VMEM count between the two prefetches as every later round, so
  // the compiler's waits at the loop head are exact on both paths into it
  __builtin_amdgcn_raw_buffer_store_b8(0, st_rsrc, kBufSkip, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b8(1, st_rsrc, kBufSkip + 64u, 0, 0);
  fetch(vw + n_waves, mB, tB, mmB);
  for (uint32_t tile = vw; tile < ntiles; tile += 2 * n_waves) {
    step(tile, mA, tA, mmA);
    fetch(tile + 2 * n_waves, mA, tA, mmA);
    if (tile + n_waves >= ntiles) break;
    step(tile + n_waves, mB, tB, mmB);
    fetch(tile + 3 * n_waves, mB, tB, mmB);
  }
  // ---- the wave's totals: hit records, payload bytes (16-B units per wave
  // piece of the payload)
  const uint32_t pay = wave_sum32(st_payload);
  const uint64_t region0 = (uint64_t)wave * out.region_bytes;  // non-fused: the wave's payload region
  const bool fits = out.fused || pay <= min(out.region_bytes, (uint64_t)UINT32_MAX);
  const uint32_t units = fits ? (pay + 15u) >> 4 : 0u;
  if (lane == 0) {
    out.work_count[wave] = n_work;
    out.tally[wave] = make_uint2(n_hit, units);
    if (!fits) {  // the host re-runs the pass with larger regions
      atomicAdd(out.arena_retries, (unsigned long long)max(n_hit, 1u));
      atomicMax(out.region_need, (unsigned long long)pay);
    }
  }
  wave_stats_flush(out, wave, lane, kStatPair, kStatPairPayload, st_q, st_payload);
  __shared__ uint2 wg_part[kScanWG / 64];
  __shared__ uint32_t wg_pre[2];
  __shared__ uint32_t wg_cls[kScanWG / 64][kNumClasses];  // per wave: SHALLOW items, staged class windows
  __shared__ uint32_t wg_cls_base[kNumClasses];
  // this wave's hit records, staged windows and counter adds have landed
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  uint32_t n_cls[kNumClasses] = {0u, 0u, 0u, 0u};
  for (uint32_t k0 = 0; k0 < n_staged; k0 += 64) {  // its staged windows per class
    const uint32_t k = k0 + lane;
    const uint32_t cl = k < n_staged ? stage[k] >> 30 : 4u;
#pragma unroll
    for (int c = 0; c < kNumClasses; ++c) n_cls[c] += (uint32_t)__builtin_popcountll(__ballot(cl == (uint32_t)c));
  }
  if (lane == 0) {
    wg_part[w_in] = make_uint2(n_hit, units);
#pragma unroll
    for (int c = 0; c < kNumClasses; ++c) wg_cls[w_in][c] = n_cls[c];
  }
  __syncthreads();
  uint32_t wg_h = 0, wg_u = 0;
  if (threadIdx.x < kNumClasses) {  // the workgroup's class totals: one atomic each (SHALLOW: lets an idle role exit)
    uint32_t tot = 0;
    for (int k = 0; k < kScanWG / 64; ++k) tot += wg_cls[k][threadIdx.x];
    wg_cls_base[threadIdx.x] = tot ? atomicAdd(&out.counters[threadIdx.x], tot) : 0u;
  }
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the class adds are done before the totals are published
    for (int k = 0; k < kScanWG / 64; ++k) {
      wg_h += wg_part[k].x;
      wg_u += wg_part[k].y;
    }
    out.wg_tally[bid] = make_uint2(wg_h, wg_u);
    if (out.fused)  // publish (8-B agent-scope store: flag and sums in one word)
      __hip_atomic_store(out.agg + bid, (1ull << 63) | ((uint64_t)wg_u << 32) | wg_h, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  // The first kPreChunks x 64 hit records, their payload sizes (LDS) and
  // wave-relative offsets are taken after this workgroup published its totals and before its
  // look-back, so that this work overlaps the wait for the workgroups before this one
  const uint2* rec = (const uint2*)(wl + out.work_region);  // record k at rec[-1 - k]
  const uint32_t nh_copy = (out.dbg & 1) ? 0 : n_hit;
  uint2 rr[kPreChunks];
  uint32_t pbv[kPreChunks], inclv[kPreChunks], rel[kPreChunks + 1];
  rel[0] = 0;
#pragma unroll
  for (int c = 0; c < kPreChunks; ++c) {
    const uint32_t k = c * 64 + lane;
    rr[c] = k < nh_copy ? *(rec - 1 - k) : make_uint2(0, 0);
  }
#pragma unroll
  for (int c = 0; c < kPreChunks; ++c) {
    const uint32_t k = c * 64 + lane, cnt = rr[c].y >> 16;
    pbv[c] = (k < nh_copy && cnt <= q.cap32) ? pair_bytes(pl, rr[c].y & 0xFFFFu, cnt) + 2u : 0u;
    inclv[c] = wave_incl_scan32(pbv[c]);
    rel[c + 1] = rel[c] + (uint32_t)__builtin_amdgcn_readlane((int)inclv[c], 63);
  }
  uint64_t hbase = 0, pbase = region0;
  if (out.fused) {
    // Wave 0 sums the aggregates of the workgroups before this one (decoupled
    // look-back over workgroups: each publishes once, when its tiles are
    // done); the last workgroup also has every total and writes the header
    if (w_in == 0) {
      const uint32_t b = bid;
      uint32_t ph = 0, pu = 0;
      for (uint32_t k0 = 0; k0 < b; k0 += 64) {
        const uint32_t k = k0 + lane;
        uint64_t v = 0;
        if (k < b && !(out.dbg & 4))
          for (;;) {
            v = __hip_atomic_load(out.agg + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (v >> 63) break;
            __builtin_amdgcn_s_sleep(4);
          }
        ph += (uint32_t)v;
        pu += (uint32_t)(v >> 32) & 0x7FFFFFFFu;
      }
      ph = wave_sum32(ph);
      pu = wave_sum32(pu);
      if (lane == 0) {
        wg_pre[0] = ph;
        wg_pre[1] = pu;
        if (b == nbid - 1) {  // every workgroup before this one has published: the totals
          uint64_t* ctl = out.cursor;  // the pass's control block
          const uint64_t ctr01 = ctl_read(ctl, kCtlCounters), ctr23 = ctl_read(ctl, kCtlCounters + 1);
          const uint64_t total = ((uint64_t)pu + wg_u) << 4;
          // the scan's part of the dense payload is bounded by the regions part of the
          // arena (a tail pack appends the spill bytes behind it): re-run with larger regions
          const bool over = total > out.spill_base;
          uint64_t h[kHdrWords];
          h[kHdrHits] = (uint64_t)ph + wg_h;
          h[kHdrPayload] = total;
          h[kHdrRouted] = (ctr01 & 0xFFFFFFFFu) + (ctr01 >> 32) + (ctr23 & 0xFFFFFFFFu) + (ctr23 >> 32);
          h[kHdrExactRetries] = 0;
          if (over) atomicAdd(out.arena_retries, 1ull);  // also seen by a later tail pack's header
          h[kHdrArenaRetries] = ctl_read(ctl, kCtlArenaRetries);
          h[kHdrCursor] = 0;
          h[kHdrPass] = out.pass_id;
          h[kHdrRegionNeed] = ctl_read(ctl, kCtlRegionNeed);
          write_header(out.hdr, out.hdr_host, h);
        }
      }
    }
    __syncthreads();
    uint32_t eh = 0, eu = 0;
    for (uint32_t k = 0; k < w_in; ++k) {
      eh += wg_part[k].x;
      eu += wg_part[k].y;
    }
    hbase = (uint64_t)wg_pre[0] + eh;
    pbase = ((uint64_t)wg_pre[1] + eu) << 4;
  }
  if (!out.fused) __syncthreads();  // wg_cls_base (the fused path synchronised after its look-back)
  if (n_staged) {  // this wave's staged class windows -> the class lists, behind the waves before it
    uint32_t run[kNumClasses];
#pragma unroll
    for (int c = 0; c < kNumClasses; ++c) {
      run[c] = wg_cls_base[c];
      for (uint32_t k = 0; k < w_in; ++k) run[c] += wg_cls[k][c];
    }
    for (uint32_t k0 = 0; k0 < n_staged; k0 += 64) {
      const uint32_t k = k0 + lane;
      const bool live = k < n_staged;
      const uint32_t item = live ? stage[k] : 0u;
      const uint32_t cl = item >> 30;
      uint32_t slot = 0;
#pragma unroll
      for (int c = 0; c < kNumClasses; ++c) {
        const uint64_t bc = __ballot(live && cl == (uint32_t)c);
        if (live && cl == (uint32_t)c) slot = run[c] + mbcnt(bc);
        run[c] += (uint32_t)__builtin_popcountll(bc);
      }
      if (live) out.lists[(int64_t)cl * q.n + slot] = item & 0x3FFFFFFFu;
    }
  }
  // ---- the wave's hit records -> result: payload bytes from the LDS pair
  // list (one dword store per record, pair_store), dense 16-B records (fused)
  // or the k_result_pack records in place
  const bool write_pay = out.fused ? pbase + pay <= out.spill_base : fits;
  uint8_t* pdst = out.fused ? out.dense : out.payload;
  auto emit = [&](uint32_t k, uint2 r, uint32_t pb, uint64_t off) {
    const uint32_t cnt = r.y >> 16, first = r.y & 0xFFFFu;
    if (pb && write_pay && !(out.dbg & 2)) pair_store(pl, first, cnt, pdst + off);
    if (k < n_hit) {
      if (out.fused) {
        const uint64_t word = pb ? off : (uint64_t)cnt;  // OVERFLOW: the exact count, no payload
        out.hits_out[hbase + k] = make_uint4(r.x, cnt, (uint32_t)word, (uint32_t)(word >> 32));
        out.hit_refs[hbase + k] = (uint16_t)(first | (pb ? 0u : 0x8000u));  // sst_result_pair_hits
      } else {
        *((uint2*)rec - 1 - k) = make_uint2(r.x, cnt | (pb << 16));
      }
    }
  };
#pragma unroll
  for (int c = 0; c < kPreChunks; ++c)
    if (c * 64 < nh_copy) emit(c * 64 + lane, rr[c], pbv[c], pbase + rel[c] + (inclv[c] - pbv[c]));
  uint64_t run = pbase + rel[kPreChunks];
  for (uint32_t k0 = kPreChunks * 64; k0 < nh_copy; k0 += 64) {
    const uint32_t k = k0 + lane;
    const uint2 r = k < n_hit ? *(rec - 1 - k) : make_uint2(0, 0);
    const uint32_t cnt = r.y >> 16;
    const uint32_t pb = (k < n_hit && cnt <= q.cap32) ? pair_bytes(pl, r.y & 0xFFFFu, cnt) + 2u : 0u;
    const uint32_t incl = wave_incl_scan32(pb);
    emit(k, r, pb, run + (incl - pb));
    run += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  }
}
template <bool THR, bool MODS>
__global__ __launch_bounds__(kScanWG, 8) void k_explain_scan(TableArgs t, QueryArgs q, OutArgs out) {
  explain_scan_wg<THR, MODS>(t, q, out, blockIdx.x, gridDim.x);
}
// One launch for a step of both predicates (sst_step_device): the pair
// scan's grid, then a7_blocks workgroups of is_valid over peaks x 4 breakage
// weights (1 024 peaks each).  The scan's workgroups are dispatched first (its
// look-back only ever waits for scan workgroups dispatched before it); the
// host gives a fused step one scan workgroup per CU (step_scan_wg_per_cu), so
// the is_valid workgroups run in each CU's other half beside the scan from
// the start, and the step pays one launch.  (is_valid in front of the scan
// instead: 8 us slower per step; two scan workgroups per CU, is_valid only in
// the scan's tail: 2 us slower; same-box A/Bs.)
template <bool THR, bool MODS>
__global__ __launch_bounds__(kScanWG, 8) void k_step(TableArgs t, QueryArgs q, OutArgs out, ValidArgs v, PeakShifts sh,
                                                   uint32_t a7_blocks) {
  const uint32_t n_scan = gridDim.x - a7_blocks;
  if (blockIdx.x >= n_scan) {
    is_valid_peak<4>(v, sh, (blockIdx.x - n_scan) * kScanWG + threadIdx.x);
    return;
  }
  explain_scan_wg<THR, MODS>(t, q, out, blockIdx.x, n_scan);
}

// the extent ceil((max(kept) * 35 + 1) / C) * C of query i's reduced table
// (per-query alphabets; the top kept row below the table's row count)
__device__ __forceinline__ int64_t reduced_limit(const TableArgs& t, const QueryArgs& q, int64_t i) {
  const int64_t g = q.spec ? (int64_t)q.spec[i] : 0;
  const M128 am = mand(M128{q.alpha[2 * g], q.alpha[2 * g + 1]}, rows_upto(t.n_rows - 1));
  const int top = am.b ? 127 - __builtin_clzll(am.b) : 63 - __builtin_clzll(am.a | 1ull);
  const int64_t max_mass = (int64_t)t.w[top] * 35;
  return (max_mass + q.comp) / q.comp * q.comp;
}

// Tables without the pair list (uploaded tables, literal-sweep rows): every
// non-empty window is checked against the valid bitset here, then queued for
// the expand kernel (<= 3 items) or the deferred class lists.
__global__ __launch_bounds__(kScanWG, 8) void k_bitset_scan(TableArgs t, QueryArgs q, OutArgs out) {
  if (blockIdx.x == 0) {
    if (threadIdx.x < (unsigned)out.ctl_words) out.ctl_next[threadIdx.x] = 0;
    for (uint32_t k = threadIdx.x; k < gridDim.x; k += blockDim.x) out.agg_next[k] = 0;
  }
  const int lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * (kScanWG / 64) + (threadIdx.x >> 6);
  const uint32_t n_waves = gridDim.x * (kScanWG / 64);
  const uint32_t n = (uint32_t)q.n;  // < 2^32 - 64 (host checks)
  const uint32_t ntiles = (n + 63) >> 6;
  uint4* wl = out.work + (uint64_t)wave * out.work_region;
  uint32_t n_work = 0;  // wave-uniform
  for (uint32_t tile = wave; tile < ntiles; tile += n_waves) {
    const uint32_t i = tile * 64 + lane;
    const bool live = i < n;
    double lof = 1.0, hif = 0.0;
    int64_t mm = q.max_mods_scalar;
    if (live) {
      quantise_f(q.mass[i], q.thr ? q.thr[i] : 0.0, q.thr == nullptr, q.tol, q.prec, q.rprec, lof, hif);
      if (q.max_mods) mm = q.max_mods[i];
    }
    const bool nonempty = live && lof <= hif;
    // the table's extent; with a per-query alphabet, its reduced table's
    // (max(kept) * 35, mass_table.py:114-117): every window value at or past
    // it raises, reachable or not (mass_explanation.py:134-138, NameError)
    double limf = (double)t.limit;
    if (q.alpha && live) limf = fmin(limf, (double)reduced_limit(t, q, i));
    const bool oot = nonempty && !(hif < limf);
    const bool zero = nonempty && !oot && lof <= 0.0 && hif >= 0.0;  // v == 0 -> [[]] (:130-131)
    const double af = lof < 1.0 ? 1.0 : lof;
    const bool active = nonempty && !oot && af <= hif;
    const uint32_t a = active ? (uint32_t)af : 0u, hi = active ? (uint32_t)hif : 0u;
    const int A0 = clamp_budget(mm);
    const bool a0ok = !t.any_mod || A0 >= kInfBudget || (uint64_t)hi < (uint64_t)(A0 + 1) * (uint64_t)t.w_min_mod;
    const uint32_t nl = q.qlen && live ? q.never_len[q.qlen[i]] : t.never_lim;  // per-query budgets
    const bool never = hi < nl && a0ok;
    int8_t status = oot ? (int8_t)SST_OUT_OF_TABLE : (zero ? (int8_t)SST_EMPTY : (int8_t)SST_NONE);
    bool work = false;
    uint4 item = make_uint4(0, 0, 0, 0);
    int route = -1;
    if (active && window_has_roots(t.valid, a, hi)) {
      int cls;
      if (never) cls = hi < t.shallow_hi ? kClassShallow : kClassDeep;
      else cls = q.with_memo ? kClassExact : kClassNomemo;
      if (cls == kClassShallow) {
        work = true;  // the expand kernel writes status, count and offset
        item = make_uint4(i, a, hi, zero ? kItemZero : 0u);
      } else {
        route = cls;
        status = (int8_t)kStatusPending;
      }
    }
    route_append(out, q.n, route, i);
    if (live && !work) out.status[i] = status;
    const uint64_t bal = __ballot(work);
    if (work) wl[n_work + __builtin_popcountll(bal & lane_mask_lt(lane))] = item;
    n_work += (uint32_t)__builtin_popcountll(bal);
  }
  if (lane == 0) {
    out.work_count[wave] = n_work;
    out.tally[wave] = make_uint2(0, 0);  // no hit records: the expand kernel emits them
    if (n_work) atomicAdd(&out.counters[kClassShallow], n_work);  // lets an idle expand launch exit at once
  }
  if (threadIdx.x == 0) out.wg_tally[blockIdx.x] = make_uint2(0, 0);
  wave_stats_flush(out, wave, lane, kStatPair, kStatPairPayload, 0, 0);
}

// ---------------------------------------------------------------------------
// Explain, part 2 -- the SHALLOW fast path for queued windows: k_explain_expand
// after k_bitset_scan (tables without the pair list), the first role of
// k_explain_deferred after the pair scan (which routed every window).  Each wave takes
// scan-wave worklist regions in a grid stride, 64 queries at a time; payload
// goes to the wave's own arena region through a bump pointer fed by a
// wavefront prefix sum (a full region spills: one atomic per tile).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void expand_body(const TableArgs& t, const QueryArgs& q, const OutArgs& out, Lds& s,
                                            int64_t wave, int64_t n_waves) {
  const int lane = threadIdx.x & 63;
  if (out.counters[kClassShallow] == 0) return;  // nothing queued (block-uniform)
  stage_rows(s, t);
  ShallowStats st{0, 0, 0};
  for (int64_t src = wave; src < out.n_scan_waves; src += n_waves) {
    const uint32_t nw = out.work_count[src];
    const uint4* wl = out.work + (uint64_t)src * out.work_region;
    for (uint32_t k0 = 0; k0 < nw; k0 += 64) shallow_chunk(t, q, out, s, wl, k0, nw, lane, st);
  }
  for (int o = 32; o > 0; o >>= 1) {
    st.q += __shfl_down(st.q, o, 64);
    st.nodes += __shfl_down(st.nodes, o, 64);
    st.payload += __shfl_down(st.payload, o, 64);
  }
  if (lane == 0 && st.q) {
    atomicAdd(&out.stats[kStatShallow], (unsigned long long)st.q);
    atomicAdd(&out.stats[kStatNodes], (unsigned long long)st.nodes);
    atomicAdd(&out.stats[kStatPayload], (unsigned long long)st.payload);
  }
}
// The SHALLOW role of k_explain_deferred after the pair scan: the scan
// appended its <= 3-item windows (budgets cannot bind) to the dense class-0
// list; one lane per window (recomputed from the query), the waves of the
// role in a grid stride over the list.
__device__ void shallow_list_body(const TableArgs& t, const QueryArgs& q, const OutArgs& out, Lds& s, int blk,
                                  int nblk) {
  const uint32_t n_list = out.counters[kClassShallow];
  if (n_list == 0) return;  // block-uniform: nothing queued
  stage_rows(s, t);
  const int lane = threadIdx.x & 63;
  const int64_t nthreads = (int64_t)nblk * blockDim.x;
  ShallowStats st{0, 0, 0};
  // workgroup-uniform trip count: one allocation atomic per workgroup (wg_alloc)
  for (int64_t jb = (int64_t)blk * blockDim.x; jb < (int64_t)n_list; jb += nthreads) {
    const int64_t j = jb + threadIdx.x;
    const bool live = j < (int64_t)n_list;
    uint32_t i = 0, flags = 0;
    int64_t a = 1, b = 0;
    if (live) {
      i = out.lists[(int64_t)kClassShallow * q.n + j];
      int64_t lo, hi;
      quantise(q.mass[i], q.thr ? q.thr[i] : 0.0, q.thr == nullptr, q.tol, q.prec, q.rprec, lo, hi);
      flags = (lo <= 0 && hi >= 0) ? kItemZero : 0u;
      a = lo < 1 ? 1 : lo;
      b = hi;
    }
    shallow_item<true>(t, q, out, s, live, i, a, b, flags, lane, st);
  }
  for (int o = 32; o > 0; o >>= 1) {
    st.q += __shfl_down(st.q, o, 64);
    st.nodes += __shfl_down(st.nodes, o, 64);
    st.payload += __shfl_down(st.payload, o, 64);
  }
  if (lane == 0 && st.q) {
    atomicAdd(&out.stats[kStatShallow], (unsigned long long)st.q);
    atomicAdd(&out.stats[kStatNodes], (unsigned long long)st.nodes);
    atomicAdd(&out.stats[kStatPayload], (unsigned long long)st.payload);
  }
}
__global__ __launch_bounds__(kWG) void k_explain_expand(TableArgs t, QueryArgs q, OutArgs out) {
  __shared__ Lds s;
  expand_body(t, q, out, s, (int64_t)blockIdx.x * (kWG / 64) + (threadIdx.x >> 6), (int64_t)gridDim.x * (kWG / 64));
}

// ---------------------------------------------------------------------------
// Result materialisation -- k_result_pack, once per pass (and again after a
// deferred-class launch): the dense hit list and the dense payload every
// consumer reads (include/sst.h, sst_result_hit_list).
//   * block b packs scan workgroup b's 16 waves: its place in the dense
//     output is the prefix of the workgroup tallies before it plus the
//     prefix of its own waves' tallies; each wave turns its scan wave's 8-B
//     hit records into 16-B dense records (payload offsets from a wavefront
//     prefix sum of the byte counts) and copies the wave's payload region in
//     16-B pieces;
//   * the deferred paths' hit records and spill bytes follow the scan's,
//     spread over the whole grid;
//   * block 0 writes the header (sizes, routed windows, retry counters) to
//     HBM and to host-mapped memory, so that the host can settle the pass
//     without a copy.
// ---------------------------------------------------------------------------

// Latency shape: every load the block needs in the common case -- the
// workgroup tallies, its waves' tallies, the first 4 x 64 hit records and the
// first 2 KB of payload of each wave -- is issued in one round before any of
// them is used (the record and payload loads speculatively, with clamped
// indices: the worklist and arena regions are always allocated that far), so
// a block costs one memory round trip plus one workgroup reduction; larger
// waves loop.  Sums are u32: hit records (< 2^32 queries) and 16-B units.
constexpr int kPackRec = 4;  // hit records per lane in the first round
constexpr int kPackPay = 2;  // 16-B payload pieces per lane in the first round

__global__ __launch_bounds__(1024, 8) void k_result_pack(PackArgs p) {  // 2 blocks per CU
  const int t = threadIdx.x, lane = t & 63, wv = __builtin_amdgcn_readfirstlane(t >> 6);
  const int b = blockIdx.x;
  const bool scan_part = b < p.n_wg && !p.scan_packed;  // a fused scan placed its own part already
  const uint64_t w = (uint64_t)b * 16 + wv;  // wave-uniform: region bases stay in SGPRs
  // ---- round 1: issue every load (no barrier: each wave sums the workgroup
  // tallies itself, 8 B per scan workgroup from L2)
  const uint32_t nd = *(const uint32_t*)(p.ctl + kCtlDhits);  // deferred hit records
  const uint64_t cursor = p.ctl[kCtlCursor];
  const uint2 wtv = scan_part ? p.tally[(int64_t)b * 16 + (lane & 15)] : make_uint2(0, 0);
  // (plain variables, not arrays: an array here is promoted to LDS)
  uint2 r0 = make_uint2(0, 0), r1 = r0, r2 = r0, r3 = r0;
  uint4 pay0 = make_uint4(0, 0, 0, 0), pay1 = pay0;
  // record k of the wave sits at rec[top - k] (filled from the region's end)
  const uint2* rec = (const uint2*)(p.work + w * p.work_region);
  const uint32_t top = (uint32_t)(2 * p.work_region - 1);  // work_region < 2^31 (host checks)
  const uint4* src = (const uint4*)(p.arena + w * p.region_bytes);
  if (scan_part) {
    const uint32_t last_pay = (uint32_t)min<uint64_t>(p.region_bytes >> 4, 0xFFFFFFFFull) - 1;
    r0 = rec[top - min((uint32_t)lane, top)];
    r1 = rec[top - min((uint32_t)(64 + lane), top)];
    r2 = rec[top - min((uint32_t)(128 + lane), top)];
    r3 = rec[top - min((uint32_t)(192 + lane), top)];
    pay0 = src[min((uint32_t)lane, last_pay)];
    pay1 = src[min((uint32_t)(64 + lane), last_pay)];
  }
  // ---- workgroup prefix (< b) and totals of the scan's hit records / units
  uint32_t ph = 0, pu = 0, th = 0, tu = 0;
  for (int k0 = 0; k0 < p.n_wg; k0 += 8 * 64) {
    uint2 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = k0 + j * 64 + lane;
      v[j] = k < p.n_wg ? p.wg_tally[k] : make_uint2(0, 0);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = k0 + j * 64 + lane;
      th += v[j].x;
      tu += v[j].y;
      ph += k < b ? v[j].x : 0u;
      pu += k < b ? v[j].y : 0u;
    }
  }
  ph = wave_sum32(ph);
  pu = wave_sum32(pu);
  th = wave_sum32(th);
  tu = wave_sum32(tu);
  uint64_t tb = (uint64_t)tu << 4;  // scan payload bytes (16-B pieces)
  if (p.scan_packed) {  // the fused scan's totals (its header, read by the host)
    th = (uint32_t)p.scan_hits;
    tb = p.scan_bytes;
  }
  if (p.dbg & 8) {
    if (b == 0 && t == 0) p.hdr[0] = th + pu + ph + tu + r0.x + r1.x + r2.x + r3.x + pay0.x + pay1.x;
    return;
  }
  // ---- this wave's scan wave: dense hit records, then its payload region
  if (scan_part) {
    const uint32_t eh = wave_sum32(lane < wv ? wtv.x : 0u);
    const uint32_t eu = wave_sum32(lane < wv ? wtv.y : 0u);
    const uint32_t nh = (uint32_t)__builtin_amdgcn_readlane((int)wtv.x, wv);
    uint32_t n16 = (uint32_t)__builtin_amdgcn_readlane((int)wtv.y, wv);
    const uint64_t hbase = (uint64_t)ph + eh, pbase = ((uint64_t)pu + eu) << 4;
    uint64_t run = pbase;
    const uint32_t nhs = (p.dbg & 1) ? 0 : nh;
    if (nh > 0) run = pack_hits(p.hits + hbase, lane, nhs, r0, run);
    if (nh > 64) run = pack_hits(p.hits + hbase, 64 + lane, nhs, r1, run);
    if (nh > 128) run = pack_hits(p.hits + hbase, 128 + lane, nhs, r2, run);
    if (nh > 192) run = pack_hits(p.hits + hbase, 192 + lane, nhs, r3, run);
    for (uint32_t k0 = kPackRec * 64; k0 < nh; k0 += 64)
      run = pack_hits(p.hits + hbase, k0 + lane, nh, rec[top - min(k0 + lane, nh - 1)], run);
    uint4* dst = (uint4*)(p.payload + pbase);
    if (p.dbg & 2) n16 = 0;
    if ((uint32_t)lane < n16) dst[lane] = pay0;
    if ((uint32_t)(64 + lane) < n16) dst[64 + lane] = pay1;
    for (uint32_t c = kPackPay * 64 + lane; c < n16; c += 64) dst[c] = src[c];
  }
  // ---- the deferred paths' records and spill bytes, behind the scan's
  const uint64_t spill_used = cursor < p.spill_cap ? cursor : p.spill_cap;
  const uint64_t gt = (uint64_t)b * 1024 + t, G = (uint64_t)gridDim.x * 1024;
  for (uint64_t k = gt; k < nd; k += G) {
    uint4 r = p.dhits[k];
    if (r.x & kHitOffsetFlag) {
      const uint64_t o = (((uint64_t)r.w << 32) | r.z) - p.spill_base + tb;
      r = make_uint4(r.x & ~kHitOffsetFlag, r.y, (uint32_t)o, (uint32_t)(o >> 32));
    }
    p.hits[(uint64_t)th + k] = r;
  }
  const uint64_t n16s = (spill_used + 15u) >> 4;
  const uint4* ssrc = (const uint4*)(p.arena + p.spill_base);
  uint4* sdst = (uint4*)(p.payload + tb);
  for (uint64_t c = gt; c < n16s; c += G) sdst[c] = ssrc[c];
  // ---- header
  if (b == 0 && t == 0) {
    const uint32_t* ctr = (const uint32_t*)(p.ctl + kCtlCounters);
    uint64_t h[kHdrWords];
    for (int k = 0; k < kHdrWords; ++k) h[k] = 0;
    h[kHdrHits] = (uint64_t)th + nd;
    h[kHdrPayload] = tb + spill_used;
    h[kHdrRouted] = (uint64_t)ctr[0] + ctr[1] + ctr[2] + ctr[3];
    h[kHdrExactRetries] = p.ctl[kCtlExactRetries];
    h[kHdrArenaRetries] = p.ctl[kCtlArenaRetries];  // spill overflows: the host compares the cursor
    h[kHdrCursor] = cursor;
    h[kHdrPass] = p.pass_id;
    h[kHdrRegionNeed] = p.ctl[kCtlRegionNeed];
    write_header(p.hdr, (p.dbg & 4) ? nullptr : p.hdr_host, h);
  }
}

// Per-query count[] / offset[] arrays from the dense hit list (only for
// callers that ask for them: sst_result_device).  Queries without candidates
// keep undefined entries (include/sst.h).
__global__ __launch_bounds__(256) void k_hits_to_arrays(const uint4* __restrict__ hits, uint64_t n_hits,
                                                        const int8_t* __restrict__ status, uint64_t* __restrict__ count,
                                                        uint64_t* __restrict__ offset) {
  const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= n_hits) return;
  const uint4 r = hits[k];
  const uint64_t word = ((uint64_t)r.w << 32) | r.z;
  if (status[r.x] == SST_SOME) {
    count[r.x] = r.y;
    offset[r.x] = word;
  } else {
    count[r.x] = word;
    offset[r.x] = 0;
  }
}

// ---------------------------------------------------------------------------
// The gather's wire format v5 (sst_wire_pack): one launch, a role per block
// range, every output byte written by exactly one thread except the list
// entries (the rare rest: is_valid raises, statuses other than NONE /
// SOME, pair hits whose count is not 1..7), whose slots a block takes with one
// atomic (wire_slots).  HBM-bound byte work: each thread reads
// 8 code or status bytes (or 10 hit records) and writes one output
// byte (or word); no LDS beyond the block's slot arithmetic.

// 8 code bytes from q0 on (bytes past n read as 0)
__device__ __forceinline__ uint64_t wire_load8(const int8_t* p, int64_t q0, int64_t n) {
  if (q0 + 8 <= n && ((uintptr_t)(p + q0) & 7) == 0) return *(const uint64_t*)(p + q0);
  uint64_t v = 0;
  for (int k = 0; k < 8; ++k)
    if (q0 + k < n) v |= (uint64_t)(uint8_t)p[q0 + k] << (8 * k);
  return v;
}

// First list slot of this thread's n_mine entries: a block-wide prefix sum
// and one atomic on the header's counter (zeroed by the host before the
// launch) per block that has any; blocks without entries only pay the
// barrier.  Entries come in no particular order.  Block-uniform call.
__device__ __forceinline__ uint64_t wire_slots(const WireArgs& a, uint32_t n_mine) {
  __shared__ uint32_t s_wave[4];
  __shared__ unsigned long long s_base;
  if (!__syncthreads_or(n_mine != 0)) return 0;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t incl = n_mine;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) s_wave[wv] = incl;
  __syncthreads();
  if (threadIdx.x == 0)
    s_base = atomicAdd((unsigned long long*)(a.out + 8 * kWireListWord),
                       (unsigned long long)(s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3]));
  __syncthreads();
  uint64_t base = s_base + incl - n_mine;
  for (int w = 0; w < wv; ++w) base += s_wave[w];
  return base;
}

__device__ __forceinline__ void wire_entry(const WireArgs& a, uint64_t pos, uint32_t type, uint64_t idx,
                                           uint32_t value) {
  if (pos < a.list_cap) ((uint2*)(a.out + a.o_list))[pos] = make_uint2((type << 30) | (uint32_t)idx, value);
}

__global__ __launch_bounds__(256) void k_wire_pack(WireArgs a) {
  const uint32_t b = blockIdx.x;
  if (b == 0 && threadIdx.x < kWireHeaderWords && threadIdx.x != kWireListWord)  // the counter stays the host's zero
    ((uint64_t*)a.out)[threadIdx.x] = a.hdr[threadIdx.x];
  if (b < a.be_v) {  // valid: byte t = 8 queries' bits (True); raises listed
    const uint64_t t = (uint64_t)b * 256 + threadIdx.x;
    const bool act = t < a.nb_v;
    const uint64_t v = act ? wire_load8(a.valid, (int64_t)t * 8, a.n7) : 0;
    uint32_t bits = 0, exc = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int8_t c = (int8_t)(v >> (8 * k));
      bits |= (uint32_t)(c == 1) << k;
      exc |= (uint32_t)(act && (int64_t)t * 8 + k < a.n7 && c == -1) << k;
    }
    if (act) a.out[a.o_vbits + t] = (uint8_t)bits;
    uint64_t pos = wire_slots(a, __builtin_popcount(exc));
    for (; exc; exc &= exc - 1) wire_entry(a, pos++, 0u, t * 8 + __builtin_ctz(exc), 0u);
    return;
  }
  if (b < a.be_s) {  // status: byte t = 8 queries' hit bits (SOME / OVERFLOW / ABORTED); statuses other
                     // than NONE / SOME listed (EMPTY is rare: a window reaching mass 0)
    const uint64_t t = (uint64_t)(b - a.be_v) * 256 + threadIdx.x;
    const bool act = t < a.nb_s;
    const uint64_t v = act ? wire_load8(a.status, (int64_t)t * 8, a.n8) : 0;
    uint32_t bits = 0, exc = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int8_t c = (int8_t)(v >> (8 * k));
      bits |= (uint32_t)(c == SST_SOME || c == SST_OVERFLOW || c == SST_ABORTED) << k;
      exc |= (uint32_t)(act && (int64_t)t * 8 + k < a.n8 && c != SST_NONE && c != SST_SOME) << k;
    }
    if (act) a.out[a.o_sbits + t] = (uint8_t)bits;
    uint64_t pos = wire_slots(a, __builtin_popcount(exc));
    for (; exc; exc &= exc - 1) {
      const int k = __builtin_ctz(exc);
      wire_entry(a, pos++, 1u, t * 8 + k, (uint32_t)(uint8_t)(v >> (8 * k)));
    }
    return;
  }
  if (b < a.be_f) {  // u32 word t of the w-bit first entries (field i at bits i*w ..)
    const uint64_t t = (uint64_t)(b - a.be_s) * 256 + threadIdx.x;
    if (t >= a.nw_f) return;
    const uint64_t lo = t * 32, w = (uint64_t)a.w;
    uint32_t word = 0;
    for (uint64_t i = lo / w; i * w < lo + 32 && i < a.n_pair; ++i) {
      const uint64_t f = a.refs[i] & 0x7FFFu;
      const int64_t sh = (int64_t)(i * w) - (int64_t)lo;
      word |= (uint32_t)(sh >= 0 ? f << sh : f >> -sh);
    }
    ((uint32_t*)(a.out + a.o_first))[t] = word;
    return;
  }
  if (b < a.be_c) {  // u32 word t of the 3-bit count codes (10 per word): 1..7, 0 = listed count
    const uint64_t t = (uint64_t)(b - a.be_f) * 256 + threadIdx.x;
    const bool act = t < a.nw_c;
    uint32_t word = 0, exc = 0;
    for (int k = 0; k < 10; ++k) {
      const uint64_t i = t * 10 + k;
      if (!act || i >= a.n_pair) break;
      const uint32_t c = a.hits[i].y;
      if (c >= 1 && c <= 7)
        word |= c << (3 * k);
      else
        exc |= 1u << k;
    }
    if (act) ((uint32_t*)(a.out + a.o_codes))[t] = word;
    uint64_t pos = wire_slots(a, __builtin_popcount(exc));
    for (; exc; exc &= exc - 1) {
      const uint64_t i = t * 10 + __builtin_ctz(exc);
      wire_entry(a, pos++, 2u, i, a.hits[i].y);
    }
    return;
  }
  if (b < a.be_e) {  // explicit record t {query | kind << 30, a, b}
    const uint64_t t = (uint64_t)(b - a.be_c) * 256 + threadIdx.x;
    if (t >= a.n_exp) return;
    const uint4 r = a.hits[a.n_pair + t];
    const int8_t s = a.status[r.x];
    const uint32_t kind = s == SST_OVERFLOW ? 1u : (s == SST_ABORTED ? 2u : 0u);
    const uint64_t off = (((uint64_t)r.w << 32) | r.z) - a.pair_bytes;
    uint32_t* o = (uint32_t*)(a.out + a.o_exp) + 3 * t;
    o[0] = r.x | (kind << 30);
    o[1] = kind == 0 ? r.y : r.z;
    o[2] = kind == 0 ? (uint32_t)off : r.w;
  }
}

#ifdef SST_DIAG_TIME  // timing builds only (tools/c1_time.py): per-wave phase clocks of the deep role
__device__ uint64_t g_diag_time[1 << 20];
#define DIAG_T(k)                                                                                        \
  do {                                                                                                   \
    const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                                                \
    if ((threadIdx.x & 63) == 0 && MODE == MODE_FAST)                                                    \
      g_diag_time[8 * ((int64_t)blk * (blockDim.x >> 6) + (threadIdx.x >> 6)) + (k)] = t_;               \
  } while (0)
#else
#define DIAG_T(k) \
  do {            \
  } while (0)
#endif

// The row mask of query i's alphabet (sst_explain_alpha_batch_device: its
// spectrum's reduced alphabet over this table's rows; all rows otherwise).
__device__ __forceinline__ M128 query_alpha(const QueryArgs& q, int64_t i) {
  if (!q.alpha) return M128{~0ull, ~0ull};
  const int64_t g = q.spec ? (int64_t)q.spec[i] : 0;
  return M128{q.alpha[2 * g], q.alpha[2 * g + 1]};
}
// A reduced table is rebuilt up to max(kept masses) * 35 (mass_table.py:
// 114-117, MAX_SEQ_LENGTH) with ceil((max_mass + 1) / C) words per row.  A
// window reaching its extent raises (status OUT_OF_TABLE, :134-138); one in
// its last word, whose bits the reference's last-column mask may clear
// (mass_table.py:246), is not modelled by the full table's rows: ABORTED.
__device__ __forceinline__ int8_t alpha_extent_status(const TableArgs& t, const QueryArgs& q, const Lds& s, M128 am,
                                                      int64_t hi) {
  if (!q.alpha) return SST_NONE;
  am = mand(am, rows_upto(t.n_rows - 1));
  const int top = am.b ? 127 - __builtin_clzll(am.b) : 63 - __builtin_clzll(am.a | 1ull);
  const int64_t max_mass = (int64_t)s.w[top] * 35;
  const int64_t lim = (max_mass + q.comp) / q.comp * q.comp;  // ceil((max_mass + 1) / C) * C
  if (hi >= lim) return SST_OUT_OF_TABLE;
  if (hi >= lim - q.comp) return SST_ABORTED;
  return SST_NONE;
}

// Deferred fast/no-memo queries with deep stacks: persistent grid, one lane per
// query, stack in a per-lane slice of the workspace.
template <int MODE, bool NW = false>
__device__ void deep_body(const TableArgs& t, const QueryArgs& q, const OutArgs& out, int cls, GlobFrame* ws, Lds& s,
                          int blk, int nblk) {
  DIAG_T(0);
  const uint32_t n_list = out.counters[cls];
  if (n_list == 0) return;  // block-uniform: nothing queued for this role
  stage_rows(s, t);
  const int64_t gid = (int64_t)blk * blockDim.x + threadIdx.x;
  const int64_t nthreads = (int64_t)nblk * blockDim.x;
  GlobStack st{ws + gid, (uint32_t)nthreads};
  DIAG_T(1);
  uint64_t st_n = 0, st_nodes = 0;
  // workgroup-uniform trip count: the payload allocation and the hit records
  // take one atomic per workgroup (wg_alloc), not one per wave or query
  for (int64_t jb = (int64_t)blk * blockDim.x; jb < (int64_t)n_list; jb += nthreads) {
    const int64_t j = jb + threadIdx.x;
    const bool live = j < (int64_t)n_list;
    int64_t i = 0, a = 1, b = 0;
    int A0 = 0;
    EnumOut eo{0, 0, 0, 0};
    int8_t status = SST_NONE;
    uint64_t bytes = 0;
    RegSinkPaths rs;  // the first two candidates' paths, kept by the counting DFS
    M128 am{~0ull, ~0ull};
    if (live) {
      i = out.lists[(int64_t)cls * q.n + j];
      am = query_alpha(q, i);
      int64_t lo, hi;
      quantise(q.mass[i], q.thr ? q.thr[i] : 0.0, q.thr == nullptr, q.tol, q.prec, q.rprec, lo, hi);
      A0 = clamp_budget(q.max_mods ? q.max_mods[i] : q.max_mods_scalar);
      const bool has_zero = lo <= 0 && hi >= 0;
      a = lo < 1 ? 1 : lo;
      b = hi;
      const int8_t ext = alpha_extent_status(t, q, s, am, b);
      if (ext != SST_NONE) a = 1, b = 0;  // nothing to enumerate
      DIAG_T(2);
      enumerate_window<MODE, NW>(t, s, st, nullptr, a, b, A0, rs, q.node_budget, eo, am);
      status = eo.count ? SST_SOME : (has_zero ? SST_EMPTY : SST_NONE);
      bytes = eo.bytes;
      if (ext != SST_NONE) {
        status = ext;
        bytes = 0;
      } else if (eo.fail) {
        status = SST_ABORTED;
        bytes = 0;
      } else if (eo.count > q.cap_count) {
        status = SST_OVERFLOW;
        bytes = 0;
      }
    }
    if (out.dbg & 4) {  // DIAGNOSTIC 4: the counting DFS only
      if (live) {
        st_n++;
        st_nodes += eo.nodes;
      }
      continue;
    }
    DIAG_T(3);
    const TileOut to = spill_alloc_wg(out, bytes, status);
    DIAG_T(4);
    if (to.bytes && !rs.over) {
      rs.flush(out.payload + to.off, to.bytes);
    } else if (to.bytes) {  // more than 32 bytes: enumerate again straight into the arena
      MemSink ms{out.payload + to.off, ~0ull};
      EnumOut e2{0, 0, 0, 0};
      enumerate_window<MODE, NW>(t, s, st, nullptr, a, b, A0, ms, ~0ull, e2, am);
    }
    emit_result_wg(out, live, (uint32_t)i, to.status, eo.count, to.off);
    DIAG_T(5);
#ifdef SST_DIAG_TIME
    {
      uint32_t it = eo.iters;
      for (int o_ = 32; o_ > 0; o_ >>= 1) it = max(it, (uint32_t)__shfl_xor((int)it, o_, 64));
      if ((threadIdx.x & 63) == 0 && MODE == MODE_FAST)
        g_diag_time[8 * ((int64_t)blk * (blockDim.x >> 6) + (threadIdx.x >> 6)) + 7] = it;
    }
#endif
    if (live) {
      st_n++;
      st_nodes += eo.nodes;
    }
  }
  wg_stat(out.stats, MODE == MODE_FAST ? kStatDeep : kStatNomemo, st_n);
  DIAG_T(6);
  wg_stat(out.stats, kStatNodes, st_nodes);
}

// Deferred budget-binding queries: exact memo replay (phase 1) + enabled-DAG
// enumeration (phase 2).  Per lane: a hash slice and a frame slice.
__device__ void exact_body(const TableArgs& t, const QueryArgs& q, const OutArgs& out, ExactWs ws, Lds& s, int blk,
                           int64_t lanes) {
  const uint32_t n_list = out.counters[kClassExact];
  if (n_list == 0) return;  // block-uniform: nothing queued for this role
  stage_rows(s, t);
  const int64_t gid = (int64_t)blk * blockDim.x + threadIdx.x;
  const int64_t nthreads = lanes;  // the workspace's lanes (a multiple of 64; the last workgroup may have idle waves)
  if (gid - (threadIdx.x & 63) >= lanes) return;  // wave-uniform; no workgroup barrier follows
  P1Frame* fr = (P1Frame*)(ws.frames + gid * kMaxDepth * sizeof(P1Frame));
  GlobStack st{(GlobFrame*)ws.stacks + gid, (uint32_t)nthreads};
  Hash h;
  h.e = (HEntry*)(ws.hash + (size_t)gid * ws.hash_cap * sizeof(HEntry));
  h.mask = ws.hash_cap - 1;
  h.limit = (uint32_t)(ws.hash_cap * 0.7);
  h.cap = s.cap;
  h.capz0 = s.capz0;
  h.capz1 = s.capz1;
  uint64_t st_n = 0, st_nodes = 0;
  const int lane = threadIdx.x & 63;
  for (int64_t j0 = gid - lane; j0 < (int64_t)n_list; j0 += nthreads) {  // wave-uniform (see deep_body)
    const int64_t j = j0 + lane;
    const bool live = j < (int64_t)n_list;
    int64_t i = 0, a = 1, b = 0;
    int A0 = 0;
    int8_t status = SST_NONE;
    EnumOut eo{0, 0, 0, 0};
    uint64_t bytes = 0, nodes = 0;
    M128 am{~0ull, ~0ull};
    if (live) {
      i = out.lists[(int64_t)kClassExact * q.n + j];
      am = query_alpha(q, i);
      if (q.qlen) {  // this query's own budgets
        const int L = q.qlen[i];
        h.cap = q.caps_len + (int64_t)L * kMaxRows;
        h.capz0 = q.capz_len[2 * L];
        h.capz1 = q.capz_len[2 * L + 1];
      }
      int64_t lo, hi;
      quantise(q.mass[i], q.thr ? q.thr[i] : 0.0, q.thr == nullptr, q.tol, q.prec, q.rprec, lo, hi);
      A0 = clamp_budget(q.max_mods ? q.max_mods[i] : q.max_mods_scalar);
      const bool has_zero = lo <= 0 && hi >= 0;
      a = lo < 1 ? 1 : lo;
      b = hi;
      h.epoch = ++ws.epochs[gid];
      h.used = 0;
      const int8_t ext = alpha_extent_status(t, q, s, am, b);
      if (ext != SST_NONE) a = 1, b = 0;
      const int rc = ext != SST_NONE ? -4 : phase1<false>(t, s, h, fr, a, b, A0, q.node_budget, nodes, am);
      if (rc == -4) {
        status = ext;
      } else if (rc == -1) {
        status = (int8_t)kStatusExactRetry;
        atomicAdd(out.exact_retries, 1ull);  // lets the host see it without a status scan (settle)
      } else if (rc < 0) {
        status = SST_ABORTED;
      } else {
        CountSink cs;
        enumerate_window<MODE_EXACT>(t, s, st, &h, a, b, A0, cs, q.node_budget, eo);
        status = eo.count ? SST_SOME : (has_zero ? SST_EMPTY : SST_NONE);
        bytes = eo.bytes;
        if (eo.fail) {
          status = SST_ABORTED;
          bytes = 0;
        } else if (eo.count > q.cap_count) {
          status = SST_OVERFLOW;
          bytes = 0;
        }
      }
    }
    const TileOut to = spill_alloc(out, lane, bytes, status);
    if (to.bytes) {
      MemSink ms{out.payload + to.off, ~0ull};
      EnumOut e2{0, 0, 0, 0};
      enumerate_window<MODE_EXACT>(t, s, st, &h, a, b, A0, ms, ~0ull, e2);
    }
    emit_result(out, live, (uint32_t)i, to.status, eo.count, to.off);
    if (live) {
      st_n++;
      st_nodes += nodes + eo.nodes;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {  // per wave (waves of this role may have left early)
    st_n += __shfl_down(st_n, o, 64);
    st_nodes += __shfl_down(st_nodes, o, 64);
  }
  if ((threadIdx.x & 63) == 0 && st_n) {
    atomicAdd(&out.stats[kStatExact], (unsigned long long)st_n);
    atomicAdd(&out.stats[kStatNodes], (unsigned long long)st_nodes);
  }
}

// The pair scan's tail in one launch (64-lane blocks, partitioned by block
// index): SHALLOW windows (the scan waves' worklists), deep fast path, deep
// no-memo, exact replay.  The scan routed every window, so the roles are
// independent; each exits at once when its list is empty, so an idle pass
// costs one launch.  shallow_blocks = 0 after k_bitset_scan (its windows go to
// k_explain_expand, which routes them).
__global__ __launch_bounds__(kDefWG) void k_explain_deferred(TableArgs t, QueryArgs q, OutArgs out, GlobFrame* ws_deep,
                                                             ExactWs ws, int shallow_blocks, int deep_blocks,
                                                             int exact_lanes) {
  __shared__ Lds s;
  int b = blockIdx.x;
  if (b < shallow_blocks) {
    if (!(out.dbg & 1)) shallow_list_body(t, q, out, s, b, shallow_blocks);  // DIAGNOSTIC 1: no SHALLOW role
    return;
  }
  b -= shallow_blocks;
  if (out.dbg & 2) return;  // DIAGNOSTIC 2: no deep / exact roles
  if (b < deep_blocks) {
    if (t.n_rows <= 64)  // the canonical and most reduced tables: one mask word
      deep_body<MODE_FAST, true>(t, q, out, kClassDeep, ws_deep, s, b, deep_blocks);
    else
      deep_body<MODE_FAST>(t, q, out, kClassDeep, ws_deep, s, b, deep_blocks);
  }
  else if (b < 2 * deep_blocks)  // second half of the deep workspace
    deep_body<MODE_NOMEMO>(t, q, out, kClassNomemo, ws_deep + (size_t)deep_blocks * kDefWG * kMaxDepth, s,
                           b - deep_blocks, deep_blocks);
  else
    exact_body(t, q, out, ws, s, b - 2 * deep_blocks, exact_lanes);
}

// ---------------------------------------------------------------------------
// compute_sequence_length_bound (mass_table.py:343-487), batched.
//
// The reference's backtrack has the explain DFS's visit order, memo key
// (m, row) and budget flow exactly (up: B = cap[row-1]; left on a mod row:
// A-1, B-1 when A > 0 and B > 0), so the first-visit state per mass is the
// exact path's phase 1 (hv, enabled-left mask).  A node's memoised value is
//   value(m, r) = combine(default, value(m, r-1) [r > lo],
//                         value(m - w_r, r) + 1 [left enabled at first visit])
// = combine over rows s in [lo, r] of the enabled left contributions,
// combine = min (lower, default max_len+1) or max (upper, default -1).
//
// Fast path (budgets provably never bind, fast-path theorem): value(v, top)
// is the min / max item count of a multiset summing to v, i.e. the min / max
// k with v in L_k, where L_0 = {0}, L_{k+1} = U_r (L_k + w_r) -- layered
// bitsets built per call, one lane per query.
// ---------------------------------------------------------------------------
// L_{k+1} from L_k: one output word per thread, OR over the rows' shifts
__global__ void k_layer_step(const uint64_t* __restrict__ prev, uint64_t* __restrict__ next, int64_t nwords,
                             const int* __restrict__ w, int n_rows) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nwords) return;
  uint64_t acc = 0;
  for (int r = 1; r < n_rows; ++r) {
    const int64_t q = w[r] >> 6;
    const int sh = w[r] & 63;
    const int64_t jj = j - q;
    if (jj < 0) continue;
    uint64_t x = prev[jj] << sh;
    if (sh && jj > 0) x |= prev[jj - 1] >> (64 - sh);
    acc |= x;
  }
  next[j] = acc;
}


// saved ancestors of the value DP (the current frame is in registers)
struct LBFrame {
  HEntry* e;
  uint32_t m;
  int acc;
  uint8_t r, hv, pad0, pad1;
};

// values of mass `root` (and every descendant it needs), per row lo..hv in
// vals[slot * kMaxRows + row]; 0 ok, -2 depth, -3 inconsistent memo
__device__ int lb_values(const TableArgs& t, const Lds& s, const Hash& h, int8_t* vals, LBFrame* fr, HEntry* root_e,
                         uint32_t root, int dir, int dflt) {
  HEntry* e = root_e;
  uint32_t m = root;
  int acc = dflt;
  int r = (int)((e->meta >> 16) & 0xFF), hv = (int)(e->meta & 0xFF);
  M128 en{e->en0, e->en1};
  int d = 0;
  for (;;) {
    if (r > hv) {
      e->pad = 1;  // values computed
      if (d == 0) return 0;
      const LBFrame f = fr[--d];  // resume the parent at its pending row (the child is now computed)
      e = f.e;
      m = f.m;
      acc = f.acc;
      r = f.r;
      hv = f.hv;
      en = M128{e->en0, e->en1};
      continue;
    }
    if (mtest(en, r)) {
      const uint32_t c = m - (uint32_t)s.w[r];
      int cv = 0;  // total_mass == 0 -> 0 (mass_table.py:378-379)
      if (c != 0) {
        HEntry* ce = h.find(c);  // visited by phase 1 (the edge was taken)
        if (!ce) return -3;      // cannot happen for a consistent table; never dereference
        if (ce->pad == 0) {
          if (d + 1 >= kMaxDepth) return -2;
          fr[d++] = LBFrame{e, m, acc, (uint8_t)r, (uint8_t)hv, 0, 0};
          e = ce;
          m = c;
          acc = dflt;
          r = (int)((ce->meta >> 16) & 0xFF);
          hv = (int)(ce->meta & 0xFF);
          en = M128{ce->en0, ce->en1};
          continue;
        }
        cv = vals[(size_t)(ce - h.e) * kMaxRows + r];
      }
      acc = lb_combine(dir, acc, cv + 1);
    }
    vals[(size_t)(e - h.e) * kMaxRows + r] = (int8_t)acc;  // combine(default, rows lo..r)
    ++r;
  }
}

// lb_values with one query per wave.  Values are a pure function of the
// phase-1 DAG, so a node first computes every uncomputed child (depth first,
// ascending rows), then all its rows at once: lane r loads child r's value
// and a wavefront prefix min / max over rows lo..hv gives
// vals[node][r] = combine(default, rows lo..r).  One probe round per node
// instead of one dependent look-up per row.
struct LBWFrame {
  uint64_t u0, u1;  // rows whose child still has to be computed
  HEntry* e;
  uint32_t m;
  uint32_t pad;
};
__device__ __forceinline__ M128 lb_uncomputed(const TableArgs& t, const Lds& s, const Hash& h, const HEntry* e,
                                              uint32_t m, bool& bad, uint32_t pass) {
  const int lane = threadIdx.x & 63;
  const M128 en{e->en0, e->en1};
  bool u[2], miss = false;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int r = lane + 64 * half;
    u[half] = false;
    if (r < t.n_rows && mtest(en, r) && m != (uint32_t)s.w[r]) {
      const HEntry* ce = h.find(m - (uint32_t)s.w[r]);  // visited by phase 1 (the edge was taken)
      miss |= ce == nullptr;
      u[half] = ce && ce->pad != pass;
    }
  }
  bad = __ballot(miss) != 0;
  return M128{(uint64_t)__ballot(u[0]), (uint64_t)__ballot(u[1])};
}
// pass: the value of `pad` that marks a node computed by this pass (one
// phase 1 can feed two passes, the lower and the upper bound)
__device__ int lb_values_wave(const TableArgs& t, const Lds& s, const Hash& h, int8_t* vals, LBWFrame* fr,
                              HEntry* root_e, uint32_t root, int dir, int dflt, uint32_t pass = 1) {
  const int lane = threadIdx.x & 63;
  const int neutral = dir ? -128 : 127;  // identity of max / min over int8 values
  HEntry* e = root_e;
  uint32_t m = root;
  bool bad = false;
  M128 u = lb_uncomputed(t, s, h, e, m, bad, pass);
  if (bad) return -3;
  int d = 0;
  for (;;) {
    if (!mzero(u)) {  // compute the lowest uncomputed child first
      const int r = mlow(u);
      u = mclear(u, r);
      const uint32_t c = m - (uint32_t)s.w[r];
      HEntry* ce = h.find(c);
      if (!ce) return -3;
      if (ce->pad == pass) continue;  // computed meanwhile, inside an earlier sibling's subtree
      if (d + 1 >= kMaxDepth) return -2;
      fr[d++] = LBWFrame{u.a, u.b, e, m, 0};
      e = ce;
      m = c;
      u = lb_uncomputed(t, s, h, e, m, bad, pass);
      if (bad) return -3;
      continue;
    }
    // every child is computed: this node's rows lo..hv at once
    const int lo = (int)((e->meta >> 16) & 0xFF), hv = (int)(e->meta & 0xFF);
    const M128 en{e->en0, e->en1};
    int contrib[2];
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int r = lane + 64 * half;
      contrib[half] = neutral;
      if (r < t.n_rows && r >= lo && r <= hv && mtest(en, r)) {
        const uint32_t c = m - (uint32_t)s.w[r];
        int cv = 0;  // total_mass == 0 -> 0 (mass_table.py:378-379)
        if (c != 0) {
          const HEntry* ce = h.find(c);
          cv = ce ? vals[(size_t)(ce - h.e) * kMaxRows + r] : 0;
        }
        contrib[half] = cv + 1;
      }
    }
    const int p0 = lb_scan(dir, contrib[0]);
    const int tot0 = __shfl(p0, 63, 64);
    const int p1 = lb_combine(dir, lb_scan(dir, contrib[1]), tot0);
    int8_t* row = vals + (size_t)(e - h.e) * kMaxRows;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int r = lane + 64 * half;
      if (r < kMaxRows && r >= lo && r <= hv) row[r] = (int8_t)lb_combine(dir, dflt, half ? p1 : p0);
    }
    e->pad = pass;  // values computed
    if (d == 0) return 0;
    const LBWFrame f = fr[--d];
    u = M128{f.u0, f.u1};
    e = f.e;
    m = f.m;
  }
}

// per-query frame workspace of k_length_exact: phase-1 frames, then the value
// DP's frames (lane or wave form)
constexpr size_t kLBFrameBytes =
    kMaxDepth * (sizeof(P1Frame) + (sizeof(LBFrame) > sizeof(LBWFrame) ? sizeof(LBFrame) : sizeof(LBWFrame)));

__device__ __forceinline__ bool lb_window(const LBArgs& q, int64_t i, int64_t& lo, int64_t& hi) {
  const double obs = q.obs[i];
  quantise(q.su[i], q.tol * obs, false, q.tol, q.prec, q.rprec, lo, hi);  // mass_table.py:354-359
  return lo <= hi;
}

__device__ __forceinline__ int64_t lb_finish_len(int best, int dir, int max_len) {
  // mass_table.py:476-484: the default bound becomes 1 (lower) / max_len (upper)
  if (dir == 0) return best >= max_len + 1 ? 1 : best;
  return best == -1 ? max_len : best;
}
__device__ __forceinline__ int64_t lb_finish(const LBArgs& q, int best, int dir) {
  return lb_finish_len(best, dir, q.max_len);
}
__device__ __forceinline__ int64_t lb_finish(const LBArgs& q, int best) { return lb_finish(q, best, q.dir); }

__global__ __launch_bounds__(256) void k_length_fast(TableArgs t, LBArgs q) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= q.n) return;
  int64_t lo, hi;
  if (!lb_window(q, i, lo, hi)) {
    q.status[i] = (int8_t)kLBEmptyWindow;  // min([]) raises ValueError
    return;
  }
  if (hi >= t.limit) {
    q.status[i] = SST_OUT_OF_TABLE;  // NotImplementedError (mass_table.py:383-387)
    return;
  }
  if (q.alpha) {  // a reduced alphabet: its table's extent (as explain, §3), then the exact replay
    const int64_t g = q.spec ? (int64_t)q.spec[i] : 0;
    M128 am = mand(M128{q.alpha[2 * g], q.alpha[2 * g + 1]}, rows_upto(t.n_rows - 1));
    const int top = am.b ? 127 - __builtin_clzll(am.b) : 63 - __builtin_clzll(am.a | 1ull);
    const int64_t lim = ((int64_t)t.w[top] * 35 + q.comp) / q.comp * q.comp;
    if (hi >= lim - q.comp) {
      q.status[i] = hi >= lim ? (int8_t)SST_OUT_OF_TABLE : (int8_t)SST_ABORTED;
      return;
    }
  }
  const int64_t a = lo < 0 ? 0 : lo;
  const bool fast = !q.alpha && q.layers && hi < q.layer_limit && budgets_never_bind(t, hi, q.A0);
  if (!fast) {
    const uint32_t slot = atomicAdd(q.exact_count, 1u);
    q.exact_list[slot] = (uint32_t)i;
    q.status[i] = (int8_t)kStatusPending;
    return;
  }
  const int dflt = q.dir ? -1 : q.max_len + 1;
  int best = dflt;
  if (a <= hi) {
    for (int k = 0; k < q.n_layers; ++k) {
      if (any_bits(q.layers + (int64_t)k * q.layer_words, a, hi)) {
        if (q.dir == 0) {
          best = k < best ? k : best;
          break;
        }
        best = k;
      }
    }
  }
  q.out[i] = lb_finish(q, best);
  q.status[i] = 0;
}

// one lane per queued query: phase 1 (first visits) + value DP; per-lane hash
// slice and value slice, fresh (zeroed) workspace per launch
// WAVE: one query per 64-lane block (the DFS state is wave-uniform, the
// lanes split the prefetch); else one query per lane.
template <bool WAVE>
__global__ __launch_bounds__(64) void k_length_exact(TableArgs t, LBArgs q, char* hash, int8_t* vals, char* frames,
                                                     uint32_t hash_cap) {
  __shared__ Lds s;
  const uint32_t n_list = *q.exact_count;
  if (n_list == 0) return;
  stage_rows(s, t);
  const int64_t gid = WAVE ? (int64_t)blockIdx.x : (int64_t)blockIdx.x * 64 + threadIdx.x;
  const int64_t nthreads = WAVE ? (int64_t)gridDim.x : (int64_t)gridDim.x * 64;
  __shared__ P1Frame wfr[WAVE ? kMaxDepth : 1];  // wave mode: the replay's saved frames
  P1Frame* gfr = (P1Frame*)(frames + gid * kLBFrameBytes);
  P1Frame* fr = WAVE ? wfr : gfr;
  LBFrame* lf = (LBFrame*)(gfr + kMaxDepth);
  Hash h;
  h.e = (HEntry*)(hash + (size_t)gid * hash_cap * sizeof(HEntry));
  h.mask = hash_cap - 1;
  h.limit = hash_cap / 4;  // load factor <= 1/4: a wave waits for its longest probe chain
  h.cap = s.cap;
  h.capz0 = s.capz0;
  h.capz1 = s.capz1;
  const bool fuse = WAVE && q.fuse;  // both bounds' values in phase 1 (two dense value slices per wave)
  int8_t* lv = fuse ? vals + (size_t)gid * (hash_cap / 4) * kValSlots * 2 : vals + (size_t)gid * hash_cap * kMaxRows;
  if (fuse) {
    h.vals_lo = lv;
    h.vals_hi = lv + (size_t)(hash_cap / 4) * kValSlots;
    h.dense = true;
  }
  uint64_t epoch = 0;
  const int top = t.n_rows - 1;
  for (int64_t j = gid; j < (int64_t)n_list; j += nthreads) {
    const int64_t i = q.exact_list[j];
    int64_t lo, hi;
    lb_window(q, i, lo, hi);
    int A0 = q.A0, max_len = q.max_len;
    if (WAVE && q.qlen) {  // this query's budgets by its max_len (the block is one wave)
      const int L = q.qlen[i];
      const int lane = threadIdx.x & 63;
      bool z0 = false, z1 = false;
      if (lane < t.n_rows) {
        s.cap[lane] = q.caps_len[(int64_t)L * kMaxRows + lane];
        z0 = s.cap[lane] <= 0;
      }
      if (lane + 64 < t.n_rows) {
        s.cap[lane + 64] = q.caps_len[(int64_t)L * kMaxRows + lane + 64];
        z1 = s.cap[lane + 64] <= 0;
      }
      const uint64_t c0 = __ballot(z0), c1 = __ballot(z1);
      if (lane == 0) {
        s.capz0 = c0;
        s.capz1 = c1;
      }
      __syncthreads();
      A0 = q.a0_len[L];
      max_len = L;
      h.capz0 = s.capz0;
      h.capz1 = s.capz1;
    }
    h.epoch = ++epoch;  // the workspace was zeroed: epochs 1, 2, ... are fresh
    h.used = 0;
    h.dflt_lo = max_len + 1;
    uint64_t nodes = 0;
    const int64_t a = lo < 1 ? 1 : lo;
    M128 am{~0ull, ~0ull};
    if (q.alpha) {
      const int64_t g = q.spec ? (int64_t)q.spec[i] : 0;
      am = M128{q.alpha[2 * g], q.alpha[2 * g + 1]};
      if (WAVE && q.reach_bits) {  // the reduced table's pairs from its rows' reachability
        const int lane = threadIdx.x & 63;
        const M128 kept = mand(mand(am, rows_upto(t.n_rows - 1)), rows_from(1));
        const int n_lo = __builtin_popcountll(kept.a);
        const int r1 = lane + 64;
        const bool k0 = (kept.a >> lane) & 1ull, k1 = (kept.b >> lane) & 1ull;
        const int rank0 = k0 ? __builtin_popcountll(kept.a & ((1ull << lane) - 1ull)) : -1;
        const int rank1 = k1 ? n_lo + __builtin_popcountll(kept.b & ((1ull << lane) - 1ull)) : -1;
        __shared__ int s_krow[kMaxRows];
        if (k0) s_krow[rank0] = lane;
        if (k1) s_krow[rank1] = r1;
        __syncthreads();
        h.reach = true;
        h.rv.bits = q.reach_bits + q.reach_off[g];
        h.rv.W = q.reach_words[g];
        h.rv.K = n_lo + __builtin_popcountll(kept.b);
        h.rv.kept = kept;
        if (fuse && h.rv.K > kValSlots) {  // the dense value slots hold 64 kept rows: reported, not guessed
          q.status[i] = SST_ABORTED;
          continue;
        }
        h.rv.row0 = lane < h.rv.K ? s_krow[lane] : 0;
        h.rv.row1 = lane + 64 < h.rv.K ? s_krow[lane + 64] : 0;
        h.rv.w0 = s.w[h.rv.row0];
        h.rv.w1 = s.w[h.rv.row1];
        h.rv.rank0 = rank0;
        h.rv.rank1 = rank1;
        __syncthreads();
      }
    }
    h.vals_bad = false;
    int rc = phase1<WAVE>(t, s, h, fr, a, hi, A0, q.node_budget, nodes, am);
    if (rc == 0 && h.vals_bad) rc = -4;  // SST_ABORTED below
    if (q.nodes_out && (!WAVE || threadIdx.x == 0)) q.nodes_out[i] += nodes;
    if (rc == -1) {
      q.status[i] = (int8_t)kStatusExactRetry;
      continue;
    }
    if (rc == -3 && q.soft) {
      q.status[i] = (int8_t)kLBHeavy;
      continue;
    }
    if (rc < 0) {
      q.status[i] = SST_ABORTED;
      continue;
    }
    // the value DP over phase 1's DAG: one direction, or (both) the lower
    // bound then the upper from the same first visits (pass 1, 2); fused:
    // phase 1 already wrote both, the roots' top rows are combined here
    const int n_dir = WAVE && q.both ? 2 : 1;
    int64_t res[2] = {0, 0};
    if (fuse) {
      int bl = max_len + 1, bh = -1;
      if (lo <= 0 && hi >= 0) {  // total_mass == 0 -> 0
        bl = lb_combine(0, bl, 0);
        bh = lb_combine(1, bh, 0);
      }
      for (int64_t v = a; v <= hi && rc == 0; ++v) {
        if (h.reach ? !reach_bit(h.rv, h.rv.K - 1, v) : !((t.valid[v >> 6] >> (v & 63)) & 1ull)) continue;
        const HEntry* e = h.find((uint32_t)v);
        if (!e) {
          rc = -3;
          break;
        }
        const size_t at = (size_t)e->pad * kValSlots + (h.rv.K - 1);  // the top row's value: the highest kept row's
        bl = lb_combine(0, bl, h.vals_lo[at]);
        bh = lb_combine(1, bh, h.vals_hi[at]);
      }
      res[0] = lb_finish_len(bl, 0, max_len);
      res[1] = lb_finish_len(bh, 1, max_len);
    }
    for (int di = 0; di < n_dir && rc == 0 && !fuse; ++di) {
      const int dir = q.both ? di : q.dir;
      const uint32_t pass = (uint32_t)di + 1;
      const int dflt = dir ? -1 : max_len + 1;
      int best = dflt;
      if (lo <= 0 && hi >= 0) best = lb_combine(dir, best, 0);  // total_mass == 0 -> 0
      for (int64_t v = a; v <= hi && rc == 0; ++v) {
        // pair(top, v) == 0: default
        if (h.reach ? !reach_bit(h.rv, h.rv.K - 1, v) : !((t.valid[v >> 6] >> (v & 63)) & 1ull)) continue;
        HEntry* e = h.find((uint32_t)v);
        if (!e) {
          rc = -3;
          break;
        }
        if (e->pad != pass)
          rc = WAVE ? lb_values_wave(t, s, h, lv, (LBWFrame*)lf, e, (uint32_t)v, dir, dflt, pass)
                    : lb_values(t, s, h, lv, lf, e, (uint32_t)v, dir, dflt);
        if (rc == 0) best = lb_combine(dir, best, lv[(size_t)(e - h.e) * kMaxRows + top]);
      }
      res[di] = lb_finish_len(best, dir, max_len);
    }
    if (rc < 0) {
      q.status[i] = SST_ABORTED;
      continue;
    }
    q.out[i] = res[0];
    if (q.both) q.out_hi[i] = res[1];
    q.status[i] = 0;
  }
}

// ---------------------------------------------------------------------------
// explain_mass_with_recursion (mass_explanation.py:206-284), batched.
//
// dp(remaining, start, used_all, used_ind): budget check (:231-235, before
// the memo), memo keyed (remaining, start) holding the FIRST visit's list
// (:238-239), base cases |remaining| <= thr -> [[]] and remaining < 0 -> []
// (not memoised), then children i = start.. in ascending order with
// used_all + is_mod(i) and used_ind = (i != start ? 0 : used_ind + is_mod(i)).
// Phase 1 replays the DFS and stores, per memoised node, the children that
// passed their budget check at the node's first visit; phase 2 enumerates
// that DAG (twice: count, then write).  One lane per query.
// ---------------------------------------------------------------------------
struct REntry {
  uint64_t key;  // epoch << 40 | start << 32 | remaining
  uint64_t en0, en1;
  uint64_t pad;
};
struct RHash {
  REntry* e;
  uint32_t mask;
  uint64_t epoch;
  uint32_t used, limit;
  __device__ __forceinline__ uint64_t key(uint32_t rem, int start) const {
    return (epoch << 40) | ((uint64_t)start << 32) | rem;
  }
  __device__ __forceinline__ uint32_t slot(uint32_t rem, int start) const {
    return ((rem * 0x9E3779B1u) ^ ((uint32_t)start * 0x85EBCA77u)) & mask;
  }
  __device__ __forceinline__ REntry* find(uint32_t rem, int start) const {
    const uint64_t k = key(rem, start);
    for (uint32_t i = slot(rem, start);; i = (i + 1) & mask) {
      const uint64_t x = e[i].key;
      if (x == k) return &e[i];
      if ((x >> 40) != epoch) return nullptr;
    }
  }
  __device__ __forceinline__ REntry* insert(uint32_t rem, int start) {  // caller checked absence
    if (used >= limit) return nullptr;
    const uint64_t k = key(rem, start);
    for (uint32_t i = slot(rem, start);; i = (i + 1) & mask) {
      if ((e[i].key >> 40) != epoch) {
        ++used;
        e[i].key = k;
        return &e[i];
      }
    }
  }
};
// saved (not current) DFS frames: 16 B, in LDS.  The current frame lives in
// registers, so iterating a node's ~100 children touches no frame memory.
struct RFrame {
  uint32_t slot;  // memo entry
  uint32_t rem;
  int16_t ua, ui;
  uint8_t start, next, pad0, pad1;
};
constexpr int kRecLanes = 64;  // lanes (queries) per workgroup of the recursion kernel

// base case [[]]: abs(remaining) <= thr (:242-243) or remaining == 0 (:246-247)
__device__ __forceinline__ bool rec_leaf(int64_t rem, int64_t thr) { return (rem <= thr && rem >= -thr) || rem == 0; }

// children of (rem, start) that pass their budget check (:231-235)
__device__ __forceinline__ M128 rec_enabled(const TableArgs& t, const Lds& s, int start, int ua, int ui, int A) {
  M128 en = mand(rows_from(start), rows_upto(t.n_rows - 1));
  if (ua + 1 > A) {  // every modification child would exceed max_modifications
    en.a &= ~t.mod0;
    en.b &= ~t.mod1;
  }
  // a fresh row i != start carries used_ind = 0: blocked only if cap[i] < 0
  const bool keep_start = mtest(en, start) && ui + s.mod[start] <= s.cap[start];  // repeat of `start`
  en.a &= ~t.capneg0;
  en.b &= ~t.capneg1;
  en = keep_start ? (start < 64 ? M128{en.a | (1ull << start), en.b} : M128{en.a, en.b | (1ull << (start - 64))})
                  : mclear(en, start);
  return en;
}

// Overlap the memory latency of a node's child look-ups: one independent load
// per child's first probe slot (results folded into a sink the compiler must
// keep), so the sequential probes that follow hit the cache instead of paying
// one dependent HBM round trip each.
// WAVE (one query per wave): lane L takes children L and L + 64 and, one
// level deeper, the children (crem0 - w_j, j >= i0) of the first enabled
// child i0, the node the DFS most likely enters next.
template <bool WAVE>
__device__ __forceinline__ uint64_t rec_prefetch(const TableArgs& t, const Lds& s, const RHash& h, uint32_t rem,
                                                 M128 en, int64_t thr) {
  uint64_t sink = 0;
  if (WAVE) {
    const int lane = threadIdx.x & 63;
    const int i0 = mzero(en) ? kMaxRows : mlow(en);
    const int64_t crem0 = i0 < kMaxRows ? (int64_t)rem - s.w[i0] : -1;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int i = lane + 64 * half;
      if (i < t.n_rows) {
        const int64_t crem = (int64_t)rem - s.w[i];
        if (mtest(en, i) && crem > thr) sink ^= __builtin_nontemporal_load(&h.e[h.slot((uint32_t)crem, i)].key);
        const int64_t g = crem0 - s.w[i];
        if (i >= i0 && crem0 > thr && g > thr) sink ^= __builtin_nontemporal_load(&h.e[h.slot((uint32_t)g, i)].key);
      }
    }
    return sink;
  }
  for (M128 k = en; !mzero(k);) {
    const int i = mlow(k);
    k = mclear(k, i);
    const int64_t crem = (int64_t)rem - s.w[i];
    if (crem > thr) sink ^= __builtin_nontemporal_load(&h.e[h.slot((uint32_t)crem, i)].key) ^ 0;
  }
  return sink;
}

// phase 1: 0 ok, -1 memo full, -2 depth, -3 node budget.  stk: this lane's
// kMaxDepth saved frames (LDS, stride kRecLanes).
template <bool WAVE>
__device__ int rec_phase1(const TableArgs& t, const Lds& s, RHash& h, RFrame* stk, uint32_t target, int64_t thr,
                          int A, uint64_t node_budget, uint64_t& nodes) {
  REntry* e = h.insert(target, 1);
  if (!e) return -1;
  M128 rest = rec_enabled(t, s, 1, 0, 0, A);
  e->en0 = rest.a;
  e->en1 = rest.b;
  uint32_t slot = (uint32_t)(e - h.e), rem = target;
  int ua = 0, ui = 0, start = 1, d = 0;
  uint64_t sink = rec_prefetch<WAVE>(t, s, h, rem, rest, thr);
  for (;;) {
    if (mzero(rest)) {
      if (d == 0) break;
      const RFrame f = stk[(--d) * (WAVE ? 1 : kRecLanes)];
      const REntry* pe = h.e + f.slot;
      slot = f.slot;
      rem = f.rem;
      ua = f.ua;
      ui = f.ui;
      start = f.start;
      rest = mand(M128{pe->en0, pe->en1}, rows_from(f.next));
      continue;
    }
    const int i = mlow(rest);
    rest = mclear(rest, i);
    const int64_t crem = (int64_t)rem - s.w[i];
    if (rec_leaf(crem, thr) || crem < 0) continue;  // [[]] / []: base cases, not memoised
    if (h.find((uint32_t)crem, i)) continue;          // memo hit: the first visit's list
    if (++nodes > node_budget) return -3;
    if (d + 1 >= kMaxDepth) return -2;
    const int cua = ua + s.mod[i];
    const int cui = i != start ? 0 : ui + s.mod[i];
    REntry* ce = h.insert((uint32_t)crem, i);
    if (!ce) return -1;
    const M128 cen = rec_enabled(t, s, i, cua, cui, A);
    ce->en0 = cen.a;
    ce->en1 = cen.b;
    stk[(d++) * (WAVE ? 1 : kRecLanes)] = RFrame{slot, rem, (int16_t)ua, (int16_t)ui, (uint8_t)start, (uint8_t)(i + 1), 0, 0};
    slot = (uint32_t)(ce - h.e);
    rem = (uint32_t)crem;
    ua = cua;
    ui = cui;
    start = i;
    rest = cen;
    sink ^= rec_prefetch<WAVE>(t, s, h, rem, rest, thr);
  }
  return __ballot(sink == 0x5bd1e9955bd1e995ull) ? 1 : 0;  // (never) keeps every lane's prefetch loads alive
}

// Phase 1 with one query per wave.  A node's children (rem - w_i, i) have
// pairwise distinct keys, and no node inside child i's subtree can carry a
// later sibling's key (its start row would be that sibling's row j with
// w_i + ... = w_j over rows i <= ... <= j, impossible for positive masses).
// So every sibling's memo state at the moment the reference reaches it equals
// its state when the parent is first entered: the lanes probe all children at
// once (lane L: rows L and L + 64) and the DFS then walks only the children
// that need a first visit, in ascending row order -- the reference's order.
struct RWFrame {
  uint64_t d0, d1;  // children still to descend into
  uint32_t slot, rem;
  int16_t ua, ui;
  uint8_t start, pad0, pad1, pad2;
};
__device__ __forceinline__ M128 rec_descend_mask(const TableArgs& t, const Lds& s, const RHash& h, uint32_t rem,
                                                 M128 en, int64_t thr, uint64_t& sink) {
  const int lane = threadIdx.x & 63;
  bool need[2];
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int i = lane + 64 * half;
    need[half] = false;
    if (i < t.n_rows && mtest(en, i)) {
      const int64_t crem = (int64_t)rem - s.w[i];
      // [[]] / [] base cases are not memoised; otherwise a memo miss is a first visit
      if (!rec_leaf(crem, thr) && crem >= 0) need[half] = h.find((uint32_t)crem, i) == nullptr;
    }
  }
  const M128 d{(uint64_t)__ballot(need[0]), (uint64_t)__ballot(need[1])};
  // prefetch the memo slots of the first descendant's children
  if (!mzero(d)) {
    const int i0 = mlow(d);
    const int64_t crem0 = (int64_t)rem - s.w[i0];
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int j = lane + 64 * half;
      if (j < t.n_rows && j >= i0) {
        const int64_t g = crem0 - s.w[j];
        if (g > thr) sink ^= __builtin_nontemporal_load(&h.e[h.slot((uint32_t)g, j)].key);
      }
    }
  }
  return d;
}
// Whether the node's memoised list (its first visit's) is non-empty: some
// enabled child is a [[]] base case or a memo node whose own list is non-empty
// (REntry::pad bit 0, set when that node completed -- children complete before
// their parents, and memo hits were completed earlier).  Lanes probe the
// children in one round.  Phase 2 then walks only non-empty subtrees.
__device__ __forceinline__ void rec_complete(const TableArgs& t, const Lds& s, const RHash& h, REntry* e,
                                             uint32_t rem, int64_t thr) {
  const int lane = threadIdx.x & 63;
  const M128 en{e->en0, e->en1};
  bool ne = false;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int i = lane + 64 * half;
    if (i < t.n_rows && mtest(en, i)) {
      const int64_t crem = (int64_t)rem - s.w[i];
      if (rec_leaf(crem, thr)) {
        ne = true;
      } else if (crem > 0) {
        const REntry* ce = h.find((uint32_t)crem, i);
        ne |= ce && (ce->pad & 1u);
      }
    }
  }
  if (__ballot(ne)) e->pad = 1;
}
__device__ int rec_phase1_wave(const TableArgs& t, const Lds& s, RHash& h, RWFrame* stk, uint32_t target,
                               int64_t thr, int A, uint64_t node_budget, uint64_t& nodes) {
  REntry* e = h.insert(target, 1);
  if (!e) return -1;
  uint64_t sink = 0;
  M128 en = rec_enabled(t, s, 1, 0, 0, A);
  e->en0 = en.a;
  e->en1 = en.b;
  e->pad = 0;
  uint32_t slot = (uint32_t)(e - h.e), rem = target;
  int ua = 0, ui = 0, start = 1, d = 0;
  M128 rest = rec_descend_mask(t, s, h, rem, en, thr, sink);
  for (;;) {
    if (mzero(rest)) {
      rec_complete(t, s, h, h.e + slot, rem, thr);  // every child of this node is done
      if (d == 0) break;
      const RWFrame f = stk[--d];
      slot = f.slot;
      rem = f.rem;
      ua = f.ua;
      ui = f.ui;
      start = f.start;
      rest = M128{f.d0, f.d1};
      continue;
    }
    const int i = mlow(rest);
    rest = mclear(rest, i);
    const uint32_t crem = rem - (uint32_t)s.w[i];
    if (++nodes > node_budget) return -3;
    if (d + 1 >= kMaxDepth) return -2;
    const int cua = ua + s.mod[i];
    const int cui = i != start ? 0 : ui + s.mod[i];
    REntry* ce = h.insert(crem, i);
    if (!ce) return -1;
    const M128 cen = rec_enabled(t, s, i, cua, cui, A);
    ce->en0 = cen.a;
    ce->en1 = cen.b;
    ce->pad = 0;
    stk[d++] = RWFrame{rest.a, rest.b, slot, rem, (int16_t)ua, (int16_t)ui, (uint8_t)start, 0, 0, 0};
    slot = (uint32_t)(ce - h.e);
    rem = crem;
    ua = cua;
    ui = cui;
    start = i;
    rest = rec_descend_mask(t, s, h, rem, cen, thr, sink);
  }
  return __ballot(sink == 0x5bd1e9955bd1e995ull) ? 1 : 0;  // (never) keeps every lane's prefetch loads alive
}

// Phase 2 with one query per wave: the candidates in the reference's list
// order (children ascending, each child's list in its own order), walking
// only the non-empty subtrees marked by phase 1.  At each node the lanes
// classify every enabled child in one probe round; a candidate's record is
// written with one byte per lane.  dst == nullptr counts.
struct RPFrame {
  uint64_t t0, t1;  // children still to emit / enter
  uint32_t rem;
  uint32_t pad;
};
__device__ __forceinline__ M128 rec_todo(const TableArgs& t, const Lds& s, const RHash& h, uint32_t rem,
                                         const REntry* e, int64_t thr) {
  const int lane = threadIdx.x & 63;
  const M128 en{e->en0, e->en1};
  bool go[2];
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int i = lane + 64 * half;
    go[half] = false;
    if (i < t.n_rows && mtest(en, i)) {
      const int64_t crem = (int64_t)rem - s.w[i];
      if (rec_leaf(crem, thr)) {
        go[half] = true;
      } else if (crem > 0) {
        const REntry* ce = h.find((uint32_t)crem, i);
        go[half] = ce && (ce->pad & 1u);
      }
    }
  }
  return M128{(uint64_t)__ballot(go[0]), (uint64_t)__ballot(go[1])};
}
__device__ int rec_enumerate_wave(const TableArgs& t, const Lds& s, const RHash& h, RPFrame* stk, uint8_t* path,
                                  uint32_t target, int64_t thr, uint8_t* dst, uint64_t& count, uint64_t& bytes) {
  const int lane = threadIdx.x & 63;
  const REntry* e = h.find(target, 1);
  if (!e) return -3;
  if (!(e->pad & 1u)) return 0;
  uint32_t rem = target;
  M128 todo = rec_todo(t, s, h, rem, e, thr);
  int d = 0;
  for (;;) {
    if (mzero(todo)) {
      if (d == 0) break;
      const RPFrame f = stk[--d];
      rem = f.rem;
      todo = M128{f.t0, f.t1};
      continue;
    }
    const int i = mlow(todo);
    todo = mclear(todo, i);
    path[d] = (uint8_t)i;
    const int64_t crem = (int64_t)rem - s.w[i];
    if (rec_leaf(crem, thr)) {  // a candidate: rows path[0..d] (ascending)
      if (dst && lane <= d + 1) dst[bytes + lane] = lane == 0 ? (uint8_t)(d + 1) : path[lane - 1];
      count++;
      bytes += (uint64_t)d + 2;
      continue;
    }
    const REntry* ce = h.find((uint32_t)crem, i);  // non-empty memo node (rec_todo)
    if (!ce) return -3;
    if (d + 1 >= kMaxDepth) return -2;
    stk[d++] = RPFrame{todo.a, todo.b, rem, 0};
    rem = (uint32_t)crem;
    todo = rec_todo(t, s, h, rem, ce, thr);
  }
  return 0;
}

// phase 2: candidates in the reference's list order; dst == nullptr counts.
// path: this lane's row per level (LDS, stride kRecLanes).
template <bool WAVE>
__device__ int rec_enumerate(const TableArgs& t, const Lds& s, const RHash& h, RFrame* stk, uint8_t* path,
                             uint32_t target, int64_t thr, uint8_t* dst, uint64_t cap_count, uint64_t& count,
                             uint64_t& bytes) {
  const REntry* e = h.find(target, 1);
  if (!e) return -3;
  uint32_t slot = (uint32_t)(e - h.e), rem = target;
  M128 rest = M128{e->en0, e->en1};
  int d = 0;
  while (true) {
    if (mzero(rest)) {
      if (d == 0) break;
      const RFrame f = stk[(--d) * (WAVE ? 1 : kRecLanes)];
      const REntry* pe = h.e + f.slot;
      slot = f.slot;
      rem = f.rem;
      rest = mand(M128{pe->en0, pe->en1}, rows_from(f.next));
      continue;
    }
    const int i = mlow(rest);
    rest = mclear(rest, i);
    path[d * (WAVE ? 1 : kRecLanes)] = (uint8_t)i;
    const int64_t crem = (int64_t)rem - s.w[i];
    if (rec_leaf(crem, thr)) {  // a candidate: rows path[0..d] (ascending)
      if (dst && count < cap_count) {
        dst[bytes] = (uint8_t)(d + 1);
        for (int k = 0; k <= d; ++k) dst[bytes + 1 + k] = path[k * (WAVE ? 1 : kRecLanes)];
      }
      count++;
      bytes += (uint64_t)d + 2;
      continue;
    }
    if (crem < 0) continue;
    const REntry* ce = h.find((uint32_t)crem, i);
    if (!ce) return -3;  // phase 1 memoised every non-base child it reached
    if (d + 1 >= kMaxDepth) return -2;
    stk[(d++) * (WAVE ? 1 : kRecLanes)] = RFrame{slot, rem, 0, 0, 0, (uint8_t)(i + 1), 0, 0};
    slot = (uint32_t)(ce - h.e);
    rem = (uint32_t)crem;
    rest = M128{ce->en0, ce->en1};
  }
  return 0;
}

// WAVE: one query per 64-lane block; the DFS state (and its LDS stack) is
// wave-uniform, the lanes split the prefetch loads.  Else one query per lane.
template <bool WAVE>
__global__ __launch_bounds__(kRecLanes) void k_explain_recursion(TableArgs t, QueryArgs q, OutArgs out, char* hash,
                                                                 uint32_t hash_cap) {
  constexpr int kLanesPerStack = WAVE ? 1 : kRecLanes;
  __shared__ Lds s;
  __shared__ RFrame stk_all[kMaxDepth * kLanesPerStack];  // 96 KB per block in lane mode
  __shared__ uint8_t path_all[kMaxDepth * kLanesPerStack];
  __shared__ RWFrame wstk[WAVE ? kMaxDepth : 1];           // phase 1 of the wave mode
  __shared__ RPFrame pstk[WAVE ? kMaxDepth : 1];           // phase 2 of the wave mode
  stage_rows(s, t);
  const int64_t gid = WAVE ? (int64_t)blockIdx.x : (int64_t)blockIdx.x * kRecLanes + threadIdx.x;
  const int64_t nthreads = WAVE ? (int64_t)gridDim.x : (int64_t)gridDim.x * kRecLanes;
  RFrame* stk = stk_all + (WAVE ? 0 : threadIdx.x);
  uint8_t* path = path_all + (WAVE ? 0 : threadIdx.x);
  RHash h;
  h.e = (REntry*)(hash + (size_t)gid * hash_cap * sizeof(REntry));
  h.mask = hash_cap - 1;
  h.limit = hash_cap / 4;  // load factor <= 1/4: a wave waits for its longest probe chain
  uint64_t epoch = 0;
  for (int64_t i = gid; i < q.n; i += nthreads) {
    int64_t target, thr;
    {
      int64_t lo, hi;  // lo = target - thr, hi = target + thr (mass_explanation.py:218-225)
      quantise(q.mass[i], q.thr ? q.thr[i] : 0.0, q.thr == nullptr, q.tol, q.prec, q.rprec, lo, hi);
      target = (lo + hi) / 2;
      thr = (hi - lo) / 2;
    }
    const int A = clamp_budget(q.max_mods ? q.max_mods[i] : q.max_mods_scalar);
    int8_t status;
    uint64_t count = 0, bytes = 0, off = 0;
    if (rec_leaf(target, thr)) {
      status = SST_EMPTY;  // [[]]: the empty composition only (:242-247)
    } else if (target < 0) {
      status = SST_NONE;  // [] (:250-251)
    } else if (target >= (int64_t)UINT32_MAX) {
      status = SST_ABORTED;
    } else {
      h.epoch = ++epoch;  // the workspace was zeroed: epochs 1, 2, ... are fresh
      h.used = 0;
      uint64_t nodes = 0;
      int rc = WAVE ? rec_phase1_wave(t, s, h, wstk, (uint32_t)target, thr, A, q.node_budget, nodes)
                    : rec_phase1<WAVE>(t, s, h, stk, (uint32_t)target, thr, A, q.node_budget, nodes);
      if (rc > 0) rc = 0;
      if (rc == 0)
        rc = WAVE ? rec_enumerate_wave(t, s, h, pstk, path, (uint32_t)target, thr, nullptr, count, bytes)
                  : rec_enumerate<WAVE>(t, s, h, stk, path, (uint32_t)target, thr, nullptr, 0, count, bytes);
      if (rc == -1) {
        status = (int8_t)kStatusExactRetry;
      } else if (rc < 0) {
        status = SST_ABORTED;
        count = 0;
      } else if (count == 0) {
        status = SST_NONE;
      } else if (count > q.cap_count) {
        status = SST_OVERFLOW;
      } else {
        status = SST_SOME;
        if (WAVE) {  // one allocation per wave, broadcast
          unsigned long long sb = 0;
          if ((threadIdx.x & 63) == 0) sb = atomicAdd((unsigned long long*)out.cursor, (unsigned long long)bytes);
          off = out.spill_base + (((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(sb >> 32)) << 32) |
                                  (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)sb));
        } else {
          off = out.spill_base + atomicAdd((unsigned long long*)out.cursor, (unsigned long long)bytes);
        }
        if (off + bytes > out.arena_bytes) {
          status = (int8_t)kStatusArenaRetry;
        } else {
          uint64_t c2 = 0, b2 = 0;
          if (WAVE)
            rec_enumerate_wave(t, s, h, pstk, path, (uint32_t)target, thr, out.payload + off, c2, b2);
          else
            rec_enumerate<WAVE>(t, s, h, stk, path, (uint32_t)target, thr, out.payload + off, ~0ull, c2, b2);
        }
      }
    }
    // WAVE: every lane holds the same query; lane 0 owns its hit record
    emit_result(out, true, (uint32_t)i, status, count, off, !WAVE || (threadIdx.x & 63) == 0);
  }
}

// ---------------------------------------------------------------------------
// host-side launchers (C++ linkage, used by sst_api.cpp)
// ---------------------------------------------------------------------------
static inline unsigned blocks_for(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

hipError_t launch_bits_seed(uint64_t* R0, int64_t nwords, hipStream_t st) {
  hipLaunchKernelGGL(k_bits_seed, dim3(blocks_for(nwords, 256)), dim3(256), 0, st, R0, nwords);
  return hipGetLastError();
}
hipError_t launch_bits_shift_or(uint64_t* dst, const uint64_t* src, int64_t k, int64_t nwords, int64_t nbits,
                                hipStream_t st) {
  hipLaunchKernelGGL(k_bits_shift_or, dim3(blocks_for(nwords, 256)), dim3(256), 0, st, dst, src, k, nwords, nbits);
  return hipGetLastError();
}
hipError_t launch_pack(int C, const uint64_t* R, int64_t rw, int n_rows, const int64_t* w, int64_t ncols, int64_t M,
                       uint64_t last_mask, const uint8_t* literal, void* out, hipStream_t st) {
  dim3 grid(blocks_for(ncols, 256), n_rows);
#define SST_PACK(CC) \
  hipLaunchKernelGGL(k_pack<CC>, grid, dim3(256), 0, st, R, rw, n_rows, w, ncols, M, last_mask, literal, out)
  switch (C) {
    case 4: SST_PACK(4); break;
    case 8: SST_PACK(8); break;
    case 16: SST_PACK(16); break;
    default: SST_PACK(32);
  }
#undef SST_PACK
  return hipGetLastError();
}
hipError_t launch_row_literal(int C, const uint64_t* Rprev, int64_t ncols, int shift, void* row, int64_t rw,
                              uint64_t* Rout, hipStream_t st) {
#define SST_ROW(CC)                                                                                   \
  hipLaunchKernelGGL(k_row_init<CC>, dim3(blocks_for(ncols, 256)), dim3(256), 0, st, Rprev, ncols, row); \
  hipLaunchKernelGGL(k_row_sweep_literal<CC>, dim3(1), dim3(64), 0, st, row, ncols, shift);            \
  hipLaunchKernelGGL(k_unpack_any<CC>, dim3(blocks_for(rw, 256)), dim3(256), 0, st, row, ncols, rw, Rout)
  switch (C) {
    case 4: SST_ROW(4); break;
    case 8: SST_ROW(8); break;
    case 16: SST_ROW(16); break;
    default: SST_ROW(32);
  }
#undef SST_ROW
  return hipGetLastError();
}
hipError_t launch_index(int C, const void* packed, int n_rows, int64_t ncols, int64_t M, ulonglong2* index,
                        uint64_t* valid, int* err, hipStream_t st) {
  dim3 grid(blocks_for(M, 256));
  switch (C) {
    case 4: hipLaunchKernelGGL(k_index<4>, grid, dim3(256), 0, st, packed, n_rows, ncols, M, index, valid, err); break;
    case 8: hipLaunchKernelGGL(k_index<8>, grid, dim3(256), 0, st, packed, n_rows, ncols, M, index, valid, err); break;
    case 16: hipLaunchKernelGGL(k_index<16>, grid, dim3(256), 0, st, packed, n_rows, ncols, M, index, valid, err); break;
    default: hipLaunchKernelGGL(k_index<32>, grid, dim3(256), 0, st, packed, n_rows, ncols, M, index, valid, err);
  }
  return hipGetLastError();
}
hipError_t launch_is_valid(const uint64_t* valid, int64_t limit, int64_t full_lo, int64_t full_hi, int64_t first_reach,
                           const double* mass, const double* thr, int64_t n, double tol, double prec, int8_t* out,
                           hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int grid = (int)blocks_for(n, 256);
  ValidArgs v{valid, limit, full_lo, full_hi, first_reach, mass, thr, n, tol, prec, 1.0 / prec, out};
  if (thr)
    hipLaunchKernelGGL(k_is_valid<true>, dim3(grid), dim3(256), 0, st, v);
  else
    hipLaunchKernelGGL(k_is_valid<false>, dim3(grid), dim3(256), 0, st, v);
  return hipGetLastError();
}
hipError_t launch_is_valid_peaks(const uint64_t* valid, int64_t limit, int64_t full_lo, int64_t full_hi,
                                 int64_t first_reach, const double* obs, int64_t n, const double* shifts, int n_w,
                                 double tol, double prec, int8_t* out, hipStream_t st) {
  if (n <= 0 || n_w <= 0) return hipSuccess;
  const int grid = (int)blocks_for(n, 256);
  ValidArgs v{valid, limit, full_lo, full_hi, first_reach, obs, nullptr, n, tol, prec, 1.0 / prec, out};
  PeakShifts sh{};  // 4 slots: the default branch below builds its own per group of 4
  for (int k = 0; k < n_w && k < 4; ++k) sh.shift[k] = shifts[k];
  switch (n_w) {  // the reference's breakage dicts: 4 weights (FULL_BREAKAGE_DICT: up to 16)
    case 1: hipLaunchKernelGGL(k_is_valid_peaks<1>, dim3(grid), dim3(256), 0, st, v, sh); break;
    case 2: hipLaunchKernelGGL(k_is_valid_peaks<2>, dim3(grid), dim3(256), 0, st, v, sh); break;
    case 3: hipLaunchKernelGGL(k_is_valid_peaks<3>, dim3(grid), dim3(256), 0, st, v, sh); break;
    case 4: hipLaunchKernelGGL(k_is_valid_peaks<4>, dim3(grid), dim3(256), 0, st, v, sh); break;
    default:
      for (int k0 = 0; k0 < n_w; k0 += 4) {  // four weights per launch, output block k0 on
        const int m = n_w - k0 < 4 ? n_w - k0 : 4;
        PeakShifts s2{};
        for (int k = 0; k < m; ++k) s2.shift[k] = shifts[k0 + k];
        ValidArgs v2 = v;
        v2.out = out + (size_t)k0 * n;
        if (m == 4) hipLaunchKernelGGL(k_is_valid_peaks<4>, dim3(grid), dim3(256), 0, st, v2, s2);
        if (m == 3) hipLaunchKernelGGL(k_is_valid_peaks<3>, dim3(grid), dim3(256), 0, st, v2, s2);
        if (m == 2) hipLaunchKernelGGL(k_is_valid_peaks<2>, dim3(grid), dim3(256), 0, st, v2, s2);
        if (m == 1) hipLaunchKernelGGL(k_is_valid_peaks<1>, dim3(grid), dim3(256), 0, st, v2, s2);
      }
  }
  return hipGetLastError();
}
size_t scan_dyn_lds(const TableArgs& t) {
  if (!t.pairs_enabled) return 0;
  return ((size_t)(2 * (t.n_pairs + 2) + t.n_buckets) * sizeof(uint32_t) + 15) / 16 * 16;
}
hipError_t launch_explain_scan(const TableArgs& t, const QueryArgs& q, const OutArgs& o, int n_blocks,
                               hipStream_t st) {
  if (q.n <= 0) return hipSuccess;
  const size_t dyn = scan_dyn_lds(t);
  if (!t.pairs_enabled)
    hipLaunchKernelGGL(k_bitset_scan, dim3(n_blocks), dim3(kScanWG), 0, st, t, q, o);
  else if (q.thr && q.max_mods)
    hipLaunchKernelGGL((k_explain_scan<true, true>), dim3(n_blocks), dim3(kScanWG), dyn, st, t, q, o);
  else if (q.thr)
    hipLaunchKernelGGL((k_explain_scan<true, false>), dim3(n_blocks), dim3(kScanWG), dyn, st, t, q, o);
  else if (q.max_mods)
    hipLaunchKernelGGL((k_explain_scan<false, true>), dim3(n_blocks), dim3(kScanWG), dyn, st, t, q, o);
  else
    hipLaunchKernelGGL((k_explain_scan<false, false>), dim3(n_blocks), dim3(kScanWG), dyn, st, t, q, o);
  return hipGetLastError();
}
hipError_t launch_step(const TableArgs& t, const QueryArgs& q, const OutArgs& o, int n_blocks, const double* obs,
                       int64_t n_peaks, const double* shifts4, double tol, double prec, int8_t* valid_out,
                       hipStream_t st) {
  if (!t.pairs_enabled || q.n <= 0) return hipErrorInvalidValue;
  const size_t dyn = scan_dyn_lds(t);
  ValidArgs v{t.valid, t.limit, t.full_lo, t.full_hi, t.first_reach, obs, nullptr, n_peaks, tol, prec, 1.0 / prec,
              valid_out};
  PeakShifts sh{};
  for (int k = 0; k < 4; ++k) sh.shift[k] = shifts4[k];
  const uint32_t a7 = (uint32_t)((n_peaks + kScanWG - 1) / kScanWG);
  const dim3 grid(a7 + (uint32_t)n_blocks);
  if (q.thr && q.max_mods)
    hipLaunchKernelGGL((k_step<true, true>), grid, dim3(kScanWG), dyn, st, t, q, o, v, sh, a7);
  else if (q.thr)
    hipLaunchKernelGGL((k_step<true, false>), grid, dim3(kScanWG), dyn, st, t, q, o, v, sh, a7);
  else if (q.max_mods)
    hipLaunchKernelGGL((k_step<false, true>), grid, dim3(kScanWG), dyn, st, t, q, o, v, sh, a7);
  else
    hipLaunchKernelGGL((k_step<false, false>), grid, dim3(kScanWG), dyn, st, t, q, o, v, sh, a7);
  return hipGetLastError();
}
hipError_t launch_explain_expand(const TableArgs& t, const QueryArgs& q, const OutArgs& o, int n_blocks,
                                 hipStream_t st) {
  if (q.n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_explain_expand, dim3(n_blocks), dim3(kWG), 0, st, t, q, o);
  return hipGetLastError();
}
static int occupancy(const void* k, int threads, size_t dyn) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, threads, dyn) != hipSuccess) {
    (void)hipGetLastError();
    return 1;
  }
  return nb > 0 ? nb : 1;
}
int explain_scan_blocks_per_cu(size_t dyn) {
  // every variant of the pair scan is held to 8 waves/SIMD by its launch bounds
  return dyn ? occupancy((const void*)k_explain_scan<true, false>, kScanWG, dyn)
             : occupancy((const void*)k_bitset_scan, kScanWG, 0);
}
int explain_expand_blocks_per_cu() { return occupancy((const void*)k_explain_expand, kWG, 0); }
hipError_t launch_result_pack(const PackArgs& p, hipStream_t st) {
  hipLaunchKernelGGL(k_result_pack, dim3(p.n_wg > 0 ? p.n_wg : 1), dim3(1024), 0, st, p);
  return hipGetLastError();
}
hipError_t launch_hits_to_arrays(const uint4* hits, uint64_t n_hits, const int8_t* status, uint64_t* count,
                                 uint64_t* offset, hipStream_t st) {
  if (n_hits == 0) return hipSuccess;
  hipLaunchKernelGGL(k_hits_to_arrays, dim3(blocks_for((int64_t)n_hits, 256)), dim3(256), 0, st, hits, n_hits, status,
                     count, offset);
  return hipGetLastError();
}
hipError_t launch_wire_pack(const WireArgs& a, hipStream_t st) {
  if (a.be_e == 0) return hipSuccess;
  hipLaunchKernelGGL(k_wire_pack, dim3(a.be_e), dim3(256), 0, st, a);
  return hipGetLastError();
}
#ifdef SST_DIAG_TIME
hipError_t diag_time_read(void* dst, size_t bytes) { return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_diag_time), bytes); }
hipError_t diag_time_clear() {
  static uint64_t zeros[1 << 16];
  for (size_t o = 0; o < sizeof(g_diag_time); o += sizeof(zeros)) {
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_diag_time), zeros, sizeof(zeros), o);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
#endif

hipError_t launch_explain_deferred(const TableArgs& t, const QueryArgs& q, const OutArgs& o, void* ws_deep,
                                   int shallow_blocks, int deep_blocks, const ExactWs& ws, int exact_blocks,
                                   hipStream_t st) {
  if (q.n <= 0) return hipSuccess;
  // the host counts 64-lane waves; the kernel runs kDefWG-lane workgroups
  constexpr int kW = kDefWG / 64;
  const int sb = (shallow_blocks + kW - 1) / kW, db = deep_blocks / kW, eb = (exact_blocks + kW - 1) / kW;
  hipLaunchKernelGGL(k_explain_deferred, dim3(sb + 2 * db + eb), dim3(kDefWG), 0, st, t, q, o, (GlobFrame*)ws_deep, ws,
                     sb, db, exact_blocks * 64);
  return hipGetLastError();
}

size_t glob_frame_bytes() { return sizeof(GlobFrame); }
size_t p1_frame_bytes() { return sizeof(P1Frame); }
size_t hash_entry_bytes() { return sizeof(HEntry); }

hipError_t launch_layer_step(const uint64_t* prev, uint64_t* next, int64_t nwords, const int* w, int n_rows,
                             hipStream_t st) {
  hipLaunchKernelGGL(k_layer_step, dim3(blocks_for(nwords, 256)), dim3(256), 0, st, prev, next, nwords, w, n_rows);
  return hipGetLastError();
}
hipError_t launch_length_bound(const TableArgs& t, const LBArgs& q, char* hash, int8_t* vals, char* frames,
                               uint32_t hash_cap, int exact_units, bool fast_pass, hipStream_t st) {
  if (q.n <= 0) return hipSuccess;
  if (fast_pass) hipLaunchKernelGGL(k_length_fast, dim3(blocks_for(q.n, 256)), dim3(256), 0, st, t, q);
  if (exact_units >= 1)  // one 64-lane block per query in flight
    hipLaunchKernelGGL(k_length_exact<true>, dim3(exact_units), dim3(64), 0, st, t, q, hash, vals, frames, hash_cap);
  return hipGetLastError();
}
size_t lb_frame_bytes() { return kLBFrameBytes; }

hipError_t launch_explain_recursion(const TableArgs& t, const QueryArgs& q, const OutArgs& o, char* hash,
                                   char* /*frames: in LDS*/, uint32_t hash_cap, int units, hipStream_t st) {
  if (q.n <= 0 || units < 1) return hipSuccess;  // one 64-lane block per query in flight
  hipLaunchKernelGGL(k_explain_recursion<true>, dim3(units), dim3(kRecLanes), 0, st, t, q, o, hash, hash_cap);
  return hipGetLastError();
}
size_t rec_frame_bytes() { return 64; }  // frames live in LDS; kept for the host's workspace sizing
size_t rec_entry_bytes() { return sizeof(REntry); }
hipError_t launch_is_singleton(const int64_t* masses, int n_masses, const double* mass, const double* thr, int64_t n,
                               double tol, double prec, int8_t* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_is_singleton, dim3(blocks_for(n, 256)), dim3(256), 0, st, masses, n_masses, mass, thr, n, tol,
                     prec, 1.0 / prec, out);
  return hipGetLastError();
}
}  // namespace sst

