// sst_pipe.hip -- the prediction pipeline's explanation stages over many
// spectra, device-resident, gfx950.
//
//   k_classify_rows  classify_fragments (fragment_classification.py:17-101)
//                    per spectrum: is_valid of every peak x breakage weight,
//                    the intensity / mass / sequence-mass filters, is_singleton
//                    (:104-119) and the SU order of the kept rows (a merge of
//                    the breakages' sorted streams, ties breakage-major as the
//                    reference's stable sort; a spectrum whose peaks are not in
//                    mass order is ranked in LDS first, equal masses in their
//                    given order).  Rows go to fixed slots
//                    (spectrum g: 4 * peak_off[g] + i), no compaction pass.
//   k_fix_round      one filter_by_explanation round (prediction.py:170-227)
//                    of every spectrum still reducing: the alive rows, the
//                    sliding-window pairs of both sides (closed form, as the
//                    rows step) and the singletons; every query against the
//                    spectrum's alphabet (the full table's pair list with the
//                    row mask: the reduced table's answers); the explanation
//                    dict's last-writer semantics (a side pair is stored only
//                    with >= 1 explanation, a singleton always, a later equal
//                    key replaces an earlier one) in an LDS hash; the union of
//                    the surviving answers' rows -> the reduced alphabet
//                    (canonical rows kept); the spectrum stays active while
//                    the alphabet shrinks.  is_valid on the reduced tables
//                    follows in k_valid_alpha (sst_alpha.hip, AND-ed into the
//                    rows' alive flags).
//   k_bins_count /   SkeletonBuilder._predict_skeleton's speculative bin
//   k_bins_emit      queries (skeleton_building.py:114-160) over the rows the
//                    fixpoint kept: per side, bins are runs of rows whose SU
//                    step is within the pair threshold; the side's first bin
//                    explains its whole masses (against 0), every later bin
//                    each (predecessor row, row) difference; a side's last bin
//                    only when it has two rows or more (:150-153).  Count pass,
//                    exclusive scan (k_scan_u32), then every query answered on
//                    its spectrum's alphabet into a dense spectrum-major list
//                    (per spectrum: START side, then END; per side its bins in
//                    order, a bin's pairs predecessor-row-major).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sst_internal.h"
#include "sst_quant.h"

namespace sst {

namespace {

constexpr int kPipeWG = 1024;
constexpr int kHashSlots = 4096;
constexpr uint64_t kEmptyKey = ~0ull;

__device__ __forceinline__ bool in_mask(uint64_t m0, uint64_t m1, int r) {
  return r < 64 ? ((m0 >> r) & 1ull) : ((m1 >> (r - 64)) & 1ull);
}

// pair-list window [a, hi] (a >= 1, hi < pair_hi) against a row mask: the
// number of entries whose rows are all in the mask and the union of their rows
__device__ __forceinline__ uint32_t masked_walk(const TableArgs& t, uint32_t a, uint32_t hi, uint64_t m0, uint64_t m1,
                                                uint64_t& u0, uint64_t& u1) {
  const uint32_t* sums = t.pair_data;
  const uint32_t* recs = sums + (t.n_pairs + 2);
  const uint32_t* bk = recs + (t.n_pairs + 2);
  const uint32_t rel = a > t.pair_base ? a - t.pair_base : 0u;
  uint32_t k = bk[rel >> t.pair_shift] & 0xFFFFu;
  const uint32_t a2 = a << 1, h2 = (hi << 1) | 1u;
  while (sums[k] < a2) ++k;
  uint32_t cnt = 0;
  for (; sums[k] <= h2; ++k) {
    const uint32_t rec = recs[k];
    const int top = (int)((rec >> ((rec & 0xFFu) == 1u ? 8 : 16)) & 0xFFu);
    const int low = (int)((rec >> 8) & 0xFFu);
    if (in_mask(m0, m1, top) && in_mask(m0, m1, low)) {
      ++cnt;
      if (top < 64) u0 |= 1ull << top; else u1 |= 1ull << (top - 64);
      if (low < 64) u0 |= 1ull << low; else u1 |= 1ull << (low - 64);
    }
  }
  return cnt;
}

// explain status of a pair-class window against the mask (NONE / EMPTY / SOME)
__device__ __forceinline__ int8_t masked_answer(const TableArgs& t, double mass, double thr, double prec,
                                                double rprec, uint64_t m0, uint64_t m1, uint64_t& u0, uint64_t& u1,
                                                bool& pair_class) {
  double lof, hif;
  quantise_lean(mass, thr, prec, rprec, lof, hif);
  u0 = u1 = 0;
  pair_class = hif < (double)t.pair_hi;
  if (!pair_class || hif < 0.0) return SST_NONE;
  const double af = lof < 1.0 ? 1.0 : lof;
  uint32_t cnt = 0;
  if (af <= hif) cnt = masked_walk(t, (uint32_t)af, (uint32_t)hif, m0, m1, u0, u1);
  return cnt ? (int8_t)SST_SOME : lof <= 0.0 ? (int8_t)SST_EMPTY : (int8_t)SST_NONE;
}

// every peak's mass <= the next one's (whole list, any P)
__device__ __forceinline__ bool peaks_sorted(const double* obs, uint32_t P) {
  bool ok = true;
  for (uint32_t p = threadIdx.x; p + 1 < P; p += blockDim.x) ok &= obs[p] <= obs[p + 1];
  return __syncthreads_and(ok);
}

struct ClsLds {
  double obs[kPipeMaxPeaks];
  uint16_t ord[kPipeMaxPeaks];      // peaks in (mass, position) order
  uint16_t kidx[4][kPipeMaxPeaks];
  uint8_t keep[kPipeMaxPeaks];
};
struct ClsSmall {  // both variants: the block scan's words, the row masses
  uint32_t kcnt[4];
  int64_t masses[kMaxRows];
  uint32_t w[16];
};
// one spectrum's peak arrays: the LDS ones (<= kPipeMaxPeaks peaks) or a
// workgroup's slice of the pipeline's HBM scratch (k_classify_rows_big)
struct ClsView {
  double* obs;
  uint16_t* ord;
  uint16_t* kidx[4];
  uint8_t* keep;
};
// the slice bytes the big variant needs for P peaks
__device__ __forceinline__ uint64_t cls_slice_bytes(uint32_t P) { return 29ull * P + 4 * 256; }
__device__ __forceinline__ ClsView cls_big_view(uint8_t* p, uint32_t P) {
  auto up = [](uint64_t x) { return (x + 255) & ~255ull; };
  ClsView V;
  uint64_t o = 0;
  V.obs = (double*)(p + o);
  o += up(8ull * P);
  V.ord = (uint16_t*)(p + o);
  o += up(2ull * P);
  for (int k = 0; k < 4; ++k) {
    V.kidx[k] = (uint16_t*)(p + o);
    o += up(2ull * P);
  }
  V.keep = p + o;
  return V;
}

// classify_fragments (fragment_classification.py:17-101) for spectrum g of P
// peaks, one workgroup: A7 per peak and breakage, the filters, the SU order
// of the kept rows (breakage streams merged), is_singleton
__device__ __forceinline__ void classify_spec(const TableArgs& t, const PipeArgs& a, ClsSmall& S, const ClsView& V,
                                              int64_t g, int64_t p0, uint32_t P) {
  const double su_seq = a.su_seq[g];
  for (uint32_t p = threadIdx.x; p < P; p += blockDim.x) {
    const double o = a.obs[p0 + p];
    V.obs[p] = o;
    uint8_t kp = 0;
    for (int k = 0; k < a.n_shifts; ++k) {
      const double su = o - a.shift[k];
      double lof, hif;
      quantise_lean(su, a.tol * o, a.prec, a.rprec, lof, hif);
      const int8_t code =
          valid_window(t.valid, t.limit, (int64_t)lof, (int64_t)hif, t.full_lo, t.full_hi, t.first_reach);
      if (a.valid_out) a.valid_out[(int64_t)k * a.n_peaks + p0 + p] = code;
      if (code < 0) atomicOr(a.err, 8u);  // is_valid_mass raises: the reference's classify would too
      const bool inten = a.intensity ? a.intensity[p0 + p] > a.intensity_cutoff : true;
      const bool full = (a.sides[k] & 3) == 3;
      const bool keep = code == 1 && inten && o < a.mass_cutoff && su < su_seq + a.max_variance &&
                        (su > su_seq - a.max_variance || !full);
      kp |= (uint8_t)keep << k;
    }
    V.keep[p] = kp;
  }
  __syncthreads();
  // the peaks in ascending mass order, equal masses in their given order (a
  // peak list need not be sorted; a breakage's rows are then in SU order)
  const bool sorted = peaks_sorted(V.obs, P);
  for (uint32_t p = threadIdx.x; p < P; p += blockDim.x) {
    uint32_t rank = p;
    if (!sorted) {
      const double o = V.obs[p];
      rank = 0;
      for (uint32_t q = 0; q < P; ++q) {
        const double v = V.obs[q];
        rank += (v < o) | ((v == o) & (q < p));
      }
    }
    V.ord[rank] = (uint16_t)p;
  }
  __syncthreads();
  for (int k = 0; k < a.n_shifts; ++k) {
    uint32_t carry = 0;
    for (uint32_t q0 = 0; q0 < P; q0 += blockDim.x) {
      const uint32_t i = q0 + threadIdx.x;
      const uint32_t p = i < P ? V.ord[i] : 0u;
      const uint32_t f = i < P ? (V.keep[p] >> k) & 1u : 0u;
      uint32_t tot;
      const uint32_t ex = block_excl(f, S.w, tot);
      if (f) V.kidx[k][carry + ex] = (uint16_t)p;
      carry += tot;
    }
    if (threadIdx.x == 0) S.kcnt[k] = carry;
  }
  __syncthreads();
  // every kept row's place in the spectrum's SU order (all breakages)
  uint32_t n = 0;
  for (int k = 0; k < a.n_shifts; ++k) n += S.kcnt[k];
  const int64_t base = 4 * p0;
  for (int k = 0; k < a.n_shifts; ++k) {
    const double sk = a.shift[k];
    for (uint32_t j = threadIdx.x; j < S.kcnt[k]; j += blockDim.x) {
      const uint32_t p = V.kidx[k][j];
      const double su = V.obs[p] - sk;
      uint32_t pos = j;
      for (int k2 = 0; k2 < a.n_shifts; ++k2) {
        if (k2 == k) continue;
        const double s2 = a.shift[k2];
        uint32_t lo = 0, hi = S.kcnt[k2];
        while (lo < hi) {
          const uint32_t mid = (lo + hi) >> 1;
          const double v = V.obs[V.kidx[k2][mid]] - s2;
          if (v < su || (v == su && k2 < k)) lo = mid + 1;
          else hi = mid;
        }
        pos += lo;
      }
      // is_singleton (:104-119): a table row mass (the sentinel 0 included) in the window
      int64_t lo, hi;
      quantise(su, a.tol * V.obs[p], false, a.tol, a.prec, a.rprec, lo, hi);
      int l = 0, r = a.n_masses;
      while (l < r) {
        const int mid = (l + r) >> 1;
        if (S.masses[mid] < lo) l = mid + 1;
        else r = mid;
      }
      const bool single = lo <= hi && l < a.n_masses && S.masses[l] <= hi;
      a.r_su[base + pos] = su;
      a.r_ob[base + pos] = V.obs[p];
      a.r_meta[base + pos] = (uint32_t)k | ((uint32_t)a.sides[k] << 2) | ((uint32_t)single << 4) | (p << 8);
      a.alive[base + pos] = 1;
    }
  }
  if (threadIdx.x == 0) a.cnt[g] = n;
  __syncthreads();
}

}  // namespace

__global__ __launch_bounds__(kPipeWG) void k_classify_rows(TableArgs t, PipeArgs a) {
  __shared__ ClsLds L;
  __shared__ ClsSmall S;
  for (int r = threadIdx.x; r < a.n_masses; r += blockDim.x) S.masses[r] = a.masses[r];
  __syncthreads();
  ClsView V;  // (assigned, not a constant initializer: LDS addresses are not constants)
  V.obs = L.obs;
  V.ord = L.ord;
  for (int k = 0; k < 4; ++k) V.kidx[k] = L.kidx[k];
  V.keep = L.keep;
  for (int64_t g = blockIdx.x; g < a.n_spec; g += gridDim.x) {
    const int64_t p0 = a.peak_off[g];
    const uint32_t P = (uint32_t)(a.peak_off[g + 1] - p0);
    if (P > (uint32_t)kPipeMaxPeaks) {  // k_classify_rows_big's (or rejected there)
      if (threadIdx.x == 0 && !a.big) {
        atomicOr(a.err, 1u);
        a.cnt[g] = 0;
      }
      continue;
    }
    classify_spec(t, a, S, V, g, p0, P);
  }
}

// spectra of more than kPipeMaxPeaks peaks: the same code over a workgroup's
// slice of the pipeline's HBM scratch (sst_pipe_reserve_rows); spectrum g
// goes to workgroup g % gridDim.x, found by a coalesced scan of the peak counts
__global__ __launch_bounds__(kPipeWG) void k_classify_rows_big(TableArgs t, PipeArgs a) {
  __shared__ ClsSmall S;
  __shared__ uint32_t s_list[kPipeWG];
  __shared__ uint32_t s_n;
  for (int r = threadIdx.x; r < a.n_masses; r += blockDim.x) S.masses[r] = a.masses[r];
  uint8_t* slice = a.big + (uint64_t)blockIdx.x * a.big_stride;
  const int64_t G = gridDim.x;
  for (int64_t c0 = 0; (int64_t)blockIdx.x + c0 * G < a.n_spec; c0 += blockDim.x) {
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    const int64_t gi = (int64_t)blockIdx.x + (c0 + threadIdx.x) * G;
    if (gi < a.n_spec && a.peak_off[gi + 1] - a.peak_off[gi] > kPipeMaxPeaks) s_list[atomicAdd(&s_n, 1u)] = threadIdx.x;
    __syncthreads();
    const uint32_t n = s_n;
    for (uint32_t k = 0; k < n; ++k) {
      const int64_t g = (int64_t)blockIdx.x + (c0 + s_list[k]) * G;
      const int64_t p0 = a.peak_off[g];
      const uint32_t P = (uint32_t)(a.peak_off[g + 1] - p0);
      if (P > (uint32_t)kPipeMaxPeaksBig || (uint64_t)P * (uint64_t)a.n_shifts > a.big_rows ||
          cls_slice_bytes(P) > a.big_stride) {
        if (threadIdx.x == 0) {
          atomicOr(a.err, 1u);
          a.cnt[g] = 0;
        }
        continue;
      }
      classify_spec(t, a, S, cls_big_view(slice, P), g, p0, P);
    }
  }
}

namespace {

// One spectrum's alive rows, a round's query offsets and the explanation
// dict's hash, as views: of LDS arrays for a spectrum of <= kPipeMaxRows
// rows, of the workgroup's HBM slice (pipe_big_layout) in the *_big variants.
// Both instantiate the same code; the LDS views stay in the LDS address space
// after inlining (ds_* instructions), the HBM ones are global accesses.
struct FixView {
  double* su;
  double* ob;
  uint16_t* s0;      // alive rows of the START side (indices into su / ob), SU order
  uint16_t* s1;      // ... of the END side
  uint16_t* single;  // alive singleton rows
  uint32_t* q0;      // per side: exclusive prefix of each row's pair queries
  uint32_t* q1;
  uint64_t* hkey;
  uint32_t* hidx;
  uint32_t hmask;    // hash slots - 1
  __device__ __forceinline__ uint16_t* side(int sd) const { return sd ? s1 : s0; }
  __device__ __forceinline__ uint32_t* qoff(int sd) const { return sd ? q1 : q0; }
};
struct FixLdsArrays {
  double su[kPipeMaxRows];
  double ob[kPipeMaxRows];
  uint16_t side[2][kPipeMaxRows];
  uint16_t single[kPipeMaxRows];
  uint32_t qoff[2][kPipeMaxRows + 1];
  uint64_t hkey[kHashSlots];
  uint32_t hidx[kHashSlots];
};
struct FixMeta {
  uint32_t n_side[2], n_single, n_alive;
  int sstar[2];
  uint32_t w[16];
  unsigned long long u0, u1;
  uint32_t writers, n_ent;
};

__device__ __forceinline__ FixView lds_view(FixLdsArrays& S) {
  return FixView{S.su, S.ob, S.side[0], S.side[1], S.single, S.qoff[0], S.qoff[1], S.hkey, S.hidx,
                 (uint32_t)kHashSlots - 1};
}
__device__ __forceinline__ uint8_t* big_slice(const PipeArgs& a) { return a.big + (uint64_t)blockIdx.x * a.big_stride; }
__device__ __forceinline__ FixView big_view(const PipeArgs& a) {
  const PipeBigLayout B = pipe_big_layout(a.big_rows, a.big_slots);
  uint8_t* p = big_slice(a);
  return FixView{(double*)(p + B.su),     (double*)(p + B.ob),   (uint16_t*)(p + B.s0),
                 (uint16_t*)(p + B.s1),   (uint16_t*)(p + B.single), (uint32_t*)(p + B.q0),
                 (uint32_t*)(p + B.q1),   (uint64_t*)(p + B.hkey), (uint32_t*)(p + B.hidx),
                 a.big_slots - 1};
}

// the big variants' spectra: rows > kPipeMaxRows; spectrum g goes to
// workgroup g % gridDim.x, found by a coalesced scan of the row counts
template <class F>
__device__ __forceinline__ void for_big_spectra(const PipeArgs& a, F&& f) {
  __shared__ uint32_t s_list[kPipeWG];
  __shared__ uint32_t s_n;
  const int64_t G = gridDim.x;
  for (int64_t c0 = 0; (int64_t)blockIdx.x + c0 * G < a.n_spec; c0 += blockDim.x) {
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    const int64_t gi = (int64_t)blockIdx.x + (c0 + threadIdx.x) * G;
    if (gi < a.n_spec && a.cnt[gi] > (uint32_t)kPipeMaxRows) s_list[atomicAdd(&s_n, 1u)] = threadIdx.x;
    __syncthreads();
    const uint32_t n = s_n;
    for (uint32_t k = 0; k < n; ++k) {
      const int64_t g = (int64_t)blockIdx.x + (c0 + s_list[k]) * G;
      f(g, a.cnt[g]);
      __syncthreads();
    }
  }
}
// a spectrum neither variant holds (more rows than the big slices, or no slices)
__device__ __forceinline__ bool pipe_too_big(const PipeArgs& a, uint32_t nr) {
  return nr > (uint32_t)kPipeMaxRows && (a.big == nullptr || nr > a.big_rows);
}

// reads of hash slots written by atomics (device-scope loads: the slots may be HBM)
__device__ __forceinline__ uint64_t ld_key(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_idx(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the alive rows of a spectrum (SU order) and each side's / the singletons' lists
__device__ __forceinline__ void fix_load(FixMeta& M, const FixView& V, const PipeArgs& a, int64_t base,
                                         uint32_t nr) {
  uint32_t carry[4] = {0, 0, 0, 0};
  for (uint32_t r0 = 0; r0 < nr; r0 += blockDim.x) {
    const uint32_t r = r0 + threadIdx.x;
    const bool al = r < nr && a.alive[base + r];
    const uint32_t meta = al ? a.r_meta[base + r] : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl(al ? 1u : 0u, M.w, tot);
    const uint32_t i = carry[0] + ex;
    if (al) {
      V.su[i] = a.r_su[base + r];
      V.ob[i] = a.r_ob[base + r];
    }
    carry[0] += tot;
    for (int c = 0; c < 3; ++c) {
      const bool f = al && ((meta >> (2 + c)) & 1u);  // START, END, singleton
      const uint32_t x = block_excl(f ? 1u : 0u, M.w, tot);
      if (f) (c == 0 ? V.s0 : c == 1 ? V.s1 : V.single)[carry[c + 1] + x] = (uint16_t)i;
      carry[c + 1] += tot;
    }
  }
  if (threadIdx.x == 0) {
    M.n_alive = carry[0];
    M.n_side[0] = carry[1];
    M.n_side[1] = carry[2];
    M.n_single = carry[3];
    M.u0 = M.u1 = 0;
    M.writers = 0;
    M.n_ent = 0;
  }
}

__device__ __forceinline__ void hash_clear(const FixView& V) {
  for (uint32_t k = threadIdx.x; k <= V.hmask; k += blockDim.x) {
    V.hkey[k] = kEmptyKey;
    V.hidx[k] = 0;
  }
}

__device__ __forceinline__ double side_su(const FixView& V, int sd, uint32_t r) { return V.su[V.side(sd)[r]]; }

// s* and the per-row pair counts' prefix of side sd (the rows step's closed form)
__device__ __forceinline__ uint32_t fix_side_pairs(FixMeta& M, const FixView& V, int sd, double mw) {
  const uint32_t n = M.n_side[sd];
  if (threadIdx.x == 0) M.sstar[sd] = n ? (int)n - 1 : 0;
  __syncthreads();
  for (uint32_t r = threadIdx.x; r + 1 < n; r += blockDim.x)
    if (!(side_su(V, sd, n - 1) - side_su(V, sd, r) > mw)) atomicMin(&M.sstar[sd], (int)r);
  __syncthreads();
  const uint32_t ss = (uint32_t)M.sstar[sd];
  uint32_t* qoff = V.qoff(sd);
  uint32_t carry = 0;
  for (uint32_t r0 = 0; r0 < n; r0 += blockDim.x) {
    const uint32_t r = r0 + threadIdx.x;
    uint32_t c = 0;
    if (r + 1 < n) {
      if (r < ss) {
        uint32_t lo = r + 1, hi = n - 1;
        const double sr = side_su(V, sd, r);
        while (lo < hi) {
          const uint32_t mid = (lo + hi) >> 1;
          if (side_su(V, sd, mid) - sr > mw) hi = mid;
          else lo = mid + 1;
        }
        c = lo - r - 1;
      } else if (r == ss) {
        c = n - 1 - r;
      } else {
        c = 1;
      }
    }
    uint32_t tot;
    const uint32_t ex = block_excl(c, M.w, tot);
    if (r < n) qoff[r] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) qoff[n] = carry;
  __syncthreads();
  return carry;
}

// query o of the round (START pairs, END pairs, singletons): its key, mass and threshold
__device__ __forceinline__ void fix_query(const FixMeta& M, const FixView& V, uint32_t o, uint32_t q0, uint32_t q1,
                                          double tol, double& mass, double& thr, bool& single) {
  single = o >= q0 + q1;
  if (single) {
    const uint32_t r = V.single[o - q0 - q1];
    mass = V.su[r];
    thr = tol * V.ob[r];  // prediction.py:280
    return;
  }
  const int sd = o >= q0;
  const uint32_t q = sd ? o - q0 : o;
  const uint32_t n = M.n_side[sd];
  const uint32_t* qoff = V.qoff(sd);
  uint32_t lo = 0, hi = n;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (qoff[mid] <= q) lo = mid;
    else hi = mid;
  }
  const uint32_t s = lo;
  const uint32_t e = s <= (uint32_t)M.sstar[sd] ? s + 1 + (q - qoff[s]) : n - 1;
  const uint16_t* rows = V.side(sd);
  const uint32_t rs = rows[s], re = rows[e];
  mass = V.su[re] - V.su[rs];
  thr = tol * (V.ob[rs] + V.ob[re]);  // calculate_error_threshold, l1 (common.py:37-44)
}

__device__ __forceinline__ uint64_t key_bits(double k) {
  if (k == 0.0) k = 0.0;  // -0.0 and 0.0 are one dict key
  return (uint64_t)__double_as_longlong(k);
}
__device__ __forceinline__ uint32_t key_hash(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  return (uint32_t)x;
}

// the dict's writers: insert the key, the last (largest order) writer wins
__device__ __forceinline__ void hash_put(const FixView& V, uint32_t* writers, uint64_t key, uint32_t o) {
  uint32_t h = key_hash(key) & V.hmask;
  for (uint32_t probe = 0; probe <= V.hmask; ++probe, h = (h + 1) & V.hmask) {
    const unsigned long long prev = atomicCAS((unsigned long long*)&V.hkey[h], kEmptyKey, key);
    if (prev == kEmptyKey || prev == key) {
      atomicMax(&V.hidx[h], o + 1);
      if (prev == kEmptyKey) atomicAdd(writers, 1u);
      return;
    }
  }
}
// query o is the last writer of its key
__device__ __forceinline__ bool hash_last(const FixView& V, uint64_t key, uint32_t o) {
  uint32_t h = key_hash(key) & V.hmask;
  uint64_t k = ld_key(&V.hkey[h]);
  for (uint32_t probe = 0; probe < V.hmask && k != key; ++probe) {
    h = (h + 1) & V.hmask;
    k = ld_key(&V.hkey[h]);
  }
  return k == key && ld_idx(&V.hidx[h]) == o + 1;
}
__device__ __forceinline__ void hash_check(const FixMeta& M, const FixView& V, const PipeArgs& a) {
  // too full to trust the probe bound: reported
  if (threadIdx.x == 0 && (uint64_t)M.writers * 4 > 3ull * (V.hmask + 1ull)) atomicOr(a.err, 16u);
}

// exact mode: the round's queries (START pairs, END pairs, singletons) of
// spectrum g listed for the masked explain, in order (one block per spectrum)
__device__ __forceinline__ void fix_list(const FixMeta& M, const FixView& V, const PipeArgs& a, int64_t g,
                                         uint32_t q0, uint32_t q1, uint32_t Q) {
  __shared__ uint32_t s_start;
  if (threadIdx.x == 0) {
    s_start = atomicAdd(a.xq_count, Q);
    if ((uint64_t)s_start + Q > a.xq_cap) atomicOr(a.err, 64u);
  }
  __syncthreads();
  const uint32_t start = s_start;
  if ((uint64_t)start + Q <= a.xq_cap) {
    for (uint32_t o = threadIdx.x; o < Q; o += blockDim.x) {
      double mass, thr;
      bool single;
      fix_query(M, V, o, q0, q1, a.tol, mass, thr, single);
      a.xq_mass[start + o] = mass;
      a.xq_thr[start + o] = thr;
      a.xq_spec[start + o] = (int32_t)g;
      a.xq_single[start + o] = single;
    }
    if (threadIdx.x == 0) a.xq_block[g] = ((uint64_t)start << 32) | Q;
  } else if (threadIdx.x == 0) {
    a.xq_block[g] = 0;
  }
  __syncthreads();
}

// the round's outcome: canonical rows stay, a modification stays iff a
// surviving explanation names it (adapt_individual_modification_rates_by_
// alphabet_reduction, mass_table.py:94-121); the spectrum stays active while
// its alphabet shrinks
__device__ __forceinline__ void fix_outcome(const FixMeta& M, const PipeArgs& a, int64_t g, uint32_t Q) {
  if (threadIdx.x == 0) {
    const uint64_t m0 = a.alpha[2 * g], m1 = a.alpha[2 * g + 1];
    const uint64_t n0 = a.canon[0] | (m0 & M.u0), n1 = a.canon[1] | (m1 & M.u1);
    a.alpha_next[2 * g] = n0;
    a.alpha_next[2 * g + 1] = n1;
    const bool changed = __builtin_popcountll(n0) + __builtin_popcountll(n1) !=
                         __builtin_popcountll(m0) + __builtin_popcountll(m1);
    a.active_next[g] = changed;
    a.rounds[g] += 1;
    a.queries[g] += Q;
    if (changed) atomicAdd(a.n_active, 1u);
  }
  __syncthreads();
}

// one filter_by_explanation round of spectrum g (nr row slots)
__device__ __forceinline__ void fix_round_spec(const TableArgs& t, const PipeArgs& a, FixMeta& M, const FixView& V,
                                               int64_t g, uint32_t nr) {
  fix_load(M, V, a, 4 * a.peak_off[g], nr);
  hash_clear(V);
  __syncthreads();
  const uint32_t q0 = fix_side_pairs(M, V, 0, a.max_weight);
  const uint32_t q1 = fix_side_pairs(M, V, 1, a.max_weight);
  const uint32_t Q = q0 + q1 + M.n_single;
  const uint64_t m0 = a.alpha[2 * g], m1 = a.alpha[2 * g + 1];
  if (a.pair_ok && !a.pair_ok[g]) {  // budgets can bind: list the round's queries for the exact explain
    fix_list(M, V, a, g, q0, q1, Q);
    return;
  }
  // pass A: every query's answer; writers insert their key, the last (largest order) wins
  for (uint32_t o = threadIdx.x; o < Q; o += blockDim.x) {
    double mass, thr;
    bool single, pc;
    fix_query(M, V, o, q0, q1, a.tol, mass, thr, single);
    uint64_t u0, u1;
    const int8_t st = masked_answer(t, mass, thr, a.prec, a.rprec, m0, m1, u0, u1, pc);
    if (!pc) atomicOr(a.err, 4u);  // not pair-class: never for these windows (the host checks)
    if (single || st == SST_SOME) hash_put(V, &M.writers, key_bits(mass), o);
  }
  __syncthreads();
  hash_check(M, V, a);
  // pass B: the dict's surviving entries -> the observed rows
  for (uint32_t o = threadIdx.x; o < Q; o += blockDim.x) {
    double mass, thr;
    bool single, pc;
    fix_query(M, V, o, q0, q1, a.tol, mass, thr, single);
    uint64_t u0, u1;
    const int8_t st = masked_answer(t, mass, thr, a.prec, a.rprec, m0, m1, u0, u1, pc);
    if (st != SST_SOME) continue;  // None / set() entries name no nucleotide
    if (hash_last(V, key_bits(mass), o)) {
      if (u0) atomicOr(&M.u0, (unsigned long long)u0);
      if (u1) atomicOr(&M.u1, (unsigned long long)u1);
    }
  }
  __syncthreads();
  fix_outcome(M, a, g, Q);
}

// a spectrum no variant holds: reported, its alphabet carried over
__device__ __forceinline__ void fix_reject(const PipeArgs& a, int64_t g) {
  if (threadIdx.x == 0) {
    atomicOr(a.err, 2u);
    a.alpha_next[2 * g] = a.alpha[2 * g];
    a.alpha_next[2 * g + 1] = a.alpha[2 * g + 1];
    a.active_next[g] = 0;
  }
}

// the rest of an exact-mode round after the caller answered the list (see k_fix_finish)
__device__ __forceinline__ void fix_finish_spec(const PipeArgs& a, FixMeta& M, const FixView& V, int64_t g) {
  const uint64_t blk = a.xq_block[g];
  const uint32_t start = (uint32_t)(blk >> 32), Q = (uint32_t)blk;
  hash_clear(V);
  if (threadIdx.x == 0) {
    M.u0 = M.u1 = 0;
    M.writers = 0;
  }
  __syncthreads();
  for (uint32_t o = threadIdx.x; o < Q; o += blockDim.x) {
    const int8_t st = a.xa_st[start + o];
    if (st != SST_NONE && st != SST_EMPTY && st != SST_SOME) atomicOr(a.err, 128u);  // raised / capped
    if (a.xq_single[start + o] || st == SST_SOME) hash_put(V, &M.writers, key_bits(a.xq_mass[start + o]), o);
  }
  __syncthreads();
  hash_check(M, V, a);
  for (uint32_t o = threadIdx.x; o < Q; o += blockDim.x) {
    if (a.xa_st[start + o] != SST_SOME) continue;  // None / set() entries name no nucleotide
    if (!hash_last(V, key_bits(a.xq_mass[start + o]), o)) continue;
    const uint8_t* p = (const uint8_t*)a.xa_ptr[start + o];
    uint64_t u0 = 0, u1 = 0;
    for (uint32_t c = 0; c < a.xa_n[start + o]; ++c) {
      const int k = p[0];
      for (int j = 0; j < k; ++j) {
        const int r = p[1 + j];
        if (r < 64) u0 |= 1ull << r;
        else u1 |= 1ull << (r - 64);
      }
      p += 1 + k;
    }
    if (u0) atomicOr(&M.u0, (unsigned long long)u0);
    if (u1) atomicOr(&M.u1, (unsigned long long)u1);
  }
  __syncthreads();
  fix_outcome(M, a, g, Q);
}

}  // namespace

// the rest of an exact-mode round (after the caller answered the list): the
// dict's last writer per key (a side pair only with >= 1 explanation, a
// singleton always), the rows its surviving answers name (their candidates'
// payload records), the reduced alphabet and the round's counters
__global__ __launch_bounds__(kPipeWG) void k_fix_finish(PipeArgs a) {
  __shared__ uint64_t hkey[kHashSlots];
  __shared__ uint32_t hidx[kHashSlots];
  __shared__ FixMeta M;
  const FixView V{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, hkey, hidx, (uint32_t)kHashSlots - 1};
  for (int64_t g = blockIdx.x; g < a.n_spec; g += gridDim.x) {
    if (!a.active[g] || !a.pair_ok || a.pair_ok[g]) continue;  // k_fix_round settled it
    const uint32_t nr = a.cnt[g];
    if (nr > (uint32_t)kPipeMaxRows) continue;  // k_fix_finish_big's, or rejected by k_fix_round
    fix_finish_spec(a, M, V, g);
  }
}
__global__ __launch_bounds__(kPipeWG) void k_fix_finish_big(PipeArgs a) {
  __shared__ FixMeta M;
  const FixView V = big_view(a);
  for_big_spectra(a, [&](int64_t g, uint32_t nr) {
    if (a.active[g] && a.pair_ok && !a.pair_ok[g] && !pipe_too_big(a, nr)) fix_finish_spec(a, M, V, g);
  });
}

__global__ __launch_bounds__(kPipeWG) void k_fix_round(TableArgs t, PipeArgs a) {
  __shared__ FixLdsArrays S;
  __shared__ FixMeta M;
  const FixView V = lds_view(S);
  for (int64_t g = blockIdx.x; g < a.n_spec; g += gridDim.x) {
    if (!a.active[g]) {  // settled earlier: its alphabet carries over
      if (threadIdx.x == 0) {
        a.alpha_next[2 * g] = a.alpha[2 * g];
        a.alpha_next[2 * g + 1] = a.alpha[2 * g + 1];
        a.active_next[g] = 0;
      }
      continue;
    }
    const uint32_t nr = a.cnt[g];
    if (nr > (uint32_t)kPipeMaxRows) {  // k_fix_round_big's
      if (pipe_too_big(a, nr)) fix_reject(a, g);
      continue;
    }
    fix_round_spec(t, a, M, V, g, nr);
  }
}
__global__ __launch_bounds__(kPipeWG) void k_fix_round_big(TableArgs t, PipeArgs a) {
  __shared__ FixMeta M;
  const FixView V = big_view(a);
  for_big_spectra(a, [&](int64_t g, uint32_t nr) {
    if (a.active[g] && !pipe_too_big(a, nr)) fix_round_spec(t, a, M, V, g, nr);
  });
}

namespace {

// k_dict's entries of one spectrum by key into its region: few in the LDS
// variant (a rank count over the occupied slots), a bitonic sort of (key,
// slot) pairs in the HBM slice in the big one
__device__ __forceinline__ void dict_emit_lds(FixMeta& M, const FixView& V, const PipeArgs& a, const DictArgs& d,
                                              int64_t g, uint32_t q0, uint32_t q1, uint32_t* ent) {
  for (uint32_t k = threadIdx.x; k <= V.hmask; k += blockDim.x)
    if (ld_key(&V.hkey[k]) != kEmptyKey) ent[atomicAdd(&M.n_ent, 1u)] = k;
  __syncthreads();
  const uint32_t E = M.n_ent;
  const uint64_t out0 = d.off[g];
  for (uint32_t e = threadIdx.x; e < E; e += blockDim.x) {
    const uint64_t key = ld_key(&V.hkey[ent[e]]);
    uint32_t rank = 0;
    for (uint32_t f = 0; f < E; ++f) rank += ld_key(&V.hkey[ent[f]]) < key;  // keys are distinct
    double mass, thr;
    bool single;
    fix_query(M, V, ld_idx(&V.hidx[ent[e]]) - 1, q0, q1, a.tol, mass, thr, single);
    d.key[out0 + rank] = key;
    d.thr[out0 + rank] = thr;
  }
  if (threadIdx.x == 0) d.n_ent[g] = E;
}
__device__ __forceinline__ void dict_emit_big(FixMeta& M, const FixView& V, const PipeArgs& a, const DictArgs& d,
                                              int64_t g, uint32_t q0, uint32_t q1) {
  const PipeBigLayout B = pipe_big_layout(a.big_rows, a.big_slots);
  uint64_t* sk = (uint64_t*)(big_slice(a) + B.sk);
  uint32_t* si = (uint32_t*)(big_slice(a) + B.si);
  for (uint32_t k = threadIdx.x; k <= V.hmask; k += blockDim.x) {
    const uint64_t key = ld_key(&V.hkey[k]);
    if (key != kEmptyKey) {
      const uint32_t e = atomicAdd(&M.n_ent, 1u);
      sk[e] = key;
      si[e] = k;
    }
  }
  __syncthreads();
  const uint32_t E = M.n_ent;
  uint32_t N = 1;
  while (N < E) N <<= 1;
  for (uint32_t e = E + threadIdx.x; e < N; e += blockDim.x) {
    sk[e] = kEmptyKey;  // never a key (no mass has these bits): sorts last
    si[e] = 0;
  }
  __syncthreads();
  for (uint32_t k = 2; k <= N; k <<= 1)
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = threadIdx.x; i < N; i += blockDim.x) {
        const uint32_t l = i ^ j;
        if (l <= i) continue;
        const uint64_t x = sk[i], y = sk[l];
        if ((x > y) == ((i & k) == 0)) {
          sk[i] = y;
          sk[l] = x;
          const uint32_t t = si[i];
          si[i] = si[l];
          si[l] = t;
        }
      }
      __syncthreads();
    }
  const uint64_t out0 = d.off[g];
  for (uint32_t e = threadIdx.x; e < E; e += blockDim.x) {
    double mass, thr;
    bool single;
    fix_query(M, V, ld_idx(&V.hidx[si[e]]) - 1, q0, q1, a.tol, mass, thr, single);
    d.key[out0 + e] = sk[e];
    d.thr[out0 + e] = thr;
  }
  if (threadIdx.x == 0) d.n_ent[g] = E;
}

// k_dict on one spectrum (mode as launch_dict)
template <bool BIG>
__device__ __forceinline__ void dict_spec(const TableArgs& t, const PipeArgs& a, const DictArgs& d, int mode,
                                          FixMeta& M, const FixView& V, int64_t g, uint32_t nr, uint32_t* ent) {
  fix_load(M, V, a, 4 * a.peak_off[g], nr);
  if (mode == 0) hash_clear(V);
  __syncthreads();
  const uint32_t q0 = fix_side_pairs(M, V, 0, a.max_weight);
  const uint32_t q1 = fix_side_pairs(M, V, 1, a.max_weight);
  const uint32_t Q = q0 + q1 + M.n_single;
  const bool exact = a.pair_ok && !a.pair_ok[g];  // budgets can bind: the listed answers
  if (mode == 1) {
    if (threadIdx.x == 0) d.n_q[g] = Q;
    __syncthreads();
    return;
  }
  if (mode == 2) {  // list the exact-mode spectra's queries for the masked explain
    if (exact) fix_list(M, V, a, g, q0, q1, Q);
    return;
  }
  const uint64_t m0 = a.alpha[2 * g], m1 = a.alpha[2 * g + 1];
  const uint32_t xstart = exact ? (uint32_t)(a.xq_block[g] >> 32) : 0u;
  for (uint32_t o = threadIdx.x; o < Q; o += blockDim.x) {
    double mass, thr;
    bool single, pc = true;
    fix_query(M, V, o, q0, q1, a.tol, mass, thr, single);
    uint64_t u0, u1;
    const int8_t st = exact ? a.xa_st[xstart + o] : masked_answer(t, mass, thr, a.prec, a.rprec, m0, m1, u0, u1, pc);
    if (!pc) atomicOr(a.err, 4u);
    if (single || st == SST_SOME) hash_put(V, &M.writers, key_bits(mass), o);
  }
  __syncthreads();
  hash_check(M, V, a);
  if constexpr (BIG) dict_emit_big(M, V, a, d, g, q0, q1);
  else dict_emit_lds(M, V, a, d, g, q0, q1, ent);
  __syncthreads();
}

}  // namespace

// filter_by_explanation's final dict (DictArgs): the last round's queries
// over the final alive rows, answered on the final alphabet; count pass: the
// query count per spectrum; build pass: the last writer per key (the hash of
// k_fix_round), then the entries sorted by key into the spectrum's region.
__global__ __launch_bounds__(kPipeWG) void k_dict(TableArgs t, PipeArgs a, DictArgs d, int mode) {
  __shared__ FixLdsArrays S;
  __shared__ FixMeta M;
  __shared__ uint32_t ent[kHashSlots];
  const FixView V = lds_view(S);
  for (int64_t g = blockIdx.x; g < a.n_spec; g += gridDim.x) {
    const uint32_t nr = a.cnt[g];
    if (nr > (uint32_t)kPipeMaxRows) {  // k_dict_big's
      if (pipe_too_big(a, nr) && threadIdx.x == 0) {
        atomicOr(a.err, 2u);
        if (mode == 1) d.n_q[g] = 0;
        else if (mode == 0) d.n_ent[g] = 0;
        else if (a.pair_ok && !a.pair_ok[g]) a.xq_block[g] = 0;
      }
      continue;
    }
    dict_spec<false>(t, a, d, mode, M, V, g, nr, ent);
  }
}
__global__ __launch_bounds__(kPipeWG) void k_dict_big(TableArgs t, PipeArgs a, DictArgs d, int mode) {
  __shared__ FixMeta M;
  const FixView V = big_view(a);
  for_big_spectra(a, [&](int64_t g, uint32_t nr) {
    if (!pipe_too_big(a, nr)) dict_spec<true>(t, a, d, mode, M, V, g, nr, nullptr);
  });
}

namespace {

// SkeletonBuilder's bins over one spectrum's alive rows (views as FixView)
struct BinView {
  double* su;
  double* ob;
  uint16_t* s0;  // alive rows of each side, SU order
  uint16_t* s1;
  uint16_t* b0;  // per side: first row of each bin, then the row count
  uint16_t* b1;
  uint32_t* q0;  // per side: exclusive prefix of each bin's queries
  uint32_t* q1;
  __device__ __forceinline__ uint16_t* side(int sd) const { return sd ? s1 : s0; }
  __device__ __forceinline__ uint16_t* bstart(int sd) const { return sd ? b1 : b0; }
  __device__ __forceinline__ uint32_t* qoff(int sd) const { return sd ? q1 : q0; }
};
struct BinLdsArrays {
  double su[kPipeMaxRows];
  double ob[kPipeMaxRows];
  uint16_t side[2][kPipeMaxRows];
  uint16_t bstart[2][kPipeMaxRows + 1];
  uint32_t qoff[2][kPipeMaxRows + 1];
};
struct BinMeta {
  uint32_t n_side[2], nb[2];
  uint32_t w[16];
};
__device__ __forceinline__ BinView lds_bin_view(BinLdsArrays& S) {
  return BinView{S.su, S.ob, S.side[0], S.side[1], S.bstart[0], S.bstart[1], S.qoff[0], S.qoff[1]};
}
__device__ __forceinline__ BinView big_bin_view(const PipeArgs& a) {
  const PipeBigLayout B = pipe_big_layout(a.big_rows, a.big_slots);
  uint8_t* p = big_slice(a);
  return BinView{(double*)(p + B.su),   (double*)(p + B.ob),   (uint16_t*)(p + B.s0), (uint16_t*)(p + B.s1),
                 (uint16_t*)(p + B.b0), (uint16_t*)(p + B.b1), (uint32_t*)(p + B.q0), (uint32_t*)(p + B.q1)};
}

// the alive rows of spectrum g and each side's list
__device__ __forceinline__ void bins_load(BinMeta& M, const BinView& V, const PipeArgs& a, int64_t g, uint32_t nr) {
  const int64_t base = 4 * a.peak_off[g];
  uint32_t carry[3] = {0, 0, 0};
  for (uint32_t r0 = 0; r0 < nr; r0 += blockDim.x) {
    const uint32_t r = r0 + threadIdx.x;
    const bool al = r < nr && a.alive[base + r];
    const uint32_t meta = al ? a.r_meta[base + r] : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl(al ? 1u : 0u, M.w, tot);
    const uint32_t i = carry[0] + ex;
    if (al) {
      V.su[i] = a.r_su[base + r];
      V.ob[i] = a.r_ob[base + r];
    }
    carry[0] += tot;
    for (int c = 0; c < 2; ++c) {
      const bool f = al && ((meta >> (2 + c)) & 1u);  // START, END
      const uint32_t x = block_excl(f ? 1u : 0u, M.w, tot);
      if (f) V.side(c)[carry[c + 1] + x] = (uint16_t)i;
      carry[c + 1] += tot;
    }
  }
  if (threadIdx.x == 0) {
    M.n_side[0] = carry[1];
    M.n_side[1] = carry[2];
  }
  __syncthreads();
}

// side sd's bins and each bin's query count prefix; returns the side's queries
__device__ __forceinline__ uint32_t bins_side(BinMeta& M, const BinView& V, int sd, double tol) {
  const uint32_t n = M.n_side[sd];
  const uint16_t* rs = V.side(sd);
  uint16_t* bs = V.bstart(sd);
  uint32_t* qoff = V.qoff(sd);
  uint32_t carry = 0;
  for (uint32_t i0 = 0; i0 < n; i0 += blockDim.x) {
    const uint32_t i = i0 + threadIdx.x;
    // row i joins row i - 1's bin when their SU step is within the pair threshold (:130-136)
    const bool starts =
        i < n && (i == 0 || !(V.su[rs[i]] - V.su[rs[i - 1]] <= tol * (V.ob[rs[i - 1]] + V.ob[rs[i]])));
    uint32_t tot;
    const uint32_t ex = block_excl(starts ? 1u : 0u, M.w, tot);
    if (starts) bs[carry + ex] = (uint16_t)i;
    carry += tot;
  }
  const uint32_t nb = carry;
  if (threadIdx.x == 0) {
    bs[nb] = (uint16_t)n;
    M.nb[sd] = nb;
  }
  __syncthreads();
  carry = 0;
  for (uint32_t b0 = 0; b0 < nb; b0 += blockDim.x) {
    const uint32_t b = b0 + threadIdx.x;
    uint32_t c = 0;
    if (b < nb) {
      const uint32_t size = (uint32_t)bs[b + 1] - bs[b];
      const bool closed = b + 1 < nb || size > 1;  // a later row closes it, or the side's last row joined it
      if (closed) c = b == 0 ? size : ((uint32_t)bs[b] - bs[b - 1]) * size;
    }
    uint32_t tot;
    const uint32_t ex = block_excl(c, M.w, tot);
    if (b < nb) qoff[b] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) qoff[nb] = carry;
  __syncthreads();
  return carry;
}

// query q of side sd: the first bin's whole mass against 0, a later bin's
// (predecessor row, row) difference; threshold as calculate_error_threshold
__device__ __forceinline__ void bins_query(const BinMeta& M, const BinView& V, int sd, uint32_t q, double tol,
                                           double& mass, double& thr) {
  const uint32_t* qoff = V.qoff(sd);
  const uint16_t* bs = V.bstart(sd);
  uint32_t lo = 0, hi = M.nb[sd];  // last bin with qoff <= q (empty bins share their successor's offset)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (qoff[mid] <= q) lo = mid;
    else hi = mid;
  }
  const uint32_t b = lo, local = q - qoff[b];
  const uint16_t* rs = V.side(sd);
  if (b == 0) {
    const uint32_t m = rs[bs[0] + local];
    mass = V.su[m];
    thr = tol * (0.0 + V.ob[m]);
    return;
  }
  const uint32_t csz = (uint32_t)bs[b + 1] - bs[b];
  const uint32_t p = rs[bs[b - 1] + local / csz], r = rs[bs[b] + local % csz];
  mass = V.su[r] - V.su[p];
  thr = tol * (V.ob[p] + V.ob[r]);
}

__device__ __forceinline__ void bins_count_spec(const PipeArgs& a, BinMeta& M, const BinView& V, int64_t g,
                                                uint32_t nr) {
  bins_load(M, V, a, g, nr);
  const uint32_t q0 = bins_side(M, V, 0, a.tol);
  const uint32_t q1 = bins_side(M, V, 1, a.tol);
  if (threadIdx.x == 0) {
    a.n_q[g] = q0 + q1;
    if (a.n_q0) a.n_q0[g] = q0;
  }
  __syncthreads();
}

__device__ __forceinline__ void bins_emit_spec(const TableArgs& t, const PipeArgs& a, BinMeta& M, const BinView& V,
                                               int64_t g, uint32_t nr) {
  bins_load(M, V, a, g, nr);
  const uint32_t q0 = bins_side(M, V, 0, a.tol);
  const uint32_t q1 = bins_side(M, V, 1, a.tol);
  const uint64_t base = a.q_off[g];
  const uint64_t m0 = a.alpha[2 * g], m1 = a.alpha[2 * g + 1];
  for (uint32_t o = threadIdx.x; o < q0 + q1; o += blockDim.x) {
    const int sd = o >= q0;
    double mass, thr;
    bins_query(M, V, sd, sd ? o - q0 : o, a.tol, mass, thr);
    double lof, hif;
    quantise_lean(mass, thr, a.prec, a.rprec, lof, hif);
    int8_t st = SST_NONE;
    uint32_t cnt = 0;
    // off the pair class, or budgets that can bind: listed for the masked explain
    const bool pend = !(hif < (double)t.pair_hi) || (a.pair_ok && !a.pair_ok[g]);
    if (pend) {
      st = (int8_t)kStatusPending;
    } else if (hif >= 0.0) {
      const double af = lof < 1.0 ? 1.0 : lof;
      uint64_t u0 = 0, u1 = 0;
      if (af <= hif) cnt = masked_walk(t, (uint32_t)af, (uint32_t)hif, m0, m1, u0, u1);
      st = cnt ? (int8_t)SST_SOME : lof <= 0.0 ? (int8_t)SST_EMPTY : (int8_t)SST_NONE;
    }
    a.q_status[base + o] = st;
    a.q_count[base + o] = cnt;
    if (a.n_def) {  // one returning atomic per wave instruction
      const uint64_t bal = __ballot(pend);
      if (pend) {
        const int lane = threadIdx.x & 63, leader = __builtin_ctzll(bal);
        uint32_t pos = 0;
        if (lane == leader) pos = atomicAdd(a.n_def, (uint32_t)__builtin_popcountll(bal));
        pos = __shfl(pos, leader, 64) + (uint32_t)__builtin_popcountll(bal & ((1ull << lane) - 1ull));
        a.def_mass[pos] = mass;
        a.def_thr[pos] = thr;
        a.def_spec[pos] = (int32_t)g;
        a.def_q[pos] = base + o;
      }
    }
  }
  __syncthreads();
}

}  // namespace

__global__ __launch_bounds__(kPipeWG) void k_bins_count(PipeArgs a) {
  __shared__ BinLdsArrays S;
  __shared__ BinMeta M;
  const BinView V = lds_bin_view(S);
  for (int64_t g = blockIdx.x; g < a.n_spec; g += gridDim.x) {
    const uint32_t nr = a.cnt[g];
    if (nr > (uint32_t)kPipeMaxRows) {  // k_bins_count_big's
      if (pipe_too_big(a, nr) && threadIdx.x == 0) {
        atomicOr(a.err, 2u);
        a.n_q[g] = 0;
        if (a.n_q0) a.n_q0[g] = 0;
      }
      continue;
    }
    bins_count_spec(a, M, V, g, nr);
  }
}
__global__ __launch_bounds__(kPipeWG) void k_bins_count_big(PipeArgs a) {
  __shared__ BinMeta M;
  const BinView V = big_bin_view(a);
  for_big_spectra(a, [&](int64_t g, uint32_t nr) {
    if (!pipe_too_big(a, nr)) bins_count_spec(a, M, V, g, nr);
  });
}

__global__ __launch_bounds__(kPipeWG) void k_bins_emit(TableArgs t, PipeArgs a) {
  __shared__ BinLdsArrays S;
  __shared__ BinMeta M;
  const BinView V = lds_bin_view(S);
  for (int64_t g = blockIdx.x; g < a.n_spec; g += gridDim.x) {
    const uint32_t nr = a.cnt[g];
    if (nr > (uint32_t)kPipeMaxRows) continue;  // k_bins_emit_big's (or no queries: rejected)
    bins_emit_spec(t, a, M, V, g, nr);
  }
}
__global__ __launch_bounds__(kPipeWG) void k_bins_emit_big(TableArgs t, PipeArgs a) {
  __shared__ BinMeta M;
  const BinView V = big_bin_view(a);
  for_big_spectra(a, [&](int64_t g, uint32_t nr) {
    if (!pipe_too_big(a, nr)) bins_emit_spec(t, a, M, V, g, nr);
  });
}

// exclusive prefix of n u32 counts into n + 1 u64 offsets (one workgroup,
// chunks staged through LDS so that loads and stores are coalesced)
__global__ __launch_bounds__(kPipeWG) void k_scan_u32(const uint32_t* in, uint64_t* out, int64_t n) {
  constexpr int kPer = 8, kChunk = kPer * kPipeWG;
  __shared__ uint64_t s_buf[kChunk];
  __shared__ uint64_t s_w[16];
  uint64_t carry = 0;
  for (int64_t c0 = 0; c0 < n; c0 += kChunk) {
    const int m = (int)(n - c0 < kChunk ? n - c0 : kChunk);
    uint32_t x[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int i = threadIdx.x + k * kPipeWG;
      x[k] = i < m ? in[c0 + i] : 0u;
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) s_buf[threadIdx.x + k * kPipeWG] = x[k];
    __syncthreads();
    uint64_t v[kPer], run = 0;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      v[j] = s_buf[threadIdx.x * kPer + j];
      run += v[j];
    }
    // block-wide exclusive scan of the runs (wave shuffles, then the waves' sums)
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint64_t incl = run;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t y = __shfl_up(incl, d, 64);
      if (lane >= d) incl += y;
    }
    if (lane == 63) s_w[wv] = incl;
    __syncthreads();
    uint64_t base = carry, tot = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
      if (w < wv) base += s_w[w];
      tot += s_w[w];
    }
    base += incl - run;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      s_buf[threadIdx.x * kPer + j] = base;
      base += v[j];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < m; i += blockDim.x) out[c0 + i] = s_buf[i];
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) out[n] = carry;
}

hipError_t launch_dict(const TableArgs& t, const PipeArgs& a, const DictArgs& d, int mode, int n_wg,
                       hipStream_t st) {
  if (a.n_spec <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_dict, dim3(n_wg), dim3(kPipeWG), 0, st, t, a, d, mode);
  if (a.big) hipLaunchKernelGGL(k_dict_big, dim3(a.big_wg), dim3(kPipeWG), 0, st, t, a, d, mode);
  return hipGetLastError();
}
hipError_t launch_scan_u32(const uint32_t* in, uint64_t* out, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL(k_scan_u32, dim3(1), dim3(kPipeWG), 0, st, in, out, n);
  return hipGetLastError();
}

hipError_t launch_bins_count(const PipeArgs& a, int n_wg, hipStream_t st) {
  if (a.n_spec > 0) hipLaunchKernelGGL(k_bins_count, dim3(n_wg), dim3(kPipeWG), 0, st, a);
  if (a.n_spec > 0 && a.big) hipLaunchKernelGGL(k_bins_count_big, dim3(a.big_wg), dim3(kPipeWG), 0, st, a);
  hipLaunchKernelGGL(k_scan_u32, dim3(1), dim3(kPipeWG), 0, st, (const uint32_t*)a.n_q, a.q_off, a.n_spec);
  return hipGetLastError();
}
hipError_t launch_bins_emit(const TableArgs& t, const PipeArgs& a, int n_wg, hipStream_t st) {
  if (a.n_spec <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_bins_emit, dim3(n_wg), dim3(kPipeWG), 0, st, t, a);
  if (a.big) hipLaunchKernelGGL(k_bins_emit_big, dim3(a.big_wg), dim3(kPipeWG), 0, st, t, a);
  return hipGetLastError();
}

hipError_t launch_classify_rows(const TableArgs& t, const PipeArgs& a, int n_wg, hipStream_t st) {
  if (a.n_spec <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_classify_rows, dim3(n_wg), dim3(kPipeWG), 0, st, t, a);
  if (a.big) hipLaunchKernelGGL(k_classify_rows_big, dim3(a.big_wg), dim3(kPipeWG), 0, st, t, a);
  return hipGetLastError();
}
hipError_t launch_fix_finish(const PipeArgs& a, int n_wg, hipStream_t st) {
  if (a.n_spec <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_fix_finish, dim3(n_wg), dim3(kPipeWG), 0, st, a);
  if (a.big) hipLaunchKernelGGL(k_fix_finish_big, dim3(a.big_wg), dim3(kPipeWG), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_fix_round(const TableArgs& t, const PipeArgs& a, int n_wg, hipStream_t st) {
  if (a.n_spec <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_fix_round, dim3(n_wg), dim3(kPipeWG), 0, st, t, a);
  if (a.big) hipLaunchKernelGGL(k_fix_round_big, dim3(a.big_wg), dim3(kPipeWG), 0, st, t, a);
  return hipGetLastError();
}

}  // namespace sst
