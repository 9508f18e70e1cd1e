// sst_rows.hip -- one step of the hot path from the peaks (gfx950):
// classify_fragments' is_valid and filters (fragment_classification.py:17-101)
// and the first filter_by_explanation round's sliding-window explains
// (prediction.py:261-329, without the singletons) with every producer on the
// device, so the explain queries are never written to HBM.
//
// Per spectrum (peaks sorted by mass, as a peak list is):
//   * A7: every peak x breakage weight (su = obs - shift_k, thr = tol * obs)
//     against the full table's last-row bitset, written breakage-major as
//     sst_is_valid_peaks; a row is kept when valid and it passes the
//     intensity / mass / sequence-mass filters (:84-95, :122-139);
//   * each side's rows (START: the breakages naming START, END likewise) in
//     SU order: a breakage's kept rows are already sorted (su = obs - shift
//     with the peaks sorted), so a side is a merge of <= 4 sorted streams --
//     each row's place is its rank in its own stream plus a binary search in
//     each other stream (ties: the breakage-major concat order the
//     reference's stable sort keeps);
//   * the sliding window in closed form (prediction.py:293-328): with s* the
//     first start whose difference to the side's last row is <= max_weight,
//     a start r < s* pairs with r+1 .. E_r (E_r: the last end within
//     max_weight, the reference's exact float test), s* with every later row,
//     and every start after s* only with the last row (the loop's end stays
//     there); pairs in start, then end order;
//   * each pair (s, e): diff = su[e] - su[s], thr = tol * (obs[s] + obs[e])
//     (calculate_error_threshold, l1) -> a pair-class window answered from
//     the LDS pair list (every difference is <= max_weight < 3 w_min).
//
// Three launches: k_rows_count (A7, rows to scratch, per-spectrum totals of
// queries / hits / payload bytes), k_rows_scan (spectrum offsets), k_rows_emit
// (statuses, dense hit list with pair-list refs, dense payload; the last
// workgroup writes the header).  Both spectrum kernels are persistent (one
// 1024-lane workgroup per CU, the 40 KB pair image staged once) and walk the
// spectra grid-stride.  The result is sst_result's dense layout in query order
// (spectrum-major; START pairs, then END pairs).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sst_internal.h"
#include "sst_quant.h"

namespace sst {

namespace {

constexpr int kRowsWG = 1024;

struct PairImg {
  const uint32_t* sums;
  const uint32_t* recs;
  const uint32_t* bk;
  uint32_t base;
  int shift;
};

// the pair-list entries with sums in [a, hi] (a >= 1): count, first entry, record bytes
__device__ __forceinline__ uint32_t img_walk(const PairImg& p, uint32_t a, uint32_t hi, uint32_t& first,
                                             uint32_t& bytes) {
  const uint32_t rel = a > p.base ? a - p.base : 0u;
  uint32_t k = p.bk[rel >> p.shift] & 0xFFFFu;
  const uint32_t a2 = a << 1, h2 = (hi << 1) | 1u;
  while (p.sums[k] < a2) ++k;
  first = k;
  uint32_t nb = 0;
  for (; p.sums[k] <= h2; ++k) nb += 2u + (p.sums[k] & 1u);
  bytes = nb;
  return k - first;
}

typedef uint32_t __attribute__((aligned(1))) u32_unal;

struct SpecLds {
  double obs[kRowsMaxPeaks];
  double su[kRowsMaxSide];
  double ob[kRowsMaxSide];
  uint32_t qoff[kRowsMaxSide + 1];  // exclusive prefix of pairs per start row
  uint16_t kidx[4][kRowsMaxPeaks];  // peak of the j-th kept row of breakage k
  uint8_t keep[kRowsMaxPeaks];      // bit k: the row (k, p) is kept
  uint32_t kcnt[4];
  uint32_t w[16];
  int sstar;
  uint32_t n_side[2];
};

// The side's window pairs: s*, per-row counts and their prefix (rows in
// L.su / L.ob [0, n)); returns the number of pairs.
__device__ uint32_t side_pairs(SpecLds& L, uint32_t n, double mw) {
  if (threadIdx.x == 0) L.sstar = n ? (int)n - 1 : 0;
  __syncthreads();
  for (uint32_t r = threadIdx.x; r + 1 < n; r += blockDim.x)
    if (!(L.su[n - 1] - L.su[r] > mw)) atomicMin(&L.sstar, (int)r);
  __syncthreads();
  const uint32_t ss = (uint32_t)L.sstar;
  uint32_t carry = 0;
  for (uint32_t r0 = 0; r0 < n; r0 += blockDim.x) {
    const uint32_t r = r0 + threadIdx.x;
    uint32_t c = 0;
    if (r + 1 < n) {
      if (r < ss) {  // the last end within max_weight: first e with su[e] - su[r] > mw, minus one
        uint32_t lo = r + 1, hi = n - 1;  // predicate true at n - 1 (r < s*)
        while (lo < hi) {
          const uint32_t mid = (lo + hi) >> 1;
          if (L.su[mid] - L.su[r] > mw) hi = mid;
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
    const uint32_t ex = block_excl(c, L.w, tot);
    if (r < n) L.qoff[r] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) L.qoff[n] = carry;
  __syncthreads();
  return carry;
}

// pair q of the side -> (start, end)
__device__ __forceinline__ void pair_of(const SpecLds& L, uint32_t n, uint32_t q, uint32_t& s, uint32_t& e) {
  uint32_t lo = 0, hi = n;  // last r with qoff[r] <= q
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (L.qoff[mid] <= q) lo = mid;
    else hi = mid;
  }
  s = lo;
  e = s <= (uint32_t)L.sstar ? s + 1 + (q - L.qoff[s]) : n - 1;
}

struct QAns {
  int8_t status;
  uint32_t cnt, first, bytes;
};

__device__ __forceinline__ QAns answer(const SpecLds& L, const PairImg& img, const RowsArgs& a, uint32_t s,
                                       uint32_t e) {
  const double diff = L.su[e] - L.su[s];
  const double thr = a.tol * (L.ob[s] + L.ob[e]);
  double lof, hif;
  quantise_lean(diff, thr, a.prec, a.rprec, lof, hif);
  QAns r{SST_NONE, 0, 0, 0};
  if (lof <= hif && hif >= 0.0) {
    const double af = lof < 1.0 ? 1.0 : lof;
    if (af <= hif) r.cnt = img_walk(img, (uint32_t)af, (uint32_t)hif, r.first, r.bytes);
    if (r.cnt > a.cap) r.status = SST_OVERFLOW;
    else if (r.cnt) r.status = SST_SOME;
    else if (lof <= 0.0) r.status = SST_EMPTY;  // v == 0 in the window: the empty solution only
  }
  return r;
}

__device__ void stage_img(const TableArgs& t, uint32_t* dyn, PairImg& img) {
  const int n_s = t.n_pairs + 2;
  const int words = 2 * n_s + t.n_buckets;
  for (int k = threadIdx.x; k < words; k += blockDim.x) dyn[k] = t.pair_data[k];
  img.sums = dyn;
  img.recs = dyn + n_s;
  img.bk = dyn + 2 * n_s;
  img.base = t.pair_base;
  img.shift = t.pair_shift;
  __syncthreads();
}

// A7, filters, kept-row compaction and both sides' merged rows of spectrum g
// (rows to L and, when `to_scratch`, to the scratch rows); returns false for a
// spectrum larger than the workgroup's LDS (reported to the host)
__device__ bool load_spectrum(SpecLds& L, const TableArgs& t, const RowsArgs& a, int64_t g, bool classify) {
  const int64_t p0 = a.peak_off[g];
  const uint32_t P = (uint32_t)(a.peak_off[g + 1] - p0);
  if (P > (uint32_t)kRowsMaxPeaks) return false;
  const double su_seq = a.su_seq[g];
  for (uint32_t p = threadIdx.x; p < P; p += blockDim.x) {
    const double o = a.obs[p0 + p];
    L.obs[p] = o;
    uint8_t kp = 0;
    for (int k = 0; k < a.n_shifts; ++k) {
      const double su = o - a.shift[k];
      int8_t code;
      if (classify) {
        double lof, hif;
        quantise_lean(su, a.tol * o, a.prec, a.rprec, lof, hif);
        code = valid_window(t.valid, t.limit, (int64_t)lof, (int64_t)hif, t.full_lo, t.full_hi, t.first_reach);
        a.valid_out[(int64_t)k * a.n_peaks + p0 + p] = code;
      } else {
        code = a.valid_out[(int64_t)k * a.n_peaks + p0 + p];  // k_rows_emit: the codes k_rows_count wrote
      }
      const bool inten = a.intensity ? a.intensity[p0 + p] > a.intensity_cutoff : true;
      const bool full = (a.sides[k] & 3) == 3;  // START and END: filter_by_sequence_mass's lower cut
      const bool keep = code == 1 && inten && o < a.mass_cutoff && su < su_seq + a.max_variance &&
                        (su > su_seq - a.max_variance || !full);
      kp |= (uint8_t)keep << k;
    }
    L.keep[p] = kp;
  }
  __syncthreads();
  // per breakage: kept rows in peak order (= SU order)
  for (int k = 0; k < a.n_shifts; ++k) {
    uint32_t carry = 0;
    for (uint32_t p0_ = 0; p0_ < P; p0_ += blockDim.x) {
      const uint32_t p = p0_ + threadIdx.x;
      const uint32_t f = p < P ? (L.keep[p] >> k) & 1u : 0u;
      uint32_t tot;
      const uint32_t ex = block_excl(f, L.w, tot);
      if (f) L.kidx[k][carry + ex] = (uint16_t)p;
      carry += tot;
    }
    if (threadIdx.x == 0) L.kcnt[k] = carry;
  }
  __syncthreads();
  return true;
}

// merge side `sd` (0 START, 1 END) into L.su / L.ob; returns its row count
__device__ uint32_t merge_side(SpecLds& L, const RowsArgs& a, int sd) {
  uint32_t n = 0;
  for (int k = 0; k < a.n_shifts; ++k)
    if ((a.sides[k] >> sd) & 1) n += L.kcnt[k];
  if (n > (uint32_t)kRowsMaxSide) return 0xFFFFFFFFu;
  for (int k = 0; k < a.n_shifts; ++k) {
    if (!((a.sides[k] >> sd) & 1)) continue;
    const double sk = a.shift[k];
    for (uint32_t j = threadIdx.x; j < L.kcnt[k]; j += blockDim.x) {
      const uint32_t p = L.kidx[k][j];
      const double su = L.obs[p] - sk;
      uint32_t pos = j;
      for (int k2 = 0; k2 < a.n_shifts; ++k2) {
        if (k2 == k || !((a.sides[k2] >> sd) & 1)) continue;
        const double s2 = a.shift[k2];
        // rows of k2 before (su, k): su2 < su, or su2 == su for an earlier breakage
        uint32_t lo = 0, hi = L.kcnt[k2];
        while (lo < hi) {
          const uint32_t mid = (lo + hi) >> 1;
          const double v = L.obs[L.kidx[k2][mid]] - s2;
          if (v < su || (v == su && k2 < k)) lo = mid + 1;
          else hi = mid;
        }
        pos += lo;
      }
      L.su[pos] = su;
      L.ob[pos] = L.obs[p];
    }
  }
  __syncthreads();
  return n;
}

}  // namespace

__global__ __launch_bounds__(kRowsWG) void k_rows_count(TableArgs t, RowsArgs a) {
  extern __shared__ uint32_t dyn[];
  __shared__ SpecLds L;
  __shared__ uint32_t s_acc[3];
  PairImg img;
  stage_img(t, dyn, img);
  for (int64_t g = blockIdx.x; g < a.n_spec; g += gridDim.x) {
    if (!load_spectrum(L, t, a, g, true)) {
      if (threadIdx.x == 0) {
        atomicOr(a.err, 1u);
        a.totals[3 * g] = a.totals[3 * g + 1] = a.totals[3 * g + 2] = 0;
        a.side_rows[2 * g] = a.side_rows[2 * g + 1] = 0;
      }
      continue;
    }
    if (threadIdx.x < 3) s_acc[threadIdx.x] = 0;
    uint32_t nq = 0, nside[2] = {0, 0};
    for (int sd = 0; sd < 2; ++sd) {
      const uint32_t n = merge_side(L, a, sd);
      if (n == 0xFFFFFFFFu) {
        if (threadIdx.x == 0) atomicOr(a.err, 2u);
        break;
      }
      nside[sd] = n;
      // the side's rows to scratch (k_rows_emit reads them back)
      double* rs = a.rows_su + 4 * a.peak_off[g] + (sd ? 2 * (a.peak_off[g + 1] - a.peak_off[g]) : 0);
      double* ro = a.rows_ob + 4 * a.peak_off[g] + (sd ? 2 * (a.peak_off[g + 1] - a.peak_off[g]) : 0);
      for (uint32_t r = threadIdx.x; r < n; r += blockDim.x) {
        rs[r] = L.su[r];
        ro[r] = L.ob[r];
      }
      const uint32_t Q = side_pairs(L, n, a.max_weight);
      uint32_t h = 0, b = 0;
      for (uint32_t q = threadIdx.x; q < Q; q += blockDim.x) {
        uint32_t s, e;
        pair_of(L, n, q, s, e);
        const QAns r = answer(L, img, a, s, e);
        h += (r.status == SST_SOME || r.status == SST_OVERFLOW);
        b += r.status == SST_SOME ? r.bytes + 2u : 0u;
      }
      if (h) atomicAdd(&s_acc[1], h);
      if (b) atomicAdd(&s_acc[2], b);
      nq += Q;
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      a.totals[3 * g] = nq;
      a.totals[3 * g + 1] = s_acc[1];
      a.totals[3 * g + 2] = s_acc[2];
      a.side_rows[2 * g] = nside[0];
      a.side_rows[2 * g + 1] = nside[1];
    }
    __syncthreads();
  }
}

// exclusive offsets of every spectrum's queries, hits and payload bytes (one
// workgroup) and the totals
__global__ __launch_bounds__(kRowsWG) void k_rows_scan(RowsArgs a) {
  __shared__ uint32_t s_w[16];
  uint64_t carry[3] = {0, 0, 0};
  for (int64_t g0 = 0; g0 < a.n_spec; g0 += blockDim.x) {
    const int64_t g = g0 + threadIdx.x;
    for (int c = 0; c < 3; ++c) {
      const uint32_t v = g < a.n_spec ? a.totals[3 * g + c] : 0u;
      uint32_t tot;
      const uint32_t ex = block_excl(v, s_w, tot);
      if (g < a.n_spec) a.offs[3 * g + c] = carry[c] + ex;
      carry[c] += tot;
    }
  }
  if (threadIdx.x == 0) {
    a.ctl[0] = carry[0];
    a.ctl[1] = carry[1];
    a.ctl[2] = carry[2];
    if (carry[0] > a.cap_queries || carry[1] > a.cap_queries || carry[2] > a.cap_bytes) atomicOr(a.err, 4u);
  }
}

__global__ __launch_bounds__(kRowsWG) void k_rows_emit(TableArgs t, RowsArgs a) {
  extern __shared__ uint32_t dyn[];
  __shared__ SpecLds L;
  PairImg img;
  stage_img(t, dyn, img);
  const bool room = !(*(volatile uint32_t*)a.err & 4u);
  for (int64_t g = blockIdx.x; g < a.n_spec && room; g += gridDim.x) {
    if (a.peak_off[g + 1] - a.peak_off[g] > kRowsMaxPeaks) continue;
    uint64_t qb = a.offs[3 * g], hb = a.offs[3 * g + 1], bb = a.offs[3 * g + 2];
    for (int sd = 0; sd < 2; ++sd) {
      const uint32_t n = a.side_rows[2 * g + sd];
      const double* rs = a.rows_su + 4 * a.peak_off[g] + (sd ? 2 * (a.peak_off[g + 1] - a.peak_off[g]) : 0);
      const double* ro = a.rows_ob + 4 * a.peak_off[g] + (sd ? 2 * (a.peak_off[g + 1] - a.peak_off[g]) : 0);
      for (uint32_t r = threadIdx.x; r < n; r += blockDim.x) {
        L.su[r] = rs[r];
        L.ob[r] = ro[r];
      }
      __syncthreads();
      const uint32_t Q = side_pairs(L, n, a.max_weight);
      for (uint32_t q0 = 0; q0 < Q; q0 += blockDim.x) {
        const uint32_t q = q0 + threadIdx.x;
        QAns r{SST_NONE, 0, 0, 0};
        if (q < Q) {
          uint32_t s, e;
          pair_of(L, n, q, s, e);
          r = answer(L, img, a, s, e);
          a.status[qb + q] = r.status;
        }
        const bool hit = r.status == SST_SOME || r.status == SST_OVERFLOW;
        uint32_t th, tb;
        const uint32_t xh = block_excl(hit ? 1u : 0u, L.w, th);
        const uint32_t xb = block_excl(r.status == SST_SOME ? r.bytes + 2u : 0u, L.w, tb);
        if (hit) {
          const uint64_t off = bb + xb;
          const uint64_t word = r.status == SST_SOME ? off : (uint64_t)r.cnt;
          a.hits[hb + xh] = make_uint4((uint32_t)(qb + q), r.cnt, (uint32_t)word, (uint32_t)(word >> 32));
          a.refs[hb + xh] = (uint16_t)(r.first | (r.status == SST_OVERFLOW ? 0x8000u : 0u));
          if (r.status == SST_SOME) {
            uint8_t* dst = a.dense + off;
            for (uint32_t k = r.first; k < r.first + r.cnt; ++k) {
              const uint32_t rec = img.recs[k];
              *(u32_unal*)dst = rec;  // the 2 pad bytes after the query's last record take the overhang
              dst += (rec & 0xFFu) + 1u;
            }
          }
        }
        hb += th;
        bb += tb;
      }
      qb += Q;
      __syncthreads();
    }
  }
  // the last workgroup to finish writes the header the host polls
  __shared__ uint32_t s_last;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    s_last = atomicAdd(a.done, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (s_last && threadIdx.x == 0) {
    __threadfence();
    *a.done = 0;  // the next pass's counters
    const uint32_t err = *(volatile uint32_t*)a.err;
    *a.err = 0;
    uint64_t h[kHdrWords] = {0};
    h[kHdrHits] = a.ctl[1];
    h[kHdrPayload] = a.ctl[2];
    h[kHdrPass] = a.pass_id;
    h[kHdrQueries] = a.ctl[0];
    h[kHdrRowsErr] = err;
    for (int k = 0; k < kHdrWords; ++k) a.hdr[k] = h[k];
    for (int k = 0; k < kHdrWords; ++k)
      __hip_atomic_store(a.hdr_host + k, h[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

size_t rows_lds_bytes() { return sizeof(SpecLds); }

hipError_t launch_rows_step(const TableArgs& t, const RowsArgs& a, int n_wg, size_t dyn, hipStream_t st) {
  if (a.n_spec <= 0 || !t.pairs_enabled) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_rows_count, dim3(n_wg), dim3(kRowsWG), dyn, st, t, a);
  hipLaunchKernelGGL(k_rows_scan, dim3(1), dim3(kRowsWG), 0, st, a);
  hipLaunchKernelGGL(k_rows_emit, dim3(n_wg), dim3(kRowsWG), dyn, st, t, a);
  return hipGetLastError();
}

}  // namespace sst
