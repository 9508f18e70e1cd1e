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
// Launches: k_rows_count_w (one wave per contiguous chunk of spectra, each
// spectrum of <= 160 peaks in turn; larger spectra are listed for
// k_rows_count, one workgroup each): A7, every window pair answered once
// (each 64-query window's mask of answers other than NONE, and those
// answers' 4-B words, to scratch: the pass's one answer per pair), per-spectrum
// totals of queries / hits / payload bytes and each chunk's sums;
// k_rows_emit_w: each chunk's exclusive offsets from the 64-chunk tiles' sums
// (added up by the count kernels) and its own tile's earlier chunks (no scan
// launch), each spectrum's offsets (its chunk's plus the chunk's earlier
// spectra's totals), then a pass over its windows writing every status byte,
// and per block of 64 stored answers the dense hit records with pair-list
// refs and the dense payload; k_rows_count / k_rows_emit do the same for the
// big spectra (rows to scratch, answered in both passes); the last workgroup
// writes the header.  The result is sst_result's dense layout
// in query order (spectrum-major; START pairs, then END pairs).
#include <hip/hip_runtime.h>
#include <mutex>
#include <stdint.h>

#include "sst_internal.h"
#include "sst_quant.h"

namespace sst {

#ifdef SST_ROWS_PROF  // phase clocks of the wave kernels (diagnostic builds; printed by the last workgroup)
__device__ unsigned long long g_rows_prof[12];
#define RPROF_T(v) const uint64_t v = wall_clock64()
#define RPROF_ADD(i, d) \
  if ((threadIdx.x & 63) == 0) atomicAdd(&g_rows_prof[i], (unsigned long long)(d))
#else
#define RPROF_T(v)
#define RPROF_ADD(i, d)
#endif

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
  uint16_t ord[kRowsMaxPeaks];      // peaks in (mass, position) order when they do not come sorted
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

// A stored answer (the count pass's 4 B per query): count << 16 | first
// entry; a pair without entries stores its status instead (0 NONE, 1 EMPTY).
// SOME / OVERFLOW follow from the count and the cap; the record bytes from
// the records themselves (ans_bytes), which the emit reads anyway.
__device__ __forceinline__ uint32_t ans_word(const QAns& r) {
  return r.cnt ? ((r.cnt & 0xFFFFu) << 16 | (r.first & 0xFFFFu)) : (r.status == SST_EMPTY ? 1u : 0u);
}
__device__ __forceinline__ QAns ans_read(uint32_t v, uint32_t cap) {
  QAns r{SST_NONE, v >> 16, 0, 0};
  if (r.cnt) {
    r.first = v & 0xFFFFu;
    r.status = r.cnt > cap ? SST_OVERFLOW : SST_SOME;
  } else if (v & 1u) {
    r.status = SST_EMPTY;
  }
  return r;
}
// The count pass's stored answers: per 64-query window of a side, the mask
// of its queries with an answer other than NONE (ans_mask, 8 B at 128 g +
// 64 sd + window: a stored side has <= 60 windows), and the side's answers
// other than NONE, in query order (ans_ent, 4-B words from 64 ans_win_base
// on).  Side sd of spectrum g owns ceil(kRowsAnsPerPeak P / 64) 64-word
// blocks from ans_win_base on, which never reach the next side's first
// (floor(x + y) - floor(x) >= floor(y), plus one per side).
__device__ __forceinline__ uint64_t ans_win_base(int64_t p0, uint32_t P, int sd, int64_t g) {
  return (uint64_t)kRowsAnsPerPeak * (2 * (uint64_t)p0 + (uint64_t)sd * P) / 64 + 2 * (uint64_t)g + (uint64_t)sd;
}
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// the payload bytes of records [first, first + cnt): record k takes
// (recs[k] & 0xFF) + 1 bytes
__device__ __forceinline__ uint32_t ans_bytes(const uint32_t* recs, uint32_t first, uint32_t cnt) {
  uint32_t nb = 0;
  for (uint32_t k0 = first; k0 < first + cnt; k0 += 4) {
    uint32_t rec[4];
#pragma unroll
    for (int x = 0; x < 4; ++x) rec[x] = k0 + x < first + cnt ? recs[k0 + x] : 0xFFFFFFFFu;
#pragma unroll
    for (int x = 0; x < 4; ++x) nb += rec[x] != 0xFFFFFFFFu ? (rec[x] & 0xFFu) + 1u : 0u;
  }
  return nb;
}

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
  // peaks in mass order (ranked here when the list is not sorted; equal
  // masses in their given order): each breakage's kept rows in SU order
  bool ok = true;
  for (uint32_t p = threadIdx.x; p + 1 < P; p += blockDim.x) ok &= L.obs[p] <= L.obs[p + 1];
  const bool sorted = __syncthreads_and(ok);
  if (!sorted) {
    for (uint32_t p = threadIdx.x; p < P; p += blockDim.x) {
      const double o = L.obs[p];
      uint32_t rank = 0;
      for (uint32_t q = 0; q < P; ++q) {
        const double v = L.obs[q];
        rank += (v < o) | ((v == o) & (q < p));
      }
      L.ord[rank] = (uint16_t)p;
    }
    __syncthreads();
  }
  for (int k = 0; k < a.n_shifts; ++k) {
    uint32_t carry = 0;
    for (uint32_t p0_ = 0; p0_ < P; p0_ += blockDim.x) {
      const uint32_t i = p0_ + threadIdx.x;
      const uint32_t p = i < P ? (sorted ? i : L.ord[i]) : 0u;
      const uint32_t f = i < P ? (L.keep[p] >> k) & 1u : 0u;
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
  const uint32_t n_big = a.tickets[2];  // spectra k_rows_count_w left to the block kernels
  if (n_big == 0) return;
  PairImg img;
  stage_img(t, dyn, img);
  for (uint32_t i = blockIdx.x; i < n_big; i += gridDim.x) {
    const int64_t g = a.big[i];
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
      // into its chunk's totals (the wave kernel wrote the chunk's other spectra's)
      unsigned long long* ct = a.chunk_tot + 3 * (g / a.chunk);
      unsigned long long* tt = a.tile_tot + a.tile_par * 3 * a.n_tiles + 3 * (g / a.chunk / kRowsTile);
      if (nq) atomicAdd(ct, (unsigned long long)nq);
      if (s_acc[1]) atomicAdd(ct + 1, (unsigned long long)s_acc[1]);
      if (s_acc[2]) atomicAdd(ct + 2, (unsigned long long)s_acc[2]);
      if (nq) atomicAdd(tt, (unsigned long long)nq);
      if (s_acc[1]) atomicAdd(tt + 1, (unsigned long long)s_acc[1]);
      if (s_acc[2]) atomicAdd(tt + 2, (unsigned long long)s_acc[2]);
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(kRowsWG) void k_rows_emit(TableArgs t, RowsArgs a) {
  extern __shared__ uint32_t dyn[];
  __shared__ SpecLds L;
  // the spectra over kWP peaks (both sides from the rows the workgroup count
  // left in scratch) and the wave kernels' spectra with a side past its answer
  // slots (that side from its scratch rows, the other's stored answers)
  const uint32_t n_big = a.tickets[2], n_all = n_big + a.tickets[1];
  PairImg img;
  if (n_all) stage_img(t, dyn, img);
  const bool room = !(*(volatile uint32_t*)a.err & 4u);
  for (uint32_t i = blockIdx.x; i < n_all && room; i += gridDim.x) {
    const bool redo = i >= n_big;
    const int64_t g = redo ? a.redo[i - n_big] : a.big[i];
    if (a.peak_off[g + 1] - a.peak_off[g] > kRowsMaxPeaks) continue;
    // its offsets: its chunk's plus the chunk's earlier spectra's totals
    __shared__ unsigned long long s_off[3];
    const int64_t ch = g / a.chunk;
    if (threadIdx.x < 3) s_off[threadIdx.x] = a.chunk_off[3 * ch + threadIdx.x];
    __syncthreads();
    for (int64_t h = ch * a.chunk + threadIdx.x; h < g; h += blockDim.x)
      for (int c = 0; c < 3; ++c)
        if (a.totals[3 * h + c]) atomicAdd(&s_off[c], (unsigned long long)a.totals[3 * h + c]);
    __syncthreads();
    uint64_t qb = s_off[0], hb = s_off[1], bb = s_off[2];
    __syncthreads();
    const int64_t P = a.peak_off[g + 1] - a.peak_off[g];
    for (int sd = 0; sd < 2; ++sd) {
      const uint32_t n = a.side_rows[2 * g + sd];
      const bool stored = redo && a.ans_q[2 * g + sd] != 0xFFFFFFFFu;  // the count pass's answers, in query order
      const uint64_t wb = ans_win_base(a.peak_off[g], (uint32_t)P, sd, g);
      uint32_t Q;
      if (stored) {
        Q = a.ans_q[2 * g + sd];
      } else {
        const double* rs = a.rows_su + 4 * a.peak_off[g] + (sd ? 2 * P : 0);
        const double* ro = a.rows_ob + 4 * a.peak_off[g] + (sd ? 2 * P : 0);
        for (uint32_t r = threadIdx.x; r < n; r += blockDim.x) {
          L.su[r] = rs[r];
          L.ob[r] = ro[r];
        }
        __syncthreads();
        Q = side_pairs(L, n, a.max_weight);
      }
      for (uint32_t q0 = 0; q0 < Q; q0 += blockDim.x) {
        const uint32_t q = q0 + threadIdx.x;
        QAns r{SST_NONE, 0, 0, 0};
        if (q < Q) {
          if (stored) {
            const uint64_t* mk = a.ans_mask + 128 * g + 64 * sd;
            const uint64_t m = mk[q / 64], below = (1ull << (q & 63)) - 1ull;
            if ((m >> (q & 63)) & 1ull) {
              uint32_t e = (uint32_t)__builtin_popcountll(m & below);  // the side's answers before q
              for (uint32_t w = 0; w < q / 64; ++w) e += (uint32_t)__builtin_popcountll(mk[w]);
              r = ans_read(a.ans_ent[wb * 64 + e], a.cap);
            }
            if (r.status == SST_SOME) r.bytes = ans_bytes(img.recs, r.first, r.cnt);
          } else {
            uint32_t s, e;
            pair_of(L, n, q, s, e);
            r = answer(L, img, a, s, e);
          }
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
    a.tickets[0] = a.tickets[1] = a.tickets[2] = 0;
    const uint32_t err = *(volatile uint32_t*)a.err;
    *a.err = 0;
    uint64_t h[kHdrWords] = {0};
    h[kHdrHits] = a.ctl[1];
    h[kHdrPayload] = a.ctl[2];
    h[kHdrPass] = a.pass_id;
    h[kHdrQueries] = a.ctl[0];
    h[kHdrRowsErr] = err;
#ifdef SST_ROWS_PROF
    printf("rows prof (wall_clock64 ticks, summed over spectra): head %llu load %llu merge %llu answer %llu tail %llu n %llu | emit head %llu body %llu | wave life %llu waves %llu grid %llu\n",
           g_rows_prof[0], g_rows_prof[1], g_rows_prof[2], g_rows_prof[3], g_rows_prof[4], g_rows_prof[5],
           g_rows_prof[6], g_rows_prof[7], g_rows_prof[8], g_rows_prof[9], g_rows_prof[10]);
    for (int k = 0; k < 12; ++k) g_rows_prof[k] = 0;
#endif
    for (int k = 0; k < kHdrWords; ++k) a.hdr[k] = h[k];
    for (int k = 0; k < kHdrWords; ++k)
      __hip_atomic_store(a.hdr_host + k, h[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---------------------------------------------------------------------------
// One wave per spectrum (spectra of <= kRowsWaveMaxPeaks peaks, i.e. every
// spectrum of a 10..20-mer): a spectrum's phases are short dependent chains
// (bitset loads, LDS binary searches, pair-list walks), so many spectra must
// be in flight per CU -- one wave per workgroup, many workgroups per CU,
// each wave its own spectrum, wave-level prefix sums (no barriers).  The
// pair list is read through L2 (40 KB, resident); the block kernels above
// take the larger spectra.
namespace {

constexpr int kWP = kRowsWaveMaxPeaks;
constexpr int kWS = 2 * kRowsWaveMaxPeaks;  // rows per side: two breakages per side
constexpr int kWavesPerWG = 1;  // one wave per workgroup: a finished spectrum frees its slot at once
                                 // (4-wave workgroups held theirs until the slowest of the four: 168 vs 140 us)

struct WaveLds {
  double obs[kWP];           // the spectrum's peaks in mass order (equal masses in their given order)
  double su[kWS];            // the side's rows in SU order
  uint8_t rp[kWS];           // each row's peak (its observed mass: the pair threshold)
  uint16_t qoff[kWS + 1];    // a side has < 2^16 pairs (kWS (kWS - 1) / 2)
  uint8_t kidx[4][kWP];      // peak of the j-th kept row of breakage k (mass order)
  uint8_t keep[kWP];         // bit k: the row (k, p) is kept
  uint32_t kcnt[4];
  uint32_t sstar;
  uint32_t hist[64];  // wave_pair_window: starts per position of a 64-query window
};
static_assert(kWP < 256, "u8 peak indices and kept-row counts");
static_assert(kRowsAnsPerPeak * kWP <= 64 * 64, "a stored side's window masks: one per lane of a wave (<= 64 windows)");

// LDS written by some lanes of the wave, read by others: order the accesses
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// inclusive prefix sum over the wave's 64 lanes: DPP row shifts within each
// 16-lane row, then row broadcasts of lanes 15 and 31 (VALU only, no LDS
// round trip as a ds_bpermute-based shuffle would take)
__device__ __forceinline__ uint32_t wave_incl(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return x;
}
__device__ __forceinline__ uint32_t wave_excl(uint32_t v, uint32_t& total) {
  const uint32_t incl = wave_incl(v);
  total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  return incl - v;
}
__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint32_t y = __shfl_xor(v, d, 64);
    v = y < v ? y : v;
  }
  return v;
}

// A7, filters and the kept rows of every breakage (mass order) of spectrum g.
// (Hoisting every breakage's bitset loads ahead of the code stores measured
// no faster: most windows meet the all-reachable run and load nothing, and
// the hoisted form took 17 more VGPRs.)
__device__ void wave_load(WaveLds& L, const TableArgs& t, const RowsArgs& a, int64_t p0, uint32_t P, double su_seq,
                          bool write_a7) {
  const int lane = threadIdx.x & 63;
  for (uint32_t p = lane; p < P; p += 64) {
    const double o = a.obs[p0 + p];
    uint8_t kp = 0;
    for (int k = 0; k < a.n_shifts; ++k) {
      const double su = o - a.shift[k];
      double lof, hif;
      quantise_lean(su, a.tol * o, a.prec, a.rprec, lof, hif);
      const int8_t code =
          valid_window(t.valid, t.limit, (int64_t)lof, (int64_t)hif, t.full_lo, t.full_hi, t.first_reach);
      if (write_a7) a.valid_out[(int64_t)k * a.n_peaks + p0 + p] = code;
      const bool inten = a.intensity ? a.intensity[p0 + p] > a.intensity_cutoff : true;
      const bool full = (a.sides[k] & 3) == 3;
      const bool keep = code == 1 && inten && o < a.mass_cutoff && su < su_seq + a.max_variance &&
                        (su > su_seq - a.max_variance || !full);
      kp |= (uint8_t)keep << k;
    }
    L.obs[p] = o;
    L.keep[p] = kp;
  }
  wsync();
  // a peak list need not be sorted: rank the peaks by mass (equal masses in
  // their given order) and rewrite them in that order (the rows need only
  // their masses, never the peak's position in the list)
  bool sorted = true;
  for (uint32_t p = lane; p + 1 < P; p += 64) sorted &= L.obs[p] <= L.obs[p + 1];
  sorted = __ballot(!sorted) == 0;
  if (!sorted) {
    double ov[(kWP + 63) / 64];
    uint8_t kv[(kWP + 63) / 64];
    uint32_t rv[(kWP + 63) / 64];
#pragma unroll
    for (int i = 0; i < (kWP + 63) / 64; ++i) {
      const uint32_t p = lane + 64u * i;
      rv[i] = 0xFFFFFFFFu;
      if (p >= P) continue;
      const double o = L.obs[p];
      uint32_t rank = 0;
      for (uint32_t q = 0; q < P; ++q) {
        const double v = L.obs[q];
        rank += (v < o) | ((v == o) & (q < p));
      }
      ov[i] = o;
      kv[i] = L.keep[p];
      rv[i] = rank;
    }
    wsync();
#pragma unroll
    for (int i = 0; i < (kWP + 63) / 64; ++i)
      if (rv[i] != 0xFFFFFFFFu) {
        L.obs[rv[i]] = ov[i];
        L.keep[rv[i]] = kv[i];
      }
    wsync();
  }
  for (int k = 0; k < a.n_shifts; ++k) {
    uint32_t carry = 0;
    for (uint32_t q0 = 0; q0 < P; q0 += 64) {
      const uint32_t i = q0 + lane;
      const bool f = i < P && ((L.keep[i] >> k) & 1u);
      const uint64_t bal = __ballot(f);
      if (f)
        L.kidx[k][carry + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u))] = (uint8_t)i;
      carry += (uint32_t)__builtin_popcountll(bal);
    }
    if (lane == 0) L.kcnt[k] = carry;
  }
}

// side sd's rows into L.su / L.rp (SU order) and its window pairs' prefix;
// returns the row count (or ~0 when it does not fit) and the pair count.  Row
// j of breakage k goes to j plus, for each other breakage k2 of the side, the
// kept rows of k2 before it (binary search; ties: the earlier breakage first).
__device__ uint32_t wave_side(WaveLds& L, const RowsArgs& a, int sd, uint32_t& Q) {
  const int lane = threadIdx.x & 63;
  uint32_t n = 0;
  for (int k = 0; k < a.n_shifts; ++k)
    if ((a.sides[k] >> sd) & 1) n += L.kcnt[k];
  Q = 0;
  if (n > (uint32_t)kWS) return 0xFFFFFFFFu;
  for (int k = 0; k < a.n_shifts; ++k) {
    if (!((a.sides[k] >> sd) & 1)) continue;
    const double sk = a.shift[k];
    for (uint32_t j = lane; j < L.kcnt[k]; j += 64) {
      const uint32_t p = L.kidx[k][j];
      const double su = L.obs[p] - sk;
      uint32_t pos = j;
      for (int k2 = 0; k2 < a.n_shifts; ++k2) {
        if (k2 == k || !((a.sides[k2] >> sd) & 1)) continue;
        const double s2 = a.shift[k2];
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
      L.rp[pos] = (uint8_t)p;
    }
  }
  wsync();
  // s*: the first start whose difference to the last row is within max_weight
  uint32_t ss = n ? n - 1 : 0;
  for (uint32_t r = lane; r + 1 < n; r += 64)
    if (!(L.su[n - 1] - L.su[r] > a.max_weight)) ss = r < ss ? r : ss;
  ss = wave_min(ss);
  uint32_t carry = 0;
  for (uint32_t r0 = 0; r0 < n; r0 += 64) {
    const uint32_t r = r0 + lane;
    uint32_t c = 0;
    if (r + 1 < n) {
      if (r < ss) {
        uint32_t lo = r + 1, hi = n - 1;
        const double sr = L.su[r];
        while (lo < hi) {
          const uint32_t mid = (lo + hi) >> 1;
          if (L.su[mid] - sr > a.max_weight) hi = mid;
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
    const uint32_t ex = wave_excl(c, tot);
    if (r < n) L.qoff[r] = carry + ex;
    carry += tot;
  }
  if (lane == 0) {
    L.qoff[n] = carry;
    L.sstar = ss;
  }
  wsync();
  Q = carry;
  return n;
}

__device__ __forceinline__ void wave_pair(const WaveLds& L, uint32_t n, uint32_t q, uint32_t& s, uint32_t& e) {
  uint32_t lo = 0, hi = n;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (L.qoff[mid] <= q) lo = mid;
    else hi = mid;
  }
  s = lo;
  e = s <= L.sstar ? s + 1 + (q - L.qoff[s]) : n - 1;
}

// The pairs of queries q0 + lane (q0 a multiple of 64; qoff[s0] <= q0):
// lane j looks at start r = s0 + 1 + j, whose first query sits at position
// qoff[r] - q0 of the window; a histogram of those positions and its prefix
// give each lane its start, the last r with qoff[r] <= q (as wave_pair's
// binary search, without one per lane).  Returns the start of query q0 + 64;
// a window whose 64 looked-at starts all begin in it (starts without pairs)
// falls back to the binary search.
__device__ __forceinline__ uint32_t wave_pair_window(WaveLds& L, uint32_t n, uint32_t q0, uint32_t s0, uint32_t& s,
                                                     uint32_t& e) {
  const int lane = threadIdx.x & 63;
  const uint32_t r = s0 + 1u + (uint32_t)lane;
  const uint32_t pos = r < n ? L.qoff[r] - q0 : 0xFFFFFFFFu;
  L.hist[lane] = 0u;
  wsync();
  if (pos < 64u) atomicAdd(&L.hist[pos], 1u);
  wsync();
  uint32_t tot;
  const uint32_t cnt = wave_excl(L.hist[lane], tot) + L.hist[lane];  // starts at positions <= lane
  const uint64_t at64 = __ballot(pos == 64u);
  const bool full = (uint32_t)__builtin_amdgcn_readlane((int)pos, 63) <= 64u;  // lane 63's start begins by q0 + 64: maybe more beyond it
  const uint32_t q = q0 + (uint32_t)lane;
  wsync();  // the histogram is rewritten by the next window
  if (!full) {
    s = s0 + cnt;
    e = s <= L.sstar ? s + 1u + (q - L.qoff[s]) : n - 1u;
    return s0 + tot + (uint32_t)__builtin_popcountll(at64);
  }
  wave_pair(L, n, q, s, e);
  uint32_t s1, e1;
  wave_pair(L, n, q0 + 64u, s1, e1);
  return s1;
}

// A pair's answer: wave_ask quantises the pair's window and loads its two
// census words (the pair-list entries with sums <= each end: none for an
// inactive lane or a window without a whole mass), wave_reply forms the
// status, count, first entry and record bytes from them.
struct QAsk {
  uint32_t x, y;  // census words at the window's lower and upper end
  uint32_t mode;  // bit0: the window holds 0 or more (lof <= hif, hif >= 0); bit1: census words; bit2: lof <= 0
};
__device__ __forceinline__ QAsk wave_ask(const WaveLds& L, const TableArgs& t, const RowsArgs& a, bool act,
                                         uint32_t s, uint32_t e) {
  QAsk k{0u, 0u, 0u};
  if (!act) return k;
  const double diff = L.su[e] - L.su[s];
  const double thr = a.tol * (L.obs[L.rp[s]] + L.obs[L.rp[e]]);
  double lof, hif;
  quantise_lean(diff, thr, a.prec, a.rprec, lof, hif);
  if (lof <= hif && hif >= 0.0) {
    const double af = lof < 1.0 ? 1.0 : lof;
    k.mode = 1u | (lof <= 0.0 ? 4u : 0u);
    if (af <= hif) {  // census_walk's two loads
      const uint32_t c0 = t.pair_base - 1u, lo = (uint32_t)af - 1u, hi = (uint32_t)hif;
      k.x = t.census[(lo < c0 ? c0 : lo) - c0];
      k.y = t.census[(hi < c0 ? c0 : hi) - c0];
      k.mode |= 2u;
    }
  }
  return k;
}
__device__ __forceinline__ QAns wave_reply(const RowsArgs& a, const QAsk& k) {
  QAns r{SST_NONE, 0, 0, 0};
  if (k.mode & 1u) {
    if (k.mode & 2u) {
      r.first = k.x & 0xFFFFu;
      r.bytes = (k.y >> 16) - (k.x >> 16);
      r.cnt = (k.y & 0xFFFFu) - r.first;
    }
    if (r.cnt > a.cap) r.status = SST_OVERFLOW;
    else if (r.cnt) r.status = SST_SOME;
    else if (k.mode & 4u) r.status = SST_EMPTY;
  }
  return r;
}

__device__ __forceinline__ PairImg global_img(const TableArgs& t) {
  const int n_s = t.n_pairs + 2;
  return PairImg{t.pair_data, t.pair_data + n_s, t.pair_data + 2 * n_s, t.pair_base, t.pair_shift};
}

}  // namespace

// six waves per SIMD (<= 80 VGPRs: same-box A/B 179-180 against 186 us/step at 90 VGPRs and five)
__global__ __launch_bounds__(64 * kWavesPerWG) __attribute__((amdgpu_waves_per_eu(6))) void k_rows_count_w(TableArgs t, RowsArgs a) {
  __shared__ WaveLds Ls[kWavesPerWG];
  WaveLds& L = Ls[threadIdx.x >> 6];
  const int lane = threadIdx.x & 63;
  RPROF_T(w0);
  // this wave's chunk: spectra [w * chunk, (w + 1) * chunk)
  const int64_t w = (int64_t)blockIdx.x * kWavesPerWG + (threadIdx.x >> 6);
  const int64_t g_end = (w + 1) * a.chunk < a.n_spec ? (w + 1) * a.chunk : a.n_spec;
  uint64_t cq = 0, chh = 0, cb = 0;  // the chunk's totals (its big spectra: the workgroup kernel adds theirs)
  for (int64_t g = w * a.chunk; g < g_end; ++g) {
    RPROF_T(c0);
    const int64_t p0 = a.peak_off[g];
    const uint32_t P = (uint32_t)(a.peak_off[g + 1] - p0);
    if (P > (uint32_t)kWP) {  // the block kernels'
      if (lane == 0) a.big[atomicAdd(&a.tickets[2], 1u)] = (uint32_t)g;
      continue;
    }
    RPROF_T(c1);
    RPROF_ADD(0, c1 - c0);
    wave_load(L, t, a, p0, P, a.su_seq[g], true);
    wsync();
    RPROF_T(c2);
    RPROF_ADD(1, c2 - c1);
    uint32_t nq = 0, nh = 0, nb = 0, n0 = 0, n1 = 0;
    bool ok = true;
    for (int sd = 0; sd < 2; ++sd) {
      uint32_t Q;
      RPROF_T(c3);
      const uint32_t n = wave_side(L, a, sd, Q);
      RPROF_T(c4);
      RPROF_ADD(2, c4 - c3);
      if (n == 0xFFFFFFFFu) {
        ok = false;
        break;
      }
      if (sd) n1 = n;
      else n0 = n;
      // every pair is answered here, once (4 B: ans_word): the emit pass reads the answers
      // back in query order instead of re-forming and re-answering the pairs
      // (the side's fixed slots; a side with more queries keeps its rows in
      // scratch and is answered again by the emit pass)
      const uint64_t wb = ans_win_base(p0, P, sd, g);
      const bool fits = Q <= (uint32_t)kRowsAnsPerPeak * P;
      if (lane == 0) a.ans_q[2 * g + sd] = fits ? Q : 0xFFFFFFFFu;
      // a side past its slots: the workgroup emit answers it again (listed once per spectrum)
      if (!fits && lane == 0 && (sd == 0 || a.ans_q[2 * g] != 0xFFFFFFFFu)) a.redo[atomicAdd(&a.tickets[1], 1u)] = (uint32_t)g;
      if (!fits) {
        double* rs = a.rows_su + 4 * p0 + (sd ? 2 * (int64_t)P : 0);
        double* ro = a.rows_ob + 4 * p0 + (sd ? 2 * (int64_t)P : 0);
        for (uint32_t r = lane; r < n; r += 64) {
          rs[r] = L.su[r];
          ro[r] = L.obs[L.rp[r]];
        }
      }
      uint32_t s0 = 0;  // the start of query q0
      uint64_t mka = 0;   // lane w: window w's mask (stored once, after the side)
      uint32_t ne = 0;    // the side's answers other than NONE so far
      for (uint32_t q0 = 0; q0 < Q; q0 += 64) {
        const uint32_t q = q0 + lane;
        uint32_t s, e;
        s0 = wave_pair_window(L, n, q0, s0, s, e);
        QAns r{SST_NONE, 0, 0, 0};
        if (q < Q) r = wave_reply(a, wave_ask(L, t, a, true, s, e));
        nh += (r.status == SST_SOME || r.status == SST_OVERFLOW);
        nb += r.status == SST_SOME ? r.bytes + 2u : 0u;
        const bool kept = r.status != SST_NONE;  // NONE (most pairs) is stored as a clear mask bit only
        const uint64_t m = __ballot(kept);
        if ((uint32_t)lane == q0 / 64) mka = m;
        if (fits && kept) a.ans_ent[wb * 64 + ne + mbcnt64(m)] = ans_word(r);
        ne += (uint32_t)__builtin_popcountll(m);
      }
      if (fits && (uint32_t)lane < (Q + 63) / 64) a.ans_mask[128 * g + 64 * sd + lane] = mka;
      nq += Q;
      wsync();
      RPROF_T(c5);
      RPROF_ADD(3, c5 - c4);
    }
    RPROF_T(c6);
    uint32_t th, tb;
    wave_excl(nh, th);
    wave_excl(nb, tb);
    if (lane == 0) {
      if (!ok) atomicOr(a.err, 2u);
      a.totals[3 * g] = ok ? nq : 0u;
      a.totals[3 * g + 1] = ok ? th : 0u;
      a.totals[3 * g + 2] = ok ? tb : 0u;
      a.side_rows[2 * g] = ok ? n0 : 0u;
      a.side_rows[2 * g + 1] = ok ? n1 : 0u;
    }
    if (ok) {
      cq += nq;
      chh += th;
      cb += tb;
    }
    wsync();
    RPROF_T(c7);
    RPROF_ADD(4, c7 - c6);
    RPROF_ADD(5, 1);
  }
  if (lane == 0 && w < a.n_chunks) {
    a.chunk_tot[3 * w] = cq;
    a.chunk_tot[3 * w + 1] = chh;
    a.chunk_tot[3 * w + 2] = cb;
    unsigned long long* tt = a.tile_tot + a.tile_par * 3 * a.n_tiles + 3 * (w / kRowsTile);
    if (cq) atomicAdd(tt, (unsigned long long)cq);
    if (chh) atomicAdd(tt + 1, (unsigned long long)chh);
    if (cb) atomicAdd(tt + 2, (unsigned long long)cb);
  }
  if (w == 0)  // the next pass's tile sums start from zero
    for (int64_t i = lane; i < 3 * a.n_tiles; i += 64) a.tile_tot[(a.tile_par ^ 1u) * 3 * a.n_tiles + i] = 0;
  RPROF_T(w1);
  RPROF_ADD(8, w1 - w0);
  RPROF_ADD(9, 1);
  if (threadIdx.x == 0 && blockIdx.x == 0) RPROF_ADD(10, gridDim.x);
}

namespace {

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// Chunk w's exclusive offsets (queries, hits, payload bytes): the totals of
// the 64-chunk tiles before its own (tile_tot, summed by the count kernels)
// plus its own tile's earlier chunks -- at most five coalesced loads per lane
// and a wave sum, no launch of its own and no wait on other waves.
__device__ void chunk_prefix(const RowsArgs& a, int64_t w, uint64_t off[3]) {
  const int lane = threadIdx.x & 63;
  const unsigned long long* tt = a.tile_tot + a.tile_par * 3 * a.n_tiles;
  const int64_t t = w / kRowsTile;
  uint64_t v[3] = {0, 0, 0};
  for (int64_t i = lane; i < t; i += 64)
    for (int c = 0; c < 3; ++c) v[c] += tt[3 * i + c];
  const int64_t j = t * kRowsTile + lane;
  if (j < w)
    for (int c = 0; c < 3; ++c) v[c] += a.chunk_tot[3 * j + c];
  for (int c = 0; c < 3; ++c) off[c] = wave_sum64(v[c]);
}

struct EmitLds {
  uint64_t mask[2][64];   // each side's window masks
  uint32_t ebase[2][64];  // the side's answers before each window
  uint32_t ne[2];         // the side's answers other than NONE
  uint16_t qring[128];    // the queries of answers [64 c, 64 c + 128), at answer & 127
};

}  // namespace

__global__ __launch_bounds__(64 * kWavesPerWG) void k_rows_emit_w(TableArgs t, RowsArgs a) {
  // the answers the count pass stored, streamed back in query order (a
  // spectrum with a side past its slots, or over kWP peaks, is the workgroup
  // emit's); 1.5 KB of LDS per wave for the spectrum's window masks, so the
  // waves per CU are set by registers
  __shared__ EmitLds Es[kWavesPerWG];
  EmitLds& E = Es[threadIdx.x >> 6];
  const int lane = threadIdx.x & 63;
  const PairImg img = global_img(t);
  const int64_t w = (int64_t)blockIdx.x * kWavesPerWG + (threadIdx.x >> 6);
  if (w >= a.n_chunks) return;
  const int64_t g_end = (w + 1) * a.chunk < a.n_spec ? (w + 1) * a.chunk : a.n_spec;
  uint64_t off[3];
  chunk_prefix(a, w, off);
  const uint64_t ct[3] = {a.chunk_tot[3 * w], a.chunk_tot[3 * w + 1], a.chunk_tot[3 * w + 2]};
  if (lane == 0) {  // this chunk's offsets (the workgroup emit's big spectra); the last chunk's end: the pass totals
    for (int c = 0; c < 3; ++c) a.chunk_off[3 * w + c] = off[c];
    if (w == a.n_chunks - 1) {
      a.ctl[0] = off[0] + ct[0];
      a.ctl[1] = off[1] + ct[1];
      a.ctl[2] = off[2] + ct[2];
    }
  }
  // past the result's capacity: nothing written (the header reports it)
  const bool room = off[0] + ct[0] <= a.cap_queries && off[1] + ct[1] <= a.cap_queries && off[2] + ct[2] <= a.cap_bytes;
  if (!room) {
    if (lane == 0) atomicOr(a.err, 4u);
    return;
  }
  for (int64_t g = w * a.chunk; g < g_end; ++g) {
    const int64_t p0 = a.peak_off[g];
    const uint32_t P = (uint32_t)(a.peak_off[g + 1] - p0);
    const uint32_t Q0 = a.ans_q[2 * g], Q1 = a.ans_q[2 * g + 1];
    uint64_t qb = off[0], hb = off[1], bb = off[2];
    // the next spectrum's offsets (this one's totals: the count kernels')
    off[0] += a.totals[3 * g];
    off[1] += a.totals[3 * g + 1];
    off[2] += a.totals[3 * g + 2];
    if (P > (uint32_t)kWP || Q0 == 0xFFFFFFFFu || Q1 == 0xFFFFFFFFu) continue;  // the workgroup kernel's
    // both sides' window masks and each window's first answer (the answers
    // before it: a wave prefix of the masks' popcounts) to LDS, and each
    // side's first 64 answer words, in one round trip
    {
      const uint64_t m0 = (uint32_t)lane < (Q0 + 63) / 64 ? __builtin_nontemporal_load(&a.ans_mask[128 * g + lane]) : 0ull;
      const uint64_t m1 = (uint32_t)lane < (Q1 + 63) / 64 ? __builtin_nontemporal_load(&a.ans_mask[128 * g + 64 + lane]) : 0ull;
      uint32_t n0, n1;
      const uint32_t e0 = wave_excl((uint32_t)__builtin_popcountll(m0), n0);
      const uint32_t e1 = wave_excl((uint32_t)__builtin_popcountll(m1), n1);
      E.mask[0][lane] = m0;
      E.mask[1][lane] = m1;
      E.ebase[0][lane] = e0;
      E.ebase[1][lane] = e1;
      if (lane == 0) {
        E.ne[0] = n0;
        E.ne[1] = n1;
      }
      wsync();
    }
    const uint32_t* ent0 = a.ans_ent + ans_win_base(p0, P, 0, g) * 64;
    const uint32_t* ent1 = a.ans_ent + ans_win_base(p0, P, 1, g) * 64;
    uint32_t cur = Q0 ? __builtin_nontemporal_load(&ent0[lane]) : 0u;
    const uint32_t pre1 = Q1 ? __builtin_nontemporal_load(&ent1[lane]) : 0u;
    for (int sd = 0; sd < 2; ++sd) {
      const uint32_t Q = sd ? Q1 : Q0;
      const uint32_t nwin = (Q + 63) / 64;
      const uint32_t* ent = sd ? ent1 : ent0;
      const uint32_t ne = E.ne[sd];
      if (sd) cur = pre1;
      // The side's answers other than NONE stream through two 64-word
      // registers (answers [64 c, 64 c + 128)), the next block loaded as
      // the stream enters the last.  A pass over the windows writes every
      // status byte (an answer reaches its query's lane by ds_bpermute) and
      // each answer's query to an LDS ring; each block of 64 answers, once
      // the windows have passed it, is emitted in one go: one lane per
      // answer, its first records loaded together, one pair of wave prefix
      // sums per 64 answers (hit records, refs and payload in query order).
      uint32_t c = 0;
      uint32_t nxt = 64u < ne ? __builtin_nontemporal_load(&ent[64 + lane]) : 0u;
      auto emit_block = [&](uint32_t words, uint32_t k) {
        const uint32_t e = 64u * k + lane;
        wsync();  // the ring's query indices
        const QAns r = e < ne ? ans_read(words, a.cap) : QAns{SST_NONE, 0, 0, 0};
        const uint32_t q = E.qring[e & 127u];
        const bool some = r.status == SST_SOME;
        uint32_t rec[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int x = 0; x < 4; ++x)
          if (some && (uint32_t)x < r.cnt) rec[x] = img.recs[r.first + x];
        uint32_t nb = 0;
        if (some) {
#pragma unroll
          for (int x = 0; x < 4; ++x) nb += (uint32_t)x < r.cnt ? (rec[x] & 0xFFu) + 1u : 0u;
          if (r.cnt > 4) nb += ans_bytes(img.recs, r.first + 4, r.cnt - 4);
        }
        uint32_t th, tb;
        const bool hit = some || r.status == SST_OVERFLOW;
        const uint32_t xh = wave_excl(hit ? 1u : 0u, th);
        const uint32_t xb = wave_excl(some ? nb + 2u : 0u, tb);
        if (hit) {
          const uint64_t o = bb + xb;
          const uint64_t word = some ? o : (uint64_t)r.cnt;
          a.hits[hb + xh] = make_uint4((uint32_t)(qb + q), r.cnt, (uint32_t)word, (uint32_t)(word >> 32));
          a.refs[hb + xh] = (uint16_t)(r.first | (r.status == SST_OVERFLOW ? 0x8000u : 0u));
          if (some) {
            // the 2 pad bytes after the query's last record take the overhang
            uint8_t* dst = a.dense + o;
#pragma unroll
            for (int x = 0; x < 4; ++x)
              if ((uint32_t)x < r.cnt) {
                *(u32_unal*)dst = rec[x];
                dst += (rec[x] & 0xFFu) + 1u;
              }
            const uint32_t kend = r.first + r.cnt;
            for (uint32_t k0 = r.first + 4; k0 < kend; k0 += 4) {  // more than four records
              uint32_t rr[4];
#pragma unroll
              for (int x = 0; x < 4; ++x) rr[x] = k0 + x < kend ? img.recs[k0 + x] : 0u;
#pragma unroll
              for (int x = 0; x < 4; ++x)
                if (k0 + x < kend) {
                  *(u32_unal*)dst = rr[x];
                  dst += (rr[x] & 0xFFu) + 1u;
                }
            }
          }
        }
        hb += th;
        bb += tb;
        wsync();  // the ring's slots are rewritten
      };
      for (uint32_t wi = 0; wi < nwin; ++wi) {
        const uint64_t m = E.mask[sd][wi];
        const uint32_t base = E.ebase[sd][wi];
        if (base >= 64u * (c + 1)) {  // block c is complete: emit it, the stream enters the next
          emit_block(cur, c);
          ++c;
          cur = nxt;
          nxt = 64u * (c + 1) < ne ? __builtin_nontemporal_load(&ent[64u * (c + 1) + lane]) : 0u;
        }
        const uint32_t q = 64u * wi + lane;
        const uint32_t e = base + mbcnt64(m);
        const uint32_t v0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((e & 63u) << 2), (int)cur);
        const uint32_t v1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((e & 63u) << 2), (int)nxt);
        const bool has = (m >> lane) & 1ull;
        const uint32_t v = has ? ((e >> 6) > c ? v1 : v0) : 0u;
        if (q < Q) a.status[qb + q] = ans_read(v, a.cap).status;
        if (has) E.qring[e & 127u] = (uint16_t)q;
      }
      if (ne > 64u * c) {  // the last blocks
        emit_block(cur, c);
        if (ne > 64u * (c + 1)) emit_block(nxt, c + 1);
      }
      qb += Q;
    }
  }
}

size_t rows_lds_bytes() { return sizeof(SpecLds); }

hipError_t launch_rows_step(const TableArgs& t, const RowsArgs& a, int n_wg, size_t dyn, hipStream_t st) {
  if (a.n_spec <= 0 || !t.pairs_enabled) return hipErrorInvalidValue;
#ifndef SST_ROWS_IMG_LDS
  const size_t wdyn = 0;
#else
  const size_t wdyn = dyn;
#endif
  // 4-wave workgroups, as many as are resident (each wave a contiguous chunk of spectra)
  // (the occupancy of the two wave kernels: with no dynamic LDS a per-process
  // constant, computed once -- contexts on other threads see the finished
  // value, never a torn one; the pair-image variant asks every time)
  auto occupancy = [](size_t d, int* out) {
    int c1 = 0, c2 = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&c1, k_rows_count_w, 64 * kWavesPerWG, 0) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&c2, k_rows_emit_w, 64 * kWavesPerWG, d) != hipSuccess)
      return hipErrorLaunchFailure;
    *out = c1 < c2 ? c1 : c2;
    return hipSuccess;
  };
  static std::once_flag occ_once;
  static int occ0 = 0;
  static hipError_t occ0_err = hipSuccess;
  int occ = 0;
  if (wdyn == 0) {
    std::call_once(occ_once, [&] { occ0_err = occupancy(0, &occ0); });
    if (occ0_err != hipSuccess) return occ0_err;
    occ = occ0;
  } else if (hipError_t e = occupancy(wdyn, &occ); e != hipSuccess) {
    return e;
  }
  const int wave_wg = n_wg * (occ > 0 ? occ : 1);
  // one spectrum per wave where the chunk arrays allow (the dispatcher then
  // balances the waves: a resident-only grid of contiguous chunks left the
  // kernel waiting for its 3-spectrum waves), contiguous chunks beyond
  RowsArgs b = a;
  b.n_chunks = a.n_spec < a.chunk_cap ? a.n_spec : a.chunk_cap;
  b.chunk = (a.n_spec + b.n_chunks - 1) / b.n_chunks;
  b.n_chunks = (a.n_spec + b.chunk - 1) / b.chunk;
  if (b.n_chunks > a.chunk_cap || b.n_chunks > a.n_tiles * kRowsTile) return hipErrorInvalidValue;
  const int wgrid = (int)((b.n_chunks + kWavesPerWG - 1) / kWavesPerWG);
  (void)wave_wg;
  hipLaunchKernelGGL(k_rows_count_w, dim3(wgrid), dim3(64 * kWavesPerWG), 0, st, t, b);
  // the workgroup kernels take the few spectra over kWP peaks (none in most
  // batches: a small grid keeps their launches cheap when idle)
  const int big_wg = n_wg < 64 ? n_wg : 64;
  hipLaunchKernelGGL(k_rows_count, dim3(big_wg), dim3(kRowsWG), dyn, st, t, b);
  hipLaunchKernelGGL(k_rows_emit_w, dim3(wgrid), dim3(64 * kWavesPerWG), wdyn, st, t, b);
  hipLaunchKernelGGL(k_rows_emit, dim3(big_wg), dim3(kRowsWG), dyn, st, t, b);  // last: writes the header
  return hipGetLastError();
}

}  // namespace sst
