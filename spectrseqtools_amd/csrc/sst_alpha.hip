// sst_alpha.hip -- queries on per-spectrum reduced alphabets (gfx950).
//
// Predictor.filter_by_explanation (prediction.py:170-227) reduces each
// spectrum's alphabet to the modifications its explanations name
// (adapt_individual_modification_rates_by_alphabet_reduction,
// mass_table.py:94-121) and rebuilds the DP table for it; over a batch of
// spectra nearly every spectrum ends with its own alphabet, so a table per
// spectrum is not an option.  Two kernels answer the reduced tables' queries
// without building them:
//
//   k_pairs_alpha   explain_mass_with_table on pair-class windows (every
//                   candidate has <= 2 items: hi < 3 w_min): the candidates on
//                   the reduced table are exactly the full table's pair-list
//                   entries whose rows all lie in the spectrum's alphabet (the
//                   reduced table is the closure of those rows; budgets that
//                   cannot bind are the caller's check), in the same order.
//                   One lane per query; the 40 KB pair list is read through L2.
//   k_valid_alpha   is_valid_mass on the reduced table: reachability by the
//                   spectrum's rows (an unbounded knapsack: the reduced table's
//                   last row), computed as a bitset closure in LDS, one
//                   workgroup per spectrum.  Every row mass is >= w_min (C, a
//                   canonical row, is never dropped), so bit m depends only on
//                   bits m - w_r <= m - w_min: chunks of 8064 words (258048
//                   masses < w_min) are filled in order, each word an OR of
//                   shifted words of the ones before it (w_max < 3 * 2^18), in
//                   a 128 KB ring of 2^15 words.  The spectrum's windows (in mass order)
//                   are answered as soon as the chunk holding them is done; a
//                   run of >= w_min reachable masses (the alphabet's lightest
//                   row) ends the closure: every later mass m is reachable, as
//                   m - w_min is.  The reduced table's extent and
//                   its last-column mask (mass_table.py:212, :246) bound the
//                   reachable masses exactly as in set_up_bit_table.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sst_internal.h"
#include "sst_quant.h"

namespace sst {

namespace {

// A wave fills kParts runs of 63 consecutive words per chunk (lane 63 only
// supplies its neighbour's word), one wave-segment of 504 words: a row's
// scalar work (its mass, ring offset and shift) serves the wave's whole
// segment, and a chunk is one segment per wave.
constexpr int kValidWG = 1024;
constexpr int kValidWaves = kValidWG / 64;
constexpr int kParts = 8;
constexpr int kSegWords = 63 * kParts;                  // 504
constexpr int kChunkWords = kSegWords * kValidWaves;    // 8064 words per chunk
constexpr int64_t kChunkBits = kChunkWords * 32;        // 258048 masses (< w_min)
constexpr int kRingWords = 32768;                       // a chunk + the w_max / 32 words before it
constexpr int kRingMask = kRingWords - 1;
constexpr int kRingPad = 512;                           // the ring's first words again: reads past the end
static_assert(kChunkWords + 3 * 262144 / 32 + 2 <= kRingWords, "ring too small");
static_assert(kSegWords + 1 <= kRingPad, "ring pad too small");

__device__ __forceinline__ bool row_in(uint64_t m0, uint64_t m1, int r) {
  return r < 64 ? ((m0 >> r) & 1ull) : ((m1 >> (r - 64)) & 1ull);
}

__device__ __forceinline__ uint64_t ring_word(const uint32_t* ring, int64_t wi) {
  return wi < 0 ? 0ull : (uint64_t)ring[wi & kRingMask];
}

// 64 closure bits starting at mass x (x may be negative: zeros) from the ring
__device__ __forceinline__ uint64_t ring_bits(const uint32_t* ring, int64_t x) {
  if (x < -63) return 0ull;
  const int64_t wi = x >> 5;  // floor
  const int s = (int)(x & 31);
  const uint64_t lo = ring_word(ring, wi) | ring_word(ring, wi + 1) << 32;
  if (s == 0) return lo;
  return (lo >> s) | (ring_word(ring, wi + 2) << (64 - s));
}

// any closure bit in [a, b] (both inside the ring's chunks)
__device__ __forceinline__ bool ring_any(const uint32_t* ring, int64_t a, int64_t b) {
  for (int64_t x = a; x <= b; x += 64) {
    uint64_t v = ring_bits(ring, x);
    const int64_t left = b - x + 1;
    if (left < 64) v &= (1ull << left) - 1ull;
    if (v) return true;
  }
  return false;
}

}  // namespace

__device__ __forceinline__ void alpha_window(const AlphaArgs& a, int64_t i, int64_t& lo, int64_t& hi) {
  const double t = a.thr_obs ? a.tol * a.thr_obs[i] : a.thr ? a.thr[i] : 0.0;
  quantise(a.mass[i], t, a.thr == nullptr && a.thr_obs == nullptr, a.tol, a.prec, a.rprec, lo, hi);
}
__device__ __forceinline__ void alpha_put(const AlphaArgs& a, int64_t i, int8_t res) {
  if (!a.alive) {
    a.out[i] = res;
  } else if (a.alive[i]) {
    if (res != 1) a.alive[i] = 0;
    if (res == -1 || res == (int8_t)kStatusPending) atomicOr(a.err, res == -1 ? 8u : 32u);
  }
}

__global__ __launch_bounds__(kValidWG) void k_valid_alpha(AlphaArgs a) {
  __shared__ uint32_t ring[kRingWords + kRingPad];  // word i of the closure at i & kRingMask
  __shared__ int s_w[kMaxRows];
  __shared__ int s_n;
  __shared__ int64_t s_done;   // queries [q0, s_done) answered
  __shared__ int s_full;       // a run of >= w_min reachable masses seen: every later mass is reachable
  __shared__ int s_zmax;       // the chunk's highest unreachable mass (chunk-relative), -1: none
  __shared__ int64_t s_run;    // reachable masses ending at the last chunk's end
  __shared__ int s_wmin_all;
  const int64_t g = blockIdx.x;
  if (a.active && !a.active[g]) return;
  const int64_t q0 = a.counts ? 4 * a.offsets[g] : a.offsets[g];
  const int64_t q1 = a.counts ? q0 + a.counts[g] : a.offsets[g + 1];
  if (q0 >= q1) return;
  const uint64_t m0 = a.masks[2 * g], m1 = a.masks[2 * g + 1];
  // with every canonical row kept the closure starts from theirs (shared, in
  // L2) and only the other rows are added per spectrum
  __shared__ int s_wmax_all, s_use_c;
  if (threadIdx.x == 0) {
    int n = 0, wmax_all = 0, wmin_all = INT32_MAX;
    for (int r = 1; r < a.n_rows; ++r)
      if (row_in(m0, m1, r)) {
        wmax_all = a.w[r] > wmax_all ? a.w[r] : wmax_all;
        wmin_all = a.w[r] < wmin_all ? a.w[r] : wmin_all;
      }
    // the reduced table ends below ceil((35 w_max + 1) / 32) * 32: the shared
    // closure must cover it
    const int64_t lim = ((int64_t)wmax_all * 35 + 32) / 32 * 32;
    const int uc = a.canon_closure && (m0 & a.canon0) == a.canon0 && (m1 & a.canon1) == a.canon1 &&
                   lim <= 32 * a.canon_words;
    for (int r = 1; r < a.n_rows; ++r)
      if (row_in(m0, m1, r) && !(uc && row_in(a.canon0, a.canon1, r))) s_w[n++] = a.w[r];
    s_n = n;
    s_wmax_all = wmax_all;
    s_use_c = uc;
    s_done = q0;
    s_full = 0;
    s_zmax = -1;
    s_run = 0;
    s_wmin_all = wmin_all;
  }
  __syncthreads();
  const bool use_c = s_use_c;
  const int n_w = s_n;
  if (n_w == 0 && !use_c) {  // sentinel only: nothing >= 1 is reachable
    for (int64_t i = q0 + threadIdx.x; i < q1; i += blockDim.x) alpha_put(a, i, 0);
    return;
  }
  // words below mass 0 read as empty: zero the ring (slots are reused across spectra)
  for (int i = threadIdx.x; i < kRingWords + kRingPad; i += blockDim.x) ring[i] = 0u;
  // the row masses, lane r of every wave holding rows r and r + 64
  const int w_lo = (int)(threadIdx.x & 63) < n_w ? s_w[threadIdx.x & 63] : 0;
  const int w_hi = (int)(threadIdx.x & 63) + 64 < n_w ? s_w[(threadIdx.x & 63) + 64] : 0;
  int wmax = 0, wmin = INT32_MAX;  // of the rows added per spectrum (the ring's dependency window)
  for (int k = 0; k < n_w; ++k) {
    wmax = s_w[k] > wmax ? s_w[k] : wmax;
    wmin = s_w[k] < wmin ? s_w[k] : wmin;
  }
  if (n_w == 0) wmin = wmax = (int)kChunkBits + 1;  // the canonical closure alone
  // the reduced table (set_up_bit_table with max_mass = max(kept) * 35):
  // masses < limit exist, the last-column mask leaves masses <= vtop reachable
  const int64_t max_mass = (int64_t)s_wmax_all * 35;
  const int64_t n_cols = (max_mass + 1 + 31) / 32;
  const int64_t limit = n_cols * 32;
  const int64_t vtop = ((max_mass + 1) % 32 == 0) ? (n_cols - 1) * 32 - 1 : max_mass;
  // the highest window value any query of this spectrum looks at
  int64_t top = 0;
  for (int64_t i = q0 + threadIdx.x; i < q1; i += blockDim.x) {
    int64_t lo, hi;
    alpha_window(a, i, lo, hi);
    top = hi > top ? hi : top;
  }
  __shared__ int64_t s_top;
  if (threadIdx.x == 0) s_top = 0;
  __syncthreads();
  atomicMax((unsigned long long*)&s_top, (unsigned long long)(top < 0 ? 0 : top));
  __syncthreads();
  top = s_top < limit - 1 ? s_top : limit - 1;
  const int64_t n_chunks = top / kChunkBits + 1;
  // a chunk's words depend only on words before it (every row is heavier than
  // a chunk), and on none more than 3 * 2^18 masses back (the ring holds them)
  const bool guard_ok = wmin > kChunkBits && wmax < 3 * 262144;
  // A row's shifted word for output word o needs ring words wi and wi + 1,
  // and wi + 1 is the next lane's wi (a DPP lane shift): each of the wave's
  // kParts runs reads 64 words and writes 63.  The shift is wave-uniform.
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int seg0 = wv * kSegWords;  // the wave's first word in a chunk
  // the canonical closure's words of a chunk, per lane and part, loaded a
  // chunk ahead: one L2 latency per chunk, hidden behind the chunk before
  uint32_t cwv[kParts];
  auto load_canon = [&](int64_t jj, uint32_t* dst) {
#pragma unroll
    for (int k = 0; k < kParts; ++k) {
      const int64_t cw = jj * kChunkWords + seg0 + 63 * k + lane;
      dst[k] = use_c && lane < 63 && cw < a.canon_words ? a.canon_closure[cw] : 0u;
    }
  };
  load_canon(0, cwv);
  for (int64_t j = 0; j < n_chunks && guard_ok; ++j) {
    const int64_t cs = j * kChunkWords;  // the chunk's first word
    const int64_t base = cs * 32;
    int zmax = -1;  // this lane's highest unreachable mass in the chunk
    uint32_t nxt[kParts];
    if (j + 1 < n_chunks && !s_full) {
      load_canon(j + 1, nxt);
    } else {
#pragma unroll
      for (int k = 0; k < kParts; ++k) nxt[k] = 0u;
    }
    uint32_t v[kParts];
    if (!s_full) {
#pragma unroll
      for (int k = 0; k < kParts; ++k) v[k] = cwv[k];  // includes mass 0 (use_c); past the full table: none
      if (!use_c && j == 0 && wv == 0 && lane == 0) v[0] = 1u;  // mass 0: the empty multiset (table[0, 0] seed)
      // the wave's first output mass (masses < limit < 2^31), wave-uniform:
      // the shifts and ring offsets below are scalar arithmetic
      const int mw = __builtin_amdgcn_readfirstlane((int)(32 * (cs + seg0)));
      // rows [r0, r1), lane r - r0 holding row r's mass (read by readlane: no
      // LDS round trip); two rows per step, their LDS reads in flight together
      // (a tail repeats the last row: the same bits again)
      auto add_rows = [&](int wsrc, int r0, int r1) {
        for (int r = r0; r < r1; r += 2) {
          int x[2];
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) {
            const int rk = r + kk < r1 ? r + kk : r1 - 1;
            x[kk] = mw - __builtin_amdgcn_readlane(wsrc, rk - r0);
          }
          // ring words from the wave's first shifted word (negative masses: the
          // zeroed slots not yet filled; past the end: the pad copy of the start)
          uint32_t lo[2][kParts];
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) {
            const uint32_t* src = ring + ((x[kk] >> 5) & kRingMask) + lane;
#pragma unroll
            for (int k = 0; k < kParts; ++k) lo[kk][k] = src[63 * k];
          }
#pragma unroll
          for (int k = 0; k < kParts; ++k) {
            uint32_t t[2];
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
              // the next lane's word (wave_shl:1; lane 63's result is unused)
              const uint32_t nx = (uint32_t)__builtin_amdgcn_mov_dpp((int)lo[kk][k], 0x130, 0xF, 0xF, true);
              t[kk] = __builtin_amdgcn_alignbit(nx, lo[kk][k], (uint32_t)x[kk] & 31u);  // ({nx, lo} >> shift) low word
            }
            v[k] |= t[0] | t[1];
          }
        }
      };
      add_rows(w_lo, 0, n_w < 64 ? n_w : 64);
      if (n_w > 64) add_rows(w_hi, 64, n_w);
    } else {
#pragma unroll
      for (int k = 0; k < kParts; ++k) v[k] = ~0u;
    }
    if (lane < 63) {
#pragma unroll
      for (int k = 0; k < kParts; ++k) {
        const int o = seg0 + 63 * k + lane;  // chunk-relative; o ascends with k
        const int ri = (int)((cs + o) & kRingMask);
        ring[ri] = v[k];
        if (ri < kRingPad) ring[ri + kRingWords] = v[k];
        if (v[k] != ~0u) zmax = 32 * o + 31 - __builtin_clz(~v[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < kParts; ++k) cwv[k] = nxt[k];
    for (int off = 32; off > 0; off >>= 1) {  // the wave's highest, then one atomic per wave
      const int z2 = __shfl_xor(zmax, off, 64);
      zmax = zmax > z2 ? zmax : z2;
    }
    if (lane == 0 && zmax >= 0) atomicMax(&s_zmax, zmax);
    __syncthreads();
    if (threadIdx.x == 0) {
      // a run of >= w_min reachable masses [x, x + w_min): every m beyond is
      // reachable (m - w_min is, by induction), so the closure is full from here
      const int zm = s_zmax;
      s_zmax = -1;
      s_run = zm < 0 ? s_run + kChunkBits : kChunkBits - 1 - zm;
      if (s_run >= s_wmin_all) s_full = 1;
    }
    __syncthreads();
    // answer the queries whose windows lie below the end of this chunk (the
    // rows come sorted by mass, windows are narrow: a query whose hi is in a
    // later chunk stops the sweep and is answered there)
    const int64_t end = base + kChunkBits;
    const bool last = j == n_chunks - 1;
    for (int64_t i0 = s_done; i0 < q1; i0 += blockDim.x) {
      const int64_t i = i0 + threadIdx.x;
      bool ready = false;
      int8_t res = 0;
      if (i < q1) {
        int64_t lo, hi;
        alpha_window(a, i, lo, hi);
        ready = last || hi < end;
        if (ready) {
          // is_valid_mass (mass_explanation.py:63-88): skip v <= 0, raise at
          // the first v >= limit, True at the first reachable v
          const int64_t x0 = lo < 1 ? 1 : lo;
          const int64_t x1 = hi < vtop ? hi : vtop;
          bool any = false;
          if (x0 <= x1 && (x0 >> 5) < cs + kChunkWords - kRingWords) {
            res = (int8_t)kStatusPending;  // below the ring (rows not in mass order): reported, not guessed
          } else {
            if (x0 <= x1) any = ring_any(ring, x0, x1);
            res = any ? (int8_t)1 : (hi >= limit && hi >= lo && hi >= 1) ? (int8_t)-1 : (int8_t)0;
          }
          alpha_put(a, i, res);
        }
      }
      // the sweep advances over the leading run of answered queries
      const uint64_t not_ready = __ballot(i < q1 && !ready);
      __shared__ int s_stop[kValidWG / 64];
      if ((threadIdx.x & 63) == 0) s_stop[threadIdx.x >> 6] = not_ready ? __builtin_ctzll(not_ready) : 64;
      __syncthreads();
      int stop = -1;
      for (int wv = 0; wv < (int)(blockDim.x >> 6); ++wv)
        if (s_stop[wv] < 64) {
          stop = wv * 64 + s_stop[wv];
          break;
        }
      __syncthreads();
      if (stop >= 0) {
        if (threadIdx.x == 0) s_done = i0 + stop;
        __syncthreads();
        break;
      }
      if (threadIdx.x == 0) s_done = i0 + (int64_t)blockDim.x < q1 ? i0 + blockDim.x : q1;
      __syncthreads();
    }
    __syncthreads();
    if (s_done >= q1) break;
  }
  if (!guard_ok)  // alphabets the ring cannot hold (not produced by the reduction): reported, not guessed
    for (int64_t i = q0 + threadIdx.x; i < q1; i += blockDim.x) alpha_put(a, i, (int8_t)kStatusPending);
}

// Pair-class windows on a per-spectrum alphabet (see the file comment).  Out:
// status, the number of candidates, the union of their rows and the window's
// pair-list range [first, end) (the candidates are the entries of that range
// whose rows are all in the alphabet).  Windows that are not pair-class
// (hi >= pair_hi) get kStatusPending: the caller answers them otherwise.
__global__ __launch_bounds__(256) void k_pairs_alpha(TableArgs t, PairAlphaArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  int64_t lo, hi;
  quantise(a.mass[i], a.thr ? a.thr[i] : 0.0, a.thr == nullptr, a.tol, a.prec, a.rprec, lo, hi);
  const int32_t g = a.spec[i];
  const uint64_t m0 = a.masks[2 * (int64_t)g], m1 = a.masks[2 * (int64_t)g + 1];
  int8_t status = SST_NONE;
  uint32_t cnt = 0, first = 0, end = 0;
  uint64_t u0 = 0, u1 = 0;
  if (hi >= t.pair_hi) {
    status = (int8_t)kStatusPending;
  } else if (lo <= hi && hi >= 0) {
    const bool zero = lo <= 0;  // v == 0: the empty solution [[]]
    const int64_t x0 = lo < 1 ? 1 : lo;
    if (x0 <= hi) {
      const uint32_t* sums = t.pair_data;
      const uint32_t* recs = sums + (t.n_pairs + 2);
      const uint32_t* bk = recs + (t.n_pairs + 2);
      const uint32_t av = (uint32_t)x0, hv = (uint32_t)hi;
      const uint32_t rel = av > t.pair_base ? av - t.pair_base : 0u;
      uint32_t k = bk[rel >> t.pair_shift] & 0xFFFFu;
      const uint32_t a2 = av << 1, h2 = (hv << 1) | 1u;
      while (sums[k] < a2) ++k;
      first = k;
      for (; sums[k] <= h2; ++k) {
        const uint32_t rec = recs[k];
        const int top = (int)((rec >> ((rec & 0xFFu) == 1u ? 8 : 16)) & 0xFFu);
        const int low = (int)((rec >> 8) & 0xFFu);
        if (row_in(m0, m1, top) && row_in(m0, m1, low)) {
          ++cnt;
          if (top < 64) u0 |= 1ull << top; else u1 |= 1ull << (top - 64);
          if (low < 64) u0 |= 1ull << low; else u1 |= 1ull << (low - 64);
        }
      }
      end = k;
    }
    status = cnt ? (int8_t)SST_SOME : zero ? (int8_t)SST_EMPTY : (int8_t)SST_NONE;
  }
  a.status[i] = status;
  a.count[i] = cnt;
  a.rowmask[2 * i] = u0;
  a.rowmask[2 * i + 1] = u1;
  a.range[2 * i] = first;
  a.range[2 * i + 1] = end;
}

hipError_t launch_valid_alpha(const AlphaArgs& a, int64_t n_spec, hipStream_t st) {
  if (n_spec <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_valid_alpha, dim3((uint32_t)n_spec), dim3(kValidWG), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_pairs_alpha(const TableArgs& t, const PairAlphaArgs& a, hipStream_t st) {
  if (a.n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pairs_alpha, dim3((uint32_t)((a.n + 255) / 256)), dim3(256), 0, st, t, a);
  return hipGetLastError();
}

}  // namespace sst
