// sst_skel.hip -- SkeletonBuilder._predict_skeleton's walk over many spectra
// on the device, gfx950.
//
//   k_skel_walk   one lane per (spectrum, side): the reference's sequential
//                 loop (skeleton_building.py:114-196) over the side's rows the
//                 fixpoint kept: bins of rows whose SU step is within the pair
//                 threshold, each closed bin explained against the last bin
//                 that had explanations (explain_bin_differences :372-421, the
//                 first against mass 0), every difference looked up in
//                 filter_by_explanation's final dict first
//                 (explain_mass_difference :423-440: a hit answers the same
//                 window at the dict entry's threshold); bins without
//                 explanations reject their rows, the others update the
//                 skeleton (update_skeleton_for_given_explanations :442-482)
//                 and their rows' min_end / max_end.
//
// Answers: a pair-class window whose budgets cannot bind is answered here
// from the full table's pair list under the spectrum's row mask (the reduced
// table's candidates), in the reference's order.  Every other
// window needs the DFS (the masked explain, sst_explain_alpha_batch_device):
// the speculative bin queries (each bin against the bin before it, stage 3)
// were answered before the walk and arrive as candidate references; a bin
// that must be explained against an older bin (its predecessor had none) is
// a re-query -- when it holds such windows the lane lists them, marks its
// side suspended and stops; the host answers the list and relaunches the
// suspended sides, which replay from the start and consume the answers in
// the order they meet them (the walk is deterministic).
//
// Order: explanation lists are Python set iterations (common.py:60-65 over
// mass_explanation.py:287-320's set of name tuples) and the positions a set
// of ints, so the lane emulates CPython's set (sst_pyset.h) from the names'
// hashes (host: hash(name) of the running interpreter) -- the same order the
// reference produces under the same hash seed.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sst_internal.h"
#include "sst_pyset.h"
#include "sst_quant.h"

namespace sst {

namespace {

constexpr uint64_t kRefPtr = 1ull << 63;
constexpr uint64_t kRefLow = (1ull << 56) - 1;

__device__ __forceinline__ uint64_t ref_pair(uint32_t k, int len) { return ((uint64_t)len << 56) | k; }
__device__ __forceinline__ uint64_t ref_ptr(const uint8_t* p, int len) {
  return kRefPtr | ((uint64_t)len << 56) | ((uint64_t)p & kRefLow);
}
__device__ __forceinline__ int ref_len(uint64_t r) { return (int)((r >> 56) & 0x7F); }
// row j of a candidate: a pair-list record ([k][row_0][row_1] in a u32) or a
// payload record ([k][row_0]...[row_{k-1}] bytes); rows ascending
__device__ __forceinline__ int ref_row(const TableArgs& t, uint64_t r, int j) {
  if (r & kRefPtr) return ((const uint8_t*)(r & kRefLow))[1 + j];
  const uint32_t* recs = t.pair_data + (t.n_pairs + 2);
  return (int)((recs[(uint32_t)(r & kRefLow)] >> (8 + 8 * j)) & 0xFFu);
}

struct Lane {
  pyset::Table pos[2];   // the current and the next position set
  int cur;
  uint8_t* lkeys;        // update: explanation lengths in first-run order
  uint8_t* lseen;        // [len_cap]
  uint64_t* lval;        // [2 len_cap] the last run's names per length
  uint64_t* ex;          // [expl_cap][4]: tuple hash, mask lo, mask hi, ref
  uint32_t n_ex;
  uint64_t* cref;        // [cand_cap] the current query's candidates
  int64_t* chash;
  pyset::Table ts;       // their name-tuple set
  uint64_t* xi;          // [xmask + 1] the bin's list by tuple hash: xepoch << 32 | (index + 1)
  uint32_t xmask;
  uint32_t xepoch;       // one per bin: slots of other epochs are empty
};

// A suspended side's loop state, at the head of its scratch: a relaunch
// resumes at the bin that listed the re-queries instead of replaying.
struct WalkState {
  uint32_t tag;  // side id + 1: valid
  uint32_t f, n, spec_ctr, consumed, xepoch;
  int32_t lv0, lv1, pb0, pb1, cur0, cur;
  uint32_t pmask, pfill;
  int32_t pcur;
  uint32_t povf;
};
static_assert(sizeof(WalkState) <= 64, "walk state");
constexpr uint64_t kWalkStateBytes = 64;
__host__ __device__ inline uint32_t walk_index_slots(uint32_t expl_cap) {
  uint32_t x = 16;
  while (x < 2 * expl_cap) x <<= 1;
  return x;
}
__device__ __forceinline__ uint32_t xi_slot(int64_t h, uint32_t mask) {
  const uint64_t u = (uint64_t)h;
  return (uint32_t)(u ^ (u >> 29) ^ (u >> 47)) & mask;
}

__device__ __forceinline__ double key_of(double k) { return k == 0.0 ? 0.0 : k; }

// filter_by_explanation's final dict: the threshold the entry for `diff` was
// answered with (true), or false when diff is not a key
__device__ __forceinline__ bool dict_thr(const WalkArgs& a, int64_t g, double diff, double& thr) {
  const uint64_t key = (uint64_t)__double_as_longlong(key_of(diff));
  uint64_t lo = a.d_off[g], hi = lo + a.d_n[g];
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (a.d_key[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  if (lo < a.d_off[g] + a.d_n[g] && a.d_key[lo] == key) {
    thr = a.d_thr[lo];
    return true;
  }
  return false;
}

enum { kAnsOk = 0, kAnsBig = 1 };

// a candidate's tuple hash (hash of its name tuple, names in row order) and
// row mask
__device__ __forceinline__ void cand_props(const TableArgs& t, const WalkArgs& a, uint64_t ref, int64_t& h,
                                           uint64_t& m0, uint64_t& m1) {
  const int k = ref_len(ref);
  uint64_t acc = pyset::tuple_hash_init();
  m0 = m1 = 0;
  for (int j = 0; j < k; ++j) {
    const int r = ref_row(t, ref, j);
    acc = (uint64_t)pyset::tuple_hash_step(acc, a.name_hash[r]);
    if (r < 64) m0 |= 1ull << r;
    else m1 |= 1ull << (r - 64);
  }
  h = pyset::tuple_hash_final(acc, k);
}

// the pair-class window [lof, hif] on the mask: its candidates (the pair
// list's entries of the window whose rows are kept, sorted (sum, top row) =
// the reference's order) into the lane's list; returns the status
__device__ int8_t pair_candidates(const TableArgs& t, Lane& L, uint32_t cand_cap, double lof, double hif,
                                  uint64_t m0, uint64_t m1, uint32_t& nc, bool& big) {
  nc = 0;
  if (hif < 0.0) return SST_NONE;
  const double af = lof < 1.0 ? 1.0 : lof;
  if (af <= hif) {
    const uint32_t a = (uint32_t)af, hi = (uint32_t)hif;
    const uint32_t* sums = t.pair_data;
    const uint32_t* recs = sums + (t.n_pairs + 2);
    const uint32_t* bk = recs + (t.n_pairs + 2);
    const uint32_t rel = a > t.pair_base ? a - t.pair_base : 0u;
    uint32_t k = bk[rel >> t.pair_shift] & 0xFFFFu;
    const uint32_t a2 = a << 1, h2 = (hi << 1) | 1u;
    while (sums[k] < a2) ++k;
    for (; sums[k] <= h2; ++k) {
      const uint32_t rec = recs[k];
      const int cnt = (int)(rec & 0xFFu);
      const int r0 = (int)((rec >> 8) & 0xFFu), r1 = cnt == 2 ? (int)((rec >> 16) & 0xFFu) : r0;
      const bool in0 = r0 < 64 ? (m0 >> r0) & 1ull : (m1 >> (r0 - 64)) & 1ull;
      const bool in1 = r1 < 64 ? (m0 >> r1) & 1ull : (m1 >> (r1 - 64)) & 1ull;
      if (!(in0 && in1)) continue;
      if (nc == cand_cap) {
        big = true;
        return SST_SOME;
      }
      L.cref[nc++] = ref_pair(k, cnt);
    }
  }
  return nc ? (int8_t)SST_SOME : lof <= 0.0 ? (int8_t)SST_EMPTY : (int8_t)SST_NONE;
}

// a DFS answer's candidates (payload records) into the lane's list
__device__ bool ref_candidates(Lane& L, uint32_t cand_cap, uint64_t ptr, uint32_t n, uint32_t& nc) {
  if (n > cand_cap) return false;
  const uint8_t* p = (const uint8_t*)ptr;
  for (uint32_t c = 0; c < n; ++c) {
    const int k = p[0];
    if (k > 127) return false;  // a ref holds 7 length bits: a side with such an explanation ends SST_WALK_LIMIT
    L.cref[c] = ref_ptr(p, k);
    p += 1 + k;
  }
  nc = n;
  return true;
}

// the query's explanation list (set order of its name tuples) appended to
// the bin's list without duplicates (explain_bin_differences :406-421)
__device__ bool merge_query(const TableArgs& t, const WalkArgs& a, Lane& L, uint32_t nc) {
  for (uint32_t c = 0; c < nc; ++c) {
    int64_t h;
    uint64_t m0, m1;
    cand_props(t, a, L.cref[c], h, m0, m1);
    L.chash[c] = h;
  }
  pyset::clear(L.ts);
  for (uint32_t c = 0; c < nc; ++c) pyset::add(L.ts, (int32_t)c, L.chash[c]);
  if (L.ts.overflow) return false;
  const int32_t* keys = L.ts.key[L.ts.cur];
  for (uint32_t s = 0; s <= L.ts.mask; ++s) {
    const int32_t c = keys[s];
    if (c < 0) continue;
    const uint64_t ref = L.cref[c];
    const int64_t h = L.chash[c];
    const int len = ref_len(ref);
    // `not in` the bin's list: equal name tuples have equal hashes, so only
    // the entries filed under this hash are compared
    uint32_t x = xi_slot(h, L.xmask);
    bool dup = false;
    for (;; x = (x + 1) & L.xmask) {
      const uint64_t v = L.xi[x];
      if ((uint32_t)(v >> 32) != L.xepoch) break;  // empty
      const uint64_t* e = L.ex + 4 * ((uint32_t)v - 1u);
      if ((int64_t)e[0] != h || ref_len(e[3]) != len) continue;
      bool same = true;
      for (int j = 0; j < len && same; ++j) same = ref_row(t, e[3], j) == ref_row(t, ref, j);
      if (same) {
        dup = true;
        break;
      }
    }
    if (dup) continue;
    if (L.n_ex == a.expl_cap) return false;
    int64_t hh;
    uint64_t m0, m1;
    cand_props(t, a, ref, hh, m0, m1);
    L.xi[x] = ((uint64_t)L.xepoch << 32) | (L.n_ex + 1u);
    uint64_t* e = L.ex + 4 * L.n_ex++;
    e[0] = (uint64_t)h;
    e[1] = m0;
    e[2] = m1;
    e[3] = ref;
  }
  return true;
}

// the k-th re-query answer of side sid (earlier rounds' blocks, in order)
__device__ bool resolved(const WalkArgs& a, uint32_t sid, uint32_t k, uint64_t& ptr, uint32_t& n, int8_t& st) {
  for (int r = 0; r < a.n_rounds; ++r) {
    const uint64_t blk = a.rq_block[r][sid];
    const uint32_t cnt = (uint32_t)blk, start = (uint32_t)(blk >> 32);
    if (k < cnt) {
      ptr = a.rq_ptr[r][start + k];
      n = a.rq_n[r][start + k];
      st = a.rq_st[r][start + k];
      return true;
    }
    k -= cnt;
  }
  return false;
}

struct SideRows {
  const uint16_t* rows;
  const double* su;
  const double* ob;
};

// query j of the bin pair (P = [p0, p1) or none, E = [e0, e1)): the
// difference and calculate_error_threshold (common.py:37-44) as :378-398
__device__ __forceinline__ void bin_query(const SideRows& R, int p0, int p1, int e0, int e1, uint32_t j, double tol,
                                          double& diff, double& thr) {
  if (p0 < 0) {
    const int c = R.rows[e0 + j];
    diff = R.su[c];
    thr = tol * (0.0 + R.ob[c]);
    return;
  }
  const uint32_t ne = (uint32_t)(e1 - e0);
  const int p = R.rows[p0 + j / ne], c = R.rows[e0 + j % ne];
  diff = R.su[c] - R.su[p];
  thr = tol * (R.ob[p] + R.ob[c]);
}

enum { kBinNone = 0, kBinSome = 1, kBinSuspend = 2, kBinBig = 3, kBinRaise = 4, kBinLimit = 5, kBinMissing = 6 };

}  // namespace

__global__ __launch_bounds__(256) void k_skel_walk(TableArgs t, WalkArgs a) {
  const uint32_t li = blockIdx.x * blockDim.x + threadIdx.x;
  if (li >= a.n_sides) return;
  const uint32_t sid = a.sides[li];
  const int64_t g = sid >> 1;
  const int sd = (int)(sid & 1u);
  const int64_t base = 4 * a.peak_off[g];
  const uint32_t nr = a.cnt[g];
  const int ML = a.max_len[g];
  const uint64_t m0 = a.alpha[2 * g], m1 = a.alpha[2 * g + 1];
  const bool pair_ok = a.pair_ok[g] != 0;
  // lane scratch: the side's slot (a relaunch finds its state there)
  uint8_t* sc = a.scratch + (uint64_t)(a.slot ? a.slot[li] : li) * a.scratch_stride;
  WalkState* wst = (WalkState*)sc;
  const bool resume = a.resume && wst->tag == sid + 1u;
  sc += kWalkStateBytes;
  // the side's rows (alive, side bit), SU order, as slot indices
  uint16_t* rows = a.side_rows + (sd ? a.slots : 0) + base;
  int32_t* mn = a.min_end + (sd ? a.slots : 0) + base;
  int32_t* mx = a.max_end + (sd ? a.slots : 0) + base;
  uint8_t* kp = a.kept + (sd ? a.slots : 0) + base;
  uint64_t* sk = a.skel + 2 * (a.skel_off[g] + (sd ? (uint64_t)ML : 0));
  uint32_t n = 0;
  if (resume) {
    n = wst->n;
  } else {
    for (uint32_t r = 0; r < nr; ++r)
      if (a.alive[base + r] && ((a.r_meta[base + r] >> (2 + sd)) & 1u)) rows[n++] = (uint16_t)r;
    for (uint32_t f = 0; f < n; ++f) {  // Predictor.predict's initial min_end / max_end (prediction.py:76-79)
      mn[rows[f]] = 0;
      mx[rows[f]] = -1;
      kp[rows[f]] = 1;
    }
    for (int i = 0; i < 2 * ML; ++i) sk[i] = 0;
    if (nr > (uint32_t)kPipeBigRows || ML + 2 > (int)a.len_cap) {
      a.side_status[sid] = kWalkLimit;
      return;
    }
  }
  Lane L;
  for (int s2 = 0; s2 < 2; ++s2) {
    for (int k = 0; k < 2; ++k) {
      L.pos[s2].key[k] = (int32_t*)sc;
      sc += 4ull * a.pos_cap;
      L.pos[s2].hash[k] = (int64_t*)sc;
      sc += 8ull * a.pos_cap;
    }
    L.pos[s2].cap = a.pos_cap;
  }
  L.lval = (uint64_t*)sc;
  sc += 16ull * a.len_cap;
  L.ex = (uint64_t*)sc;
  sc += 32ull * a.expl_cap;
  L.cref = (uint64_t*)sc;
  sc += 8ull * a.cand_cap;
  L.chash = (int64_t*)sc;
  sc += 8ull * a.cand_cap;
  for (int k = 0; k < 2; ++k) {
    L.ts.key[k] = (int32_t*)sc;
    sc += 4ull * a.tset_cap;
    L.ts.hash[k] = (int64_t*)sc;
    sc += 8ull * a.tset_cap;
  }
  L.ts.cap = a.tset_cap;
  L.xi = (uint64_t*)sc;
  L.xmask = walk_index_slots(a.expl_cap) - 1u;
  sc += 8ull * (L.xmask + 1u);
  L.lkeys = sc;
  sc += a.len_cap;
  L.lseen = sc;
  uint32_t f0 = 1, spec_ctr = 0, consumed = 0;  // speculative queries of the closed bins so far, re-query answers used
  int lv0 = -1, lv1 = -1;   // last bin with explanations
  int pb0 = -1, pb1 = -1;   // the previous closed bin
  int cur0 = 0;
  if (resume) {
    f0 = wst->f;
    spec_ctr = wst->spec_ctr;
    consumed = wst->consumed;
    lv0 = wst->lv0, lv1 = wst->lv1, pb0 = wst->pb0, pb1 = wst->pb1, cur0 = wst->cur0;
    L.cur = wst->cur;
    pyset::Table& P = L.pos[L.cur];
    P.mask = wst->pmask;
    P.fill = wst->pfill;
    P.cur = wst->pcur;
    P.overflow = wst->povf != 0;
    L.xepoch = wst->xepoch;
  } else {
    for (uint32_t k = 0; k < a.len_cap; ++k) L.lseen[k] = 0;
    for (uint32_t k = 0; k <= L.xmask; ++k) L.xi[k] = 0;
    L.xepoch = 0;
    L.cur = 0;
    pyset::clear(L.pos[0]);
    pyset::add(L.pos[0], 0, 0);  // pos = {0} (:126)
  }

  SideRows R{rows, a.r_su + base, a.r_ob + base};
  const uint64_t spec_q0 = a.q_off[g] + (sd ? a.q0[g] : 0u);  // this side's speculative queries
  int status = kWalkDone;
  const double pair_hi = (double)t.pair_hi;
  for (uint32_t f = f0; f < n && status == kWalkDone; ++f) {
    if (L.pos[L.cur].fill == 0) {  // no positions left (:132-135)
      kp[rows[f]] = 0;
      continue;
    }
    const double nd = R.su[rows[f]] - R.su[rows[f - 1]];
    const double nt = a.tol * (R.ob[rows[f - 1]] + R.ob[rows[f]]);
    const bool joined = nd <= nt;
    if (joined && f + 1 < n) continue;
    const int e0 = cur0, e1 = joined ? (int)f + 1 : (int)f;
    const int ne = e1 - e0;
    const bool first = pb0 < 0;
    bool spec = first ? lv0 < 0 : lv0 == pb0;  // the bin pair stage 3 answered
    const uint32_t spec_base = spec_ctr;
    spec_ctr += first ? (uint32_t)ne : (uint32_t)((pb1 - pb0) * ne);
    const int p0 = lv0, p1 = lv1;
    const uint32_t nq = p0 < 0 ? (uint32_t)ne : (uint32_t)((p1 - p0) * ne);
    // stage 3 answered each window at the bin's own threshold; a difference
    // the final dict holds is answered at the dict writer's threshold
    // (explain_mass_difference, skeleton_building.py:429-430).  Where the two
    // differ and the walk does not answer the window itself (not pair class:
    // exact-mode spectra), stage 3's answer is not the reference's: the bin
    // is re-queried instead
    for (uint32_t j = 0; j < nq && spec; ++j) {
      double diff, thr, te;
      bin_query(R, p0, p1, e0, e1, j, a.tol, diff, thr);
      if (dict_thr(a, g, diff, te) && te != thr) {
        double lof, hif;
        quantise_lean(diff, te, a.prec, a.rprec, lof, hif);
        if (!(pair_ok && hif < pair_hi)) spec = false;
      }
    }
    // re-query: its DFS windows must have been answered
    int res = kBinNone;
    if (!spec) {
      uint32_t n_off = 0;
      for (uint32_t j = 0; j < nq; ++j) {
        double diff, thr;
        bin_query(R, p0, p1, e0, e1, j, a.tol, diff, thr);
        double te;
        if (dict_thr(a, g, diff, te)) thr = te;
        double lof, hif;
        quantise_lean(diff, thr, a.prec, a.rprec, lof, hif);
        n_off += !(pair_ok && hif < pair_hi);
      }
      uint64_t tmp_p;
      uint32_t tmp_n;
      int8_t tmp_s;
      if (n_off && !resolved(a, sid, consumed + n_off - 1, tmp_p, tmp_n, tmp_s)) {
        if (a.n_rounds >= kWalkMaxRounds) {
          status = kWalkRounds;
          break;
        }
        const uint32_t start = atomicAdd(a.req_count, n_off);
        if ((uint64_t)start + n_off > a.req_cap) {
          status = kWalkLimit;
          break;
        }
        uint32_t o = 0;
        for (uint32_t j = 0; j < nq; ++j) {
          double diff, thr;
          bin_query(R, p0, p1, e0, e1, j, a.tol, diff, thr);
          double te;
          if (dict_thr(a, g, diff, te)) thr = te;
          double lof, hif;
          quantise_lean(diff, thr, a.prec, a.rprec, lof, hif);
          if (pair_ok && hif < pair_hi) continue;
          a.req_mass[start + o] = diff;
          a.req_thr[start + o] = thr;
          a.req_spec[start + o] = (int32_t)g;
          ++o;
        }
        a.req_block[sid] = ((uint64_t)start << 32) | n_off;
        status = kWalkSuspended;
        // the loop state at this bin's start, for the relaunch
        const pyset::Table& P = L.pos[L.cur];
        WalkState w{sid + 1u, f, n, spec_base, consumed, L.xepoch, lv0, lv1, pb0, pb1, cur0, L.cur,
                    P.mask, P.fill, P.cur, P.overflow ? 1u : 0u};
        *wst = w;
        break;
      }
    }
    // the bin's explanation list
    bool all_none = true;
    L.n_ex = 0;
    ++L.xepoch;  // empties the list's index
    uint32_t off_j = 0;
    for (uint32_t j = 0; j < nq && res == kBinNone; ++j) {
      double diff, thr;
      bin_query(R, p0, p1, e0, e1, j, a.tol, diff, thr);
      double te;
      if (dict_thr(a, g, diff, te)) thr = te;
      double lof, hif;
      quantise_lean(diff, thr, a.prec, a.rprec, lof, hif);
      uint32_t nc = 0;
      int8_t st;
      bool big = false;
      if (pair_ok && hif < pair_hi) {
        st = pair_candidates(t, L, a.cand_cap, lof, hif, m0, m1, nc, big);
        if (big) res = kBinBig;
      } else {
        uint64_t ptr = 0;
        uint32_t cnt = 0;
        st = (int8_t)kStatusPending;
        if (spec) {
          const uint64_t q = spec_q0 + spec_base + j;
          ptr = a.s_ptr[q];
          cnt = a.s_n[q];
          st = a.s_st[q];
        } else if (!resolved(a, sid, consumed + off_j, ptr, cnt, st)) {
          res = kBinMissing;
        }
        ++off_j;
        if (res == kBinNone && st == SST_SOME && !ref_candidates(L, a.cand_cap, ptr, cnt, nc)) res = kBinBig;
      }
      if (res != kBinNone) break;
      if (st == SST_NONE) continue;  // None (:402-404)
      if (st == SST_EMPTY) {         // [] (set() -> empty list)
        all_none = false;
        continue;
      }
      if (st == SST_OUT_OF_TABLE) {  // the reference raises (NameError, mass_explanation.py:134-138)
        res = kBinRaise;
        break;
      }
      if (st != SST_SOME) {  // OVERFLOW / ABORTED / unanswered: no candidate list to order
        res = st == (int8_t)kStatusPending ? kBinMissing : kBinLimit;
        break;
      }
      all_none = false;
      if (!merge_query(t, a, L, nc)) res = kBinBig;
    }
    if (!spec) consumed += off_j;
    if (res == kBinBig) {
      status = kWalkBig;
      break;
    }
    if (res == kBinRaise) {
      status = kWalkRaise;
      break;
    }
    if (res == kBinLimit) {
      status = kWalkLimit;
      break;
    }
    if (res == kBinMissing) {
      status = kWalkMissing;
      break;
    }
    if (all_none) {  // skip the bin: its fragments are rejected (:161-173)
      for (int e = e0; e < e1; ++e) kp[rows[e]] = 0;
    } else {
      // update_skeleton_for_given_explanations (:442-482)
      pyset::Table& P = L.pos[L.cur];
      pyset::Table& Nx = L.pos[L.cur ^ 1];
      pyset::clear(Nx);
      const int32_t* pk = P.key[P.cur];
      for (uint32_t s = 0; s <= P.mask; ++s) {
        const int p = pk[s];
        if (p < 0) continue;
        int nk = 0, prev = -1;
        for (uint32_t u = 0; u < L.n_ex; ++u) {
          const uint64_t* e = L.ex + 4 * u;
          const int len = ref_len(e[3]);
          if (p + len - 1 >= ML) continue;  // 0 <= p + len - 1 < max_len (:457)
          if (len != prev) {                // groupby: a new run; the dict keeps the last run per length
            if (!L.lseen[len]) {
              L.lseen[len] = 1;
              L.lkeys[nk++] = (uint8_t)len;
            }
            L.lval[2 * len] = L.lval[2 * len + 1] = 0;
            prev = len;
          }
          L.lval[2 * len] |= e[1];
          L.lval[2 * len + 1] |= e[2];
        }
        for (int k = 0; k < nk; ++k) {
          const int len = L.lkeys[k];
          const uint64_t v0 = L.lval[2 * len], v1 = L.lval[2 * len + 1];
          for (int i = 0; i < len; ++i) {
            uint64_t* S = sk + 2 * (p + i);
            if ((v0 & ~S[0]) == 0 && (v1 & ~S[1]) == 0) {  // issuperset: clear, then add
              S[0] = v0;
              S[1] = v1;
            } else {
              S[0] |= v0;
              S[1] |= v1;
            }
          }
        }
        for (int k = 0; k < nk; ++k) {
          const int q = p + L.lkeys[k];
          pyset::add(Nx, q, q);
          L.lseen[L.lkeys[k]] = 0;
        }
      }
      L.cur ^= 1;
      pyset::Table& Q = L.pos[L.cur];
      if (Q.overflow) {
        status = kWalkLimit;
        break;
      }
      int lo = 1, hi = 0;  // min(pos, default=1), max(pos, default=0)
      if (Q.fill) {
        lo = 1 << 30;
        hi = -1;
        const int32_t* qk = Q.key[Q.cur];
        for (uint32_t s = 0; s <= Q.mask; ++s) {
          const int p = qk[s];
          if (p < 0) continue;
          lo = p < lo ? p : lo;
          hi = p > hi ? p : hi;
        }
      }
      for (int e = e0; e < e1; ++e) {
        mn[rows[e]] = lo;
        mx[rows[e]] = hi;
      }
      lv0 = e0;
      lv1 = e1;
    }
    pb0 = e0;
    pb1 = e1;
    cur0 = (int)f;
  }
  a.side_status[sid] = (uint8_t)status;
  if (status == kWalkSuspended) atomicAdd(a.n_suspended, 1u);
  if (status == kWalkBig) atomicAdd(a.n_big, 1u);
}

// a result's candidate references scattered to dst[i] (sst_result_refs_device)
__global__ void k_refs_status(const int8_t* __restrict__ status, int64_t n, const int64_t* __restrict__ dst,
                              uint64_t* ptr, uint32_t* cnt, int8_t* st) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t d = dst[i];
  st[d] = status[i];
  cnt[d] = 0;
  ptr[d] = 0;
}
__global__ void k_refs_hits(const uint4* __restrict__ hits, uint64_t n_hits, const uint8_t* payload,
                            const int8_t* __restrict__ status, const int64_t* __restrict__ dst, uint64_t* ptr,
                            uint32_t* cnt) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_hits) return;
  const uint4 h = hits[k];
  const int64_t d = dst[h.x];
  const uint64_t word = (uint64_t)h.z | ((uint64_t)h.w << 32);
  if (status[h.x] == SST_SOME) {
    cnt[d] = h.y;
    ptr[d] = (uint64_t)(payload + word);
  } else {  // OVERFLOW / ABORTED: the exact count, no payload
    cnt[d] = word > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)word;
  }
}
hipError_t launch_result_refs(const int8_t* status, int64_t n, const uint4* hits, uint64_t n_hits,
                              const uint8_t* payload, const int64_t* dst, uint64_t* ptr, uint32_t* cnt, int8_t* st,
                              hipStream_t stream) {
  if (n > 0) hipLaunchKernelGGL(k_refs_status, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, status, n, dst,
                                ptr, cnt, st);
  if (n_hits > 0)
    hipLaunchKernelGGL(k_refs_hits, dim3((unsigned)((n_hits + 255) / 256)), dim3(256), 0, stream, hits, n_hits,
                       payload, status, dst, ptr, cnt);
  return hipGetLastError();
}

uint64_t walk_scratch_bytes(uint32_t pos_cap, uint32_t len_cap, uint32_t expl_cap, uint32_t cand_cap,
                            uint32_t tset_cap) {
  const uint64_t b = kWalkStateBytes + 2ull * 2 * 12 * pos_cap + 16ull * len_cap + 32ull * expl_cap +
                     16ull * cand_cap + 2ull * 12 * tset_cap + 8ull * walk_index_slots(expl_cap) + 2ull * len_cap;
  return (b + 15) & ~15ull;
}

hipError_t launch_skel_walk(const TableArgs& t, const WalkArgs& a, hipStream_t st) {
  if (a.n_sides == 0) return hipSuccess;
  hipLaunchKernelGGL(k_skel_walk, dim3((a.n_sides + 255) / 256), dim3(256), 0, st, t, a);
  return hipGetLastError();
}

// select_sequence_length_with_jaccard + combine_skeleton_sequences, one lane
// per spectrum (skeleton_building.py:315-370, 485-516, 291-313)
namespace {
__device__ __forceinline__ int pop128(uint64_t a, uint64_t b) { return __builtin_popcountll(a) + __builtin_popcountll(b); }
// Python slice start of seq[len(seq) - k:] for a list of n items
__device__ __forceinline__ int tail_start(int n, int k) {
  int s = n - k;
  if (s < 0) s += n;
  return s < 0 ? 0 : s;
}
__device__ __forceinline__ int lowest(uint64_t a, uint64_t b) { return a ? __builtin_ctzll(a) : 64 + __builtin_ctzll(b); }
__device__ __forceinline__ int highest(uint64_t a, uint64_t b) { return b ? 127 - __builtin_clzll(b) : 63 - __builtin_clzll(a); }
}  // namespace

__global__ __launch_bounds__(256) void k_jaccard(sst_jaccard_args a) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= a.n_spec) return;
  const int ML = a.max_len[g];
  const uint64_t* st = a.skel + 2 * a.skel_off[g];      // START skeleton
  const uint64_t* en = a.skel + 2 * (a.skel_off[g] + ML);  // END skeleton as walked; reversed below
  // end_skeleton = end_skeleton[::-1]: position i is the walked position ML - 1 - i
  auto E0 = [&](int i) { return en[2 * (ML - 1 - i)]; };
  auto E1 = [&](int i) { return en[2 * (ML - 1 - i) + 1]; };
  if (a.status_lb[g] != 0) {
    a.status[g] = SST_JAC_BOUNDS;
    a.seq_len[g] = 0;
    return;
  }
  const int64_t lo = a.lower[g], hi = a.upper[g];
  int64_t best_len = lo;
  double best_val = -1.0;
  for (int64_t lc = lo; lc <= hi; ++lc) {
    const int ns = (int)(lc < ML ? lc : ML);  // start_skeleton[:lc]
    const int e0 = tail_start(ML, (int)(lc < (int64_t)ML + ML ? lc : (int64_t)ML + ML));  // end_skeleton[ML - lc:]
    const int ne = ML - e0;
    const int np = ns < ne ? ns : ne;  // zip
    // sum(map(jaccard_index, ...)) / lc: CPython 3.10 sum() adds the ints
    // (empty side: 1) and floats (|a & b| / |a | b|) in order in one double
    bool is_int = true;
    int64_t isum = 0;
    double fsum = 0.0;
    for (int i = 0; i < np; ++i) {
      const uint64_t a0 = st[2 * i], a1 = st[2 * i + 1], b0 = E0(e0 + i), b1 = E1(e0 + i);
      const int na = pop128(a0, a1), nb = pop128(b0, b1);
      if (na == 0 || nb == 0) {
        if (is_int) isum += 1;
        else fsum += 1.0;
      } else {
        const double j = (double)pop128(a0 & b0, a1 & b1) / (double)pop128(a0 | b0, a1 | b1);
        if (is_int) {
          fsum = (double)isum;
          is_int = false;
        }
        fsum += j;
      }
    }
    const double value = (is_int ? (double)isum : fsum) / (double)lc;
    if (!(value > best_val)) continue;
    // validate_sequence_length_by_mass on the same slices
    double mn = 0.0, mx = 0.0;
    for (int i = 0; i < np; ++i) {
      const uint64_t u0 = st[2 * i] | E0(e0 + i), u1 = st[2 * i + 1] | E1(e0 + i);
      if (!(u0 | u1)) continue;  // min([], default=0)
      mn += a.row_mass[lowest(u0, u1)];   // rows ascend by mass
      mx += a.row_mass[highest(u0, u1)];
    }
    const double su = a.su_mass[g];
    if (mn - a.max_variance <= su && su <= mx + a.max_variance) {
      best_val = value;
      best_len = lc;
    }
  }
  if (best_val < 0.0) {
    a.status[g] = SST_JAC_NO_LENGTH;
    a.seq_len[g] = 0;
    return;
  }
  a.seq_len[g] = (int32_t)best_len;
  if (best_len > ML || best_len < 0) {  // start_skeleton[i] past its end: IndexError
    a.status[g] = SST_JAC_INDEX;
    return;
  }
  const int L = (int)best_len;
  const int e0 = tail_start(ML, L);
  uint64_t* out = a.comb + 2 * a.comb_off[g];
  for (int i = 0; i < L; ++i) {
    const uint64_t s0 = st[2 * i], s1 = st[2 * i + 1], b0 = E0(e0 + i), b1 = E1(e0 + i);
    uint64_t c0 = s0 & b0, c1 = s1 & b1;  // the intersection, else the union
    if (!(c0 | c1)) {
      c0 = s0 | b0;
      c1 = s1 | b1;
    }
    out[2 * i] = c0;
    out[2 * i + 1] = c1;
  }
  a.status[g] = SST_JAC_OK;
}

hipError_t launch_jaccard(const sst_jaccard_args& a, hipStream_t st) {
  if (a.n_spec <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_jaccard, dim3((unsigned)((a.n_spec + 255) / 256)), dim3(256), 0, st, a);
  return hipGetLastError();
}

// the skeleton's alphabet reduction (skeleton_building.py:319-326,
// adapt_individual_modification_rates_by_alphabet_reduction,
// mass_table.py:94-100): the canonical rows and the kept modifications some
// position of either side's skeleton names, one lane per spectrum
__global__ __launch_bounds__(256) void k_skel_alpha(int64_t n_spec, const int32_t* max_len, const uint64_t* skel_off,
                                                    const uint64_t* skel, const uint64_t* alpha, uint64_t canon0,
                                                    uint64_t canon1, uint64_t* out) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_spec) return;
  const uint64_t* sk = skel + 2 * skel_off[g];
  uint64_t u0 = 0, u1 = 0;
  for (int i = 0; i < 2 * max_len[g]; ++i) {
    u0 |= sk[2 * i];
    u1 |= sk[2 * i + 1];
  }
  out[2 * g] = alpha[2 * g] & (canon0 | u0);
  out[2 * g + 1] = alpha[2 * g + 1] & (canon1 | u1);
}
hipError_t launch_skel_alpha(int64_t n_spec, const int32_t* max_len, const uint64_t* skel_off, const uint64_t* skel,
                             const uint64_t* alpha, uint64_t canon0, uint64_t canon1, uint64_t* out, hipStream_t st) {
  if (n_spec <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_skel_alpha, dim3((unsigned)((n_spec + 255) / 256)), dim3(256), 0, st, n_spec, max_len,
                     skel_off, skel, alpha, canon0, canon1, out);
  return hipGetLastError();
}

// After the skeleton (prediction.py:88-103): build_skeleton's fragment
// bookkeeping (skeleton_building.py:67-109) -- the START walk's kept rows
// (min_end / max_end - 1), the END walk's kept rows not already kept at START
// (len - min_end / len - max_end), the internal rows whose peak no kept
// terminal row shares, every end index outside [0, len) clamped to len - 1
// -- and the alphabet _reduce_alphabet then sets: the Jaccard stage's
// alphabet with the modifications the combined skeleton does not name dropped
// (mass_table.py:94-100).  One workgroup per spectrum; the peaks of kept
// terminal rows as an LDS bitmap.  The caller then runs is_valid on that
// alphabet (sst_valid_rows_alpha_device) over alive_out.
constexpr int kPostPeaks = kPipeMaxPeaksBig + 1;  // the classify kernels' peak limit
__global__ __launch_bounds__(256) void k_post_skel(sst_post_args a, uint64_t canon0, uint64_t canon1) {
  __shared__ uint32_t peaks[kPostPeaks / 32];
  __shared__ uint64_t names[2];
  for (int64_t g = blockIdx.x; g < a.n_spec; g += gridDim.x) {
    const int64_t off = 4 * a.peak_off[g];
    const int n = (int)a.rows[g];
    const int64_t np = a.peak_off[g + 1] - a.peak_off[g];
    const bool ok = a.jac_status[g] == SST_JAC_OK && np <= kPostPeaks;
    if (threadIdx.x == 0) {
      if (a.jac_status[g] == SST_JAC_OK && np > kPostPeaks) atomicOr(a.err, 1u);
      a.active[g] = ok ? 1 : 0;
      names[0] = names[1] = 0;
    }
    if (!ok) {  // build_skeleton raised: predict returns Prediction.default() (:89-94)
      for (int i = threadIdx.x; i < n; i += blockDim.x) a.alive_out[off + i] = 0;
      if (threadIdx.x == 0) {
        a.alpha_out[2 * g] = a.alpha[2 * g];
        a.alpha_out[2 * g + 1] = a.alpha[2 * g + 1];
      }
      __syncthreads();
      continue;
    }
    const int L = a.seq_len[g];
    for (int w = threadIdx.x; w < kPostPeaks / 32; w += blockDim.x) peaks[w] = 0;
    __syncthreads();
    const uint8_t* kept_s = a.kept;
    const uint8_t* kept_e = a.kept + a.slots;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const uint32_t m = a.meta[off + i];
      const bool al = a.alive[off + i] != 0;
      const bool st = al && ((m >> 2) & 1u) && kept_s[off + i];
      const bool en = al && ((m >> 3) & 1u) && kept_e[off + i] && !st;
      if (st || en) atomicOr(&peaks[(m >> 8) >> 5], 1u << ((m >> 8) & 31u));
    }
    // the combined skeleton's names (positions 0 .. len - 1)
    const uint64_t* cb = a.comb + 2 * a.comb_off[g];
    uint64_t u0 = 0, u1 = 0;
    for (int i = threadIdx.x; i < L; i += blockDim.x) {
      u0 |= cb[2 * i];
      u1 |= cb[2 * i + 1];
    }
    if (u0) atomicOr((unsigned long long*)&names[0], (unsigned long long)u0);
    if (u1) atomicOr((unsigned long long*)&names[1], (unsigned long long)u1);
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const uint32_t m = a.meta[off + i];
      const bool al = a.alive[off + i] != 0;
      const bool st = al && ((m >> 2) & 1u) && kept_s[off + i];
      const bool en = al && ((m >> 3) & 1u) && kept_e[off + i] && !st;
      const bool internal = al && !((m >> 2) & 3u);
      const bool fin = st || en || (internal && !((peaks[(m >> 8) >> 5] >> ((m >> 8) & 31u)) & 1u));
      int lo = 0, hi = -1;  // Predictor.predict's initial columns (prediction.py:76-79)
      if (st) {
        lo = a.min_end[off + i] - 1;
        hi = a.max_end[off + i] - 1;
      } else if (en) {
        lo = L - a.min_end[a.slots + off + i];
        hi = L - a.max_end[a.slots + off + i];
      }
      if (lo < 0 || lo >= L) lo = L - 1;
      if (hi < 0 || hi >= L) hi = L - 1;
      a.alive_out[off + i] = fin ? 1 : 0;
      a.min_end_out[off + i] = lo;
      a.max_end_out[off + i] = hi;
    }
    if (threadIdx.x == 0) {
      a.alpha_out[2 * g] = a.alpha[2 * g] & (canon0 | names[0]);
      a.alpha_out[2 * g + 1] = a.alpha[2 * g + 1] & (canon1 | names[1]);
    }
    __syncthreads();
  }
}
// the walk's re-query answers merged over rounds (skeleton_device's round
// loop): per side, the merged view's entries of the earlier rounds, then this
// round's block -- round-major per side, sides in order, as the walk's
// resolved() reads a single round.  count: per side totals; copy: one lane
// per side (its entries are few), at the exclusive scan of the totals.
__global__ void k_requery_count(const int64_t* o_block, const int64_t* block, uint32_t* tot, int64_t n_sides) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_sides) return;
  const uint32_t o = o_block ? (uint32_t)((uint64_t)o_block[i] & 0xFFFFFFFFull) : 0u;
  tot[i] = o + (uint32_t)((uint64_t)block[i] & 0xFFFFFFFFull);
}
__global__ void k_requery_copy(sst_requery_merge_args a, const uint64_t* off) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n_sides) return;
  uint64_t at = off[i];
  const uint64_t start = at;
  if (a.o_block) {
    const uint64_t b = (uint64_t)a.o_block[i];
    for (uint64_t k = b >> 32, e = (b >> 32) + (b & 0xFFFFFFFFull); k < e; ++k, ++at) {
      a.m_ptr[at] = a.o_ptr[k];
      a.m_n[at] = a.o_n[k];
      a.m_st[at] = a.o_st[k];
    }
  }
  const uint64_t b = (uint64_t)a.block[i];
  for (uint64_t k = b >> 32, e = (b >> 32) + (b & 0xFFFFFFFFull); k < e; ++k, ++at) {
    a.m_ptr[at] = a.ptr[k];
    a.m_n[at] = a.n[k];
    a.m_st[at] = a.st[k];
  }
  a.m_block[i] = (int64_t)((start << 32) | (at - start));
}
hipError_t launch_requery_merge(const sst_requery_merge_args& a, uint32_t* tot, uint64_t* off, hipStream_t st) {
  if (a.n_sides <= 0) return hipSuccess;
  const unsigned g = (unsigned)((a.n_sides + 255) / 256);
  hipLaunchKernelGGL(k_requery_count, dim3(g), dim3(256), 0, st, a.o_block, a.block, tot, a.n_sides);
  if (hipError_t e = launch_scan_u32(tot, off, a.n_sides, st)) return e;
  hipLaunchKernelGGL(k_requery_copy, dim3(g), dim3(256), 0, st, a, (const uint64_t*)off);
  return hipGetLastError();
}

hipError_t launch_post_skel(const sst_post_args& a, uint64_t canon0, uint64_t canon1, int n_wg, hipStream_t st) {
  if (a.n_spec <= 0) return hipSuccess;
  const int64_t g = a.n_spec < (int64_t)n_wg ? a.n_spec : (int64_t)n_wg;
  hipLaunchKernelGGL(k_post_skel, dim3((unsigned)g), dim3(256), 0, st, a, canon0, canon1);
  return hipGetLastError();
}

}  // namespace sst
