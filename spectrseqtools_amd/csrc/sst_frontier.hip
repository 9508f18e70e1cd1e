// sst_frontier.hip -- compute_sequence_length_bound (mass_table.py:343-487)
// on the skeleton's reduced alphabets, both directions, WITHOUT replaying the
// reference's memoised DFS (gfx950).
//
// The reference walks backtrack(m, r, A, B) depth-first: memo check, up
// branch (m, r-1) before left branch (m - w_r, r), one memo shared by every
// window value (ascending).  The memo key (m, r) ignores the budgets (A, B), so
// a node's memoised value is fixed by its FIRST visit's budgets -- the only
// order-dependent thing in the whole computation.  That first visit is not a
// property of the DFS order alone: it is the lexicographically smallest path
//     (root index, c_{K-1}, c_{K-2}, ..., c_r)      c_s = left moves in row s
// among the paths the DFS actually expands, and a node is expanded exactly
// once, at its own first visit.  So
//     FV(m, r) = lexmin( FV(m, r+1) . up,  FV(m + w_r, r) . left )
// over the two possible parents (the up parent only if m is in R_{r-1}..R_r,
// the left parent only if ITS first-visit budgets allow the move), a
// recurrence over descending masses: a left parent is heavier by w_r >= w_min,
// an up parent has the same mass.  Masses are therefore processed in bands of
// w_min (every band depends only on earlier bands and, within a mass, on the
// row above), one launch per band; the values (min / max path length, the
// reference's defaults and its -1 + 1 = 0 quirk included) then follow by a DP
// over ascending masses, one launch per band in reverse.  Nodes = the
// reference's memo entries; no node is ever revisited.  DESIGN §3.
//
// Data (per chunk of queries, HBM):
//   lr        per alphabet: byte per mass, the lowest kept rank k with the mass
//             in R_k (0xFF: none) -- pair(k, m) != 0 <=> lr[m] <= k, bit0 <=>
//             lr[m] <= k-1, bit1 <=> m - w_k == 0 or lr[m - w_k] <= k
//   groups    one per (query, mass) with at least one visited row: hash ring
//             of R tables (band mod R), 32-B entries {key, 128-bit rank mask
//             of the left candidates}; each band's fresh groups listed
//   cands     one per left edge (child (query, mass, rank)): hash ring, entry
//             {key, parent node, child budgets A B, the child's FV key}
//   nodes     ids allocated per group (ranks lo..hv ascending): flags, left
//             parent id (a node with a left parent, or its root slot), and
//             its left child's lower / upper value packed in 16 bits, pushed
//             there by the child (values run bands in reverse: the child's
//             first); a root's value goes to its root slot the same way
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sst_internal.h"
#include "sst_quant.h"

namespace sst {

namespace {

constexpr int kProbeMax = 4096;
constexpr uint32_t kRootBit = 0x80000000u;
constexpr uint32_t kRootUnset = 0xFFFFFFFFu;  // a root slot whose node has not pushed its value
constexpr uint32_t kNodeSeg = 512;  // k_lbf_nodes: ids per ticket
constexpr uint32_t kFreshBuf = 640;  // > kNodeSeg + 127: the nodes of a range moved to group starts
constexpr uint8_t kFLeft = 1, kFUp = 2, kFZero = 4, kFCand = 8;  // kFCand: k_lbf_groups' mark, until k_lbf_nodes
constexpr uint8_t kFPar = 16;  // k_lbf_nodes: the node has a left parent or is a root (lpar)

struct alignas(32) FGroup {
  uint64_t key;
  uint64_t mask[2];
  uint64_t pad;
};

template <int KW>
struct FCand {
  uint64_t key;
  uint32_t parent;
  uint8_t A, B;
  uint16_t pad;
  uint64_t fk[KW];
};

// hash keys: tag (12 bits: the chunk's epoch mod 32, band + 1 <= 127) | listed
// query (20) | mass (25) | rank (7).  A slot whose tag is not the current one
// is free: stale entries of earlier bands and chunks need no clearing.
__device__ __forceinline__ uint64_t fkey(uint32_t tagb, uint32_t j, uint32_t m, uint32_t k) {
  return ((uint64_t)tagb << 52) | ((uint64_t)j << 32) | ((uint64_t)m << 7) | (uint64_t)k;
}
__device__ __forceinline__ uint32_t ftagb(const FrontierArgs& a, uint32_t band) {
  return ((uint32_t)a.epoch << 7) | (band + 1u);
}
__device__ __forceinline__ uint32_t ftag(uint64_t key) { return (uint32_t)(key >> 52); }
__device__ __forceinline__ uint32_t fhash(uint64_t key, uint32_t mask) {
  uint64_t x = key * 0x9E3779B97F4A7C15ull;
  x ^= x >> 31;
  return (uint32_t)(x >> 17) & mask;
}

__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const int o = __shfl_xor(v, d, 64);
    v = o > v ? o : v;
  }
  return v;
}
__device__ __forceinline__ uint32_t wave_incl_u(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(v, d, 64);
    if (lane >= d) v += y;
  }
  return v;
}
__device__ __forceinline__ uint64_t lanemask_lt() {
  const int lane = threadIdx.x & 63;
  return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// the lane owning item q of a wave's items laid out by lane (incl: the
// inclusive count up to each lane): the first lane whose count exceeds q
__device__ __forceinline__ int wave_owner(uint32_t incl, uint32_t q) {
  int g = 0;
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1)
    if (__shfl(incl, g + s - 1, 64) <= q) g += s;
  return g;
}

// the t-th highest set bit (t from 0) of the 128-bit mask (h1:h0)
__device__ __forceinline__ int mask_select_top(uint64_t h1, uint64_t h0, uint32_t t) {
  const uint32_t c1 = (uint32_t)__builtin_popcountll(h1);
  const uint64_t x = t < c1 ? h1 : h0;
  const uint32_t need = (t < c1 ? t : t - c1) + 1u;
  int b = 0;
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1)
    if ((uint32_t)__builtin_popcountll(x >> (b + s)) >= need) b += s;
  return (t < c1 ? 64 : 0) + b;
}

// find-or-insert (band-tagged; a slot whose tag is not this band's is free)
__device__ __forceinline__ uint32_t group_get(FGroup* T, uint32_t mask, uint64_t key, bool& fresh) {
  const uint32_t tag = ftag(key);
  uint32_t h = fhash(key, mask);
  for (int p = 0; p < kProbeMax; ++p) {
    const uint64_t cur = __hip_atomic_load(&T[h].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == key) {
      fresh = false;
      return h;
    }
    if (ftag(cur) != tag) {
      const uint64_t prev = atomicCAS((unsigned long long*)&T[h].key, (unsigned long long)cur, (unsigned long long)key);
      if (prev == cur) {
        fresh = true;
        return h;
      }
      if (prev == key) {
        fresh = false;
        return h;
      }
    }
    h = (h + 1) & mask;
  }
  return UINT32_MAX;
}

// insert a key known to be new (a left edge has one parent)
template <int KW>
__device__ __forceinline__ uint32_t cand_put(FCand<KW>* T, uint32_t mask, uint64_t key) {
  const uint32_t tag = ftag(key);
  uint32_t h = fhash(key, mask);
  for (int p = 0; p < kProbeMax; ++p) {
    const uint64_t cur = __hip_atomic_load(&T[h].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (ftag(cur) != tag) {
      const uint64_t prev = atomicCAS((unsigned long long*)&T[h].key, (unsigned long long)cur, (unsigned long long)key);
      if (prev == cur) return h;
    }
    h = (h + 1) & mask;
  }
  return UINT32_MAX;
}

template <int KW>
__device__ __forceinline__ uint32_t cand_find(const FCand<KW>* T, uint32_t mask, uint64_t key) {
  const uint32_t tag = ftag(key);
  uint32_t h = fhash(key, mask);
  for (int p = 0; p < kProbeMax; ++p) {
    const uint64_t cur = T[h].key;
    if (cur == key) return h;
    if (ftag(cur) != tag) return UINT32_MAX;
    h = (h + 1) & mask;
  }
  return UINT32_MAX;
}

// first-visit keys: a KW x 64-bit big-endian integer (word 0 most
// significant) whose lexicographic order is the reference's DFS preorder: the
// root index in the top rb bits, then each kept rank from the top down in
// unary -- c_s ones and a zero.  (Unary keeps the order: at the first rank
// where two count vectors differ, the smaller count meets its zero where the
// larger has a one.)  A path in row k has zero counts below k, so every bit
// after its current position is zero, and one more left move in row k sets the
// bit at rb + d + (K - 1 - k) from the top (d = the path's left moves so far:
// the ones already set).  rb + max d + K bits; max d <= hi / w_min.
template <int KW>
__device__ __forceinline__ bool key_less(const uint64_t (&a)[KW], const uint64_t (&b)[KW]) {
  bool lt = false, decided = false;
#pragma unroll
  for (int i = 0; i < KW; ++i) {
    if (!decided && a[i] != b[i]) {
      lt = a[i] < b[i];
      decided = true;
    }
  }
  return lt;
}
template <int KW>
__device__ __forceinline__ int key_ones(const uint64_t (&k)[KW], int rb) {  // left moves on the path
  int d = rb > 0 ? -__builtin_popcountll(k[0] >> (64 - rb)) : 0;
#pragma unroll
  for (int i = 0; i < KW; ++i) d += __builtin_popcountll(k[i]);
  return d;
}
template <int KW>
__device__ __forceinline__ void key_set_msb(uint64_t (&k)[KW], int p) {  // bit p counted from the most significant
#pragma unroll
  for (int i = 0; i < KW; ++i)
    if (i == (p >> 6)) k[i] |= 1ull << (63 - (p & 63));
}

__device__ __forceinline__ uint32_t qrow_w(uint32_t x) { return x & 0xFFFFFu; }
__device__ __forceinline__ int qrow_cap(uint32_t x) { return (int)((x >> 20) & 0xFFu); }
__device__ __forceinline__ bool qrow_mod(uint32_t x) { return (x >> 28) & 1u; }

__device__ __forceinline__ void set_overflow(FrontierArgs& a, uint32_t why) { atomicOr(&a.ctl->overflow, why); }

}  // namespace

// per listed query (one wave each): its window, budgets, alphabet rank table
__global__ __launch_bounds__(256) void k_lbf_setup(TableArgs t, FrontierArgs a) {
  const int lane = threadIdx.x & 63;
  const uint32_t jj = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (jj >= a.n_chunk) return;
  const uint32_t i = a.list[a.chunk0 + jj];
  int64_t lo, hi;
  quantise(a.su[i], a.tol * a.obs[i], false, a.tol, a.prec, a.rprec, lo, hi);  // mass_table.py:354-359
  const uint32_t u = (uint32_t)a.spec[i];
  const int L = a.qlen ? a.qlen[i] : a.max_len;
  const int A0 = a.qlen ? a.a0_len[L] : a.A0;
  const uint64_t top = t.n_rows >= 64 ? (t.n_rows - 64 >= 64 ? ~0ull : ((1ull << (t.n_rows - 64)) - 1ull)) : 0ull;
  const uint64_t m0 = a.alpha[2 * u] & ~1ull & (t.n_rows >= 64 ? ~0ull : ((1ull << t.n_rows) - 1ull));
  const uint64_t m1 = a.alpha[2 * u + 1] & top;
  const int n_lo = __builtin_popcountll(m0);
  const int K = n_lo + __builtin_popcountll(m1);
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int r = lane + 64 * half;
    const uint64_t mm = half ? m1 : m0;
    if (r < t.n_rows && ((mm >> lane) & 1ull)) {
      const int rank = (half ? n_lo : 0) + __builtin_popcountll(mm & ((1ull << lane) - 1ull));
      int cap = a.qlen ? a.caps_len[(int64_t)L * kMaxRows + r] : t.cap[r];
      cap = cap < 0 ? 0 : (cap > 255 ? 255 : cap);
      a.qrow[(size_t)jj * 128 + rank] = (uint32_t)t.w[r] | ((uint32_t)cap << 20) | ((uint32_t)(t.mod[r] ? 1 : 0) << 28);
    }
  }
  if (lane == 0) {
    // queries the engine's layout cannot hold are answered SST_ABORTED on
    // their own (the batch's other queries are unaffected): a window wider
    // than one band (its roots would fall in several bands, and a root's left
    // child could land on another root's mass), a window top at 2^25 or
    // beyond (the keys' mass field), or a first-visit key beyond 256 bits
    // (root index bits -- at most bits(w_min - 1) once the window fits a
    // band --, one bit per kept rank, one per left move <= hi / w_min)
    int kb = 0;
    while (kb < 32 && ((uint32_t)(a.wb - 1) >> kb)) ++kb;
    const int64_t win0 = hi - lo + 1;
    const bool fits = win0 <= (int64_t)a.wb && hi < (1ll << 25) &&
                      kb + K + (int)((hi > 0 ? hi : 0) / a.wb) <= 256;
    FQInfo q;
    q.hi = fits ? hi : lo - 1;  // an excluded query has no window values: no roots, no nodes
    q.lo = lo;
    q.lr_off = a.lr_off[u];
    q.i = i;
    q.K = (uint16_t)(fits ? K : 0);
    q.L = (uint16_t)(L > 65535 ? 65535 : L);
    q.A0 = (uint16_t)(A0 < 0 ? 0 : (A0 > 255 ? 255 : A0));
    q.pad = fits ? 0 : 1;
    a.qi[jj] = q;
    if (!fits) {
      a.status[i] = SST_ABORTED;
      return;
    }
    atomicMax(&a.ctl->max_need, (uint32_t)(K + (hi > 0 ? hi : 0) / a.wb));
    if (hi >= 1) {
      atomicMax(&a.ctl->max_band, (uint32_t)((hi - 1) / a.wb));
      atomicMax((unsigned long long*)&a.ctl->max_hi, (unsigned long long)hi);
    }
    const int64_t win = hi - lo + 1;
    atomicMax(&a.ctl->max_win, (uint32_t)(win < 1 ? 1 : (win > 0x7FFFFFFF ? 0x7FFFFFFF : win)));
    atomicMax(&a.ctl->max_k, (uint32_t)K);
  }
}

// the roots: window values v >= 1 in R_{K-1}, band 0, key (v - lo, 0, ...)
template <int KW>
__global__ __launch_bounds__(256) void k_lbf_roots(FrontierArgs a) {
  const int lane = threadIdx.x & 63;
  const uint32_t jj = blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = jj < a.n_chunk;
  FQInfo q{};
  int64_t win = 0;
  if (act) {
    q = a.qi[jj];
    win = q.hi - q.lo + 1;
    if (win < 0) win = 0;
  }
  const int steps = wave_max_i((int)win);
  FGroup* G = (FGroup*)a.gtab;
  FCand<KW>* C = (FCand<KW>*)a.ctab;
  const int top = (int)q.K - 1;
  const uint32_t rtop = act && top >= 0 ? a.qrow[(size_t)jj * 128 + top] : 0u;
  for (int s = 0; s < steps; ++s) {
    const int64_t v = q.lo + s;
    bool pred = act && s < win && v >= 1 && top >= 0 && (int)a.lr[q.lr_off + v] <= top;
    bool fresh = false;
    uint32_t gs = 0;
    if (pred) {
      gs = group_get(G, a.gmask, fkey(ftagb(a, 0), jj, (uint32_t)v, 0), fresh);
      if (gs == UINT32_MAX) {
        set_overflow(a, 2);
        pred = false;
        fresh = false;
      } else {
        atomicOr((unsigned long long*)&G[gs].mask[top >> 6], 1ull << (top & 63));
      }
    }
    const uint64_t bm = __ballot(fresh);
    if (bm) {
      const int leader = __builtin_ctzll(bm);
      uint32_t b0 = 0;
      if (lane == leader) b0 = atomicAdd(&a.ctl->list_cnt[0], (uint32_t)__builtin_popcountll(bm));
      b0 = __shfl(b0, leader, 64);
      if (fresh) {
        const uint32_t at = b0 + (uint32_t)__builtin_popcountll(bm & lanemask_lt());
        if (at > a.gmask) set_overflow(a, 4);
        else a.glist[at] = gs;
      }
    }
    if (pred) {
      const uint32_t cs = cand_put<KW>(C, a.cmask, fkey(ftagb(a, 0), jj, (uint32_t)v, (uint32_t)top));
      if (cs == UINT32_MAX) {
        set_overflow(a, 2);
      } else {
        FCand<KW>& e = C[cs];
        e.parent = kRootBit | (uint32_t)(jj * a.rstride + s);
        a.root_node[(size_t)jj * a.rstride + s] = kRootUnset;  // its value, once band 0's values run
        e.A = (uint8_t)q.A0;
        e.B = (uint8_t)qrow_cap(rtop);
#pragma unroll
        for (int w = 0; w < KW; ++w) e.fk[w] = 0;
        if (a.rb > 0) e.fk[0] = (uint64_t)s << (64 - a.rb);
      }
    }
  }
}

// Band b in two launches.  Within a group (query, mass) the up move keeps
// the path's key, so the first visit of rank k is the smallest left candidate
// at ranks k .. hv: FV(m, k) = min_{j >= k} L_j (the up chain carries the
// winner down; its budgets: A from the winning candidate, B = cap[k] unless
// the winner is rank k's own).  Every node of the band is then independent:
//   k_lbf_groups  a lane per group: the group's entry (its masks consumed),
//                 lo, node ids (ranks lo .. hv ascending), node -> group and
//                 each node's flags (a rank below it, a candidate of its own)
//   k_lbf_nodes   a lane per node: its own rank's candidate from the hash
//                 (and its parent's child link), its first visit as a
//                 segmented suffix min over the group, the left attempt
//                 (mass_table.py:424-441), the left child's group and
//                 candidate in the band it falls in
template <int KW>
struct FCRec {  // a group's left candidate, copied for the node lanes
  uint64_t fk[KW];
  uint8_t A, B, rank, pad[5];
};
struct FGRec {
  uint32_t base;   // node id of rank lo
  uint32_t j;      // listed query (chunk index)
  uint32_t m;      // mass
  uint32_t cbase;  // its first candidate record (ranks descending)
  uint8_t lo, hv, nc, pad;
};

template <int KW>
__global__ __launch_bounds__(256) void k_lbf_groups(FrontierArgs a, int band) {
  __shared__ uint32_t s_ovf;  // one reading for the workgroup: its barriers below need every wave
  if (threadIdx.x == 0) s_ovf = __hip_atomic_load(&a.ctl->overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (s_ovf) return;
  const int lane = threadIdx.x & 63;
  const uint32_t slot = (uint32_t)band & ((uint32_t)a.ring - 1u);
  const uint32_t ng = a.ctl->list_cnt[slot];
  if (blockIdx.x == 0 && threadIdx.x == 0) a.band_groups[band] = ng;
  if (ng > a.grec_cap) {
    if (blockIdx.x == 0 && threadIdx.x == 0) set_overflow(a, 4);
    return;
  }
  const size_t gstride = (size_t)a.gmask + 1;
  FGroup* G = (FGroup*)a.gtab + slot * gstride;
  const uint32_t* Lst = a.glist + slot * gstride;
  FGRec* GR = (FGRec*)a.grec;
  const uint32_t band0 = a.band_start[band];
  __shared__ uint32_t s_tot[4], s_base;
  const int wib = (int)(threadIdx.x >> 6);
  for (uint32_t bbase = blockIdx.x * 256u; bbase < ng; bbase += gridDim.x * 256u) {  // block-uniform trips
    const uint32_t base = bbase + (uint32_t)wib * 64u;
    const uint32_t gi = base + lane;
    const bool act = gi < ng;
    uint32_t jj = 0, m = 0, n = 0, nc = 0;
    int hv = 0, lo = 0;
    uint64_t mk0 = 0, mk1 = 0;
    if (act) {
      const uint32_t gs = Lst[gi];
      const FGroup g = G[gs];
      G[gs].mask[0] = 0;  // consumed: the slot's next band starts from empty masks
      G[gs].mask[1] = 0;
      jj = (uint32_t)(g.key >> 32) & 0xFFFFFu;
      m = (uint32_t)(g.key >> 7) & 0x1FFFFFFu;
      mk0 = g.mask[0];
      mk1 = g.mask[1];
      hv = mk1 ? 127 - __builtin_clzll(mk1) : 63 - __builtin_clzll(mk0 | 1ull);
      lo = a.lr[a.qi[jj].lr_off + m];
      if (hv < lo || !(mk0 | mk1)) set_overflow(a, 8);  // cannot happen: a candidate's mass is in R_hv
      else n = (uint32_t)(hv - lo + 1);
      nc = (uint32_t)(__builtin_popcountll(mk0) + __builtin_popcountll(mk1));
    }
    // node ids: one atomic per workgroup (the waves' totals through LDS)
    const uint32_t incl = wave_incl_u(n), total = __shfl(incl, 63, 64);
    if (lane == 0) s_tot[wib] = total;
    __syncthreads();
    const uint32_t btotal = s_tot[0] + s_tot[1] + s_tot[2] + s_tot[3];
    if (threadIdx.x == 0) s_base = atomicAdd(&a.ctl->node_ctr, btotal);
    __syncthreads();
    const uint32_t bstart = s_base;
    uint32_t wbase = bstart;
    for (int w = 0; w < wib; ++w) wbase += s_tot[w];
    __syncthreads();  // the next trip rewrites s_tot / s_base
    if ((uint64_t)bstart + btotal > a.ncap || (uint64_t)bstart + btotal - band0 > a.ngrp_cap) {
      if (threadIdx.x == 0) set_overflow(a, 1);
      return;  // the whole workgroup
    }
    const uint32_t id0 = wbase + incl - n;
    {  // per-query node counts: one atomic per run of one query's groups in the wave
      // (a chunk of few queries otherwise sends every group's add to the same word)
      const uint32_t jprev = __shfl_up(jj, 1, 64), jnext = __shfl_down(jj, 1, 64);  // every lane shuffles
      const bool head = lane == 0 || jprev != jj;
      const bool tail = lane == 63 || jnext != jj;
      int seg = head ? lane : 0;
      uint32_t run = n;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int ps = __shfl_up(seg, d, 64);
        if (lane >= d && ps > seg) seg = ps;
      }
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(run, d, 64);
        if (lane - d >= seg) run += y;
      }
      if (tail && run) atomicAdd(&a.node_cnt[jj], run);
    }
    if (act) {
      FGRec r;
      r.base = id0;
      r.j = jj;
      r.m = m;
      r.cbase = 0;  // (candidates are read from the hash by the node pass)
      r.lo = (uint8_t)lo;
      r.hv = (uint8_t)hv;
      r.nc = (uint8_t)nc;
      r.pad = 0;
      GR[gi] = r;
    }
    // node -> group, the wave's nodes 64 at a time (ids are the wave's
    // items in lane order: coalesced, no lane waits for the largest group)
    for (uint32_t q0 = 0; q0 < total; q0 += 64u) {
      const uint32_t q = q0 + (uint32_t)lane;
      const int g = wave_owner(incl, q);
      const uint32_t gfirst = __shfl(incl - n, g, 64), glo = __shfl((uint32_t)lo, g, 64);
      const uint64_t h0 = __shfl(mk0, g, 64), h1 = __shfl(mk1, g, 64);
      if (q < total) {
        a.node_group[wbase - band0 + q] = base + (uint32_t)g;
        const uint32_t k = glo + (q - gfirst);  // its rank: a candidate of its own at rank k, a node below it
        const bool has = ((k >= 64 ? h1 : h0) >> (k & 63)) & 1ull;
        a.flags[wbase + q] = (uint8_t)((k > glo ? kFUp : 0) | (has ? kFCand : 0));
      }
    }
  }
}

// the first group start (a node without kFUp) at or after x0 in [x0, s1], 64
// flags per step
__device__ __forceinline__ uint32_t next_group_start(const FrontierArgs& a, uint32_t x0, uint32_t s1) {
  const int lane = threadIdx.x & 63;
  for (uint32_t y = x0; y < s1; y += 64u) {
    const uint32_t x = y + (uint32_t)lane;
    const uint64_t b = __ballot(x >= s1 || !(a.flags[x] & kFUp));
    if (b) return y + (uint32_t)__builtin_ctzll(b);
  }
  return s1;
}

template <int KW>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_lbf_nodes(FrontierArgs a, int band) {
  if (__hip_atomic_load(&a.ctl->overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const int lane = threadIdx.x & 63;
  const uint32_t rmask = (uint32_t)a.ring - 1u;
  const uint32_t band0 = a.band_start[band];
  const uint32_t nn = a.ctl->node_ctr - band0;  // this band's nodes (k_lbf_groups allocated them)
  const size_t gstride = (size_t)a.gmask + 1, cstride = (size_t)a.cmask + 1;
  const FGRec* GR = (const FGRec*)a.grec;
  const FCand<KW>* Cb = (const FCand<KW>*)a.ctab + ((uint32_t)band & rmask) * cstride;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
  // a wave takes a range of whole groups and runs it 64 nodes at a time from
  // the top: a node's first visit is the smallest candidate at its rank or
  // above in its group -- a segmented suffix min over consecutive ids, each
  // lane loading only its own rank's candidate record; the group open at a
  // step's top carried from the step above
  // (ranges of kNodeSeg ids, taken from a ticket, moved to group starts)
  const uint32_t e_all = band0 + nn, nseg = (nn + kNodeSeg - 1u) / kNodeSeg;
  __shared__ uint32_t s_fresh[4][2][kFreshBuf];  // per wave: the range's fresh groups of bands b+1, b+2
  const int wib = (int)(threadIdx.x >> 6);
  uint32_t next = wave;  // the first range: the wave's own; later ones from the ticket, past the grid's
  for (;;) {
  uint32_t nf0 = 0, nf1 = 0;  // (wave-uniform) fresh groups buffered per band
  const uint32_t sg = next;
  if (sg >= nseg) break;  // (a wave past a small band's ranges leaves without touching the ticket)
  const uint32_t r0 = sg ? next_group_start(a, band0 + sg * kNodeSeg, e_all) : band0;
  const uint32_t r1 = sg + 1u >= nseg ? e_all : next_group_start(a, band0 + (sg + 1u) * kNodeSeg, e_all);
  uint64_t cy_key[KW];
#pragma unroll
  for (int w = 0; w < KW; ++w) cy_key[w] = ~0ull;
  int cy_A = 0, cy_B = 0, cy_win = -1;
  for (uint32_t c1 = r1; c1 > r0;) {
    const uint32_t c0 = c1 - r0 > 64u ? c1 - 64u : r0;
    const uint32_t id = c0 + (uint32_t)lane;
    const bool live = id < c1;
    const uint32_t x = id - band0;
    c1 = c0;
    uint32_t jj = 0, m = 0;
    int k = 0, lo = 0, hv = 0;
    uint32_t rw = 0;
    uint8_t f0 = 0;
    FQInfo q{};
    if (live) {
      f0 = a.flags[id];
      const FGRec r = GR[a.node_group[x]];
      jj = r.j;
      m = r.m;
      lo = r.lo;
      hv = r.hv;
      k = lo + (int)(id - r.base);
      q = a.qi[jj];
      rw = a.qrow[(size_t)jj * 128 + k];
    }
    // the left child's lowest-rank byte, loaded now (before this rank's
    // candidate and the wave's scans) so the two random lines are in flight
    // together; only the budget test (rarely false) could have spared it
    const int64_t m2e = (int64_t)m - qrow_w(rw);
    const int lrv = live && m2e > 0 ? (int)a.lr[q.lr_off + m2e] : 0;
    const bool has = live && (f0 & kFCand);
    // the first group top (highest rank) at or above this lane; 64: the
    // group continues past the step's top (dead lanes -- above a partial
    // bottom step -- end nothing and add nothing)
    int se = (live && k == hv) ? lane : 64;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int o = __shfl_down(se, d, 64);
      if (lane + d < 64 && o < se) se = o;
    }
    const bool open = se == 64;
    const int lim = open ? 63 : se;
    uint64_t key[KW];
#pragma unroll
    for (int w = 0; w < KW; ++w) key[w] = ~0ull;
    int A = 0, B = 0, win = -1;
    bool hpar = false;  // a left parent (or a root slot): its id to lpar (this node's own slot), the value pushed later
    if (has) {  // this rank's own candidate, straight from the hash
      const uint32_t cs = cand_find<KW>(Cb, a.cmask, fkey(ftagb(a, (uint32_t)band), jj, m, (uint32_t)k));
      if (cs == UINT32_MAX) {
        set_overflow(a, 16);  // cannot happen: the mask bit follows the insertion
      } else {
        const FCand<KW>& c = Cb[cs];
#pragma unroll
        for (int w = 0; w < KW; ++w) key[w] = c.fk[w];
        A = c.A;
        B = c.B;
        win = k;
        a.lpar[id] = c.parent;
        hpar = true;
      }
    }
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      uint64_t ok[KW];
#pragma unroll
      for (int w = 0; w < KW; ++w) ok[w] = __shfl_down(key[w], d, 64);
      const int oA = __shfl_down(A, d, 64), oB = __shfl_down(B, d, 64), ow = __shfl_down(win, d, 64);
      if (lane + d <= lim && ow >= 0 && (win < 0 || key_less<KW>(ok, key))) {
#pragma unroll
        for (int w = 0; w < KW; ++w) key[w] = ok[w];
        A = oA;
        B = oB;
        win = ow;
      }
    }
    if (open && cy_win >= 0 && (win < 0 || key_less<KW>(cy_key, key))) {
#pragma unroll
      for (int w = 0; w < KW; ++w) key[w] = cy_key[w];
      A = cy_A;
      B = cy_B;
      win = cy_win;
    }
    // the step below continues lane 0's group unless lane 0 is its lowest rank
    if (__shfl(k > lo ? 1 : 0, 0, 64)) {
#pragma unroll
      for (int w = 0; w < KW; ++w) cy_key[w] = __shfl(key[w], 0, 64);
      cy_A = __shfl(A, 0, 64);
      cy_B = __shfl(B, 0, 64);
      cy_win = __shfl(win, 0, 64);
    } else {
#pragma unroll
      for (int w = 0; w < KW; ++w) cy_key[w] = ~0ull;
      cy_A = cy_B = 0;
      cy_win = -1;
    }
    if (live) {
      if (win < 0) set_overflow(a, 8);  // cannot happen: the group's top rank holds a candidate
      if (win != k) B = qrow_cap(rw);  // reached by the up chain: B = cap of this row (mass_table.py:411-420)
    }
    const int64_t wk = qrow_w(rw);
    const bool mod = qrow_mod(rw);
    // the left branch (mass_table.py:424-441): attempted iff bit1 (m - w_k in
    // R_k, the lowest-rank byte loaded above) and the budgets allow it
    const int64_t m2 = (int64_t)m - wk;
    const bool bud = !mod || (A > 0 && B > 0);
    const bool latt = live && bud && m2 >= 0 && (m2 == 0 || lrv <= k);
    if (live)
      a.flags[id] = (uint8_t)((latt ? kFLeft : 0) | (k > lo ? kFUp : 0) | (latt && m2 == 0 ? kFZero : 0) |
                              (hpar ? kFPar : 0));
    bool emit = latt && m2 > 0;
    const uint32_t band2 = emit ? (uint32_t)((q.hi - m2) / a.wb) : 0u;
    const uint32_t slot2 = band2 & rmask;
    uint32_t gs2 = 0;
    bool fresh = false;
    if (emit) {
      FGroup* G2 = (FGroup*)a.gtab + slot2 * gstride;
      gs2 = group_get(G2, a.gmask, fkey(ftagb(a, band2), jj, (uint32_t)m2, 0), fresh);
      if (gs2 == UINT32_MAX) {
        set_overflow(a, 2);
        emit = false;
        fresh = false;
      } else {
        atomicOr((unsigned long long*)&G2[gs2].mask[k >> 6], 1ull << (k & 63));
      }
    }
    for (int d = 1; d <= a.jump; ++d) {  // fresh groups join their band's list
      const bool pd = fresh && band2 == (uint32_t)band + (uint32_t)d;
      const uint64_t bm = __ballot(pd);
      if (bm && d <= 2) {  // buffered for the range: one atomic per range and band
        uint32_t& nf = d == 1 ? nf0 : nf1;
        const uint32_t at = nf + (uint32_t)__builtin_popcountll(bm & lanemask_lt());
        if (pd) {
          if (at < kFreshBuf) s_fresh[wib][d - 1][at] = gs2;
          else set_overflow(a, 4);  // cannot happen: a range holds < kFreshBuf nodes
        }
        nf += (uint32_t)__builtin_popcountll(bm);
      } else if (bm) {
        const int leader = __builtin_ctzll(bm);
        const uint32_t sl = ((uint32_t)band + (uint32_t)d) & rmask;
        uint32_t b0 = 0;
        if (lane == leader) b0 = atomicAdd(&a.ctl->list_cnt[sl], (uint32_t)__builtin_popcountll(bm));
        b0 = __shfl(b0, leader, 64);
        if (pd) {
          const uint32_t at = b0 + (uint32_t)__builtin_popcountll(bm & lanemask_lt());
          if (at > a.gmask) set_overflow(a, 4);
          else a.glist[sl * gstride + at] = gs2;
        }
      }
    }
    if (emit) {
      FCand<KW>* C2 = (FCand<KW>*)a.ctab + slot2 * cstride;
      const uint32_t cs = cand_put<KW>(C2, a.cmask, fkey(ftagb(a, band2), jj, (uint32_t)m2, (uint32_t)k));
      if (cs == UINT32_MAX) {
        set_overflow(a, 2);
      } else {
        uint64_t k2[KW];
#pragma unroll
        for (int w = 0; w < KW; ++w) k2[w] = key[w];
        key_set_msb<KW>(k2, a.rb + key_ones<KW>(key, a.rb) + ((int)q.K - 1 - k));
        FCand<KW>& e = C2[cs];
        e.parent = id;
        e.A = (uint8_t)(mod ? A - 1 : A);
        e.B = (uint8_t)(mod ? B - 1 : B);
#pragma unroll
        for (int w = 0; w < KW; ++w) e.fk[w] = k2[w];
      }
    }
  }
  // the range's fresh groups into their bands' lists
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  for (int d = 1; d <= 2; ++d) {
    const uint32_t nf = d == 1 ? nf0 : nf1;
    if (!nf) continue;
    const uint32_t sl = ((uint32_t)band + (uint32_t)d) & rmask;
    uint32_t b0 = 0;
    if (lane == 0) b0 = atomicAdd(&a.ctl->list_cnt[sl], nf);
    b0 = __shfl(b0, 0, 64);
    for (uint32_t t = (uint32_t)lane; t < nf && t < kFreshBuf; t += 64u) {
      const uint32_t at = b0 + t;
      if (at > a.gmask) set_overflow(a, 4);
      else a.glist[sl * gstride + at] = s_fresh[wib][d - 1][t];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // the buffer is refilled by the next range
  if (lane == 0) next = nwaves + atomicAdd(&a.ctl->node_ticket, 1u);
  next = __shfl(next, 0, 64);
  }
}

// between bands: record where band b's nodes start; free the list slot the
// next band's heaviest children will fill
__global__ void k_lbf_mark(FrontierArgs a, int band) {
  a.band_start[band] = a.ctl->node_ctr;
  a.ctl->crec_ctr = 0;  // the candidate records are per band
  a.ctl->list_cnt[((uint32_t)band + (uint32_t)a.jump) & ((uint32_t)a.ring - 1u)] = 0;
  a.ctl->node_ticket = 0;
}

// the memoised values of band b's nodes (mass_table.py:407-457).  Within a
// group (ranks ascending) a node's values fold its left branch into the node
// below's: lower = min, upper = max over the group's ranks up to it -- a
// segmented prefix min / max over consecutive node ids.  A wave takes a range
// of whole groups and runs it 64 nodes at a time (a lane per node; the group
// open at a step's start carried from the step before); lower with 255 as "no
// path" (min(default, x) at the roots), upper from -1.  A node's left child
// pushed its value into the node's lval slot when the child's (later) band
// ran, so the node reads its own slot; it pushes its own value to its left
// parent the same way (one random write per edge instead of the parent's
// random read of the child's value and the child's random write of a link).
__global__ __launch_bounds__(256) void k_lbf_values(FrontierArgs a, int band) {
  if (__hip_atomic_load(&a.ctl->overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const int lane = threadIdx.x & 63;
  const uint32_t s0 = a.band_start[band], s1 = a.band_start[band + 1];
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
  const uint32_t nn = s1 - s0;
  const uint32_t per = ((nn + nwaves - 1u) / nwaves + 63u) & ~63u;
  const uint64_t b0 = (uint64_t)wave * per, b1 = b0 + per;
  if (b0 >= nn) return;
  // whole groups: both ends moved to the next group start (the neighbours
  // compute the same boundary)
  const uint32_t r0 = wave ? next_group_start(a, s0 + (uint32_t)b0, s1) : s0;
  const uint32_t r1 = b1 >= nn ? s1 : next_group_start(a, s0 + (uint32_t)b1, s1);
  const uint64_t le = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
  int clo = 255, chi = -1;  // the values of the group open at the step's start
  uint32_t n_edges = 0;     // (wave-uniform) left moves onto a mass > 0: the run's edge count
  for (uint32_t c0 = r0; c0 < r1; c0 += 64u) {
    const uint32_t x = c0 + (uint32_t)lane;
    const bool live = x < r1;
    const uint8_t f = live ? a.flags[x] : (uint8_t)0;
    const uint32_t par = (f & kFPar) ? a.lpar[x] : 0u;
    n_edges += (uint32_t)__builtin_popcountll(__ballot((f & kFLeft) && !(f & kFZero)));
    int vl = 255, vh = -1;
    if (f & kFLeft) {
      vl = 1;  // a left move onto mass 0: 0 + 1
      vh = 1;
      if (!(f & kFZero)) {
        const uint32_t p = a.lval[x];  // the left child's value, pushed by the child's band
        const int l = (int)(p & 0xFFu) + 1;
        vl = l > 255 ? 255 : l;
        vh = (int)(p >> 8);  // upper + 1: -1 + 1 = 0 (the reference's default feeds the max)
      }
    }
    // segmented inclusive min / max: a segment starts at each group's lowest rank
    const bool head = live && !(f & kFUp);
    int seg = head ? lane : 0;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int ps = __shfl_up(seg, d, 64);
      if (lane >= d && ps > seg) seg = ps;
    }
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int yl = __shfl_up(vl, d, 64), yh = __shfl_up(vh, d, 64);
      if (lane - d >= seg) {
        vl = yl < vl ? yl : vl;
        vh = yh > vh ? yh : vh;
      }
    }
    if (!(__ballot(head) & le)) {  // still in the group open at the step's start
      vl = clo < vl ? clo : vl;
      vh = chi > vh ? chi : vh;
    }
    const uint16_t pk = (uint16_t)(vl | ((vh + 1) << 8));
    if (f & kFPar) {  // to the left parent, in an earlier band (a heavier mass) whose run comes later, or the root slot
      if (par & kRootBit) a.root_node[par & ~kRootBit] = pk;
      else if (par >= s0) set_overflow(a, 32);  // cannot happen
      else a.lval[par] = pk;
    }
    const int last = r1 - c0 >= 64u ? 63 : (int)(r1 - c0 - 1u);
    clo = __shfl(vl, last, 64);
    chi = __shfl(vh, last, 64);
  }
  if (lane == 0 && n_edges) atomicAdd((unsigned long long*)&a.ctl->edges, (unsigned long long)n_edges);
}

// per query: min / max over the window's roots (mass_table.py:459-487)
__global__ __launch_bounds__(256) void k_lbf_out(FrontierArgs a) {
  const uint32_t jj = blockIdx.x * blockDim.x + threadIdx.x;
  if (jj >= a.n_chunk) return;
  const FQInfo q = a.qi[jj];
  const bool bad = __hip_atomic_load(&a.ctl->overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  if (bad) return;  // the host splits the chunk and runs it again
  if (q.pad & 1) return;  // excluded by k_lbf_setup (SST_ABORTED already written)
  const int dl = (int)q.L + 1;
  int bl = dl, bh = -1;
  if (q.lo <= 0 && q.hi >= 0) {  // total_mass == 0 -> 0
    bl = 0 < bl ? 0 : bl;
    bh = 0 > bh ? 0 : bh;
  }
  const int top = (int)q.K - 1;
  for (int64_t v = q.lo < 1 ? 1 : q.lo; v <= q.hi; ++v) {
    if (top < 0 || (int)a.lr[q.lr_off + v] > top) continue;  // pair(top, v) == 0: the default
    const uint32_t p = a.root_node[(size_t)jj * a.rstride + (size_t)(v - q.lo)];  // the root's value
    if (p == kRootUnset) {  // cannot happen: every reachable root is a band-0 node
      set_overflow(a, 32);
      return;
    }
    const int l = (int)(p & 0xFFu), h = (int)(p >> 8) - 1;
    bl = l < bl ? l : bl;
    bh = h > bh ? h : bh;
  }
  if (a.nodes_out) a.nodes_out[q.i] += a.node_cnt[jj];
  a.lower[q.i] = bl >= dl ? 1 : bl;  // the default becomes 1 / max_len (:476-484)
  a.upper[q.i] = bh == -1 ? (int64_t)q.L : bh;
  a.status[q.i] = 0;
}

// the lowest kept rank reaching each mass, from sst_reach_rows' row bitsets
__global__ __launch_bounds__(256) void k_reach_lowest(ReachArgs r, const uint64_t* lr_off, uint8_t* lr) {
  for (int64_t g = blockIdx.y; g < r.n_spec; g += gridDim.y) {
    const uint64_t m0 = r.alpha[2 * g], m1 = r.alpha[2 * g + 1];
    int K = 0;
    for (int row = 1; row < r.n_rows; ++row) K += row < 64 ? (int)((m0 >> row) & 1ull) : (int)((m1 >> (row - 64)) & 1ull);
    const int64_t W = r.words[g];
    const uint32_t* bits = r.bits + r.off[g];
    uint4* out = (uint4*)(lr + lr_off[g]);
    for (int64_t jw = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; jw < W; jw += (int64_t)gridDim.x * blockDim.x) {
      uint32_t o[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = 0xFFFFFFFFu;
      uint32_t acc = 0;
      for (int k = 0; k < K && acc != 0xFFFFFFFFu; ++k) {
        const uint32_t x = bits[(int64_t)k * W + jw];
        const uint32_t nw = x & ~acc;
        if (!nw) continue;
        acc |= x;
        const uint32_t kk = (uint32_t)k * 0x01010101u;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const uint32_t nib = (nw >> (4 * q)) & 0xFu;
          const uint32_t bm = ((nib & 1u) ? 0xFFu : 0u) | ((nib & 2u) ? 0xFF00u : 0u) | ((nib & 4u) ? 0xFF0000u : 0u) |
                              ((nib & 8u) ? 0xFF000000u : 0u);
          o[q] = (o[q] & ~bm) | (kk & bm);
        }
      }
      out[2 * jw] = make_uint4(o[0], o[1], o[2], o[3]);
      out[2 * jw + 1] = make_uint4(o[4], o[5], o[6], o[7]);
    }
  }
}

hipError_t launch_reach_lowest(const ReachArgs& r, const uint64_t* lr_off, uint8_t* lr, hipStream_t st) {
  if (r.n_spec <= 0) return hipSuccess;
  const int gy = (int)(r.n_spec < 65535 ? r.n_spec : 65535);
  hipLaunchKernelGGL(k_reach_lowest, dim3(16, gy), dim3(256), 0, st, r, lr_off, lr);
  return hipGetLastError();
}

hipError_t launch_lbf_setup(const TableArgs& t, const FrontierArgs& a, hipStream_t st) {
  const uint32_t blocks = (a.n_chunk + 3) / 4;  // four 64-lane waves per block
  hipLaunchKernelGGL(k_lbf_setup, dim3(blocks), dim3(256), 0, st, t, a);
  return hipGetLastError();
}

template <int KW>
static hipError_t sweep(const FrontierArgs& a, int n_bands, int band_blocks, hipStream_t st) {
  hipLaunchKernelGGL(k_lbf_roots<KW>, dim3((a.n_chunk + 255) / 256), dim3(256), 0, st, a);
  for (int b = 0; b < n_bands; ++b) {
    hipLaunchKernelGGL(k_lbf_mark, dim3(1), dim3(1), 0, st, a, b);
    hipLaunchKernelGGL(k_lbf_groups<KW>, dim3(band_blocks), dim3(256), 0, st, a, b);
    hipLaunchKernelGGL(k_lbf_nodes<KW>, dim3(band_blocks), dim3(256), 0, st, a, b);
  }
  hipLaunchKernelGGL(k_lbf_mark, dim3(1), dim3(1), 0, st, a, n_bands);
  for (int b = n_bands - 1; b >= 0; --b) hipLaunchKernelGGL(k_lbf_values, dim3(band_blocks), dim3(256), 0, st, a, b);
  hipLaunchKernelGGL(k_lbf_out, dim3((a.n_chunk + 255) / 256), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_lbf_sweep(const FrontierArgs& a, int key_words, int n_bands, int band_blocks, hipStream_t st) {
  switch (key_words) {
    case 4: return sweep<4>(a, n_bands, band_blocks, st);
    case 1: return sweep<1>(a, n_bands, band_blocks, st);
    case 2: return sweep<2>(a, n_bands, band_blocks, st);
    default: return hipErrorInvalidValue;
  }
}

size_t lbf_cand_bytes(int key_words) {
  switch (key_words) {
    case 1: return sizeof(FCand<1>);
    case 2: return sizeof(FCand<2>);
    default: return sizeof(FCand<4>);
  }
}
size_t lbf_group_bytes() { return sizeof(FGroup); }
size_t lbf_grec_bytes() { return sizeof(FGRec); }
size_t lbf_crec_bytes(int key_words) {
  switch (key_words) {
    case 1: return sizeof(FCRec<1>);
    case 2: return sizeof(FCRec<2>);
    default: return sizeof(FCRec<4>);
  }
}

}  // namespace sst
