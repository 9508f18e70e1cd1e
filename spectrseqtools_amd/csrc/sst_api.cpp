// sst_api.cpp -- host side of libsstgpu.so: contexts, device tables, batch
// launches and the extern "C" ABI declared in include/sst.h.
//
// No CPU compute path exists here: every table build, index derivation and
// query runs in the HIP kernels of sst_kernels.hip.  The host only moves
// buffers, sizes workspaces and retries the rare batches whose outputs did not
// fit the first arena / hash sizing.
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "sst.h"
#include "sst_internal.h"
#include "sst_pyset.h"

using namespace sst;

namespace {

struct DevBuf {  // owns one device allocation (freed on release or destruction)
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), bytes(o.bytes) {
    o.p = nullptr;
    o.bytes = 0;
  }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) {
      release();
      p = o.p;
      bytes = o.bytes;
      o.p = nullptr;
      o.bytes = 0;
    }
    return *this;
  }
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  // grow-only reallocation; returns false on OOM
  bool ensure(size_t n) {
    if (n <= bytes) return true;
    release();
    if (n == 0) return true;
    if (hipMalloc(&p, n) != hipSuccess) {
      (void)hipGetLastError();
      p = nullptr;
      return false;
    }
    bytes = n;
    return true;
  }
};

}  // namespace

struct sst_ctx {
  int device = 0;
  hipStream_t stream = nullptr;  // where work is queued: `own`, or the caller's (sst_ctx_set_stream)
  hipStream_t own = nullptr;
  std::string err;
  std::recursive_mutex mu;
  // staging for host-pointer calls
  DevBuf in_mass, in_thr, in_mods, out_valid;
  // persistent workspaces of the deferred explain kernels
  DevBuf ws_deep;
  DevBuf ws_hash, ws_frames, ws_stacks, ws_epochs;
  DevBuf singleton_masses;  // sorted, de-duplicated integer masses of the last is_singleton call
  // the first-visit frontier's workspace (sst_length_bounds_frontier_device):
  // kept across calls (a config-5 run makes one call per batch of alphabets;
  // allocating tens of GB per call costs seconds), with its hash epoch and the
  // memo entries per query seen so far (the next call's first chunk size)
  struct LbfWs {
    DevBuf flags, lpar, lval, gtab, ctab, glist, ctl, bstart, bgroups, qi, qrow, roots, ncnt, grec, crec, ngrp;
    uint64_t S = 0, ncap = 0, budget = 0;
    bool by_default = false;
    int epoch = 0;
    bool dirty = true;
    uint64_t done_q = 0, done_nodes = 0;
    double band_frac = 0.3;  // the largest band's share of a chunk's nodes seen so far
  } lbf, lbf_small;  // lbf_small: sst_length_bound_batch's (one table, few queries; 4 GB)
  uint32_t hash_cap = 0;
  int exact_blocks = 0;
  int n_cu = 256;       // compute units (persistent grid sizing)
  int expand_blocks = 0;  // resident workgroups of k_explain_expand
  // measurement: hipEvents around launches on `stream`
  uint32_t prof = 0;  // kernel ids whose launches are bracketed by events
  struct Pending {
    int kid;
    hipEvent_t a, b;
  };
  std::vector<Pending> pending;
  std::vector<hipEvent_t> pool;
  double prof_ms[SST_K_COUNT] = {0};
  int64_t prof_n[SST_K_COUNT] = {0};
  uint32_t prof_every = 1;                // bracket every n-th launch of a selected kernel
  uint64_t prof_seen[SST_K_COUNT] = {0};  // launches of each kernel id since selection
  // the pipeline's big-spectrum slices (sst_pipe_reserve_rows, pipe_big_layout)
  DevBuf pipe_big;
  uint32_t pipe_big_rows = 0, pipe_big_slots = 0;
  int pipe_big_wg = 0;
};

struct sst_table {
  sst_ctx* ctx = nullptr;
  int n_rows = 0;
  int64_t n_cols = 0;
  int C = 32;
  int64_t M = 0;
  std::vector<int64_t> masses;
  std::vector<uint8_t> is_mod;
  std::vector<int64_t> cap;
  DevBuf packed, index, valid, w, capd, modd, pairs, census, canon_c;
  int64_t canon_c_words = 0;  // the canonical rows' closure (k_valid_alpha), built at first use
  std::vector<uint32_t> pair_recs;  // the pair list's payload records (host copy)
  uint64_t pair_key = 0;            // their FNV-1a (sst_wire_pack), computed on first use
  bool pair_key_set = false;
  int scan_blocks = 0;  // resident workgroups of k_explain_scan (depends on the LDS pair list size)
  bool closure = false;  // built here from masses >= C: rows are true closures (layered fast paths valid)
  TableArgs args{};
};

// per-query budgets of an explain pass (QueryArgs::qlen ...): query i's caps
// row qlen[i] of the tables
struct LenBudgets {
  const int32_t* qlen = nullptr;
  const int32_t* caps = nullptr;
  const uint64_t* capz = nullptr;
  const uint32_t* never = nullptr;
};

struct sst_result {
  sst_ctx* ctx = nullptr;
  int64_t n = 0;
  int64_t cap_n = 0;
  // the result a consumer reads (include/sst.h): status[n], the dense hit
  // list and the dense payload, all written on the device by the pass
  DevBuf status, hits, dense;
  // pass workspaces: the arena (scan-wave regions + spill area), control
  // blocks, class lists, scan worklists / hit records, tallies, deferred hits
  DevBuf payload, ctl, lists, wave_stats, work, work_count, tally, wg_tally, dhits, hdr, agg, refs, stage;
  DevBuf count, offset;  // per-query arrays: only built for sst_result_device callers that ask for them
  DevBuf lb_caps, lb_capz, lb_never;  // per-query budgets' tables (sst_explain_alpha_lens_batch_device)
  uint64_t* hdr_host = nullptr;  // host-mapped copy of the pack kernel's header (host address)
  uint64_t* hdr_host_dev = nullptr;  // its device address
  // control block (spill cursor, class counters, stats) of the current pass;
  // two of them: each pass's scan kernel zeroes the other for the next pass
  // (no memsets between passes)
  int parity = 1;
  bool ctl_ready = false;
  int n_expand_waves = 0;  // waves of k_explain_expand / the SHALLOW role
  int64_t n_scan_waves = 0;
  int n_wg = 0;             // scan workgroups (= k_result_pack blocks)
  uint64_t work_region = 0;
  uint64_t region_bytes = 0, spill_bytes = 0;
  uint64_t pass_id = 0;
  uint64_t pack_seq = 0;  // k_result_pack launches of this result: the header carries the latest
  uint32_t rows_tile_par = 0;  // the rows step's tile-sum parity of the last launched step (RowsArgs.tile_tot)
  bool tail_ran = false;   // the deferred-class launch ran for the current pass
  bool settled = true;     // the current pass has been checked (routed windows run, retries done)
  bool arrays_ready = false;  // count[] / offset[] built from the hit list for the current pass
  bool bitset_scan = false;   // the pass ran k_bitset_scan + k_explain_expand (tables without the pair list)
  bool fused_pass = false;    // the pass's scan packed its own queries' result (dense records + payload)
  struct {
    sst_table* t;
    const double *mass, *thr;
    const int64_t* mods;
    int64_t mods_scalar;
    double tol, prec;
    int with_memo;
    uint64_t cap;
    const uint64_t* alpha;  // per-query alphabets (sst_explain_alpha_batch_device) or null
    const int32_t* spec;
    LenBudgets lb;          // per-query budgets or none
  } pass{};
  uint64_t arena_bytes = 0;
  uint64_t n_hits = 0, payload_bytes = 0;
  // the fused scan's part of the result (its header): the first scan_hits
  // dense records are pair-path hits with refs[], their payload the first
  // scan_bytes of the dense payload (0 / 0 after an unfused pass)
  bool scan_hdr_pending = false;
  uint64_t scan_hits = 0, scan_bytes = 0;
  // the stream the pass was queued on; settle() queues its own launches
  // there and, when it launched any, records settle_ev after them: later
  // users of the result on another stream (sst_wire_pack on a pack stream,
  // fetch) wait for it
  hipStream_t pass_stream = nullptr;
  hipEvent_t settle_ev = nullptr;
  bool settle_ev_pending = false;
  // the step from the peaks (sst_step_rows_device): its pass writes the dense
  // result in query order and produces its own queries (n from the header)
  bool rows_pass = false;
  DevBuf rows_su, rows_ob, rows_side, rows_tot, rows_chunk, rows_ctl, rows_big, rows_redo, rows_ans, rows_aq;
  std::vector<int8_t> h_status;
  std::vector<uint64_t> h_count, h_offset;
  std::vector<uint8_t> h_payload;
  uint64_t h_stats[kNumStats] = {0};
};

namespace {

int fail(sst_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}
#define HIP_OK(ctx, expr)                                                                        \
  do {                                                                                          \
    hipError_t _e = (expr);                                                                     \
    if (_e != hipSuccess)                                                                       \
      return fail(ctx, SST_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));           \
  } while (0)

int set_device(sst_ctx* c) {
  HIP_OK(c, hipSetDevice(c->device));
  return SST_OK;
}

hipEvent_t take_event(sst_ctx* c) {
  if (!c->pool.empty()) {
    hipEvent_t e = c->pool.back();
    c->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  // timing-only events: no system-scope fence (nothing is handed to the host
  // through them), so a bracket costs the stream less and its start stamp
  // sits closer to the kernel it times
  if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return e;
}

// bracket one launch with events on the ctx stream when profiling is on
struct Prof {
  sst_ctx* c;
  int kid;
  hipEvent_t a = nullptr;
  Prof(sst_ctx* c_, int kid_) : c(c_), kid(kid_) {
    if (((c->prof >> kid) & 1u) && c->prof_seen[kid]++ % c->prof_every == 0 && (a = take_event(c)))
      (void)hipEventRecord(a, c->stream);
  }
  ~Prof() {
    if (!a) return;
    hipEvent_t b = take_event(c);
    if (!b) {
      c->pool.push_back(a);
      return;
    }
    (void)hipEventRecord(b, c->stream);
    c->pending.push_back({kid, a, b});
  }
};

void prof_resolve(sst_ctx* c) {
  for (auto& p : c->pending) {
    float ms = 0.f;
    if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
      c->prof_ms[p.kid] += ms;
      c->prof_n[p.kid] += 1;
    } else {
      (void)hipGetLastError();
    }
    c->pool.push_back(p.a);
    c->pool.push_back(p.b);
  }
  c->pending.clear();
}

uint64_t width_mask(int C) { return C == 32 ? ~0ull : ((1ull << (2 * C)) - 1ull); }

// mass_table.py:246 with numpy shift semantics (shift >= width -> 0)
uint64_t last_col_mask(int64_t max_mass, int64_t ncols, int C) {
  int64_t s = 2 * (ncols - (max_mass + 1) % ncols);
  if (s >= 2 * C || s < 0) return 0;
  return (width_mask(C) << s) & width_mask(C);
}

int64_t table_cols(int64_t max_mass, int C) {
  return (int64_t)std::ceil((double)(max_mass + 1) / (double)C);  // mass_table.py:214
}

// LDS pair list of the scan kernel: every single row mass and every sum of two
// row masses (rows >= 1), sorted by (sum, top row), with a bucket index.  Only
// for tables this library built from exactly these masses: then a window value
// below 3 * w_min is reachable iff it is such a sum, and the reference's DFS
// lists its candidates in (v, top row) order (pair fast path).
// u32 fast-path limits of the scan kernel (TableArgs::never_lim / pair_lim)
void refresh_limits(sst_table* t) {
  TableArgs& a = t->args;
  const int64_t u32max = (int64_t)UINT32_MAX;
  const int64_t nl = !a.any_mod ? u32max : (a.fast_limit_B < 0 ? 0 : std::min(a.fast_limit_B, u32max - 1) + 1);
  a.never_lim = (uint32_t)nl;
  a.pair_lim = (uint32_t)std::min<int64_t>(std::min<int64_t>(a.pair_hi, u32max), nl);
}

int build_pair_list(sst_table* t, bool self_built) {
  sst_ctx* c = t->ctx;
  t->args.pairs_enabled = 0;
  t->args.pair_hi = (int64_t)3 * t->args.w_min;
  // the literal-sweep rows (mass < C) are not a closure, and the last column
  // is masked: keep the pair path to closures strictly below the last column
  if (!self_built || t->args.pair_hi > (t->n_cols - 1) * t->C) return SST_OK;
  for (int r = 1; r < t->n_rows; ++r)
    if (t->masses[r] < t->C) return SST_OK;
  struct E {
    uint32_t sum, rows;
  };
  std::vector<E> e;
  for (int r1 = 1; r1 < t->n_rows; ++r1) {
    if (t->masses[r1] <= 0) return SST_OK;  // zero-mass rows: leave the general path in charge
    // entries carry their payload record serialised: [1][top] or [2][low][top]
    e.push_back({(uint32_t)t->masses[r1], 1u | ((uint32_t)r1 << 8)});
    for (int r2 = 1; r2 <= r1; ++r2) {
      int64_t s = t->masses[r1] + t->masses[r2];
      if (s >= t->args.pair_hi || s >= t->M) continue;  // never inside a pair-class window
      e.push_back({(uint32_t)s, 2u | ((uint32_t)r2 << 8) | ((uint32_t)r1 << 16)});
    }
  }
  // the reference's order: ascending sum, then ascending top row
  auto top = [](const E& x) { return (x.rows & 0xFFu) == 1u ? (x.rows >> 8) & 0xFFu : x.rows >> 16; };
  std::sort(e.begin(), e.end(), [&](const E& x, const E& y) { return x.sum != y.sum ? x.sum < y.sum : top(x) < top(y); });
  // the scan's 8-B hit records carry a window's count and payload bytes (<= 3 per entry + 2) as u16
  if (e.empty() || e.size() > 21000) return SST_OK;
  const size_t n_e = e.size(), n_s = n_e + 2;  // + two sentinels: the walk reads two entries per step
  // Buckets start at w_min (no sum below it) and cover every window start
  // below pair_hi, so a pair-class window needs no bucket bound check; the
  // finest buckets that fit the LDS budget.
  const int64_t base = t->args.w_min, span = t->args.pair_hi - base;
  if (span <= 0) return SST_OK;
  int shift = 4;
  while (shift < 16 && (2 * n_s + (size_t)(((span - 1) >> shift) + 1)) * 4 > (size_t)kMaxPairLds) ++shift;
  const int64_t n_b = ((span - 1) >> shift) + 1;
  if ((2 * n_s + (size_t)n_b) * 4 > (size_t)kMaxPairLds) return SST_OK;
  std::vector<uint32_t> img(2 * n_s + n_b);
  uint32_t* sums = img.data();
  uint32_t* recs = sums + n_s;
  uint32_t* bk = recs + n_s;
  for (size_t k = 0; k < n_e; ++k) {
    sums[k] = e[k].sum << 1 | ((e[k].rows & 0xFFu) == 2u ? 1u : 0u);
    recs[k] = e[k].rows;
  }
  sums[n_e] = sums[n_e + 1] = UINT32_MAX;
  recs[n_e] = recs[n_e + 1] = 0;
  size_t k = 0;
  for (int64_t b = 0; b < n_b; ++b) {
    const int64_t start = base + (b << shift);
    while (k < n_e && (int64_t)e[k].sum < start) ++k;
    const int64_t delta = k < n_e ? std::min<int64_t>((int64_t)e[k].sum - start, 0xFFFF) : 0xFFFF;
    bk[b] = (uint32_t)k | (uint32_t)delta << 16;
  }
  t->pair_recs.assign(recs, recs + n_e);  // host copy (sst_table_pair_records)
  t->args.pair_shift = shift;
  img.resize((img.size() + 3) / 4 * 4, 0u);  // the scan stages it in 16-B pieces
  if (!t->pairs.ensure(img.size() * 4)) return fail(c, SST_E_NOMEM, "device allocation failed (pair list)");
  HIP_OK(c, hipMemcpy(t->pairs.p, img.data(), img.size() * 4, hipMemcpyHostToDevice));
  t->args.pair_data = (const uint32_t*)t->pairs.p;
  t->args.census = nullptr;
  if (t->args.pair_hi - base + 1 <= ((int64_t)1 << 27)) {  // census: entries and record bytes with sum <= x, x in [base - 1, pair_hi)
    std::vector<uint32_t> cen((size_t)(t->args.pair_hi - base + 1));
    uint32_t cnt = 0, bytes = 0;
    size_t j = 0;
    for (size_t x = 0; x < cen.size(); ++x) {
      const int64_t v = base - 1 + (int64_t)x;
      for (; j < n_e && (int64_t)e[j].sum <= v; ++j) {
        ++cnt;
        bytes += (e[j].rows & 0xFFu) == 2u ? 3u : 2u;
      }
      cen[x] = cnt | bytes << 16;
    }
    if (!t->census.ensure(cen.size() * 4)) return fail(c, SST_E_NOMEM, "device allocation failed (pair census)");
    HIP_OK(c, hipMemcpy(t->census.p, cen.data(), cen.size() * 4, hipMemcpyHostToDevice));
    t->args.census = (const uint32_t*)t->census.p;
  }
  t->args.pair_base = (uint32_t)base;
  t->args.n_pairs = (int)n_e;
  t->args.n_buckets = (int)n_b;
  t->args.pairs_enabled = 1;
  return SST_OK;
}

int finish_table(sst_table* t, bool self_built) {
  t->closure = self_built;
  for (int r = 1; r < t->n_rows; ++r)
    if (t->masses[r] < t->C) t->closure = false;  // literal-sweep rows are not closures
  sst_ctx* c = t->ctx;
  const int64_t M = t->M;
  if (!t->index.ensure((size_t)M * sizeof(ulonglong2)) || !t->valid.ensure((size_t)((M + 63) / 64) * 8))
    return fail(c, SST_E_NOMEM, "device allocation failed (index)");
  HIP_OK(c, hipMemsetAsync(t->valid.p, 0, t->valid.bytes, c->stream));
  DevBuf err;
  if (!err.ensure(sizeof(int))) return fail(c, SST_E_NOMEM, "device allocation failed");
  HIP_OK(c, hipMemsetAsync(err.p, 0, sizeof(int), c->stream));
  HIP_OK(c, launch_index(t->C, t->packed.p, t->n_rows, t->n_cols, M, (ulonglong2*)t->index.p, (uint64_t*)t->valid.p,
                         (int*)err.p, c->stream));
  int h_err = 0;
  HIP_OK(c, hipMemcpyAsync(&h_err, err.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIP_OK(c, hipStreamSynchronize(c->stream));
  err.release();
  if (h_err)
    return fail(c, SST_E_TABLE,
                "packed table violates the DP row recurrence (bit0(r,m) != any(r-1,m)); it was not produced by "
                "set_up_bit_table");
  std::vector<int> w32(t->n_rows);
  for (int r = 0; r < t->n_rows; ++r) w32[r] = (int)t->masses[r];
  if (!t->w.ensure(t->n_rows * sizeof(int)) || !t->capd.ensure(t->n_rows * sizeof(int)) ||
      !t->modd.ensure(t->n_rows))
    return fail(c, SST_E_NOMEM, "device allocation failed");
  HIP_OK(c, hipMemcpy(t->w.p, w32.data(), t->n_rows * sizeof(int), hipMemcpyHostToDevice));
  t->args.index = (const ulonglong2*)t->index.p;
  t->args.valid = (const uint64_t*)t->valid.p;
  t->args.limit = M;
  t->args.w = (const int*)t->w.p;
  t->args.n_rows = t->n_rows;
  int wmin = 0;
  for (int r = 1; r < t->n_rows; ++r)
    if (t->masses[r] > 0 && (wmin == 0 || t->masses[r] < wmin)) wmin = (int)t->masses[r];
  t->args.w_min = wmin > 0 ? wmin : 1;
  t->args.shallow_hi = (int64_t)kShallowDepth * t->args.w_min;  // < 4 w_min: at most 3 items
  // longest run of reachable masses (whole bitset words): every window that
  // meets it holds a reachable value (is_valid answers without a bitset load)
  {
    std::vector<uint64_t> vb(t->valid.bytes / 8);
    HIP_OK(c, hipMemcpy(vb.data(), t->valid.p, t->valid.bytes, hipMemcpyDeviceToHost));
    int64_t best_lo = 0, best_len = 0, run_lo = 0;
    for (int64_t k = 0; k <= (int64_t)vb.size(); ++k) {
      if (k < (int64_t)vb.size() && vb[(size_t)k] == ~0ull) continue;
      if (k - run_lo > best_len) {
        best_len = k - run_lo;
        best_lo = run_lo;
      }
      run_lo = k + 1;
    }
    t->args.full_lo = best_len ? best_lo * 64 : 1;
    t->args.full_hi = best_len ? std::min<int64_t>((best_lo + best_len) * 64, M) : 1;  // [full_lo, full_hi)
    // first reachable mass >= 1: windows wholly below it hold no reachable value
    int64_t first = M;
    for (size_t k = 0; k < vb.size() && first == M; ++k) {
      const uint64_t x = k == 0 ? (vb[0] & ~1ull) : vb[k];
      if (x) first = (int64_t)k * 64 + __builtin_ctzll(x);
    }
    t->args.first_reach = first;
  }
  if (int rc = build_pair_list(t, self_built)) return rc;
  // default budgets: no modification rows (callers set them)
  std::vector<uint8_t> mod(t->n_rows, 0);
  std::vector<int64_t> cap(t->n_rows, 0);
  return sst_table_set_budgets(t, mod.data(), cap.data());
}

int check_masses(sst_ctx* c, const int64_t* masses, int n_rows) {
  if (!masses || n_rows < 1 || n_rows > kMaxRows)
    return fail(c, SST_E_ARG, "n_rows must be in [1, 120]");
  for (int r = 0; r < n_rows; ++r)
    if (masses[r] < 0 || masses[r] > (int64_t)INT32_MAX) return fail(c, SST_E_ARG, "integer masses must be in [0, 2^31)");
  return SST_OK;
}

bool valid_C(int C) { return C == 4 || C == 8 || C == 16 || C == 32; }

}  // namespace

extern "C" {

int sst_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

#ifdef SST_DIAG_TIME  // timing builds only (tools/c1_time.py)
}  // extern "C"
namespace sst {
hipError_t diag_time_read(void* dst, size_t bytes);
hipError_t diag_time_clear();
}  // namespace sst
extern "C" {
int sst_diag_time_read(void* dst, size_t bytes) { return sst::diag_time_read(dst, bytes) == hipSuccess ? 0 : -1; }
int sst_diag_time_clear() { return sst::diag_time_clear() == hipSuccess ? 0 : -1; }
#endif

int sst_ctx_create(int device, sst_ctx** out) {
  if (!out) return SST_E_ARG;
  *out = nullptr;
  int n = sst_device_count();
  if (device < 0 || device >= n) return SST_E_ARG;
  sst_ctx* c = new sst_ctx();
  c->device = device;
  {
    int cu = 0;
    if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cu > 0) c->n_cu = cu;
    (void)hipGetLastError();
  }
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return SST_E_HIP;
  }
  c->stream = c->own;
  *out = c;
  return SST_OK;
}

void sst_ctx_destroy(sst_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  (void)hipStreamSynchronize(c->own);
  for (DevBuf* b : {&c->in_mass, &c->in_thr, &c->in_mods, &c->out_valid, &c->ws_deep, &c->ws_hash, &c->ws_frames,
                    &c->ws_stacks, &c->ws_epochs, &c->singleton_masses})
    b->release();
  prof_resolve(c);
  for (hipEvent_t e : c->pool) (void)hipEventDestroy(e);
  (void)hipStreamDestroy(c->own);
  delete c;
}

const char* sst_last_error(const sst_ctx* c) { return c ? c->err.c_str() : "null context"; }

void* sst_ctx_stream(sst_ctx* c) { return c ? (void*)c->stream : nullptr; }

int sst_ctx_set_stream(sst_ctx* c, void* stream) {
  if (!c) return SST_E_ARG;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  c->stream = stream ? (hipStream_t)stream : c->own;
  return SST_OK;
}

int sst_ctx_synchronize(sst_ctx* c) {
  if (!c) return SST_E_ARG;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  HIP_OK(c, hipStreamSynchronize(c->stream));
  return SST_OK;
}

int sst_ctx_trim(sst_ctx* c) {
  if (!c) return SST_E_ARG;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  HIP_OK(c, hipStreamSynchronize(c->stream));
  c->lbf = sst_ctx::LbfWs{};  // DevBuf frees on destruction
  c->lbf_small = sst_ctx::LbfWs{};
  return SST_OK;
}

int sst_table_build(sst_ctx* c, const int64_t* masses, int n_rows, int64_t max_mass, int C, sst_table** out) {
  if (!c || !out) return SST_E_ARG;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  *out = nullptr;
  if (int rc = check_masses(c, masses, n_rows)) return rc;
  if (!valid_C(C)) return fail(c, SST_E_ARG, "The compression rate is not compatible with the table setup.");
  if (max_mass < 0) return fail(c, SST_E_ARG, "max_mass must be >= 0");
  if (int rc = set_device(c)) return rc;
  sst_table* t = new sst_table();
  t->ctx = c;
  t->n_rows = n_rows;
  t->C = C;
  t->n_cols = table_cols(max_mass, C);
  t->M = t->n_cols * C;
  if (t->M > (int64_t)INT32_MAX) {  // the query kernels hold window values in u32
    delete t;
    return fail(c, SST_E_ARG, "table would cover masses beyond 2^31 - 1");
  }
  t->masses.assign(masses, masses + n_rows);
  const int64_t M = t->M, rw = (M + 63) / 64;
  DevBuf R, tmp, wdev;
  if (!R.ensure((size_t)n_rows * rw * 8) || !tmp.ensure((size_t)2 * rw * 8) || !wdev.ensure(n_rows * 8) ||
      !t->packed.ensure((size_t)n_rows * t->n_cols * (C / 4))) {
    delete t;
    return fail(c, SST_E_NOMEM, "device allocation failed (table build)");
  }
  uint64_t* Rp = (uint64_t*)R.p;
  uint64_t* T[2] = {(uint64_t*)tmp.p, (uint64_t*)tmp.p + rw};
  HIP_OK(c, hipMemcpyAsync(wdev.p, masses, n_rows * 8, hipMemcpyHostToDevice, c->stream));
  HIP_OK(c, launch_bits_seed(Rp, rw, c->stream));
  // R_r = R_{r-1} closed under +w_r by doubling: after j passes all multiples
  // 0..2^j-1 of w_r are added; stop once 2^j * w_r >= M.
  std::vector<uint8_t> literal(n_rows, 0);
  for (int r = 1; r < n_rows; ++r) {
    const uint64_t* src = Rp + (int64_t)(r - 1) * rw;
    uint64_t* dst_final = Rp + (int64_t)r * rw;
    int64_t k = masses[r];
    if (k > 0 && k < C) {  // step == 0: the reference's single in-place sweep
      literal[r] = 1;
      void* row = (char*)t->packed.p + (size_t)r * t->n_cols * (C / 4);
      HIP_OK(c, launch_row_literal(C, src, t->n_cols, (int)k, row, rw, dst_final, c->stream));
      continue;
    }
    if (k <= 0 || k >= M) {
      HIP_OK(c, hipMemcpyAsync(dst_final, src, rw * 8, hipMemcpyDeviceToDevice, c->stream));
      continue;
    }
    int passes = 0;
    for (int64_t kk = k; kk < M; kk *= 2) ++passes;
    int cur = 0;
    for (int p = 0; p < passes; ++p, k *= 2) {
      uint64_t* dst = (p == passes - 1) ? dst_final : T[cur];
      HIP_OK(c, launch_bits_shift_or(dst, src, k, rw, M, c->stream));
      src = dst;
      cur ^= 1;
    }
  }
  DevBuf lit;
  if (!lit.ensure(n_rows)) return fail(c, SST_E_NOMEM, "device allocation failed");
  HIP_OK(c, hipMemcpyAsync(lit.p, literal.data(), n_rows, hipMemcpyHostToDevice, c->stream));
  HIP_OK(c, launch_pack(C, Rp, rw, n_rows, (const int64_t*)wdev.p, t->n_cols, M, last_col_mask(max_mass, t->n_cols, C),
                        (const uint8_t*)lit.p, t->packed.p, c->stream));
  HIP_OK(c, hipStreamSynchronize(c->stream));
  lit.release();
  R.release();
  tmp.release();
  wdev.release();
  int rc = finish_table(t, true);
  if (rc) {
    delete t;
    return rc;
  }
  *out = t;
  return SST_OK;
}

int sst_table_upload(sst_ctx* c, const int64_t* masses, int n_rows, const void* words, int64_t n_cols, int C,
                     sst_table** out) {
  if (!c || !out || !words) return SST_E_ARG;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  *out = nullptr;
  if (int rc = check_masses(c, masses, n_rows)) return rc;
  if (!valid_C(C) || n_cols < 1) return fail(c, SST_E_ARG, "bad compression or n_cols");
  if (n_cols > (int64_t)INT32_MAX / C) return fail(c, SST_E_ARG, "table covers masses beyond 2^31 - 1");
  if (int rc = set_device(c)) return rc;
  sst_table* t = new sst_table();
  t->ctx = c;
  t->n_rows = n_rows;
  t->C = C;
  t->n_cols = n_cols;
  t->M = n_cols * C;
  t->masses.assign(masses, masses + n_rows);
  size_t bytes = (size_t)n_rows * n_cols * (C / 4);
  if (!t->packed.ensure(bytes)) {
    delete t;
    return fail(c, SST_E_NOMEM, "device allocation failed (upload)");
  }
  hipError_t e = hipMemcpy(t->packed.p, words, bytes, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    delete t;
    return fail(c, SST_E_HIP, std::string("upload: ") + hipGetErrorString(e));
  }
  int rc = finish_table(t, false);
  if (rc) {
    delete t;
    return rc;
  }
  *out = t;
  return SST_OK;
}

int sst_table_set_budgets(sst_table* t, const uint8_t* is_mod, const int64_t* cap) {
  if (!t || !is_mod || !cap) return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  const int N = t->n_rows;
  t->is_mod.assign(is_mod, is_mod + N);
  t->cap.assign(cap, cap + N);
  std::vector<int> cap32(N);
  uint64_t mod0 = 0, mod1 = 0, cz0 = 0, cz1 = 0, cn0 = 0, cn1 = 0;
  int any_mod = 0;
  int64_t wmm = 0, lim = INT64_MAX;
  for (int r = 0; r < N; ++r) {
    int64_t cp = cap[r];
    cap32[r] = (int)std::max<int64_t>(std::min<int64_t>(cp, kInfBudget), -1);
    bool m = is_mod[r] != 0;
    if (m) {
      (r < 64 ? mod0 : mod1) |= 1ull << (r & 63);
      any_mod = 1;
      int64_t w = t->masses[r];
      if (w > 0 && (wmm == 0 || w < wmm)) wmm = w;
      // no per-row cap can bind for window values v <= (cap+1)*w - 1
      int64_t cpp = std::max<int64_t>(cp, 0);
      int64_t l = (w <= 0) ? (cpp > 0 ? INT64_MAX : -1)
                           : (cpp + 1 > INT64_MAX / std::max<int64_t>(w, 1) ? INT64_MAX : (cpp + 1) * w - 1);
      lim = std::min(lim, l);
    }
    if (cp <= 0) (r < 64 ? cz0 : cz1) |= 1ull << (r & 63);
    if (cp < 0) (r < 64 ? cn0 : cn1) |= 1ull << (r & 63);
  }
  if (!t->capd.ensure(N * sizeof(int)) || !t->modd.ensure(N)) return fail(c, SST_E_NOMEM, "device allocation failed");
  HIP_OK(c, hipMemcpy(t->capd.p, cap32.data(), N * sizeof(int), hipMemcpyHostToDevice));
  HIP_OK(c, hipMemcpy(t->modd.p, is_mod, N, hipMemcpyHostToDevice));
  t->args.cap = (const int*)t->capd.p;
  t->args.mod = (const uint8_t*)t->modd.p;
  t->args.mod0 = mod0;
  t->args.mod1 = mod1;
  t->args.capz0 = cz0;
  t->args.capz1 = cz1;
  t->args.capneg0 = cn0;
  t->args.capneg1 = cn1;
  t->args.any_mod = any_mod;
  t->args.w_min_mod = (int)(wmm > 0 ? wmm : 1);
  t->args.fast_limit_B = lim;
  refresh_limits(t);
  return SST_OK;
}

int sst_table_shape(const sst_table* t, int* n_rows, int64_t* n_cols, int* C) {
  if (!t) return SST_E_ARG;
  if (n_rows) *n_rows = t->n_rows;
  if (n_cols) *n_cols = t->n_cols;
  if (C) *C = t->C;
  return SST_OK;
}

int sst_table_download(sst_table* t, void* out) {
  if (!t || !out) return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  HIP_OK(c, hipStreamSynchronize(c->stream));
  HIP_OK(c, hipMemcpy(out, t->packed.p, (size_t)t->n_rows * t->n_cols * (t->C / 4), hipMemcpyDeviceToHost));
  return SST_OK;
}

void sst_table_destroy(sst_table* t) {
  if (!t) return;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  for (DevBuf* b : {&t->packed, &t->index, &t->valid, &t->w, &t->capd, &t->modd, &t->pairs, &t->census, &t->canon_c})
    b->release();
  delete t;
}

int sst_is_valid_batch_device(sst_table* t, const double* d_mass, const double* d_thr, int64_t n, double tol,
                              double prec, int8_t* d_out) {
  if (!t || n < 0 || n > INT32_MAX || (n > 0 && (!d_mass || !d_out))) return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  Prof p(c, SST_K_IS_VALID);
  HIP_OK(c, launch_is_valid(t->args.valid, t->args.limit, t->args.full_lo, t->args.full_hi, t->args.first_reach, d_mass,
                            d_thr, n, tol, prec, d_out, c->stream));
  return SST_OK;
}

int sst_is_valid_peaks_device(sst_table* t, const double* d_obs, int64_t n_peaks, const double* shifts, int n_shifts,
                              double tol, double prec, int8_t* d_out) {
  if (!t || n_peaks < 0 || n_peaks > INT32_MAX || n_shifts < 0 || n_shifts > 64 ||
      (n_peaks > 0 && n_shifts > 0 && (!d_obs || !d_out || !shifts)) ||
      (int64_t)n_shifts * n_peaks > INT32_MAX)
    return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  Prof p(c, SST_K_IS_VALID);
  HIP_OK(c, launch_is_valid_peaks(t->args.valid, t->args.limit, t->args.full_lo, t->args.full_hi, t->args.first_reach,
                                  d_obs, n_peaks, shifts, n_shifts, tol, prec, d_out, c->stream));
  return SST_OK;
}
int sst_is_valid_peaks(sst_table* t, const double* obs, int64_t n_peaks, const double* shifts, int n_shifts,
                       double tol, double prec, int8_t* out) {
  if (!t || n_peaks < 0 || n_peaks > INT32_MAX || n_shifts < 0 || n_shifts > 64 ||
      (n_peaks > 0 && n_shifts > 0 && (!obs || !out || !shifts)))
    return SST_E_ARG;
  const int64_t n = n_peaks * n_shifts;
  if (n == 0) return SST_OK;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  if (!c->in_mass.ensure(n_peaks * 8) || !c->out_valid.ensure(n))
    return fail(c, SST_E_NOMEM, "device allocation failed (staging)");
  HIP_OK(c, hipMemcpyAsync(c->in_mass.p, obs, n_peaks * 8, hipMemcpyHostToDevice, c->stream));
  if (int rc = sst_is_valid_peaks_device(t, (const double*)c->in_mass.p, n_peaks, shifts, n_shifts, tol, prec,
                                         (int8_t*)c->out_valid.p))
    return rc;
  HIP_OK(c, hipMemcpyAsync(out, c->out_valid.p, n, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(c, hipStreamSynchronize(c->stream));
  return SST_OK;
}
int sst_is_valid_batch(sst_table* t, const double* mass, const double* thr, int64_t n, double tol, double prec,
                       int8_t* out) {
  if (!t || n < 0 || n > INT32_MAX || (n > 0 && (!mass || !out))) return SST_E_ARG;
  if (n == 0) return SST_OK;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  if (!c->in_mass.ensure(n * 8) || (thr && !c->in_thr.ensure(n * 8)) || !c->out_valid.ensure(n))
    return fail(c, SST_E_NOMEM, "device allocation failed (staging)");
  HIP_OK(c, hipMemcpyAsync(c->in_mass.p, mass, n * 8, hipMemcpyHostToDevice, c->stream));
  if (thr) HIP_OK(c, hipMemcpyAsync(c->in_thr.p, thr, n * 8, hipMemcpyHostToDevice, c->stream));
  if (int rc = sst_is_valid_batch_device(t, (const double*)c->in_mass.p, thr ? (const double*)c->in_thr.p : nullptr, n,
                                         tol, prec, (int8_t*)c->out_valid.p))
    return rc;
  HIP_OK(c, hipMemcpyAsync(out, c->out_valid.p, n, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(c, hipStreamSynchronize(c->stream));
  return SST_OK;
}

}  // extern "C"

namespace {

constexpr int kDeepBlocks = 4096;       // waves (64 lanes) per deep role (fast, no-memo) of the deferred kernel:
                                        // 4 waves per SIMD, so the latency-bound DFS lanes overlap their loads
constexpr uint32_t kHashCap0 = 1u << 14;  // exact-path hash entries per lane (first attempt)
constexpr int kExactLanes0 = 2048;      // exact-path concurrent lanes (first attempt)
constexpr uint64_t kNodeBudget = 1ull << 32;
constexpr uint64_t kRecNodeBudget = 1ull << 34;  // explain_recursion: per-query DFS nodes before ABORTED (a guard only)
constexpr uint32_t kRecHashCap0 = 1u << 16;       // explain_recursion: memo nodes per lane (first attempt)
constexpr uint64_t kLBNodeBudget = 1ull << 34;  // length bound: per-query DFS nodes before ABORTED (a guard only)
constexpr size_t kMaxMemoBytes = 64ull << 30;    // largest per-launch memo workspace the retries grow to
// first memo capacity per query in flight: 2^23 entries shared by the units
// (one query per wave), at least `floor` each -- few queries get a large
// memo at once instead of re-running after each exhaustion
uint32_t memo_cap0(int units, uint32_t floor) {
  uint32_t cap = 1u << 23;
  while (cap > floor && (uint64_t)cap * (uint64_t)units > (1ull << 23)) cap >>= 1;
  return cap;
}
constexpr uint32_t kLBHashCap0 = 1u << 16;       // length bound: memo masses per lane (first attempt)

void free_result_bufs(sst_result* r) {
  for (DevBuf* b : {&r->status, &r->hits, &r->dense, &r->payload, &r->ctl, &r->lists, &r->wave_stats, &r->work,
                    &r->work_count, &r->tally, &r->wg_tally, &r->dhits, &r->hdr, &r->agg, &r->refs, &r->stage, &r->count,
                    &r->offset, &r->rows_su, &r->rows_ob, &r->rows_side, &r->rows_tot, &r->rows_chunk, &r->rows_ctl, &r->rows_big, &r->rows_redo, &r->rows_ans, &r->rows_aq,
                    &r->lb_caps, &r->lb_capz, &r->lb_never})
    b->release();
  if (r->hdr_host) (void)hipHostFree(r->hdr_host);
  r->hdr_host = nullptr;
  if (r->settle_ev) (void)hipEventDestroy(r->settle_ev);
  r->settle_ev = nullptr;
}

uint64_t* ctl_block(sst_result* r, int parity) { return (uint64_t*)r->ctl.p + parity * kCtlWords; }

OutArgs out_args(sst_result* r) {
  static_assert(kCtlArenaRetries < kCtlStats && kCtlStats + kNumStats <= kCtlDhits && kCtlDhits < kCtlWords &&
                    kCtlWords <= kScanWG && 2 * 2 >= kNumClasses,
                "control block layout");
  OutArgs o{};
  uint64_t* ctl = ctl_block(r, r->parity);
  o.status = (int8_t*)r->status.p;
  o.payload = (uint8_t*)r->payload.p;
  o.arena_bytes = r->arena_bytes;
  o.region_bytes = r->region_bytes;
  o.spill_base = (uint64_t)r->n_scan_waves * r->region_bytes;
  o.cursor = ctl + kCtlCursor;
  o.exact_retries = (unsigned long long*)(ctl + kCtlExactRetries);
  o.arena_retries = (unsigned long long*)(ctl + kCtlArenaRetries);
  o.region_need = (unsigned long long*)(ctl + kCtlRegionNeed);
  o.ctl_next = ctl_block(r, r->parity ^ 1);
  o.ctl_words = kCtlWords;
  o.wave_stats = (unsigned long long*)r->wave_stats.p;
  o.work = (uint4*)r->work.p;
  o.work_count = (uint32_t*)r->work_count.p;
  o.stage = (uint32_t*)r->stage.p;
  o.tally = (uint2*)r->tally.p;
  o.wg_tally = (uint2*)r->wg_tally.p;
  o.work_region = r->work_region;
  o.n_scan_waves = r->n_scan_waves;
  o.counters = (uint32_t*)(ctl + kCtlCounters);
  o.lists = (uint32_t*)r->lists.p;
  o.stats = (unsigned long long*)(ctl + kCtlStats);
  o.dhits = (uint4*)r->dhits.p;
  o.dhit_count = (uint32_t*)(ctl + kCtlDhits);
  o.fused = 0;
  o.agg = (uint64_t*)r->agg.p + (size_t)r->parity * r->n_wg;
  o.agg_next = (uint64_t*)r->agg.p + (size_t)(r->parity ^ 1) * r->n_wg;
  o.hits_out = (uint4*)r->hits.p;
  o.hit_refs = (uint16_t*)r->refs.p;
  o.dense = (uint8_t*)r->dense.p;
  o.hdr = (uint64_t*)r->hdr.p;
  o.hdr_host = r->hdr_host_dev;
  o.pass_id = 0;
  return o;
}

int ensure_exact_ws(sst_ctx* c, uint32_t hash_cap, int lanes) {
  if (c->hash_cap == hash_cap && c->exact_blocks * 64 == lanes) return SST_OK;
  size_t hb = (size_t)lanes * hash_cap * hash_entry_bytes();
  c->ws_hash.release();
  c->ws_epochs.release();
  if (!c->ws_hash.ensure(hb) || !c->ws_epochs.ensure((size_t)lanes * 8) ||
      !c->ws_frames.ensure((size_t)lanes * kMaxDepth * p1_frame_bytes()) ||
      !c->ws_stacks.ensure((size_t)lanes * kMaxDepth * glob_frame_bytes()))
    return fail(c, SST_E_NOMEM, "device allocation failed (exact workspace)");
  HIP_OK(c, hipMemsetAsync(c->ws_hash.p, 0, hb, c->stream));
  HIP_OK(c, hipMemsetAsync(c->ws_epochs.p, 0, (size_t)lanes * 8, c->stream));
  c->hash_cap = hash_cap;
  c->exact_blocks = lanes / 64;
  return SST_OK;
}

uint64_t round16(uint64_t x) { return (x + 15u) & ~15ull; }

// Workspaces for a retry pass: scan-wave regions 4x larger when a wave's
// region overflowed, the spill area sized to what the spill cursor counted
// (it keeps counting past the arena), the exact path's memo 8x larger per
// lane over 8x fewer lanes.
int grow_for_retry(sst_result* r, bool regions, bool spill, bool exact, uint64_t cursor, uint64_t region_need) {
  sst_ctx* c = r->ctx;
  if (regions) r->region_bytes = round16(std::max<uint64_t>(2 * r->region_bytes, region_need + region_need / 4));
  if (spill) r->spill_bytes = round16(std::max<uint64_t>(2 * r->spill_bytes, cursor + (1u << 20)));
  if (regions || spill) {
    r->payload.release();
    r->dense.release();
  }
  if (exact) {
    const uint32_t hc = c->hash_cap * 8;
    const int lanes = std::max(64, (c->exact_blocks * 64) / 8);
    if (hc > (1u << 26)) return fail(c, SST_E_INTERNAL, "explain: exact-path memo exceeds 2^26 masses");
    if (int rc = ensure_exact_ws(c, hc, lanes)) return rc;
  }
  return SST_OK;
}

// The scalar budget folded into the scan's u32 limits.  With A0 =
// clamp(max_mods_scalar), budgets_never_bind(hi, A0) holds iff
// hi < never_lim and (no mod rows, A0 = inf, or hi < (A0 + 1) * w_min_mod);
// window values are < 2^31, so clamping the products to u32 is exact.
void fold_scan_limits(const TableArgs& a, QueryArgs& q) {
  const int64_t A0 = q.max_mods_scalar < 0 ? (int64_t)kInfBudget : std::min<int64_t>(q.max_mods_scalar, kInfBudget);
  uint64_t a0lim = UINT32_MAX;
  if (a.any_mod && A0 < kInfBudget) a0lim = std::min<uint64_t>((uint64_t)(A0 + 1) * (uint64_t)a.w_min_mod, UINT32_MAX);
  q.pair_hi_lim = (uint32_t)std::min<uint64_t>(a.pair_lim, a0lim);
  q.never_hi_lim = (uint32_t)std::min<uint64_t>(a.never_lim, a0lim);
  q.cap32 = (uint32_t)std::min<uint64_t>(q.cap_count, UINT32_MAX);
}

// the deferred-class launch of a pass (after the pair scan it also runs the
// SHALLOW windows, one wave per block)
int launch_tail(sst_table* t, sst_result* r) {
  sst_ctx* c = t->ctx;
  const auto& ps = r->pass;
  QueryArgs q{ps.mass, ps.thr, ps.mods, ps.mods_scalar, r->n, ps.tol, ps.prec, 1.0 / ps.prec, ps.with_memo, ps.cap,
              kNodeBudget};
  fold_scan_limits(t->args, q);
  q.alpha = ps.alpha;
  q.spec = ps.spec;
  q.comp = (int)t->C;
  q.qlen = ps.lb.qlen;
  q.caps_len = ps.lb.caps;
  q.capz_len = ps.lb.capz;
  q.never_len = ps.lb.never;
  OutArgs o = out_args(r);
#ifdef SST_DIAG  // diagnostic builds only (make DIAG=1): roles switched off, results invalid
  {
    static const char* dbg = getenv("SST_TAIL_DBG");
    o.dbg = dbg ? atoi(dbg) : 0;
  }
#endif
  // the deep roles' DFS stacks (~1.5 GB): allocated at the first pass that
  // routes windows to them, not with every ctx
  if (!c->ws_deep.ensure((size_t)2 * kDeepBlocks * 64 * kMaxDepth * glob_frame_bytes()))
    return fail(c, SST_E_NOMEM, "device allocation failed (deep workspace)");
  ExactWs ws{(char*)c->ws_hash.p, (char*)c->ws_frames.p, (char*)c->ws_stacks.p, (uint64_t*)c->ws_epochs.p,
             c->hash_cap};
  Prof p(c, SST_K_EXPLAIN_DEEP);  // deep, no-memo and exact roles: one launch
  const int shallow_blocks = r->bitset_scan ? 0 : std::min(r->n_expand_waves, 4 * c->n_cu);
  HIP_OK(c, launch_explain_deferred(t->args, q, o, c->ws_deep.p, shallow_blocks, kDeepBlocks, ws, c->exact_blocks,
                                    c->stream));
  r->tail_ran = true;
  return SST_OK;
}

// k_result_pack: dense hit list + dense payload + header of the current pass
int launch_pack(sst_result* r, const uint64_t* scan_hdr = nullptr) {
  sst_ctx* c = r->ctx;
  r->pass_stream = c->stream;  // the header the host waits for comes from this stream
  PackArgs pa{};
  if (scan_hdr) {  // after a fused scan: its part of the result is in place
    pa.scan_packed = 1;
    pa.scan_hits = scan_hdr[kHdrHits];
    pa.scan_bytes = scan_hdr[kHdrPayload];
  }
  pa.tally = (const uint2*)r->tally.p;
  pa.wg_tally = (const uint2*)r->wg_tally.p;
  pa.work = (const uint4*)r->work.p;
  pa.work_region = r->work_region;
  pa.arena = (const uint8_t*)r->payload.p;
  pa.region_bytes = r->region_bytes;
  pa.spill_base = (uint64_t)r->n_scan_waves * r->region_bytes;
  pa.spill_cap = r->spill_bytes;
  pa.ctl = ctl_block(r, r->parity);
  pa.dhits = (const uint4*)r->dhits.p;
  pa.hits = (uint4*)r->hits.p;
  pa.payload = (uint8_t*)r->dense.p;
  pa.hdr = (uint64_t*)r->hdr.p;
  pa.hdr_host = r->hdr_host_dev;
  pa.pass_id = ++r->pack_seq;
  pa.n_wg = r->n_wg;
#ifdef SST_DIAG  // diagnostic builds only (make DIAG=1): copies skipped, results invalid
  {
    static const char* dbg = getenv("SST_PACK_DBG");
    pa.dbg = dbg ? atoi(dbg) : 0;
  }
#endif
  {
    Prof p(c, SST_K_RESULT_PACK);
    HIP_OK(c, launch_result_pack(pa, c->stream));
  }
  return SST_OK;
}

// One pass of the explain pipeline on device buffers: the scan, the
// deferred-class launch (eager_tail; otherwise settle() launches it only if
// the scan routed a window to it) and the result pack.  Tables without the
// pair list run k_bitset_scan + k_explain_expand and always the tail.
// is_valid over peaks x breakage weights issued with a pass (sst_step_device)
struct PeaksJob {
  const double* obs;
  int64_t n;
  const double* shifts;
  int n_shifts;
  int8_t* out;
};

int explain_pass(sst_table* t, sst_result* r, const double* d_mass, const double* d_thr, const int64_t* d_mods,
                 int64_t mods_scalar, double tol, double prec, int with_memo, uint64_t cap_count, bool eager_tail,
                 const PeaksJob* peaks = nullptr, const uint64_t* d_alpha = nullptr, const int32_t* d_spec = nullptr,
                 const LenBudgets* lens = nullptr) {
  sst_ctx* c = t->ctx;
  const LenBudgets lb = lens ? *lens : LenBudgets{};
  r->pass = {t, d_mass, d_thr, d_mods, mods_scalar, tol, prec, with_memo, cap_count, d_alpha, d_spec, lb};
  r->pass_stream = c->stream;
  r->settle_ev_pending = false;
  r->rows_pass = false;
  const int64_t n = r->n;
  r->arena_bytes = (uint64_t)r->n_scan_waves * r->region_bytes + r->spill_bytes;
  if (!r->ctl.ensure(2 * kCtlWords * 8) || !r->lists.ensure((size_t)kNumClasses * std::max<int64_t>(n, 1) * 4) ||
      !r->payload.ensure(r->arena_bytes) || !r->dense.ensure(r->arena_bytes))
    return fail(c, SST_E_NOMEM, "device allocation failed (result)");
  if (!r->ctl_ready) {
    HIP_OK(c, hipMemsetAsync(r->ctl.p, 0, 2 * kCtlWords * 8, c->stream));
    r->ctl_ready = true;
  }
  r->parity ^= 1;  // zeroed by the previous pass's scan (or above)
  ++r->pass_id;
  r->tail_ran = false;
  r->arrays_ready = false;
  r->bitset_scan = !t->args.pairs_enabled;
  if (n == 0 && peaks && peaks->n > 0 && peaks->n_shifts > 0) {
    Prof p(c, SST_K_IS_VALID);
    HIP_OK(c, launch_is_valid_peaks(t->args.valid, t->args.limit, t->args.full_lo, t->args.full_hi,
                                    t->args.first_reach, peaks->obs, peaks->n, peaks->shifts, peaks->n_shifts, tol,
                                    prec, peaks->out, c->stream));
  }
  if (n == 0) {  // nothing to launch: an empty, settled result
    // no scan ran to zero what the next pass reads: its control block and
    // its half of the look-back aggregates
    HIP_OK(c, hipMemsetAsync(ctl_block(r, r->parity ^ 1), 0, kCtlWords * 8, c->stream));
    HIP_OK(c, hipMemsetAsync((uint64_t*)r->agg.p + (size_t)(r->parity ^ 1) * r->n_wg, 0, (size_t)r->n_wg * 8,
                             c->stream));
    r->fused_pass = r->scan_hdr_pending = false;
    r->scan_hits = r->scan_bytes = 0;
    r->n_hits = r->payload_bytes = 0;
    r->settled = true;
    return SST_OK;
  }
  r->settled = false;
  if (c->hash_cap == 0) {
    // SST_EXACT_HASH_CAP0 (tests): a smaller first memo per lane, so that the
    // retry ladder (8x the memo over 8x fewer lanes) runs down to its last rung
    const char* e = getenv("SST_EXACT_HASH_CAP0");
    uint32_t cap0 = kHashCap0;
    if (e && atoi(e) >= 16) {
      cap0 = 16;
      while (cap0 < (uint32_t)atoi(e) && cap0 < kHashCap0) cap0 <<= 1;
    }
    if (int rc = ensure_exact_ws(c, cap0, kExactLanes0)) return rc;
  }
  // per-query alphabets: the scan answers no window itself (its pair list and
  // SHALLOW role know the full alphabet only) and routes every window with
  // values to the deferred roles, which walk the alphabet's rows only
  TableArgs ta = t->args;
  if (d_alpha) ta.pair_lim = 0, ta.shallow_hi = 0;
  QueryArgs q{d_mass, d_thr, d_mods, mods_scalar, n, tol, prec, 1.0 / prec, with_memo, cap_count, kNodeBudget};
  fold_scan_limits(ta, q);
  q.alpha = d_alpha;
  q.spec = d_spec;
  q.comp = (int)t->C;
  q.qlen = lb.qlen;
  q.caps_len = lb.caps;
  q.capz_len = lb.capz;
  q.never_len = lb.never;
  OutArgs o = out_args(r);
  // the pair scan packs its own result (and writes the header) when no
  // deferred-class launch follows it in this pass
  const bool fused = !eager_tail && !r->bitset_scan;
  r->fused_pass = fused;
  r->scan_hdr_pending = fused;
  r->scan_hits = r->scan_bytes = 0;
  if (fused) {
    o.fused = 1;
    o.pass_id = ++r->pack_seq;
#ifdef SST_DIAG  // diagnostic builds only (make DIAG=1)
    static const char* dbg = getenv("SST_PACK_DBG");
    o.dbg = dbg ? atoi(dbg) : 0;
#endif
  }
  const bool step = peaks && peaks->n > 0 && peaks->n_shifts == 4 && fused;
  if (peaks && peaks->n > 0 && peaks->n_shifts > 0 && !step) {  // A7 in its own launch, before the pass
    Prof p(c, SST_K_IS_VALID);
    HIP_OK(c, launch_is_valid_peaks(t->args.valid, t->args.limit, t->args.full_lo, t->args.full_hi,
                                    t->args.first_reach, peaks->obs, peaks->n, peaks->shifts, peaks->n_shifts, tol,
                                    prec, peaks->out, c->stream));
  }
  {
    Prof p(c, SST_K_EXPLAIN_MAIN);
    if (step)
      HIP_OK(c, launch_step(t->args, q, o, r->n_wg, peaks->obs, peaks->n, peaks->shifts, tol, prec, peaks->out,
                            c->stream));
    else
      HIP_OK(c, launch_explain_scan(ta, q, o, r->n_wg, c->stream));
  }
  if (fused) return SST_OK;
  if (r->bitset_scan) {  // the expand kernel routes the windows the bitset scan queued
    Prof p(c, SST_K_EXPLAIN_EXPAND);
    HIP_OK(c, launch_explain_expand(ta, q, o, r->n_expand_waves / (kWG / 64), c->stream));
    eager_tail = true;
  }
  if (eager_tail)
    if (int rc = launch_tail(t, r)) return rc;
  return launch_pack(r);
}

// Scan workgroups per CU of a fused step (sst_step_device with peaks): one
// 1024-lane scan workgroup per CU leaves half of each CU's lane slots to the
// is_valid workgroups behind the scan's grid, which then run beside the scan
// from the start instead of only in its tail (one box: 69.1 against 72.7 µs
// per step with two scan workgroups per CU; the scan alone is 13 % slower at
// half occupancy).  SST_STEP_SCAN_WG_PER_CU overrides (A/B).
int step_scan_wg_per_cu() {
  static const int v = [] {
    const char* e = getenv("SST_STEP_SCAN_WG_PER_CU");
    return e && atoi(e) > 0 ? atoi(e) : 1;
  }();
  return v;
}

int alloc_result(sst_table* t, int64_t n, sst_result** out, bool step = false) {
  sst_ctx* c = t->ctx;
  if (t->scan_blocks == 0) t->scan_blocks = c->n_cu * explain_scan_blocks_per_cu(scan_dyn_lds(t->args));
  if (c->expand_blocks == 0) c->expand_blocks = c->n_cu * explain_expand_blocks_per_cu();
  sst_result* r = new sst_result();
  r->ctx = c;
  r->pass_stream = c->stream;
  r->n = n;
  r->cap_n = n;
  size_t nn = (size_t)std::max<int64_t>(n, 1);
  // the scan grid: every resident workgroup, or fewer for small batches (16
  // tiles of 64 queries per workgroup at least); worklist: one region per
  // scan wave, big enough for all its tiles
  int64_t tiles = ((int64_t)nn + 63) / 64;
  const int64_t grid = step ? (int64_t)c->n_cu * std::min<int64_t>(t->scan_blocks / c->n_cu, step_scan_wg_per_cu())
                            : (int64_t)t->scan_blocks;
  r->n_wg = (int)std::max<int64_t>(1, std::min<int64_t>(grid, (tiles + 15) / 16));
  r->n_scan_waves = (int64_t)r->n_wg * (kScanWG / 64);
  r->work_region = (uint64_t)((tiles + r->n_scan_waves - 1) / r->n_scan_waves) * 64;
  // one arena region per scan wave, sized for 16 B of payload per query slot
  // of the wave (2 KB at least), then a spill area for the deferred paths
  r->n_expand_waves = c->expand_blocks * (kWG / 64);
  r->region_bytes = std::max<uint64_t>(2048, round16(16 * r->work_region));
  r->spill_bytes = round16(std::max<uint64_t>(1u << 20, 2 * (uint64_t)nn));
  void* hh = nullptr;
  bool ok = r->status.ensure(nn) && r->hits.ensure(nn * 16) && r->refs.ensure(nn * 2) && r->dhits.ensure(nn * 16) &&
            r->wave_stats.ensure((size_t)r->n_scan_waves * kNumStats * 8) &&
            r->work.ensure((size_t)r->n_scan_waves * r->work_region * 16) &&
            r->stage.ensure((size_t)r->n_scan_waves * r->work_region * 4) &&
            r->work_count.ensure((size_t)r->n_scan_waves * 4) && r->tally.ensure((size_t)r->n_scan_waves * 8) &&
            r->wg_tally.ensure((size_t)r->n_wg * 8) && r->hdr.ensure(kHdrWords * 8) &&
            r->agg.ensure((size_t)2 * r->n_wg * 8) &&
            hipMemsetAsync(r->agg.p, 0, (size_t)2 * r->n_wg * 8, c->stream) == hipSuccess;
  if (ok && hipHostMalloc(&hh, kHdrWords * 8, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
    r->hdr_host = (uint64_t*)hh;
    void* dp = nullptr;
    ok = hipHostGetDevicePointer(&dp, hh, 0) == hipSuccess && dp != nullptr;
    r->hdr_host_dev = (uint64_t*)dp;
    memset(hh, 0, kHdrWords * 8);
  } else {
    ok = false;
  }
  if (!ok) {
    (void)hipGetLastError();
    free_result_bufs(r);
    delete r;
    return fail(c, SST_E_NOMEM, "device allocation failed (result)");
  }
  *out = r;
  return SST_OK;
}

// Wait for the current pass's last pack to publish its header and read it.
// The header lives in host-mapped memory, written by the pack kernel as soon
// as its sums are known: the host polls it (no event on the stream); the
// pack's remaining stores complete in stream order before any later work of
// this ctx (fetch copies, a re-run, the caller's next kernels).
int wait_header(sst_result* r, uint64_t* h) {
  sst_ctx* c = r->ctx;
  volatile uint64_t* hv = r->hdr_host;
  auto t0 = std::chrono::steady_clock::now();
  for (uint64_t spin = 0; __atomic_load_n(&hv[kHdrPass], __ATOMIC_ACQUIRE) != r->pack_seq; ++spin) {
    if (spin < 4096) continue;
    sched_yield();
    if ((spin & 255) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
      // a long pass (or a lost write): wait for the stream itself, then insist
      HIP_OK(c, hipStreamSynchronize(r->pass_stream));
      if (__atomic_load_n(&hv[kHdrPass], __ATOMIC_ACQUIRE) != r->pack_seq)
        return fail(c, SST_E_INTERNAL, "explain: the result header was not written");
      break;
    }
  }
  for (int k = 0; k < kHdrWords; ++k) h[k] = __atomic_load_n(&hv[k], __ATOMIC_ACQUIRE);
  if (h[kHdrPass] != r->pack_seq) return fail(c, SST_E_INTERNAL, "explain: result header of another pass");
  return SST_OK;
}

// Settle the current pass: wait for it, launch the deferred classes if the
// scan routed windows to them (then pack again), and re-run the pass with
// larger workspaces if a query outgrew a payload region, the spill area or
// the exact path's memo -- from the caller's device inputs, which must still
// hold the batch (include/sst.h).
int settle(sst_result* r) {
  if (r->settled) return SST_OK;
  sst_ctx* c = r->ctx;
  // launches below go to the pass's stream, whatever the ctx's current one is
  struct StreamScope {
    sst_ctx* c;
    hipStream_t saved;
    ~StreamScope() { c->stream = saved; }
  } scope{c, c->stream};
  c->stream = r->pass_stream;
  bool launched = false;
  for (int attempt = 0;; ++attempt) {
    uint64_t h[kHdrWords];
    if (int rc = wait_header(r, h)) return rc;
    if (r->rows_pass) {  // the step from the peaks: its queries, all answered from the pair list
      if (h[kHdrRowsErr])
        return fail(c, SST_E_ARG, "rows step: " + std::string(h[kHdrRowsErr] & 1 ? "a spectrum has more than 1024 peaks"
                                                            : h[kHdrRowsErr] & 2 ? "a side has more than 2048 rows"
                                                            : "more queries / payload than the result holds"));
      r->n = (int64_t)h[kHdrQueries];
    }
    if (r->scan_hdr_pending) {  // the fused scan's own header
      r->scan_hits = h[kHdrHits];
      r->scan_bytes = h[kHdrPayload];
      r->scan_hdr_pending = false;
    }
    if (h[kHdrRouted] && !r->tail_ran) {
      if (int rc = launch_tail(r->pass.t, r)) return rc;
      if (int rc = launch_pack(r, r->fused_pass ? h : nullptr)) return rc;
      launched = true;
      --attempt;
      continue;
    }
    const bool regions = h[kHdrArenaRetries] > 0, spill = h[kHdrCursor] > r->spill_bytes;
    const bool exact = h[kHdrExactRetries] > 0;
    if (!regions && !spill && !exact) {
      r->n_hits = h[kHdrHits];
      r->payload_bytes = h[kHdrPayload];
      break;
    }
    if (attempt == 6) return fail(c, SST_E_INTERNAL, "explain: retries exhausted");
    HIP_OK(c, hipStreamSynchronize(c->stream));  // the pack may still run: buffers are about to be replaced
    if (int rc = grow_for_retry(r, regions, spill, exact, h[kHdrCursor], h[kHdrRegionNeed])) return rc;
    const auto p = r->pass;  // a copy: the pass rewrites it
    if (int rc = explain_pass(p.t, r, p.mass, p.thr, p.mods, p.mods_scalar, p.tol, p.prec, p.with_memo, p.cap, true,
                              nullptr, p.alpha, p.spec, &p.lb))
      return rc;
    launched = true;
  }
  if (launched) {
    if (!r->settle_ev && hipEventCreateWithFlags(&r->settle_ev, hipEventDisableTiming) != hipSuccess) {
      r->settle_ev = nullptr;
      return fail(c, SST_E_HIP, "hipEventCreateWithFlags failed");
    }
    HIP_OK(c, hipEventRecord(r->settle_ev, r->pass_stream));
    r->settle_ev_pending = true;
  }
  r->settled = true;
  return SST_OK;
}

// Order the ctx's current stream after the work settle() queued on the
// pass's stream (a no-op when they are the same stream or settle launched
// nothing): the pass's kernels themselves are the caller's to order.
int order_after_settle(sst_result* r) {
  sst_ctx* c = r->ctx;
  if (r->settle_ev_pending && c->stream != r->pass_stream) HIP_OK(c, hipStreamWaitEvent(c->stream, r->settle_ev, 0));
  return SST_OK;
}

// Host copies: status, the dense hit list (-> count[] / offset[] on the host)
// and the dense payload.
int fetch(sst_result* r) {
  sst_ctx* c = r->ctx;
  if (int rc = settle(r)) return rc;
  const int64_t n = r->n;  // after settling: a rows-step pass learns its query count from the header
  if (int rc = order_after_settle(r)) return rc;
  r->h_status.resize(n);
  r->h_count.assign(n, 0);
  r->h_offset.assign(n, 0);
  std::vector<uint4> hv(r->n_hits);
  std::vector<unsigned long long> ws((size_t)r->n_scan_waves * kNumStats);
  if (n && r->rows_pass) {
    HIP_OK(c, hipMemcpyAsync(r->h_status.data(), r->status.p, n, hipMemcpyDeviceToHost, c->stream));
  } else if (n) {
    HIP_OK(c, hipMemcpyAsync(r->h_status.data(), r->status.p, n, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(c, hipMemcpyAsync(r->h_stats, ctl_block(r, r->parity) + kCtlStats, kNumStats * 8, hipMemcpyDeviceToHost,
                             c->stream));
    HIP_OK(c, hipMemcpyAsync(ws.data(), r->wave_stats.p, ws.size() * 8, hipMemcpyDeviceToHost, c->stream));
  } else {
    for (auto& x : r->h_stats) x = 0;
  }
  if (r->n_hits) HIP_OK(c, hipMemcpyAsync(hv.data(), r->hits.p, r->n_hits * 16, hipMemcpyDeviceToHost, c->stream));
  r->h_payload.resize(r->payload_bytes);
  if (r->payload_bytes)
    HIP_OK(c, hipMemcpyAsync(r->h_payload.data(), r->dense.p, r->payload_bytes, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(c, hipStreamSynchronize(c->stream));
  if (r->rows_pass) {  // no scan waves: every query was a pair-list window
    for (auto& x : r->h_stats) x = 0;
    r->h_stats[kStatPair] = (uint64_t)n;
    r->h_stats[kStatPairPayload] = r->payload_bytes;
  } else if (n && !r->bitset_scan)  // k_bitset_scan's waves write zero counters
    for (int64_t w = 0; w < r->n_scan_waves; ++w)
      for (int k = 0; k < kNumStats; ++k) r->h_stats[k] += ws[(size_t)w * kNumStats + k];
  for (const uint4& h : hv) {
    if (h.x >= (uint32_t)n) return fail(c, SST_E_INTERNAL, "explain: hit record out of range");
    const uint64_t word = ((uint64_t)h.w << 32) | h.z;
    if (r->h_status[h.x] == SST_SOME) {
      r->h_count[h.x] = h.y;
      r->h_offset[h.x] = word;
    } else {
      r->h_count[h.x] = word;
    }
  }
  return SST_OK;
}

}  // namespace

extern "C" {

int sst_explain_batch_device(sst_table* t, const double* d_mass, const double* d_thr, int64_t n, double tol, double prec,
                             const int64_t* d_mods, int64_t mods_scalar, int with_memo, uint64_t cap_count,
                             sst_result** out) {
  if (!t || !out || n < 0 || n > SST_MAX_EXPLAIN_BATCH || (n > 0 && !d_mass)) return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  sst_result* r = *out;
  const bool reuse = r != nullptr;
  if (reuse) {
    if (r->ctx != c || n > r->cap_n) return fail(c, SST_E_ARG, "result reuse: other ctx or capacity < n");
    r->n = n;
  } else if (int rc = alloc_result(t, n, &r)) {
    return rc;
  }
  int rc = explain_pass(t, r, d_mass, d_thr, d_mods, mods_scalar, tol, prec, with_memo, cap_count, false);
  if (rc) {
    if (!reuse) {
      free_result_bufs(r);
      delete r;
    }
    return rc;
  }
  *out = r;
  return SST_OK;
}

int sst_explain_alpha_batch_device(sst_table* t, const double* d_mass, const double* d_thr, const int32_t* d_spec,
                                   const uint64_t* d_alpha, int64_t n, double tol, double prec,
                                   const int64_t* d_mods, int64_t mods_scalar, int with_memo, uint64_t cap_count,
                                   sst_result** out) {
  if (!t || !out || n < 0 || n > SST_MAX_EXPLAIN_BATCH || (n > 0 && (!d_mass || !d_alpha))) return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  sst_result* r = *out;
  const bool reuse = r != nullptr;
  if (reuse) {
    if (r->ctx != c || n > r->cap_n) return fail(c, SST_E_ARG, "result reuse: other ctx or capacity < n");
    r->n = n;
  } else if (int rc = alloc_result(t, n, &r)) {
    return rc;
  }
  int rc = explain_pass(t, r, d_mass, d_thr, d_mods, mods_scalar, tol, prec, with_memo, cap_count, false, nullptr,
                        d_alpha, d_spec);
  if (rc) {
    if (!reuse) {
      free_result_bufs(r);
      delete r;
    }
    return rc;
  }
  *out = r;
  return SST_OK;
}

int sst_explain_alpha_lens_batch_device(sst_table* t, const double* d_mass, const double* d_thr, const int32_t* d_spec,
                                        const uint64_t* d_alpha, const int32_t* d_qlen, const int64_t* caps_by_len,
                                        int n_lens, int64_t n, double tol, double prec, const int64_t* d_mods,
                                        uint64_t cap_count, sst_result** out) {
  if (!t || !out || n < 0 || n > SST_MAX_EXPLAIN_BATCH || n_lens < 1 || n_lens > 4096 || !caps_by_len ||
      (n > 0 && (!d_mass || !d_alpha || !d_qlen || !d_mods)))
    return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  const int N = t->n_rows;
  if ((int)t->is_mod.size() != N) return fail(c, SST_E_ARG, "explain (per-query budgets): the table has no budgets set");
  // per length: the caps (clamped as sst_table_set_budgets), the rows with
  // cap <= 0 and the fast-path limit (no per-row cap can bind below it)
  std::vector<int32_t> caps((size_t)n_lens * kMaxRows, 0);
  std::vector<uint64_t> capz(2 * (size_t)n_lens, 0);
  std::vector<uint32_t> never(n_lens);
  const int64_t u32max = (int64_t)UINT32_MAX;
  for (int L = 0; L < n_lens; ++L) {
    int64_t lim = INT64_MAX;
    bool any_mod = false;
    for (int r = 0; r < N; ++r) {
      const int64_t cp = caps_by_len[(int64_t)L * N + r];
      caps[(size_t)L * kMaxRows + r] = (int32_t)std::max<int64_t>(std::min<int64_t>(cp, kInfBudget), -1);
      if (cp <= 0) capz[2 * L + (r >> 6)] |= 1ull << (r & 63);
      if (t->is_mod[r]) {
        any_mod = true;
        const int64_t w = t->masses[r], cpp = std::max<int64_t>(cp, 0);
        const int64_t l = (w <= 0) ? (cpp > 0 ? INT64_MAX : -1)
                                   : (cpp + 1 > INT64_MAX / std::max<int64_t>(w, 1) ? INT64_MAX : (cpp + 1) * w - 1);
        lim = std::min(lim, l);
      }
    }
    never[L] = (uint32_t)(!any_mod ? u32max : (lim < 0 ? 0 : std::min(lim, u32max - 1) + 1));
  }
  sst_result* r = *out;
  const bool reuse = r != nullptr;
  if (reuse) {
    if (r->ctx != c || n > r->cap_n) return fail(c, SST_E_ARG, "result reuse: other ctx or capacity < n");
    r->n = n;
  } else if (int rc = alloc_result(t, n, &r)) {
    return rc;
  }
  auto drop = [&](int rc) {
    if (!reuse) {
      free_result_bufs(r);
      delete r;
    }
    return rc;
  };
  // the result's own copies (a retry of the pass reads them again); a reused
  // result's previous pass is settled by its consumer before it is reused
  if (!r->lb_caps.ensure(caps.size() * 4) || !r->lb_capz.ensure(capz.size() * 8) || !r->lb_never.ensure(never.size() * 4))
    return drop(fail(c, SST_E_NOMEM, "device allocation failed (result)"));
  if (hipMemcpy(r->lb_caps.p, caps.data(), caps.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(r->lb_capz.p, capz.data(), capz.size() * 8, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(r->lb_never.p, never.data(), never.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
    return drop(fail(c, SST_E_HIP, "hipMemcpy (per-query budgets)"));
  LenBudgets lb{d_qlen, (const int32_t*)r->lb_caps.p, (const uint64_t*)r->lb_capz.p, (const uint32_t*)r->lb_never.p};
  int rc = explain_pass(t, r, d_mass, d_thr, d_mods, 0, tol, prec, 1, cap_count, false, nullptr, d_alpha, d_spec, &lb);
  if (rc) return drop(rc);
  *out = r;
  return SST_OK;
}

int sst_step_device(sst_table* t, const double* d_obs, int64_t n_peaks, const double* shifts, int n_shifts,
                    int8_t* d_valid_out, const double* d_mass, const double* d_thr, int64_t n, double tol, double prec,
                    const int64_t* d_mods, int64_t mods_scalar, int with_memo, uint64_t cap_count, sst_result** out) {
  if (!t || !out || n < 0 || n > SST_MAX_EXPLAIN_BATCH || (n > 0 && !d_mass) || n_peaks < 0 ||
      n_peaks > INT32_MAX || n_shifts < 0 || n_shifts > 64 || (int64_t)n_shifts * n_peaks > INT32_MAX ||
      (n_peaks > 0 && n_shifts > 0 && (!d_obs || !d_valid_out || !shifts)))
    return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  sst_result* r = *out;
  const bool reuse = r != nullptr;
  if (reuse) {
    if (r->ctx != c || n > r->cap_n) return fail(c, SST_E_ARG, "result reuse: other ctx or capacity < n");
    r->n = n;
  } else if (int rc = alloc_result(t, n, &r, n_peaks > 0 && n_shifts > 0)) {
    return rc;
  }
  const PeaksJob job{d_obs, n_peaks, shifts, n_shifts, d_valid_out};
  int rc = explain_pass(t, r, d_mass, d_thr, d_mods, mods_scalar, tol, prec, with_memo, cap_count, false, &job);
  if (rc) {
    if (!reuse) {
      free_result_bufs(r);
      delete r;
    }
    return rc;
  }
  *out = r;
  return SST_OK;
}

int sst_step_rows_device(sst_table* t, const double* d_obs, const int64_t* d_peak_off, int64_t n_spec,
                         int64_t n_peaks, const double* d_intensity, double intensity_cutoff, double mass_cutoff,
                         const double* d_su_seq, const double* shifts, const uint8_t* sides, int n_shifts,
                         double max_weight, double tol, double prec, int64_t max_mods_scalar, uint64_t cap_per_query,
                         int64_t max_queries, int8_t* d_valid_out, sst_result** out) {
  if (!t || !out || n_spec < 1 || n_peaks < 0 || n_peaks > INT32_MAX || n_shifts < 1 || n_shifts > 4 || !shifts ||
      !sides || !d_obs || !d_peak_off || !d_su_seq || !d_valid_out || max_queries < 1 ||
      max_queries > SST_MAX_EXPLAIN_BATCH || (int64_t)n_shifts * n_peaks > INT32_MAX)
    return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  if (!t->args.pairs_enabled || !t->args.census) return fail(c, SST_E_ARG, "rows step: the table has no pair list");
  // every window must be pair-class with budgets that cannot bind: a
  // difference <= max_weight, a threshold <= tol * 2 * mass_cutoff
  const double hi_max = (max_weight + tol * 2.0 * mass_cutoff) / prec + 2.0;
  if (!(hi_max < (double)t->args.pair_hi))
    return fail(c, SST_E_ARG, "rows step: windows may leave the pair class (max_weight / mass_cutoff too large)");
  if (t->args.any_mod) {
    if (max_mods_scalar >= 0 && max_mods_scalar < 2)
      return fail(c, SST_E_ARG, "rows step: max_modifications < 2 can bind on pair windows");
    for (int r = 1; r < t->n_rows; ++r)
      if (t->is_mod[r] && t->cap[r] < 2) return fail(c, SST_E_ARG, "rows step: a modification cap < 2 can bind");
  }
  sst_result* r = *out;
  const bool reuse = r != nullptr;
  if (reuse) {
    if (r->ctx != c || max_queries > r->cap_n) return fail(c, SST_E_ARG, "result reuse: other ctx or capacity");
  } else if (int rc = alloc_result(t, max_queries, &r)) {
    return rc;
  }
  auto bail = [&](int rc) {
    if (!reuse) {
      free_result_bufs(r);
      delete r;
    }
    return rc;
  };
  const size_t P = (size_t)n_peaks, S = (size_t)n_spec;
  const size_t NC = (size_t)c->n_cu * 64;  // chunk capacity: >= the wave kernels' waves (launch_rows_step checks)
  const bool fresh = !r->rows_ctl.p;
  if (!r->dense.ensure(std::max<uint64_t>(r->arena_bytes, (uint64_t)16 * r->cap_n + (1u << 20))) ||
      !r->rows_su.ensure(std::max<size_t>(1, 4 * P) * 8) || !r->rows_ob.ensure(std::max<size_t>(1, 4 * P) * 8) ||
      !r->rows_side.ensure(2 * S * 4) || !r->rows_tot.ensure(3 * S * 4) || !r->rows_chunk.ensure((6 * NC + 6 * (NC / kRowsTile + 1)) * 8) ||
      !r->rows_big.ensure(S * 4) || !r->rows_redo.ensure(S * 4) || !r->rows_ctl.ensure(64) ||
      !r->rows_ans.ensure(128 * S * 8 + (2 * kRowsAnsPerPeak * P / 64 + 2 * S + 2) * 64 * 4) || !r->rows_aq.ensure(2 * S * 4))
    return bail(fail(c, SST_E_NOMEM, "device allocation failed (rows step)"));
  if (fresh) {
    HIP_OK(c, hipMemsetAsync(r->rows_ctl.p, 0, 64, c->stream));
    HIP_OK(c, hipMemsetAsync((uint64_t*)r->rows_chunk.p + 6 * NC, 0, 6 * (NC / kRowsTile + 1) * 8, c->stream));  // tile sums
  }
  r->pass = {t, nullptr, nullptr, nullptr, max_mods_scalar, tol, prec, 1, cap_per_query, nullptr, nullptr};
  r->pass_stream = c->stream;
  r->settle_ev_pending = false;
  r->rows_pass = true;
  ++r->pass_id;
  r->tail_ran = true;  // nothing to route
  r->arrays_ready = false;
  r->bitset_scan = false;
  r->fused_pass = true;
  r->scan_hdr_pending = true;
  r->scan_hits = r->scan_bytes = 0;
  r->settled = false;
  RowsArgs a{};
  a.obs = d_obs;
  a.peak_off = d_peak_off;
  a.n_spec = n_spec;
  a.n_peaks = n_peaks;
  a.intensity = d_intensity;
  a.intensity_cutoff = intensity_cutoff;
  a.mass_cutoff = mass_cutoff;
  a.max_variance = 1.0;  // fragment_classification.py:8
  a.su_seq = d_su_seq;
  for (int k = 0; k < n_shifts; ++k) {
    a.shift[k] = shifts[k];
    a.sides[k] = sides[k];
  }
  a.n_shifts = n_shifts;
  a.max_weight = max_weight;
  a.tol = tol;
  a.prec = prec;
  a.rprec = 1.0 / prec;
  a.cap = (uint32_t)std::min<uint64_t>(cap_per_query, UINT32_MAX);
  a.valid_out = d_valid_out;
  a.rows_su = (double*)r->rows_su.p;
  a.rows_ob = (double*)r->rows_ob.p;
  a.side_rows = (uint32_t*)r->rows_side.p;
  a.ans_mask = (uint64_t*)r->rows_ans.p;
  a.ans_ent = (uint32_t*)(a.ans_mask + 128 * S);
  a.ans_q = (uint32_t*)r->rows_aq.p;
  a.totals = (uint32_t*)r->rows_tot.p;
  a.chunk_tot = (unsigned long long*)r->rows_chunk.p;
  a.chunk_off = (uint64_t*)r->rows_chunk.p + 3 * NC;
  a.tile_tot = (unsigned long long*)r->rows_chunk.p + 6 * NC;
  a.n_tiles = (int64_t)(NC / kRowsTile + 1);
  a.chunk_cap = (int64_t)NC;
  a.ctl = (uint64_t*)r->rows_ctl.p;
  a.err = (uint32_t*)((char*)r->rows_ctl.p + 32);
  a.done = (uint32_t*)((char*)r->rows_ctl.p + 40);
  a.tickets = (uint32_t*)((char*)r->rows_ctl.p + 48);
  a.big = (uint32_t*)r->rows_big.p;
  a.redo = (uint32_t*)r->rows_redo.p;
  a.cap_queries = (uint64_t)r->cap_n;
  a.cap_bytes = r->dense.bytes;
  a.status = (int8_t*)r->status.p;
  a.hits = (uint4*)r->hits.p;
  a.refs = (uint16_t*)r->refs.p;
  a.dense = (uint8_t*)r->dense.p;
  a.hdr = (uint64_t*)r->hdr.p;
  a.hdr_host = r->hdr_host_dev;
  a.pass_id = ++r->pack_seq;
  a.tile_par = r->rows_tile_par ^ 1u;  // the last step zeroed these tile sums
  {
    Prof p(c, SST_K_EXPLAIN_MAIN);
    HIP_OK(c, launch_rows_step(t->args, a, c->n_cu, scan_dyn_lds(t->args), c->stream));
  }
  r->rows_tile_par = a.tile_par;
  *out = r;
  return SST_OK;
}

int sst_explain_batch(sst_table* t, const double* mass, const double* thr, int64_t n, double tol, double prec,
                      const int64_t* mods, int64_t mods_scalar, int with_memo, uint64_t cap_count, sst_result** out) {
  if (!t || !out || n < 0 || n > SST_MAX_EXPLAIN_BATCH || (n > 0 && !mass)) return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  *out = nullptr;
  if (int rc = set_device(c)) return rc;
  size_t nn = (size_t)std::max<int64_t>(n, 1);
  if (!c->in_mass.ensure(nn * 8) || (thr && !c->in_thr.ensure(nn * 8)) || (mods && !c->in_mods.ensure(nn * 8)))
    return fail(c, SST_E_NOMEM, "device allocation failed (staging)");
  if (n) {
    HIP_OK(c, hipMemcpyAsync(c->in_mass.p, mass, n * 8, hipMemcpyHostToDevice, c->stream));
    if (thr) HIP_OK(c, hipMemcpyAsync(c->in_thr.p, thr, n * 8, hipMemcpyHostToDevice, c->stream));
    if (mods) HIP_OK(c, hipMemcpyAsync(c->in_mods.p, mods, n * 8, hipMemcpyHostToDevice, c->stream));
  }
  const double* dm = (const double*)c->in_mass.p;
  const double* dt = thr ? (const double*)c->in_thr.p : nullptr;
  const int64_t* dmo = mods ? (const int64_t*)c->in_mods.p : nullptr;
  sst_result* r = nullptr;
  if (int rc = alloc_result(t, n, &r)) return rc;
  int rc = explain_pass(t, r, dm, dt, dmo, mods_scalar, tol, prec, with_memo, cap_count, true);
  if (!rc) rc = fetch(r);  // settles: retries with larger workspaces happen there
  for (int64_t i = 0; !rc && i < n; ++i)
    if (r->h_status[i] <= kStatusPending) rc = fail(c, SST_E_INTERNAL, "explain: query left unresolved (internal error)");
  if (rc) {
    free_result_bufs(r);
    delete r;
    return rc;
  }
  *out = r;
  return SST_OK;
}

int sst_explain_recursion_batch(sst_table* t, const double* mass, const double* thr, int64_t n, double tol,
                                double prec, const int64_t* mods, int64_t mods_scalar, uint64_t cap_count,
                                sst_result** out) {
  if (!t || !out || n < 0 || n > SST_MAX_EXPLAIN_BATCH || (n > 0 && !mass)) return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  *out = nullptr;
  if (int rc = set_device(c)) return rc;
  const size_t nn = (size_t)std::max<int64_t>(n, 1);
  if (!c->in_mass.ensure(nn * 8) || (thr && !c->in_thr.ensure(nn * 8)) || (mods && !c->in_mods.ensure(nn * 8)))
    return fail(c, SST_E_NOMEM, "device allocation failed (staging)");
  if (n) {
    HIP_OK(c, hipMemcpyAsync(c->in_mass.p, mass, n * 8, hipMemcpyHostToDevice, c->stream));
    if (thr) HIP_OK(c, hipMemcpyAsync(c->in_thr.p, thr, n * 8, hipMemcpyHostToDevice, c->stream));
    if (mods) HIP_OK(c, hipMemcpyAsync(c->in_mods.p, mods, n * 8, hipMemcpyHostToDevice, c->stream));
  }
  sst_result* r = nullptr;
  if (int rc = alloc_result(t, n, &r)) return rc;
  // no scan: the pack finds empty scan tallies and takes the kernel's hit
  // records and spill bytes
  HIP_OK(c, hipMemsetAsync(r->tally.p, 0, r->tally.bytes, c->stream));
  HIP_OK(c, hipMemsetAsync(r->wg_tally.p, 0, r->wg_tally.bytes, c->stream));
  QueryArgs q{(const double*)c->in_mass.p, thr ? (const double*)c->in_thr.p : nullptr,
              mods ? (const int64_t*)c->in_mods.p : nullptr, mods_scalar, n, tol, prec, 1.0 / prec, 1, cap_count,
              kRecNodeBudget};
  // one 64-lane block per query in flight (k_explain_recursion<WAVE>), each
  // with its own memo slice
  int units = (int)std::min<int64_t>(256, n);
  uint32_t cap = memo_cap0(units, kRecHashCap0);
  int rc = SST_OK;
  for (int attempt = 0; n > 0; ++attempt) {
    if (attempt == 8) {
      rc = fail(c, SST_E_INTERNAL, "explain_recursion: retries exhausted");
      break;
    }
    r->arena_bytes = (uint64_t)r->n_scan_waves * r->region_bytes + r->spill_bytes;
    DevBuf hash, frames;
    if (!r->ctl.ensure(2 * kCtlWords * 8) || !r->payload.ensure(r->arena_bytes) ||
        !r->dense.ensure(r->arena_bytes) || !hash.ensure((size_t)units * cap * rec_entry_bytes()) ||
        !frames.ensure((size_t)units * rec_frame_bytes())) {
      rc = fail(c, SST_E_NOMEM, "device allocation failed (recursion)");
      break;
    }
    r->parity = 0;  // one pass per attempt: block 0, zeroed here
    r->ctl_ready = true;
    ++r->pass_id;
    r->bitset_scan = true;  // no scan-wave counters
    HIP_OK(c, hipMemsetAsync(r->ctl.p, 0, 2 * kCtlWords * 8, c->stream));
    HIP_OK(c, hipMemsetAsync(hash.p, 0, hash.bytes, c->stream));
    HIP_OK(c, launch_explain_recursion(t->args, q, out_args(r), (char*)hash.p, (char*)frames.p, cap, units,
                                       c->stream));
    if ((rc = launch_pack(r))) break;
    uint64_t h[kHdrWords];
    if ((rc = wait_header(r, h))) break;
    r->n_hits = h[kHdrHits];
    r->payload_bytes = h[kHdrPayload];
    r->settled = true;
    r->tail_ran = true;
    if ((rc = fetch(r))) break;
    bool memo_retry = false;
    for (int64_t i = 0; i < n; ++i) memo_retry |= r->h_status[i] == kStatusExactRetry;
    const bool arena_retry = h[kHdrCursor] > r->spill_bytes;
    if (!arena_retry && !memo_retry) break;
    if (arena_retry) {
      r->spill_bytes = round16(std::max<uint64_t>(2 * r->spill_bytes, h[kHdrCursor] + (1u << 20)));
      r->payload.release();
      r->dense.release();
    }
    if (memo_retry) {
      if ((size_t)std::max(1, units / 8) * cap * 8 * rec_entry_bytes() > kMaxMemoBytes) {
        rc = fail(c, SST_E_NOMEM, "explain_recursion: memo would exceed the workspace limit");
        break;
      }
      cap *= 8;
      units = std::max(1, units / 8);
    }
  }
  if (!rc && n == 0) {
    r->settled = true;
    rc = fetch(r);
  }
  if (rc) {
    free_result_bufs(r);
    delete r;
    return rc;
  }
  *out = r;
  return SST_OK;
}

int sst_result_settle(sst_result* r, uint64_t* n_hits, uint64_t* payload_bytes) {
  if (!r) return SST_E_ARG;
  std::lock_guard<std::recursive_mutex> g(r->ctx->mu);
  if (int rc = set_device(r->ctx)) return rc;
  if (int rc = settle(r)) return rc;
  if (n_hits) *n_hits = r->n_hits;
  if (payload_bytes) *payload_bytes = r->payload_bytes;
  return SST_OK;
}

int sst_result_queries(sst_result* r, int64_t* n) {
  if (!r || !n) return SST_E_ARG;
  std::lock_guard<std::recursive_mutex> g(r->ctx->mu);
  if (int rc = set_device(r->ctx)) return rc;
  if (int rc = settle(r)) return rc;
  *n = r->n;
  return SST_OK;
}

int sst_result_host(sst_result* r, const int8_t** status, const uint64_t** count, const uint64_t** offset,
                    const uint8_t** payload, uint64_t* payload_bytes) {
  if (!r) return SST_E_ARG;
  if (status) *status = r->h_status.data();
  if (count) *count = r->h_count.data();
  if (offset) *offset = r->h_offset.data();
  if (payload) *payload = r->h_payload.data();
  if (payload_bytes) *payload_bytes = r->h_payload.size();
  return SST_OK;
}

int sst_result_device(sst_result* r, int8_t** d_status, uint64_t** d_count, uint64_t** d_offset, uint8_t** d_payload,
                      uint64_t* payload_bytes) {
  if (!r) return SST_E_ARG;
  sst_ctx* c = r->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  if (int rc = settle(r)) return rc;
  if (int rc = order_after_settle(r)) return rc;
  if ((d_count || d_offset) && !r->arrays_ready) {  // per-query arrays: built from the hit list on request
    const size_t nn = (size_t)std::max<int64_t>(r->n, 1);
    if (!r->count.ensure(nn * 8) || !r->offset.ensure(nn * 8))
      return fail(c, SST_E_NOMEM, "device allocation failed (count / offset arrays)");
    HIP_OK(c, launch_hits_to_arrays((const uint4*)r->hits.p, r->n_hits, (const int8_t*)r->status.p,
                                    (uint64_t*)r->count.p, (uint64_t*)r->offset.p, c->stream));
    r->arrays_ready = true;
  }
  if (d_status) *d_status = (int8_t*)r->status.p;
  if (d_count) *d_count = (uint64_t*)r->count.p;
  if (d_offset) *d_offset = (uint64_t*)r->offset.p;
  if (d_payload) *d_payload = (uint8_t*)r->dense.p;
  if (payload_bytes) *payload_bytes = r->payload_bytes;
  return SST_OK;
}

int sst_result_hit_list(sst_result* r, void** d_hits, uint64_t* n_hits) {
  if (!r || !d_hits || !n_hits) return SST_E_ARG;
  sst_ctx* c = r->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  if (int rc = settle(r)) return rc;
  if (int rc = order_after_settle(r)) return rc;  // settling's extra launches wrote these buffers
  *d_hits = r->hits.p;
  *n_hits = r->n_hits;
  return SST_OK;
}

int sst_result_pair_hits(sst_result* r, void** d_refs, uint64_t* n_pair_hits, uint64_t* pair_bytes, int* n_scan_wg) {
  if (!r) return SST_E_ARG;
  sst_ctx* c = r->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  if (int rc = settle(r)) return rc;
  if (int rc = order_after_settle(r)) return rc;
  if (d_refs) *d_refs = r->refs.p;
  if (n_pair_hits) *n_pair_hits = r->scan_hits;
  if (pair_bytes) *pair_bytes = r->scan_bytes;
  if (n_scan_wg) *n_scan_wg = r->rows_pass ? 0 : r->n_wg;  // 0: the hits come in query order
  return SST_OK;
}

int sst_table_pair_records(sst_table* t, uint32_t* recs, int64_t cap, int64_t* n) {
  if (!t || !n) return SST_E_ARG;
  *n = t->args.pairs_enabled ? (int64_t)t->pair_recs.size() : 0;
  if (!recs || *n == 0) return SST_OK;
  if (cap < *n) return fail(t->ctx, SST_E_ARG, "pair records: buffer too small");
  memcpy(recs, t->pair_recs.data(), (size_t)*n * 4);
  return SST_OK;
}

// FNV-1a (63 bits) of the pair records' bytes: parallel.pair_key
static uint64_t pair_key_of(const std::vector<uint32_t>& recs) {
  uint64_t h = 0xCBF29CE484222325ull;
  const uint8_t* p = (const uint8_t*)recs.data();
  for (size_t i = 0; i < recs.size() * 4; ++i) h = (h ^ p[i]) * 0x100000001B3ull;
  return h & 0x7FFFFFFFFFFFFFFFull;
}

static uint64_t align8(uint64_t x) { return (x + 7) & ~7ull; }

int64_t sst_wire_pack(sst_result* r, const int8_t* d_valid, int64_t n_valid, void* d_out, int64_t cap) {
  if (!r || n_valid < 0 || (n_valid > 0 && !d_valid) || (d_out && cap < 0)) return SST_E_ARG;
  sst_ctx* c = r->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  if (int rc = settle(r)) return rc;
  if (int rc = order_after_settle(r)) return rc;
  sst_table* t = r->pass.t;
  const uint64_t n_pair = r->scan_hits, n_exp = r->n_hits - r->scan_hits;
  const uint64_t xpay = r->payload_bytes - r->scan_bytes;
  if (r->n_hits < r->scan_hits || r->payload_bytes < r->scan_bytes)
    return fail(c, SST_E_INTERNAL, "wire pack: pair part larger than the result");
  if (n_valid >= (1ll << 30) || r->n >= (1ll << 30))
    return fail(c, SST_E_ARG, "wire pack: list entries index at most 2^30 queries");
  if (xpay >= (1ull << 32)) return fail(c, SST_E_ARG, "wire pack: explicit payload offsets are 32-bit");
  const uint64_t E = (n_pair && t) ? t->pair_recs.size() : 0;
  int w = 1;
  while (E > 1 && (1ull << w) < E) ++w;  // first entries are < E
  WireArgs a{};
  a.valid = d_valid;
  a.status = (const int8_t*)r->status.p;
  a.hits = (const uint4*)r->hits.p;
  a.refs = (const uint16_t*)r->refs.p;
  a.out = (uint8_t*)d_out;
  a.n7 = n_valid;
  a.n8 = r->n;
  a.n_pair = n_pair;
  a.n_exp = n_exp;
  a.pair_bytes = r->scan_bytes;
  a.w = w;
  a.nb_v = align8(((uint64_t)n_valid + 7) / 8);
  a.nb_s = align8(((uint64_t)r->n + 7) / 8);
  a.nw_f = (n_pair * w + 63) / 64 * 2;
  a.nw_c = (n_pair + 19) / 20 * 2;
  a.o_vbits = 8 * kWireHeaderWords;
  a.o_sbits = a.o_vbits + a.nb_v;
  a.o_first = a.o_sbits + a.nb_s;
  a.o_codes = a.o_first + 4 * a.nw_f;
  a.o_exp = a.o_codes + 4 * a.nw_c;
  const uint64_t o_pay = a.o_exp + align8(12 * n_exp);
  a.o_list = o_pay + align8(xpay);
  if (!d_out) return (int64_t)a.o_list;  // the fixed part's bytes: sizing only
  if ((uint64_t)cap < a.o_list) return fail(c, SST_E_ARG, "wire pack: buffer smaller than the fixed part");
  if ((uintptr_t)d_out & 7) return fail(c, SST_E_ARG, "wire pack: buffer not 8-byte aligned");
  a.list_cap = ((uint64_t)cap - a.o_list) / 8;
  if (n_pair && !t->pair_key_set) {
    t->pair_key = pair_key_of(t->pair_recs);
    t->pair_key_set = true;
  }
  const uint64_t hdr[kWireHeaderWords] = {kWireMagic, (uint64_t)n_valid, (uint64_t)r->n, n_pair, n_exp, xpay,
                                          (uint64_t)(r->rows_pass ? 0 : r->n_wg), n_pair ? t->pair_key : 0, (uint64_t)w, 0, a.list_cap,
                                          a.o_list, 0, 0, 0, 0};
  for (int k = 0; k < kWireHeaderWords; ++k) a.hdr[k] = hdr[k];
  auto blocks = [](uint64_t n) { return (uint32_t)((n + 255) / 256); };
  a.be_v = blocks(a.nb_v);
  a.be_s = a.be_v + blocks(a.nb_s);
  a.be_f = a.be_s + blocks(a.nw_f);
  a.be_c = a.be_f + blocks(a.nw_c);
  a.be_e = std::max<uint32_t>(1, a.be_c + blocks(n_exp));  // >= 1 block: the header
  uint8_t* out = (uint8_t*)d_out;
  HIP_OK(c, hipMemsetAsync(out + 8 * kWireListWord, 0, 8, c->stream));  // the list counter
  if (n_exp & 1) HIP_OK(c, hipMemsetAsync(out + a.o_exp + 12 * n_exp, 0, 4, c->stream));
  HIP_OK(c, launch_wire_pack(a, c->stream));
  if (xpay)
    HIP_OK(c, hipMemcpyAsync(out + o_pay, (const uint8_t*)r->dense.p + r->scan_bytes, xpay, hipMemcpyDeviceToDevice,
                             c->stream));
  if (align8(xpay) != xpay) HIP_OK(c, hipMemsetAsync(out + o_pay + xpay, 0, align8(xpay) - xpay, c->stream));
  return (int64_t)a.o_list;
}

int sst_result_fetch(sst_result* r) {
  if (!r) return SST_E_ARG;
  std::lock_guard<std::recursive_mutex> g(r->ctx->mu);
  if (int rc = set_device(r->ctx)) return rc;
  return fetch(r);
}

void sst_result_free(sst_result* r) {
  if (!r) return;
  std::lock_guard<std::recursive_mutex> g(r->ctx->mu);
  (void)hipSetDevice(r->ctx->device);
  (void)hipStreamSynchronize(r->ctx->stream);
  free_result_bufs(r);
  delete r;
}

int sst_result_stats(const sst_result* r, uint64_t* s) {
  if (!r || !s) return SST_E_ARG;
  for (int i = 0; i < kNumStats; ++i) s[i] = r->h_stats[i];
  return SST_OK;
}

int sst_profile_enable(sst_ctx* c, int on) { return sst_profile_select(c, on ? (1u << SST_K_COUNT) - 1u : 0u); }

int sst_profile_select(sst_ctx* c, uint32_t kernel_mask) {
  if (!c) return SST_E_ARG;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  prof_resolve(c);
  for (int i = 0; i < SST_K_COUNT; ++i) {
    c->prof_ms[i] = 0;
    c->prof_n[i] = 0;
    c->prof_seen[i] = 0;
  }
  c->prof = kernel_mask & ((1u << SST_K_COUNT) - 1u);
  return SST_OK;
}

int sst_profile_sample(sst_ctx* c, uint32_t every) {
  if (!c || every == 0) return SST_E_ARG;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  c->prof_every = every;
  for (int i = 0; i < SST_K_COUNT; ++i) c->prof_seen[i] = 0;
  return SST_OK;
}

int sst_profile_read(sst_ctx* c, double* ms, int64_t* n) {
  if (!c) return SST_E_ARG;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  prof_resolve(c);
  for (int i = 0; i < SST_K_COUNT; ++i) {
    if (ms) ms[i] = c->prof_ms[i];
    if (n) n[i] = c->prof_n[i];
    c->prof_ms[i] = 0;
    c->prof_n[i] = 0;
  }
  return SST_OK;
}


// sorted, de-duplicated copy of the caller's integer masses on the device
static int singleton_masses(sst_ctx* c, const int64_t* masses, int n_masses, DevBuf& d, int* n_unique) {
  if ((!masses && n_masses > 0) || n_masses < 0 || n_masses > kMaxSingletonMasses)
    return fail(c, SST_E_ARG, "is_singleton: 0..1024 integer masses");
  std::vector<int64_t> m(masses, masses + n_masses);
  std::sort(m.begin(), m.end());
  m.erase(std::unique(m.begin(), m.end()), m.end());
  if (!d.ensure(std::max<size_t>(1, m.size()) * 8)) return fail(c, SST_E_NOMEM, "device allocation failed");
  if (!m.empty()) HIP_OK(c, hipMemcpyAsync(d.p, m.data(), m.size() * 8, hipMemcpyHostToDevice, c->stream));
  HIP_OK(c, hipStreamSynchronize(c->stream));  // m is a host temporary
  *n_unique = (int)m.size();
  return SST_OK;
}

int sst_is_singleton_batch_device(sst_ctx* c, const int64_t* masses, int n_masses, const double* d_mass,
                                  const double* d_thr, int64_t n, double tol, double prec, int8_t* d_out) {
  if (!c || n < 0 || n > INT32_MAX || (n > 0 && (!d_mass || !d_out))) return SST_E_ARG;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  int nm = 0;
  if (int rc = singleton_masses(c, masses, n_masses, c->singleton_masses, &nm)) return rc;
  HIP_OK(c, launch_is_singleton((const int64_t*)c->singleton_masses.p, nm, d_mass, d_thr, n, tol, prec, d_out,
                                c->stream));
  return SST_OK;
}

int sst_is_singleton_batch(sst_ctx* c, const int64_t* masses, int n_masses, const double* mass, const double* thr,
                           int64_t n, double tol, double prec, int8_t* out) {
  if (!c || n < 0 || n > INT32_MAX || (n > 0 && (!mass || !out))) return SST_E_ARG;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  if (n == 0) return SST_OK;
  const size_t nn = (size_t)n;
  if (!c->in_mass.ensure(nn * 8) || (thr && !c->in_thr.ensure(nn * 8)) || !c->out_valid.ensure(nn))
    return fail(c, SST_E_NOMEM, "device allocation failed (staging)");
  HIP_OK(c, hipMemcpyAsync(c->in_mass.p, mass, nn * 8, hipMemcpyHostToDevice, c->stream));
  if (thr) HIP_OK(c, hipMemcpyAsync(c->in_thr.p, thr, nn * 8, hipMemcpyHostToDevice, c->stream));
  if (int rc = sst_is_singleton_batch_device(c, masses, n_masses, (const double*)c->in_mass.p,
                                             thr ? (const double*)c->in_thr.p : nullptr, n, tol, prec,
                                             (int8_t*)c->out_valid.p))
    return rc;
  HIP_OK(c, hipMemcpyAsync(out, c->out_valid.p, nn, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(c, hipStreamSynchronize(c->stream));
  return SST_OK;
}

// ---- per-spectrum reduced alphabets (sst_alpha.hip) --------------------
static int check_masks(sst_table* t) {
  if (t->n_rows > 120) return fail(t->ctx, SST_E_ARG, "alphabet masks cover 120 rows");
  return SST_OK;
}

// k_valid_alpha's shared start: the closure of the canonical rows over the
// table's masses [0, M), as u32 words (bit m: m is a sum of canonical rows).
// Host-built once per table (every row mass is >= 64, so word i depends only
// on earlier words).
static int canon_closure(sst_table* t, AlphaArgs& a) {
  sst_ctx* c = t->ctx;
  a.canon0 = a.canon1 = 0;
  std::vector<int64_t> cw;
  for (int r = 1; r < t->n_rows; ++r)
    if (!t->is_mod[r]) {
      (r < 64 ? a.canon0 : a.canon1) |= 1ull << (r & 63);
      cw.push_back(t->masses[r]);
    }
  a.canon_closure = nullptr;
  a.canon_words = 0;
  for (int64_t w : cw)
    if (w < 64) return SST_OK;  // not word-separable: every spectrum runs its whole closure
  if (!t->canon_c_words) {
    const int64_t nw = (t->M + 31) / 32;
    std::vector<uint32_t> bits((size_t)nw, 0u);
    auto get = [&](int64_t m) -> uint32_t {  // 32 bits from mass m on (m may be negative: zeros)
      if (m <= -32) return 0u;
      const int64_t wi = m >= 0 ? m / 32 : -1 - (-m - 1) / 32;
      const int s = (int)(m - wi * 32);
      const uint64_t lo = wi >= 0 ? bits[(size_t)wi] : 0u, hi = wi + 1 >= 0 && wi + 1 < nw ? bits[(size_t)wi + 1] : 0u;
      return (uint32_t)(((hi << 32) | lo) >> s);
    };
    for (int64_t i = 0; i < nw; ++i) {
      uint32_t v = i == 0 ? 1u : 0u;
      for (int64_t w : cw) v |= get(32 * i - w);
      bits[(size_t)i] = v;
    }
    if (!t->canon_c.ensure((size_t)nw * 4)) return fail(c, SST_E_NOMEM, "device allocation failed (canonical closure)");
    HIP_OK(c, hipMemcpy(t->canon_c.p, bits.data(), (size_t)nw * 4, hipMemcpyHostToDevice));
    t->canon_c_words = nw;
  }
  a.canon_closure = (const uint32_t*)t->canon_c.p;
  a.canon_words = t->canon_c_words;
  return SST_OK;
}

int sst_explain_pairs_alpha_device(sst_table* t, const double* d_mass, const double* d_thr, const int32_t* d_spec,
                                   const uint64_t* d_masks, int64_t n, double tol, double prec, int8_t* d_status,
                                   uint32_t* d_count, uint64_t* d_rowmask, uint32_t* d_range) {
  if (!t || n < 0 || n > SST_MAX_EXPLAIN_BATCH ||
      (n > 0 && (!d_mass || !d_spec || !d_masks || !d_status || !d_count || !d_rowmask || !d_range)))
    return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  if (int rc = check_masks(t)) return rc;
  if (!t->args.pairs_enabled) return fail(c, SST_E_ARG, "pairs on reduced alphabets: the table has no pair list");
  PairAlphaArgs a{d_mass, d_thr, d_spec, d_masks, n, tol, prec, 1.0 / prec, d_status, d_count, d_rowmask, d_range};
  Prof p(c, SST_K_PAIRS_ALPHA);
  HIP_OK(c, launch_pairs_alpha(t->args, a, c->stream));
  return SST_OK;
}

// host buffers in, host buffers out (synchronous); scratch on the device
struct Scratch {
  std::vector<DevBuf> b;
  void* get(size_t bytes) {
    b.emplace_back();
    return b.back().ensure(bytes ? bytes : 1) ? b.back().p : nullptr;
  }
  ~Scratch() {
    for (auto& x : b) x.release();
  }
};

int sst_explain_pairs_alpha(sst_table* t, const double* mass, const double* thr, const int32_t* spec,
                            const uint64_t* masks, int64_t n_spec, int64_t n, double tol, double prec, int8_t* status,
                            uint32_t* count, uint64_t* rowmask, uint32_t* range) {
  if (!t || n < 0 || n_spec < 0 || (n > 0 && (!mass || !spec || !masks || !status || !count || !rowmask || !range)))
    return SST_E_ARG;
  if (n == 0) return SST_OK;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  for (int64_t i = 0; i < n; ++i)
    if (spec[i] < 0 || spec[i] >= n_spec) return fail(c, SST_E_ARG, "pairs on reduced alphabets: spectrum id out of range");
  Scratch sc;
  void *dm = sc.get(n * 8), *dt = thr ? sc.get(n * 8) : nullptr, *ds = sc.get(n * 4), *dk = sc.get(n_spec * 16);
  void *o1 = sc.get(n), *o2 = sc.get(n * 4), *o3 = sc.get(n * 16), *o4 = sc.get(n * 8);
  if (!dm || (thr && !dt) || !ds || !dk || !o1 || !o2 || !o3 || !o4)
    return fail(c, SST_E_NOMEM, "device allocation failed (pairs on reduced alphabets)");
  HIP_OK(c, hipMemcpyAsync(dm, mass, n * 8, hipMemcpyHostToDevice, c->stream));
  if (thr) HIP_OK(c, hipMemcpyAsync(dt, thr, n * 8, hipMemcpyHostToDevice, c->stream));
  HIP_OK(c, hipMemcpyAsync(ds, spec, n * 4, hipMemcpyHostToDevice, c->stream));
  HIP_OK(c, hipMemcpyAsync(dk, masks, n_spec * 16, hipMemcpyHostToDevice, c->stream));
  if (int rc = sst_explain_pairs_alpha_device(t, (const double*)dm, (const double*)dt, (const int32_t*)ds,
                                              (const uint64_t*)dk, n, tol, prec, (int8_t*)o1, (uint32_t*)o2,
                                              (uint64_t*)o3, (uint32_t*)o4))
    return rc;
  HIP_OK(c, hipMemcpyAsync(status, o1, n, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(c, hipMemcpyAsync(count, o2, n * 4, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(c, hipMemcpyAsync(rowmask, o3, n * 16, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(c, hipMemcpyAsync(range, o4, n * 8, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(c, hipStreamSynchronize(c->stream));
  return SST_OK;
}

int sst_is_valid_alpha_device(sst_table* t, const double* d_mass, const double* d_thr, const int64_t* d_offsets,
                              int64_t n_spec, const uint64_t* d_masks, double tol, double prec, int8_t* d_out) {
  if (!t || n_spec < 0 || n_spec > INT32_MAX || (n_spec > 0 && (!d_mass || !d_offsets || !d_masks || !d_out)))
    return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  if (int rc = check_masks(t)) return rc;
  AlphaArgs a{};
  a.mass = d_mass;
  a.thr = d_thr;
  a.offsets = d_offsets;
  a.masks = d_masks;
  a.w = t->args.w;
  a.n_rows = t->n_rows;
  a.tol = tol;
  a.prec = prec;
  a.rprec = 1.0 / prec;
  a.out = d_out;
  if (int rc = canon_closure(t, a)) return rc;
  Prof p(c, SST_K_VALID_ALPHA);
  HIP_OK(c, launch_valid_alpha(a, n_spec, c->stream));
  return SST_OK;
}

// ---- config 5 on the device (sst_pipe.hip) ---------------------------
static int pipe_args(sst_table* t, const double* d_obs, const int64_t* d_peak_off, int64_t n_spec, int64_t n_peaks,
                     const double* d_intensity, double intensity_cutoff, double mass_cutoff, const double* d_su_seq,
                     const double* shifts, const uint8_t* sides, int n_shifts, double max_weight, double tol,
                     double prec, PipeArgs& a) {
  if (!t || n_spec < 0 || n_spec > INT32_MAX || n_peaks < 0 || n_shifts < 1 || n_shifts > 4 || !shifts || !sides ||
      (n_spec > 0 && (!d_obs || !d_peak_off || !d_su_seq)))
    return SST_E_ARG;
  if (!t->args.pairs_enabled) return fail(t->ctx, SST_E_ARG, "pipeline: the table has no pair list");
  const double hi_max = (max_weight + tol * 2.0 * mass_cutoff) / prec + 2.0;
  if (!(hi_max < (double)t->args.pair_hi))
    return fail(t->ctx, SST_E_ARG, "pipeline: windows may leave the pair class (max_weight / mass_cutoff too large)");
  a = PipeArgs{};
  a.obs = d_obs;
  a.peak_off = d_peak_off;
  a.n_spec = n_spec;
  a.n_peaks = n_peaks;
  a.intensity = d_intensity;
  a.intensity_cutoff = intensity_cutoff;
  a.mass_cutoff = mass_cutoff;
  a.max_variance = 1.0;  // fragment_classification.py:8
  a.su_seq = d_su_seq;
  for (int k = 0; k < n_shifts; ++k) {
    a.shift[k] = shifts[k];
    a.sides[k] = sides[k];
  }
  a.n_shifts = n_shifts;
  a.max_weight = max_weight;
  a.tol = tol;
  a.prec = prec;
  a.rprec = 1.0 / prec;
  for (int r = 1; r < t->n_rows; ++r)
    if (!t->is_mod[r]) a.canon[r >> 6] |= 1ull << (r & 63);
  return SST_OK;
}

// the context's big-spectrum slices into the stage's arguments (none reserved:
// a spectrum of more than kPipeMaxRows rows is reported, bit 2)
static void big_args(sst_ctx* c, sst::PipeArgs& a) {
  if (!c->pipe_big_rows) return;
  a.big = (uint8_t*)c->pipe_big.p;
  a.big_rows = c->pipe_big_rows;
  a.big_slots = c->pipe_big_slots;
  a.big_stride = sst::pipe_big_layout(a.big_rows, a.big_slots).stride;
  a.big_wg = c->pipe_big_wg;
}

int sst_classify_rows_device(sst_table* t, const double* d_obs, const int64_t* d_peak_off, int64_t n_spec,
                             int64_t n_peaks, const double* d_intensity, double intensity_cutoff, double mass_cutoff,
                             const double* d_su_seq, const double* shifts, const uint8_t* sides, int n_shifts,
                             double max_weight, double tol, double prec, int8_t* d_valid_out, double* d_rows_su,
                             double* d_rows_ob, uint32_t* d_rows_meta, uint8_t* d_alive, uint32_t* d_rows,
                             uint32_t* d_err) {
  PipeArgs a;
  if (int rc = pipe_args(t, d_obs, d_peak_off, n_spec, n_peaks, d_intensity, intensity_cutoff, mass_cutoff, d_su_seq,
                         shifts, sides, n_shifts, max_weight, tol, prec, a))
    return rc;
  if (n_spec > 0 && (!d_rows_su || !d_rows_ob || !d_rows_meta || !d_alive || !d_rows || !d_err)) return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  if (!c->singleton_masses.ensure((size_t)t->n_rows * 8)) return fail(c, SST_E_NOMEM, "device allocation failed");
  HIP_OK(c, hipMemcpyAsync(c->singleton_masses.p, t->masses.data(), (size_t)t->n_rows * 8, hipMemcpyHostToDevice,
                           c->stream));
  a.masses = (const int64_t*)c->singleton_masses.p;
  a.n_masses = t->n_rows;
  a.valid_out = d_valid_out;
  a.r_su = d_rows_su;
  a.r_ob = d_rows_ob;
  a.r_meta = d_rows_meta;
  a.alive = d_alive;
  a.cnt = d_rows;
  a.err = d_err;
  big_args(c, a);  // spectra of more than kPipeMaxPeaks peaks: k_classify_rows_big in the reserved slices
  Prof p(c, SST_K_CLASSIFY_ROWS);
  HIP_OK(c, launch_classify_rows(t->args, a, c->n_cu, c->stream));
  return SST_OK;
}

// the exact-mode arrays (sst_exact_io) into the stage's arguments
static int exact_io(sst_ctx* c, const sst_exact_io* x, sst::PipeArgs& a) {
  if (!x) return SST_OK;
  if (!x->pair_ok || !x->xq_mass || !x->xq_thr || !x->xq_spec || !x->xq_single || !x->xq_count || !x->xq_block)
    return fail(c, SST_E_ARG, "exact-mode arrays");
  a.pair_ok = x->pair_ok;
  a.xq_mass = x->xq_mass;
  a.xq_thr = x->xq_thr;
  a.xq_spec = x->xq_spec;
  a.xq_single = x->xq_single;
  a.xq_count = x->xq_count;
  a.xq_cap = x->xq_cap;
  a.xq_block = x->xq_block;
  a.xa_st = x->xa_st;
  a.xa_n = x->xa_n;
  a.xa_ptr = x->xa_ptr;
  return SST_OK;
}


int sst_requery_merge_device(sst_table* t, const sst_requery_merge_args* args, uint32_t* d_tot, uint64_t* d_off) {
  if (!t || !args || args->n_sides < 0 || (args->n_sides > 0 && (!args->block || !args->m_block || !d_tot || !d_off)))
    return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  Prof p(c, SST_K_REQUERY_MERGE);
  HIP_OK(c, sst::launch_requery_merge(*args, d_tot, d_off, c->stream));
  return SST_OK;
}

int sst_pipe_reserve_rows(sst_table* t, int64_t max_rows) {
  if (!t || max_rows < 0) return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (max_rows <= kPipeMaxRows || (uint32_t)max_rows <= c->pipe_big_rows) return SST_OK;
  if (max_rows > kPipeBigRows)
    return fail(c, SST_E_ARG, "pipeline: more than " + std::to_string(kPipeBigRows) + " rows per spectrum");
  if (int rc = set_device(c)) return rc;
  const uint32_t rows = (uint32_t)max_rows;
  uint32_t slots = 1u << 15;  // the dict hash: >= 16 slots per row (writers <= 3/4 of them)
  while (slots < 16u * rows) slots <<= 1;
  const int wg = std::max(1, std::min(c->n_cu, 32));
  const uint64_t bytes = sst::pipe_big_layout(rows, slots).stride * (uint64_t)wg;
  HIP_OK(c, hipStreamSynchronize(c->stream));  // earlier launches may still read the old slices
  if (!c->pipe_big.ensure(bytes)) return fail(c, SST_E_NOMEM, "device allocation failed");
  c->pipe_big_rows = rows;
  c->pipe_big_slots = slots;
  c->pipe_big_wg = wg;
  return SST_OK;
}

int sst_fix_round_device(sst_table* t, const int64_t* d_peak_off, int64_t n_spec, const double* d_rows_su,
                         const double* d_rows_ob, const uint32_t* d_rows_meta, uint8_t* d_alive,
                         const uint32_t* d_rows, const uint64_t* d_alpha, uint64_t* d_alpha_next,
                         const uint8_t* d_active, uint8_t* d_active_next, uint32_t* d_rounds, uint32_t* d_queries,
                         uint32_t* d_n_active, double max_weight, double tol, double prec, uint32_t* d_err,
                         const sst_exact_io* x) {
  const double zero_shift = 0.0;
  const uint8_t zero_side = 0;
  PipeArgs a;
  if (int rc = pipe_args(t, d_rows_su, d_peak_off, n_spec, 0, nullptr, 0.0, 0.0, d_rows_su, &zero_shift,
                         &zero_side, 1, max_weight, tol, prec, a))
    return rc;
  if (n_spec > 0 && (!d_rows_ob || !d_rows_meta || !d_alive || !d_rows || !d_alpha || !d_alpha_next || !d_active ||
                     !d_active_next || !d_rounds || !d_queries || !d_n_active || !d_err))
    return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  if (int rc = check_masks(t)) return rc;
  a.r_su = const_cast<double*>(d_rows_su);
  a.r_ob = const_cast<double*>(d_rows_ob);
  a.r_meta = const_cast<uint32_t*>(d_rows_meta);
  a.alive = d_alive;
  a.cnt = const_cast<uint32_t*>(d_rows);
  a.alpha = d_alpha;
  a.alpha_next = d_alpha_next;
  a.active = d_active;
  a.active_next = d_active_next;
  a.rounds = d_rounds;
  a.queries = d_queries;
  a.n_active = d_n_active;
  a.err = d_err;
  if (int rc = exact_io(c, x, a)) return rc;
  if (n_spec > 0) HIP_OK(c, hipMemsetAsync(d_n_active, 0, sizeof(uint32_t), c->stream));  // this round's count
  big_args(c, a);
  Prof p(c, SST_K_FIX_ROUND);
  HIP_OK(c, launch_fix_round(t->args, a, c->n_cu, c->stream));
  return SST_OK;
}

static int bins_args(sst_table* t, const int64_t* d_peak_off, int64_t n_spec, const double* d_rows_su,
                     const double* d_rows_ob, const uint32_t* d_rows_meta, const uint8_t* d_alive,
                     const uint32_t* d_rows, double tol, double prec, uint64_t* d_q_off, uint32_t* d_err, PipeArgs& a) {
  if (!t || n_spec < 0 || n_spec > INT32_MAX || !d_q_off ||
      (n_spec > 0 && (!d_peak_off || !d_rows_su || !d_rows_ob || !d_rows_meta || !d_alive || !d_rows || !d_err)))
    return SST_E_ARG;
  if (!t->args.pairs_enabled) return fail(t->ctx, SST_E_ARG, "skeleton bins: the table has no pair list");
  a = PipeArgs{};
  a.peak_off = d_peak_off;
  a.n_spec = n_spec;
  a.r_su = const_cast<double*>(d_rows_su);
  a.r_ob = const_cast<double*>(d_rows_ob);
  a.r_meta = const_cast<uint32_t*>(d_rows_meta);
  a.alive = const_cast<uint8_t*>(d_alive);
  a.cnt = const_cast<uint32_t*>(d_rows);
  a.tol = tol;
  a.prec = prec;
  a.rprec = 1.0 / prec;
  a.q_off = d_q_off;
  a.err = d_err;
  return SST_OK;
}

int sst_bins_count_device(sst_table* t, const int64_t* d_peak_off, int64_t n_spec, const double* d_rows_su,
                          const double* d_rows_ob, const uint32_t* d_rows_meta, const uint8_t* d_alive,
                          const uint32_t* d_rows, double tol, uint32_t* d_n_q, uint64_t* d_q_off, uint32_t* d_err,
                          uint32_t* d_n_q0) {
  PipeArgs a;
  if (int rc = bins_args(t, d_peak_off, n_spec, d_rows_su, d_rows_ob, d_rows_meta, d_alive, d_rows, tol, 1.0,
                         d_q_off, d_err, a))
    return rc;
  if (n_spec > 0 && !d_n_q) return SST_E_ARG;
  a.n_q = d_n_q;
  a.n_q0 = d_n_q0;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  big_args(c, a);
  Prof p(c, SST_K_BINS_COUNT);
  HIP_OK(c, launch_bins_count(a, c->n_cu, c->stream));
  return SST_OK;
}

int sst_bins_emit_device(sst_table* t, const int64_t* d_peak_off, int64_t n_spec, const double* d_rows_su,
                         const double* d_rows_ob, const uint32_t* d_rows_meta, const uint8_t* d_alive,
                         const uint32_t* d_rows, const uint64_t* d_alpha, double tol, double prec,
                         const uint64_t* d_q_off, int8_t* d_status, uint32_t* d_count, double* d_def_mass,
                         double* d_def_thr, int32_t* d_def_spec, uint64_t* d_def_q, uint32_t* d_n_def,
                         uint32_t* d_err, const uint8_t* d_pair_ok) {
  PipeArgs a;
  if (int rc = bins_args(t, d_peak_off, n_spec, d_rows_su, d_rows_ob, d_rows_meta, d_alive, d_rows, tol, prec,
                         const_cast<uint64_t*>(d_q_off), d_err, a))
    return rc;
  if (n_spec > 0 && (!d_alpha || !d_status || !d_count)) return SST_E_ARG;
  a.alpha = d_alpha;
  a.q_status = d_status;
  a.q_count = d_count;
  if (d_n_def && (!d_def_mass || !d_def_thr || !d_def_spec || !d_def_q)) return SST_E_ARG;
  a.def_mass = d_def_mass;
  a.def_thr = d_def_thr;
  a.def_spec = d_def_spec;
  a.def_q = d_def_q;
  a.n_def = d_n_def;
  a.pair_ok = d_pair_ok;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  if (int rc = check_masks(t)) return rc;
  big_args(c, a);
  Prof p(c, SST_K_BINS_EMIT);
  HIP_OK(c, launch_bins_emit(t->args, a, c->n_cu, c->stream));
  return SST_OK;
}

int sst_valid_rows_alpha_device(sst_table* t, const int64_t* d_peak_off, int64_t n_spec, const double* d_rows_su,
                                const double* d_rows_ob, const uint32_t* d_rows, const uint64_t* d_alpha,
                                const uint8_t* d_active, uint8_t* d_alive, double tol, double prec, uint32_t* d_err) {
  if (!t || n_spec < 0 || n_spec > INT32_MAX ||
      (n_spec > 0 && (!d_peak_off || !d_rows_su || !d_rows_ob || !d_rows || !d_alpha || !d_alive || !d_err)))
    return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  if (int rc = check_masks(t)) return rc;
  AlphaArgs a{};
  a.mass = d_rows_su;
  a.thr_obs = d_rows_ob;  // the rows' thresholds: tolerance * observed mass (prediction.py:219)
  a.offsets = d_peak_off;
  a.counts = d_rows;
  a.masks = d_alpha;
  a.active = d_active;
  a.alive = d_alive;
  a.err = d_err;
  a.w = t->args.w;
  a.n_rows = t->n_rows;
  a.tol = tol;
  a.prec = prec;
  a.rprec = 1.0 / prec;
  if (int rc = canon_closure(t, a)) return rc;
  Prof p(c, SST_K_VALID_ALPHA);
  HIP_OK(c, launch_valid_alpha(a, n_spec, c->stream));
  return SST_OK;
}

int sst_is_valid_alpha(sst_table* t, const double* mass, const double* thr, const int64_t* offsets, int64_t n_spec,
                       const uint64_t* masks, double tol, double prec, int8_t* out) {
  if (!t || n_spec < 0 || (n_spec > 0 && (!offsets || !masks))) return SST_E_ARG;
  if (n_spec == 0) return SST_OK;
  const int64_t n = offsets[n_spec];
  if (offsets[0] != 0 || n < 0 || (n > 0 && (!mass || !out))) return SST_E_ARG;
  for (int64_t g = 0; g < n_spec; ++g)
    if (offsets[g + 1] < offsets[g]) return SST_E_ARG;
  if (n == 0) return SST_OK;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  Scratch sc;
  void *dm = sc.get(n * 8), *dt = thr ? sc.get(n * 8) : nullptr, *doff = sc.get((n_spec + 1) * 8),
       *dk = sc.get(n_spec * 16), *dout = sc.get(n);
  if (!dm || (thr && !dt) || !doff || !dk || !dout)
    return fail(c, SST_E_NOMEM, "device allocation failed (is_valid on reduced alphabets)");
  HIP_OK(c, hipMemcpyAsync(dm, mass, n * 8, hipMemcpyHostToDevice, c->stream));
  if (thr) HIP_OK(c, hipMemcpyAsync(dt, thr, n * 8, hipMemcpyHostToDevice, c->stream));
  HIP_OK(c, hipMemcpyAsync(doff, offsets, (n_spec + 1) * 8, hipMemcpyHostToDevice, c->stream));
  HIP_OK(c, hipMemcpyAsync(dk, masks, n_spec * 16, hipMemcpyHostToDevice, c->stream));
  if (int rc = sst_is_valid_alpha_device(t, (const double*)dm, (const double*)dt, (const int64_t*)doff, n_spec,
                                         (const uint64_t*)dk, tol, prec, (int8_t*)dout))
    return rc;
  HIP_OK(c, hipMemcpyAsync(out, dout, n, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(c, hipStreamSynchronize(c->stream));
  return SST_OK;
}

}  // extern "C"
static int lbf_frontier(sst_table* t, sst_ctx::LbfWs& W, const double* d_su, const double* d_obs,
                        const int32_t* d_spec, const uint64_t* d_alpha, const uint8_t* d_lr, const uint64_t* d_lr_off,
                        int64_t n, double tol, double prec, int max_len, int64_t max_mods, int64_t* d_lower,
                        int64_t* d_upper, int8_t* d_status, const int32_t* d_qlen, const int32_t* d_caps_len,
                        const int32_t* d_a0_len, uint64_t* d_nodes, uint64_t workspace_bytes, sst_lbf_stats* stats);
namespace {
constexpr uint64_t kBatchFrontierBytes = 4ull << 30;  // sst_length_bound_batch's frontier workspace

static int length_bound_batch(sst_table* t, const double* su, const double* obs, int64_t n, double tol, double prec,
                              int max_len, int64_t max_mods, int direction, int64_t* out, int8_t* status,
                              const int32_t* spec, const uint64_t* alpha, int64_t n_alpha) {
  const bool exact_only = (direction & SST_LB_EXACT_ONLY) != 0;
  const bool replay_only = (direction & SST_LB_REPLAY) != 0;
  direction &= ~(SST_LB_EXACT_ONLY | SST_LB_REPLAY);
  if (!t || n < 0 || n > INT32_MAX || (n > 0 && (!su || !obs || !out || !status)) || (direction != 0 && direction != 1) ||
      max_len < 0 || max_len > 253)
    return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  if (n == 0) return SST_OK;
  const size_t nn = (size_t)n;
  DevBuf d_su, d_obs, d_out, d_st, d_list, d_cnt, layers, d_spec, d_alpha;
  if (!d_su.ensure(nn * 8) || !d_obs.ensure(nn * 8) || !d_out.ensure(nn * 8) || !d_st.ensure(nn) ||
      !d_list.ensure(nn * 4) || !d_cnt.ensure(4))
    return fail(c, SST_E_NOMEM, "device allocation failed (length bound)");
  if (alpha) {
    for (int64_t i = 0; spec && i < n; ++i)
      if (spec[i] < 0 || spec[i] >= n_alpha) return fail(c, SST_E_ARG, "length bound: alphabet index out of range");
    if (!d_alpha.ensure((size_t)n_alpha * 16) || (spec && !d_spec.ensure(nn * 4)))
      return fail(c, SST_E_NOMEM, "device allocation failed (length bound alphabets)");
    HIP_OK(c, hipMemcpyAsync(d_alpha.p, alpha, (size_t)n_alpha * 16, hipMemcpyHostToDevice, c->stream));
    if (spec) HIP_OK(c, hipMemcpyAsync(d_spec.p, spec, nn * 4, hipMemcpyHostToDevice, c->stream));
  }
  HIP_OK(c, hipMemcpyAsync(d_su.p, su, nn * 8, hipMemcpyHostToDevice, c->stream));
  HIP_OK(c, hipMemcpyAsync(d_obs.p, obs, nn * 8, hipMemcpyHostToDevice, c->stream));
  HIP_OK(c, hipMemsetAsync(d_cnt.p, 0, 4, c->stream));
  LBArgs q{};
  q.su = (const double*)d_su.p;
  q.obs = (const double*)d_obs.p;
  q.n = n;
  q.tol = tol;
  q.prec = prec;
  q.rprec = 1.0 / prec;
  q.A0 = (int)std::max<int64_t>(0, std::min<int64_t>(max_mods, kInfBudget));  // round(rate * max_len) >= 0
  q.dir = direction;
  q.max_len = max_len;
  q.out = (int64_t*)d_out.p;
  q.status = (int8_t*)d_st.p;
  q.exact_list = (uint32_t*)d_list.p;
  q.exact_count = (uint32_t*)d_cnt.p;
  q.node_budget = kLBNodeBudget;
  q.alpha = alpha ? (const uint64_t*)d_alpha.p : nullptr;
  q.spec = alpha && spec ? (const int32_t*)d_spec.p : nullptr;
  q.comp = (int)t->C;
  // fast path: layered reachability up to the largest window (a host-side
  // over-estimate; the kernel re-checks hi < layer_limit exactly), kept below
  // the reference's masked last column
  if (t->closure && t->args.w_min > 0 && !exact_only && !alpha) {
    double hmax = 0;
    for (int64_t i = 0; i < n; ++i) hmax = std::max(hmax, (su[i] + tol * std::fabs(obs[i])) / prec + 4.0);
    const int64_t safe = (t->n_cols - 1) * t->C;
    const int64_t lim = std::min<int64_t>(safe, (int64_t)std::min(hmax, (double)safe));
    if (lim > 0) {
      const int64_t words = (lim + 63) / 64;
      const int n_layers = (int)(lim / t->args.w_min) + 2;
      if (!layers.ensure((size_t)n_layers * words * 8)) return fail(c, SST_E_NOMEM, "device allocation failed (layers)");
      uint64_t* L = (uint64_t*)layers.p;
      const uint64_t one = 1;
      HIP_OK(c, hipMemsetAsync(L, 0, (size_t)words * 8, c->stream));
      HIP_OK(c, hipMemcpyAsync(L, &one, 8, hipMemcpyHostToDevice, c->stream));
      for (int k = 0; k + 1 < n_layers; ++k)
        HIP_OK(c, launch_layer_step(L + (size_t)k * words, L + (size_t)(k + 1) * words, words, t->args.w, t->n_rows,
                                    c->stream));
      q.layers = L;
      q.layer_words = words;
      q.n_layers = n_layers;
      q.layer_limit = lim;
    }
  }
  // fast kernel (queues the rest), then the exact kernel; retried with a
  // larger per-lane memo while any query reports hash exhaustion
  uint32_t n_exact = 0;
  {
    Prof p(c, SST_K_LENGTH_BOUND);
    HIP_OK(c, launch_length_bound(t->args, q, nullptr, nullptr, nullptr, 0, 0, true, c->stream));
  }
  HIP_OK(c, hipMemcpyAsync(&n_exact, d_cnt.p, 4, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(c, hipStreamSynchronize(c->stream));
  std::vector<int8_t> st(nn);
  DevBuf f_alpha, f_words, f_off, f_bits, f_lr, f_lro, f_spec, f_lo, f_hi, f_st;
  bool frontier_ok = t->closure && !alpha && !replay_only && t->args.w_min >= 1024;  // (the reach rows' LDS ring)
  int64_t w_top = 0;
  for (int r = 1; r < t->n_rows && frontier_ok; ++r) {
    frontier_ok = t->masses[r] < (1 << 20);
    w_top = std::max<int64_t>(w_top, t->masses[r]);
  }
  // the frontier applies the reduced-alphabet extent ceil((w_top * 35 + 1) / C) * C
  // (mass_table.py:116): only a table of exactly that extent (every table built
  // here, the reference's cache) is answered by it; an uploaded table of another
  // extent goes to the replay, which reads the table's own
  frontier_ok = frontier_ok && (w_top * 35 + t->C) / t->C == t->n_cols;
  if (n_exact && frontier_ok) {
    // the first-visit frontier on the table's own rows, both
    // directions, for the queries the fast path left pending only (its own
    // answers stay); a window in the table's last packed word, where the
    // frontier's reachability cannot see the last-column mask (SST_ABORTED
    // there), or one the frontier's layout cannot hold, goes on to the replay
    const size_t m = n_exact;
    std::vector<uint32_t> pend(m);
    HIP_OK(c, hipMemcpyAsync(pend.data(), d_list.p, m * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(c, hipStreamSynchronize(c->stream));
    std::vector<double> psu(m), pob(m);
    int64_t hmax = 1;
    for (size_t j = 0; j < m; ++j) {
      psu[j] = su[pend[j]];
      pob[j] = obs[pend[j]];
      hmax = std::max<int64_t>(hmax, (int64_t)((psu[j] + tol * std::fabs(pob[j])) / prec) + 4);
    }
    hmax = std::min<int64_t>(hmax, t->n_cols * t->C);
    const int64_t words = hmax / 32 + 2;
    uint64_t am[2] = {0, 0};
    for (int r = 1; r < t->n_rows; ++r) am[r >> 6] |= 1ull << (r & 63);
    const int64_t zero = 0;
    const size_t K = (size_t)(t->n_rows - 1);
    DevBuf f_su, f_ob;
    if (!f_alpha.ensure(16) || !f_words.ensure(8) || !f_off.ensure(8) || !f_bits.ensure(K * words * 4) ||
        !f_lr.ensure((size_t)words * 32) || !f_lro.ensure(8) || !f_spec.ensure(m * 4) || !f_lo.ensure(m * 8) ||
        !f_hi.ensure(m * 8) || !f_st.ensure(m) || !f_su.ensure(m * 8) || !f_ob.ensure(m * 8))
      return fail(c, SST_E_NOMEM, "device allocation failed (length bound, frontier)");
    HIP_OK(c, hipMemcpyAsync(f_alpha.p, am, 16, hipMemcpyHostToDevice, c->stream));
    HIP_OK(c, hipMemcpyAsync(f_words.p, &words, 8, hipMemcpyHostToDevice, c->stream));
    HIP_OK(c, hipMemcpyAsync(f_off.p, &zero, 8, hipMemcpyHostToDevice, c->stream));
    HIP_OK(c, hipMemcpyAsync(f_lro.p, &zero, 8, hipMemcpyHostToDevice, c->stream));
    HIP_OK(c, hipMemcpyAsync(f_su.p, psu.data(), m * 8, hipMemcpyHostToDevice, c->stream));
    HIP_OK(c, hipMemcpyAsync(f_ob.p, pob.data(), m * 8, hipMemcpyHostToDevice, c->stream));
    HIP_OK(c, hipMemsetAsync(f_spec.p, 0, m * 4, c->stream));
    if (int rc = sst_reach_rows_device(t, (const uint64_t*)f_alpha.p, (const int64_t*)f_words.p,
                                       (const uint64_t*)f_off.p, 1, (uint32_t*)f_bits.p))
      return rc;
    if (int rc = sst_reach_lowest_device(t, (const uint64_t*)f_alpha.p, (const int64_t*)f_words.p,
                                         (const uint64_t*)f_off.p, 1, (const uint32_t*)f_bits.p,
                                         (const uint64_t*)f_lro.p, (uint8_t*)f_lr.p))
      return rc;
    if (int rc = lbf_frontier(t, c->lbf_small, (const double*)f_su.p, (const double*)f_ob.p,
                              (const int32_t*)f_spec.p, (const uint64_t*)f_alpha.p, (const uint8_t*)f_lr.p,
                              (const uint64_t*)f_lro.p, (int64_t)m, tol, prec, max_len, max_mods, (int64_t*)f_lo.p,
                              (int64_t*)f_hi.p, (int8_t*)f_st.p, nullptr, nullptr, nullptr, nullptr, kBatchFrontierBytes,
                              nullptr))
      return rc;
    // scatter the frontier's answers over the fast pass's (host copies: nn x 9 bytes)
    std::vector<int64_t> fv(m), ov(nn);
    std::vector<int8_t> fs(m);
    HIP_OK(c, hipMemcpyAsync(fv.data(), direction ? f_hi.p : f_lo.p, m * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(c, hipMemcpyAsync(fs.data(), f_st.p, m, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(c, hipMemcpyAsync(ov.data(), d_out.p, nn * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(c, hipMemcpyAsync(st.data(), d_st.p, nn, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(c, hipStreamSynchronize(c->stream));
    std::vector<uint32_t> rest;
    for (size_t j = 0; j < m; ++j) {
      ov[pend[j]] = fv[j];
      st[pend[j]] = fs[j];
      if (fs[j] == SST_ABORTED) rest.push_back(pend[j]);
    }
    HIP_OK(c, hipMemcpyAsync(d_out.p, ov.data(), nn * 8, hipMemcpyHostToDevice, c->stream));
    HIP_OK(c, hipMemcpyAsync(d_st.p, st.data(), nn, hipMemcpyHostToDevice, c->stream));
    n_exact = (uint32_t)rest.size();
    if (n_exact) {
      HIP_OK(c, hipMemcpyAsync(d_list.p, rest.data(), rest.size() * 4, hipMemcpyHostToDevice, c->stream));
      HIP_OK(c, hipMemcpyAsync(d_cnt.p, &n_exact, 4, hipMemcpyHostToDevice, c->stream));
    }
    HIP_OK(c, hipStreamSynchronize(c->stream));  // the host vectors above are read by the copies
  }
  if (n_exact && max_len > 120)  // the frontier answers up to 253; the replay's int8 value slots hold 121
    return fail(c, SST_E_ARG,
                "length bound: max_len " + std::to_string(max_len) + " above 120 for a window only the DFS replay "
                "answers (the table's last packed word, or beyond the frontier's layout)");
  if (n_exact) {
    // one 64-lane block per query in flight (k_length_exact<WAVE>), each with
    // its own memo slice: up to 1 024 at once (4 waves per CU; the memo slices
    // then take ~10 GB of HBM), batches of many spectra keep the chip busy
    int units = (int)std::min<uint32_t>(1024, n_exact);
    uint32_t cap = memo_cap0(units, kLBHashCap0);
    for (;;) {
      DevBuf hash, vals, frames;
      if (!hash.ensure((size_t)units * cap * hash_entry_bytes()) || !vals.ensure((size_t)units * cap * kMaxRows) ||
          !frames.ensure((size_t)units * lb_frame_bytes()))
        return fail(c, SST_E_NOMEM, "device allocation failed (length-bound memo)");
      HIP_OK(c, hipMemsetAsync(hash.p, 0, hash.bytes, c->stream));
      Prof p(c, SST_K_LENGTH_BOUND);
      HIP_OK(c, launch_length_bound(t->args, q, (char*)hash.p, (int8_t*)vals.p, (char*)frames.p, cap, units, false,
                                    c->stream));
      HIP_OK(c, hipMemcpyAsync(st.data(), d_st.p, nn, hipMemcpyDeviceToHost, c->stream));
      HIP_OK(c, hipStreamSynchronize(c->stream));
      bool retry = false;
      for (size_t i = 0; i < nn; ++i) retry |= st[i] == kStatusExactRetry;
      if (!retry) break;
      if ((size_t)std::max(1, units / 8) * cap * 8 * (hash_entry_bytes() + kMaxRows) > kMaxMemoBytes)
        return fail(c, SST_E_NOMEM, "length bound: memo would exceed the workspace limit");
      cap *= 8;
      units = std::max(1, units / 8);
    }
  }
  HIP_OK(c, hipMemcpyAsync(out, d_out.p, nn * 8, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(c, hipMemcpyAsync(status, d_st.p, nn, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(c, hipStreamSynchronize(c->stream));
  for (size_t i = 0; i < nn; ++i)
    if (status[i] == kStatusPending || status[i] == kStatusExactRetry)
      return fail(c, SST_E_INTERNAL, "length bound: query left unresolved (internal error)");
  return SST_OK;
}

}  // namespace
extern "C" {

int sst_length_bound_batch(sst_table* t, const double* su, const double* obs, int64_t n, double tol, double prec,
                           int max_len, int64_t max_mods, int direction, int64_t* out, int8_t* status) {
  return length_bound_batch(t, su, obs, n, tol, prec, max_len, max_mods, direction, out, status, nullptr, nullptr,
                            0);
}

int sst_length_bound_alpha_batch(sst_table* t, const double* su, const double* obs, const int32_t* spec,
                                 const uint64_t* alpha, int64_t n_alpha, int64_t n, double tol, double prec,
                                 int max_len, int64_t max_mods, int direction, int64_t* out, int8_t* status) {
  // "lower" only: a left child that is reachable in the full table but not with
  // the kept rows returns the default (-1) there, and the reference's upper
  // bound counts such a visited child as -1 + 1 = 0 where the rebuilt table
  // would not visit it at all; the lower bound's default (max_len
  // + 1) can never win a min, so its masked replay is exact
  if (!alpha || n_alpha <= 0 || (direction & ~SST_LB_EXACT_ONLY) != 0) return SST_E_ARG;
  return length_bound_batch(t, su, obs, n, tol, prec, max_len, max_mods, direction, out, status, spec, alpha,
                            n_alpha);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Query producers (host): the sliding window of collect_explanations_per_side
// (prediction.py:286-329), the same state machine over every side.
// ---------------------------------------------------------------------------
int64_t sst_window_pairs(const double* su, const int64_t* offsets, int64_t n_sides, double max_weight,
                         int64_t* start_out, int64_t* end_out, int64_t cap) {
  if (n_sides < 0 || (n_sides > 0 && (!su || !offsets)) || cap < 0 || (cap > 0 && (!start_out || !end_out)))
    return SST_E_ARG;
  int64_t k = 0;
  for (int64_t j = 0; j < n_sides; ++j) {
    const int64_t b = offsets[j], n = offsets[j + 1] - offsets[j];
    if (n < 0) return SST_E_ARG;
    int64_t start = 0, end = 1;
    while (end < n) {
      if (end - start <= 0) {  // :297-300
        ++end;
        continue;
      }
      const double diff = su[b + end] - su[b + start];  // :303
      if (diff > max_weight) {  // :306-309
        ++start;
        end = start + 1;
        continue;
      }
      if (k < cap) {
        start_out[k] = b + start;
        end_out[k] = b + end;
      }
      ++k;
      if (end == n - 1)  // :324-327
        ++start;
      else
        ++end;
    }
  }
  return k;
}

// One side's sliding window (the state machine above) over rows idx[0..n):
// emits the pairs through f(a, b) in the reference's order.
template <typename F>
static void window_side(const double* su, const int64_t* idx, int64_t n, double max_weight, F&& f) {
  int64_t start = 0, end = 1;
  while (end < n) {
    if (end - start <= 0) {
      ++end;
      continue;
    }
    if (su[idx[end]] - su[idx[start]] > max_weight) {
      ++start;
      end = start + 1;
      continue;
    }
    f(idx[start], idx[end]);
    if (end == n - 1)
      ++start;
    else
      ++end;
  }
}

// the host producers' worker threads: at most 16 (the GPU box's CPU share)
static unsigned host_threads() { return std::max(1u, std::min(16u, std::thread::hardware_concurrency())); }
template <typename F>
static void parallel_ranges(int64_t n, int64_t grain, F&& f) {  // f(lo, hi) over [0, n) in contiguous pieces
  const unsigned hw = host_threads();
  if (n < grain || hw == 1) {
    f((int64_t)0, n);
    return;
  }
  const int64_t per = (n + hw - 1) / hw;
  std::vector<std::thread> th;
  for (unsigned t = 0; t < hw; ++t) {
    const int64_t lo = std::min<int64_t>(n, (int64_t)t * per), hi = std::min<int64_t>(n, lo + per);
    if (lo < hi) th.emplace_back(f, lo, hi);
  }
  for (auto& x : th) x.join();
}

int64_t sst_su_diff_queries(const double* su, const double* obs, const uint8_t* flags, const int64_t* offsets,
                            int64_t n_spec, double max_weight, double tolerance, double* diff, double* thr,
                            int64_t* spec, int8_t* kind, int64_t cap) {
  if (n_spec < 0 || (n_spec > 0 && (!su || !obs || !flags || !offsets)) || cap < 0 ||
      (cap > 0 && (!diff || !thr || !spec || !kind)))
    return SST_E_ARG;
  for (int64_t g = 0; g < n_spec; ++g)
    if (offsets[g + 1] < offsets[g]) return SST_E_ARG;
  // one spectrum's queries in the reference's order: START pairs, END pairs, singletons
  auto produce = [&](int64_t g, std::vector<int64_t>& side, auto&& emit) {
    const int64_t lo = offsets[g], hi = offsets[g + 1];
    for (int sd = 0; sd < 2; ++sd) {
      side.clear();
      for (int64_t r = lo; r < hi; ++r)
        if (flags[r] & (1u << sd)) side.push_back(r);
      window_side(su, side.data(), (int64_t)side.size(), max_weight,
                  [&](int64_t a, int64_t b) { emit(su[b] - su[a], tolerance * (obs[a] + obs[b]), (int8_t)sd); });
    }
    for (int64_t r = lo; r < hi; ++r)
      if (flags[r] & 4u) emit(su[r], tolerance * obs[r], (int8_t)2);
  };
  // pass 1: queries per spectrum; pass 2 (if they fit): each spectrum's at its prefix
  std::vector<int64_t> base((size_t)n_spec + 1, 0);
  parallel_ranges(n_spec, 256, [&](int64_t g0, int64_t g1) {
    std::vector<int64_t> side;
    for (int64_t g = g0; g < g1; ++g) {
      int64_t c = 0;
      produce(g, side, [&](double, double, int8_t) { ++c; });
      base[(size_t)g + 1] = c;
    }
  });
  for (int64_t g = 0; g < n_spec; ++g) base[(size_t)g + 1] += base[(size_t)g];
  const int64_t total = base[(size_t)n_spec];
  if (total > cap) return total;
  parallel_ranges(n_spec, 256, [&](int64_t g0, int64_t g1) {
    std::vector<int64_t> side;
    for (int64_t g = g0; g < g1; ++g) {
      int64_t k = base[(size_t)g];
      produce(g, side, [&](double d, double t, int8_t kd) {
        diff[k] = d;
        thr[k] = t;
        spec[k] = g;
        kind[k] = kd;
        ++k;
      });
    }
  });
  return total;
}

int64_t sst_dict_union(const int64_t* offsets, int64_t n_spec, const double* key, const int8_t* kind,
                       const int8_t* status, const uint64_t* rowmask, uint8_t* keep, uint64_t* union_out) {
  if (!offsets || n_spec < 0) return SST_E_ARG;
  if (n_spec == 0) return 0;
  const int64_t n = offsets[n_spec];
  if (n > 0 && (!key || !kind || !status || !rowmask || !keep || !union_out)) return SST_E_ARG;
  std::atomic<int64_t> kept{0};
  parallel_ranges(n_spec, 64, [&](int64_t g0, int64_t g1) {
    std::vector<std::pair<double, int64_t>> v;
    int64_t mine = 0;
    for (int64_t gs = g0; gs < g1; ++gs) {
      const int64_t a = offsets[gs], b = offsets[gs + 1];
      union_out[2 * gs] = union_out[2 * gs + 1] = 0;
      v.clear();
      for (int64_t i = a; i < b; ++i) {
        keep[i] = 0;
        // side pairs are stored only with >= 1 explanation (prediction.py:322-323);
        // singletons always (:277-282)
        const bool writes = kind[i] == 2 || status[i] == SST_SOME;
        if (writes) v.push_back({key[i] == 0.0 ? 0.0 : key[i], i});  // -0.0 == 0.0 as dict keys
      }
      // the last writer of every key survives (dict assignment order: START
      // pairs, END pairs, singletons = the queries' order)
      std::stable_sort(v.begin(), v.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
      for (size_t k = 0; k < v.size(); ++k) {
        if (k + 1 < v.size() && v[k + 1].first == v[k].first) continue;
        const int64_t i = v[k].second;
        keep[i] = 1;
        ++mine;
        if (status[i] == SST_SOME) {
          union_out[2 * gs] |= rowmask[2 * i];
          union_out[2 * gs + 1] |= rowmask[2 * i + 1];
        }
      }
    }
    kept += mine;
  });
  return kept.load();
}

int sst_sort_rows(const int64_t* group, const double* key, int64_t n, int64_t n_groups, int64_t* order) {
  if (n < 0 || n_groups < 0 || (n > 0 && (!group || !key || !order))) return SST_E_ARG;
  std::vector<int64_t> start((size_t)n_groups + 1, 0);
  for (int64_t i = 0; i < n; ++i) {
    if (group[i] < 0 || group[i] >= n_groups) return SST_E_ARG;
    ++start[(size_t)group[i] + 1];
  }
  for (int64_t g = 0; g < n_groups; ++g) start[(size_t)g + 1] += start[(size_t)g];
  {
    std::vector<int64_t> pos(start.begin(), start.end() - 1);
    for (int64_t i = 0; i < n; ++i) order[pos[(size_t)group[i]]++] = i;  // stable: input order per group
  }
  // each group by key, ties in input order; groups split over a few threads
  const unsigned hw = host_threads();
  const int64_t per = (n_groups + hw - 1) / hw;
  auto work = [&](int64_t g0, int64_t g1) {
    for (int64_t g = g0; g < g1; ++g)
      std::stable_sort(order + start[(size_t)g], order + start[(size_t)g + 1],
                       [&](int64_t a, int64_t b) { return key[a] < key[b]; });
  };
  if (n < (1 << 16) || hw == 1) {
    work(0, n_groups);
  } else {
    std::vector<std::thread> th;
    for (unsigned t = 0; t < hw; ++t) {
      const int64_t g0 = std::min<int64_t>(n_groups, (int64_t)t * per), g1 = std::min<int64_t>(n_groups, g0 + per);
      if (g0 < g1) th.emplace_back(work, g0, g1);
    }
    for (auto& x : th) x.join();
  }
  return SST_OK;
}

// ---- CPython set order (sst_pyset.h), for the skeleton walk's tests -------
extern "C" int64_t sst_py_tuple_hash(const int64_t* item_hashes, int64_t n) {
  uint64_t acc = sst::pyset::tuple_hash_init();
  for (int64_t i = 0; i < n; ++i) acc = (uint64_t)sst::pyset::tuple_hash_step(acc, item_hashes[i]);
  return sst::pyset::tuple_hash_final(acc, n);
}

extern "C" int64_t sst_pyset_order(const int32_t* keys, const int64_t* hashes, int64_t n, int32_t* order) {
  if (n < 0 || n > (1 << 24) || (n > 0 && (!keys || !hashes || !order))) return SST_E_ARG;
  const uint32_t cap = sst::pyset::table_size_for((uint32_t)n);
  std::vector<int32_t> k0(cap), k1(cap);
  std::vector<int64_t> h0(cap), h1(cap);
  sst::pyset::Table t{{k0.data(), k1.data()}, {h0.data(), h1.data()}, cap, 0, 0, 0, false};
  sst::pyset::clear(t);
  for (int64_t i = 0; i < n; ++i) {
    if (keys[i] < 0) return SST_E_ARG;
    sst::pyset::add(t, keys[i], hashes[i]);
  }
  if (t.overflow) return SST_E_ARG;
  int64_t m = 0;
  for (uint32_t s = 0; s <= t.mask; ++s)
    if (t.key[t.cur][s] >= 0) order[m++] = t.key[t.cur][s];
  return m;
}

// ---- config 5: final dict, skeleton walk, candidate references -----------
extern "C" int sst_dict_count_device(sst_table* t, const int64_t* d_peak_off, int64_t n_spec, const double* d_rows_su,
                                     const double* d_rows_ob, const uint32_t* d_rows_meta, const uint8_t* d_alive,
                                     const uint32_t* d_rows, double max_weight, double tol, uint32_t* d_n_q,
                                     uint64_t* d_off, uint32_t* d_err) {
  if (!t || n_spec < 0 || n_spec > INT32_MAX || !d_off ||
      (n_spec > 0 && (!d_peak_off || !d_rows_su || !d_rows_ob || !d_rows_meta || !d_alive || !d_rows || !d_n_q ||
                      !d_err)))
    return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  sst::PipeArgs a{};
  a.peak_off = d_peak_off;
  a.n_spec = n_spec;
  a.r_su = const_cast<double*>(d_rows_su);
  a.r_ob = const_cast<double*>(d_rows_ob);
  a.r_meta = const_cast<uint32_t*>(d_rows_meta);
  a.alive = const_cast<uint8_t*>(d_alive);
  a.cnt = const_cast<uint32_t*>(d_rows);
  a.max_weight = max_weight;
  a.tol = tol;
  a.err = d_err;
  sst::DictArgs d{};
  d.n_q = d_n_q;
  big_args(c, a);
  Prof p(c, SST_K_DICT);
  HIP_OK(c, sst::launch_dict(t->args, a, d, 1, c->n_cu, c->stream));
  HIP_OK(c, sst::launch_scan_u32(d_n_q, d_off, n_spec, c->stream));
  return SST_OK;
}

extern "C" int sst_dict_build_device(sst_table* t, const int64_t* d_peak_off, int64_t n_spec, const double* d_rows_su,
                                     const double* d_rows_ob, const uint32_t* d_rows_meta, const uint8_t* d_alive,
                                     const uint32_t* d_rows, const uint64_t* d_alpha, double max_weight, double tol,
                                     double prec, const uint64_t* d_off, uint64_t* d_key, double* d_thr,
                                     uint32_t* d_n_ent, uint32_t* d_err, const sst_exact_io* x) {
  if (!t || n_spec < 0 || n_spec > INT32_MAX ||
      (n_spec > 0 && (!d_peak_off || !d_rows_su || !d_rows_ob || !d_rows_meta || !d_alive || !d_rows || !d_alpha ||
                      !d_off || !d_n_ent || !d_err)))
    return SST_E_ARG;
  if (!t->args.pairs_enabled) return fail(t->ctx, SST_E_ARG, "final dict: the table has no pair list");
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  if (int rc = check_masks(t)) return rc;
  sst::PipeArgs a{};
  a.peak_off = d_peak_off;
  a.n_spec = n_spec;
  a.r_su = const_cast<double*>(d_rows_su);
  a.r_ob = const_cast<double*>(d_rows_ob);
  a.r_meta = const_cast<uint32_t*>(d_rows_meta);
  a.alive = const_cast<uint8_t*>(d_alive);
  a.cnt = const_cast<uint32_t*>(d_rows);
  a.alpha = d_alpha;
  a.max_weight = max_weight;
  a.tol = tol;
  a.prec = prec;
  a.rprec = 1.0 / prec;
  a.err = d_err;
  sst::DictArgs d{};
  d.off = d_off;
  d.key = d_key;
  d.thr = d_thr;
  d.n_ent = d_n_ent;
  if (int rc = exact_io(c, x, a)) return rc;
  if (x && (!x->xa_st || !x->xa_n || !x->xa_ptr)) return fail(c, SST_E_ARG, "final dict: the exact-mode answers");
  big_args(c, a);
  Prof p(c, SST_K_DICT);
  HIP_OK(c, sst::launch_dict(t->args, a, d, 0, c->n_cu, c->stream));
  return SST_OK;
}

extern "C" int sst_dict_list_device(sst_table* t, const int64_t* d_peak_off, int64_t n_spec, const double* d_rows_su,
                                    const double* d_rows_ob, const uint32_t* d_rows_meta, const uint8_t* d_alive,
                                    const uint32_t* d_rows, double max_weight, double tol, uint32_t* d_err,
                                    const sst_exact_io* x) {
  if (!t || !x || n_spec < 0 || n_spec > INT32_MAX ||
      (n_spec > 0 && (!d_peak_off || !d_rows_su || !d_rows_ob || !d_rows_meta || !d_alive || !d_rows || !d_err)))
    return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  sst::PipeArgs a{};
  a.peak_off = d_peak_off;
  a.n_spec = n_spec;
  a.r_su = const_cast<double*>(d_rows_su);
  a.r_ob = const_cast<double*>(d_rows_ob);
  a.r_meta = const_cast<uint32_t*>(d_rows_meta);
  a.alive = const_cast<uint8_t*>(d_alive);
  a.cnt = const_cast<uint32_t*>(d_rows);
  a.max_weight = max_weight;
  a.tol = tol;
  a.err = d_err;
  if (int rc = exact_io(c, x, a)) return rc;
  sst::DictArgs d{};
  big_args(c, a);
  Prof p(c, SST_K_DICT);
  HIP_OK(c, sst::launch_dict(t->args, a, d, 2, c->n_cu, c->stream));
  return SST_OK;
}

extern "C" int sst_fix_finish_device(sst_table* t, int64_t n_spec, const uint32_t* d_rows, const uint64_t* d_alpha,
                                     uint64_t* d_alpha_next,
                                     const uint8_t* d_active, uint8_t* d_active_next, uint32_t* d_rounds,
                                     uint32_t* d_queries, uint32_t* d_n_active, uint32_t* d_err,
                                     const sst_exact_io* x) {
  if (!t || !x || n_spec < 0 || n_spec > INT32_MAX ||
      (n_spec > 0 && (!d_rows || !d_alpha || !d_alpha_next || !d_active || !d_active_next || !d_rounds || !d_queries ||
                      !d_n_active || !d_err || !x->xa_st || !x->xa_n || !x->xa_ptr)))
    return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  sst::PipeArgs a{};
  a.n_spec = n_spec;
  a.cnt = const_cast<uint32_t*>(d_rows);
  a.alpha = d_alpha;
  a.alpha_next = d_alpha_next;
  a.active = d_active;
  a.active_next = d_active_next;
  a.rounds = d_rounds;
  a.queries = d_queries;
  a.n_active = d_n_active;
  a.err = d_err;
  for (int r = 1; r < t->n_rows; ++r)
    if (!t->is_mod[r]) a.canon[r >> 6] |= 1ull << (r & 63);
  if (int rc = exact_io(c, x, a)) return rc;
  big_args(c, a);
  Prof p(c, SST_K_FIX_ROUND);
  HIP_OK(c, sst::launch_fix_finish(a, c->n_cu, c->stream));
  return SST_OK;
}

extern "C" uint32_t sst_pyset_table_size(uint32_t n) { return sst::pyset::table_size_for(n); }

extern "C" uint64_t sst_walk_scratch_bytes(uint32_t pos_cap, uint32_t len_cap, uint32_t expl_cap, uint32_t cand_cap,
                                           uint32_t tset_cap) {
  return sst::walk_scratch_bytes(pos_cap, len_cap, expl_cap, cand_cap, tset_cap);
}

extern "C" int sst_skel_walk_device(sst_table* t, const sst_walk_args* a) {
  if (!t || !a) return SST_E_ARG;
  if (a->n_sides == 0) return SST_OK;
  if (!a->peak_off || !a->cnt || !a->r_su || !a->r_ob || !a->r_meta || !a->alive || !a->alpha || !a->max_len ||
      !a->pair_ok || !a->d_off || !a->d_n || !a->q_off || !a->q0 || !a->s_ptr || !a->s_n || !a->s_st ||
      !a->req_block || !a->req_mass || !a->req_thr || !a->req_spec || !a->req_count || !a->name_hash || !a->sides ||
      !a->scratch || !a->side_rows || !a->skel_off || !a->skel || !a->min_end || !a->max_end || !a->kept ||
      !a->side_status || !a->n_suspended || !a->n_big || a->n_rounds < 0 || a->n_rounds > SST_WALK_MAX_ROUNDS)
    return SST_E_ARG;
  for (int r = 0; r < a->n_rounds; ++r)
    if (!a->rq_block[r] || !a->rq_ptr[r] || !a->rq_n[r] || !a->rq_st[r]) return SST_E_ARG;
  if (a->pos_cap < sst::pyset::kMinSize || a->tset_cap < sst::pyset::kMinSize || (a->pos_cap & (a->pos_cap - 1)) ||
      (a->tset_cap & (a->tset_cap - 1)) || a->len_cap < 2 || a->len_cap > 255 ||
      a->scratch_stride < sst::walk_scratch_bytes(a->pos_cap, a->len_cap, a->expl_cap, a->cand_cap, a->tset_cap))
    return fail(t->ctx, SST_E_ARG, "skeleton walk: scratch capacities");
  if (!t->args.pairs_enabled) return fail(t->ctx, SST_E_ARG, "skeleton walk: the table has no pair list");
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  if (int rc = check_masks(t)) return rc;
  Prof p(c, SST_K_SKEL_WALK);
  HIP_OK(c, sst::launch_skel_walk(t->args, *a, c->stream));
  return SST_OK;
}

extern "C" int sst_result_refs_device(sst_result* r, const int64_t* d_dst, uint64_t* d_ptr, uint32_t* d_n,
                                      int8_t* d_st) {
  if (!r) return SST_E_ARG;
  sst_ctx* c = r->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  if (int rc = settle(r)) return rc;
  if (int rc = order_after_settle(r)) return rc;
  if (r->n > 0 && (!d_dst || !d_ptr || !d_n || !d_st)) return SST_E_ARG;
  HIP_OK(c, sst::launch_result_refs((const int8_t*)r->status.p, r->n, (const uint4*)r->hits.p, r->n_hits,
                                    (const uint8_t*)r->dense.p, d_dst, d_ptr, d_n, d_st, c->stream));
  return SST_OK;
}

// ---- config 5: both length bounds on the skeleton alphabets ---------------
extern "C" int sst_reach_rows_device(sst_table* t, const uint64_t* d_alpha, const int64_t* d_words,
                                     const uint64_t* d_off, int64_t n_spec, uint32_t* d_bits) {
  if (!t || n_spec < 0 || (n_spec > 0 && (!d_alpha || !d_words || !d_off || !d_bits))) return SST_E_ARG;
  if (t->args.w_min < 1024) return fail(t->ctx, SST_E_ARG, "reach rows: row masses below 1024 (the LDS ring)");
  for (int r = 1; r < t->n_rows; ++r)
    if (t->masses[r] >= (1 << 20)) return fail(t->ctx, SST_E_ARG, "reach rows: a row mass of 2^20 or more");
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  sst::ReachArgs a{d_alpha, d_words, d_off, d_bits, t->args.w, t->n_rows, n_spec};
  Prof p(c, SST_K_REACH_ROWS);
  HIP_OK(c, sst::launch_reach_rows(a, c->n_cu, c->stream));
  return SST_OK;
}

// replay waves in flight for the reach-mode bounds (16 per CU: the DFS is
// latency-bound, one query per wave; memo 2^16 entries each on the first try)
constexpr uint32_t kReachUnits = 4096;
constexpr size_t kReachMemoBytes = 96ull << 30;  // the replay's memo workspace per launch (HBM: 288 GB)

extern "C" int sst_length_bounds_reach_device(sst_table* t, const double* d_su, const double* d_obs,
                                              const int32_t* d_spec, const uint64_t* d_alpha,
                                              const uint32_t* d_reach_bits, const uint64_t* d_reach_off,
                                              const int64_t* d_reach_words, int64_t n, double tol, double prec,
                                              int max_len, int64_t max_mods, int64_t* d_lower, int64_t* d_upper,
                                              int8_t* d_status, const int32_t* d_qlen, const int32_t* d_caps_len,
                                              const int32_t* d_a0_len, uint64_t* d_nodes, int64_t soft_nodes,
                                              uint32_t memo_first, int fuse) {
  if (!t || n < 0 || n > INT32_MAX || max_len < 0 || (d_qlen && (!d_caps_len || !d_a0_len)) ||
      (n > 0 && (!d_su || !d_obs || !d_spec || !d_alpha || !d_reach_bits || !d_reach_off || !d_reach_words ||
                 !d_lower || !d_upper || !d_status)))
    return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (max_len > 120) return fail(c, SST_E_ARG, "length bounds (replay): max_len above 120 (the int8 value slots)");
  if (int rc = set_device(c)) return rc;
  if (n == 0) return SST_OK;
  // the memo workspace: at most kReachMemoBytes, and at most 60 % of what the
  // device has free now (a smaller or shared device runs fewer waves)
  size_t memo_bytes = kReachMemoBytes;
  {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess) memo_bytes = std::min(memo_bytes, fr / 10 * 6);
    else (void)hipGetLastError();
  }
  const size_t nn = (size_t)n;
  DevBuf d_list, d_cnt;
  if (!d_list.ensure(nn * 4) || !d_cnt.ensure(4)) return fail(c, SST_E_NOMEM, "device allocation failed (length bound)");
  HIP_OK(c, hipMemsetAsync(d_cnt.p, 0, 4, c->stream));
  LBArgs q{};
  q.su = d_su;
  q.obs = d_obs;
  q.n = n;
  q.tol = tol;
  q.prec = prec;
  q.rprec = 1.0 / prec;
  q.A0 = (int)std::max<int64_t>(0, std::min<int64_t>(max_mods, kInfBudget));
  q.dir = 0;
  q.max_len = max_len;
  q.out = d_lower;
  q.status = d_status;
  q.exact_list = (uint32_t*)d_list.p;
  q.exact_count = (uint32_t*)d_cnt.p;
  q.node_budget = kLBNodeBudget;
  q.alpha = d_alpha;
  q.spec = d_spec;
  q.comp = (int)t->C;
  q.reach_bits = d_reach_bits;
  q.reach_off = d_reach_off;
  q.reach_words = d_reach_words;
  q.both = 1;
  q.out_hi = d_upper;
  q.qlen = d_qlen;
  q.caps_len = d_caps_len;
  q.a0_len = d_a0_len;
  q.nodes_out = d_nodes;
  q.fuse = fuse ? 1 : 0;  // the caller checks every alphabet has <= 64 kept rows
  if (soft_nodes > 0) {
    q.node_budget = (uint64_t)soft_nodes;
    q.soft = 1;
  }
  if (memo_first && (memo_first & (memo_first - 1))) return fail(c, SST_E_ARG, "length bound: memo_first not a power of two");
  uint32_t n_exact = 0;
  {
    Prof p(c, SST_K_LENGTH_BOUND);  // windows, extents; every live query is listed for the replay
    HIP_OK(c, launch_length_bound(t->args, q, nullptr, nullptr, nullptr, 0, 0, true, c->stream));
  }
  HIP_OK(c, hipMemcpyAsync(&n_exact, d_cnt.p, 4, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(c, hipStreamSynchronize(c->stream));
  std::vector<int8_t> st(nn);
  // memo per wave: 2^16 masses on the first try (most spectra), 8x per retry
  // for the queries that ran out; the waves in flight are what the
  // workspace budget allows at that size (a retry keeps its parallelism)
  // per memo slot: the hash entry, plus (fused) 2 x 64 value bytes per
  // inserted mass at load factor 1/4, or (not fused) 120 value bytes per slot
  const size_t per_entry = hash_entry_bytes() + (fuse ? 2 * 64 / 4 : kMaxRows);
  uint32_t cap = memo_first ? std::max<uint32_t>(memo_first, 64) : kLBHashCap0;
  auto units_for = [&](uint32_t n_q) {
    const size_t by_mem = memo_bytes / ((size_t)cap * per_entry);
    return (int)std::max<size_t>(1, std::min<size_t>({(size_t)kReachUnits, (size_t)std::max<uint32_t>(1, n_q), by_mem}));
  };
  int units = units_for(n_exact);
  while (n_exact) {
    DevBuf hash, vals, frames;
    if (!hash.ensure((size_t)units * cap * hash_entry_bytes()) ||
        !vals.ensure(fuse ? (size_t)units * (cap / 4) * 2 * 64 : (size_t)units * cap * kMaxRows) ||
        !frames.ensure((size_t)units * lb_frame_bytes()))
      return fail(c, SST_E_NOMEM, "device allocation failed (length-bound memo)");
    HIP_OK(c, hipMemsetAsync(hash.p, 0, hash.bytes, c->stream));
    {
      Prof p(c, SST_K_LENGTH_BOUND);
      HIP_OK(c, launch_length_bound(t->args, q, (char*)hash.p, (int8_t*)vals.p, (char*)frames.p, cap, units, false,
                                    c->stream));
    }
    HIP_OK(c, hipMemcpyAsync(st.data(), d_status, nn, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(c, hipStreamSynchronize(c->stream));
    // the queries whose memo ran out: again, alone, with 8x the memo
    std::vector<uint32_t> retry;
    for (size_t i = 0; i < nn; ++i)
      if (st[i] == kStatusExactRetry) retry.push_back((uint32_t)i);
    if (retry.empty()) break;
    if ((size_t)cap * 8 * per_entry > memo_bytes)
      return fail(c, SST_E_NOMEM, "length bound: memo would exceed the workspace limit");
    cap *= 8;
    units = units_for((uint32_t)retry.size());
    n_exact = (uint32_t)retry.size();
    HIP_OK(c, hipMemcpyAsync(d_list.p, retry.data(), retry.size() * 4, hipMemcpyHostToDevice, c->stream));
    HIP_OK(c, hipMemcpyAsync(d_cnt.p, &n_exact, 4, hipMemcpyHostToDevice, c->stream));
  }
  for (size_t i = 0; i < nn; ++i)
    if (st[i] == kStatusPending || st[i] == kStatusExactRetry)
      return fail(c, SST_E_INTERNAL, "length bound: query left unresolved (internal error)");
  return SST_OK;
}

// ---- the first-visit frontier (sst_frontier.hip) ---------------------------
extern "C" int sst_reach_lowest_device(sst_table* t, const uint64_t* d_alpha, const int64_t* d_words,
                                       const uint64_t* d_off, int64_t n_spec, const uint32_t* d_bits,
                                       const uint64_t* d_lr_off, uint8_t* d_lr) {
  if (!t || n_spec < 0 || (n_spec > 0 && (!d_alpha || !d_words || !d_off || !d_bits || !d_lr_off || !d_lr)))
    return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  sst::ReachArgs a{d_alpha, d_words, d_off, const_cast<uint32_t*>(d_bits), t->args.w, t->n_rows, n_spec};
  Prof p(c, SST_K_REACH_ROWS);
  HIP_OK(c, sst::launch_reach_lowest(a, d_lr_off, d_lr, c->stream));
  return SST_OK;
}

namespace {
int bits_for(uint64_t x) {  // bits needed to hold 0..x
  int b = 0;
  while (b < 64 && (x >> b)) ++b;
  return b;
}
uint64_t pow2_floor(uint64_t x) {
  uint64_t p = 1;
  while (p <= x / 2) p <<= 1;
  return p;
}
}  // namespace

static int lbf_frontier(sst_table* t, sst_ctx::LbfWs& W, const double* d_su, const double* d_obs,
                        const int32_t* d_spec, const uint64_t* d_alpha, const uint8_t* d_lr, const uint64_t* d_lr_off,
                        int64_t n, double tol, double prec, int max_len, int64_t max_mods, int64_t* d_lower,
                        int64_t* d_upper, int8_t* d_status, const int32_t* d_qlen, const int32_t* d_caps_len,
                        const int32_t* d_a0_len, uint64_t* d_nodes, uint64_t workspace_bytes, sst_lbf_stats* stats) {
  if (!t || n < 0 || n > INT32_MAX || max_len < 0 || (d_qlen && (!d_caps_len || !d_a0_len)) ||
      (n > 0 && (!d_su || !d_obs || !d_spec || !d_alpha || !d_lr || !d_lr_off || !d_lower || !d_upper || !d_status)))
    return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  if (stats) *stats = sst_lbf_stats{};
  if (n == 0) return SST_OK;
  for (int r = 1; r < t->n_rows; ++r)
    if (t->masses[r] >= (1 << 20)) return fail(c, SST_E_ARG, "length bounds (frontier): a row mass of 2^20 or more");
  const int wb = (int)t->args.w_min;
  int64_t w_max = 0;
  for (int r = 1; r < t->n_rows; ++r) w_max = std::max<int64_t>(w_max, t->masses[r]);
  if (wb < 1) return fail(c, SST_E_ARG, "length bounds (frontier): no row mass");
  const int jump = (int)((w_max + wb - 1) / wb);  // bands one left move can cross
  int ring = 1;
  while (ring <= jump) ring <<= 1;
  if (ring > 8) return fail(c, SST_E_ARG, "length bounds (frontier): row masses span more than 7 bands");
  const size_t nn = (size_t)n;
  DevBuf d_list, d_cnt;
  if (!d_list.ensure(nn * 4) || !d_cnt.ensure(4)) return fail(c, SST_E_NOMEM, "device allocation failed (length bound)");
  HIP_OK(c, hipMemsetAsync(d_cnt.p, 0, 4, c->stream));
  // the list pass: windows, the reduced table's extent (SST_OUT_OF_TABLE /
  // SST_ABORTED in its last word), empty windows; every live query listed
  LBArgs q{};
  q.su = d_su;
  q.obs = d_obs;
  q.n = n;
  q.tol = tol;
  q.prec = prec;
  q.rprec = 1.0 / prec;
  q.A0 = (int)std::max<int64_t>(0, std::min<int64_t>(max_mods, kInfBudget));
  q.max_len = max_len;
  q.out = d_lower;
  q.status = d_status;
  q.exact_list = (uint32_t*)d_list.p;
  q.exact_count = (uint32_t*)d_cnt.p;
  q.node_budget = kLBNodeBudget;
  q.alpha = d_alpha;
  q.spec = d_spec;
  q.comp = (int)t->C;
  uint32_t n_live = 0;
  {
    Prof p(c, SST_K_LENGTH_BOUND);
    HIP_OK(c, launch_length_bound(t->args, q, nullptr, nullptr, nullptr, 0, 0, true, c->stream));
  }
  HIP_OK(c, hipMemcpyAsync(&n_live, d_cnt.p, 4, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(c, hipStreamSynchronize(c->stream));
  if (stats) stats->live = n_live;
  if (n_live == 0) return SST_OK;
  {  // the list pass appends with atomics: sorted, the chunks (and so every
     // dispatch of a run) are the same from run to run (matched profiles)
    std::vector<uint32_t> lst(n_live);
    HIP_OK(c, hipMemcpyAsync(lst.data(), d_list.p, (size_t)n_live * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(c, hipStreamSynchronize(c->stream));
    std::sort(lst.begin(), lst.end());
    HIP_OK(c, hipMemcpyAsync(d_list.p, lst.data(), (size_t)n_live * 4, hipMemcpyHostToDevice, c->stream));
    HIP_OK(c, hipStreamSynchronize(c->stream));
  }
  // workspace per "slot": 8 nodes of 7 B, a 4-B node -> group entry for the
  // band in hand, per ring table a group entry (32 B) + its list entry (4 B)
  // and a candidate entry (32 B: 128-bit keys), and the band's group record
  // (20 B) and candidate record (24 B); S slots, S a power of two (hashing)
  size_t budget = workspace_bytes;
  if (budget == 0 && W.S && W.by_default) {
    budget = W.budget;  // the default workspace of an earlier call
  } else if (budget == 0) {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
      (void)hipGetLastError();
      fr = 16ull << 30;
    }
    budget = std::min<size_t>(96ull << 30, fr / 2);
  }
  constexpr uint64_t kNodesPerSlot = 8;
  const size_t per_slot = kNodesPerSlot * 7 + 4 + (size_t)ring * (lbf_group_bytes() + 4 + lbf_cand_bytes(2)) +
                          lbf_grec_bytes() + lbf_crec_bytes(2);
  if (W.budget != budget) {  // (re)size the ctx's workspace: the first call, or another budget
    W = sst_ctx::LbfWs{};
    W.budget = budget;
    W.by_default = workspace_bytes == 0;
    W.S = pow2_floor(std::max<size_t>(1024, budget / per_slot));
    if (W.S > (1ull << 31)) W.S = 1ull << 31;
    W.ncap = std::min<uint64_t>(kNodesPerSlot * W.S, 0xFFFFFFF0ull);
  }
  const uint64_t S = W.S, ncap = W.ncap;
  DevBuf &flags = W.flags, &lpar = W.lpar, &lval = W.lval, &gtab = W.gtab, &ctab = W.ctab,
         &glist = W.glist, &ctl = W.ctl, &bstart = W.bstart, &bgroups = W.bgroups, &qi = W.qi, &qrow = W.qrow,
         &roots = W.roots, &ncnt = W.ncnt, &grec = W.grec, &crec = W.crec, &ngrp = W.ngrp;
  if (!flags.ensure(ncap) || !lpar.ensure(ncap * 4) || !lval.ensure(ncap * 2) ||
      !gtab.ensure((size_t)ring * S * lbf_group_bytes()) || !ctab.ensure((size_t)ring * S * lbf_cand_bytes(2)) ||
      !glist.ensure((size_t)ring * S * 4) || !ctl.ensure(sizeof(FCtl)) || !grec.ensure(S * lbf_grec_bytes()) ||
      !crec.ensure(S * lbf_crec_bytes(2)) || !ngrp.ensure(S * 4)) {
    W = sst_ctx::LbfWs{};
    return fail(c, SST_E_NOMEM, "device allocation failed (length-bound frontier workspace)");
  }
  constexpr uint32_t kChunkMax = 1u << 20;  // the keys' query field
  // one sweep over list entries [c0, c1): 1 done, 0 overflow (split and rerun), < 0 error
  uint64_t last_nodes = 0;
  int& epoch = W.epoch;  // hash tags per chunk: tables are cleared only when the epoch wraps
  bool& dirty = W.dirty;  // or after an overflowed chunk (its groups' masks were not consumed)
  auto run_chunk = [&](uint32_t c0, uint32_t c1) -> int {
    const uint32_t nc = c1 - c0;
    FrontierArgs a{};
    a.list = (const uint32_t*)d_list.p;
    a.chunk0 = c0;
    a.n_chunk = nc;
    a.su = d_su;
    a.obs = d_obs;
    a.tol = tol;
    a.prec = prec;
    a.rprec = 1.0 / prec;
    a.spec = d_spec;
    a.alpha = d_alpha;
    a.lr = d_lr;
    a.lr_off = d_lr_off;
    a.qlen = d_qlen;
    a.caps_len = d_caps_len;
    a.a0_len = d_a0_len;
    a.A0 = q.A0;
    a.max_len = max_len;
    a.wb = wb;
    a.ring = ring;
    a.jump = jump;
    a.lower = d_lower;
    a.upper = d_upper;
    a.status = d_status;
    a.nodes_out = d_nodes;
    if (!qi.ensure((size_t)nc * sizeof(FQInfo)) || !qrow.ensure((size_t)nc * 128 * 4) || !ncnt.ensure((size_t)nc * 4))
      return fail(c, SST_E_NOMEM, "device allocation failed (length-bound frontier queries)");
    a.qi = (FQInfo*)qi.p;
    a.qrow = (uint32_t*)qrow.p;
    a.node_cnt = (uint32_t*)ncnt.p;
    a.ctl = (FCtl*)ctl.p;
    HIP_OK(c, hipMemsetAsync(ctl.p, 0, sizeof(FCtl), c->stream));
    HIP_OK(c, hipMemsetAsync(ncnt.p, 0, (size_t)nc * 4, c->stream));
    {
      Prof p(c, SST_K_LENGTH_BOUND);
      HIP_OK(c, launch_lbf_setup(t->args, a, c->stream));
    }
    FCtl h{};
    HIP_OK(c, hipMemcpyAsync(&h, ctl.p, sizeof(FCtl), hipMemcpyDeviceToHost, c->stream));
    HIP_OK(c, hipStreamSynchronize(c->stream));
    const int n_bands = h.max_hi >= 1 ? (int)h.max_band + 1 : 0;
    if (n_bands > 126) return fail(c, SST_E_ARG, "length bounds (frontier): a window beyond 126 bands");
    if (h.max_hi >= (1ull << 25)) return fail(c, SST_E_ARG, "length bounds (frontier): a window at 2^25 or beyond");
    a.rb = bits_for(h.max_win > 0 ? h.max_win - 1 : 0);
    // unary keys: root bits, one zero per kept rank, one 1 per left move (<= hi / w_min)
    const int need = a.rb + (int)h.max_need;  // (k_lbf_setup excluded every query beyond 256 bits)
    int kw = need <= 64 ? 1 : need <= 128 ? 2 : need <= 256 ? 4 : 0;
    // (tests: SST_LBF_MIN_KEY_WORDS=2|4 runs a batch with wider keys than it
    // needs -- wide keys are otherwise reached only by windows whose memo no
    // oracle could check; the results must not change)
    if (const char* mk = getenv("SST_LBF_MIN_KEY_WORDS")) {
      const int m = atoi(mk);
      if (kw && (m == 2 || m == 4) && m > kw) kw = m;
    }
    if (!kw || a.rb > 32) return fail(c, SST_E_ARG, "length bounds (frontier): first-visit keys beyond 256 bits");
    a.rstride = (int)std::max<uint32_t>(1, h.max_win);
    a.n_bands = n_bands;
    if (!roots.ensure((size_t)nc * a.rstride * 4))
      return fail(c, SST_E_NOMEM, "device allocation failed (length-bound frontier roots)");
    a.root_node = (uint32_t*)roots.p;
    a.flags = (uint8_t*)flags.p;
    a.lpar = (uint32_t*)lpar.p;
    a.lval = (uint16_t*)lval.p;
    a.ncap = ncap;
    a.gtab = (char*)gtab.p;
    a.gmask = (uint32_t)(S - 1);
    const uint64_t cslots = pow2_floor(ctab.bytes / ((size_t)ring * lbf_cand_bytes(kw)));
    a.ctab = (char*)ctab.p;
    a.cmask = (uint32_t)(cslots - 1);
    a.glist = (uint32_t*)glist.p;
    if (!bstart.ensure((size_t)(n_bands + 2) * 4) || !bgroups.ensure((size_t)(n_bands + 2) * 4))
      return fail(c, SST_E_NOMEM, "device allocation failed (length-bound frontier bands)");
    a.band_start = (uint32_t*)bstart.p;
    a.band_groups = (uint32_t*)bgroups.p;
    a.grec = (char*)grec.p;
    a.grec_cap = S;
    a.crec = (char*)crec.p;
    a.crec_cap = crec.bytes / lbf_crec_bytes(kw);
    a.node_group = (uint32_t*)ngrp.p;
    a.ngrp_cap = S;
    if (dirty || epoch == 0) {  // empty tables: tag 0 matches no band
      HIP_OK(c, hipMemsetAsync(gtab.p, 0, gtab.bytes, c->stream));
      HIP_OK(c, hipMemsetAsync(ctab.p, 0, ctab.bytes, c->stream));
      epoch = 0;
      dirty = false;
    }
    a.epoch = epoch;
    epoch = (epoch + 1) & 31;
    {
      Prof p(c, SST_K_LENGTH_BOUND);
      HIP_OK(c, launch_lbf_sweep(a, kw, n_bands, c->n_cu * 8, c->stream));
    }
    HIP_OK(c, hipMemcpyAsync(&h, ctl.p, sizeof(FCtl), hipMemcpyDeviceToHost, c->stream));
    std::vector<uint32_t> band_groups((size_t)n_bands, 0), band_start((size_t)n_bands + 1, 0);
    if (n_bands) {
      HIP_OK(c, hipMemcpyAsync(band_groups.data(), bgroups.p, (size_t)n_bands * 4, hipMemcpyDeviceToHost, c->stream));
      HIP_OK(c, hipMemcpyAsync(band_start.data(), bstart.p, ((size_t)n_bands + 1) * 4, hipMemcpyDeviceToHost,
                               c->stream));
    }
    HIP_OK(c, hipStreamSynchronize(c->stream));
    if (h.overflow & 56u) return fail(c, SST_E_INTERNAL, "length bounds (frontier): inconsistent first-visit tables");
    if (h.overflow) {
      dirty = true;
      if (stats) {
        stats->splits++;
        stats->overflow_bits |= h.overflow;
      }
      if (nc == 1) {  // one query beyond the whole workspace: reported, not guessed
        FQInfo one{};
        HIP_OK(c, hipMemcpyAsync(&one, qi.p, sizeof(FQInfo), hipMemcpyDeviceToHost, c->stream));
        HIP_OK(c, hipStreamSynchronize(c->stream));
        const int8_t ab = SST_ABORTED;
        HIP_OK(c, hipMemcpyAsync(d_status + one.i, &ab, 1, hipMemcpyHostToDevice, c->stream));
        if (stats) stats->aborted++;
        return 1;
      }
      return 0;
    }
    last_nodes = h.node_ctr;
    if (h.node_ctr > (1u << 24)) {  // the bands' shape: sizes the next chunks against the per-band capacities
      uint32_t mb = 0;
      for (int b = 0; b < n_bands; ++b) mb = std::max<uint32_t>(mb, band_start[b + 1] - band_start[b]);
      W.band_frac = std::max(W.band_frac * 0.9, (double)mb / (double)h.node_ctr);
    }
    if (stats) {
      stats->chunks++;
      stats->nodes += h.node_ctr;
      stats->bands = std::max<int64_t>(stats->bands, n_bands);
      stats->key_words = std::max<int64_t>(stats->key_words, kw);
      for (uint32_t x : band_groups) {
        stats->max_band_groups = std::max<int64_t>(stats->max_band_groups, x);
        stats->groups += x;
      }
      stats->edges += (int64_t)h.edges;
      for (int b = 0; b < n_bands; ++b)
        stats->max_band_nodes = std::max<int64_t>(stats->max_band_nodes, band_start[b + 1] - band_start[b]);
      stats->table_slots = (int64_t)S;
      stats->node_cap = (int64_t)ncap;
    }
    return 1;
  };
  // chunks sized from the nodes per query seen so far (this ctx's earlier
  // calls included; a first chunk of 256), aiming at half the node capacity;
  // a chunk that overflows is split in halves
  // (this call's queries once it has some: alphabets differ between calls)
  uint64_t done_q = 0, done_nodes = 0;
  uint32_t c0 = 0;
  while (c0 < n_live) {
    uint32_t nc = std::min<uint32_t>(n_live - c0, 256);
    if ((done_q && done_nodes) || (W.done_q && W.done_nodes)) {
      // nodes per chunk: half the node capacity, and a largest band of at most
      // 40 % of the per-band capacities (S node -> group entries, hash slots)
      const double per_q = done_q && done_nodes ? (double)done_nodes / (double)done_q
                                                : 4.0 * (double)W.done_nodes / (double)W.done_q;
      const double target = std::min(0.5 * (double)ncap, 0.4 * (double)S / std::max(0.02, W.band_frac));
      nc = (uint32_t)std::max<double>(1.0, std::min<double>({(double)(n_live - c0), (double)kChunkMax, target / per_q}));
    } else if (done_q) {
      nc = std::min<uint32_t>(n_live - c0, kChunkMax);
    }
    std::vector<std::pair<uint32_t, uint32_t>> todo{{c0, c0 + nc}};
    while (!todo.empty()) {
      const auto [a0, a1] = todo.back();
      todo.pop_back();
      const int rc = run_chunk(a0, a1);
      if (rc < 0) return rc;
      if (rc == 0) {
        const uint32_t mid = a0 + (a1 - a0) / 2;
        todo.push_back({mid, a1});
        todo.push_back({a0, mid});
        continue;
      }
      done_q += a1 - a0;
      done_nodes += last_nodes;
      W.done_q += a1 - a0;
      W.done_nodes += last_nodes;
    }
    c0 += nc;
  }
  HIP_OK(c, hipStreamSynchronize(c->stream));
  return SST_OK;
}

extern "C" int sst_length_bounds_frontier_device(sst_table* t, const double* d_su, const double* d_obs,
                                                 const int32_t* d_spec, const uint64_t* d_alpha, const uint8_t* d_lr,
                                                 const uint64_t* d_lr_off, int64_t n, double tol, double prec,
                                                 int max_len, int64_t max_mods, int64_t* d_lower, int64_t* d_upper,
                                                 int8_t* d_status, const int32_t* d_qlen, const int32_t* d_caps_len,
                                                 const int32_t* d_a0_len, uint64_t* d_nodes, uint64_t workspace_bytes,
                                                 sst_lbf_stats* stats) {
  if (!t) return SST_E_ARG;
  return lbf_frontier(t, t->ctx->lbf, d_su, d_obs, d_spec, d_alpha, d_lr, d_lr_off, n, tol, prec, max_len, max_mods,
                      d_lower, d_upper, d_status, d_qlen, d_caps_len, d_a0_len, d_nodes, workspace_bytes, stats);
}

extern "C" int sst_jaccard_device(sst_table* t, const sst_jaccard_args* a) {
  if (!t || !a || a->n_spec < 0) return SST_E_ARG;
  if (a->n_spec == 0) return SST_OK;
  if (!a->max_len || !a->skel_off || !a->skel || !a->lower || !a->upper || !a->status_lb || !a->su_mass ||
      !a->row_mass || !a->comb_off || !a->comb || !a->seq_len || !a->status)
    return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  Prof p(c, SST_K_JACCARD);
  HIP_OK(c, sst::launch_jaccard(*a, c->stream));
  return SST_OK;
}

extern "C" int sst_post_skeleton_device(sst_table* t, const sst_post_args* a) {
  if (!t || !a || a->n_spec < 0) return SST_E_ARG;
  if (a->n_spec == 0) return SST_OK;
  if (!a->peak_off || !a->rows || !a->meta || !a->alive || !a->kept || !a->min_end || !a->max_end || a->slots < 0 ||
      !a->seq_len || !a->jac_status || !a->comb_off || !a->comb || !a->alpha || !a->alpha_out || !a->active ||
      !a->alive_out || !a->min_end_out || !a->max_end_out || !a->err)
    return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  uint64_t canon[2] = {0, 0};
  for (int r = 1; r < t->n_rows; ++r)
    if (!t->is_mod[r]) canon[r >> 6] |= 1ull << (r & 63);
  Prof p(c, SST_K_JACCARD);
  HIP_OK(c, sst::launch_post_skel(*a, canon[0], canon[1], 4 * c->n_cu, c->stream));
  return SST_OK;
}

extern "C" int sst_skeleton_alpha_device(sst_table* t, int64_t n_spec, const int32_t* d_max_len,
                                         const uint64_t* d_skel_off, const uint64_t* d_skel, const uint64_t* d_alpha,
                                         uint64_t* d_out) {
  if (!t || n_spec < 0 || (n_spec > 0 && (!d_max_len || !d_skel_off || !d_skel || !d_alpha || !d_out))) return SST_E_ARG;
  sst_ctx* c = t->ctx;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (int rc = set_device(c)) return rc;
  uint64_t canon[2] = {0, 0};
  for (int r = 1; r < t->n_rows; ++r)
    if (!t->is_mod[r]) canon[r >> 6] |= 1ull << (r & 63);
  Prof p(c, SST_K_JACCARD);
  HIP_OK(c, sst::launch_skel_alpha(n_spec, d_max_len, d_skel_off, d_skel, d_alpha, canon[0], canon[1], d_out,
                                   c->stream));
  return SST_OK;
}
