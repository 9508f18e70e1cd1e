// sst_internal.h -- shared definitions between the HIP kernels and the host
// side of libsstgpu.so.  Not part of the public ABI (see include/sst.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sst.h"

namespace sst {

constexpr int kMaxRows = 120;      // rows 0..119; index record keeps lo in bits 56..63
static_assert(kMaxRows == SST_MAX_ROWS, "the ABI's row stride");
constexpr int kWG = 256;           // workgroup of the lane-per-query kernels (4 waves)
#ifndef SST_DEF_WG
#define SST_DEF_WG 256
#endif
constexpr int kDefWG = SST_DEF_WG;        // k_explain_deferred workgroup (4 waves; the deep role allocates per workgroup)
constexpr int kShallowDepth = 4;   // register-stack depth of the main kernel
constexpr int kMaxDepth = 96;      // >= max items of any multiset in a table (73 for the full alphabet)
constexpr int kInfBudget = 1 << 30;  // np.inf budget (decremented at most kMaxDepth times)
constexpr int kScanWG = 1024;        // scan kernel workgroup (2 per CU share the LDS pair list)
constexpr int kMaxSingletonMasses = 1024;  // is_singleton: integer masses staged in LDS
constexpr int kMaxPairLds = 44 * 1024;  // pair-list image per scan workgroup (staged at launch; 78 KB: 2 us slower)
// worklist item flags ({query, a, b, flags}): v == 0 lies in the window; the
// window was not classified by the scan (the expand kernel checks the bitset
// and routes it); budgets cannot bind (fast-path theorem)
constexpr uint32_t kItemZero = 1u, kItemUnclassified = 2u, kItemNever = 4u;

enum { kClassShallow = 0, kClassDeep = 1, kClassExact = 2, kClassNomemo = 3, kNumClasses = 4 };
// internal statuses (never returned to callers)
constexpr int kStatusPending = -10;
constexpr int kStatusArenaRetry = -11;
constexpr int kStatusExactRetry = -12;
constexpr int kLBEmptyWindow = -5;  // length bound: empty window (the reference's min([]) raises ValueError)
constexpr int kLBHeavy = SST_LB_HEAVY;  // length bound: over the caller's soft node budget (replayed later)

enum {
  kStatShallow = 0,
  kStatDeep = 1,
  kStatExact = 2,
  kStatNomemo = 3,
  kStatNodes = 4,
  kStatPayload = 5,
  kStatPair = 6,         // queries answered from the LDS pair list
  kStatPairPayload = 7,  // payload bytes of those
  kNumStats = 8
};

struct TableArgs {
  const ulonglong2* index;  // M records
  const uint64_t* valid;    // ceil(M/64) words
  int64_t limit;            // M = n_cols * compression
  const int* w;             // [n_rows] integer masses
  const int* cap;           // [n_rows] round(max_len * rate)
  const uint8_t* mod;       // [n_rows] is_modification
  uint64_t mod0, mod1;      // row masks of modification rows
  uint64_t capz0, capz1;    // row masks with cap <= 0
  uint64_t capneg0, capneg1;  // row masks with cap < 0
  int64_t fast_limit_B;     // max window value for which no per-row cap can bind
  int64_t full_lo, full_hi;  // every mass in [full_lo, full_hi) is reachable (pair(N-1, m) != 0)
  int64_t first_reach;       // smallest reachable mass >= 1
  int64_t shallow_hi;       // window values < shallow_hi (= 4 * w_min) fit in <= 3 items
  // LDS pair list: every 1- and 2-item sum of the alphabet, sorted by
  // (sum, top row), as one u32 image staged to LDS whole:
  //   sums[n_pairs + 2]  sum << 1 | (record is a pair), two UINT32_MAX sentinels
  //   recs[n_pairs + 2]  serialised payload record: [1][top] or [2][low][top]
  //   bk[n_buckets]      bucket b covers masses pair_base + [b, b+1) << pair_shift:
  //                      bits 0-15 first entry with sum >= the bucket start,
  //                      bits 16-31 that sum minus the bucket start (clamped)
  // Valid only for tables known to follow the reference recurrence over
  // exactly these masses (built here); window values < pair_hi (= 3 * w_min)
  // have no candidate with more than 2 items.
  const uint32_t* pair_data;
  int64_t pair_hi;
  int n_pairs;
  int n_buckets;
  int pair_shift;
  uint32_t pair_base;  // = w_min: no sum lies below it
  // census of the pair list, one u32 per value x in [pair_base - 1, pair_hi):
  // bits 0-15 entries with sum <= x, bits 16-31 their record bytes.  A window's
  // count, first entry and payload bytes are two independent loads (the rows
  // step reads it through L2; the pair list is <= 21000 entries, <= 63000 B)
  const uint32_t* census;
  // u32 forms of the fast-path limits (window values are < 2^31):
  // hi < never_lim  <=>  hi <= fast_limit_B (no per-row cap binds);
  // hi < pair_lim   <=>  pair-list window with no per-row cap binding
  uint32_t never_lim, pair_lim;
  int pairs_enabled;
  int n_rows;
  int any_mod;
  int w_min;                // smallest positive row mass
  int w_min_mod;            // smallest modification row mass
};

struct QueryArgs {
  const double* mass;
  const double* thr;        // may be null: tolerance * mass
  const int64_t* max_mods;  // may be null: max_mods_scalar
  int64_t max_mods_scalar;
  int64_t n;
  double tol, prec;
  double rprec;  // 1 / prec (host-rounded): quotient fast path, see quantise()
  int with_memo;
  uint64_t cap_count;
  uint64_t node_budget;
  // pair-list scan, folded on the host (fold_scan_limits): with one scalar
  // budget, hi < pair_hi_lim <=> pair-class window whose budgets cannot bind,
  // hi < never_hi_lim <=> fast-path theorem; cap32 = min(cap_count, 2^32-1)
  uint32_t pair_hi_lim = 0, never_hi_lim = 0, cap32 = 0;
  // per-query alphabets (sst_explain_alpha_batch_device): alpha[2 g], [2 g + 1]
  // = row mask of alphabet g over the table's rows, spec[i] = query i's alphabet
  const uint64_t* alpha = nullptr;
  const int32_t* spec = nullptr;
  int comp = 32;  // the table's compression (masses per packed word)
  // per-query budgets (sst_explain_alpha_lens_batch_device; null: the
  // table's caps for every query): query i's row caps caps_len[qlen[i] *
  // kMaxRows + r], the rows with cap <= 0 capz_len[2 qlen[i]], [+ 1], and its
  // fast-path limit never_len[qlen[i]] (never_lim for those caps); its
  // max_modifications come in max_mods[i]
  const int32_t* qlen = nullptr;
  const int32_t* caps_len = nullptr;
  const uint64_t* capz_len = nullptr;
  const uint32_t* never_len = nullptr;
};

// Arena layout of one explain pass:
//   [0, spill_base)        one region per scan wave (bump allocated by that
//                          wave alone: no atomics), spill_base =
//                          n_scan_waves * region_bytes
//   [spill_base, arena)    spill area, atomically allocated (the deferred
//                          paths: SHALLOW worklists, deep / exact / no-memo,
//                          recursion)
// k_result_pack turns the pass's output into the result every consumer
// reads: status[n] (written in place by the kernels), a dense hit list (one
// 16-B record {query, count, word} per query with candidates) and a dense
// payload (see include/sst.h, sst_result_hit_list).
struct OutArgs {
  int8_t* status;
  uint8_t* payload;           // the arena
  uint64_t arena_bytes;
  uint64_t region_bytes;      // per-wave region of the scan kernel (multiple of 16)
  uint64_t spill_base;        // = n_scan_waves * region_bytes
  uint64_t* cursor;           // spill bytes taken (keeps counting past the arena: > spill area = arena retries)
  unsigned long long* exact_retries;  // queries the exact path left for a retry with a larger memo
  unsigned long long* arena_retries;  // SOME queries whose scan-wave region was full (retried with larger regions)
  unsigned long long* region_need;    // atomicMax: payload bytes a wave with a full region would have needed
  uint64_t* ctl_next;         // the next pass's control block: zeroed by the scan kernel
  int ctl_words;
  unsigned long long* wave_stats;  // [n_scan_waves][kNumStats] scan-wave counters
  uint4* work;                // [n_scan_waves][work_region] queued SHALLOW {query, a, b, has_zero} from the
                              // front; the scan's hit records {query, count | bytes << 16} (uint2) from the back
  uint32_t* work_count;       // [n_scan_waves] worklist lengths (k_explain_scan)
  uint32_t* stage;            // [n_scan_waves][work_region] the pair scan's deferred-class windows (query | class << 30)
  uint2* tally;               // [n_scan_waves] {hit records, region bytes used in 16-B units}
  uint2* wg_tally;            // [scan workgroups] the sums over its 16 waves
  uint64_t work_region;
  int64_t n_scan_waves;
  uint32_t* counters;  // [kNumClasses]
  uint32_t* lists;     // [kNumClasses][n]
  unsigned long long* stats;  // [kNumStats] deferred-kernel counters
  uint4* dhits;        // [n] hit records of the deferred paths (final format; kHitOffsetFlag: word = arena offset)
  uint32_t* dhit_count;
  // fused result pack (k_explain_scan on the device path): each workgroup
  // publishes its {hits, 16-B units} in agg[] (bit 63 = published), sums its
  // predecessors' and writes its waves' dense records and payload; the last
  // workgroup writes the header
  int fused;
  uint64_t* agg;       // [n_wg] this pass
  uint64_t* agg_next;  // [n_wg] the next pass's: zeroed by block 0
  uint4* hits_out;     // dense hit list
  uint16_t* hit_refs;  // per scan hit: its first pair-list entry | 0x8000 for OVERFLOW (sst_result_pair_hits)
  uint8_t* dense;      // dense payload
  uint64_t* hdr;       // device header
  uint64_t* hdr_host;  // host-mapped header (device address)
  uint64_t pass_id;
  int dbg;  // DIAGNOSTIC (SST_PACK_DBG): 1 no record copy, 2 no payload copy, 4 no look-back wait
};

// hit records: {query | flags, count (saturated to u32), word lo, word hi};
// word = the byte offset of the query's candidates (SOME) or its exact
// candidate count (OVERFLOW / ABORTED, no payload).  The deferred paths set
// kHitOffsetFlag on SOME records (word = arena offset, rebased by the pack).
constexpr uint32_t kHitOffsetFlag = 1u << 31;

// control block layout (u64 words of one pass).  The counters the deferred
// kernel's waves all add to (spill cursor, hit records, stats) sit 2 KB
// apart: same-line atomics from every wave serialise in one memory channel
// (config 1: deferred kernel 96.5 -> 94.2 us with them apart)
enum {
  kCtlCursor = 0,       // spill cursor
  kCtlCounters = 1,     // [1..2]: u32 class counters x kNumClasses
  kCtlExactRetries = 3,
  kCtlArenaRetries = 13,
  kCtlRegionNeed = 14,  // largest region a scan wave would have needed (when one overflowed)
  kCtlStats = 256,      // [256..264): deferred-kernel stats
  kCtlDhits = 512,      // u32 deferred hit records
  kCtlWords = 1024      // zeroed by one 1024-lane scan workgroup
};

// result header written by k_result_pack (u64 words)
enum {
  kHdrHits = 0,         // dense hit records
  kHdrPayload = 1,      // dense payload bytes
  kHdrRouted = 2,       // windows the scan queued for the deferred kernel (SHALLOW items + class lists)
  kHdrExactRetries = 3,
  kHdrArenaRetries = 4, // SOME queries whose scan-wave region was full
  kHdrCursor = 5,       // raw spill cursor (sizes a retry's spill area)
  kHdrPass = 6,         // pass id the header belongs to
  kHdrRegionNeed = 7,   // largest region a scan wave would have needed (sizes a retry's regions)
  kHdrQueries = 8,      // explain queries of the pass (the rows step produces its own)
  kHdrRowsErr = 9,      // rows step: 1 a spectrum over kRowsMaxPeaks, 2 a side over kRowsMaxSide, 4 no room
  kHdrWords = 10
};

struct PackArgs {
  const uint2* tally;
  const uint2* wg_tally;
  const uint4* work;
  uint64_t work_region;
  const uint8_t* arena;
  uint64_t region_bytes, spill_base, spill_cap;
  const uint64_t* ctl;
  const uint4* dhits;
  uint4* hits;         // dense hit list out
  uint8_t* payload;    // dense payload out
  uint64_t* hdr;       // device copy of the header
  uint64_t* hdr_host;  // host-mapped copy (may be null)
  uint64_t pass_id;
  int n_wg;
  int dbg;  // DIAGNOSTIC (SST_PACK_DBG): 1 no hit stores, 2 no payload copy, 4 no host header, 8 only round 1
  // after a fused scan (which wrote the dense records and payload of its own
  // queries): only the deferred paths' records and spill bytes are packed,
  // behind the scan's totals
  int scan_packed;
  uint64_t scan_hits, scan_bytes;
};

struct ValidArgs {  // is_valid_mass batch
  const uint64_t* valid;
  int64_t limit, full_lo, full_hi, first_reach;
  const double* mass;
  const double* thr;  // may be null: tolerance * mass
  int64_t n;
  double tol, prec, rprec;
  int8_t* out;
};

struct PeakShifts {  // breakage weight x precision per output block (k_is_valid_peaks)
  double shift[4];
};

struct LBArgs {
  const double* su;
  const double* obs;
  int64_t n;
  double tol, prec, rprec;
  int A0;         // round(seq.modification_rate * seq.max_len)
  int dir;        // 0 lower, 1 upper
  int max_len;
  int64_t* out;
  int8_t* status;
  uint32_t* exact_list;
  uint32_t* exact_count;
  const uint64_t* layers;  // [n_layers][layer_words]; null: no fast path
  int64_t layer_words;
  int n_layers;
  int64_t layer_limit;     // layers cover masses [0, layer_limit)
  uint64_t node_budget;
  // per-query alphabets (sst_length_bound_alpha_batch): row masks alpha[2 g],
  // [2 g + 1] over the table's rows, spec[i] = query i's; null: all rows
  const uint64_t* alpha = nullptr;
  const int32_t* spec = nullptr;
  int comp = 32;
  // with the alphabets' per-row reachability (ReachArgs layout, spectrum
  // spec[i]): the replay reads the reduced table's pairs from it instead of
  // the full table's index -- exact for both directions; both = 1: one replay
  // gives the lower bound in out[] and the upper in out_hi[]
  const uint32_t* reach_bits = nullptr;
  const uint64_t* reach_off = nullptr;
  const int64_t* reach_words = nullptr;
  int both = 0;
  int64_t* out_hi = nullptr;
  // per-query max_len (wave mode; null: max_len, A0 and the table's caps for
  // every query): query i's caps caps_len[qlen[i] * kMaxRows + r] and
  // max_modifications a0_len[qlen[i]] (the host's round(L * rate))
  const int32_t* qlen = nullptr;
  const int32_t* caps_len = nullptr;
  const int32_t* a0_len = nullptr;
  uint64_t* nodes_out = nullptr;  // may be null: per query, phase-1 nodes visited (summed over attempts)
  int fuse = 0;  // wave mode with both: the values computed inside phase 1 (vals holds 2 slices per wave)
  int soft = 0;  // node_budget is the caller's soft budget: a query over it gets kLBHeavy, not SST_ABORTED
};

// per-row reachability of reduced alphabets (sst_reach.hip): spectrum g's
// kept rows r_0 < r_1 < ... (alpha, row 0 excluded), row k's bitset of
// masses [0, 32 words[g]) at bits + off[g] + k * words[g] (u32 words)
struct ReachArgs {
  const uint64_t* alpha;   // [2 n_spec]
  const int64_t* words;    // [n_spec]
  const uint64_t* off;     // [n_spec]
  uint32_t* bits;
  const int* w;            // the table's row masses
  int n_rows;
  int64_t n_spec;
};
hipError_t launch_reach_rows(const ReachArgs& a, int n_wg, hipStream_t st);
// lr[lr_off[g] + m] = the lowest kept rank k with m in R_k (0xFF: none)
hipError_t launch_reach_lowest(const ReachArgs& r, const uint64_t* lr_off, uint8_t* lr, hipStream_t st);

// the first-visit frontier (sst_frontier.hip): length bounds on reduced
// alphabets without replaying the DFS
struct FQInfo {       // per listed query of a chunk
  int64_t hi, lo;     // quantised window
  uint64_t lr_off;    // its alphabet's lowest-rank bytes
  uint32_t i;         // query index
  uint16_t K;         // kept rows (row 0 excluded)
  uint16_t L;         // max_len
  uint16_t A0;        // max_modifications (clamped to 255)
  uint16_t pad;       // bit 0: excluded by k_lbf_setup (answered SST_ABORTED)
};
struct FCtl {
  uint32_t node_ctr;
  uint32_t overflow;  // bit 0 nodes, 1 a hash table, 2 a band list, 3/4/5 internal
  uint32_t list_cnt[8];
  uint32_t max_band, max_win, max_k, crec_ctr;
  uint64_t max_hi;
  uint32_t node_ticket;  // k_lbf_nodes' next id range (reset per band by k_lbf_mark)
  uint32_t max_need;     // max over the chunk's queries of K + hi / w_min (key bits besides the root index)
  uint64_t edges;        // left moves onto a mass > 0 (k_lbf_values: one add per wave and band)
};
struct FrontierArgs {
  const uint32_t* list;  // the list pass's live queries
  uint32_t chunk0, n_chunk;
  const double* su;
  const double* obs;
  double tol, prec, rprec;
  const int32_t* spec;
  const uint64_t* alpha;
  const uint8_t* lr;
  const uint64_t* lr_off;
  const int32_t* qlen;
  const int32_t* caps_len;
  const int32_t* a0_len;
  int A0, max_len;
  int wb;          // band width: the table's lightest row (every left move crosses >= 1 band)
  int ring, jump;  // hash / list ring size (power of two > jump), max bands one left move crosses
  int rb;          // key: root index bits (then the ranks in unary)
  int epoch;       // hash tags of this chunk (0..31; the tables are cleared when it wraps)
  int rstride;     // root slots per query
  int n_bands;     // band_start[n_bands] = the chunk's node count (after the last band)
  FQInfo* qi;
  uint32_t* qrow;  // [n_chunk][128]: rank -> w | cap << 20 | is_mod << 28
  uint32_t* root_node;  // per root slot: the root node's packed value (pushed by k_lbf_values)
  uint8_t* flags;
  uint32_t* lpar;  // per node with a left parent: the parent's id, or kRootBit | its root slot (kFPar)
  uint16_t* lval;  // per node with a left move onto a mass > 0: its left child's lower | (upper + 1) << 8,
                   // pushed by the child
  uint64_t ncap;
  char* gtab;
  uint32_t gmask;
  char* ctab;
  uint32_t cmask;
  uint32_t* glist;
  FCtl* ctl;
  uint32_t* band_start;
  uint32_t* band_groups;
  int64_t* lower;
  int64_t* upper;
  int8_t* status;
  uint64_t* nodes_out;
  uint32_t* node_cnt;  // [n_chunk] memo entries per listed query (added to nodes_out when the chunk completes)
  // the band being processed: its groups' records (list order), their left
  // candidates, and node (id - band start) -> group
  char* grec;
  uint64_t grec_cap;
  char* crec;
  uint64_t crec_cap;
  uint32_t* node_group;
  uint64_t ngrp_cap;
};
hipError_t launch_lbf_setup(const TableArgs& t, const FrontierArgs& a, hipStream_t st);
hipError_t launch_lbf_sweep(const FrontierArgs& a, int key_words, int n_bands, int band_blocks, hipStream_t st);
size_t lbf_cand_bytes(int key_words);
size_t lbf_group_bytes();
size_t lbf_grec_bytes();
size_t lbf_crec_bytes(int key_words);

struct ExactWs {
  char* hash;
  char* frames;
  char* stacks;
  uint64_t* epochs;
  uint32_t hash_cap;
};

// The gather's wire format v5 (sst_wire_pack, include/sst.h).  Header words
// (u64): magic, n_valid, n_explain, n_pair, n_explicit, explicit payload
// bytes, n_wg, key, w, n_list (the device counter), list capacity, list
// offset, 4 reserved.  Sections (8-B aligned): valid bits, hit bits,
// w-bit first entries, 3-bit count codes (10 per u32), 12-B explicit records, explicit
// payload, 8-B list entries.
constexpr uint64_t kWireMagic = 0x3557545353ull;  // "SSTW5"
constexpr int kWireHeaderWords = 16;
constexpr int kWireListWord = 9;
struct WireArgs {
  const int8_t* valid;
  const int8_t* status;
  const uint4* hits;
  const uint16_t* refs;
  uint8_t* out;
  int64_t n7, n8;
  uint64_t n_pair, n_exp, pair_bytes, list_cap;
  uint64_t o_vbits, o_sbits, o_first, o_codes, o_exp, o_list;
  uint64_t nb_v, nb_s, nw_f, nw_c;  // region sizes: bytes, bytes, u32 words, u32 words
  uint32_t be_v, be_s, be_f, be_c, be_e;  // cumulative block ends per role
  int w;
  uint64_t hdr[kWireHeaderWords];
};
hipError_t launch_wire_pack(const WireArgs& a, hipStream_t st);

// queries on per-spectrum reduced alphabets (sst_alpha.hip): spectrum g's
// alphabet is the row set masks[2g] (rows 0..63) | masks[2g+1] (rows 64..119)
// of the full table
struct AlphaArgs {  // k_valid_alpha: is_valid_mass on the reduced tables
  const double* mass;
  const double* thr;       // may be null: tolerance * mass
  const double* thr_obs;   // may be null: else thr = tolerance * thr_obs[i] (the rows' observed masses)
  const int64_t* offsets;  // [n_spec + 1] query ranges (each in mass order); with `base`: peak offsets
  const uint32_t* counts;  // may be null; else spectrum g's queries are [4 offsets[g], + counts[g]) (row slots)
  const uint8_t* active;   // may be null; else only spectra with active[g] are answered
  uint8_t* alive;          // may be null; else alive[i] &= (answer == 1) instead of writing out
  uint32_t* err;           // with alive: | 8 when a row's window leaves its reduced table
  const uint64_t* masks;
  const int* w;            // full table row masses
  int n_rows;
  double tol, prec, rprec;
  int8_t* out;
  // the closure of the table's canonical rows (every alphabet the reduction
  // produces keeps them): bit m of u32 word m / 32 set iff m is a sum of
  // canonical rows, for m < 32 canon_words; a spectrum whose mask holds every
  // canonical row starts its closure from it and adds only its other rows
  const uint32_t* canon_closure;  // may be null
  int64_t canon_words;
  uint64_t canon0, canon1;  // the canonical rows' mask
};
struct PairAlphaArgs {  // k_pairs_alpha: explain on pair-class windows
  const double* mass;
  const double* thr;
  const int32_t* spec;
  const uint64_t* masks;
  int64_t n;
  double tol, prec, rprec;
  int8_t* status;
  uint32_t* count;
  uint64_t* rowmask;  // [2n]
  uint32_t* range;    // [2n] pair-list entries [first, end)
};
hipError_t launch_valid_alpha(const AlphaArgs& a, int64_t n_spec, hipStream_t st);

// the step from the peaks (sst_rows.hip)
constexpr int kRowsMaxPeaks = 1024;   // peaks per spectrum a workgroup holds
constexpr int kRowsMaxSide = 2048;    // rows per side (two breakages per side at most ... x 2 headroom)
constexpr int kRowsWaveMaxPeaks = 160;  // spectra up to this many peaks: one wave each (k_rows_*_w)
// answer slots per peak and side of the rows step's count pass (config 3:
// 10 queries per peak over both sides)
constexpr int kRowsAnsPerPeak = 24;
constexpr int kRowsTile = 64;  // chunks per tile of the rows step's offsets
struct RowsArgs {
  const double* obs;          // [n_peaks] sorted within each spectrum
  const int64_t* peak_off;    // [n_spec + 1]
  int64_t n_spec, n_peaks;
  const double* intensity;    // may be null: every peak passes
  double intensity_cutoff, mass_cutoff, max_variance;
  const double* su_seq;       // [n_spec] SequenceInformation.su_mass per spectrum
  double shift[4];
  uint8_t sides[4];           // per breakage: bit0 START side, bit1 END side
  int n_shifts;
  double max_weight, tol, prec, rprec;
  uint32_t cap;               // candidate cap (OVERFLOW beyond)
  int8_t* valid_out;          // [n_shifts * n_peaks]
  double* rows_su;            // scratch [4 * n_peaks]
  double* rows_ob;
  uint32_t* side_rows;        // [2 n_spec]
  // the wave kernels' answers, written once by the count pass, per 64-query
  // window of a side: the mask of queries with an answer other than NONE and
  // those answers' words (count << 16 | first entry, or 1 for EMPTY;
  // sst_rows.hip ans_word), side sd of spectrum g from window
  // ans_win_base(peak_off[g], P_g, sd, g) on (masks at 128 g + 64 sd) when
  // its queries fit its kRowsAnsPerPeak * P_g slots (else the emit pass
  // answers that side again from its scratch rows)
  uint64_t* ans_mask;         // [128 n_spec]
  uint32_t* ans_ent;          // [64 (2 kRowsAnsPerPeak n_peaks / 64 + 2 n_spec + 2)]
  uint32_t* ans_q;            // [2 n_spec] the side's queries, ~0: did not fit
  uint32_t* totals;           // [3 n_spec] queries, hits, payload bytes
  unsigned long long* chunk_tot;  // [3 n_chunks] totals of each wave's contiguous chunk of spectra
  uint64_t* chunk_off;        // [3 n_chunks] their exclusive offsets (k_rows_emit_w)
  unsigned long long* tile_tot;  // [2][3 n_tiles] sums of kRowsTile consecutive chunks, by step parity: the
                              // count kernels add into tile_par's and zero the other's (zeroed at allocation)
  int64_t n_tiles;
  uint32_t tile_par;          // alternates between consecutive rows steps on one result
  int64_t chunk, n_chunks;    // spectra per chunk, chunks (= waves of the wave kernels' grid; set at launch)
  int64_t chunk_cap;          // chunk arrays' capacity (chunks)
  uint64_t* ctl;              // [4] totals
  uint32_t* err;
  uint32_t* done;
  uint32_t* tickets;          // [3]: [2] spectra listed in `big`, [1] in `redo` ([0] spare)
  uint32_t* big;              // [n_spec] spectra over kRowsWaveMaxPeaks peaks (the block kernels')
  uint32_t* redo;             // [n_spec] the wave kernels' spectra with a side past its answer slots (tickets[1])
  uint64_t cap_queries, cap_bytes;
  int8_t* status;
  uint4* hits;
  uint16_t* refs;
  uint8_t* dense;
  uint64_t* hdr;
  uint64_t* hdr_host;
  uint64_t pass_id;
};
hipError_t launch_rows_step(const TableArgs& t, const RowsArgs& a, int n_wg, size_t dyn, hipStream_t st);

// config 5 on the device (sst_pipe.hip)
constexpr int kPipeMaxPeaks = 4096;  // peaks per spectrum the classify workgroup holds (77 KB of LDS)
constexpr int kPipeMaxRows = 2048;   // rows per spectrum the LDS variants of the row kernels hold
constexpr int kPipeMaxPeaksBig = 16383;  // peaks per spectrum k_classify_rows_big takes (u16 peak and row indices)
constexpr int kPipeBigRows = 4 * kPipeMaxPeaksBig;  // rows per spectrum in the HBM-scratch variants (< 2^16)
// A spectrum of more than kPipeMaxRows rows is handled by the *_big variants
// of k_fix_round / k_dict / k_fix_finish / k_bins_*: the same code over a
// workgroup's slice of HBM scratch (PipeArgs big*) instead of LDS arrays,
// with a dict hash of big_slots entries.  Layout of one slice:
struct PipeBigLayout {
  uint64_t su, ob, q0, q1, hkey, hidx, sk, si, s0, s1, single, b0, b1, stride;
};
__host__ __device__ inline PipeBigLayout pipe_big_layout(uint32_t rows, uint32_t slots) {
  PipeBigLayout L{};
  uint64_t o = 0;
  auto take = [&o](uint64_t bytes) {
    const uint64_t at = o;
    o += (bytes + 255) & ~255ull;
    return at;
  };
  L.su = take(8ull * rows);
  L.ob = take(8ull * rows);
  L.q0 = take(4ull * (rows + 1));
  L.q1 = take(4ull * (rows + 1));
  L.hkey = take(8ull * slots);
  L.hidx = take(4ull * slots);
  L.sk = take(8ull * slots);  // the dict's entries sorted by key (bitonic, k_dict_big)
  L.si = take(4ull * slots);
  L.s0 = take(2ull * rows);
  L.s1 = take(2ull * rows);
  L.single = take(2ull * rows);
  L.b0 = take(2ull * (rows + 1));
  L.b1 = take(2ull * (rows + 1));
  L.stride = o;
  return L;
}
struct PipeArgs {
  const double* obs;          // [n_peaks], any order within each spectrum
  const int64_t* peak_off;    // [n_spec + 1]; rows of spectrum g live at slots 4 * peak_off[g] + i
  int64_t n_spec, n_peaks;
  const double* intensity;
  double intensity_cutoff, mass_cutoff, max_variance;
  const double* su_seq;
  double shift[4];
  uint8_t sides[4];
  int n_shifts;
  double max_weight, tol, prec, rprec;
  const int64_t* masses;      // the table's integer masses (is_singleton)
  int n_masses;
  int8_t* valid_out;          // may be null: A7 codes [n_shifts * n_peaks]
  double* r_su;
  double* r_ob;
  uint32_t* r_meta;           // breakage | sides << 2 | singleton << 4 | peak << 8
  uint8_t* alive;
  uint32_t* cnt;              // [n_spec] rows
  const uint64_t* alpha;      // [2 n_spec] this round's alphabets
  uint64_t* alpha_next;
  const uint8_t* active;      // [n_spec] spectra running this round
  uint8_t* active_next;
  uint32_t* rounds;           // [n_spec]
  uint32_t* queries;          // [n_spec] explain queries issued over the rounds
  uint32_t* n_active;         // spectra whose alphabet shrank this round
  uint64_t canon[2];          // the canonical rows (never dropped)
  uint32_t* n_q;              // [n_spec] skeleton bin queries (k_bins count pass)
  uint32_t* n_q0;             // may be null: [n_spec] of those, the START side's
  uint64_t* q_off;            // [n_spec + 1] their exclusive offsets (total last)
  int8_t* q_status;           // [total] per bin query: SST_NONE / EMPTY / SOME, kStatusPending off the pair class
  uint32_t* q_count;          // [total] candidates on the spectrum's alphabet
  // off-pair-class bin queries listed for the masked explain (may be null):
  // window mass, threshold, spectrum and bin-query index; n_def their count
  double* def_mass;
  double* def_thr;
  int32_t* def_spec;
  uint64_t* def_q;
  uint32_t* n_def;
  uint32_t* err;
  // spectra whose budgets can bind on pair-class windows (pair_ok[g] == 0;
  // null: none): their windows need the exact masked explain.  k_fix_round /
  // k_dict list such a spectrum's queries (xq_*, a block per spectrum in
  // xq_block[g] = start << 32 | count) instead of answering them; the caller
  // answers the list (sst_explain_alpha_batch_device, sst_result_refs_device
  // into xa_*) and k_fix_finish / k_dict's build pass read the answers
  const uint8_t* pair_ok;
  double* xq_mass;
  double* xq_thr;
  int32_t* xq_spec;
  uint8_t* xq_single;
  uint32_t* xq_count;
  uint64_t xq_cap;
  uint64_t* xq_block;
  const int8_t* xa_st;
  const uint32_t* xa_n;
  const uint64_t* xa_ptr;
  // HBM scratch of the big-spectrum variants (null: a spectrum of more than
  // kPipeMaxRows rows is an error, bit 2); big_wg slices of big_stride bytes
  uint8_t* big;
  uint64_t big_stride;
  uint32_t big_rows, big_slots;
  int big_wg;
};
hipError_t launch_fix_finish(const PipeArgs& a, int n_wg, hipStream_t st);
// filter_by_explanation's final explanation dict per spectrum (sst_pipe.hip,
// k_dict): the dict the last round built (prediction.py:261-329: a side pair
// is stored only with >= 1 explanation, a singleton always, a later equal key
// replaces an earlier one) over the final alive rows and alphabet.  The
// skeleton walk looks its bin differences up in it (skeleton_building.py:
// 429-430) -- a hit answers with the dict's value, i.e. the same window at
// the last writer's threshold.
struct DictArgs {
  uint32_t* n_q;         // count pass: [n_spec] the final round's queries (>= its entries)
  const uint64_t* off;   // build pass: [n_spec + 1] region offsets (exclusive scan of n_q)
  uint64_t* key;         // [total] keys ascending (double bits, -0.0 folded into 0.0)
  double* thr;           // [total] the last writer's threshold
  uint32_t* n_ent;       // [n_spec] entries
};
// mode 1: count, 2: list the exact-mode spectra's queries (PipeArgs xq_*),
// 0: build (exact-mode spectra read their listed answers xa_*)
hipError_t launch_dict(const TableArgs& t, const PipeArgs& a, const DictArgs& d, int mode, int n_wg,
                       hipStream_t st);
hipError_t launch_scan_u32(const uint32_t* in, uint64_t* out, int64_t n, hipStream_t st);
hipError_t launch_requery_merge(const sst_requery_merge_args& a, uint32_t* tot, uint64_t* off, hipStream_t st);
// the skeleton walk (sst_skel.hip, k_skel_walk): the public sst_walk_args
constexpr int kWalkMaxRounds = SST_WALK_MAX_ROUNDS;
enum { kWalkDone = SST_WALK_DONE, kWalkSuspended = SST_WALK_SUSPENDED, kWalkBig = SST_WALK_BIG,
       kWalkRaise = SST_WALK_RAISE, kWalkLimit = SST_WALK_LIMIT, kWalkRounds = SST_WALK_ROUNDS,
       kWalkMissing = SST_WALK_MISSING };
using WalkArgs = sst_walk_args;
hipError_t launch_skel_walk(const TableArgs& t, const WalkArgs& a, hipStream_t st);
hipError_t launch_jaccard(const sst_jaccard_args& a, hipStream_t st);
hipError_t launch_post_skel(const sst_post_args& a, uint64_t canon0, uint64_t canon1, int n_wg, hipStream_t st);
hipError_t launch_skel_alpha(int64_t n_spec, const int32_t* max_len, const uint64_t* skel_off, const uint64_t* skel,
                             const uint64_t* alpha, uint64_t canon0, uint64_t canon1, uint64_t* out, hipStream_t st);
hipError_t launch_result_refs(const int8_t* status, int64_t n, const uint4* hits, uint64_t n_hits,
                              const uint8_t* payload, const int64_t* dst, uint64_t* ptr, uint32_t* cnt, int8_t* st,
                              hipStream_t stream);
uint64_t walk_scratch_bytes(uint32_t pos_cap, uint32_t len_cap, uint32_t expl_cap, uint32_t cand_cap,
                            uint32_t tset_cap);
hipError_t launch_bins_count(const PipeArgs& a, int n_wg, hipStream_t st);
hipError_t launch_bins_emit(const TableArgs& t, const PipeArgs& a, int n_wg, hipStream_t st);
hipError_t launch_classify_rows(const TableArgs& t, const PipeArgs& a, int n_wg, hipStream_t st);
hipError_t launch_fix_round(const TableArgs& t, const PipeArgs& a, int n_wg, hipStream_t st);
size_t rows_lds_bytes();
hipError_t launch_pairs_alpha(const TableArgs& t, const PairAlphaArgs& a, hipStream_t st);

hipError_t launch_bits_seed(uint64_t* R0, int64_t nwords, hipStream_t st);
hipError_t launch_bits_shift_or(uint64_t* dst, const uint64_t* src, int64_t k, int64_t nwords, int64_t nbits,
                                hipStream_t st);
hipError_t launch_pack(int C, const uint64_t* R, int64_t rw, int n_rows, const int64_t* w, int64_t ncols, int64_t M,
                       uint64_t last_mask, const uint8_t* literal, void* out, hipStream_t st);
hipError_t launch_row_literal(int C, const uint64_t* Rprev, int64_t ncols, int shift, void* row, int64_t rw,
                              uint64_t* Rout, hipStream_t st);
hipError_t launch_index(int C, const void* packed, int n_rows, int64_t ncols, int64_t M, ulonglong2* index,
                        uint64_t* valid, int* err, hipStream_t st);
hipError_t launch_is_valid(const uint64_t* valid, int64_t limit, int64_t full_lo, int64_t full_hi, int64_t first_reach,
                           const double* mass, const double* thr, int64_t n, double tol, double prec, int8_t* out,
                           hipStream_t st);
hipError_t launch_is_valid_peaks(const uint64_t* valid, int64_t limit, int64_t full_lo, int64_t full_hi,
                                 int64_t first_reach, const double* obs, int64_t n, const double* shifts, int n_w,
                                 double tol, double prec, int8_t* out, hipStream_t st);
// the pair scan with is_valid over peaks x 4 breakage weights in front of it, one launch (k_step)
hipError_t launch_step(const TableArgs& t, const QueryArgs& q, const OutArgs& o, int n_blocks, const double* obs,
                       int64_t n_peaks, const double* shifts4, double tol, double prec, int8_t* valid_out,
                       hipStream_t st);
hipError_t launch_explain_scan(const TableArgs& t, const QueryArgs& q, const OutArgs& o, int n_blocks,
                               hipStream_t st);
hipError_t launch_explain_expand(const TableArgs& t, const QueryArgs& q, const OutArgs& o, int n_blocks,
                                 hipStream_t st);
int explain_scan_blocks_per_cu(size_t dyn_lds);
int explain_expand_blocks_per_cu();
size_t scan_dyn_lds(const TableArgs& t);
hipError_t launch_result_pack(const PackArgs& p, hipStream_t st);
hipError_t launch_hits_to_arrays(const uint4* hits, uint64_t n_hits, const int8_t* status, uint64_t* count,
                                 uint64_t* offset, hipStream_t st);
hipError_t launch_explain_deferred(const TableArgs& t, const QueryArgs& q, const OutArgs& o, void* ws_deep,
                                   int shallow_blocks, int deep_blocks, const ExactWs& ws, int exact_blocks,
                                   hipStream_t st);
size_t glob_frame_bytes();
hipError_t launch_layer_step(const uint64_t* prev, uint64_t* next, int64_t nwords, const int* w, int n_rows,
                             hipStream_t st);
hipError_t launch_length_bound(const TableArgs& t, const LBArgs& q, char* hash, int8_t* vals, char* frames,
                               uint32_t hash_cap, int exact_units, bool fast_pass, hipStream_t st);
size_t lb_frame_bytes();
hipError_t launch_is_singleton(const int64_t* masses, int n_masses, const double* mass, const double* thr, int64_t n,
                               double tol, double prec, int8_t* out, hipStream_t st);
hipError_t launch_explain_recursion(const TableArgs& t, const QueryArgs& q, const OutArgs& o, char* hash,
                                   char* frames, uint32_t hash_cap, int units, hipStream_t st);
size_t rec_frame_bytes();
size_t rec_entry_bytes();
size_t p1_frame_bytes();
size_t hash_entry_bytes();

}  // namespace sst
