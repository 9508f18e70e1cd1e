/*
 * sst.h -- C ABI of the MI355X mass-explanation engine (libsstgpu.so).
 *
 * Drop-in boundary for spectrseq/spectrseqtools' per-peak combinatorial
 * search.  The reference has no FFI (it is pure Python); these entry points
 * are what its hot-path functions call through ctypes in
 * spectrseqtools_amd/_native.py.  Each declaration cites the reference
 * interface it replaces (paths relative to the reference repo root).
 *
 * Conventions
 *   - plain C types only; host pointers unless the name ends in _device;
 *   - every function returns 0 on success or a negative SST_E* code; the
 *     message is available from sst_last_error(ctx);
 *   - one sst_ctx per HIP device; calls on one ctx are serialised; a table
 *     belongs to the ctx that made it;
 *   - masses are f64 Da; windows are quantised exactly as the reference does
 *     (mass_explanation.py:107,110-114): target = round(mass/precision) with
 *     ties-to-even, thr = ceil((thr_abs or tolerance*mass)/precision).
 */
#ifndef SST_H
#define SST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- return codes ---------------------------------------------------- */
#define SST_OK 0
#define SST_E_ARG (-1)      /* bad argument / shape                         */
#define SST_E_HIP (-2)      /* HIP runtime error                            */
#define SST_E_NOMEM (-3)    /* device allocation failed                     */
#define SST_E_TABLE (-4)    /* packed table violates the DP recurrence      */
#define SST_E_INTERNAL (-5) /* depth/budget guard tripped                   */

/* ---- per-query status of sst_explain_batch -------------------------- */
#define SST_NONE 0          /* reference returns MassExplanations(None)      */
#define SST_EMPTY 1         /* reference returns MassExplanations(set())     */
#define SST_SOME 2          /* >= 1 candidate composition                    */
#define SST_OUT_OF_TABLE (-1) /* reference raises NotImplementedError naming */
                              /* its window value (mass_explanation.py:68-72, */
                              /* :134-138 with `value` bound at :192)        */
#define SST_OVERFLOW (-2)   /* count > cap_per_query: exact count, no payload */
#define SST_ABORTED (-4)    /* DFS node guard (2^34 nodes) exhausted: count is a lower bound */

/* ---- per-query result of sst_is_valid_batch ------------------------- */
/*  1 = True, 0 = False, -1 = reference raises NotImplementedError          */

typedef struct sst_ctx sst_ctx;
typedef struct sst_table sst_table;
typedef struct sst_result sst_result;

/* Number of visible HIP devices (0 when none). */
int sst_device_count(void);

/* One context per GPU (one process per GPU in multi-GPU runs). */
int sst_ctx_create(int device, sst_ctx** out);
void sst_ctx_destroy(sst_ctx* ctx);
const char* sst_last_error(const sst_ctx* ctx);
/* The HIP stream all work of this ctx is queued on (hipStream_t). */
void* sst_ctx_stream(sst_ctx* ctx);
/* Queue this ctx's subsequent work on `stream` (a hipStream_t of the ctx's
 * device, owned by the caller), or on the ctx's own stream again when NULL.
 * Set-stream semantics as in rocBLAS: nothing is ordered across the switch,
 * the caller orders work on different streams (events).  A result's later
 * operations (compaction, fetch, free) go to the ctx's stream at that time.  Used to overlap the A7
 * batch with the A8 chain (bench.py).  No reference equivalent (the
 * reference is single-threaded Python). */
int sst_ctx_set_stream(sst_ctx* ctx, void* stream);
/* Wait for all queued work of this ctx. */
int sst_ctx_synchronize(sst_ctx* ctx);
/* Release the ctx's cached work buffers: the first-visit frontier's
 * workspaces that sst_length_bounds_frontier_device and
 * sst_length_bound_batch keep across calls (up to min(96 GB, free / 2) and
 * 4 GB), so that later stages, other allocators or another process on the
 * same GPU get that HBM back.  Waits for the ctx's queued work first; the
 * next frontier call allocates again.  No reference equivalent (the
 * reference's memo dict is freed when compute_sequence_length_bound returns,
 * mass_table.py:361). */
int sst_ctx_trim(sst_ctx* ctx);

/* Build the packed 2-bit DP reachability table on the GPU.
 * Replaces set_up_bit_table(integer_masses, max_mass, compression_rate)
 * (spectrseqtools/mass_table.py:207-248; settings :251-289) and therefore
 * load_dp_table / _reduce_nucleotide_list (:319-340, :102-121).
 * masses: sorted unique integer masses incl. the 0 sentinel (row 0),
 * n_rows <= 120; compression in {4, 8, 16, 32}. */
int sst_table_build(sst_ctx* ctx, const int64_t* masses, int n_rows, int64_t max_mass, int compression,
                    sst_table** out);

/* Adopt an existing packed table (e.g. the reference's .npy cache,
 * load_dp_table mass_table.py:319-340): words are n_rows x n_cols elements
 * of compression/4 bytes, C order.  Fails with SST_E_TABLE if the table
 * does not satisfy the row recurrence the engine's index relies on. */
int sst_table_upload(sst_ctx* ctx, const int64_t* masses, int n_rows, const void* words, int64_t n_cols,
                     int compression, sst_table** out);

/* Row budgets the explain DFS reads from DynamicProgrammingTable.masses:
 * is_mod[r] = NucleotideMass.is_modification, cap[r] =
 * round(seq.max_len * NucleotideMass.modification_rate)
 * (mass_explanation.py:158-172, :200). */
int sst_table_set_budgets(sst_table* t, const uint8_t* is_mod, const int64_t* cap);

int sst_table_shape(const sst_table* t, int* n_rows, int64_t* n_cols, int* compression);
/* Copy the packed table to host (n_rows*n_cols*(compression/4) bytes):
 * the DynamicProgrammingTable.table ndarray (mass_table.py:54). */
int sst_table_download(sst_table* t, void* words_out);
void sst_table_destroy(sst_table* t);

/* is_valid_mass (mass_explanation.py:45-89), one result per query.
 * thr_abs may be NULL (reference default threshold = tolerance*mass). */
int sst_is_valid_batch(sst_table* t, const double* mass, const double* thr_abs, int64_t n, double tolerance,
                       double precision, int8_t* out);
/* Same on device buffers, queued on the ctx stream (no synchronisation). */
int sst_is_valid_batch_device(sst_table* t, const double* d_mass, const double* d_thr_abs, int64_t n,
                              double tolerance, double precision, int8_t* d_out);

/* is_valid_mass over peaks x breakage weights, as classify_fragments maps it
 * over its concatenated frame (fragment_classification.py:39-67): for every
 * peak p and shift k, mass = obs[p] - shifts[k] and threshold = tolerance *
 * obs[p] (shifts[k] = breakage weight x precision, computed by the caller as
 * the reference does); out[k * n_peaks + p] as sst_is_valid_batch
 * (breakage-major, the reference's row order).  Reads each peak once. */
int sst_is_valid_peaks(sst_table* t, const double* obs, int64_t n_peaks, const double* shifts, int n_shifts,
                       double tolerance, double precision, int8_t* out);
int sst_is_valid_peaks_device(sst_table* t, const double* d_obs, int64_t n_peaks, const double* shifts, int n_shifts,
                              double tolerance, double precision, int8_t* d_out);

/* is_singleton (fragment_classification.py:104-119), one result per query:
 * 1 if some value of the quantised window [round(mass/precision) -
 * ceil(thr/precision), ... + ...] is one of masses[0..n_masses) (the caller's
 * integer masses; classify_fragments passes the table's rows, :73-80), else 0.
 * n_masses <= 1024.  thr_abs may be NULL (tolerance*mass). */
int sst_is_singleton_batch(sst_ctx* ctx, const int64_t* masses, int n_masses, const double* mass,
                           const double* thr_abs, int64_t n, double tolerance, double precision, int8_t* out);
/* Same on device buffers, queued on the ctx stream (masses: host array). */
int sst_is_singleton_batch_device(sst_ctx* ctx, const int64_t* masses, int n_masses, const double* d_mass,
                                  const double* d_thr_abs, int64_t n, double tolerance, double precision,
                                  int8_t* d_out);

/* explain_mass_with_table (mass_explanation.py:92-203), batched.
 *   max_mods: per-query budget array (may be NULL) else max_mods_scalar;
 *             a negative value means np.inf (the reference default);
 *   with_memo: the reference's with_memo flag (memo semantics reproduced
 *             exactly, including budget-dependent first-visit effects);
 *   cap_per_query: candidate cap; larger sets report SST_OVERFLOW with the
 *             exact count and no payload.
 *   n <= SST_MAX_EXPLAIN_BATCH per call (the kernels address per-query
 *             arrays with 32-bit byte offsets; split larger batches).
 * Results (host copies) through sst_result_* below. */
#define SST_MAX_EXPLAIN_BATCH (1ll << 29)
int sst_explain_batch(sst_table* t, const double* mass, const double* thr_abs, int64_t n, double tolerance,
                      double precision, const int64_t* max_mods, int64_t max_mods_scalar, int with_memo,
                      uint64_t cap_per_query, sst_result** out);
/* Same with inputs already in HBM; results stay on the device.  Queued on
 * the ctx stream, no host synchronisation: on tables built here the pass is
 * one scan launch that writes the complete result (status bytes, dense hit
 * list, dense payload; see sst_result_hit_list) plus a small header into
 * host-mapped memory (uploaded tables: scan, expand, deferred and pack
 * launches).  If *out is non-NULL it must be a result of the same
 * ctx with capacity >= n: its buffers are reused (no allocation).  The inputs
 * (and the table) must stay valid and unchanged until the pass is settled
 * (sst_result_settle, or the first view / fetch, which settle implicitly):
 * settling waits for the pass and reads its header; only if the scan routed
 * windows to the deferred classes (deep, exact, no-memo and > 2-item windows;
 * the pass launches only the scan and the pack on tables with the pair list)
 * does it launch them and pack again, and only if a query outgrew a payload
 * region, the spill area or the exact path's memo does it re-run the pass
 * with larger workspaces. */
int sst_explain_batch_device(sst_table* t, const double* d_mass, const double* d_thr, int64_t n,
                             double tolerance, double precision, const int64_t* d_max_mods, int64_t max_mods_scalar,
                             int with_memo, uint64_t cap_per_query, sst_result** out);

/* sst_explain_batch_device against per-query reduced alphabets without
 * rebuilding a table: query i is answered as explain_mass_with_table on the
 * table DynamicProgrammingTable._reduce_nucleotide_list (mass_table.py:
 * 94-121) would rebuild for the rows of alphabet d_spec[i] (d_spec null: all
 * queries alphabet 0), given as a row mask over this table's rows:
 * d_alpha[2 g] rows 0..63, d_alpha[2 g + 1] rows 64..127 (row 0, the
 * sentinel, is implied).  The kept rows keep their caps (sst_table_set_budgets
 * of this table).  Every window with values goes to the deferred DFS roles,
 * which walk the alphabet's rows only (the pair scan answers none); a window
 * reaching the reduced table's extent max(kept) * 35 is SST_OUT_OF_TABLE as in
 * the reference, one inside that table's last packed word SST_ABORTED (the
 * reference's last-column mask is not modelled).  Replaces a table rebuild +
 * explain_mass_with_table per alphabet (prediction.py:207 -> :216-227,
 * skeleton_building.py:212 -> :436).  Results, reuse and settling as for
 * sst_explain_batch_device; every d_spec[i] must index d_alpha (device
 * buffers are not range-checked), and d_spec / d_alpha must stay valid until
 * the pass is settled. */
int sst_explain_alpha_batch_device(sst_table* t, const double* d_mass, const double* d_thr, const int32_t* d_spec,
                                   const uint64_t* d_alpha, int64_t n, double tolerance, double precision,
                                   const int64_t* d_max_mods, int64_t max_mods_scalar, int with_memo,
                                   uint64_t cap_per_query, sst_result** out);

/* sst_explain_alpha_batch_device with per-query budgets: query i's row caps
 * are row d_qlen[i] of caps_by_len (host, [n_lens][n_rows]: the caps
 * sst_table_set_budgets would set for that length, round(L * rate)), its
 * max_modifications d_mods[i]; the table's is_modification flags (set by
 * sst_table_set_budgets) are kept.  Every query is answered as one
 * sst_explain_alpha_batch_device call with those budgets set would answer it
 * (the exact memo path: with_memo = 1), so windows of many max_len values
 * go in one pass instead of one pass per value (skeleton_building.py:212 ->
 * :436 per spectrum, each spectrum's SequenceInformation.max_len).  Results,
 * reuse and settling as for sst_explain_batch_device; d_qlen / d_mods must
 * stay valid until the pass is settled. */
int sst_explain_alpha_lens_batch_device(sst_table* t, const double* d_mass, const double* d_thr, const int32_t* d_spec,
                                        const uint64_t* d_alpha, const int32_t* d_qlen, const int64_t* caps_by_len,
                                        int n_lens, int64_t n, double tolerance, double precision,
                                        const int64_t* d_mods, uint64_t cap_per_query, sst_result** out);

/* One step of both predicates on device buffers, as classify_fragments and
 * the explanation stage issue them: sst_is_valid_peaks_device(d_obs, n_peaks,
 * shifts, n_shifts -> d_valid_out) and sst_explain_batch_device(d_mass, ...,
 * out), with the same results.  With 4 breakage weights and a pass whose scan
 * packs its own result, both run in one launch (the pair scan's grid, the
 * is_valid workgroups behind it); otherwise as two launches.  No
 * reference equivalent (it issues the two per row). */
int sst_step_device(sst_table* t, const double* d_obs, int64_t n_peaks, const double* shifts, int n_shifts,
                    int8_t* d_valid_out, const double* d_mass, const double* d_thr, int64_t n, double tolerance,
                    double precision, const int64_t* d_max_mods, int64_t max_mods_scalar, int with_memo,
                    uint64_t cap_per_query, sst_result** out);

/* explain_mass_with_recursion (mass_explanation.py:206-284), batched: the
 * table-free enumerator (target = round(mass/precision), base case
 * |remaining| <= thr at every level, memo keyed (remaining, start) with the
 * first visit's list, per-row caps from sst_table_set_budgets).  max_mods:
 * per-query array or scalar; negative = np.inf; a fractional reference budget
 * is passed floored.  Results as for sst_explain_batch (status, count,
 * offset, payload of ascending row indices); SST_ABORTED when a query
 * exhausts the DFS node budget.  Synchronous. */
int sst_explain_recursion_batch(sst_table* t, const double* mass, const double* thr_abs, int64_t n,
                                double tolerance, double precision, const int64_t* max_mods, int64_t max_mods_scalar,
                                uint64_t cap_per_query, sst_result** out);

/* The step from the peaks: classify_fragments' is_valid and filters
 * (fragment_classification.py:17-101: A7 of every peak x breakage weight into
 * d_valid_out as sst_is_valid_peaks_device, the intensity / mass cuts and
 * filter_by_sequence_mass against d_su_seq[spectrum]) and the first
 * filter_by_explanation round's sliding-window explains of both sides
 * (prediction.py:261-329; no singletons), every producer on the device:
 * per spectrum the kept rows of each side in SU order (a merge of the
 * breakages' sorted streams), the window pairs in closed form and each pair's
 * difference and threshold formed in the kernels.  Spectrum g's peaks are
 * d_obs[d_peak_off[g] .. d_peak_off[g+1]) in any order (at most 1024; a list
 * not in mass order is ranked on the device, equal masses in their given
 * order); sides[k]: bit 0 = breakage k's rows are on the START side, bit 1 = on
 * the END side (both: the sequence-mass lower cut applies); d_intensity may
 * be NULL (every peak passes).  The result holds the explain answers in query
 * order (spectrum-major; START pairs then END pairs; the order
 * collect_diff_explanations_for_su issues them) and the number of queries
 * (sst_result_queries; at most max_queries); its hits all come from the pair
 * list (sst_result_pair_hits, n_scan_wg = 0: query order).  Every window must
 * be pair-class with budgets that cannot bind (checked: SST_E_ARG otherwise).
 * No reference equivalent (the reference issues these one row at a time). */
int sst_step_rows_device(sst_table* t, const double* d_obs, const int64_t* d_peak_off, int64_t n_spec,
                         int64_t n_peaks, const double* d_intensity, double intensity_cutoff, double mass_cutoff,
                         const double* d_su_seq, const double* shifts, const uint8_t* sides, int n_shifts,
                         double max_weight, double tolerance, double precision, int64_t max_mods_scalar,
                         uint64_t cap_per_query, int64_t max_queries, int8_t* d_valid_out, sst_result** out);
/* Number of explain queries of a result (settles it first). */
int sst_result_queries(sst_result* r, int64_t* n);

/* Wait for a result's pass and complete it (see sst_explain_batch_device);
 * reports the dense hit list's length and the dense payload's size.  Other
 * work queued on the ctx stream after the pass keeps running.  No reference
 * equivalent. */
int sst_result_settle(sst_result* r, uint64_t* n_hits, uint64_t* payload_bytes);

/* Host views of a result (valid until sst_result_free; filled by
 * sst_result_fetch, which sst_explain_batch calls):
 *   status[n] (SST_NONE..), count[n] candidates, offset[n] byte offset of the
 *   query's candidates in payload; payload = per candidate one length byte k
 *   followed by k row indices (ascending, i.e. ascending mass); a query's
 *   candidates may be followed by unused bytes (count delimits them).
 *   count[i] and offset[i] are 0 unless status[i] is SST_SOME, SST_OVERFLOW
 *   or SST_ABORTED (the host builds them from the hit list). */
int sst_result_host(sst_result* r, const int8_t** status, const uint64_t** count, const uint64_t** offset,
                    const uint8_t** payload, uint64_t* payload_bytes);
/* Ordering of a result's device buffers: they are written on the stream that
 * was the ctx's stream when the pass was queued (the pass stream); settling
 * queues any further launches (deferred classes, pack, retries) on that same
 * stream, whatever the ctx's stream is at the time.  sst_wire_pack, the views
 * and fetch wait (hipStreamWaitEvent) for the work settling queued when they
 * run on another stream; the pass's own kernels are the caller's to order
 * (e.g. an event recorded on the pass stream right after the launch). */
/* Device views (no copy; settle the result first).  d_status and d_payload
 * (the dense payload) are the pass's own output.  d_count / d_offset are
 * per-query u64 arrays built from the hit list only when asked for (pass
 * NULL to skip them: 16 B per query of extra HBM traffic); their entries are
 * undefined for queries without candidates. */
int sst_result_device(sst_result* r, int8_t** d_status, uint64_t** d_count, uint64_t** d_offset,
                      uint8_t** d_payload, uint64_t* payload_bytes);
/* The dense hit list of a result, on the device (settles it first): one
 * 16-B record {u32 query, u32 count (saturated), u32 word lo, u32 word hi}
 * per query with candidates (SOME, OVERFLOW, ABORTED), where word is the
 * byte offset of the query's candidates in the dense payload (SOME) or the
 * exact candidate count (OVERFLOW, ABORTED: no payload).  Records come in the
 * engine's order (per scan wave, then the deferred paths).  With the status
 * bytes and the payload this is the whole result in ~1 B/query + 16 B per hit
 * (the wire format bench.py --gather sends over RCCL).  Valid until the next
 * pass on this result or its free.  No reference equivalent. */
int sst_result_hit_list(sst_result* r, void** d_hits, uint64_t* n_hits);
/* The pair-path part of a device-path result (settles it first): its first
 * *n_pair_hits dense records are the hits the scan answered from the pair
 * list, and their candidates occupy the first *pair_bytes of the dense
 * payload.  d_refs (u16, one per such record): the first pair-list entry of
 * the query's candidates (entries first .. first + count - 1, records as
 * sst_table_pair_records returns them), | 0x8000 for OVERFLOW.  The records
 * come in the scan's order: workgroup b < *n_scan_wg, its wave w < 16, then
 * that wave's tiles (64 queries each; wave w of workgroup b takes tiles
 * v, v + 16 * n_scan_wg, ... with v = ((w >> 1) * n_scan_wg + b) * 2 + (w & 1)),
 * ascending query within a tile.  0 pair hits after passes that were not
 * fused (host entry points, retries, tables without the pair list).  With
 * the status codes this is the whole pair-path result in ~4 B per hit and
 * no payload (parallel.wire_pack).  No reference equivalent. */
int sst_result_pair_hits(sst_result* r, void** d_refs, uint64_t* n_pair_hits, uint64_t* pair_bytes, int* n_scan_wg);
/* The table's pair list: payload record of entry e (u32: [k][row..] in its
 * low 2-3 bytes, the bytes sst_result_host's payload holds for that
 * candidate); *n = 0 for tables without the list.  recs may be NULL (size
 * query). */
int sst_table_pair_records(sst_table* t, uint32_t* recs, int64_t cap, int64_t* n);
/* One rank's complete step result in the gather's wire format v5, packed on
 * the device by one kernel on the ctx stream (settles r first): d_valid the
 * step's n_valid is_valid codes (int8 -1 / 0 / 1), r its explain result.
 * The layout (8-B aligned sections; spectrseqtools_amd/parallel.py,
 * wire_unpack, decodes it):
 *   header   16 x u64: magic "SSTW5", n_valid, n_explain, n_pair, n_explicit,
 *            explicit payload bytes, n_scan_wg, pair key (FNV-1a of the pair
 *            records), w, n_list, list capacity, list offset, 4 x 0
 *   valid    1 bit per is_valid query: True
 *   status   1 bit per explain query: 1 = SOME / OVERFLOW / ABORTED (a hit),
 *            0 = NONE or listed
 *   first    per pair hit (sst_result_pair_hits, scan order) its first
 *            pair-list entry in w bits, w = ceil(log2(pair-list entries))
 *   codes    per pair hit 3 bits, 10 per u32: its count 1..7, 0 = listed
 *   explicit 12-B records {u32 query | kind << 30, u32 a, u32 b} of the
 *            other hits: kind 0 SOME (a = candidates, b = payload offset),
 *            1 OVERFLOW / 2 ABORTED (a, b = the exact count)
 *   payload  the explicit hits' payload
 *   list     n_list 8-B entries {u32 index | type << 30, u32 value}, in no
 *            particular order: type 0 an is_valid raise, 1 an explain status
 *            other than NONE / SOME (value: the status byte; EMPTY, raises,
 *            OVERFLOW, ABORTED), 2 a pair hit's
 *            count outside 1..7 (index: the pair hit, value: the count)
 * d_out NULL: returns the fixed part's bytes (the list's offset) and packs
 * nothing; otherwise cap (>= that) bounds the buffer and entries beyond it
 * are dropped (the header's n_list still counts them: the receiver checks).
 * d_out must be 8-byte aligned.  Returns the fixed part's bytes or a
 * negative SST_E_*.  No reference equivalent (the north star's RCCL gather of
 * candidate compositions). */
int64_t sst_wire_pack(sst_result* r, const int8_t* d_valid, int64_t n_valid, void* d_out, int64_t cap);
/* Copy device results to the host views (synchronises the ctx stream). */
int sst_result_fetch(sst_result* r);
void sst_result_free(sst_result* r);

/* Counters of the last explain launch (valid after a fetch), for measurement:
 * [0] queries run by the shallow (<= 3 item) fast path, [1] deep fast path,
 * [2] exact (budget-binding) path, [3] no-memo path, [4] index records loaded
 * (node expansions of the counting pass), [5] payload bytes written by those
 * paths, [6] queries answered from the on-chip pair list (<= 2 item windows),
 * [7] payload bytes written by the pair-list path. */
int sst_result_stats(const sst_result* r, uint64_t* stats_out /* [8] */);

/* compute_sequence_length_bound (spectrseqtools/mass_table.py:343-487),
 * batched over (su_mass, obs_mass) pairs: window = round(su/precision) +-
 * ceil(tolerance*obs/precision); max_mods = round(seq.modification_rate *
 * seq.max_len) (:351); per-row caps from sst_table_set_budgets; direction 0 =
 * "lower", 1 = "upper", optionally | SST_LB_EXACT_ONLY | SST_LB_REPLAY.
 * Windows whose budgets provably never bind come from layered reachability;
 * the others, on a table built here (a closure of its rows), from the
 * first-visit frontier (as sst_length_bounds_frontier_device, with the
 * table's own rows; a 4 GB workspace kept in the ctx), or from the replay
 * of the memoised DFS (windows in the table's last packed word, tables
 * uploaded as they are, SST_LB_REPLAY).  out[i] = the bound; status[i]: 0
 * ok, SST_OUT_OF_TABLE (the reference raises NotImplementedError),
 * SST_LB_EMPTY_WINDOW (its min([]) raises ValueError), SST_ABORTED (DFS node
 * budget exhausted: no bound).  max_len <= 253 (the frontier's u8 values);
 * a window only the replay answers needs max_len <= 120 (SST_E_ARG with a
 * message otherwise).  Synchronous, host buffers. */
#define SST_LB_EMPTY_WINDOW (-5)
/* sst_length_bound_batch on per-query reduced alphabets (the table
 * adapt_individual_modification_rates_by_alphabet_reduction would rebuild,
 * mass_table.py:94-121, as select_sequence_length_with_jaccard / _with_lp
 * call it after reducing to the skeleton's nucleotides, skeleton_building.py:
 * 212-224, 324-336): query i on alphabet spec[i] (spec NULL: alphabet 0) of
 * n_alpha row masks alpha[2 g], alpha[2 g + 1] over the table's rows; the
 * exact replay with the mask, no table rebuilt.  A window reaching the reduced
 * table's extent is SST_OUT_OF_TABLE, one in its last packed word
 * SST_ABORTED (as sst_explain_alpha_batch_device).  direction must be 0
 * ("lower"; SST_E_ARG otherwise): the reference's upper bound counts a
 * visited child that returned the default as -1 + 1 = 0, and the masked walk
 * visits children the rebuilt table would not (reachable only with dropped
 * rows), so "upper" needs the rebuilt table.  Host buffers. */
int sst_length_bound_alpha_batch(sst_table* t, const double* su_mass, const double* obs_mass, const int32_t* spec,
                                 const uint64_t* alpha, int64_t n_alpha, int64_t n, double tolerance,
                                 double precision, int max_len, int64_t max_mods, int direction, int64_t* out,
                                 int8_t* status);
#define SST_LB_EXACT_ONLY 2 /* direction flag: skip the layered fast path (tests) */
#define SST_LB_REPLAY 4     /* direction flag: the replay instead of the first-visit frontier (tests) */
int sst_length_bound_batch(sst_table* t, const double* su_mass, const double* obs_mass, int64_t n, double tolerance,
                           double precision, int max_len, int64_t max_mods, int direction, int64_t* out,
                           int8_t* status);

/* ---- per-spectrum reduced alphabets ---------------------------------- */
/* Predictor.filter_by_explanation (prediction.py:170-227) reduces every
 * spectrum's alphabet to the modifications its explanations name
 * (adapt_individual_modification_rates_by_alphabet_reduction,
 * mass_table.py:94-121) and then queries the table rebuilt for that alphabet
 * (set_up_bit_table over the kept rows, max_mass = max(kept) * 35).  Over many
 * spectra these entry points answer those rebuilt tables' queries without
 * building them: spectrum g's alphabet is a row subset of t, the bits of
 * masks[2g] (rows 0..63) and masks[2g + 1] (rows 64..119); row 0 is implied;
 * the canonical rows are never dropped by the reference, so every alphabet
 * holds t's lightest row. */

/* explain_mass_with_table (mass_explanation.py:92-203) on pair-class windows
 * (hi < 3 * the lightest row mass: every candidate has <= 2 items) of query i
 * against the table of spectrum spec[i]'s alphabet: the candidates are t's
 * pair-list entries whose rows lie in the alphabet, in the reference's order.
 * The caller guarantees the budgets cannot bind (as for any pair-class window
 * with max_modifications >= 2 and per-row caps >= 2).  Out per query: status
 * (SST_NONE / SST_EMPTY / SST_SOME; -10 for a window that is not pair-class,
 * which the caller answers otherwise), the candidate count, the union of the
 * candidates' rows (rowmask[2i], rowmask[2i + 1]) and the window's pair-list
 * entry range range[2i] .. range[2i + 1] (its candidates are the entries of
 * that range whose rows are all in the alphabet; sst_table_pair_records).
 * t must carry the pair list.  No reference equivalent (batched). */
int sst_explain_pairs_alpha_device(sst_table* t, const double* d_mass, const double* d_thr, const int32_t* d_spec,
                                   const uint64_t* d_masks, int64_t n, double tolerance, double precision,
                                   int8_t* d_status, uint32_t* d_count, uint64_t* d_rowmask, uint32_t* d_range);
int sst_explain_pairs_alpha(sst_table* t, const double* mass, const double* thr, const int32_t* spec,
                            const uint64_t* masks, int64_t n_spec, int64_t n, double tolerance, double precision,
                            int8_t* status, uint32_t* count, uint64_t* rowmask, uint32_t* range);
/* is_valid_mass (mass_explanation.py:45-89) against the table of each
 * spectrum's alphabet (its last row: reachability by the alphabet's rows,
 * the reduced table's extent and last-column mask included): spectrum g's
 * queries are mass/thr[offsets[g] .. offsets[g+1]), in ascending mass order
 * (classify_fragments' SU order).  out as sst_is_valid_batch; -10 marks a
 * query the kernel could not answer (queries out of mass order). */
int sst_is_valid_alpha_device(sst_table* t, const double* d_mass, const double* d_thr, const int64_t* d_offsets,
                              int64_t n_spec, const uint64_t* d_masks, double tolerance, double precision,
                              int8_t* d_out);
int sst_is_valid_alpha(sst_table* t, const double* mass, const double* thr, const int64_t* offsets, int64_t n_spec,
                       const uint64_t* masks, double tolerance, double precision, int8_t* out);

/* ---- query producers (host code, no device) --------------------------- */
/* The sliding window of collect_explanations_per_side
 * (spectrseqtools/prediction.py:286-329) over many sides at once: side j is
 * su[offsets[j] .. offsets[j+1]) (SU masses sorted ascending); every (start,
 * end) pair whose difference the reference explains, in its order (including
 * its quirk: once `end` reaches the last fragment, later starts pair only with
 * it until a difference exceeds max_weight), as indices into su.  cap: room in
 * start_out / end_out; the return value is the number of pairs (> cap: nothing
 * beyond cap written, call again with more room) or a negative SST_E* code. */
int64_t sst_window_pairs(const double* su, const int64_t* offsets, int64_t n_sides, double max_weight,
                         int64_t* start_out, int64_t* end_out, int64_t cap);
/* The first filter_by_explanation round's queries over many spectra
 * (spectrseqtools/prediction.py:261-329, collect_diff_explanations_for_su):
 * spectrum g's rows su/obs[offsets[g] .. offsets[g+1]) (classify_fragments'
 * rows, ascending SU mass); flags per row: 1 START side, 2 END side, 4
 * singleton.  Per spectrum, in the reference's order: the START side's
 * sliding-window pairs, the END side's, then the singletons: diff = su[end] -
 * su[start] (a singleton: its su), thr = tolerance * (obs[start] + obs[end])
 * (a singleton: tolerance * obs), spec = g, kind = 0 / 1 / 2.  Returns the
 * number of queries (> cap: nothing written) or SST_E*.  Spectra are split
 * over up to 16 host threads. */
int64_t sst_su_diff_queries(const double* su, const double* obs, const uint8_t* flags, const int64_t* offsets,
                            int64_t n_spec, double max_weight, double tolerance, double* diff, double* thr,
                            int64_t* spec, int8_t* kind, int64_t cap);
/* ---- config 5 on the device ---------------------------------------------
 * classify_fragments and the filter_by_explanation fixpoint over many spectra
 * with every array in HBM.  Rows of spectrum g live in slots
 * 4 * d_peak_off[g] + i, i < d_rows[g] (d_rows_* arrays of 4 * n_peaks):
 * su, observed mass, meta = breakage | sides << 2 | is_singleton << 4 | peak
 * position << 8, alive.  Peaks in any order (ranked by mass on the device, equal
 * masses in their given order), <= 16383 per spectrum (above 4096 in the
 * reserved HBM slices); shifts / sides as sst_step_rows_device.  A spectrum of
 * more than 2048 rows is held in HBM slices the table's context reserves
 * (sst_pipe_reserve_rows, before the stages run); without them it is an
 * error.  d_err collects | 1 a spectrum over 16383 peaks (or over 4096 with
 * no slices reserved), 2 over 2048 rows with no slices reserved (or over
 * the reserved rows), 4 a window outside the pair class, 8 a window past a
 * table's end (the reference raises), 16 a dict too large for its hash, 32
 * rows out of mass order; the caller checks it. */
/* Reserve the context's slices for spectra of up to max_rows rows (<= 65532:
 * 4 breakages x 16383 peaks) in the row stages (classify above 4096 peaks, fix
 * rounds, final dict, bins);
 * a no-op for max_rows <= 2048 or at most what is reserved.  Synchronises the
 * context's stream when it grows. */
int sst_pipe_reserve_rows(sst_table* t, int64_t max_rows);
/* classify_fragments (fragment_classification.py:17-101): A7 into d_valid_out
 * (may be NULL), the filters, is_singleton against t's masses, SU order. */
int sst_classify_rows_device(sst_table* t, const double* d_obs, const int64_t* d_peak_off, int64_t n_spec,
                             int64_t n_peaks, const double* d_intensity, double intensity_cutoff, double mass_cutoff,
                             const double* d_su_seq, const double* shifts, const uint8_t* sides, int n_shifts,
                             double max_weight, double tolerance, double precision, int8_t* d_valid_out,
                             double* d_rows_su, double* d_rows_ob, uint32_t* d_rows_meta, uint8_t* d_alive,
                             uint32_t* d_rows, uint32_t* d_err);
/* Budget-binding ("exact mode") spectra of the device pipeline: a spectrum
 * whose max_modifications or modification caps are < 2 (a small
 * --modification_rate, or max_len <= 2: mass_explanation.py:158-172) can have
 * its budgets bind on pair-class windows, where the pair list's answers are
 * not the reference's.  With x->pair_ok[g] == 0 the stage lists the
 * spectrum's queries instead of answering them: x->xq_mass / xq_thr /
 * xq_spec / xq_single[...] in one block per spectrum (x->xq_block[g] = start
 * << 32 | count; *x->xq_count the list length, x->xq_cap its capacity, d_err
 * bit 64 on overflow); the caller answers the list with the exact masked
 * explain (sst_explain_alpha_batch_device, per max_len group) and
 * sst_result_refs_device into x->xa_st / xa_n / xa_ptr, then runs the stage's
 * second half (sst_fix_finish_device, sst_dict_build_device).  x may be NULL:
 * every spectrum's pair-class answers are exact. */
typedef struct sst_exact_io {
  const uint8_t* pair_ok;  /* [n_spec] */
  double* xq_mass;
  double* xq_thr;
  int32_t* xq_spec;
  uint8_t* xq_single;      /* 1: a singleton's query (stored in the dict even when empty) */
  uint32_t* xq_count;
  uint64_t xq_cap;
  uint64_t* xq_block;      /* [n_spec] */
  const int8_t* xa_st;
  const uint32_t* xa_n;
  const uint64_t* xa_ptr;
} sst_exact_io;

/* One filter_by_explanation round (prediction.py:170-202) of the spectra with
 * d_active[g]: their alive rows' window pairs and singletons explained
 * against d_alpha[2g..2g+1] (row masks of t; the caller keeps budgets from
 * binding, see sst_explain_pairs_alpha), the explanation dict's surviving
 * entries, d_alpha_next = the canonical rows | (alphabet & observed rows),
 * d_active_next[g] = the alphabet shrank (*d_n_active, zeroed by the call, counts those);
 * d_rounds[g] += 1, d_queries[g] += the round's explain queries.  Settled
 * spectra carry their alphabet over. */
int sst_fix_round_device(sst_table* t, const int64_t* d_peak_off, int64_t n_spec, const double* d_rows_su,
                         const double* d_rows_ob, const uint32_t* d_rows_meta, uint8_t* d_alive,
                         const uint32_t* d_rows, const uint64_t* d_alpha, uint64_t* d_alpha_next,
                         const uint8_t* d_active, uint8_t* d_active_next, uint32_t* d_rounds, uint32_t* d_queries,
                         uint32_t* d_n_active, double max_weight, double tolerance, double precision,
                         uint32_t* d_err, const sst_exact_io* x);
/* The exact-mode spectra's half of the round, after their listed queries
 * were answered (same arrays as the round; x required). */
int sst_fix_finish_device(sst_table* t, int64_t n_spec, const uint32_t* d_rows, const uint64_t* d_alpha,
                          uint64_t* d_alpha_next,
                          const uint8_t* d_active, uint8_t* d_active_next, uint32_t* d_rounds, uint32_t* d_queries,
                          uint32_t* d_n_active, uint32_t* d_err, const sst_exact_io* x);
/* SkeletonBuilder._predict_skeleton's speculative bin queries
 * (skeleton_building.py:114-160; replaces the per-bin explain calls of
 * :131-160 for every spectrum at once) over the rows a fixpoint kept
 * (d_alive), on each spectrum's alphabet d_alpha: per side, bins are runs of
 * rows whose SU step is <= tol * (obs_prev + obs); the side's first bin
 * explains its rows' SU masses against 0 (threshold tol * obs), every later
 * bin each (predecessor row, row) difference (tol * (obs_p + obs_r)); a
 * side's last bin only with >= 2 rows.  Two calls: count (d_n_q[S] queries
 * per spectrum, d_q_off[S + 1] their exclusive offsets, the total last), then
 * emit into d_status / d_count [total], spectrum-major (START side, then END;
 * bins in order; a bin's pairs predecessor-row-major).  Statuses SST_NONE /
 * EMPTY / SOME, or -10 for a window outside the pair class (hi >= 3 w_min:
 * the caller's general path).  With d_n_def non-null (zeroed by the caller),
 * those windows are also listed, in any order, for
 * sst_explain_alpha_batch_device: d_def_mass / d_def_thr / d_def_spec /
 * d_def_q[*d_n_def] = window mass, threshold, spectrum and index into
 * d_status (capacity: the total).  d_err bit 2: a spectrum over 2048 rows
 * with no slices reserved (sst_pipe_reserve_rows). */
int sst_bins_count_device(sst_table* t, const int64_t* d_peak_off, int64_t n_spec, const double* d_rows_su,
                          const double* d_rows_ob, const uint32_t* d_rows_meta, const uint8_t* d_alive,
                          const uint32_t* d_rows, double tol, uint32_t* d_n_q, uint64_t* d_q_off, uint32_t* d_err,
                          uint32_t* d_n_q0 /* may be NULL: the START side's count per spectrum */);
int sst_bins_emit_device(sst_table* t, const int64_t* d_peak_off, int64_t n_spec, const double* d_rows_su,
                         const double* d_rows_ob, const uint32_t* d_rows_meta, const uint8_t* d_alive,
                         const uint32_t* d_rows, const uint64_t* d_alpha, double tol, double prec,
                         const uint64_t* d_q_off, int8_t* d_status, uint32_t* d_count, double* d_def_mass,
                         double* d_def_thr, int32_t* d_def_spec, uint64_t* d_def_q, uint32_t* d_n_def,
                         uint32_t* d_err, const uint8_t* d_pair_ok /* may be NULL; 0: list every window */);

/* _reduce_alphabet's filter (prediction.py:211-227): is_valid_mass of the
 * alive rows of the d_active spectra against their reduced tables (d_alpha),
 * AND-ed into d_alive.  A spectrum whose alphabet did not change needs no
 * re-filter (its rows already passed that table), so a fixpoint passes the
 * round's changed flags (sst_fix_round_device's d_active_next). */
int sst_valid_rows_alpha_device(sst_table* t, const int64_t* d_peak_off, int64_t n_spec, const double* d_rows_su,
                                const double* d_rows_ob, const uint32_t* d_rows, const uint64_t* d_alpha,
                                const uint8_t* d_active, uint8_t* d_alive, double tolerance, double precision,
                                uint32_t* d_err);

/* The explanation dict collect_diff_explanations_for_su builds per spectrum
 * (prediction.py:261-284): spectrum g's queries [offsets[g], offsets[g+1])
 * in its order (START pairs, END pairs, singletons) with kind 0 / 1 / 2, their
 * dict key (the difference, or the singleton's SU mass), explain status and
 * candidate row union (2 x u64).  Side pairs are stored only with >= 1
 * explanation, singletons always; a later store of an equal key replaces the
 * earlier one.  keep[i] = 1 for the queries whose answers the finished dict
 * holds; union_out[2g..2g+1] = the rows of those answers (the observed
 * nucleotides of filter_by_explanation, :189-195).  Returns the number of
 * dict entries over all spectra, or SST_E*.  Host code, up to 16 threads. */
int64_t sst_dict_union(const int64_t* offsets, int64_t n_spec, const double* key, const int8_t* kind,
                       const int8_t* status, const uint64_t* rowmask, uint8_t* keep, uint64_t* union_out);
/* order[0..n): the row permutation that sorts by group (0 <= group < n_groups)
 * then key ascending, ties in row order -- classify_fragments' per-spectrum
 * sort by standard_unit_mass (fragment_classification.py:84), for many
 * spectra (numpy.lexsort((rows, key, group))). */
int sst_sort_rows(const int64_t* group, const double* key, int64_t n, int64_t n_groups, int64_t* order);

/* ---- config 5: SkeletonBuilder._predict_skeleton's walk --------------- */
/* One lane per (spectrum, side) walks the side's rows the fixpoint kept
 * (skeleton_building.py:114-196): bins, each closed bin explained against the
 * last bin with explanations (explain_bin_differences :372-421, the first
 * against 0) after filter_by_explanation's final dict (:423-440),
 * update_skeleton_for_given_explanations (:442-482) with CPython's set order
 * (sst_pyset_order; name hashes from the caller's interpreter), min_end /
 * max_end per bin.  Pair-class windows are answered in the lane; the others
 * come from the masked explain: stage 3's speculative queries (s_*), and
 * re-queries (a bin explained against an older bin) listed by the lane when
 * their answers are missing -- the side is then SST_WALK_SUSPENDED, and the
 * caller answers req_* (sst_explain_alpha_batch_device), adds them as round
 * n_rounds (rq_*: per side its block start << 32 | count in the round's
 * lists) and walks the suspended sides again: with resume set and the same
 * scratch slots, each resumes at the bin that suspended it (its loop state
 * is kept at the head of its slot), otherwise it replays from the start.
 * SST_WALK_BIG: a bin outgrew the lane's scratch capacities (walk that side
 * again with larger ones).  All pointers are device pointers. */
#define SST_WALK_MAX_ROUNDS 16
#define SST_WALK_DONE 0
#define SST_WALK_SUSPENDED 1
#define SST_WALK_BIG 2
#define SST_WALK_RAISE 3   /* an answer raised in the reference (window past the reduced table) */
#define SST_WALK_LIMIT 4   /* an engine limit: rows, positions, request list, OVERFLOW / ABORTED answer */
#define SST_WALK_ROUNDS 5  /* more than SST_WALK_MAX_ROUNDS re-query rounds */
#define SST_WALK_MISSING 6 /* a DFS answer was not supplied */
typedef struct sst_walk_args {
  const int64_t* peak_off;   /* [n_spec + 1]: rows of spectrum g at slots 4 peak_off[g] + i (SU order) */
  const uint32_t* cnt;       /* [n_spec] rows */
  const double* r_su;
  const double* r_ob;
  const uint32_t* r_meta;    /* breakage | sides << 2 | singleton << 4 | peak << 8 */
  const uint8_t* alive;      /* the rows the fixpoint kept */
  const uint64_t* alpha;     /* [2 n_spec] the fixpoint's alphabets (row masks) */
  const int32_t* max_len;    /* [n_spec] SequenceInformation.max_len */
  const uint8_t* pair_ok;    /* [n_spec] budgets cannot bind on pair-class windows */
  int64_t n_spec;
  int64_t slots;             /* 4 * peaks */
  double tol, prec, rprec;
  const uint64_t* d_off;     /* the final dict (sst_dict_build_device) */
  const uint32_t* d_n;
  const uint64_t* d_key;
  const double* d_thr;
  const uint64_t* q_off;     /* stage 3 (sst_bins_count_device): per spectrum its queries' offset */
  const uint32_t* q0;        /* and its START side's count */
  const uint64_t* s_ptr;     /* per stage-3 query off the pair class: first payload record (sst_result_refs_device) */
  const uint32_t* s_n;
  const int8_t* s_st;
  int n_rounds;
  const uint64_t* rq_block[SST_WALK_MAX_ROUNDS];
  const uint64_t* rq_ptr[SST_WALK_MAX_ROUNDS];
  const uint32_t* rq_n[SST_WALK_MAX_ROUNDS];
  const int8_t* rq_st[SST_WALK_MAX_ROUNDS];
  uint64_t* req_block;       /* [2 n_spec] this round's blocks (zeroed by the caller) */
  double* req_mass;
  double* req_thr;
  int32_t* req_spec;
  uint32_t* req_count;
  uint64_t req_cap;
  const int64_t* name_hash;  /* [n_rows] hash() of each row's nucleoside name */
  const uint32_t* sides;     /* side ids 2 g + (0 START, 1 END) to walk */
  uint32_t n_sides;
  uint8_t* scratch;          /* scratch_stride bytes per slot (sst_walk_scratch_bytes) */
  uint64_t scratch_stride;
  uint32_t pos_cap, len_cap, expl_cap, cand_cap, tset_cap;  /* len_cap = max max_len + 2 <= 255 */
  uint16_t* side_rows;       /* [2 slots] */
  const uint64_t* skel_off;  /* [n_spec] exclusive prefix of 2 max_len */
  uint64_t* skel;            /* spectrum g, side sd, position i: masks at 2 (skel_off[g] + sd max_len[g] + i) */
  int32_t* min_end;          /* [2 slots] per side */
  int32_t* max_end;
  uint8_t* kept;             /* [2 slots] per side: not rejected by the walk */
  uint8_t* side_status;      /* [2 n_spec] SST_WALK_* */
  uint32_t* n_suspended;
  uint32_t* n_big;
  const uint32_t* slot;      /* [n_sides] each walked side's scratch slot (NULL: its index in sides) */
  int resume;                /* a side whose slot holds its suspended state resumes there (else it
                                walks from the start; slots of a first launch hold no state) */
} sst_walk_args;
/* Scratch bytes per walked side for the given capacities (pos_cap, tset_cap:
 * powers of two >= the set tables the positions / a query's candidates need,
 * sst_pyset_table_size). */
uint64_t sst_walk_scratch_bytes(uint32_t pos_cap, uint32_t len_cap, uint32_t expl_cap, uint32_t cand_cap,
                                uint32_t tset_cap);

/* The walk's re-query answers merged over rounds (skeleton_device's round
 * loop; skeleton_building.py:114-196 issues them one explain call at a time,
 * the device walk suspends and resumes, so a side's k-th re-query answer must
 * be entry k of its merged list).  Per side sid of n_sides: the earlier
 * rounds' merged entries (o_block[sid] = start << 32 | count into o_ptr /
 * o_n / o_st; o_block NULL for the first round), then this round's
 * (block[sid] likewise into ptr / n / st) -> m_block[sid] = start << 32 |
 * count into m_ptr / m_n / m_st, sides in order.  m_* must hold the earlier
 * rounds' total plus this round's entries; tot (u32[n_sides]) and off
 * (u64[n_sides + 1]) are device scratch.  Device pointers, the ctx's stream. */
typedef struct sst_requery_merge_args {
  const int64_t* o_block;
  const uint64_t* o_ptr;
  const uint32_t* o_n;
  const int8_t* o_st;
  const int64_t* block;
  const uint64_t* ptr;
  const uint32_t* n;
  const int8_t* st;
  int64_t n_sides;
  int64_t* m_block;
  uint64_t* m_ptr;
  uint32_t* m_n;
  int8_t* m_st;
} sst_requery_merge_args;
int sst_requery_merge_device(sst_table* t, const sst_requery_merge_args* args, uint32_t* d_tot, uint64_t* d_off);
/* CPython's table size after n distinct additions to an empty set. */
uint32_t sst_pyset_table_size(uint32_t n);
int sst_skel_walk_device(sst_table* t, const sst_walk_args* a);
/* Candidate references of a result's queries (settles it first): for query
 * i, d_st[d_dst[i]] = its status, d_n[...] = its candidates (SOME) or exact
 * count (OVERFLOW / ABORTED), d_ptr[...] = the device address of its first
 * payload record (SOME; else 0).  Valid while the result lives unchanged. */
int sst_result_refs_device(sst_result* r, const int64_t* d_dst, uint64_t* d_ptr, uint32_t* d_n, int8_t* d_st);
/* filter_by_explanation's final explanation dict per spectrum
 * (prediction.py:261-329 over the final rows and alphabet).  Count pass:
 * d_n_q[g] = the last round's queries, d_off = their exclusive offsets
 * (n_spec + 1 entries, total last); build pass: keys ascending (double bits)
 * and the last writer's threshold into [d_off[g], + d_n_ent[g]). */
int sst_dict_count_device(sst_table* t, const int64_t* d_peak_off, int64_t n_spec, const double* d_rows_su,
                          const double* d_rows_ob, const uint32_t* d_rows_meta, const uint8_t* d_alive,
                          const uint32_t* d_rows, double max_weight, double tol, uint32_t* d_n_q, uint64_t* d_off,
                          uint32_t* d_err);
int sst_dict_build_device(sst_table* t, const int64_t* d_peak_off, int64_t n_spec, const double* d_rows_su,
                          const double* d_rows_ob, const uint32_t* d_rows_meta, const uint8_t* d_alive,
                          const uint32_t* d_rows, const uint64_t* d_alpha, double max_weight, double tol, double prec,
                          const uint64_t* d_off, uint64_t* d_key, double* d_thr, uint32_t* d_n_ent, uint32_t* d_err,
                          const sst_exact_io* x);
/* The exact-mode spectra's final-round queries listed for the masked
 * explain (before sst_dict_build_device, which then reads x->xa_*). */
int sst_dict_list_device(sst_table* t, const int64_t* d_peak_off, int64_t n_spec, const double* d_rows_su,
                         const double* d_rows_ob, const uint32_t* d_rows_meta, const uint8_t* d_alive,
                         const uint32_t* d_rows, double max_weight, double tol, uint32_t* d_err, const sst_exact_io* x);

/* select_sequence_length_with_jaccard (skeleton_building.py:315-370) and
 * combine_skeleton_sequences (:494-516) per spectrum, one lane each: the
 * START skeleton and the reversed END skeleton (sst_walk_args.skel layout),
 * the two length bounds on the skeleton alphabet (sst_length_bounds_reach_
 * device) and that alphabet's row masses; validate_sequence_length_by_mass
 * (:291-313) in the reference's float order (sequential f64 sums, CPython
 * 3.10's sum()).  Outputs: seq_len[g], the combined skeleton (masks at
 * 2 (comb_off[g] + i), i < seq_len[g]; comb_off[g] + max_len[g] positions
 * reserved) and status[g]: SST_JAC_OK, SST_JAC_NO_LENGTH (the reference's
 * "No sequence length fitting ..." Exception), SST_JAC_INDEX (an IndexError
 * in combine_skeleton_sequences: seq_len > max_len), SST_JAC_BOUNDS (a
 * length bound raised: status_lb[g] != 0). */
#define SST_JAC_OK 0
#define SST_JAC_NO_LENGTH 1
#define SST_JAC_INDEX 2
#define SST_JAC_BOUNDS 3
typedef struct sst_jaccard_args {
  int64_t n_spec;
  const int32_t* max_len;     /* [n_spec] */
  const uint64_t* skel_off;   /* [n_spec] as sst_walk_args.skel_off */
  const uint64_t* skel;
  const int64_t* lower;       /* [n_spec] the length bounds */
  const int64_t* upper;
  const int8_t* status_lb;
  const double* su_mass;      /* [n_spec] SequenceInformation.su_mass */
  const double* row_mass;     /* [n_rows] integer mass * precision (nucleoside_masses) */
  const uint64_t* comb_off;   /* [n_spec] exclusive prefix of max_len */
  uint64_t* comb;             /* combined skeleton masks */
  int32_t* seq_len;
  int8_t* status;
  double max_variance;        /* fragment_classification.MAX_VARIANCE */
} sst_jaccard_args;
int sst_jaccard_device(sst_table* t, const sst_jaccard_args* a);
/* The skeleton's alphabet per spectrum (skeleton_building.py:319-326):
 * d_out[2g..2g+1] = d_alpha[2g..] & (the table's canonical rows | every row
 * either side's skeleton names at any of its max_len positions). */
int sst_skeleton_alpha_device(sst_table* t, int64_t n_spec, const int32_t* d_max_len, const uint64_t* d_skel_off,
                              const uint64_t* d_skel, const uint64_t* d_alpha, uint64_t* d_out);

/* After the skeleton (Predictor.predict, prediction.py:88-103), for the
 * spectra whose Jaccard length stands (status SST_JAC_OK; the others get
 * active 0 and no rows: predict returns Prediction.default()):
 * build_skeleton's fragments (skeleton_building.py:67-109) -- rows the START
 * walk kept (min_end - 1, max_end - 1), rows the END walk kept that START did
 * not (len - min_end, len - max_end), the alive internal rows whose peak no kept
 * terminal row shares (0, -1), every end index outside [0, len) clamped to
 * len - 1 -- in alive_out / min_end_out / max_end_out per row slot, and the
 * alphabet _reduce_alphabet sets (:99-103): alpha (the Jaccard stage's, as
 * sst_skeleton_alpha_device gives it) without the modifications the combined
 * skeleton's positions 0 .. seq_len - 1 do not name.  The caller applies the
 * reduction's is_valid filter with sst_valid_rows_alpha_device(alpha_out,
 * active, alive_out).  kept / min_end / max_end are sst_walk_args' [2][slots]
 * arrays (side-major).  err bit 0: a spectrum of more than 4096 peaks. */
typedef struct sst_post_args {
  int64_t n_spec;
  const int64_t* peak_off;   /* [n_spec + 1] */
  const uint32_t* rows;      /* [n_spec] */
  const uint32_t* meta;      /* row slots, as sst_classify_rows_device writes them */
  const uint8_t* alive;      /* the fixpoint's survivors */
  const uint8_t* kept;       /* [2][slots] */
  const int32_t* min_end;    /* [2][slots] */
  const int32_t* max_end;
  int64_t slots;
  const int32_t* seq_len;    /* [n_spec] sst_jaccard_device's */
  const int8_t* jac_status;  /* [n_spec] */
  const uint64_t* comb_off;  /* [n_spec] */
  const uint64_t* comb;
  const uint64_t* alpha;     /* [2 n_spec] the Jaccard stage's alphabets */
  uint64_t* alpha_out;       /* [2 n_spec] */
  uint8_t* active;           /* [n_spec] */
  uint8_t* alive_out;        /* row slots */
  int32_t* min_end_out;
  int32_t* max_end_out;
  uint32_t* err;
} sst_post_args;
int sst_post_skeleton_device(sst_table* t, const sst_post_args* a);

/* compute_sequence_length_bound (mass_table.py:343-487) after the skeleton's
 * alphabet reduction (skeleton_building.py:315-336), both directions, for
 * queries on per-spectrum reduced alphabets, exact without a table rebuild:
 * sst_reach_rows_device writes, per spectrum g, the reachability bitset of
 * each kept row k (row 0 excluded, ascending): bit m of u32 word
 * d_bits[d_off[g] + k * d_words[g] + m / 32] <=> m is a sum of kept rows up
 * to that one (the rebuilt table's pair(r_k, m) != 0), for m < 32 d_words[g]
 * (>= the highest window value + 1).  sst_length_bounds_reach_device then
 * replays the reference's memoised DFS once per query (spectrum d_spec[i])
 * on those pairs and derives both bounds from it: d_lower[i] / d_upper[i],
 * d_status[i] 0 ok, SST_OUT_OF_TABLE (the reference raises), SST_ABORTED (a
 * window in the reduced table's masked last word, or a guard), -5 an empty
 * window.  Budgets: max_len, max_mods and the table's caps
 * (sst_table_set_budgets) as in sst_length_bound_batch -- or, with d_qlen
 * non-NULL, per query: max_len d_qlen[i], caps d_caps_len[d_qlen[i] *
 * SST_MAX_ROWS + r] and max_mods d_a0_len[d_qlen[i]] (the caller's
 * round(L * rate)), so spectra of every max_len share one launch (the
 * table's is_modification flags still come from sst_table_set_budgets).
 * d_nodes (may be NULL; zeroed by the caller): per query, the replay's
 * visited nodes summed over its attempts.  soft_nodes > 0: a query whose
 * replay passes that many nodes stops with status SST_LB_HEAVY (the caller
 * replays such queries together later, with soft_nodes 0), so that a few
 * heavy spectra do not hold up a batch.  memo_first: the first attempt's
 * memo masses per query (0: 2^16; a power of two).  fuse: both bounds'
 * values computed inside the replay, in dense per-mass slots (allowed when
 * every alphabet has <= 64 kept rows; 0: the separate value passes).
 * Device pointers. */
#define SST_MAX_ROWS 120
#define SST_LB_HEAVY (-7)
int sst_reach_rows_device(sst_table* t, const uint64_t* d_alpha, const int64_t* d_words, const uint64_t* d_off,
                          int64_t n_spec, uint32_t* d_bits);
int sst_length_bounds_reach_device(sst_table* t, const double* d_su, const double* d_obs, const int32_t* d_spec,
                                   const uint64_t* d_alpha, const uint32_t* d_reach_bits, const uint64_t* d_reach_off,
                                   const int64_t* d_reach_words, int64_t n, double tol, double prec, int max_len,
                                   int64_t max_mods, int64_t* d_lower, int64_t* d_upper, int8_t* d_status,
                                   const int32_t* d_qlen, const int32_t* d_caps_len, const int32_t* d_a0_len,
                                   uint64_t* d_nodes, int64_t soft_nodes, uint32_t memo_first, int fuse);

/* The same bounds WITHOUT replaying the DFS (sst_frontier.hip, DESIGN §3
 * "first-visit frontier"): the reference's memo is keyed by (mass, row) and
 * ignores the budgets, so each node's memoised value is fixed by its first
 * visit; which visit comes first is the lexicographic minimum over the node's
 * up and left parents (mass_table.py:373-457: up before left, window values
 * ascending), computed in bands of the lightest row mass over descending
 * masses, then the values by a DP over ascending masses.  Same result as the
 * replay for every query, in time linear in the memo's size and independent of
 * any one spectrum's depth.
 * sst_reach_lowest_device first turns sst_reach_rows_device's bitsets into one
 * byte per mass: d_lr[d_lr_off[g] + m] = the lowest kept rank k with m in
 * R_k (0xFF: none), m < 32 d_words[g] (d_lr_off[g] a multiple of 32).
 * sst_length_bounds_frontier_device: arguments as sst_length_bounds_reach_device
 * (d_lr / d_lr_off instead of the bitsets); d_nodes (may be NULL; zeroed by the
 * caller) = per query, the memo entries (distinct (mass, row) nodes) its DFS
 * creates.  workspace_bytes: the device workspace (0: half the free memory, at
 * most 48 GB); queries are processed in chunks sized from the memo entries
 * per query seen so far (a chunk that overflows is split; a single query
 * beyond the workspace gets SST_ABORTED).
 * stats may be NULL. */
typedef struct sst_lbf_stats {
  int64_t live;            /* queries the list pass handed to the frontier */
  int64_t nodes;           /* memo entries created */
  int64_t chunks;          /* chunks run to completion */
  int64_t splits;          /* chunks that overflowed the workspace and were split */
  int64_t aborted;         /* single queries beyond the workspace (SST_ABORTED) */
  int64_t bands;           /* mass bands of the largest chunk */
  int64_t key_words;       /* 64-bit words per first-visit key (1, 2 or 4) */
  int64_t max_band_groups; /* (query, mass) groups of the fullest band */
  int64_t max_band_nodes;  /* memo entries of the fullest band */
  int64_t table_slots;     /* slots per hash table of the ring */
  int64_t node_cap;        /* node capacity per chunk */
  int64_t overflow_bits;   /* why chunks were split: 1 nodes / a band's records, 2 a hash table, 4 a band list */
  int64_t groups;          /* (query, mass) groups of the completed chunks (the memo's distinct masses) */
  int64_t edges;           /* left moves onto a mass > 0 of the completed chunks (candidate inserts) */
} sst_lbf_stats;
int sst_reach_lowest_device(sst_table* t, const uint64_t* d_alpha, const int64_t* d_words, const uint64_t* d_off,
                            int64_t n_spec, const uint32_t* d_bits, const uint64_t* d_lr_off, uint8_t* d_lr);
int sst_length_bounds_frontier_device(sst_table* t, const double* d_su, const double* d_obs, const int32_t* d_spec,
                                      const uint64_t* d_alpha, const uint8_t* d_lr, const uint64_t* d_lr_off, int64_t n,
                                      double tol, double prec, int max_len, int64_t max_mods, int64_t* d_lower,
                                      int64_t* d_upper, int8_t* d_status, const int32_t* d_qlen,
                                      const int32_t* d_caps_len, const int32_t* d_a0_len, uint64_t* d_nodes,
                                      uint64_t workspace_bytes, sst_lbf_stats* stats);

/* ---- CPython set order (the skeleton walk's emulation, sst_pyset.h) ---- */
/* hash(tuple) of a tuple whose items hash to item_hashes[0..n) (CPython
 * 3.8+ tuplehash, 64-bit): the hash of an explanation's name tuple
 * (mass_explanation.py:302-318) from the names' str hashes. */
int64_t sst_py_tuple_hash(const int64_t* item_hashes, int64_t n);
/* The iteration order of a set built by adding elements keys[0..n) (distinct
 * keys = distinct elements, hashes[i] = hash(element i)) in that order to an
 * empty set (CPython 3.7-3.12 setobject.c): order[0..m) receives the keys in
 * iteration order; returns m (the distinct elements) or SST_E*.  Host code:
 * it exists so that tests can pin the walk's emulation to the interpreter. */
int64_t sst_pyset_order(const int32_t* keys, const int64_t* hashes, int64_t n, int32_t* order);

/* ---- measurement ------------------------------------------------------ */
/* Kernel ids for sst_profile_read. */
#define SST_K_IS_VALID 0
#define SST_K_EXPLAIN_MAIN 1
#define SST_K_EXPLAIN_DEFERRED 2 /* deep, no-memo and exact roles share one launch */
#define SST_K_EXPLAIN_DEEP SST_K_EXPLAIN_DEFERRED
#define SST_K_EXPLAIN_NOMEMO 3 /* reserved (merged into SST_K_EXPLAIN_DEFERRED) */
#define SST_K_EXPLAIN_EXACT 4  /* reserved (merged into SST_K_EXPLAIN_DEFERRED) */
#define SST_K_EXPLAIN_EXPAND 5
#define SST_K_RESULT_PACK 6 /* k_result_pack: dense hit list + payload of a pass */
/* config 5 (the device-resident pipeline stages) */
#define SST_K_CLASSIFY_ROWS 7 /* k_classify_rows (sst_classify_rows_device) */
#define SST_K_FIX_ROUND 8     /* k_fix_round (sst_fix_round_device) */
#define SST_K_VALID_ALPHA 9   /* k_valid_alpha (sst_valid_rows_alpha_device, sst_is_valid_alpha*) */
#define SST_K_BINS_COUNT 10   /* k_bins_count + k_scan_u32 (sst_bins_count_device) */
#define SST_K_BINS_EMIT 11    /* k_bins_emit (sst_bins_emit_device) */
#define SST_K_DICT 12         /* k_dict_count / k_dict_build (sst_dict_final_device) */
#define SST_K_SKEL_WALK 13    /* k_skel_walk (sst_skeleton_walk_device) */
#define SST_K_REACH_ROWS 14   /* k_reach_rows (sst_reach_rows_device) */
#define SST_K_LENGTH_BOUND 15 /* k_length_fast / k_length_exact (length-bound batches) */
#define SST_K_JACCARD 16      /* k_jaccard (sst_jaccard_device) */
#define SST_K_PAIRS_ALPHA 17  /* k_pairs_alpha (sst_explain_pairs_alpha*) */
#define SST_K_REQUERY_MERGE 18 /* k_requery_count + k_scan_u32 + k_requery_copy (sst_requery_merge_device) */
#define SST_K_COUNT 24
/* When enabled, every kernel launch of this ctx is bracketed by hipEvents
 * recorded on the ctx stream; sst_profile_read synchronises and returns the
 * summed milliseconds and launch counts per kernel id since the last read
 * (or enable), then resets them. */
int sst_profile_enable(sst_ctx* ctx, int on);
/* Same, restricted to the kernel ids set in kernel_mask (bit k = id k): each
 * bracketed launch costs two event records on the stream, so a benchmark
 * brackets only the kernels it reports. */
int sst_profile_select(sst_ctx* ctx, uint32_t kernel_mask);
/* Bracket only every `every`-th launch of each selected kernel (default 1):
 * the events' own cost on the stream is then spread over `every` launches
 * while the durations are still sampled from the live launch stream. */
int sst_profile_sample(sst_ctx* ctx, uint32_t every);
int sst_profile_read(sst_ctx* ctx, double* ms_total /* [SST_K_COUNT] */, int64_t* launches /* [SST_K_COUNT] */);

#ifdef __cplusplus
}
#endif
#endif /* SST_H */
