"""ctypes binding of libsstgpu.so (the C ABI in include/sst.h).

This is the only way the Python mirror reaches the engine.  There is no CPU
fallback: if the library is missing or no HIP device is visible, every entry
point raises.  ctypes releases the GIL for the duration of each call.
"""
import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SST_LIBRARY", os.path.join(_HERE, "libsstgpu.so"))

# status codes (include/sst.h)
SST_NONE, SST_EMPTY, SST_SOME = 0, 1, 2
SST_OUT_OF_TABLE, SST_OVERFLOW, SST_ABORTED = -1, -2, -4
SST_LB_EMPTY_WINDOW = -5

# every function include/sst.h declares (checked by tests/test_boundary.py)
EXPORTS = (
    "sst_device_count", "sst_ctx_create", "sst_ctx_destroy", "sst_last_error", "sst_ctx_stream",
    "sst_ctx_synchronize", "sst_table_build", "sst_table_upload", "sst_table_set_budgets", "sst_table_shape",
    "sst_table_download", "sst_table_destroy", "sst_is_valid_batch", "sst_is_valid_batch_device",
    "sst_explain_batch", "sst_explain_batch_device", "sst_explain_alpha_batch_device", "sst_explain_alpha_lens_batch_device", "sst_result_host", "sst_result_device", "sst_result_fetch",
    "sst_result_free", "sst_result_stats", "sst_profile_enable", "sst_profile_select",
    "sst_profile_sample", "sst_profile_read", "sst_length_bound_batch", "sst_explain_recursion_batch", "sst_is_singleton_batch",
    "sst_is_singleton_batch_device", "sst_ctx_set_stream", "sst_result_hit_list", "sst_result_settle",
    "sst_window_pairs", "sst_is_valid_peaks", "sst_is_valid_peaks_device", "sst_result_pair_hits",
    "sst_table_pair_records", "sst_su_diff_queries", "sst_sort_rows", "sst_step_device",
    "sst_wire_pack", "sst_explain_pairs_alpha", "sst_explain_pairs_alpha_device", "sst_is_valid_alpha",
    "sst_is_valid_alpha_device", "sst_dict_union", "sst_step_rows_device", "sst_result_queries",
    "sst_classify_rows_device", "sst_fix_round_device", "sst_valid_rows_alpha_device",
    "sst_bins_count_device", "sst_bins_emit_device", "sst_length_bound_alpha_batch",
    "sst_py_tuple_hash", "sst_pyset_order", "sst_pyset_table_size", "sst_walk_scratch_bytes",
    "sst_skel_walk_device", "sst_result_refs_device", "sst_dict_count_device", "sst_dict_build_device",
    "sst_reach_rows_device", "sst_length_bounds_reach_device", "sst_jaccard_device", "sst_skeleton_alpha_device",
    "sst_dict_list_device", "sst_fix_finish_device", "sst_pipe_reserve_rows", "sst_reach_lowest_device",
    "sst_length_bounds_frontier_device", "sst_post_skeleton_device", "sst_ctx_trim", "sst_requery_merge_device",
)

# kernel ids of sst_profile_read
K_IS_VALID, K_EXPLAIN_SCAN, K_EXPLAIN_DEEP, K_EXPLAIN_NOMEMO, K_EXPLAIN_EXACT, K_EXPLAIN_EXPAND = 0, 1, 2, 3, 4, 5
K_RESULT_PACK = 6
(K_CLASSIFY_ROWS, K_FIX_ROUND, K_VALID_ALPHA, K_BINS_COUNT, K_BINS_EMIT, K_DICT, K_SKEL_WALK, K_REACH_ROWS,
 K_LENGTH_BOUND, K_JACCARD, K_PAIRS_ALPHA, K_REQUERY_MERGE) = range(7, 19)
K_COUNT = 24  # SST_K_COUNT
KERNEL_NAMES = {K_IS_VALID: "k_is_valid", K_EXPLAIN_SCAN: "k_explain_scan", K_EXPLAIN_DEEP: "k_explain_deferred",
                K_EXPLAIN_EXPAND: "k_explain_expand",
                K_RESULT_PACK: "k_result_pack",  # ids 3, 4: reserved (merged into the deferred launch)
                K_CLASSIFY_ROWS: "k_classify_rows", K_FIX_ROUND: "k_fix_round", K_VALID_ALPHA: "k_valid_alpha",
                K_BINS_COUNT: "k_bins_count", K_BINS_EMIT: "k_bins_emit", K_DICT: "k_dict_build",
                K_SKEL_WALK: "k_skel_walk", K_REACH_ROWS: "k_reach_rows", K_LENGTH_BOUND: "k_length_bound",
                K_JACCARD: "k_jaccard", K_PAIRS_ALPHA: "k_pairs_alpha", K_REQUERY_MERGE: "k_requery_merge"}

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_U64 = ctypes.c_uint64
_I = ctypes.c_int
_D = ctypes.c_double
_PP = ctypes.POINTER(ctypes.c_void_p)


class EngineError(RuntimeError):
    pass


WALK_MAX_ROUNDS = 16  # SST_WALK_MAX_ROUNDS
MAX_ROWS = 120  # SST_MAX_ROWS (row stride of per-length cap tables)
LB_HEAVY = -7  # SST_LB_HEAVY
(WALK_DONE, WALK_SUSPENDED, WALK_BIG, WALK_RAISE, WALK_LIMIT, WALK_ROUNDS, WALK_MISSING) = range(7)


JAC_OK, JAC_NO_LENGTH, JAC_INDEX, JAC_BOUNDS = range(4)


class ExactIO(ctypes.Structure):
    """sst_exact_io (include/sst.h): budget-binding spectra's query lists."""
    _fields_ = [("pair_ok", ctypes.c_void_p), ("xq_mass", ctypes.c_void_p), ("xq_thr", ctypes.c_void_p),
                ("xq_spec", ctypes.c_void_p), ("xq_single", ctypes.c_void_p), ("xq_count", ctypes.c_void_p),
                ("xq_cap", ctypes.c_uint64), ("xq_block", ctypes.c_void_p), ("xa_st", ctypes.c_void_p),
                ("xa_n", ctypes.c_void_p), ("xa_ptr", ctypes.c_void_p)]


class PostArgs(ctypes.Structure):
    """sst_post_args (include/sst.h): build_skeleton's fragments and the skeleton-based reduction."""
    _fields_ = [("n_spec", ctypes.c_int64), ("peak_off", ctypes.c_void_p), ("rows", ctypes.c_void_p),
                ("meta", ctypes.c_void_p), ("alive", ctypes.c_void_p), ("kept", ctypes.c_void_p),
                ("min_end", ctypes.c_void_p), ("max_end", ctypes.c_void_p), ("slots", ctypes.c_int64),
                ("seq_len", ctypes.c_void_p), ("jac_status", ctypes.c_void_p), ("comb_off", ctypes.c_void_p),
                ("comb", ctypes.c_void_p), ("alpha", ctypes.c_void_p), ("alpha_out", ctypes.c_void_p),
                ("active", ctypes.c_void_p), ("alive_out", ctypes.c_void_p), ("min_end_out", ctypes.c_void_p),
                ("max_end_out", ctypes.c_void_p), ("err", ctypes.c_void_p)]


class RequeryMergeArgs(ctypes.Structure):
    """sst_requery_merge_args (include/sst.h): the walk's re-query answers merged over rounds."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("o_block", "o_ptr", "o_n", "o_st", "block", "ptr", "n", "st")] + \
        [("n_sides", ctypes.c_int64)] + [(n, ctypes.c_void_p) for n in ("m_block", "m_ptr", "m_n", "m_st")]


class LbfStats(ctypes.Structure):
    """sst_lbf_stats (include/sst.h): the first-visit frontier's record."""
    _fields_ = [(n, ctypes.c_int64) for n in ("live", "nodes", "chunks", "splits", "aborted", "bands", "key_words",
                                             "max_band_groups", "max_band_nodes", "table_slots", "node_cap",
                                             "overflow_bits", "groups", "edges")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


class JaccardArgs(ctypes.Structure):
    """sst_jaccard_args (include/sst.h)."""
    _fields_ = [("n_spec", ctypes.c_int64), ("max_len", ctypes.c_void_p), ("skel_off", ctypes.c_void_p),
                ("skel", ctypes.c_void_p), ("lower", ctypes.c_void_p), ("upper", ctypes.c_void_p),
                ("status_lb", ctypes.c_void_p), ("su_mass", ctypes.c_void_p), ("row_mass", ctypes.c_void_p),
                ("comb_off", ctypes.c_void_p), ("comb", ctypes.c_void_p), ("seq_len", ctypes.c_void_p),
                ("status", ctypes.c_void_p), ("max_variance", ctypes.c_double)]


class WalkArgs(ctypes.Structure):
    """sst_walk_args (include/sst.h): device pointers of the skeleton walk."""
    _R = WALK_MAX_ROUNDS
    _fields_ = [("peak_off", ctypes.c_void_p), ("cnt", ctypes.c_void_p), ("r_su", ctypes.c_void_p),
                ("r_ob", ctypes.c_void_p), ("r_meta", ctypes.c_void_p), ("alive", ctypes.c_void_p),
                ("alpha", ctypes.c_void_p), ("max_len", ctypes.c_void_p), ("pair_ok", ctypes.c_void_p),
                ("n_spec", ctypes.c_int64), ("slots", ctypes.c_int64), ("tol", ctypes.c_double),
                ("prec", ctypes.c_double), ("rprec", ctypes.c_double), ("d_off", ctypes.c_void_p),
                ("d_n", ctypes.c_void_p), ("d_key", ctypes.c_void_p), ("d_thr", ctypes.c_void_p),
                ("q_off", ctypes.c_void_p), ("q0", ctypes.c_void_p), ("s_ptr", ctypes.c_void_p),
                ("s_n", ctypes.c_void_p), ("s_st", ctypes.c_void_p), ("n_rounds", ctypes.c_int),
                ("rq_block", ctypes.c_void_p * _R), ("rq_ptr", ctypes.c_void_p * _R),
                ("rq_n", ctypes.c_void_p * _R), ("rq_st", ctypes.c_void_p * _R), ("req_block", ctypes.c_void_p),
                ("req_mass", ctypes.c_void_p), ("req_thr", ctypes.c_void_p), ("req_spec", ctypes.c_void_p),
                ("req_count", ctypes.c_void_p), ("req_cap", ctypes.c_uint64), ("name_hash", ctypes.c_void_p),
                ("sides", ctypes.c_void_p), ("n_sides", ctypes.c_uint32), ("scratch", ctypes.c_void_p),
                ("scratch_stride", ctypes.c_uint64), ("pos_cap", ctypes.c_uint32), ("len_cap", ctypes.c_uint32),
                ("expl_cap", ctypes.c_uint32), ("cand_cap", ctypes.c_uint32), ("tset_cap", ctypes.c_uint32),
                ("side_rows", ctypes.c_void_p), ("skel_off", ctypes.c_void_p), ("skel", ctypes.c_void_p),
                ("min_end", ctypes.c_void_p), ("max_end", ctypes.c_void_p), ("kept", ctypes.c_void_p),
                ("side_status", ctypes.c_void_p), ("n_suspended", ctypes.c_void_p), ("n_big", ctypes.c_void_p),
                ("slot", ctypes.c_void_p), ("resume", ctypes.c_int)]


def _share_hip_runtime_with_torch():
    """One HIP runtime per process.  PyTorch-ROCm wheels bundle their own
    libamdhip64 (same SONAME, libamdhip64.so.7, as /opt/rocm's) and load it
    by its unversioned name: if this library loaded /opt/rocm's copy first, a
    later torch import would load a second runtime that sees no GPU.  When
    torch is installed, pre-load its copy (by path, without importing torch)
    so that libsstgpu.so and torch bind to the same runtime in either order."""
    try:
        import importlib.util

        spec = importlib.util.find_spec("torch")
        if spec is None or not spec.origin:
            return
        hip = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
        if os.path.exists(hip):
            ctypes.CDLL(hip, mode=ctypes.RTLD_GLOBAL)
    except OSError:
        pass


def load_library(path=LIB_PATH):
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build the HIP engine first (python -c 'import __graft_entry__ as g; g.build()' "
            "or make -C spectrseqtools_amd/csrc)")
    if path == LIB_PATH and not os.environ.get("SST_LIBRARY"):
        from . import build_record

        why = build_record.check(path)
        if why:
            raise ImportError(f"{path}: {why}; rebuild it (make -B -C spectrseqtools_amd/csrc: -B also "
                              "when the library looks up to date)")
    _share_hip_runtime_with_torch()
    lib = ctypes.CDLL(path)
    lib.sst_device_count.restype = _I
    lib.sst_ctx_create.argtypes = [_I, _PP]
    lib.sst_ctx_destroy.argtypes = [_P]
    lib.sst_ctx_destroy.restype = None
    lib.sst_last_error.argtypes = [_P]
    lib.sst_last_error.restype = ctypes.c_char_p
    lib.sst_ctx_stream.argtypes = [_P]
    lib.sst_ctx_stream.restype = _P
    lib.sst_ctx_set_stream.argtypes = [_P, _P]
    lib.sst_ctx_set_stream.restype = _I
    lib.sst_ctx_trim.argtypes = [_P]
    lib.sst_ctx_trim.restype = _I
    lib.sst_ctx_synchronize.argtypes = [_P]
    lib.sst_table_build.argtypes = [_P, _P, _I, _I64, _I, _PP]
    lib.sst_table_upload.argtypes = [_P, _P, _I, _P, _I64, _I, _PP]
    lib.sst_table_set_budgets.argtypes = [_P, _P, _P]
    lib.sst_table_shape.argtypes = [_P, ctypes.POINTER(_I), ctypes.POINTER(_I64), ctypes.POINTER(_I)]
    lib.sst_table_download.argtypes = [_P, _P]
    lib.sst_table_destroy.argtypes = [_P]
    lib.sst_table_destroy.restype = None
    lib.sst_is_valid_batch.argtypes = [_P, _P, _P, _I64, _D, _D, _P]
    lib.sst_is_valid_batch_device.argtypes = [_P, _P, _P, _I64, _D, _D, _P]
    lib.sst_explain_batch.argtypes = [_P, _P, _P, _I64, _D, _D, _P, _I64, _I, _U64, _PP]
    lib.sst_explain_batch_device.argtypes = [_P, _P, _P, _I64, _D, _D, _P, _I64, _I, _U64, _PP]
    lib.sst_explain_alpha_batch_device.argtypes = [_P, _P, _P, _P, _P, _I64, _D, _D, _P, _I64, _I, _U64, _PP]
    lib.sst_explain_alpha_lens_batch_device.argtypes = [_P, _P, _P, _P, _P, _P, _P, _I, _I64, _D, _D, _P, _U64, _PP]
    lib.sst_result_host.argtypes = [_P, _PP, _PP, _PP, _PP, ctypes.POINTER(_U64)]
    lib.sst_result_device.argtypes = [_P, _PP, _PP, _PP, _PP, ctypes.POINTER(_U64)]
    lib.sst_result_hit_list.argtypes = [_P, _PP, ctypes.POINTER(_U64)]
    lib.sst_result_hit_list.restype = _I
    lib.sst_result_settle.argtypes = [_P, ctypes.POINTER(_U64), ctypes.POINTER(_U64)]
    lib.sst_result_settle.restype = _I
    lib.sst_result_fetch.argtypes = [_P]
    lib.sst_result_free.argtypes = [_P]
    lib.sst_result_free.restype = None
    lib.sst_result_stats.argtypes = [_P, _P]
    lib.sst_profile_enable.argtypes = [_P, _I]
    lib.sst_profile_select.argtypes = [_P, ctypes.c_uint32]
    lib.sst_profile_sample.argtypes = [_P, ctypes.c_uint32]
    lib.sst_profile_read.argtypes = [_P, _P, _P]
    lib.sst_length_bound_batch.argtypes = [_P, _P, _P, _I64, _D, _D, _I, _I64, _I, _P, _P]
    lib.sst_length_bound_alpha_batch.argtypes = [_P, _P, _P, _P, _P, _I64, _I64, _D, _D, _I, _I64, _I, _P, _P]
    lib.sst_explain_recursion_batch.argtypes = [_P, _P, _P, _I64, _D, _D, _P, _I64, _U64, _PP]
    lib.sst_is_singleton_batch.argtypes = [_P, _P, _I, _P, _P, _I64, _D, _D, _P]
    lib.sst_is_singleton_batch_device.argtypes = [_P, _P, _I, _P, _P, _I64, _D, _D, _P]
    lib.sst_is_valid_peaks.argtypes = [_P, _P, _I64, _P, _I, _D, _D, _P]
    lib.sst_is_valid_peaks_device.argtypes = [_P, _P, _I64, _P, _I, _D, _D, _P]
    lib.sst_window_pairs.argtypes = [_P, _P, _I64, _D, _P, _P, _I64]
    lib.sst_window_pairs.restype = _I64
    lib.sst_result_pair_hits.argtypes = [_P, _PP, ctypes.POINTER(_U64), ctypes.POINTER(_U64), ctypes.POINTER(_I)]
    lib.sst_result_pair_hits.restype = _I
    lib.sst_table_pair_records.argtypes = [_P, _P, _I64, ctypes.POINTER(_I64)]
    lib.sst_table_pair_records.restype = _I
    lib.sst_wire_pack.argtypes = [_P, _P, _I64, _P, _I64]
    lib.sst_wire_pack.restype = _I64
    lib.sst_su_diff_queries.argtypes = [_P, _P, _P, _P, _I64, _D, _D, _P, _P, _P, _P, _I64]
    lib.sst_su_diff_queries.restype = _I64
    lib.sst_py_tuple_hash.argtypes = [_P, _I64]
    lib.sst_py_tuple_hash.restype = _I64
    lib.sst_pyset_order.argtypes = [_P, _P, _I64, _P]
    lib.sst_pyset_order.restype = _I64
    lib.sst_sort_rows.argtypes = [_P, _P, _I64, _I64, _P]
    lib.sst_sort_rows.restype = _I
    lib.sst_step_device.argtypes = [_P, _P, _I64, _P, _I, _P, _P, _P, _I64, _D, _D, _P, _I64, _I, _U64, _PP]
    lib.sst_step_device.restype = _I
    lib.sst_explain_pairs_alpha.argtypes = [_P, _P, _P, _P, _P, _I64, _I64, _D, _D, _P, _P, _P, _P]
    lib.sst_explain_pairs_alpha.restype = _I
    lib.sst_explain_pairs_alpha_device.argtypes = [_P, _P, _P, _P, _P, _I64, _D, _D, _P, _P, _P, _P]
    lib.sst_explain_pairs_alpha_device.restype = _I
    lib.sst_is_valid_alpha.argtypes = [_P, _P, _P, _P, _I64, _P, _D, _D, _P]
    lib.sst_is_valid_alpha.restype = _I
    lib.sst_is_valid_alpha_device.argtypes = [_P, _P, _P, _P, _I64, _P, _D, _D, _P]
    lib.sst_is_valid_alpha_device.restype = _I
    lib.sst_dict_union.argtypes = [_P, _I64, _P, _P, _P, _P, _P, _P]
    lib.sst_dict_union.restype = _I64
    lib.sst_step_rows_device.argtypes = [_P, _P, _P, _I64, _I64, _P, _D, _D, _P, _P, _P, _I, _D, _D, _D, _I64, _U64,
                                         _I64, _P, _PP]
    lib.sst_step_rows_device.restype = _I
    lib.sst_result_queries.argtypes = [_P, ctypes.POINTER(_I64)]
    lib.sst_result_queries.restype = _I
    lib.sst_classify_rows_device.argtypes = [_P, _P, _P, _I64, _I64, _P, _D, _D, _P, _P, _P, _I, _D, _D, _D, _P, _P,
                                             _P, _P, _P, _P, _P]
    lib.sst_classify_rows_device.restype = _I
    lib.sst_fix_round_device.argtypes = [_P, _P, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _D, _D, _D, _P,
                                         ctypes.POINTER(ExactIO)]
    lib.sst_fix_round_device.restype = _I
    lib.sst_valid_rows_alpha_device.argtypes = [_P, _P, _I64, _P, _P, _P, _P, _P, _P, _D, _D, _P]
    lib.sst_valid_rows_alpha_device.restype = _I
    lib.sst_bins_count_device.argtypes = [_P, _P, _I64, _P, _P, _P, _P, _P, _D, _P, _P, _P, _P]
    lib.sst_bins_count_device.restype = _I
    lib.sst_bins_emit_device.argtypes = [_P, _P, _I64, _P, _P, _P, _P, _P, _P, _D, _D, _P, _P, _P, _P, _P, _P, _P,
                                         _P, _P, _P]
    lib.sst_bins_emit_device.restype = _I
    lib.sst_pyset_table_size.argtypes = [ctypes.c_uint32]
    lib.sst_pyset_table_size.restype = ctypes.c_uint32
    lib.sst_walk_scratch_bytes.argtypes = [ctypes.c_uint32] * 5
    lib.sst_walk_scratch_bytes.restype = ctypes.c_uint64
    lib.sst_skel_walk_device.argtypes = [_P, ctypes.POINTER(WalkArgs)]
    lib.sst_skel_walk_device.restype = _I
    lib.sst_result_refs_device.argtypes = [_P, _P, _P, _P, _P]
    lib.sst_result_refs_device.restype = _I
    lib.sst_dict_count_device.argtypes = [_P, _P, _I64, _P, _P, _P, _P, _P, _D, _D, _P, _P, _P]
    lib.sst_dict_count_device.restype = _I
    lib.sst_dict_build_device.argtypes = [_P, _P, _I64, _P, _P, _P, _P, _P, _P, _D, _D, _D, _P, _P, _P, _P, _P,
                                          ctypes.POINTER(ExactIO)]
    lib.sst_dict_list_device.argtypes = [_P, _P, _I64, _P, _P, _P, _P, _P, _D, _D, _P, ctypes.POINTER(ExactIO)]
    lib.sst_dict_list_device.restype = _I
    lib.sst_fix_finish_device.argtypes = [_P, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P, ctypes.POINTER(ExactIO)]
    lib.sst_pipe_reserve_rows.argtypes = [_P, _I64]
    lib.sst_pipe_reserve_rows.restype = _I
    lib.sst_fix_finish_device.restype = _I
    lib.sst_dict_build_device.restype = _I
    lib.sst_reach_rows_device.argtypes = [_P, _P, _P, _P, _I64, _P]
    lib.sst_reach_rows_device.restype = _I
    lib.sst_length_bounds_reach_device.argtypes = [_P, _P, _P, _P, _P, _P, _P, _P, _I64, _D, _D, _I, _I64, _P, _P, _P,
                                                   _P, _P, _P, _P, _I64, ctypes.c_uint32, _I]
    lib.sst_length_bounds_reach_device.restype = _I
    lib.sst_reach_lowest_device.argtypes = [_P, _P, _P, _P, _I64, _P, _P, _P]
    lib.sst_reach_lowest_device.restype = _I
    lib.sst_length_bounds_frontier_device.argtypes = [_P, _P, _P, _P, _P, _P, _P, _I64, _D, _D, _I, _I64, _P, _P,
                                                      _P, _P, _P, _P, _P, _U64, ctypes.POINTER(LbfStats)]
    lib.sst_length_bounds_frontier_device.restype = _I
    lib.sst_post_skeleton_device.argtypes = [_P, ctypes.POINTER(PostArgs)]
    lib.sst_post_skeleton_device.restype = _I
    lib.sst_requery_merge_device.argtypes = [_P, ctypes.POINTER(RequeryMergeArgs), _P, _P]
    lib.sst_requery_merge_device.restype = _I
    lib.sst_jaccard_device.argtypes = [_P, ctypes.POINTER(JaccardArgs)]
    lib.sst_jaccard_device.restype = _I
    lib.sst_skeleton_alpha_device.argtypes = [_P, _I64, _P, _P, _P, _P, _P]
    lib.sst_skeleton_alpha_device.restype = _I
    return lib


_lib = None
_lib_lock = threading.Lock()


def lib():
    global _lib
    with _lib_lock:
        if _lib is None:
            _lib = load_library()
        return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def su_diff_queries(su, obs, flags, offsets, max_weight, tolerance):
    """sst_su_diff_queries: (diff, thr, spec, kind) of the first
    filter_by_explanation round over many spectra (host code)."""
    su = np.ascontiguousarray(su, dtype=np.float64)
    obs = np.ascontiguousarray(obs, dtype=np.float64)
    flags = np.ascontiguousarray(flags, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    L = lib()
    cap = 0  # the first call counts (cheap: no output), the second fills
    while True:
        d, t = np.empty(cap, np.float64), np.empty(cap, np.float64)
        g, k = np.empty(cap, np.int64), np.empty(cap, np.int8)
        n = L.sst_su_diff_queries(_ptr(su), _ptr(obs), _ptr(flags), _ptr(offsets), len(offsets) - 1,
                                  float(max_weight), float(tolerance), _ptr(d), _ptr(t), _ptr(g), _ptr(k), cap)
        if n < 0:
            raise EngineError(f"sst_su_diff_queries failed ({n})")
        if n <= cap:
            return d[:n], t[:n], g[:n], k[:n]
        cap = int(n)


def dict_union(offsets, key, kind, status, rowmask):
    """sst_dict_union: per spectrum the surviving entries of
    collect_diff_explanations_for_su's dict (keep[i]) and the union of their
    candidate rows ([n_spec, 2] u64 masks).  Host code."""
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    key = np.ascontiguousarray(key, dtype=np.float64)
    kind = np.ascontiguousarray(kind, dtype=np.int8)
    status = np.ascontiguousarray(status, dtype=np.int8)
    rowmask = np.ascontiguousarray(rowmask, dtype=np.uint64).reshape(-1, 2)
    n_spec = len(offsets) - 1
    keep = np.zeros(len(key), np.uint8)
    union = np.zeros((max(n_spec, 0), 2), np.uint64)
    rc = lib().sst_dict_union(_ptr(offsets), n_spec, _ptr(key), _ptr(kind), _ptr(status), _ptr(rowmask), _ptr(keep),
                              _ptr(union))
    if rc < 0:
        raise EngineError(f"sst_dict_union failed ({rc})")
    return keep.astype(bool), union


def py_tuple_hash(item_hashes):
    """sst_py_tuple_hash: hash(tuple) from its items' hashes (host code)."""
    h = np.ascontiguousarray(item_hashes, dtype=np.int64)
    return int(lib().sst_py_tuple_hash(_ptr(h), len(h)))


def pyset_order(keys, hashes):
    """sst_pyset_order: the iteration order of a set built by adding the
    elements `keys` (hashes `hashes`) in order (host code)."""
    k = np.ascontiguousarray(keys, dtype=np.int32)
    h = np.ascontiguousarray(hashes, dtype=np.int64)
    out = np.empty(len(k), np.int32)
    m = lib().sst_pyset_order(_ptr(k), _ptr(h), len(k), _ptr(out))
    if m < 0:
        raise EngineError(f"sst_pyset_order failed ({m})")
    return out[:m].tolist()


def pyset_table_size(n):
    """CPython's set table size after n distinct additions (sst_pyset_table_size)."""
    return int(lib().sst_pyset_table_size(int(n)))


def walk_scratch_bytes(pos_cap, len_cap, expl_cap, cand_cap, tset_cap):
    return int(lib().sst_walk_scratch_bytes(pos_cap, len_cap, expl_cap, cand_cap, tset_cap))


def sort_rows(group, key, n_groups):
    """sst_sort_rows: permutation sorting by group, then key, ties in row
    order (numpy.lexsort((rows, key, group)); host code)."""
    group = np.ascontiguousarray(group, dtype=np.int64)
    key = np.ascontiguousarray(key, dtype=np.float64)
    order = np.empty(len(group), np.int64)
    rc = lib().sst_sort_rows(_ptr(group), _ptr(key), len(group), int(n_groups), _ptr(order))
    if rc:
        raise EngineError(f"sst_sort_rows failed ({rc})")
    return order


def window_pairs(su, offsets, max_weight):
    """sst_window_pairs: the (start, end) index pairs of the reference's
    sliding window (prediction.py:286-329) over every side su[offsets[j]:
    offsets[j+1]] (host code in libsstgpu.so; no device needed)."""
    su = np.ascontiguousarray(su, dtype=np.float64)
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    L = lib()
    cap = max(16, 4 * len(su))
    while True:
        s = np.empty(cap, np.int64)
        e = np.empty(cap, np.int64)
        k = L.sst_window_pairs(_ptr(su), _ptr(offsets), len(offsets) - 1, float(max_weight), _ptr(s), _ptr(e), cap)
        if k < 0:
            raise EngineError(f"sst_window_pairs failed ({k})")
        if k <= cap:
            return s[:k], e[:k]
        cap = int(k)


_DT = {4: np.uint8, 8: np.uint16, 16: np.uint32, 32: np.uint64}


class Engine:
    """One HIP device context (one per process per GPU)."""

    def __init__(self, device=0):
        L = lib()
        n = L.sst_device_count()
        if n <= 0:
            raise EngineError("no HIP device visible: the mass-explanation engine runs on MI355X only")
        if device >= n:
            raise EngineError(f"HIP device {device} not present ({n} visible)")
        h = ctypes.c_void_p()
        rc = L.sst_ctx_create(int(device), ctypes.byref(h))
        if rc != 0:
            raise EngineError(f"sst_ctx_create({device}) failed with {rc}")
        self.handle = h
        self.device = device
        self._lib = L

    def check(self, rc, what):
        if rc != 0:
            msg = self._lib.sst_last_error(self.handle)
            raise EngineError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")

    @property
    def stream(self):
        return self._lib.sst_ctx_stream(self.handle)

    def set_stream(self, stream=None):
        """Queue subsequent work on `stream` (a hipStream_t handle, e.g.
        torch.cuda.Stream().cuda_stream), or on the engine's own stream when
        None.  The caller orders work across streams (sst_ctx_set_stream)."""
        self.check(self._lib.sst_ctx_set_stream(self.handle, stream), "sst_ctx_set_stream")

    def synchronize(self):
        self.check(self._lib.sst_ctx_synchronize(self.handle), "sst_ctx_synchronize")

    def trim(self):
        """Release the cached frontier workspaces (sst_ctx_trim)."""
        self.check(self._lib.sst_ctx_trim(self.handle), "sst_ctx_trim")

    def is_singleton(self, integer_masses, masses, thresholds, tolerance, precision):
        """fragment_classification.is_singleton for each mass: int8 {0, 1}."""
        w = np.ascontiguousarray(integer_masses, dtype=np.int64)
        m = np.ascontiguousarray(masses, dtype=np.float64)
        t = None if thresholds is None else np.ascontiguousarray(thresholds, dtype=np.float64)
        out = np.zeros(len(m), np.int8)
        self.check(self._lib.sst_is_singleton_batch(self.handle, _ptr(w), len(w), _ptr(m), _ptr(t), len(m),
                                                    float(tolerance), float(precision), _ptr(out)),
                   "sst_is_singleton_batch")
        return out

    def profile(self, on=True, kernels=None, every=1):
        """Bracket launches with HIP events: all kernels, or only the ids in
        `kernels`; only every `every`-th launch of each (sst_profile_sample)."""
        self.check(self._lib.sst_profile_sample(self.handle, int(every)), "sst_profile_sample")
        if kernels is None or not on:
            self.check(self._lib.sst_profile_enable(self.handle, int(bool(on))), "sst_profile_enable")
        else:
            mask = 0
            for k in kernels:
                mask |= 1 << int(k)
            self.check(self._lib.sst_profile_select(self.handle, mask), "sst_profile_select")

    def profile_read(self):
        """{kernel id: (total ms, launches)} since the last read."""
        ms = np.zeros(K_COUNT, np.float64)
        n = np.zeros(K_COUNT, np.int64)
        self.check(self._lib.sst_profile_read(self.handle, _ptr(ms), _ptr(n)), "sst_profile_read")
        return {k: (float(ms[k]), int(n[k])) for k in range(K_COUNT) if n[k]}

    def close(self):
        if self.handle:
            self._lib.sst_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_engines = {}
_engines_lock = threading.Lock()


def default_device():
    for k in ("SST_DEVICE", "LOCAL_RANK"):
        if os.environ.get(k, "").isdigit():
            return int(os.environ[k])
    return 0


def get_engine(device=None):
    device = default_device() if device is None else device
    with _engines_lock:
        if device not in _engines:
            _engines[device] = Engine(device)
        return _engines[device]


class ExplainResult:
    """Host (or device) views of one sst_explain_batch* call."""

    def __init__(self, engine, handle, n):
        self.engine = engine
        self.handle = handle
        self.n = n
        self.status = self.count = self.offset = self.payload = None

    def fetch(self):
        """Host views of the fetched result (sst_result_host): status,
        count / offset (0 for queries without candidates) and the dense
        payload."""
        L = self.engine._lib
        st, cnt, off, pay = (ctypes.c_void_p() for _ in range(4))
        nb = _U64()
        self.engine.check(L.sst_result_host(self.handle, ctypes.byref(st), ctypes.byref(cnt), ctypes.byref(off),
                                            ctypes.byref(pay), ctypes.byref(nb)), "sst_result_host")
        n = self.n = self.queries()

        def view(p, dtype, k):
            if k == 0 or not p.value:
                return np.zeros(0, dtype)
            return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(np.ctypeslib.as_ctypes_type(dtype))),
                                         shape=(k,)).copy()

        self.status = view(st, np.int8, n)
        self.count = view(cnt, np.uint64, n)
        self.offset = view(off, np.uint64, n)
        self.payload = view(pay, np.uint8, int(nb.value))
        return self

    def queries(self):
        """Number of explain queries (sst_result_queries; the rows step learns
        it from its pass)."""
        n = _I64()
        self.engine.check(self.engine._lib.sst_result_queries(self.handle, ctypes.byref(n)), "sst_result_queries")
        return int(n.value)

    def settle(self):
        """Wait for the pass and complete it (sst_result_settle):
        (hit records, dense payload bytes)."""
        nh, nb = _U64(), _U64()
        self.engine.check(self.engine._lib.sst_result_settle(self.handle, ctypes.byref(nh), ctypes.byref(nb)),
                          "sst_result_settle")
        return int(nh.value), int(nb.value)

    def stats(self):
        out = np.zeros(8, np.uint64)
        self.engine.check(self.engine._lib.sst_result_stats(self.handle, _ptr(out)), "sst_result_stats")
        return out

    def device_views(self, arrays=True):
        """(status, count, offset, payload, payload bytes) device pointers;
        arrays=False skips building the per-query count / offset arrays
        (their pointers are then None)."""
        L = self.engine._lib
        st, cnt, off, pay = (ctypes.c_void_p() for _ in range(4))
        nb = _U64()
        self.engine.check(L.sst_result_device(self.handle, ctypes.byref(st), ctypes.byref(cnt) if arrays else None,
                                              ctypes.byref(off) if arrays else None, ctypes.byref(pay),
                                              ctypes.byref(nb)), "sst_result_device")
        return st.value, cnt.value, off.value, pay.value, int(nb.value)

    def hit_list_device(self):
        """(device pointer, n_hits) of the dense hit list: u32x4 records
        {query, count, word lo, word hi}; word = payload offset (SOME) or the
        exact count (OVERFLOW / ABORTED) (sst_result_hit_list)."""
        p = ctypes.c_void_p()
        nh = _U64()
        self.engine.check(self.engine._lib.sst_result_hit_list(self.handle, ctypes.byref(p), ctypes.byref(nh)),
                          "sst_result_hit_list")
        return p.value, int(nh.value)

    def pair_hits_device(self):
        """(refs device pointer, n_pair_hits, pair_bytes, n_scan_wg): the
        pair-path part of the dense hit list (sst_result_pair_hits)."""
        p = ctypes.c_void_p()
        nh, nb, wg = _U64(), _U64(), _I()
        self.engine.check(self.engine._lib.sst_result_pair_hits(self.handle, ctypes.byref(p), ctypes.byref(nh),
                                                                ctypes.byref(nb), ctypes.byref(wg)),
                          "sst_result_pair_hits")
        return p.value, int(nh.value), int(nb.value), int(wg.value)

    def wire_pack(self, d_valid, n_valid, d_out=None, cap=0):
        """sst_wire_pack: this result plus n_valid is_valid codes at d_valid
        in the gather's wire format v4, packed on the device into d_out (cap
        bytes).  d_out None: sizing only.  Returns the fixed part's bytes."""
        n = self.engine._lib.sst_wire_pack(self.handle, d_valid, int(n_valid), d_out, int(cap))
        if n < 0:
            self.engine.check(int(n), "sst_wire_pack")
        return int(n)

    def fetch_device(self):
        self.engine.check(self.engine._lib.sst_result_fetch(self.handle), "sst_result_fetch")
        return self.fetch()

    def candidates(self, i):
        """Row-index tuples of query i (ascending rows), in engine order."""
        k = int(self.count[i])
        p = int(self.offset[i])
        out = []
        pay = self.payload
        for _ in range(k):
            ln = int(pay[p])
            out.append(tuple(int(x) for x in pay[p + 1:p + 1 + ln]))
            p += 1 + ln
        return out

    def close(self):
        if self.handle:
            self.engine._lib.sst_result_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceTable:
    """A packed DP table plus its derived index, resident in HBM."""

    def __init__(self, engine, handle, n_rows, n_cols, compression, masses):
        self.engine = engine
        self.handle = handle
        self.n_rows = n_rows
        self.n_cols = n_cols
        self.compression = compression
        self.masses = list(masses)
        self._budgets = None

    @classmethod
    def build(cls, masses, max_mass, compression, engine=None):
        engine = engine or get_engine()
        w = np.ascontiguousarray(masses, dtype=np.int64)
        h = ctypes.c_void_p()
        engine.check(engine._lib.sst_table_build(engine.handle, _ptr(w), len(w), int(max_mass), int(compression),
                                                 ctypes.byref(h)), "sst_table_build")
        return cls._wrap(engine, h, w)

    @classmethod
    def upload(cls, masses, words, compression, engine=None):
        engine = engine or get_engine()
        w = np.ascontiguousarray(masses, dtype=np.int64)
        words = np.ascontiguousarray(words, dtype=_DT[compression])
        if words.ndim != 2 or words.shape[0] != len(w):
            raise ValueError("packed table must have one row per integer mass")
        h = ctypes.c_void_p()
        engine.check(engine._lib.sst_table_upload(engine.handle, _ptr(w), len(w), _ptr(words), words.shape[1],
                                                  int(compression), ctypes.byref(h)), "sst_table_upload")
        return cls._wrap(engine, h, w)

    @classmethod
    def _wrap(cls, engine, h, w):
        nr, nc, C = _I(), _I64(), _I()
        engine._lib.sst_table_shape(h, ctypes.byref(nr), ctypes.byref(nc), ctypes.byref(C))
        return cls(engine, h, nr.value, nc.value, C.value, w.tolist())

    def set_budgets(self, is_mod, caps):
        key = (tuple(bool(x) for x in is_mod), tuple(int(c) for c in caps))
        if key == self._budgets:
            return
        m = np.ascontiguousarray(key[0], dtype=np.uint8)
        c = np.ascontiguousarray(key[1], dtype=np.int64)
        self.engine.check(self.engine._lib.sst_table_set_budgets(self.handle, _ptr(m), _ptr(c)),
                          "sst_table_set_budgets")
        self._budgets = key

    def pair_records(self):
        """u32 payload record per pair-list entry (sst_table_pair_records);
        empty for tables without the list."""
        L = self.engine._lib
        n = _I64()
        self.engine.check(L.sst_table_pair_records(self.handle, None, 0, ctypes.byref(n)), "sst_table_pair_records")
        out = np.zeros(n.value, np.uint32)
        if n.value:
            self.engine.check(L.sst_table_pair_records(self.handle, _ptr(out), n.value, ctypes.byref(n)),
                              "sst_table_pair_records")
        return out

    def download(self):
        out = np.empty((self.n_rows, self.n_cols), dtype=_DT[self.compression])
        self.engine.check(self.engine._lib.sst_table_download(self.handle, _ptr(out)), "sst_table_download")
        return out

    def is_valid(self, masses, thresholds, tolerance, precision):
        m = np.ascontiguousarray(masses, dtype=np.float64)
        t = None if thresholds is None else np.ascontiguousarray(thresholds, dtype=np.float64)
        out = np.zeros(len(m), np.int8)
        self.engine.check(self.engine._lib.sst_is_valid_batch(self.handle, _ptr(m), _ptr(t), len(m), float(tolerance),
                                                              float(precision), _ptr(out)), "sst_is_valid_batch")
        return out

    def length_bound(self, su_masses, obs_masses, tolerance, precision, max_len, max_mods, direction,
                     exact_only=False, replay=False):
        """compute_sequence_length_bound for each (su, obs) pair: (bounds int64[n], status int8[n]).
        exact_only: skip the layered fast path; replay: the DFS replay instead of
        the first-visit frontier (cross-checks in tests)."""
        su = np.ascontiguousarray(su_masses, dtype=np.float64)
        ob = np.ascontiguousarray(obs_masses, dtype=np.float64)
        if su.shape != ob.shape:
            raise ValueError("su_masses and obs_masses differ in length")
        out = np.zeros(len(su), np.int64)
        st = np.zeros(len(su), np.int8)
        d = {"lower": 0, "upper": 1}[direction] if isinstance(direction, str) else int(direction)
        d |= 2 if exact_only else 0  # SST_LB_EXACT_ONLY
        d |= 4 if replay else 0  # SST_LB_REPLAY
        self.engine.check(self.engine._lib.sst_length_bound_batch(self.handle, _ptr(su), _ptr(ob), len(su),
                                                                  float(tolerance), float(precision), int(max_len),
                                                                  int(max_mods), d, _ptr(out), _ptr(st)),
                          "sst_length_bound_batch")
        return out, st

    def length_bound_alpha(self, su_masses, obs_masses, spec, alpha, tolerance, precision, max_len, max_mods,
                           direction):
        """length_bound with query i on the reduced alphabet alpha[spec[i]]
        ([n_alpha, 2] u64 row masks; sst_length_bound_alpha_batch)."""
        su = np.ascontiguousarray(su_masses, dtype=np.float64)
        ob = np.ascontiguousarray(obs_masses, dtype=np.float64)
        sp = np.ascontiguousarray(spec, dtype=np.int32)
        al = np.ascontiguousarray(alpha, dtype=np.uint64).reshape(-1, 2)
        if su.shape != ob.shape or sp.shape != su.shape:
            raise ValueError("su_masses, obs_masses and spec differ in length")
        out = np.zeros(len(su), np.int64)
        st = np.zeros(len(su), np.int8)
        d = {"lower": 0, "upper": 1}[direction] if isinstance(direction, str) else int(direction)
        self.engine.check(self.engine._lib.sst_length_bound_alpha_batch(
            self.handle, _ptr(su), _ptr(ob), _ptr(sp), _ptr(al), len(al), len(su), float(tolerance),
            float(precision), int(max_len), int(max_mods), d, _ptr(out), _ptr(st)), "sst_length_bound_alpha_batch")
        return out, st

    def is_valid_peaks(self, observed, shifts, tolerance, precision):
        """is_valid over peaks x breakage shifts (sst_is_valid_peaks): int8
        [len(shifts) * n_peaks], breakage-major."""
        o = np.ascontiguousarray(observed, dtype=np.float64)
        sh = np.ascontiguousarray(shifts, dtype=np.float64)
        out = np.zeros(len(o) * len(sh), np.int8)
        self.engine.check(self.engine._lib.sst_is_valid_peaks(self.handle, _ptr(o), len(o), _ptr(sh), len(sh),
                                                              float(tolerance), float(precision), _ptr(out)),
                          "sst_is_valid_peaks")
        return out

    def explain_pairs_alpha(self, masses, thresholds, spec, masks, tolerance, precision):
        """sst_explain_pairs_alpha: pair-class windows against per-spectrum
        reduced alphabets (masks [n_spec, 2] u64 row bits of this table).
        -> (status i8, count u32, rowmask [n, 2] u64, range [n, 2] u32)."""
        m = np.ascontiguousarray(masses, dtype=np.float64)
        t = None if thresholds is None else np.ascontiguousarray(thresholds, dtype=np.float64)
        sp = np.ascontiguousarray(spec, dtype=np.int32)
        mk = np.ascontiguousarray(masks, dtype=np.uint64).reshape(-1, 2)
        n = len(m)
        st, cnt = np.zeros(n, np.int8), np.zeros(n, np.uint32)
        rm, rg = np.zeros((n, 2), np.uint64), np.zeros((n, 2), np.uint32)
        self.engine.check(self.engine._lib.sst_explain_pairs_alpha(self.handle, _ptr(m), _ptr(t), _ptr(sp), _ptr(mk),
                                                                   len(mk), n, float(tolerance), float(precision),
                                                                   _ptr(st), _ptr(cnt), _ptr(rm), _ptr(rg)),
                          "sst_explain_pairs_alpha")
        return st, cnt, rm, rg

    def is_valid_alpha(self, masses, thresholds, offsets, masks, tolerance, precision):
        """sst_is_valid_alpha: is_valid_mass against per-spectrum reduced
        alphabets; spectrum g's queries are [offsets[g], offsets[g+1]) in
        ascending mass order.  -> int8 (1 / 0 / -1 raise)."""
        m = np.ascontiguousarray(masses, dtype=np.float64)
        t = None if thresholds is None else np.ascontiguousarray(thresholds, dtype=np.float64)
        off = np.ascontiguousarray(offsets, dtype=np.int64)
        mk = np.ascontiguousarray(masks, dtype=np.uint64).reshape(-1, 2)
        out = np.zeros(len(m), np.int8)
        self.engine.check(self.engine._lib.sst_is_valid_alpha(self.handle, _ptr(m), _ptr(t), _ptr(off), len(off) - 1,
                                                              _ptr(mk), float(tolerance), float(precision), _ptr(out)),
                          "sst_is_valid_alpha")
        if (out == -10).any():
            raise EngineError("sst_is_valid_alpha: queries out of mass order within a spectrum")
        return out

    def is_valid_peaks_device(self, d_obs, n_peaks, shifts, tolerance, precision, d_out):
        sh = np.ascontiguousarray(shifts, dtype=np.float64)
        self.engine.check(self.engine._lib.sst_is_valid_peaks_device(self.handle, d_obs, int(n_peaks), _ptr(sh),
                                                                     len(sh), float(tolerance), float(precision),
                                                                     d_out), "sst_is_valid_peaks_device")

    def is_valid_device(self, d_mass, d_thr, n, tolerance, precision, d_out):
        self.engine.check(self.engine._lib.sst_is_valid_batch_device(self.handle, d_mass, d_thr, int(n),
                                                                     float(tolerance), float(precision), d_out),
                          "sst_is_valid_batch_device")

    def explain(self, masses, thresholds, tolerance, precision, max_mods, with_memo=True, cap=2 ** 32):
        m = np.ascontiguousarray(masses, dtype=np.float64)
        t = None if thresholds is None else np.ascontiguousarray(thresholds, dtype=np.float64)
        mods_arr, scalar = _mods(max_mods, len(m))
        h = ctypes.c_void_p()
        self.engine.check(self.engine._lib.sst_explain_batch(self.handle, _ptr(m), _ptr(t), len(m), float(tolerance),
                                                             float(precision), _ptr(mods_arr), scalar,
                                                             int(bool(with_memo)), int(cap), ctypes.byref(h)),
                          "sst_explain_batch")
        return ExplainResult(self.engine, h, len(m)).fetch()

    def explain_recursion(self, masses, thresholds, tolerance, precision, max_mods, cap=2 ** 32):
        """explain_mass_with_recursion, batched; max_mods: np.inf / non-negative integers (scalar or per mass)."""
        m = np.ascontiguousarray(masses, dtype=np.float64)
        t = None if thresholds is None else np.ascontiguousarray(thresholds, dtype=np.float64)
        mods_arr, scalar = _mods(max_mods, len(m))
        h = ctypes.c_void_p()
        self.engine.check(self.engine._lib.sst_explain_recursion_batch(self.handle, _ptr(m), _ptr(t), len(m),
                                                                       float(tolerance), float(precision),
                                                                       _ptr(mods_arr), scalar, int(cap),
                                                                       ctypes.byref(h)),
                          "sst_explain_recursion_batch")
        return ExplainResult(self.engine, h, len(m)).fetch()

    def explain_device(self, d_mass, d_thr, n, tolerance, precision, max_mods_scalar, d_mods=None, with_memo=True,
                       cap=2 ** 32, reuse=None):
        """Queue an explain batch on device buffers (no host sync).  `reuse`: an
        ExplainResult of this engine with capacity >= n whose buffers are reused."""
        h = ctypes.c_void_p(reuse.handle.value if reuse is not None else None)
        self.engine.check(self.engine._lib.sst_explain_batch_device(self.handle, d_mass, d_thr, int(n),
                                                                    float(tolerance), float(precision), d_mods,
                                                                    int(max_mods_scalar), int(bool(with_memo)),
                                                                    int(cap), ctypes.byref(h)),
                          "sst_explain_batch_device")
        if reuse is not None:
            reuse.n = n
            return reuse
        return ExplainResult(self.engine, h, n)

    def explain_alpha_device(self, d_mass, d_thr, d_spec, d_alpha, n, tolerance, precision, max_mods_scalar,
                             d_mods=None, with_memo=True, cap=2 ** 32, reuse=None):
        """sst_explain_alpha_batch_device: explain_device with query i answered
        on the reduced alphabet d_alpha[d_spec[i]] (u64 row-mask pairs over this
        table's rows), as the rebuilt reduced table would answer it."""
        h = ctypes.c_void_p(reuse.handle.value if reuse is not None else None)
        self.engine.check(self.engine._lib.sst_explain_alpha_batch_device(
            self.handle, d_mass, d_thr, d_spec, d_alpha, int(n), float(tolerance), float(precision), d_mods,
            int(max_mods_scalar), int(bool(with_memo)), int(cap), ctypes.byref(h)), "sst_explain_alpha_batch_device")
        if reuse is not None:
            reuse.n = n
            return reuse
        return ExplainResult(self.engine, h, n)

    def explain_alpha_lens_device(self, d_mass, d_thr, d_spec, d_alpha, d_qlen, caps_by_len, n, tolerance,
                                  precision, d_mods, cap=2 ** 32):
        """sst_explain_alpha_lens_batch_device: explain_alpha_device with
        per-query budgets -- query i's row caps caps_by_len[d_qlen[i]] (host
        [n_lens, n_rows] ints), its max_modifications d_mods[i]."""
        caps = np.ascontiguousarray(caps_by_len, dtype=np.int64)
        h = ctypes.c_void_p(None)
        self.engine.check(self.engine._lib.sst_explain_alpha_lens_batch_device(
            self.handle, d_mass, d_thr, d_spec, d_alpha, d_qlen, caps.ctypes.data, int(caps.shape[0]), int(n),
            float(tolerance), float(precision), d_mods, int(cap), ctypes.byref(h)),
            "sst_explain_alpha_lens_batch_device")
        return ExplainResult(self.engine, h, n)

    def explain_alpha(self, masses, thresholds, spec, alpha, tolerance, precision, max_mods, with_memo=True,
                      cap=2 ** 32):
        """Host-buffer form of explain_alpha_device (tests, small batches):
        uploads the inputs, settles and fetches the result."""
        import torch

        dev = torch.device("cuda", self.engine.device)
        n = len(masses)
        dm = torch.as_tensor(np.ascontiguousarray(masses, dtype=np.float64), device=dev)
        dt = torch.as_tensor(np.ascontiguousarray(thresholds, dtype=np.float64), device=dev)
        ds = torch.as_tensor(np.ascontiguousarray(spec, dtype=np.int32), device=dev)
        da = torch.as_tensor(np.ascontiguousarray(alpha, dtype=np.uint64).view(np.int64), device=dev)
        mods = np.broadcast_to(np.asarray(max_mods, dtype=np.int64), (n,))
        dmods = torch.as_tensor(np.ascontiguousarray(mods), device=dev)
        torch.cuda.synchronize(dev)
        res = self.explain_alpha_device(dm.data_ptr(), dt.data_ptr(), ds.data_ptr(), da.data_ptr(), n, tolerance,
                                        precision, 0, d_mods=dmods.data_ptr(), with_memo=with_memo, cap=cap)
        res.fetch_device()
        del dm, dt, ds, da, dmods
        return res

    def explain_alpha_lens(self, masses, thresholds, spec, alpha, qlen, caps_by_len, max_mods, tolerance, precision):
        """Host-buffer form of explain_alpha_lens_device (tests): query i with
        row caps caps_by_len[qlen[i]] and max_mods[i]; settles and fetches."""
        import torch

        dev = torch.device("cuda", self.engine.device)
        n = len(masses)
        dm = torch.as_tensor(np.ascontiguousarray(masses, dtype=np.float64), device=dev)
        dt = torch.as_tensor(np.ascontiguousarray(thresholds, dtype=np.float64), device=dev)
        ds = torch.as_tensor(np.ascontiguousarray(spec, dtype=np.int32), device=dev)
        da = torch.as_tensor(np.ascontiguousarray(alpha, dtype=np.uint64).view(np.int64), device=dev)
        dq = torch.as_tensor(np.ascontiguousarray(qlen, dtype=np.int32), device=dev)
        dmods = torch.as_tensor(np.ascontiguousarray(np.broadcast_to(np.asarray(max_mods, np.int64), (n,))),
                                device=dev)
        torch.cuda.synchronize(dev)
        res = self.explain_alpha_lens_device(dm.data_ptr(), dt.data_ptr(), ds.data_ptr(), da.data_ptr(),
                                             dq.data_ptr(), caps_by_len, n, tolerance, precision, dmods.data_ptr())
        res.fetch_device()
        del dm, dt, ds, da, dq, dmods
        return res

    def step_rows_device(self, d_obs, d_peak_off, n_spec, n_peaks, d_su_seq, shifts, sides, d_valid_out, max_weight,
                         tolerance, precision, max_mods_scalar, max_queries, d_intensity=None, intensity_cutoff=0.5e6,
                         mass_cutoff=50000.0, cap=2 ** 32, reuse=None):
        """sst_step_rows_device: classify_fragments' is_valid + filters and
        the first filter_by_explanation round's window explains from the
        peaks, all on the device (queued, no host sync)."""
        sh = np.ascontiguousarray(shifts, dtype=np.float64)
        sd = np.ascontiguousarray(sides, dtype=np.uint8)
        h = ctypes.c_void_p(reuse.handle.value if reuse is not None else None)
        self.engine.check(self.engine._lib.sst_step_rows_device(
            self.handle, d_obs, d_peak_off, int(n_spec), int(n_peaks), d_intensity, float(intensity_cutoff),
            float(mass_cutoff), d_su_seq, _ptr(sh), _ptr(sd), len(sh), float(max_weight), float(tolerance),
            float(precision), int(max_mods_scalar), int(cap), int(max_queries), d_valid_out, ctypes.byref(h)),
            "sst_step_rows_device")
        if reuse is not None:
            return reuse
        return ExplainResult(self.engine, h, int(max_queries))

    def step_device(self, d_obs, n_peaks, shifts, d_valid_out, d_mass, d_thr, n, tolerance, precision,
                    max_mods_scalar, d_mods=None, with_memo=True, cap=2 ** 32, reuse=None):
        """sst_step_device: is_valid over peaks x breakage shifts (into
        d_valid_out, breakage-major) and an explain batch, queued together (one
        launch when the scan packs its own result).  Returns the ExplainResult."""
        sh = np.ascontiguousarray(shifts, dtype=np.float64)
        h = ctypes.c_void_p(reuse.handle.value if reuse is not None else None)
        self.engine.check(self.engine._lib.sst_step_device(self.handle, d_obs, int(n_peaks), _ptr(sh), len(sh),
                                                           d_valid_out, d_mass, d_thr, int(n), float(tolerance),
                                                           float(precision), d_mods, int(max_mods_scalar),
                                                           int(bool(with_memo)), int(cap), ctypes.byref(h)),
                          "sst_step_device")
        if reuse is not None:
            reuse.n = n
            return reuse
        return ExplainResult(self.engine, h, n)

    def close(self):
        if self.handle:
            self.engine._lib.sst_table_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _mods(max_mods, n):
    """np.inf / None -> -1 (the engine's inf); scalar or per-query array."""
    if np.ndim(max_mods) == 0:
        return None, _budget(max_mods)
    arr = np.array([_budget(x) for x in max_mods], dtype=np.int64)
    if len(arr) != n:
        raise ValueError("max_modifications array must have one entry per mass")
    return arr, 0


def _budget(a):
    if a is None:
        return -1
    a = float(a)
    if np.isinf(a):
        return -1 if a > 0 else 0
    # the reference only ever tests `A > 0`; negative budgets behave like 0
    return max(int(np.ceil(a)) if a != int(a) else int(a), 0)
