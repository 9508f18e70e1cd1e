"""ctypes binding of the CPU oracle (oracle/sst_oracle.c).

TEST INFRASTRUCTURE: imported only by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by spectrseqtools_amd/.
"""
import ctypes
import math
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "_build", "libsst_oracle.so")
NONE = float("nan")

_DT = {4: np.uint8, 8: np.uint16, 16: np.uint32, 32: np.uint64}


class _Res(ctypes.Structure):
    _fields_ = [
        ("status", ctypes.c_int),
        ("n_solutions", ctypes.c_int64),
        ("n_empty", ctypes.c_int64),
        ("n_items", ctypes.c_int64),
        ("lookups", ctypes.c_int64),
        ("lens", ctypes.POINTER(ctypes.c_int32)),
        ("rows", ctypes.POINTER(ctypes.c_int16)),
    ]


def _load():
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    lib = ctypes.CDLL(ORACLE_SO)
    P, I64, I, D = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_double
    lib.ora_table_cols.restype = I64
    lib.ora_table_cols.argtypes = [I64, I]
    lib.ora_build_table.argtypes = [P, I, I64, I, P]
    lib.ora_is_valid.argtypes = [P, I, I64, I, D, D, D, D]
    lib.ora_explain_table.argtypes = [P, I, I64, I, P, P, P, D, D, D, D, I64, I, I, ctypes.POINTER(_Res)]
    lib.ora_explain_recursion.argtypes = [I, P, P, P, D, D, D, D, I64, ctypes.POINTER(_Res)]
    lib.ora_result_free.argtypes = [ctypes.POINTER(_Res)]
    lib.ora_length_bound.restype = I64
    lib.ora_length_bound.argtypes = [P, I, I64, I, P, P, P, D, D, D, D, I64, I64, I]
    lib.ora_length_bound_memo.restype = I64
    lib.ora_length_bound_memo.argtypes = [P, I, I64, I, P, P, P, D, D, D, D, I64, I64, I, ctypes.POINTER(I64)]
    lib.ora_is_valid_batch.restype = I64
    lib.ora_is_valid_batch.argtypes = [P, I, I64, I, P, P, I64, D, D, I, P]
    lib.ora_explain_batch.restype = I64
    lib.ora_explain_batch.argtypes = [P, I, I64, I, P, P, P, P, P, P, I64, D, D, I, I, P, P, P]
    lib.ora_num_threads.restype = I
    return lib


LIB = _load()


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def build_table(masses, max_mass, C=32):
    cols = LIB.ora_table_cols(int(max_mass), C)
    out = np.zeros((len(masses), cols), dtype=_DT[C])
    w = np.ascontiguousarray(masses, dtype=np.int64)
    assert LIB.ora_build_table(_p(w), len(masses), int(max_mass), C, _p(out)) == 0
    return out


class Alphabet:
    """Row data the reference reads from dp_table.masses (mass, is_modification,
    round(max_len * modification_rate))."""

    def __init__(self, masses, is_mod, caps):
        self.w = np.ascontiguousarray(masses, dtype=np.int64)
        self.is_mod = np.ascontiguousarray(is_mod, dtype=np.uint8)
        self.cap = np.ascontiguousarray(caps, dtype=np.int64)


def _thr(t):
    return NONE if t is None else float(t)


def _A(a):
    return -1 if (a is None or a == "inf" or (isinstance(a, float) and math.isinf(a))) else int(a)


def is_valid(table, C, mass, threshold, tolerance, precision=1e-3):
    return LIB.ora_is_valid(_p(table), table.shape[0], table.shape[1], C, float(mass), _thr(threshold),
                            float(tolerance), float(precision))


def _collect(r):
    sols = []
    p = 0
    for i in range(r.n_solutions):
        k = r.lens[i]
        sols.append(tuple(int(r.rows[p + j]) for j in range(k)))
        p += k
    return sols


def explain_table(table, C, alph, mass, threshold, tolerance, A, with_memo=True, precision=1e-3):
    """-> (status, [row tuples in reference list order], n_empty, lookups);
    status 0 None, 1 set, -1 raise."""
    r = _Res()
    LIB.ora_explain_table(_p(table), table.shape[0], table.shape[1], C, _p(alph.w), _p(alph.is_mod), _p(alph.cap),
                          float(mass), _thr(threshold), float(tolerance), float(precision), _A(A), int(with_memo), 1,
                          ctypes.byref(r))
    out = (r.status, _collect(r) if r.status == 1 else [], r.n_empty, r.lookups)
    LIB.ora_result_free(ctypes.byref(r))
    return out


def explain_recursion(alph, mass, threshold, tolerance, A, precision=1e-3):
    r = _Res()
    LIB.ora_explain_recursion(len(alph.w), _p(alph.w), _p(alph.is_mod), _p(alph.cap), float(mass), _thr(threshold),
                              float(tolerance), float(precision), _A(A), ctypes.byref(r))
    out = (r.status, _collect(r) if r.status == 1 else [], r.n_empty)
    LIB.ora_result_free(ctypes.byref(r))
    return out


def length_bound(table, C, alph, su_mass, obs_mass, tolerance, max_len, max_mods, direction, precision=1e-3):
    v = LIB.ora_length_bound(_p(table), table.shape[0], table.shape[1], C, _p(alph.w), _p(alph.is_mod),
                             _p(alph.cap), float(su_mass), float(obs_mass), float(tolerance), float(precision),
                             int(max_len), int(max_mods), 1 if direction == "upper" else 0)
    return None if v == -(2 ** 63) else int(v)


def length_bound_memo(table, C, alph, su_mass, obs_mass, tolerance, max_len, max_mods, direction, precision=1e-3):
    """length_bound and the memo entries with non-zero pair bits when the
    reference's call returns (the (mass, row) nodes its DFS expanded; the
    memo's dead entries -- window values whose pair is 0, memoised with the
    default through the %C quirk of mass_table.py:403 -- are not counted), or
    (None, n) where it raises."""
    n = ctypes.c_int64(0)
    v = LIB.ora_length_bound_memo(_p(table), table.shape[0], table.shape[1], C, _p(alph.w), _p(alph.is_mod),
                                  _p(alph.cap), float(su_mass), float(obs_mass), float(tolerance), float(precision),
                                  int(max_len), int(max_mods), 1 if direction == "upper" else 0, ctypes.byref(n))
    return (None if v == -(2 ** 63) else int(v)), int(n.value)

def explain_batch(table, C, alph, masses, thrs, A, tolerance, with_memo=True, nthreads=1, precision=1e-3):
    n = len(masses)
    masses = np.ascontiguousarray(masses, dtype=np.float64)
    thrs = None if thrs is None else np.ascontiguousarray(thrs, dtype=np.float64)
    Aa = np.ascontiguousarray(np.broadcast_to(np.asarray(A, dtype=np.int64), (n,)))
    st = np.zeros(n, np.int8)
    cnt = np.zeros(n, np.int64)
    lk = np.zeros(n, np.int64)
    LIB.ora_explain_batch(_p(table), table.shape[0], table.shape[1], C, _p(alph.w), _p(alph.is_mod), _p(alph.cap),
                          _p(masses), _p(thrs), _p(Aa), n, float(tolerance), float(precision), int(with_memo),
                          int(nthreads), _p(st), _p(cnt), _p(lk))
    return st, cnt, lk


def is_valid_batch(table, C, masses, thrs, tolerance, nthreads=1, precision=1e-3):
    n = len(masses)
    masses = np.ascontiguousarray(masses, dtype=np.float64)
    thrs = None if thrs is None else np.ascontiguousarray(thrs, dtype=np.float64)
    out = np.zeros(n, np.int8)
    LIB.ora_is_valid_batch(_p(table), table.shape[0], table.shape[1], C, _p(masses), _p(thrs), n, float(tolerance),
                           float(precision), int(nthreads), _p(out))
    return out


def is_singleton_batch(masses, thrs, integer_masses, tolerance, precision=1e-3):
    """fragment_classification.py:104-119 restated (numpy, exact): target =
    round(mass/precision) (ties-to-even on the f64 quotient), thr =
    ceil(threshold/precision), threshold default tolerance*mass; True iff some
    value in [target - thr, target + thr] is one of integer_masses."""
    masses = np.asarray(masses, dtype=np.float64)
    thrs = tolerance * masses if thrs is None else np.asarray(thrs, dtype=np.float64)
    target = np.rint(masses / precision).astype(np.int64)
    th = np.ceil(thrs / precision).astype(np.int64)
    lo, hi = target - th, target + th
    w = np.unique(np.asarray(integer_masses, dtype=np.int64))
    k = np.searchsorted(w, lo, side="left")
    hit = (k < len(w)) & (w[np.minimum(k, len(w) - 1)] <= hi) & (lo <= hi)
    return hit
