"""Query producers of the reference pipeline, as array generators.

The reference issues its hot-path queries one Python call at a time:
  * fragment_classification.py:39-67  -- every observed mass x every breakage
    weight of build_breakage_dict -> is_valid_mass(su, thr = tolerance*obs);
  * prediction.py:286-329             -- a sliding window over the valid,
    SU-sorted fragments of each side -> explain_mass_with_table(diff,
    thr = tolerance*(obs_start + obs_end)) via calculate_explanations.
These functions emit the same queries as flat float64 arrays so the GPU
engine answers a whole batch in one call.  (The dataframe bookkeeping around
them -- intensity / sequence-mass filters, singletons -- is restated only as far
as it selects which fragments feed the window.)
"""
from dataclasses import dataclass

import numpy as np

from .masses import EXPLANATION_MASSES, PHOSPHATE_LINK_MASS

MAX_VARIANCE = 1  # fragment_classification.py:8


def max_nucleotide_weight(explanation_masses=EXPLANATION_MASSES):
    """prediction.py:287-290."""
    return max(explanation_masses.get_column("monoisotopic_mass").to_list()) + PHOSPHATE_LINK_MASS


@dataclass
class ClassifyQueries:
    su_mass: np.ndarray       # [n_obs * n_breakages]
    threshold: np.ndarray     # tolerance * observed mass
    observed: np.ndarray
    fragment: np.ndarray      # index of the observed mass
    breakage: list            # breakage label per query (first name of the dict entry)


def classify_queries(observed, breakage_dict, precision, tolerance):
    """fragment_classification.py:39-67: one is_valid query per (breakage,
    fragment), breakage-major like the reference's pl.concat."""
    obs = np.asarray(observed, dtype=np.float64)
    su, thr, frag, brk, ob = [], [], [], [], []
    for weight, names in breakage_dict.items():
        su.append(obs - (weight * precision))
        thr.append(tolerance * obs)
        frag.append(np.arange(len(obs)))
        ob.append(obs)
        brk += [names[0]] * len(obs)
    cat = (lambda x: np.concatenate(x)) if len(obs) else (lambda x: np.zeros(0))
    return ClassifyQueries(cat(su), cat(thr), cat(ob), cat(frag).astype(np.int64) if len(obs) else np.zeros(0, np.int64),
                           brk)


def sliding_window_pairs(su_sorted, max_weight):
    """prediction.py:293-328 restated: the (start, end) index pairs whose mass
    difference the reference explains, in the reference's order."""
    pairs = []
    n = len(su_sorted)
    start, end = 0, 1
    while end < n:
        if (end - start) <= 0:
            end += 1
            continue
        diff = su_sorted[end] - su_sorted[start]
        if diff > max_weight:
            start += 1
            end = start + 1
            continue
        pairs.append((start, end))
        if end == n - 1:
            start += 1
        else:
            end += 1
    return pairs


def window_pairs(su_sorted, max_weight):
    """sliding_window_pairs as index arrays, by the library's host-native
    producer (sst_window_pairs)."""
    from ._native import window_pairs as _wp

    return _wp(su_sorted, [0, len(su_sorted)], max_weight)


def diff_queries(su_sorted, obs_sorted, tolerance, max_weight):
    """Adjacent-difference explain queries of one side (prediction.py:286-329):
    diff = su[end] - su[start], threshold = tolerance*(obs[start]+obs[end])
    (calculate_error_threshold, common.py:37-44, l1_norm)."""
    pairs = sliding_window_pairs(su_sorted, max_weight)
    if not pairs:
        return np.zeros(0), np.zeros(0), pairs
    s = np.array([p[0] for p in pairs])
    e = np.array([p[1] for p in pairs])
    su = np.asarray(su_sorted, dtype=np.float64)
    ob = np.asarray(obs_sorted, dtype=np.float64)
    return su[e] - su[s], tolerance * (ob[s] + ob[e]), pairs


def side_fragments(su, obs, breakage, side):
    """Fragments of one side sorted by SU mass (classify_fragments sorts by
    standard_unit_mass, :86; prediction.py:265-268 filters by side)."""
    keep = np.array([side in b for b in breakage], dtype=bool)
    su_s, ob_s = np.asarray(su)[keep], np.asarray(obs)[keep]
    order = np.argsort(su_s, kind="stable")
    return su_s[order], ob_s[order]
