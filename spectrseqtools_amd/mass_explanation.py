"""Mass explanation queries, answered by the GPU engine.

Mirror of spectrseqtools/mass_explanation.py (reference v0.1.2) with the same
signatures and return/raise behaviour, plus batched entry points
(explain_masses, is_valid_masses) that cross the host/device boundary once per
batch.  The per-peak search itself runs in libsstgpu.so; this module only
defaults arguments and expands integer masses to nucleoside names
(convert_nucleotide_masses_to_names, :287-320).
"""
import math
from dataclasses import dataclass
from itertools import chain, combinations_with_replacement, product
from typing import List, Set, Tuple

import numpy as np

from . import _native
from .mass_table import DynamicProgrammingTable
from .masses import EXPLANATION_MASSES, UNMODIFIED_BASES


@dataclass
class MassExplanations:
    explanations: Set[Tuple[str]]


def _names_by_mass(frame):
    out = {}
    for m, n in zip(frame.get_column("tolerated_integer_masses").to_list(), frame.get_column("nucleoside").to_list()):
        out.setdefault(m, []).append(n)
    return out


MASS_NAMES = _names_by_mass(EXPLANATION_MASSES)  # mass_explanation.py:17-27
IS_MOD = {m: any(b not in UNMODIFIED_BASES for b in names) for m, names in MASS_NAMES.items()}  # :29-42


def _check_finite(mass):
    # int(round(nan)) / int(round(inf)) raise in the reference (:51, :107)
    if isinstance(mass, float) or isinstance(mass, np.floating):
        if math.isnan(mass):
            raise ValueError("cannot convert float NaN to integer")
        if math.isinf(mass):
            raise OverflowError("cannot convert float infinity to integer")


def _not_in_table(value):
    """The reference's out-of-table message (mass_explanation.py:68-72,
    :134-138; mass_table.py:383-387)."""
    return f"The value {value} is not in the DP table. Extend its size if you want to compute larger masses."


def _table_limit(dp_table):
    return dp_table.device_table.n_cols * dp_table.compression_per_cell


def first_value_beyond(mass, threshold, dp_table, tolerance_mass=None):
    """The `value` the reference's raise formats: its window loop runs
    ascending over [target - thr, target + thr] (mass_explanation.py:110-114,
    :189-192), and a DFS only moves to smaller masses, so the first root that
    meets a mass beyond the table is the first window value >= the table end
    (n_cols * compression).  tolerance_mass: the mass the default threshold
    scales (the length bound passes obs_mass, mass_table.py:357-359)."""
    target = int(round(mass / dp_table.precision, 0))
    if threshold is None:
        threshold = dp_table.tolerance * (mass if tolerance_mass is None else tolerance_mass)
    thr = int(np.ceil(threshold / dp_table.precision))
    return max(target - thr, _table_limit(dp_table))


def is_valid_mass(mass: float, dp_table: DynamicProgrammingTable, threshold: float = None) -> bool:
    """mass_explanation.py:45-89."""
    _check_finite(mass)
    r = is_valid_masses([mass], dp_table, None if threshold is None else [threshold], errors="status")[0]
    if r < 0:
        raise NotImplementedError(_not_in_table(first_value_beyond(mass, threshold, dp_table)))
    return bool(r)


def is_valid_masses(masses, dp_table: DynamicProgrammingTable, thresholds=None, errors="raise"):
    """Batched is_valid_mass.  thresholds: absolute (Da) per mass or None for
    the reference default tolerance*mass.  errors="raise" raises
    NotImplementedError if any mass falls out of the table (like the
    reference); errors="status" returns int8 {1, 0, -1} instead of bools."""
    masses = np.ascontiguousarray(masses, dtype=np.float64)
    if thresholds is not None:
        thresholds = np.ascontiguousarray(thresholds, dtype=np.float64)
    out = dp_table.device_table.is_valid(masses, thresholds, dp_table.tolerance, dp_table.precision)
    if errors == "status":
        return out
    bad = np.nonzero(out < 0)[0]
    if len(bad):
        k = bad[0]
        thr = None if thresholds is None else float(thresholds[k])
        raise NotImplementedError(_not_in_table(first_value_beyond(float(masses[k]), thr, dp_table)))
    return out.astype(bool)


def explain_mass_with_table(mass: float, dp_table: DynamicProgrammingTable, max_modifications=np.inf,
                            compression_rate=None, threshold=None, with_memo=True) -> MassExplanations:
    """mass_explanation.py:92-203: all multisets of the table's nucleotide masses
    summing to a value in the ppm window, with the reference's memo semantics."""
    _check_finite(mass)
    if compression_rate is not None and compression_rate != dp_table.compression_per_cell:
        if compression_rate == 1:
            raise TypeError("'DynamicProgrammingTable' object is not subscriptable")
        raise ValueError("compression_rate must match the table's compression_per_cell")
    return explain_masses([mass], dp_table, max_modifications=max_modifications,
                          thresholds=None if threshold is None else [threshold], with_memo=with_memo)[0]


def explain_masses(masses, dp_table: DynamicProgrammingTable, max_modifications=np.inf, thresholds=None,
                   with_memo=True, cap_per_query=2 ** 32, errors="raise"):
    """Batched explain_mass_with_table: one engine call for all masses.

    max_modifications: scalar (np.inf default) or one budget per mass.
    Returns a list of MassExplanations.  A query that the reference would
    raise on (window beyond the table) raises the reference's
    NotImplementedError, naming the same window value (errors="raise"), or
    yields None in the list (errors="none").  Queries with
    more than cap_per_query candidates raise OverflowError."""
    res = explain_masses_raw(masses, dp_table, max_modifications, thresholds, with_memo, cap_per_query)
    row_mass = [m.mass for m in dp_table.masses]
    out = []
    for i in range(res.n):
        st = int(res.status[i])
        if st == _native.SST_OUT_OF_TABLE:
            if errors == "raise":
                thr = None if thresholds is None else float(np.asarray(thresholds, dtype=np.float64)[i])
                raise NotImplementedError(_not_in_table(first_value_beyond(float(masses[i]), thr, dp_table)))
            out.append(None)
            continue
        if st in (_native.SST_OVERFLOW, _native.SST_ABORTED):
            raise OverflowError(f"query {i}: {int(res.count[i])} candidate compositions exceed cap_per_query")
        if st == _native.SST_NONE:
            out.append(MassExplanations(None))
        elif st == _native.SST_EMPTY:
            out.append(MassExplanations(set()))
        else:
            sols = [[row_mass[r] for r in c] for c in res.candidates(i)]
            out.append(convert_nucleotide_masses_to_names(sols))
    return out


def explain_masses_raw(masses, dp_table, max_modifications=np.inf, thresholds=None, with_memo=True,
                       cap_per_query=2 ** 32):
    """Engine result (status / count / offset / row-index payload) without
    name expansion."""
    masses = np.ascontiguousarray(masses, dtype=np.float64)
    for m in masses[~np.isfinite(masses)]:
        _check_finite(float(m))
    if thresholds is not None:
        thresholds = np.ascontiguousarray(thresholds, dtype=np.float64)
    return dp_table.device_table.explain(masses, thresholds, dp_table.tolerance, dp_table.precision,
                                         max_modifications, with_memo=with_memo, cap=cap_per_query)


def explain_mass_with_recursion(mass: float, dp_table: DynamicProgrammingTable, max_modifications=np.inf,
                                threshold=None) -> MassExplanations:
    """mass_explanation.py:206-284: the table-free enumerator (base case
    |remaining| <= threshold at every level, first-visit memo), on the GPU."""
    _check_finite(mass)
    return explain_masses_with_recursion([mass], dp_table, max_modifications,
                                         None if threshold is None else [threshold])[0]


def explain_masses_with_recursion(masses, dp_table: DynamicProgrammingTable, max_modifications=np.inf,
                                  thresholds=None, cap_per_query=2 ** 32):
    """Batched explain_mass_with_recursion (one engine call)."""
    masses = np.ascontiguousarray(masses, dtype=np.float64)
    for m in masses[~np.isfinite(masses)]:
        _check_finite(float(m))
    if thresholds is not None:
        thresholds = np.ascontiguousarray(thresholds, dtype=np.float64)
    # the reference compares used_mods_all > max_modifications: a fractional
    # budget acts floored, a negative one rejects the root call ([] -> None)
    def floored(x):
        return np.inf if not np.isfinite(x) else float(np.floor(max(x, 0.0)))

    if np.ndim(max_modifications) == 0:
        negative = np.full(masses.shape, float(max_modifications) < 0)
        engine_mods = floored(float(max_modifications))
    else:
        negative = np.asarray(max_modifications, dtype=np.float64) < 0
        engine_mods = [floored(float(x)) for x in max_modifications]
    res = dp_table.device_table.explain_recursion(masses, thresholds, dp_table.tolerance, dp_table.precision,
                                                  engine_mods, cap=cap_per_query)
    row_mass = [m.mass for m in dp_table.masses]
    out = []
    for i in range(res.n):
        st = int(res.status[i])
        if negative[i]:
            out.append(MassExplanations(None))
        elif st in (_native.SST_OVERFLOW, _native.SST_ABORTED):
            raise OverflowError(f"query {i}: recursion enumeration exceeds the engine's caps (status {st})")
        elif st == _native.SST_NONE:
            out.append(MassExplanations(None))
        elif st == _native.SST_EMPTY:
            out.append(MassExplanations(set()))
        else:
            out.append(convert_nucleotide_masses_to_names([[row_mass[r] for r in c] for c in res.candidates(i)]))
    return out


def convert_nucleotide_masses_to_names(solutions: List[List[int]]) -> MassExplanations:
    """mass_explanation.py:287-320 (host-side name expansion)."""
    solution_names = set()
    if len(solutions) == 0:
        return MassExplanations(None)
    for solution in solutions:
        if len(solution) == 0:
            continue
        distinct = [solution[idx] for idx in range(len(solution)) if idx == 0 or solution[idx - 1] != solution[idx]]
        solution_names.update(
            tuple(chain.from_iterable(entry))
            for entry in product(*[list(combinations_with_replacement(MASS_NAMES[m], solution.count(m)))
                                   for m in distinct])
        )
    return MassExplanations(solution_names)
