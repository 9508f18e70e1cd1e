"""Explanation wrapper and error model.

Mirror of the hot-path half of spectrseqtools/common.py (reference v0.1.2,
:12-65).  The RAW-file iterator (:68-93, ms_deisotope/mono) is out of scope.
"""
import re
from typing import List

from .mass_explanation import explain_mass_with_table, explain_masses
from .mass_table import DynamicProgrammingTable

ERROR_METHOD = "l1_norm"
_NUCLEOSIDE_RE = re.compile(r"\d*[ACGU]")


def parse_nucleosides(sequence: str):
    return _NUCLEOSIDE_RE.findall(sequence)


class Explanation:
    def __init__(self, *nucleosides):
        self.nucleosides = tuple(sorted(nucleosides))

    def __iter__(self):
        yield from self.nucleosides

    def __len__(self):
        return len(self.nucleosides)

    def __repr__(self):
        return f"{{{','.join(self.nucleosides)}}}"

    def __eq__(self, other):
        return self.nucleosides == other

    __hash__ = None  # as the reference (defines __eq__ without __hash__)


def calculate_error_threshold(mass1: float, mass2: float, threshold: float) -> float:
    match ERROR_METHOD:
        case "l1_norm":
            return threshold * (mass1 + mass2)
        case "l2_norm":
            return threshold * ((mass1 ** 2 + mass2 ** 2) ** 0.5)
        case _:
            raise NotImplementedError("This error method is not implemented.")


def _wrap(explanation_set):
    if explanation_set is None:
        return None
    explanation_list = list(explanation_set)
    return [Explanation(*explanation_list[i]) for i in range(len(explanation_list))]


def calculate_explanations(diff: float, threshold: float, dp_table: DynamicProgrammingTable) -> List[Explanation]:
    """common.py:47-65."""
    explanation_list = explain_mass_with_table(
        diff,
        dp_table=dp_table,
        max_modifications=round(dp_table.seq.modification_rate * dp_table.seq.max_len),
        threshold=threshold,
    ).explanations
    return _wrap(explanation_list)


def calculate_explanations_batch(diffs, thresholds, dp_table: DynamicProgrammingTable):
    """calculate_explanations over many (diff, threshold) pairs in one engine call."""
    res = explain_masses(diffs, dp_table,
                         max_modifications=round(dp_table.seq.modification_rate * dp_table.seq.max_len),
                         thresholds=thresholds)
    return [_wrap(r.explanations) for r in res]
