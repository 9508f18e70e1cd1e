"""fragment_classification.py hot-path functions on the GPU engine.

Only the per-fragment predicates that classify_fragments maps over every
row (:52-82) are here; the polars frame plumbing around them is the batched
producer in producers.py.
"""
import numpy as np

from . import _native
from .mass_table import DynamicProgrammingTable


def is_singleton(mass, integer_masses, dp_table: DynamicProgrammingTable, threshold=None) -> bool:
    """fragment_classification.py:104-119: some value of the quantised window
    (target = round(mass / precision), threshold default tolerance * mass) is one
    of integer_masses."""
    return bool(is_singletons([mass], integer_masses, dp_table, None if threshold is None else [threshold])[0])


def is_singletons(masses, integer_masses, dp_table: DynamicProgrammingTable, thresholds=None):
    """Batched is_singleton: bool per mass (one engine call)."""
    eng = dp_table.device_table.engine
    out = eng.is_singleton(integer_masses, masses, thresholds, dp_table.tolerance, dp_table.precision)
    return out.astype(bool)


__all__ = ["is_singleton", "is_singletons", "_native"]
