"""Turn the golden fixtures' contexts into oracle / engine inputs (tests only)."""
import hashlib
import math

import numpy as np

import _oracle as oracle

_TABLES = {}


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def ctx_table(ctx):
    """Oracle-built packed table of a golden context, pinned by the context's
    reference SHA-256."""
    key = tuple(ctx["masses"])
    if key not in _TABLES:
        t = oracle.build_table(ctx["masses"], max(ctx["masses"]) * 35, 32)
        assert sha(t) == ctx["table_sha256"], ctx["id"]
        _TABLES[key] = t
    return _TABLES[key]


def ctx_alphabet(ctx):
    return oracle.Alphabet(ctx["masses"], ctx["is_mod"], ctx["caps"])


def budget(a):
    return math.inf if a == "inf" else a


def expected_status(case):
    """golden case -> (status code as the engine reports it, sorted row tuples)."""
    from spectrseqtools_amd import _native

    if case["status"] == "raise":
        return _native.SST_OUT_OF_TABLE, None
    if case["status"] == "none":
        return _native.SST_NONE, []
    rows = sorted(tuple(r) for r in case["rows"])
    return (_native.SST_SOME if rows else _native.SST_EMPTY), rows
