"""The skeleton walk's emulation of CPython set iteration order and tuple
hashing (spectrseqtools_amd/csrc/sst_pyset.h) against the running
interpreter (CPU suite: host code of libsstgpu.so, no device).

SkeletonBuilder's output depends on that order (skeleton_building.py:442-482
iterates a set of positions and groups explanation lists -- the iteration
order of a set of name tuples, mass_explanation.py:287-320 -- by length), so
the device walk reproduces it from the elements' hashes."""
import random

import pytest

from spectrseqtools_amd import _native
from spectrseqtools_amd.masses import EXPLANATION_MASSES


def test_tuple_hash_matches_interpreter():
    names = EXPLANATION_MASSES.get_column("nucleoside").to_list()
    rng = random.Random(5)
    for _ in range(3000):
        t = tuple(rng.choice(names) for _ in range(rng.randint(0, 12)))
        assert _native.py_tuple_hash([hash(x) for x in t]) == hash(t), t
    for t in [(), (0,), (-1,), (1, 2, 3), (-2, 2 ** 61, -(2 ** 62))]:
        assert _native.py_tuple_hash([hash(x) for x in t]) == hash(t), t


@pytest.mark.parametrize("kind", ["ints", "small_ints", "name_tuples"])
def test_set_order_matches_interpreter(kind):
    names = EXPLANATION_MASSES.get_column("nucleoside").to_list()
    rng = random.Random({"ints": 1, "small_ints": 2, "name_tuples": 3}[kind])
    for trial in range(2500):
        n = rng.choice([1, 2, 3, 4, 5, 6, 8, 12, 18, 19, 20, 40, 76, 77, 80, 200, 400])
        if kind == "ints":
            elems = [rng.randint(-50, 10 ** 6) for _ in range(n)]
        elif kind == "small_ints":  # the walk's positions: p + len(explanation) <= max_len
            elems = [rng.randint(0, 160) for _ in range(n)]
        else:
            elems = [tuple(sorted((rng.choice(names) for _ in range(rng.randint(1, 6))), key=names.index))
                     for _ in range(n)]
        ids = {}
        keys = [ids.setdefault(e, len(ids)) for e in elems]  # equal elements share a key (re-adds are no-ops)
        s = set()
        for e in elems:
            s.add(e)
        want = [ids[e] for e in s]
        got = _native.pyset_order(keys, [hash(e) for e in elems])
        assert got == want, (kind, trial, elems)


def test_set_update_and_literal_order():
    """The walk's sets are built as the reference builds them: {0}, then
    set() + update(generator) (skeleton_building.py:126, 448-481)."""
    rng = random.Random(9)
    for _ in range(500):
        vals = [rng.randint(0, 40) for _ in range(rng.randint(1, 30))]
        s = set()
        s.update(v for v in vals)
        ids = {}
        keys = [ids.setdefault(v, len(ids)) for v in vals]
        assert _native.pyset_order(keys, vals) == [ids[v] for v in s]
