"""Pin the CPU oracle (oracle/sst_oracle.c) to the reference's own outputs
(tests/golden/, produced by running spectrseq/spectrseqtools unmodified; see
tests/golden/make_golden.py).  CPU only."""
import hashlib

import numpy as np
import pytest

import _oracle as oracle
from _golden_ctx import budget, ctx_alphabet, ctx_table, sha
from conftest import load_golden


def test_tiny_tables_verbatim(golden_tables):
    for tiny in golden_tables["tiny"]:
        t = oracle.build_table(tiny["masses"], tiny["max_mass"], tiny["compression"])
        assert list(t.shape) == tiny["shape"]
        assert t.tolist() == tiny["words"], (tiny["masses"], tiny["max_mass"], tiny["compression"])


def test_packed_tables_sha(golden_tables):
    for p in golden_tables["packed"]:
        t = oracle.build_table(p["masses"], p["max_mass"], 32)
        assert list(t.shape) == p["shape"]
        assert sha(t) == p["sha256"], p["what"]
        assert [int(np.bitwise_xor.reduce(t[r])) for r in range(t.shape[0])] == p["checksums_per_row"]


def _table_cases(golden_cases, fn):
    return [c for c in golden_cases["cases"] if c["fn"] == fn]


def test_explain_with_table_cases(golden_cases):
    ctxs = golden_cases["contexts"]
    n = 0
    for c in _table_cases(golden_cases, "table"):
        ctx = ctxs[c["ctx"]]
        st, sols, n_empty, _ = oracle.explain_table(ctx_table(ctx), 32, ctx_alphabet(ctx), c["mass"], c["threshold"],
                                                    ctx["tolerance"], budget(c["max_modifications"]),
                                                    with_memo=c["with_memo"])
        if c["status"] == "raise":
            assert st == -1, c
            continue
        if c["status"] == "none":
            assert st == 0 and not sols, c
            continue
        assert st == 1
        assert sorted(sols) == sorted(tuple(r) for r in c["rows"]), (c["tag"], c["mass"], c["max_modifications"])
        assert len(set(sols)) == len(sols)  # the reference's list has no duplicates either
        n += 1
    assert n > 1500


def test_memo_quirk_is_exercised(golden_cases):
    """Some golden queries differ between with_memo=True and False: the oracle
    must reproduce the memo-on semantics, not the budget-exact one."""
    ctxs = golden_cases["contexts"]
    differ = 0
    for c in _table_cases(golden_cases, "table"):
        if c["status"] != "set" or c["ctx"] not in ("full_L2", "full_L3"):
            continue
        ctx = ctxs[c["ctx"]]
        st, sols, _, _ = oracle.explain_table(ctx_table(ctx), 32, ctx_alphabet(ctx), c["mass"], c["threshold"],
                                              ctx["tolerance"], budget(c["max_modifications"]), with_memo=False)
        if sorted(sols) != sorted(tuple(r) for r in c["rows"]):
            differ += 1
    assert differ > 0


def test_recursion_cases(golden_cases):
    ctxs = golden_cases["contexts"]
    for c in _table_cases(golden_cases, "recursion"):
        ctx = ctxs[c["ctx"]]
        st, sols, _ = oracle.explain_recursion(ctx_alphabet(ctx), c["mass"], c["threshold"], ctx["tolerance"],
                                               budget(c["max_modifications"]))
        assert st == 1
        assert sorted(sols) == sorted(tuple(r) for r in c["rows"]), (c["ctx"], c["mass"])


def test_is_valid_cases(golden_cases):
    ctxs = golden_cases["contexts"]
    for c in _table_cases(golden_cases, "is_valid"):
        ctx = ctxs[c["ctx"]]
        r = oracle.is_valid(ctx_table(ctx), 32, c["mass"], c["threshold"], ctx["tolerance"])
        want = -1 if c["result"] == "raise" else int(c["result"])
        assert r == want, c


def test_length_bound_cases(golden_cases):
    ctxs = golden_cases["contexts"]
    cases = _table_cases(golden_cases, "length_bound")
    assert cases
    for c in cases:
        ctx = ctxs[c["ctx"]]
        su = c.get("su_mass", ctx["su_mass"])
        obs = c.get("obs_mass", ctx["obs_mass"])
        A = round(ctx["mod_rate"] * ctx["max_len"])
        got = oracle.length_bound(ctx_table(ctx), 32, ctx_alphabet(ctx), su, obs, ctx["tolerance"], ctx["max_len"], A,
                                  c["dir"])
        assert got == c["result"], c


def test_population_a7(golden_population):
    ctxs = golden_population["contexts"]
    by_ctx = {}
    for cid, m, t, v in golden_population["a7"]:
        by_ctx.setdefault(cid, []).append((m, t, v))
    for cid, rows in by_ctx.items():
        ctx = ctxs[cid]
        m = np.array([r[0] for r in rows])
        t = np.array([r[1] for r in rows])
        got = oracle.is_valid_batch(ctx_table(ctx), 32, m, t, ctx["tolerance"])
        assert got.tolist() == [int(r[2]) for r in rows], cid


def test_population_a8(golden_population):
    ctxs = golden_population["contexts"]
    for cid, m, t, A, rows in golden_population["a8"][::3]:
        ctx = ctxs[cid]
        st, sols, n_empty, _ = oracle.explain_table(ctx_table(ctx), 32, ctx_alphabet(ctx), m, t, ctx["tolerance"], A)
        if rows is None:
            assert st == 0, (cid, m)
        else:
            assert st == 1 and sorted(sols) == sorted(tuple(r) for r in rows), (cid, m)


def test_is_singleton_restatement_vs_reference():
    g = load_golden("singleton.json.gz")
    ctx = g["context"]
    q = np.array([[x[0], x[1]] for x in g["queries"]])
    want = np.array([x[2] for x in g["queries"]])
    got = oracle.is_singleton_batch(q[:, 0], q[:, 1], ctx["masses"], ctx["tolerance"], ctx["precision"])
    assert want.sum() > 1000 and np.array_equal(got, want)


def test_length_bound_reference_depth():
    """compute_sequence_length_bound at config 5's depth (length_cases.json.gz,
    tests/golden/make_length_golden.py: the reference's own call on 40 reduced
    alphabets it rebuilt itself, windows of 6..20 nucleotides, per-row rate
    profiles and max_modifications of 0..3 or round(0.5 L)): the oracle's
    rebuilt tables have the reference's SHA-256, and both directions equal the
    reference on every window (None: the reference raised).  Budgets bind:
    enough windows' bounds differ from the budget-free ones."""
    import concurrent.futures as cf

    g = load_golden("length_cases.json.gz")
    tabs = {}
    for ai, a in enumerate(g["alphabets"]):
        t = oracle.build_table(a["masses"], max(a["masses"]) * 35, 32)
        assert list(t.shape) == a["table_shape"] and sha(t) == a["table_sha256"], ai
        tabs[ai] = t
    cases = g["cases"]
    assert len(cases) >= 280 and sum(c["lower"] is None for c in cases) == len(g["alphabets"])
    assert sum(c["nucleotides"] >= 15 for c in cases) >= 20  # windows of 15..20 nucleotides

    def one(c, free=False):
        a = g["alphabets"][c["alpha"]]
        caps = [255] * len(c["caps"]) if free else c["caps"]
        alph = oracle.Alphabet(a["masses"], c["is_mod"], caps)
        return tuple(oracle.length_bound(tabs[c["alpha"]], 32, alph, c["su_mass"], c["obs_mass"], c["tolerance"],
                                         c["max_len"], 255 if free else c["max_modifications"], d)
                     for d in ("lower", "upper"))

    with cf.ThreadPoolExecutor(8) as ex:  # ctypes releases the GIL
        got = list(ex.map(one, cases))
    for c, (lo, up) in zip(cases, got):
        assert (lo, up) == (c["lower"], c["upper"]), (c["alpha"], c["su_mass"], lo, up, c["lower"], c["upper"])
    # budgets bind on these windows (the first 60 answered ones are enough to show it)
    live = [c for c in cases if c["lower"] is not None][:60]
    with cf.ThreadPoolExecutor(8) as ex:
        free = list(ex.map(lambda c: one(c, True), live))
    assert sum(f != (c["lower"], c["upper"]) for c, f in zip(live, free)) >= 20
