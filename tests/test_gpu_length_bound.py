"""GPU parity of compute_sequence_length_bound (mass_table.py:343-487):
the reference's golden answers, the CPU oracle on seeded random sequences
(full, reduced and canonical alphabets), and the layered fast path against
the exact first-visit replay on the same queries."""
import numpy as np
import pytest

import _oracle as oracle
from conftest import load_golden
from spectrseqtools_amd import _native

pytestmark = pytest.mark.gpu

CANON = (305042, 306026, 329053, 345048)


@pytest.fixture(scope="module")
def engine():
    return _native.get_engine(0)


@pytest.fixture(scope="module")
def alphabet_rows():
    g = load_golden("alphabet.json")
    return sorted({r["tolerated_integer_masses"] for r in g["rows"]} | {0})


_DEV = {}
_HOST = {}


def _host(ms):
    if tuple(ms) not in _HOST:
        _HOST[tuple(ms)] = oracle.build_table(ms, max(ms) * 35, 32)
    return _HOST[tuple(ms)]


def dev_for(engine, masses):
    key = tuple(masses)
    if key not in _DEV:
        _DEV[key] = _native.DeviceTable.build(list(masses), max(masses) * 35, 32, engine=engine)
    return _DEV[key]


def test_golden_length_bounds(engine, golden_cases):
    ctxs = golden_cases["contexts"]
    cases = [c for c in golden_cases["cases"] if c["fn"] == "length_bound"]
    assert cases
    for c in cases:
        ctx = ctxs[c["ctx"]]
        dev = dev_for(engine, ctx["masses"])
        dev.set_budgets(ctx["is_mod"], ctx["caps"])
        su = c.get("su_mass", ctx["su_mass"])
        obs = c.get("obs_mass", ctx["obs_mass"])
        A = round(ctx["mod_rate"] * ctx["max_len"])
        for exact_only, replay in ((False, False), (True, False), (True, True)):
            got, st = dev.length_bound([su], [obs], ctx["tolerance"], ctx["precision"], ctx["max_len"], A, c["dir"],
                                       exact_only=exact_only, replay=replay)
            assert int(st[0]) == 0 and int(got[0]) == c["result"], (c, exact_only, replay)


def _alph(ms, max_len, rate=0.5):
    is_mod = [m not in CANON and m != 0 for m in ms]
    caps = [round(max_len * (rate if md else (1.0 if m else 0.0))) for m, md in zip(ms, is_mod)]
    return is_mod, caps


def _check(engine, ms, max_len, su, obs, tol=1e-5):
    dev = dev_for(engine, ms)
    host = _host(ms)
    is_mod, caps = _alph(ms, max_len)
    dev.set_budgets(is_mod, caps)
    alph = oracle.Alphabet(ms, is_mod, caps)
    A = round(0.5 * max_len)
    for d in ("lower", "upper"):
        got, st = dev.length_bound(su, obs, tol, 1e-3, max_len, A, d)
        got_x, st_x = dev.length_bound(su, obs, tol, 1e-3, max_len, A, d, exact_only=True)  # the frontier
        got_r, st_r = dev.length_bound(su, obs, tol, 1e-3, max_len, A, d, exact_only=True, replay=True)
        assert (st == 0).all() and (st_x == 0).all() and (st_r == 0).all()
        for i in range(len(su)):
            want = oracle.length_bound(host, 32, alph, su[i], obs[i], tol, max_len, A, d)
            assert int(got[i]) == want, (d, i, su[i], max_len)
            assert int(got_x[i]) == want, ("frontier", d, i, su[i], max_len)
            assert int(got_r[i]) == want, ("replay", d, i, su[i], max_len)


@pytest.mark.parametrize("max_len", [8, 14, 20])
def test_canonical_vs_oracle(engine, max_len):
    rng = np.random.default_rng(max_len)
    ms = [0, *CANON]
    su = np.array([rng.choice(CANON, rng.integers(1, max_len + 1)).sum() * 1e-3 for _ in range(24)])
    obs = su + rng.normal(0, 0.002, len(su))
    _check(engine, ms, max_len, su, obs)


def test_reduced_alphabet_with_mods_vs_oracle(engine, alphabet_rows):
    # canonical + a handful of modifications: budgets bind, first visits matter
    rng = np.random.default_rng(7)
    mods = [m for m in alphabet_rows if m not in CANON and m != 0]
    ms = sorted({0, *CANON, *rng.choice(mods, 6, replace=False).tolist()})
    for max_len in (4, 7, 10):
        su = np.array([rng.choice(ms[1:], rng.integers(1, max_len + 1)).sum() * 1e-3 for _ in range(12)])
        _check(engine, ms, max_len, su, su)


def test_full_alphabet_short_vs_oracle(engine, alphabet_rows):
    rng = np.random.default_rng(11)
    ms = alphabet_rows
    for max_len in (3, 5):
        su = np.array([rng.choice(ms[1:], rng.integers(1, max_len + 1)).sum() * 1e-3 for _ in range(8)])
        _check(engine, ms, max_len, su, su * (1 + 1e-6))


def test_length_bound_errors(engine, alphabet_rows):
    ms = alphabet_rows
    dev = dev_for(engine, ms)
    is_mod, caps = _alph(ms, 4)
    dev.set_budgets(is_mod, caps)
    limit = dev.n_cols * 32
    got, st = dev.length_bound([limit * 1e-3 + 1.0, 500.0, -3.0], [limit * 1e-3 + 1.0, -1e9, -3.0], 1e-5, 1e-3, 4, 2,
                               "lower")
    assert int(st[0]) == _native.SST_OUT_OF_TABLE
    assert int(st[1]) == _native.SST_LB_EMPTY_WINDOW
    assert int(st[2]) == 0 and int(got[2]) == 1  # only negative values: default -> 1


def test_full_alphabet_6mer_vs_oracle(engine, alphabet_rows):
    # whole 6-mers over the full alphabet: budgets bind (A = 3 < 6 items), so
    # the exact replay's first-visit classification is exercised at depth
    rng = np.random.default_rng(6)
    ms = alphabet_rows
    su = np.array([rng.choice(ms[1:], 6).sum() * 1e-3 for _ in range(2)])
    _check(engine, ms, 6, su, su)


def test_last_word_windows_go_to_the_replay(engine):
    """A window in the table's last packed word: the reference's last-column
    mask (mass_table.py:246) may clear pair bits the closure has, so the
    frontier reports SST_ABORTED there and the batch call answers those
    windows by the replay (the table's real bits); equal to the oracle."""
    ms = [0, 1100, 1500, 2200]
    dev = dev_for(engine, ms)
    host = _host(ms)
    is_mod, caps = [False, False, True, True], [0, 20, 2, 1]
    dev.set_budgets(is_mod, caps)
    alph = oracle.Alphabet(ms, is_mod, caps)
    limit = dev.n_cols * 32
    su = np.array([(limit - 20) * 1e-3, (limit - 40) * 1e-3, (limit - 5) * 1e-3, 30.0, 21.5])
    obs = np.full(len(su), 0.5)  # windows of +-5 masses
    for d in ("lower", "upper"):
        got, st = dev.length_bound(su, obs, 1e-5, 1e-3, 40, 3, d, exact_only=True)
        for i in range(len(su)):
            want = oracle.length_bound(host, 32, alph, su[i], obs[i], 1e-5, 40, 3, d)
            if want is None:
                assert int(st[i]) == _native.SST_OUT_OF_TABLE, (d, i)
            else:
                assert int(st[i]) == 0 and int(got[i]) == want, (d, i, int(st[i]), int(got[i]), want)
