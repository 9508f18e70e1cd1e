"""GPU tests of sst_explain_alpha_batch_device: explain_mass_with_table on
per-query reduced alphabets, answered from the full table's rows with a row
mask (no table rebuild), against the CPU oracle on each alphabet's own
rebuilt table (set_up_bit_table over the kept rows, max_mass = max(kept) *
35, mass_table.py:94-121).  Whole masses of up to 10 items with binding
budgets (the exact memo replay), the fast path, with_memo=False, windows
reaching 0 and windows at the reduced table's extent."""
import numpy as np
import pytest

import _oracle as oracle
from conftest import load_golden
from spectrseqtools_amd import _native
from spectrseqtools_amd.pipeline import row_masks

pytestmark = pytest.mark.gpu
TOL, PREC = 1e-5, 1e-3
CANONICAL = (305042, 306026, 329053, 345048)
RATES = (0.02, 0.05, 0.1, 0.25, 0.5)


@pytest.fixture(scope="module")
def setup():
    g = load_golden("alphabet.json")
    rows = sorted({r["tolerated_integer_masses"] for r in g["rows"]} | {0})
    eng = _native.get_engine(0)
    dev = _native.DeviceTable.build(rows, max(rows) * 35, 32, engine=eng)
    rng = np.random.default_rng(71)
    max_len = 20
    is_mod = [m not in CANONICAL and m != 0 for m in rows]
    rate = [float(rng.choice(RATES)) if md else (1.0 if m else 0.0) for m, md in zip(rows, is_mod)]
    caps = [round(max_len * r) for r in rate]
    dev.set_budgets(is_mod, caps)
    return rows, dev, is_mod, caps


def _alphabets(rows, rng, n):
    canon = [i for i, m in enumerate(rows) if m in CANONICAL]
    mods = [i for i, m in enumerate(rows) if i > 0 and m not in CANONICAL]
    out = [sorted(canon)]
    for _ in range(n - 1):
        pick = rng.choice(mods, size=int(rng.integers(1, 16)), replace=False).tolist()
        out.append(sorted(set(canon + pick)))
    return out


def _queries(rows, alphas, rng, per, kmax):
    mass, thr, spec = [], [], []
    for g, a in enumerate(alphas):
        w = np.array([rows[r] for r in a])
        k = rng.integers(1, kmax + 1, per)
        m = np.array([w[rng.integers(0, len(w), kk)].sum() for kk in k]) * PREC + rng.normal(0, 0.003, per)
        lim = (max(w) * 35 + 32) // 32 * 32  # the reduced table's extent (words x 32)
        m = np.concatenate([m, rng.uniform(-0.02, 0.02, 4)])
        t = TOL * np.abs(m) * rng.uniform(0.3, 2.0, len(m)) + 1e-4
        # narrow windows past the extent (raise) and inside its last word
        m = np.concatenate([m, [(lim + 40) * PREC, (lim + 900) * PREC, (lim - 16) * PREC]])
        t = np.concatenate([t, [0.02, 0.5, 0.004]])
        mass.append(m)
        thr.append(t)
        spec.append(np.full(len(m), g, np.int32))
    return np.concatenate(mass), np.concatenate(thr), np.concatenate(spec)


def _check(rows, dev, is_mod, caps, alphas, mass, thr, spec, A, with_memo):
    masks = row_masks(np.array([[r in a for r in range(len(rows))] for a in alphas]))
    res = dev.explain_alpha(mass, thr, spec, masks, TOL, PREC, A, with_memo=with_memo)
    tabs = {}
    n = {"some": 0, "oot": 0, "aborted": 0, "empty": 0}
    for i in range(len(mass)):
        a = alphas[spec[i]]
        full = [0] + a
        ms = [rows[r] for r in full]
        lim = (max(ms) * 35 + 32) // 32 * 32
        whi = np.rint(mass[i] / PREC) + np.ceil(thr[i] / PREC)
        if whi >= 1 and lim - 32 <= whi < lim:  # the reduced table's last word: not modelled
            assert int(res.status[i]) == _native.SST_ABORTED, i
            n["aborted"] += 1
            continue
        if spec[i] not in tabs:
            tabs[spec[i]] = (oracle.build_table(ms, max(ms) * 35, 32),
                             oracle.Alphabet(ms, [is_mod[r] for r in full], [caps[r] for r in full]))
        tab, alph = tabs[spec[i]]
        st, sols, n_e, _ = oracle.explain_table(tab, 32, alph, mass[i], thr[i], TOL, int(A[i]), with_memo=with_memo)
        if st < 0:
            assert int(res.status[i]) == _native.SST_OUT_OF_TABLE, i
            n["oot"] += 1
            continue
        want = [tuple(full[x] for x in t) for t in sols]
        want_st = _native.SST_SOME if want else (_native.SST_EMPTY if n_e else _native.SST_NONE)
        assert int(res.status[i]) == want_st, (i, mass[i], thr[i], int(A[i]), a)
        assert res.candidates(i) == want, (i, mass[i], int(A[i]))  # the reference's list order
        n["some"] += want_st == _native.SST_SOME
        n["empty"] += want_st == _native.SST_EMPTY
    return n


def test_explain_alpha_exact_vs_rebuilt_tables(setup):
    """Binding budgets (A small against the masses' modification counts):
    the scan routes the windows to the exact memo replay."""
    rows, dev, is_mod, caps = setup
    rng = np.random.default_rng(72)
    alphas = _alphabets(rows, rng, 8)
    mass, thr, spec = _queries(rows, alphas, rng, 120, 10)
    A = rng.choice([0, 1, 2, 3, 5], len(mass))
    n = _check(rows, dev, is_mod, caps, alphas, mass, thr, spec, A, True)
    assert n["some"] > 200 and n["oot"] >= 16 and n["aborted"] >= 8 and n["empty"] > 0


def test_explain_alpha_fast_and_nomemo_vs_rebuilt_tables(setup):
    """Budgets that never bind (A = inf: the deep fast path) and
    with_memo=False (budgets carried along the path)."""
    rows, dev, is_mod, caps = setup
    rng = np.random.default_rng(73)
    alphas = _alphabets(rows, rng, 6)
    mass, thr, spec = _queries(rows, alphas, rng, 60, 6)
    for A, with_memo in ((np.full(len(mass), -1), True), (rng.choice([1, 2, 4], len(mass)), False)):
        n = _check(rows, dev, is_mod, caps, alphas, mass, thr, spec, A, with_memo)
        assert n["some"] > 100


def test_explain_alpha_full_mask_equals_plain_explain(setup):
    """With every row kept the masked pass answers exactly as the plain one."""
    rows, dev, is_mod, caps = setup
    rng = np.random.default_rng(74)
    ints = np.array(rows[1:])
    k = rng.integers(1, 5, 600)  # <= 4 items: at most a few hundred candidates per window on all 104 rows
    mass = np.array([ints[rng.integers(0, len(ints), kk)].sum() for kk in k]) * PREC + rng.normal(0, 0.003, 600)
    thr = 0.2 * TOL * mass
    A = rng.choice([1, 3, 10], len(mass))
    full = row_masks(np.array([[r > 0 for r in range(len(rows))]]))
    res = dev.explain_alpha(mass, thr, np.zeros(len(mass), np.int32), full, TOL, PREC, A)
    ref = dev.explain(mass, thr, TOL, PREC, A)
    assert np.array_equal(res.status, ref.status)
    for i in range(len(mass)):
        assert res.candidates(i) == ref.candidates(i), i


def test_length_bound_alpha_vs_rebuilt_tables(setup, direction="lower"):
    """compute_sequence_length_bound(dir="lower") after the skeleton's
    alphabet reduction (skeleton_building.py:212-224): sequence masses of
    5..14-mers over each alphabet's rows, A = round(0.5 max_len) with binding
    caps, on the masked full table against the oracle on the rebuilt table;
    "upper" is refused (the reference's upper bound sees the visits the mask
    adds)."""
    rows, dev, is_mod, caps = setup
    rng = np.random.default_rng(75)
    alphas = _alphabets(rows, rng, 6)
    masks = row_masks(np.array([[r in a for r in range(len(rows))] for a in alphas]))
    su, spec = [], []
    for g, a in enumerate(alphas):
        w = np.array([rows[r] for r in a])
        k = rng.integers(5, 15, 12)
        su.append(np.array([w[rng.integers(0, len(w), kk)].sum() for kk in k]) * PREC + rng.normal(0, 0.002, 12))
        spec.append(np.full(12, g, np.int32))
    su, spec = np.concatenate(su), np.concatenate(spec)
    obs = su + 912.303  # a START_END fragment's observed mass
    max_len, A = 20, 10
    out, st = dev.length_bound_alpha(su, obs, spec, masks, TOL, PREC, max_len, A, direction)
    n_ok = 0
    for i in range(len(su)):
        full = [0] + alphas[spec[i]]
        ms = [rows[r] for r in full]
        tab = oracle.build_table(ms, max(ms) * 35, 32)
        alph = oracle.Alphabet(ms, [is_mod[r] for r in full], [caps[r] for r in full])
        want = oracle.length_bound(tab, 32, alph, su[i], obs[i], TOL, max_len, A, direction)
        if want is None:
            assert int(st[i]) != 0, i
            continue
        assert int(st[i]) == 0 and int(out[i]) == want, (i, int(st[i]), int(out[i]), want)
        n_ok += 1
    assert n_ok >= 60
    with pytest.raises(_native.EngineError):  # "upper" needs the rebuilt table (include/sst.h)
        dev.length_bound_alpha(su, obs, spec, masks, TOL, PREC, max_len, A, "upper")


def test_explain_alpha_rootless_window_past_reduced_extent():
    """A window at or past the REDUCED table's extent raises in the reference
    (mass_explanation.py:133-138) whether or not any of its values is
    reachable; on a table without the pair list (an uploaded table: the
    bitset scan answers rootless windows itself) such a window must still be
    SST_OUT_OF_TABLE, as the oracle on the rebuilt table says."""
    eng = _native.get_engine(0)
    ms = [0, 1000, 1500, 2200]
    words = oracle.build_table(ms, max(ms) * 35, 32)
    dev = _native.DeviceTable.upload(ms, words, 32, engine=eng)
    dev.set_budgets([False, False, False, False], [0, 20, 20, 20])
    kept = [0, 1, 2]  # max(kept) * 35 = 52500 < the full table's 77000
    red = [ms[r] for r in kept]
    red_tab = oracle.build_table(red, max(red) * 35, 32)
    alph = oracle.Alphabet(red, [False] * 3, [0, 20, 20])
    masks = row_masks(np.array([[r in kept for r in range(len(ms))]]))
    # rootless (no sum of 1000/1500/2200 ends in ...01..03) in the reduced table's last word,
    # past its extent, and a reachable control below it
    mass = np.array([60.002, 52.530, 70.0015, 45.000, 52.499])
    thr = np.array([0.001, 0.0005, 0.0005, 0.001, 0.0004])
    res = dev.explain_alpha(mass, thr, np.zeros(len(mass), np.int32), masks, TOL, PREC, -1)
    n_oot = 0
    for i in range(len(mass)):
        st, sols, n_e, _ = oracle.explain_table(red_tab, 32, alph, mass[i], thr[i], TOL, -1)
        if st < 0:
            assert int(res.status[i]) == _native.SST_OUT_OF_TABLE, (i, int(res.status[i]))
            n_oot += 1
        else:
            want = [tuple(kept[x] for x in t) for t in sols]
            want_st = _native.SST_SOME if want else (_native.SST_EMPTY if n_e else _native.SST_NONE)
            assert int(res.status[i]) in (want_st, _native.SST_ABORTED), (i, int(res.status[i]), want_st)
            if int(res.status[i]) == want_st == _native.SST_SOME:
                assert res.candidates(i) == want
    assert n_oot >= 2


def test_explain_alpha_lens_vs_rebuilt_tables(setup):
    """Per-query budgets (sst_explain_alpha_lens_batch_device): every query
    with the caps round(L * rate) of its own max_len L and its own
    max_modifications, in one pass, against the oracle on its alphabet's
    rebuilt table with those budgets -- windows of many max_len values, as the
    skeleton walk's re-queries carry them."""
    rows, dev, is_mod, _ = setup
    rng = np.random.default_rng(76)
    alphas = _alphabets(rows, rng, 8)
    mass, thr, spec = _queries(rows, alphas, rng, 90, 10)
    rate = [float(rng.choice(RATES)) if md else (1.0 if m else 0.0) for m, md in zip(rows, is_mod)]
    lens = [2, 4, 7, 12, 20]
    caps_by_len = np.array([[round(L * r) for r in rate] for L in lens], np.int64)
    qlen = rng.integers(0, len(lens), len(mass))
    A = np.array([round(0.5 * lens[k]) if rng.random() < 0.7 else int(rng.integers(0, 4)) for k in qlen])
    masks = row_masks(np.array([[r in a for r in range(len(rows))] for a in alphas]))
    res = dev.explain_alpha_lens(mass, thr, spec, masks, qlen, caps_by_len, A, TOL, PREC)
    tabs = {}
    n_some = n_bind = 0
    for i in range(len(mass)):
        a = alphas[spec[i]]
        full = [0] + a
        ms = [rows[r] for r in full]
        lim = (max(ms) * 35 + 32) // 32 * 32
        whi = np.rint(mass[i] / PREC) + np.ceil(thr[i] / PREC)
        if whi >= 1 and lim - 32 <= whi < lim:
            assert int(res.status[i]) == _native.SST_ABORTED, i
            continue
        if spec[i] not in tabs:
            tabs[spec[i]] = oracle.build_table(ms, max(ms) * 35, 32)
        tab = tabs[spec[i]]
        caps = caps_by_len[qlen[i]]
        alph = oracle.Alphabet(ms, [is_mod[r] for r in full], [int(caps[r]) for r in full])
        st, sols, n_e, _ = oracle.explain_table(tab, 32, alph, mass[i], thr[i], TOL, int(A[i]))
        if st < 0:
            assert int(res.status[i]) == _native.SST_OUT_OF_TABLE, i
            continue
        want = [tuple(full[x] for x in t) for t in sols]
        want_st = _native.SST_SOME if want else (_native.SST_EMPTY if n_e else _native.SST_NONE)
        assert int(res.status[i]) == want_st, (i, mass[i], thr[i], int(A[i]), lens[qlen[i]])
        assert res.candidates(i) == want, (i, lens[qlen[i]])
        n_some += want_st == _native.SST_SOME
        free = oracle.Alphabet(ms, [is_mod[r] for r in full], [99] * len(full))
        n_bind += oracle.explain_table(tab, 32, free, mass[i], thr[i], TOL, 99)[1] != sols
    assert n_some > 150 and n_bind > 20
