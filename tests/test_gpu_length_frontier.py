"""GPU parity of config 5's stage-5 engines against the CPU oracle on each
skeleton alphabet's REBUILT table (set_up_bit_table over the kept rows,
max_mass = max(kept) * 35, mass_table.py:94-121, skeleton_building.py:315-336):
compute_sequence_length_bound (mass_table.py:343-487) in both directions for
~200 synthetic spectra of 5..20 nucleotides, per-spectrum max_len, random
modification rates (caps round(L * rate)) and max_modifications from 0 up
to round(0.5 L), so that budgets bind.

  * the first-visit frontier (sst_length_bounds_frontier_device, what
    pipeline_device.length_device runs): alphabets of 4..104 kept rows, so
    that first-visit keys of 64, 128 and 256 bits all run; then again in a
    workspace too small for the batch (chunks split and rerun, counted) and
    in one too small for the heaviest spectra (those report SST_ABORTED,
    every other spectrum unchanged);
  * the round-4 DFS replay (sst_length_bounds_reach_device) on the same
    spectra with a small soft node budget (the heavy second pass runs) and a
    small first memo (memo retries run), fused (<= 64 kept rows) and unfused.
"""
import concurrent.futures as cf

import numpy as np
import pytest

import _oracle as oracle
from conftest import load_golden
from spectrseqtools_amd import _native

pytestmark = pytest.mark.gpu
TOL, PREC = 1e-5, 1e-3
CANONICAL = (305042, 306026, 329053, 345048)
RATES = (0.02, 0.05, 0.1, 0.25, 0.5)


@pytest.fixture(scope="module")
def setup():
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE

    eng = _native.get_engine(0)
    seq = SequenceInformation(max_len=20, su_mass=2000.0, obs_mass=2000.0, modification_rate=0.5)
    dp = DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=MATCHING_THRESHOLD,
                                 precision=TOLERANCE, seq=seq, engine=eng)
    rows = [m.mass for m in dp.masses]
    g = load_golden("alphabet.json")
    assert rows == sorted({r["tolerated_integer_masses"] for r in g["rows"]} | {0})
    rng = np.random.default_rng(2025)
    n_rows = len(rows)
    # per max_len budgets: caps round(L * rate_r) with random per-row rates,
    # max_modifications drawn per L from {0, 1, 2, 3, round(0.5 L)}
    rate = np.array([0.0] + [float(rng.choice(RATES)) if m.is_modification else 1.0 for m in dp.masses[1:]])
    caps_len = np.zeros((21, _native.MAX_ROWS), np.int32)
    for L in range(21):
        caps_len[L, :n_rows] = [round(L * r) for r in rate]
    a0_len = np.array([int(rng.choice([0, 1, 2, 3, round(0.5 * L)])) for L in range(21)], np.int32)
    return dp, rows, caps_len, a0_len


def _spectra(rows, dp, rng):
    canon = [i for i, m in enumerate(rows) if m in CANONICAL]
    mods = [i for i in range(1, len(rows)) if rows[i] not in CANONICAL]
    plan = [(0, 4, 10, 20)] * 40 + [(1, 8, 10, 20)] * 60 + [(9, 16, 10, 16)] * 60 + [(40, 60, 7, 9)] * 24 + \
        [(100, 100, 5, 6)] * 16
    alphas, su, ob, ml = [], [], [], []
    for lo_m, hi_m, lo_k, hi_k in plan:
        nm = int(rng.integers(lo_m, hi_m + 1))
        a = sorted(set(canon + rng.choice(mods, size=min(nm, len(mods)), replace=False).tolist()))
        w = np.array([rows[r] for r in a])
        k = int(rng.integers(lo_k, hi_k + 1))
        s = float(w[rng.integers(0, len(w), k)].sum()) * PREC + rng.normal(0, 0.002)
        alphas.append(a)
        su.append(s)
        ob.append(s + 912.303)  # a START_END fragment's observed mass
        ml.append(int(np.clip(k + rng.integers(-2, 3), 3, 20)))
    masks = np.zeros((len(alphas), 2), np.uint64)
    for g, a in enumerate(alphas):
        for r in a:
            masks[g, r >> 6] |= np.uint64(1) << np.uint64(r & 63)
    return alphas, masks, np.array(su), np.array(ob), np.array(ml)


def _oracle_bounds(rows, dp, caps_len, a0_len, alphas, su, ob, ml):
    def one(g):
        full = [0] + alphas[g]
        ms = [rows[r] for r in full]
        L = int(ml[g])
        tab = oracle.build_table(ms, max(ms) * 35, 32)
        alph = oracle.Alphabet(ms, [dp.masses[r].is_modification for r in full], [int(caps_len[L, r]) for r in full])
        lo, n_lo = oracle.length_bound_memo(tab, 32, alph, su[g], ob[g], TOL, L, int(a0_len[L]), "lower")
        up, n_up = oracle.length_bound_memo(tab, 32, alph, su[g], ob[g], TOL, L, int(a0_len[L]), "upper")
        assert n_lo == n_up  # the visits do not depend on the direction
        return lo, up, n_lo

    with cf.ThreadPoolExecutor(16) as ex:  # ctypes releases the GIL: the oracle calls run in parallel
        return list(ex.map(one, range(len(alphas))))


@pytest.fixture(scope="module")
def cases(setup):
    dp, rows, caps_len, a0_len = setup
    rng = np.random.default_rng(77)
    alphas, masks, su, ob, ml = _spectra(rows, dp, rng)
    want = _oracle_bounds(rows, dp, caps_len, a0_len, alphas, su, ob, ml)
    return alphas, masks, su, ob, ml, want


def _check(want, lower, upper, st, skip=(), nodes=None):
    """Bounds and status against the oracle; with nodes, every completed
    spectrum's memo entries too (the same (mass, row) nodes as the
    reference's memo: the first-visit structure itself, not only its result)."""
    n_ok = 0
    for g, (wl, wu, wn) in enumerate(want):
        if g in skip:
            continue
        if wl is None:  # the reference raises (a window past the reduced table)
            assert int(st[g]) != 0, g
            continue
        assert int(st[g]) == 0 and (int(lower[g]), int(upper[g])) == (wl, wu), \
            (g, int(st[g]), int(lower[g]), int(upper[g]), wl, wu)
        if nodes is not None:
            assert int(nodes[g]) == wn, (g, int(nodes[g]), wn)
        n_ok += 1
    return n_ok


def test_frontier_vs_oracle_rebuilt_tables(setup, cases):
    from spectrseqtools_amd import pipeline_device as PD

    dp, rows, caps_len, a0_len = setup
    alphas, masks, su, ob, ml, want = cases
    lower, upper, st, nodes, stats = PD.length_bounds_alpha_device(dp, masks, su, ob, ml, caps_len, a0_len)
    fr = stats["frontier"]
    assert _check(want, lower, upper, st, nodes=nodes) >= 190
    # keys: root bits + the query's kept ranks + its left moves (<= hi / w_min), the
    # widest query of the batch: 104 rows and 6-mers need more than 64 bits
    assert fr["key_words"] == 2 and fr["splits"] == 0 and fr["aborted"] == 0, fr
    assert fr["nodes"] == int(nodes.sum()) > 10 ** 6, fr  # memo entries, summed over the spectra
    # the same spectra with other key widths: the <= 12-row alphabets alone
    # (64-bit keys), and the whole batch forced to 256-bit keys (a width only
    # windows with memos beyond any oracle's reach need: SST_LBF_MIN_KEY_WORDS)
    import os

    K = np.array([len(a) for a in alphas])
    for sel, kw, force in ((np.flatnonzero(K <= 12), 1, None), (np.arange(len(K)), 4, "4")):
        if force:
            os.environ["SST_LBF_MIN_KEY_WORDS"] = force
        try:
            lo1, up1, st1, nd1, s1 = PD.length_bounds_alpha_device(dp, masks, su, ob, ml, caps_len, a0_len, sel=sel)
        finally:
            os.environ.pop("SST_LBF_MIN_KEY_WORDS", None)
        assert np.array_equal(nd1[sel], nodes[sel])
        assert s1["frontier"]["key_words"] == kw and len(sel) >= 20, (kw, s1["frontier"])
        assert np.array_equal(lo1[sel], lower[sel]) and np.array_equal(up1[sel], upper[sel])
        assert np.array_equal(st1[sel], st[sel])
    # binding budgets: some spectra's bounds differ from their budget-free ones
    free = np.full((21, _native.MAX_ROWS), 255, np.int32)
    lo2, up2, st2, _, _ = PD.length_bounds_alpha_device(dp, masks, su, ob, ml, free, np.full(21, 255, np.int32))
    assert ((lo2 != lower) | (up2 != upper)).sum() >= 10


def test_frontier_split_and_abort(setup, cases):
    """A workspace far smaller than the batch: chunks overflow and are split
    until they fit (same results); one smaller than the heaviest spectra:
    those alone report SST_ABORTED."""
    from spectrseqtools_amd import pipeline_device as PD

    dp, rows, caps_len, a0_len = setup
    alphas, masks, su, ob, ml, want = cases
    _, _, _, nodes, _ = PD.length_bounds_alpha_device(dp, masks, su, ob, ml, caps_len, a0_len)
    per_slot = 376  # workspace bytes per slot (sst_api.cpp: 8 x 7 + 4 + 4 x (32 + 4 + 32) + 20 + 24)
    # the spectra without the four heaviest: tables of >= the heaviest one's
    # nodes, node capacity below the batch's
    keep = np.argsort(nodes)[:-4]
    big, tot = int(nodes[keep].max()), int(nodes[keep].sum())
    S = 1 << int(np.ceil(np.log2(max(big, 1024))))
    assert 8 * S < tot, (big, tot)
    lower, upper, st, nd, stats = PD.length_bounds_alpha_device(dp, masks, su, ob, ml, caps_len, a0_len, sel=keep,
                                                                frontier_workspace=per_slot * S)
    fr = stats["frontier"]
    assert fr["splits"] > 0 and fr["aborted"] == 0 and fr["node_cap"] == 8 * S, fr
    assert _check(want, lower, upper, st, nodes=nd, skip=set(range(len(want))) - set(keep.tolist())) >= 186
    small = int(np.sort(nodes)[-8])  # node capacity below the 8 heaviest spectra's
    S2 = 1 << int(np.floor(np.log2(small // 8)))
    lower, upper, st, _, stats = PD.length_bounds_alpha_device(dp, masks, su, ob, ml, caps_len, a0_len,
                                                               frontier_workspace=per_slot * S2)
    fr = stats["frontier"]
    ab = set(np.flatnonzero(st == _native.SST_ABORTED).tolist())
    assert fr["aborted"] == len(ab) >= 8 and fr["node_cap"] == 8 * S2, fr
    assert all(nodes[g] >= S2 // 4 for g in ab), sorted(int(nodes[g]) for g in ab)  # no light spectrum aborts
    assert _check(want, lower, upper, st, skip=ab) >= 150


@pytest.mark.parametrize("fused", [True, False])
def test_replay_heavy_pass_and_retries_vs_oracle(setup, cases, fused):
    """The round-4 engine: a soft node budget of 2^12 (every spectrum above it
    is replayed again in the heavy pass) and a 2^8-mass first memo (memo
    retries), on the spectra of <= 64 kept rows (fused values) or all of
    them at <= 9 nucleotides (unfused)."""
    from spectrseqtools_amd import pipeline_device as PD

    dp, rows, caps_len, a0_len = setup
    alphas, masks, su, ob, ml, want = cases
    K = np.array([len(a) for a in alphas])
    sel = np.flatnonzero(K <= 64) if fused else np.flatnonzero((K > 64) | (np.arange(len(K)) % 4 == 0))
    lower, upper, st, nodes, _ = PD.length_bounds_alpha_device(dp, masks, su, ob, ml, caps_len, a0_len, sel=sel,
                                                               engine="replay", soft_nodes=1 << 12,
                                                               heavy_memo=1 << 8)
    assert (nodes[sel] > (1 << 12)).sum() >= 10  # the heavy pass ran
    skip = set(range(len(alphas))) - set(sel.tolist())
    assert _check(want, lower, upper, st, skip=skip) >= len(sel) - 2


def _reference_cases(rows):
    """length_cases.json.gz (tests/golden/make_length_golden.py): the
    reference's own compute_sequence_length_bound on 40 alphabets it rebuilt
    itself, windows of 6..20 nucleotides, binding budgets, one window past
    each rebuilt table's end."""
    g = load_golden("length_cases.json.gz")
    cases = g["cases"]
    masks = np.zeros((len(cases), 2), np.uint64)
    for j, c in enumerate(cases):
        a = g["alphabets"][c["alpha"]]
        assert [rows[r] for r in a["rows"]] == a["masses"]
        for r in a["rows"][1:]:
            masks[j, r >> 6] |= np.uint64(1) << np.uint64(r & 63)
    su = np.array([c["su_mass"] for c in cases])
    ob = np.array([c["obs_mass"] for c in cases])
    ml = np.array([c["max_len"] for c in cases])
    return g, cases, masks, su, ob, ml


@pytest.mark.parametrize("engine", ["frontier", "replay"])
def test_length_bounds_vs_reference_fixtures(setup, engine):
    """Both stage-5 engines (length_bounds_alpha_device: the first-visit
    frontier config 5 runs, and the round-4 DFS replay) against the
    REFERENCE's results directly, not the oracle: lower, upper and the raise
    past the reduced table's end, with each case's per-row caps (rate
    profile) and max_modifications, grouped into one call per (profile,
    max_modifications)."""
    from spectrseqtools_amd import pipeline_device as PD

    dp, rows, _, _ = setup
    g, cases, masks, su, ob, ml = _reference_cases(rows)
    n_rows = len(rows)
    groups = {}
    for j, c in enumerate(cases):
        groups.setdefault((c["profile"], c["max_modifications"]), []).append(j)
    n_ok = n_raise = 0
    for (p, A), idx in sorted(groups.items()):
        prof = g["profiles"][p]
        caps_len = np.zeros((21, _native.MAX_ROWS), np.int32)
        for L in range(21):
            caps_len[L, :n_rows] = [round(L * r) for r in prof]
        for j in idx:  # the case's own caps are the profile's (as the generator asserted)
            a = g["alphabets"][cases[j]["alpha"]]
            assert [int(caps_len[cases[j]["max_len"], r]) for r in a["rows"][1:]] == cases[j]["caps"][1:]
        lower, upper, st, _, _ = PD.length_bounds_alpha_device(dp, masks, su, ob, ml, caps_len, np.full(21, A),
                                                               sel=np.array(idx), engine=engine)
        for j in idx:
            c = cases[j]
            if c["lower"] is None:  # the reference raises NotImplementedError (mass_table.py:389-393)
                assert int(st[j]) != 0, (j, int(st[j]))
                n_raise += 1
                continue
            assert int(st[j]) == 0 and (int(lower[j]), int(upper[j])) == (c["lower"], c["upper"]), \
                (j, engine, int(st[j]), int(lower[j]), int(upper[j]), c["lower"], c["upper"])
            n_ok += 1
    assert n_ok >= 240 and n_raise == len(g["alphabets"])


def test_length_bound_mirror_vs_reference_fixtures(setup):
    """The drop-in call itself: mass_table.compute_sequence_length_bound on a
    DynamicProgrammingTable reduced by
    adapt_individual_modification_rates_by_alphabet_reduction (a GPU rebuild
    of the reference's SHA-256) with the case's per-row rates and
    SequenceInformation -- the reference's call sequence at
    skeleton_building.py:212-224 -- equals the reference, and raises its
    NotImplementedError past the table."""
    from spectrseqtools_amd import mass_table as MTm
    from spectrseqtools_amd.mass_explanation import MASS_NAMES
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE

    dp0, rows, _, _ = setup
    g, cases, _, _, _, _ = _reference_cases(rows)
    eng = _native.get_engine(0)
    n_ok = 0
    for ai, a in enumerate(g["alphabets"]):
        seq = MTm.SequenceInformation(max_len=20, su_mass=0.0, obs_mass=0.0, modification_rate=1.0)
        dp = MTm.DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=MATCHING_THRESHOLD,
                                         precision=TOLERANCE, seq=seq, engine=eng)
        try:
            keep = {"A", "C", "G", "U"} | {MASS_NAMES[m][0] for m in a["masses"][1:]}
            dp.adapt_individual_modification_rates_by_alphabet_reduction(keep)
            assert [m.mass for m in dp.masses] == a["masses"]
            import hashlib

            assert hashlib.sha256(np.ascontiguousarray(dp.table).tobytes()).hexdigest() == a["table_sha256"], ai
            for c in (c for c in cases if c["alpha"] == ai):
                prof = g["profiles"][c["profile"]]
                for i, m in enumerate(dp.masses):
                    if m.is_modification:
                        m.modification_rate = prof[a["rows"][i]]
                dp.seq = MTm.SequenceInformation(max_len=c["max_len"], su_mass=c["su_mass"],
                                                 obs_mass=c["obs_mass"], modification_rate=c["modification_rate"])
                for d in ("lower", "upper"):
                    if c[d] is None:
                        with pytest.raises(NotImplementedError):
                            MTm.compute_sequence_length_bound(dp, d)
                    else:
                        assert MTm.compute_sequence_length_bound(dp, d) == c[d], (ai, c["su_mass"], d)
                        n_ok += 1
        finally:
            dp.close()
    assert n_ok >= 480


def test_wide_windows_vs_oracle():
    """Windows wider than one band (w_min masses: a tolerance far above the
    reference's 10 ppm) cannot be laid out by the frontier (their roots would
    span bands): the frontier answers them SST_ABORTED on their own and the
    drop-in compute_sequence_length_bound hands them to the DFS replay, equal
    to the oracle; windows just inside one band stay on the frontier."""
    from spectrseqtools_amd import mass_table as MTm
    from spectrseqtools_amd import pipeline_device as PD
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, TOLERANCE

    eng = _native.get_engine(0)
    rng = np.random.default_rng(5)
    for tol in (0.02, 0.2, 0.3):  # window widths 2 tol obs / 1e-3 masses: inside one band, then beyond w_min
        seq = MTm.SequenceInformation(max_len=8, su_mass=1500.0, obs_mass=1500.0, modification_rate=0.25)
        dp = MTm.DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=tol,
                                         precision=TOLERANCE, seq=seq, engine=eng)
        try:
            dp.adapt_individual_modification_rates_by_alphabet_reduction({"A", "C", "G", "U", "2C", "71C"})
            ms = [m.mass for m in dp.masses]
            tab = oracle.build_table(ms, max(ms) * 35, 32)
            alph = oracle.Alphabet(ms, [m.is_modification for m in dp.masses],
                                   [round(8 * m.modification_rate) for m in dp.masses])
            sus = [float(x) for x in rng.uniform(650.0, 800.0, 3)]
            for su in sus:
                dp.seq = MTm.SequenceInformation(max_len=8, su_mass=su, obs_mass=su, modification_rate=0.25)
                for d in ("lower", "upper"):
                    want = oracle.length_bound(tab, 32, alph, su, su, tol, 8, 2, d)
                    assert MTm.compute_sequence_length_bound(dp, d) == want, (tol, su, d)
        finally:
            dp.close()
    # length_bounds_alpha_device (config 5's path, no replay behind it) at a
    # wide tolerance: the wide windows alone report SST_ABORTED
    seq = MTm.SequenceInformation(max_len=8, su_mass=1500.0, obs_mass=1500.0, modification_rate=0.25)
    dp = MTm.DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=0.09, precision=TOLERANCE,
                                     seq=seq, engine=eng)
    try:
        rows_full = [m.mass for m in dp.masses]
        keep = [r for r, m in enumerate(rows_full) if m in CANONICAL]
        masks = np.zeros((4, 2), np.uint64)
        for r in keep:
            masks[:, 0] |= np.uint64(1) << np.uint64(r)
        su = np.array([1200.0, 2600.0, 3500.0, 4100.0])
        ob = np.array([1200.0, 2000.0, 3500.0, 4100.0])
        wb = min(rows_full[1:])
        wide = np.ceil(0.09 * ob / TOLERANCE) * 2 + 1 > wb
        assert wide.any() and not wide.all()
        caps_len = np.full((21, _native.MAX_ROWS), 4, np.int32)
        lower, upper, st, _, _ = PD.length_bounds_alpha_device(dp, masks, su, ob, np.full(4, 8), caps_len,
                                                               np.full(21, 4))
        ms = [0] + [rows_full[r] for r in keep]
        tab = oracle.build_table(ms, max(ms) * 35, 32)
        alph = oracle.Alphabet(ms, [False] * len(ms), [4] * len(ms))
        for g in range(4):
            if wide[g]:
                assert int(st[g]) == _native.SST_ABORTED, (g, int(st[g]))
                continue
            want = [oracle.length_bound(tab, 32, alph, su[g], ob[g], 0.09, 8, 4, d) for d in ("lower", "upper")]
            assert int(st[g]) == 0 and [int(lower[g]), int(upper[g])] == want, (g, int(st[g]), want)
    finally:
        dp.close()
