"""GPU tests of the per-spectrum reduced-alphabet kernels (sst_alpha.hip,
through the C ABI) against the CPU oracle on each alphabet's own table
(set_up_bit_table over the kept rows, max_mass = max(kept) * 35,
mass_table.py:102-121): k_valid_alpha (is_valid_mass on the reduced table:
whole fragment masses, windows at the table's extent and its last-column
mask, windows reaching 0) and k_pairs_alpha (explain_mass_with_table on
pair-class windows: statuses, counts, candidate rows and order)."""
import numpy as np
import pytest

import _oracle as oracle
from conftest import load_golden
from spectrseqtools_amd import _native
from spectrseqtools_amd.pipeline import row_masks

pytestmark = pytest.mark.gpu
TOL, PREC = 1e-5, 1e-3
CANONICAL = (305042, 306026, 329053, 345048)


@pytest.fixture(scope="module")
def setup():
    g = load_golden("alphabet.json")
    rows = sorted({r["tolerated_integer_masses"] for r in g["rows"]} | {0})
    eng = _native.get_engine(0)
    dev = _native.DeviceTable.build(rows, max(rows) * 35, 32, engine=eng)
    return rows, dev


def _alphabets(rows, rng, n):
    """n random alphabets: the canonical rows plus a random subset of the
    modifications; one whose heaviest row puts (max_mass + 1) % 32 == 0 (the
    last column fully masked, mass_table.py:246) when the alphabet has one."""
    canon = [i for i, m in enumerate(rows) if m in CANONICAL]
    mods = [i for i, m in enumerate(rows) if i > 0 and m not in CANONICAL]
    out = []
    for k in range(n):
        pick = rng.choice(mods, size=int(rng.integers(0, min(40, len(mods)))), replace=False).tolist()
        out.append(sorted(set(canon + pick)))
    quirk = [i for i in mods if (rows[i] * 35 + 1) % 32 == 0 and rows[i] > max(CANONICAL)]
    if quirk:
        out[0] = sorted(set(canon + [i for i in mods if rows[i] < rows[quirk[0]]][:5] + [quirk[0]]))
        assert max(rows[i] for i in out[0]) == rows[quirk[0]]
    out[1] = sorted(canon)  # canonical only
    return out


def test_valid_alpha_vs_oracle(setup):
    rows, dev = setup
    rng = np.random.default_rng(51)
    alphas = _alphabets(rows, rng, 12)
    masks = row_masks(np.array([[r in a for r in range(len(rows))] for a in alphas]))
    masses, thrs, offsets = [], [], [0]
    for a in alphas:
        top = max(rows[r] for r in a) * 35  # the reduced table's max_mass
        m = np.concatenate([rng.uniform(0.2, 9000.0, 1500), rng.uniform(top * PREC - 3, top * PREC + 3, 200),
                            rng.uniform(0.0, 0.05, 20)])
        m.sort()
        masses.append(m)
        thrs.append(TOL * np.abs(m) * rng.uniform(0.5, 30.0, len(m)))
        offsets.append(offsets[-1] + len(m))
    mass, thr = np.concatenate(masses), np.concatenate(thrs)
    got = dev.is_valid_alpha(mass, thr, offsets, masks, TOL, PREC)
    for g, a in enumerate(alphas):
        ms = [rows[0]] + [rows[r] for r in a]
        tab = oracle.build_table(ms, max(ms) * 35, 32)
        sl = slice(offsets[g], offsets[g + 1])
        want = oracle.is_valid_batch(tab, 32, mass[sl], thr[sl], TOL)
        assert np.array_equal(got[sl], want), (g, np.flatnonzero(got[sl] != want)[:5])
    assert set(np.unique(got).tolist()) == {-1, 0, 1}


def test_pairs_alpha_vs_oracle(setup):
    rows, dev = setup
    rng = np.random.default_rng(52)
    alphas = _alphabets(rows, rng, 10)
    masks = row_masks(np.array([[r in a for r in range(len(rows))] for a in alphas]))
    ints = np.array(rows[1:])
    n = 4000
    k = rng.integers(1, 3, n)
    mass = np.array([ints[rng.integers(0, len(ints), kk)].sum() for kk in k]) * PREC + rng.normal(0, 0.01, n)
    mass = np.concatenate([mass, rng.uniform(-0.05, 0.05, 50), [1000.0, 950.0]])  # windows at 0; beyond the pair class
    thr = TOL * rng.uniform(300, 14000, len(mass))
    spec = rng.integers(0, len(alphas), len(mass)).astype(np.int32)
    st, cnt, rm, rg = dev.explain_pairs_alpha(mass, thr, spec, masks, TOL, PREC)
    recs = dev.pair_records()
    tabs = {}
    n_some = n_empty = 0
    whi = np.rint(mass / PREC) + np.ceil(thr / PREC)
    n_other = 0
    for i in range(len(mass)):
        a = alphas[spec[i]]
        if whi[i] >= 3 * min(r for r in rows if r > 0):
            assert st[i] == -10, i  # not pair-class: the caller's to answer
            n_other += 1
            continue
        if spec[i] not in tabs:
            ms = [rows[0]] + [rows[r] for r in a]
            tabs[spec[i]] = (oracle.build_table(ms, max(ms) * 35, 32), oracle.Alphabet(ms, [0] * len(ms), [0] * len(ms)))
        tab, alph = tabs[spec[i]]
        s_, sols, n_e, _ = oracle.explain_table(tab, 32, alph, mass[i], thr[i], TOL, "inf")
        full = [tuple(([0] + a)[x] for x in t) for t in sols]
        want_st = _native.SST_SOME if full else (_native.SST_EMPTY if n_e else _native.SST_NONE)
        assert int(st[i]) == want_st and int(cnt[i]) == len(full), i
        lo, hi = (int(x) for x in rg[i])
        got = [tuple((int(e) >> (8 * (j + 1))) & 0xFF for j in range(int(e) & 0xFF)) for e in recs[lo:hi]]
        got = [t for t in got if all(r in a for r in t)]
        assert got == full, i  # the reference's order
        u = 0
        for t in full:
            for r in t:
                u |= 1 << r
        assert (int(rm[i, 0]) | (int(rm[i, 1]) << 64)) == u, i
        n_some += want_st == _native.SST_SOME
        n_empty += want_st == _native.SST_EMPTY
    assert n_some > 100 and n_empty > 0 and n_other >= 2
