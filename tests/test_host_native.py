"""CPU suite for the host-native helpers in libsstgpu.so that the columnar
stages call (no device needed): sst_window_pairs, sst_su_diff_queries and
sst_sort_rows against their plain-Python statements (producers.py, which
test_host.py / test_callers.py pin to the reference), on random and edge
inputs -- empty spectra, one-row sides, equal SU masses, a side that lies
within one window."""
import numpy as np
import pytest

from spectrseqtools_amd import _native
from spectrseqtools_amd.producers import diff_queries, sliding_window_pairs

MAX_W = 633.2
TOL = 5e-6


def _spectra(rng, n_spec, max_rows, equal_frac=0.0):
    """Random spectra: per spectrum a sorted SU column (ties when
    equal_frac > 0), observed masses, side/singleton flags, offsets."""
    lens = rng.integers(0, max_rows + 1, n_spec)
    offsets = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    su, obs, flags = [], [], []
    for n in lens:
        s = np.sort(rng.uniform(0.0, 3000.0, n))
        if equal_frac and n > 1:
            tie = rng.random(n - 1) < equal_frac
            for i in np.flatnonzero(tie):
                s[i + 1] = s[i]
        su.append(s)
        obs.append(s + rng.uniform(0.0, 50.0, n))
        f = rng.integers(1, 4, n).astype(np.uint8)  # 1 START, 2 END, 3 both
        f |= (rng.random(n) < 0.2).astype(np.uint8) << 2  # 4 singleton
        flags.append(f)
    cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)
    return cat(su, np.float64), cat(obs, np.float64), cat(flags, np.uint8), offsets


def _python_su_diffs(su, obs, flags, offsets, max_w, tol):
    """collect_diff_explanations_for_su's order (prediction.py:261-329): per
    spectrum the START pairs, the END pairs, then the singletons."""
    d, t, g, k = [], [], [], []
    for s in range(len(offsets) - 1):
        r = np.arange(offsets[s], offsets[s + 1])
        for kind, bit in ((0, 1), (1, 2)):
            side = r[(flags[r] & bit) != 0]
            dd, tt, _ = diff_queries(su[side], obs[side], tol, max_w)
            d += dd.tolist(); t += tt.tolist(); g += [s] * len(dd); k += [kind] * len(dd)
        sing = r[(flags[r] & 4) != 0]
        d += su[sing].tolist(); t += (tol * obs[sing]).tolist(); g += [s] * len(sing); k += [2] * len(sing)
    return d, t, g, k


@pytest.mark.parametrize("seed,n_spec,max_rows,equal_frac", [
    (0, 40, 30, 0.0), (1, 200, 6, 0.0), (2, 30, 60, 0.3), (3, 1, 0, 0.0), (4, 5, 1, 0.0),
    (5, 1500, 12, 0.1)])  # > 256 spectra: the threaded pass
def test_su_diff_queries_equal_python(seed, n_spec, max_rows, equal_frac):
    rng = np.random.default_rng(seed)
    su, obs, flags, offsets = _spectra(rng, n_spec, max_rows, equal_frac)
    d, t, g, k = _native.su_diff_queries(su, obs, flags, offsets, MAX_W, TOL)
    wd, wt, wg, wk = _python_su_diffs(su, obs, flags, offsets, MAX_W, TOL)
    assert d.tolist() == wd
    assert t.tolist() == wt
    assert g.tolist() == wg
    assert k.tolist() == wk


def test_su_diff_queries_no_spectra_and_dense_window():
    z = np.zeros(0)
    d, t, g, k = _native.su_diff_queries(z, z, np.zeros(0, np.uint8), np.zeros(1, np.int64), MAX_W, TOL)
    assert len(d) == len(t) == len(g) == len(k) == 0
    # one START side whose rows all fit in one window: the reference's window
    # walks the end to the last row, then the start up to it (2n - 3 pairs)
    su = np.arange(12, dtype=np.float64)
    d, t, g, k = _native.su_diff_queries(su, su + 1.0, np.ones(12, np.uint8), np.array([0, 12]), MAX_W, TOL)
    assert len(d) == 2 * 12 - 3
    assert d.tolist() == list(range(1, 12)) + list(range(10, 0, -1))
    assert set(k.tolist()) == {0} and set(g.tolist()) == {0}


def test_window_pairs_equal_python():
    rng = np.random.default_rng(7)
    su, _, _, offsets = _spectra(rng, 60, 25, 0.2)
    s, e = _native.window_pairs(su, offsets, MAX_W)
    want = []
    for j in range(len(offsets) - 1):
        b = offsets[j]
        want += [(b + i, b + k) for i, k in sliding_window_pairs(su[b:offsets[j + 1]], MAX_W)]
    assert list(zip(s.tolist(), e.tolist())) == want


@pytest.mark.parametrize("seed,n,n_groups,n_keys", [(0, 1000, 17, 50), (1, 5000, 1, 5000), (2, 300, 300, 3),
                                                      (3, 200000, 3000, 1000)])  # >= 2^16 rows: threaded
def test_sort_rows_equal_lexsort(seed, n, n_groups, n_keys):
    rng = np.random.default_rng(seed)
    group = rng.integers(0, n_groups, n)
    key = rng.integers(0, n_keys, n).astype(np.float64) * 0.5  # ties within a group
    got = _native.sort_rows(group, key, n_groups)
    assert got.tolist() == np.lexsort((np.arange(n), key, group)).tolist()


def test_sort_rows_edges():
    assert _native.sort_rows(np.zeros(0, np.int64), np.zeros(0), 0).tolist() == []
    assert _native.sort_rows([0], [1.0], 1).tolist() == [0]
    # already sorted and reverse-sorted single group
    k = np.arange(10, dtype=np.float64)
    assert _native.sort_rows(np.zeros(10, np.int64), k, 1).tolist() == list(range(10))
    assert _native.sort_rows(np.zeros(10, np.int64), k[::-1], 1).tolist() == list(range(9, -1, -1))
    with pytest.raises(_native.EngineError):
        _native.sort_rows([0, 5], [1.0, 2.0], 2)  # group id out of range
