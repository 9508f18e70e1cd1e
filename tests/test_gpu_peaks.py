"""GPU test of sst_is_valid_peaks (through the C ABI): is_valid_mass over
peaks x breakage weights, as classify_fragments issues it, equals the
per-query entry point and the CPU oracle on the expanded (mass, threshold)
rows, including windows below the first reachable mass and past the table
end (-1: the reference raises)."""
import numpy as np
import pytest

import _oracle as oracle
from conftest import load_golden
from spectrseqtools_amd import _native
from spectrseqtools_amd.masses import build_breakage_dict

pytestmark = pytest.mark.gpu
TOL, PREC = 1e-5, 1e-3


@pytest.fixture(scope="module")
def rows():
    g = load_golden("alphabet.json")
    return sorted({r["tolerated_integer_masses"] for r in g["rows"]} | {0})


def test_is_valid_peaks_vs_expanded_and_oracle(rows):
    eng = _native.get_engine(0)
    dev = _native.DeviceTable.build(rows, max(rows) * 35, 32, engine=eng)
    limit_da = dev.n_cols * dev.compression * PREC
    rng = np.random.default_rng(21)
    obs = np.concatenate([rng.uniform(300, 9000, 20000), rng.uniform(0.0, 2.0, 200),
                          rng.uniform(limit_da - 2, limit_da + 5, 200)])
    for tags in ((555.1294, 455.1491), (0.0, 0.0)):
        brk = build_breakage_dict(*tags)
        shifts = np.array([w * PREC for w in brk])
        got = dev.is_valid_peaks(obs, shifts, TOL, PREC)
        su = np.concatenate([obs - s for s in shifts])
        thr = TOL * np.tile(obs, len(shifts))
        want = dev.is_valid(su, thr, TOL, PREC)
        assert np.array_equal(got, want)
        host = oracle.build_table(rows, max(rows) * 35, 32) if tags[0] else host
        sample = rng.integers(0, len(su), 3000)
        for i in np.concatenate([sample, np.arange(len(su) - 400 * len(shifts), len(su))]):
            assert int(got[i]) == oracle.is_valid(host, 32, su[i], thr[i], TOL), i
        assert (got == -1).any() and (got == 1).any() and (got == 0).any()
    dev.close()


def test_is_valid_peaks_many_shifts(rows):
    """More than 4 breakage weights (the reference's FULL_BREAKAGE_DICT gives
    up to 16): launched four weights at a time, equal to the expanded
    per-query batch and the oracle."""
    eng = _native.get_engine(0)
    dev = _native.DeviceTable.build(rows, max(rows) * 35, 32, engine=eng)
    host = oracle.build_table(rows, max(rows) * 35, 32)
    rng = np.random.default_rng(22)
    obs = rng.uniform(300, 9000, 5000)
    for n_w in (5, 7, 16, 64):
        shifts = np.sort(rng.uniform(0.0, 1500.0, n_w))
        got = dev.is_valid_peaks(obs, shifts, TOL, PREC)
        su = np.concatenate([obs - s for s in shifts])
        thr = TOL * np.tile(obs, n_w)
        assert np.array_equal(got, dev.is_valid(su, thr, TOL, PREC)), n_w
        for i in rng.integers(0, len(su), 500):
            assert int(got[i]) == oracle.is_valid(host, 32, su[i], thr[i], TOL), (n_w, i)
    dev.close()
