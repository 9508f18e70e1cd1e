"""GPU parity tests: libsstgpu.so (through the C ABI) against the reference's
golden vectors and the CPU oracle, bit-exact (integer/index work)."""
import hashlib
import math

import numpy as np
import pytest

import _oracle as oracle
from conftest import load_golden
from spectrseqtools_amd import _native

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    return _native.get_engine(0)


@pytest.fixture(scope="module")
def alphabet_rows():
    g = load_golden("alphabet.json")
    return sorted({r["tolerated_integer_masses"] for r in g["rows"]} | {0})


@pytest.fixture(scope="module")
def full_dev(engine, alphabet_rows):
    ms = alphabet_rows
    return _native.DeviceTable.build(ms, max(ms) * 35, 32, engine=engine)


@pytest.fixture(scope="module")
def full_host(alphabet_rows):
    ms = alphabet_rows
    return oracle.build_table(ms, max(ms) * 35, 32)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_full_table_matches_reference_sha(full_dev):
    g = load_golden("tables.json")["packed"][0]
    t = full_dev.download()
    assert list(t.shape) == g["shape"]
    assert sha(t) == g["sha256"]
    assert int(t[-1, -1]) == g["last_word_last_row"]


def test_subset_tables_match_reference_sha(engine):
    for p in load_golden("tables.json")["packed"][1:]:
        dev = _native.DeviceTable.build(p["masses"], p["max_mass"], 32, engine=engine)
        assert sha(dev.download()) == p["sha256"], p["what"]
        dev.close()


def test_tiny_tables_every_compression(engine):
    for tiny in load_golden("tables.json")["tiny"]:
        dev = _native.DeviceTable.build(tiny["masses"], tiny["max_mass"], tiny["compression"], engine=engine)
        assert dev.download().tolist() == tiny["words"], (tiny["masses"], tiny["max_mass"], tiny["compression"])
        dev.close()


def test_upload_rejects_inconsistent_table(engine, alphabet_rows):
    t = oracle.build_table([0, 3, 5], 200, 32)
    t[1, 2] ^= np.uint64(1) << np.uint64(40)  # flip one bit0
    with pytest.raises(_native.EngineError):
        _native.DeviceTable.upload([0, 3, 5], t, 32, engine=engine)


def _alph(ms, max_len, mod_rate=0.5, canonical=(305042, 306026, 329053, 345048)):
    is_mod = [m not in canonical and m != 0 for m in ms]
    caps = [round(max_len * (mod_rate if md else (1.0 if m else 0.0))) for m, md in zip(ms, is_mod)]
    return is_mod, caps


def _random_queries(rng, ms, n, kmax=3, thr_hi=14000):
    ints = np.array(ms[1:])
    k = rng.integers(1, kmax + 1, n)
    masses = np.array([ints[rng.integers(0, len(ints), kk)].sum() for kk in k]) * 1e-3
    masses = masses + rng.normal(0, 0.004, n)
    thr = 1e-5 * rng.uniform(300, thr_hi, n)
    return masses, thr


def _check_explain(dev, host, ms, is_mod, caps, masses, thr, A, with_memo, tol=1e-5):
    dev.set_budgets(is_mod, caps)
    res = dev.explain(masses, thr, tol, 1e-3, A, with_memo=with_memo)
    alph = oracle.Alphabet(ms, is_mod, caps)
    Aa = np.broadcast_to(np.asarray(A, dtype=object), (len(masses),))
    for i in range(len(masses)):
        st, sols, n_empty, _ = oracle.explain_table(host, 32, alph, masses[i], None if thr is None else thr[i], tol,
                                                    Aa[i], with_memo=with_memo)
        if st < 0:
            assert int(res.status[i]) == _native.SST_OUT_OF_TABLE, i
            continue
        want_st = _native.SST_SOME if sols else (_native.SST_EMPTY if n_empty else _native.SST_NONE)
        assert int(res.status[i]) == want_st, (i, masses[i], thr[i] if thr is not None else None, Aa[i])
        # same candidate list in the reference's list order
        assert res.candidates(i) == sols, (i, masses[i], Aa[i], with_memo)
    return res


@pytest.mark.parametrize("max_len", [2, 3, 4, 20])
def test_explain_random_vs_oracle(full_dev, full_host, alphabet_rows, max_len):
    rng = np.random.default_rng(100 + max_len)
    ms = alphabet_rows
    is_mod, caps = _alph(ms, max_len)
    masses, thr = _random_queries(rng, ms, 300, kmax=3 if max_len < 20 else 2)
    for A in (0, 1, 2, round(0.5 * max_len), math.inf):
        _check_explain(full_dev, full_host, ms, is_mod, caps, masses, thr, A, True)
    m2, t2 = _random_queries(rng, ms, 120, kmax=2, thr_hi=6000)
    for A in (0, 1, math.inf):
        _check_explain(full_dev, full_host, ms, is_mod, caps, m2, t2, A, False)


def test_explain_per_query_budgets(full_dev, full_host, alphabet_rows):
    rng = np.random.default_rng(5)
    ms = alphabet_rows
    is_mod, caps = _alph(ms, 3)
    masses, thr = _random_queries(rng, ms, 256, kmax=3)
    A = rng.choice([0, 1, 2, 5], 256).tolist()
    _check_explain(full_dev, full_host, ms, is_mod, caps, masses, thr, A, True)


def test_explain_edge_windows(full_dev, full_host, alphabet_rows):
    ms = alphabet_rows
    is_mod, caps = _alph(ms, 20)
    limit = full_host.shape[1] * 32
    masses = np.array([0.0, 0.0004, -0.5, -3.0, 0.3, 305.042, 305.042, 633.169, limit * 1e-3 + 5, 1.0e3])
    thr = np.array([0.05, 0.01, 0.2, 0.01, 0.01, 0.0, 1e-9, 0.0005, 0.01, -1.0])
    _check_explain(full_dev, full_host, ms, is_mod, caps, masses, thr, math.inf, True)
    _check_explain(full_dev, full_host, ms, is_mod, caps, masses, None, math.inf, True)


def test_explain_whole_masses_binding_budget(full_dev, full_host, alphabet_rows):
    # tests/test_explain_masses.py style: whole masses, A = round(0.5 * len)
    rng = np.random.default_rng(9)
    ms = alphabet_rows
    for L in (2, 3, 4):
        seqs = [rng.choice([305042, 306026, 329053, 345048], L) for _ in range(12)]
        masses = np.array([s.sum() * 1e-3 for s in seqs])
        max_len = int(masses.max() / 1e-3 / 305042)
        is_mod, caps = _alph(ms, max_len)
        _check_explain(full_dev, full_host, ms, is_mod, caps, masses, None, round(0.5 * L), True, tol=10e-6)


def test_is_valid_vs_oracle(full_dev, full_host, alphabet_rows):
    rng = np.random.default_rng(3)
    ms = alphabet_rows
    masses, thr = _random_queries(rng, ms, 20000, kmax=20)
    limit = full_host.shape[1] * 32
    extra = np.array([0.0, -1.0, 0.0005, limit * 1e-3 - 0.01, limit * 1e-3 + 2, limit * 1e-3 - 0.3, 305.042])
    masses = np.concatenate([masses, extra])
    thr = np.concatenate([thr, [0.01, 0.5, 0.001, 0.05, 0.01, 0.4, 0.0]])
    got = full_dev.is_valid(masses, thr, 1e-5, 1e-3)
    want = oracle.is_valid_batch(full_host, 32, masses, thr, 1e-5)
    assert np.array_equal(got, want)
    got = full_dev.is_valid(masses, None, 1e-5, 1e-3)
    want = oracle.is_valid_batch(full_host, 32, masses, None, 1e-5)
    assert np.array_equal(got, want)


def test_canonical_reduced_table(engine):
    ms = [0, 305042, 306026, 329053, 345048]
    dev = _native.DeviceTable.build(ms, max(ms) * 35, 32, engine=engine)
    host = oracle.build_table(ms, max(ms) * 35, 32)
    rng = np.random.default_rng(1)
    seqs = [rng.choice(ms[1:], rng.integers(1, 9)) for _ in range(400)]
    masses = np.array([s.sum() * 1e-3 for s in seqs])
    _check_explain(dev, host, ms, [False] * 5, [0, 20, 20, 20, 20], masses, None, math.inf, True, tol=10e-6)


def _boundary_queries(prec, ks, ulps=6):
    """Masses whose quotient mass/prec sits within a few ulps of a half-integer
    (rint ties) and thresholds whose quotient sits on an integer (ceil edge),
    placed so that the window [target - thr, target + thr] starts exactly on
    or next to a reachable multiple of 1000: a one-unit rounding difference
    flips the answer."""
    masses, thr = [], []
    for k in ks:
        for half in (3.5, 4.5):  # ties to even go down at 4.5, up at 3.5
            base = (1000 * k + half) * prec
            mb = [base]
            for _ in range(ulps):
                mb.append(np.nextafter(mb[-1], np.inf))
            mb2 = [base]
            for _ in range(ulps):
                mb2.append(np.nextafter(mb2[-1], -np.inf))
            tb = (3.0 if half == 3.5 else 4.0) * prec
            tv = [tb, np.nextafter(tb, np.inf), np.nextafter(tb, -np.inf)]
            for m in mb + mb2[1:]:
                for t in tv:
                    masses.append(m)
                    thr.append(t)
    return np.array(masses), np.array(thr)


@pytest.mark.parametrize("prec", [1e-3, 3e-3, 7.77e-4])
def test_quantisation_boundaries_vs_oracle(engine, prec):
    ms = [0, 1000]
    dev = _native.DeviceTable.build(ms, 1000 * 35, 32, engine=engine)
    host = oracle.build_table(ms, 1000 * 35, 32)
    masses, thr = _boundary_queries(prec, range(1, 31))
    got = dev.is_valid(masses, thr, 1e-5, prec)
    want = oracle.is_valid_batch(host, 32, masses, thr, 1e-5, precision=prec)
    assert np.array_equal(got, want)
    # the same windows through the explain scan (pair list below 3000, expand/deep above)
    dev.set_budgets([False, False], [0, 40])
    res = dev.explain(masses, thr, 1e-5, prec, math.inf)
    alph = oracle.Alphabet(ms, [False, False], [0, 40])
    for i in range(len(masses)):
        st, sols, n_empty, _ = oracle.explain_table(host, 32, alph, masses[i], thr[i], 1e-5, math.inf, precision=prec)
        want_st = _native.SST_SOME if sols else (_native.SST_EMPTY if n_empty else _native.SST_NONE)
        assert int(res.status[i]) == want_st, (i, masses[i], thr[i])
        assert res.candidates(i) == sols, (i, masses[i], thr[i])
    dev.close()


def test_profile_sampling(full_dev, alphabet_rows):
    # sst_profile_sample: only every n-th launch of a selected kernel is
    # bracketed with events (bench.py --event-every)
    eng = full_dev.engine
    rng = np.random.default_rng(2)
    masses, thr = _random_queries(rng, alphabet_rows, 512, kmax=2)
    eng.profile(True, kernels=(_native.K_EXPLAIN_SCAN,), every=3)
    for _ in range(7):
        full_dev.explain(masses, thr, 1e-5, 1e-3, 10)
    prof = eng.profile_read()
    eng.profile(False)
    assert set(prof) == {_native.K_EXPLAIN_SCAN}
    assert prof[_native.K_EXPLAIN_SCAN][1] == 3  # launches 0, 3 and 6
    assert prof[_native.K_EXPLAIN_SCAN][0] > 0


def test_exact_retry_ladder():
    """The exact path's memo-exhaustion retries, down to the last rung (64
    lanes: one deferred-kernel workgroup with idle waves), in a child process
    whose first per-lane memo is 16 entries (SST_EXACT_HASH_CAP0)."""
    import os
    import subprocess
    import sys

    env = dict(os.environ, SST_EXACT_HASH_CAP0="16")
    here = os.path.dirname(os.path.abspath(__file__))
    p = subprocess.run([sys.executable, os.path.join(here, "_exact_retry_check.py")], env=env, capture_output=True,
                       text=True, timeout=110)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    assert "exact retry ladder ok" in p.stdout
