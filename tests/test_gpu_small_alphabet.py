"""The canonical four-row table (config 1's alphabet): every candidate list --
order included -- against the oracle's literal explain_mass_with_table on the
same table, for whole masses of 1..11 canonical items, windows wide enough to
hold several window values with candidates and many candidates per window,
and windows reaching 0 (the pair scan, the SHALLOW role and the deep DFS all
take part).  A closed-form enumeration of four-row windows was measured
against the deep DFS on config 1 and rejected (41 -> 58 us: DESIGN §9); this
test pinned it while it existed."""
import numpy as np
import pytest

import _oracle as oracle
from spectrseqtools_amd import _native

pytestmark = pytest.mark.gpu
CANONICAL = [0, 305042, 306026, 329053, 345048]
TOL, PREC = 1e-5, 1e-3


def test_four_row_table_vs_oracle():
    eng = _native.get_engine(0)
    dev = _native.DeviceTable.build(CANONICAL, max(CANONICAL) * 35, 32, engine=eng)
    dev.set_budgets([False] * 5, [0, 20, 20, 20, 20])
    host = oracle.build_table(CANONICAL, max(CANONICAL) * 35, 32)
    alph = oracle.Alphabet(CANONICAL, [False] * 5, [0, 20, 20, 20, 20])
    rng = np.random.default_rng(91)
    k = rng.integers(1, 12, 3000)
    m = np.array([sum(rng.choice(CANONICAL[1:], kk)) for kk in k]) * PREC + rng.normal(0, 0.002, len(k))
    # tolerances from tight to ~40 Da wide (many window values, many candidates)
    thr = np.where(rng.random(len(k)) < 0.8, TOL * m, rng.uniform(0.05, 40.0, len(k)))
    m = np.concatenate([m, [0.1, 0.3, 305.042]])
    thr = np.concatenate([thr, [0.2, 0.4, 0.001]])
    res = dev.explain(m, thr, TOL, PREC, -1)
    n_multi = n_big = 0
    for i in range(len(m)):
        st, sols, n_e, _ = oracle.explain_table(host, 32, alph, m[i], thr[i], TOL, -1)
        want = _native.SST_OUT_OF_TABLE if st < 0 else (_native.SST_SOME if sols else
                                                         (_native.SST_EMPTY if n_e else _native.SST_NONE))
        assert int(res.status[i]) == want, (i, m[i], thr[i])
        if sols:
            assert res.candidates(i) == sols, (i, m[i], thr[i])
            sums = {sum(CANONICAL[r] for r in c) for c in sols}
            n_multi += len(sums) > 1
            n_big += len(sols) > 16
    assert n_multi > 20 and n_big > 5
