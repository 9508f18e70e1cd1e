"""GPU suite for the hot path's callers on the HIP engine (through the C ABI):
classify_fragments, Predictor.filter_by_explanation /
collect_explanations_per_side, SkeletonBuilder._predict_skeleton and
calculate_explanations, against the reference-run fixtures
(callers.json.gz, population.json.gz).  The CPU suite (test_callers.py) runs
the same checks on oracle-backed tables."""
import pytest

import _callers_checks as C
from conftest import load_golden
from spectrseqtools_amd import _native, common

pytestmark = pytest.mark.gpu

SPECTRA = ["test_01", "test_02", "test_03", "test_04", "test_05", "test_06", "test_07", "test_08"]


@pytest.fixture(scope="module")
def engine():
    return _native.get_engine(0)


@pytest.fixture(scope="module")
def callers():
    return load_golden("callers.json.gz")


@pytest.fixture(scope="module")
def population():
    return load_golden("population.json.gz")


@pytest.mark.parametrize("tc", SPECTRA)
def test_classify_filter_skeleton(engine, callers, tc):
    """classify_fragments == the reference's output; filter_by_explanation ==
    the reference's alphabet / kept fragments / explanation dict; the batched
    skeleton walk == the reference loop."""
    rec = callers[tc]
    dp = C.make_dp(rec["ctx"], engine=engine)
    C.check_classify(rec, dp)
    frags, expl = C.check_filter(rec, dp)
    C.check_skeleton(dp, frags, expl)


@pytest.mark.parametrize("tc", SPECTRA)
def test_per_side_and_calculate_explanations(engine, population, tc):
    cid = f"pop_{tc}"
    dp = C.make_dp(population["contexts"][cid], engine=engine)
    assert C.check_per_side(population, cid, dp) >= 0
    recs = [r for r in population["a8"] if r[0] == cid]
    batch = common.calculate_explanations_batch([r[1] for r in recs], [r[2] for r in recs], dp)
    for r, b in zip(recs, batch):
        assert C.rows_of_expl(dp, b) == (None if r[4] is None else sorted(tuple(x) for x in r[4]))
    for r in recs[:50]:
        one = common.calculate_explanations(r[1], r[2], dp)
        assert C.rows_of_expl(dp, one) == (None if r[4] is None else sorted(tuple(x) for x in r[4]))


@pytest.mark.parametrize("tc", SPECTRA)
def test_fixpoint_vs_reference(engine, callers, tc):
    """pipeline.filter_fixpoint on the HIP engine (k_pairs_alpha and
    k_valid_alpha against every round's reduced alphabet) == the reference's
    own filter_by_explanation: alphabets and kept fragments after every
    round, the final explanation dict."""
    rec = callers[tc]
    dp = C.make_dp(rec["ctx"], engine=engine)
    C.check_fixpoint(rec, dp)


@pytest.mark.parametrize("tc", SPECTRA)
def test_skeleton_vs_reference(tc):
    """The batched skeleton walk and the Jaccard length selection (its two
    length bounds on the GPU) against the reference's own results, under the
    reference run's hash seed (child process on GPU 0)."""
    import os
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, PYTHONHASHSEED="0")
    p = subprocess.run([sys.executable, os.path.join(here, "_skeleton_check.py"), tc, "gpu"], env=env,
                       capture_output=True, text=True, timeout=250)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert f"skeleton ok {tc}" in p.stdout


def test_classify_batch(engine, callers):
    groups = {tc: (C.make_dp(callers[tc]["ctx"], engine=engine), [callers[tc]]) for tc in ("test_01", "test_05")}
    C.check_classify_batch(None, groups)
