"""The engine and the Python mirror against the reference's golden vectors
(tests/golden/): every explain/is_valid known answer, the reference's own
test spectra query streams, and tests/test_explain_masses.py's assertions."""
import math

import numpy as np
import pytest

from _golden_ctx import budget, expected_status
from spectrseqtools_amd import _native

pytestmark = pytest.mark.gpu

_DEV = {}


def ctx_device(ctx):
    key = tuple(ctx["masses"])
    if key not in _DEV:
        _DEV[key] = _native.DeviceTable.build(ctx["masses"], max(ctx["masses"]) * 35, 32)
    dev = _DEV[key]
    dev.set_budgets(ctx["is_mod"], ctx["caps"])
    return dev


def _run(dev, ctx, cases, with_memo):
    masses = np.array([c["mass"] for c in cases])
    thr_list = [c["threshold"] for c in cases]
    A = [budget(c["max_modifications"]) for c in cases]
    out = []
    # thresholds None -> tolerance*mass; keep the None cases in their own batch
    for none in (True, False):
        idx = [i for i, t in enumerate(thr_list) if (t is None) == none]
        if not idx:
            continue
        thr = None if none else np.array([thr_list[i] for i in idx])
        r = dev.explain(masses[idx], thr, ctx["tolerance"], ctx["precision"], [A[i] for i in idx],
                        with_memo=with_memo)
        out += [(i, int(r.status[j]), sorted(r.candidates(j))) for j, i in enumerate(idx)]
    return sorted(out)


def test_explain_cases(golden_cases):
    ctxs = golden_cases["contexts"]
    groups = {}
    for c in golden_cases["cases"]:
        if c["fn"] == "table":
            groups.setdefault((c["ctx"], c["with_memo"]), []).append(c)
    checked = 0
    for (cid, wm), cases in groups.items():
        ctx = ctxs[cid]
        got = _run(ctx_device(ctx), ctx, cases, wm)
        for i, st, rows in got:
            want_st, want_rows = expected_status(cases[i])
            assert st == want_st, (cid, cases[i]["tag"], cases[i]["mass"], st, want_st)
            if want_rows is not None:
                assert rows == want_rows, (cid, cases[i]["tag"], cases[i]["mass"])
            checked += 1
    assert checked > 1900


def test_is_valid_cases(golden_cases):
    ctxs = golden_cases["contexts"]
    for c in golden_cases["cases"]:
        if c["fn"] != "is_valid":
            continue
        ctx = ctxs[c["ctx"]]
        thr = None if c["threshold"] is None else [c["threshold"]]
        r = int(ctx_device(ctx).is_valid([c["mass"]], thr, ctx["tolerance"], ctx["precision"])[0])
        assert r == (-1 if c["result"] == "raise" else int(c["result"])), c


def test_population_streams(golden_population):
    """A7 and A8 query streams of the reference's test spectra test_01..08."""
    ctxs = golden_population["contexts"]
    for cid, ctx in ctxs.items():
        dev = ctx_device(ctx)
        a7 = [r for r in golden_population["a7"] if r[0] == cid]
        got = dev.is_valid([r[1] for r in a7], [r[2] for r in a7], ctx["tolerance"], ctx["precision"])
        assert got.tolist() == [int(r[3]) for r in a7], cid
        a8 = [r for r in golden_population["a8"] if r[0] == cid]
        if not a8:
            continue
        res = dev.explain([r[1] for r in a8], [r[2] for r in a8], ctx["tolerance"], ctx["precision"], a8[0][3])
        for j, r in enumerate(a8):
            if r[4] is None:
                assert int(res.status[j]) == _native.SST_NONE, (cid, r[1])
            else:
                want = sorted(tuple(x) for x in r[4])
                assert int(res.status[j]) == (_native.SST_SOME if want else _native.SST_EMPTY), (cid, r[1])
                assert sorted(res.candidates(j)) == want, (cid, r[1])


def test_mirror_api_test_explain_masses(golden_cases):
    """tests/test_explain_masses.py:97-136 through the mirror's own
    DynamicProgrammingTable + explain_mass_with_table, full name sets."""
    from spectrseqtools_amd.mass_explanation import explain_mass_with_table, is_valid_mass
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, TOLERANCE

    ctxs = golden_cases["contexts"]
    tables = {}
    for c in golden_cases["cases"]:
        if not c["tag"].startswith("test_explain_masses/") or c["fn"] not in ("table", "is_valid"):
            continue
        ctx = ctxs[c["ctx"]]
        key = (ctx["max_len"], ctx["tolerance"])
        if key not in tables:
            seq = SequenceInformation(max_len=ctx["max_len"], su_mass=ctx["su_mass"], obs_mass=ctx["obs_mass"],
                                      modification_rate=ctx["mod_rate"])
            tables[key] = DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=ctx["tolerance"],
                                                  precision=TOLERANCE, seq=seq)
        dp = tables[key]
        assert [m.mass for m in dp.masses] == ctx["masses"]
        if c["fn"] == "is_valid":
            assert is_valid_mass(c["mass"], dp) == c["result"]
            continue
        got = explain_mass_with_table(c["mass"], dp_table=dp, max_modifications=budget(c["max_modifications"]),
                                      with_memo=True).explanations
        assert got is not None
        assert sorted(list(t) for t in got) == c["names"], (c["ctx"], c["mass"])


def test_mirror_errors_like_reference():
    from spectrseqtools_amd.mass_explanation import explain_mass_with_table, is_valid_mass
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE

    seq = SequenceInformation(max_len=20, su_mass=1000.0, obs_mass=1000.0, modification_rate=0.5)
    dp = DynamicProgrammingTable(EXPLANATION_MASSES, 32, MATCHING_THRESHOLD, TOLERANCE, seq)
    limit = dp.device_table.n_cols * 32
    beyond = limit * 1e-3 + 10
    msg = f"The value {limit + 10000 - 10} is not in the DP table. Extend its size if you want to compute larger masses."
    with pytest.raises(NotImplementedError) as e:
        explain_mass_with_table(beyond, dp, threshold=0.01)
    assert str(e.value) == msg
    with pytest.raises(NotImplementedError) as e:
        is_valid_mass(beyond, dp, threshold=0.01)
    assert str(e.value) == msg
    with pytest.raises(ValueError):
        is_valid_mass(float("nan"), dp)
    assert explain_mass_with_table(0.0001, dp, threshold=0.01).explanations == set()
    assert explain_mass_with_table(-5.0, dp, threshold=0.01).explanations is None
    with pytest.raises(TypeError):
        explain_mass_with_table(300.0, dp, compression_rate=1)
    assert len(dp.table) == len(dp.masses) and dp.table.dtype == np.uint64


def test_alphabet_reduction_rebuilds_on_gpu(golden_cases):
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE

    ctx = golden_cases["contexts"]["canonical_L20"]
    seq = SequenceInformation(max_len=20, su_mass=1000.0, obs_mass=1000.0, modification_rate=0.5)
    dp = DynamicProgrammingTable(EXPLANATION_MASSES, 32, MATCHING_THRESHOLD, TOLERANCE, seq)
    dp.adapt_individual_modification_rates_by_alphabet_reduction({"A", "C", "G", "U"})
    assert [m.mass for m in dp.masses] == ctx["masses"]
    import hashlib

    assert hashlib.sha256(dp.table.tobytes()).hexdigest() == ctx["table_sha256"]
    assert [round(20 * m.modification_rate) for m in dp.masses] == ctx["caps"]


def _mirror_table(keep, max_len):
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE

    frame = EXPLANATION_MASSES.filter_rows(lambda r: r["nucleoside"] in keep)
    seq = SequenceInformation(max_len=max_len, su_mass=0.0, obs_mass=0.0, modification_rate=0.5)
    return DynamicProgrammingTable(frame, 32, MATCHING_THRESHOLD, TOLERANCE, seq)


def test_raise_cases_type_and_message(golden_raise_cases):
    """Every out-of-table case of tests/golden/raise_cases.json (the reference
    run by make_raise_golden.py): same exception type, same message (the
    reference formats its window-loop `value`), same non-raising results."""
    from spectrseqtools_amd.mass_explanation import explain_mass_with_table, is_valid_mass
    from spectrseqtools_amd.mass_table import compute_sequence_length_bound

    g = golden_raise_cases
    dp = _mirror_table(set(g["keep"]), g["max_len"])
    assert [m.mass for m in dp.masses] == g["masses"]
    assert dp.device_table.n_cols * 32 == g["limit"]
    n_raise = 0
    for c in g["cases"]:
        if c["fn"] == "explain":
            call = lambda: explain_mass_with_table(c["mass"], dp, threshold=c["threshold"])  # noqa: E731
        elif c["fn"] == "is_valid":
            call = lambda: is_valid_mass(c["mass"], dp, threshold=c["threshold"])  # noqa: E731
        else:
            dp.seq.su_mass, dp.seq.obs_mass = c["su_mass"], c["obs_mass"]
            call = lambda: compute_sequence_length_bound(dp, c["dir"])  # noqa: E731
        if c["status"] == "raise":
            with pytest.raises(Exception) as e:
                call()
            assert type(e.value).__name__ == c["error"], c
            assert str(e.value) == c["message"], c
            n_raise += 1
        else:
            got = call()
            if c["fn"] == "explain":
                got = None if got.explanations is None else sorted(list(t) for t in got.explanations)
            assert got == c["result"], c
    assert n_raise >= 15


def test_golden_raise_cases_through_mirror(golden_cases):
    """Every explain_cases.json.gz case with status "raise" through the
    mirror's explain_mass_with_table / is_valid_mass: the reference's
    exception type (NotImplementedError), never NameError."""
    from spectrseqtools_amd.mass_explanation import explain_mass_with_table, is_valid_mass
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, TOLERANCE

    ctxs = golden_cases["contexts"]
    dps = {}
    n = 0
    for c in golden_cases["cases"]:
        raising = c.get("status") == "raise" or c.get("result") == "raise"
        if not raising or c["fn"] not in ("table", "is_valid"):
            continue
        ctx = ctxs[c["ctx"]]
        if c["ctx"] not in dps:
            seq = SequenceInformation(max_len=ctx["max_len"], su_mass=ctx["su_mass"], obs_mass=ctx["obs_mass"],
                                      modification_rate=ctx["mod_rate"])
            dps[c["ctx"]] = DynamicProgrammingTable(EXPLANATION_MASSES, 32, ctx["tolerance"], TOLERANCE, seq)
        dp = dps[c["ctx"]]
        assert [m.mass for m in dp.masses] == ctx["masses"]
        limit = dp.device_table.n_cols * 32
        with pytest.raises(Exception) as e:
            if c["fn"] == "table":
                explain_mass_with_table(c["mass"], dp, max_modifications=budget(c["max_modifications"]),
                                        threshold=c["threshold"], with_memo=c["with_memo"])
            else:
                is_valid_mass(c["mass"], dp, threshold=c["threshold"])
        assert type(e.value).__name__ == c["error"], c
        target = int(round(c["mass"] / TOLERANCE, 0))
        thr = int(np.ceil(c["threshold"] / TOLERANCE))
        assert str(e.value).startswith(f"The value {max(target - thr, limit)} is not in the DP table."), c
        n += 1
    assert n >= 8
