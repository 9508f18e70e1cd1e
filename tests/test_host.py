"""Host-side logic of the mirror: alphabet, constants, breakage dicts, table
objects' alphabet bookkeeping, name expansion, result decoding, producers.
CPU only, checked against the reference's golden vectors."""
import numpy as np
import pytest

from spectrseqtools_amd import _native, masses
from spectrseqtools_amd.mass_explanation import IS_MOD, MASS_NAMES, convert_nucleotide_masses_to_names
from spectrseqtools_amd.mass_table import (SequenceInformation, initialize_nucleotide_masses,
                                           select_table_building_settings)


def test_explanation_masses_match_reference(golden_alphabet):
    want = [(r["monoisotopic_mass"], r["nucleoside"], r["nucleoside_list"], r["modification_rate"],
             r["theoretical_mz"], r["tolerated_integer_masses"]) for r in golden_alphabet["rows"]]
    assert [tuple(r) for r in masses.EXPLANATION_MASSES.rows()] == want
    assert masses.EXPLANATION_MASSES.columns == ["monoisotopic_mass", "nucleoside", "nucleoside_list",
                                                 "modification_rate", "theoretical_mz", "tolerated_integer_masses"]


def test_constants_match_reference(golden_alphabet):
    g = golden_alphabet
    assert masses.PHOSPHATE_LINK_MASS == g["phosphate_link_mass"]
    assert masses.TOLERANCE == g["tolerance"]
    assert masses.MATCHING_THRESHOLD == g["matching_threshold"]
    assert masses.COMPRESSION_RATE == g["compression_rate"]
    assert masses.UNMODIFIED_BASES == g["unmodified_bases"]
    assert masses.ELEMENT_MASSES == g["element_masses"]
    assert masses.NUC_REPS == g["nuc_reps"]
    assert MASS_NAMES == {int(k): v for k, v in g["mass_names"].items()}
    assert IS_MOD == {int(k): v for k, v in g["is_mod"].items()}


def test_breakage_dicts(golden_alphabet):
    for b in golden_alphabet["breakage_dicts"]:
        d = masses.build_breakage_dict(b["mass_5_prime"], b["mass_3_prime"])
        assert [[k, v] for k, v in d.items()] == b["dict"]


def test_nucleotide_masses_of_contexts(golden_cases):
    """initialize_nucleotide_masses + universal-rate capping reproduce the
    reference's row lists (the full-alphabet contexts)."""
    for cid, ctx in golden_cases["contexts"].items():
        if not cid.startswith("full_"):
            continue
        rows = initialize_nucleotide_masses(masses.EXPLANATION_MASSES)
        seq = SequenceInformation(ctx["max_len"], 0.0, 0.0, ctx["mod_rate"])
        for r in rows:
            if r.is_modification and r.modification_rate > seq.modification_rate:
                r.modification_rate = seq.modification_rate
        assert [r.mass for r in rows] == ctx["masses"]
        assert [r.names for r in rows] == ctx["names"]
        assert [r.is_modification for r in rows] == ctx["is_mod"]
        assert [r.modification_rate for r in rows] == ctx["rates"]
        assert [round(ctx["max_len"] * r.modification_rate) for r in rows] == ctx["caps"]


def test_name_expansion_matches_golden(golden_cases):
    ctxs = golden_cases["contexts"]
    n = 0
    for c in golden_cases["cases"]:
        if c["fn"] != "table" or c["status"] != "set" or "names" not in c:
            continue
        ms = ctxs[c["ctx"]]["masses"]
        sols = [[ms[r] for r in rows] for rows in c["rows"]] or [[]]  # set() <- only the v=0 solution
        got = convert_nucleotide_masses_to_names(sols).explanations
        assert sorted(list(t) for t in got) == c["names"]
        n += 1
    assert n > 500
    assert convert_nucleotide_masses_to_names([]).explanations is None
    assert convert_nucleotide_masses_to_names([[]]).explanations == set()


def test_table_settings():
    assert select_table_building_settings(32)["init"] == 0xC000000000000000
    with pytest.raises(ValueError):
        select_table_building_settings(7)


def test_result_payload_decoding():
    r = _native.ExplainResult(None, None, 3)
    r.status = np.array([2, 0, 2], np.int8)
    r.count = np.array([2, 0, 1], np.uint64)
    r.offset = np.array([0, 0, 5], np.uint64)
    r.payload = np.array([1, 7, 2, 3, 9, 3, 1, 1, 4], np.uint8)
    assert r.candidates(0) == [(7,), (3, 9)]
    assert r.candidates(1) == []
    assert r.candidates(2) == [(1, 1, 4)]
    r.handle = None


def test_producers_replay_reference_query_streams(golden_population):
    """classify_queries (fragment_classification.py:39-67) and the sliding
    window (prediction.py:286-329) regenerate the reference's exact A7 and A8
    query streams of its test spectra (test_01..08) from the observed masses,
    given the reference's is_valid answers."""
    from spectrseqtools_amd.producers import MAX_VARIANCE, classify_queries, diff_queries, max_nucleotide_weight

    a7, a8 = {}, {}
    for cid, m, t, v in golden_population["a7"]:
        a7.setdefault(cid, []).append((m, t, v))
    for cid, m, t, A, rows in golden_population["a8"]:
        a8.setdefault(cid, []).append((m, t))
    maxw = max_nucleotide_weight()
    for cid, ctx in golden_population["contexts"].items():
        sp = ctx["spectrum"]
        brk = masses.build_breakage_dict(*sp["tags"])
        cq = classify_queries(sp["observed"], brk, ctx["precision"], ctx["tolerance"])
        assert cq.su_mass.tolist() == [r[0] for r in a7[cid]]
        assert cq.threshold.tolist() == [r[1] for r in a7[cid]]
        valid = np.array([r[2] for r in a7[cid]])
        cutoff = sp["intensity_cutoff"]
        inten = [cutoff * 1.1 if x is None else x for x in sp["intensity"]] * len(brk)
        kept = [(cq.su_mass[i], cq.observed[i], cq.breakage[i], inten[i]) for i in range(len(valid)) if valid[i]]
        kept = sorted(kept, key=lambda c: c[0])
        kept = [c for c in kept if c[3] > cutoff and c[1] < 50000]
        su_seq = sp["su_seq"]
        kept = [c for c in kept if c[0] < su_seq + MAX_VARIANCE and
                (c[0] > su_seq - MAX_VARIANCE or not ("START" in c[2] and "END" in c[2]))]
        got = []
        for side in ("START", "END"):
            fr = [c for c in kept if side in c[2]]
            d, t, _ = diff_queries(np.array([c[0] for c in fr]), np.array([c[1] for c in fr]), ctx["tolerance"], maxw)
            got += list(zip(d.tolist(), t.tolist()))
        assert got == a8.get(cid, []), cid


def test_sliding_window_small():
    from spectrseqtools_amd.producers import sliding_window_pairs

    assert sliding_window_pairs([1.0, 2.0, 700.0, 701.0], 633.2) == [(0, 1), (2, 3)]
    assert sliding_window_pairs([1.0, 2.0, 3.0], 633.2) == [(0, 1), (0, 2), (1, 2)]
    assert sliding_window_pairs([5.0], 633.2) == []
