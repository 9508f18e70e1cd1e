"""GPU tests of the device-resident config-5 stages (pipeline_device:
sst_classify_rows_device, sst_fix_round_device, sst_valid_rows_alpha_device):
  * on the reference's 8 test spectra: the classified rows equal the
    reference's own classify_fragments frame row for row, and every
    filter_by_explanation round's alphabet and kept fragments equal the
    reference's (tests/golden/callers.json.gz);
  * on synthetic spectra (peaks sorted and as generated): rows, final
    alphabets, surviving rows and round counts equal the host-driven columnar
    stages (pipeline.classify / filter_fixpoint, pinned to the per-spectrum
    mirrors in the CPU suite), and the device skeleton-bin answers equal the
    host-built bin queries (pipeline.bin_queries) answered on the same
    alphabets."""
import os

import numpy as np
import pytest

import _callers_checks as C
from conftest import load_golden

pytestmark = pytest.mark.gpu
SPECTRA = ["test_01", "test_02", "test_03", "test_04", "test_05", "test_06", "test_07", "test_08"]


@pytest.fixture(scope="module")
def engine():
    from spectrseqtools_amd import _native

    return _native.get_engine(0)


@pytest.fixture(scope="module")
def callers():
    return load_golden("callers.json.gz")


@pytest.mark.parametrize("tc", SPECTRA)
def test_device_classify_and_fixpoint_vs_reference(engine, callers, tc):
    from spectrseqtools_amd import pipeline_device as PD
    from spectrseqtools_amd.masses import build_breakage_dict
    from spectrseqtools_amd.pipeline import mask_rows

    rec = callers[tc]
    dp = C.make_dp(rec["ctx"], engine=engine)
    cols = rec["input"]["columns"]
    inp = {c: [r[i] for r in rec["input"]["rows"]] for i, c in enumerate(cols)}
    obs = np.asarray(inp["observed_mass" if "observed_mass" in inp else "neutral_mass"], dtype=np.float64)
    inten = np.asarray(inp["intensity"], dtype=np.float64) if "intensity" in inp else None
    bd = build_breakage_dict(*rec["tags"])  # the reference's own input, in its peak order
    rows = PD.classify_device(dp, obs, [0, len(obs)], [dp.seq.su_mass], bd, intensity=inten,
                              intensity_cutoff=rec["intensity_cutoff"])
    n = int(rows.rows.cpu()[0])
    want = rec["classify"]
    wc = {c: [r[i] for r in want["rows"]] for i, c in enumerate(want["columns"])}
    assert n == len(want["rows"])
    meta = rows.meta.cpu().numpy()[:n].astype(np.int64)
    assert rows.su.cpu().numpy()[:n].tolist() == wc["standard_unit_mass"]
    assert rows.obs.cpu().numpy()[:n].tolist() == wc["observed_mass"]
    assert [rows.names[m & 3] for m in meta] == wc["breakage"]
    assert [bool((m >> 4) & 1) for m in meta] == wc["is_singleton"]
    assert (meta >> 8).tolist() == wc["fragment_index"]
    fx = PD.fixpoint_device(dp, rows, [dp.seq.max_len], record=True)
    rounds = rec["filter"]["rounds"]
    assert fx.n_rounds == len(rounds) == int(fx.rounds[0])
    for k, (act, alpha, alive) in enumerate(fx.history):
        rr = mask_rows(alpha, len(dp.masses))[0]
        assert [0] + [dp.masses[r].mass for r in range(1, len(dp.masses)) if rr[r]] == rounds[k]["masses"], k
        assert np.flatnonzero(alive[:n]).tolist() == rounds[k]["kept_index"], k


@pytest.mark.parametrize("peak_order", ["sorted", "as_generated"])
def test_device_stages_equal_host_driven(engine, peak_order):
    from spectrseqtools_amd import pipeline, pipeline_device as PD
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE, build_breakage_dict
    from spectrseqtools_amd.synthetic import make_spectra

    b = make_spectra(600, seed=31)
    # as generated, each spectrum's noise peaks follow its fragment peaks (not
    # in mass order): the device ranks them, the host sorts the rows
    obs = b.observed[np.lexsort((b.observed, b.spectrum))] if peak_order == "sorted" else b.observed
    bd = build_breakage_dict(555.1294, 455.1491)
    w_full = [k for k, v in bd.items() if "START_END" in v][0]
    su_seq = b.seq_mass - w_full * TOLERANCE
    seq = SequenceInformation(max_len=20, su_mass=float(su_seq[0]), obs_mass=float(b.seq_mass[0]),
                              modification_rate=0.5)
    dp = DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=MATCHING_THRESHOLD,
                                 precision=TOLERANCE, seq=seq, engine=engine)
    max_len = pipeline.max_len_of(su_seq, TOLERANCE, min(m.mass for m in dp.masses[1:]))
    c = pipeline.classify(obs, b.offsets, su_seq, dp, bd)
    rows = PD.classify_device(dp, obs, b.offsets, su_seq, bd)
    cnt = rows.rows.cpu().numpy()
    assert np.array_equal(cnt, np.diff(c.offsets))
    slot = (4 * b.offsets[:-1])[c.spec] + (np.arange(len(c.spec)) - c.offsets[c.spec])
    assert np.array_equal(rows.su.cpu().numpy()[slot], c.su)
    meta = rows.meta.cpu().numpy()[slot].astype(np.int64)
    assert np.array_equal(meta & 3, c.brk) and np.array_equal(((meta >> 4) & 1).astype(bool), c.singleton)
    assert np.array_equal(meta >> 8, c.frag)  # the caller's peak positions
    assert np.array_equal(PD.to_classified(rows, alive_only=False).frag, c.frag)
    fx_h = pipeline.filter_fixpoint(c, dp, max_len, EXPLANATION_MASSES)
    fx_d = PD.fixpoint_device(dp, rows, max_len)
    assert np.array_equal(fx_d.alpha, fx_h.alpha)
    assert np.array_equal(fx_d.rounds, fx_h.rounds)
    assert np.array_equal(rows.alive.cpu().numpy()[slot].astype(bool), fx_h.alive)
    assert int(fx_d.queries.sum()) == sum(q[0] for q in fx_h.queries)
    # stage 3: the skeleton's bin queries on the device against the host-built
    # queries (pipeline.bin_queries, pinned to the per-spectrum walk in the CPU
    # suite) answered by explain_pairs_alpha; host order -> spectrum-major
    c3 = pipeline.subset(c, fx_h.alive)
    q3 = pipeline.bin_queries(c3)
    st3, cnt3, _, _ = dp.device_table.explain_pairs_alpha(q3.diff, q3.thr, q3.spec, fx_h.alpha, dp.tolerance,
                                                          dp.precision)
    order = np.lexsort((q3.side, q3.spec))  # stable: a side's queries keep their order
    db = PD.bins_device(dp, rows, fx_d.alpha)
    S = len(b.offsets) - 1
    assert np.array_equal(np.diff(db.q_off), np.bincount(q3.spec, minlength=S))
    assert np.array_equal(db.status.cpu().numpy(), st3[order])
    assert np.array_equal(db.count.cpu().numpy().astype(np.int64), cnt3[order].astype(np.int64))
    assert (st3 == 2).sum() > 0


def test_device_bins_deferred_vs_rebuilt_tables(engine):
    """Stage 3's off-pair-class bin queries (the sides' first bins' whole
    masses, wide bin differences) answered by the masked explain on each
    spectrum's final alphabet with its own budgets (max_len groups), against
    the oracle on that alphabet's rebuilt table; the pair-class answers are
    those of the plain emit."""
    import _oracle as oracle
    from spectrseqtools_amd import _native, pipeline, pipeline_device as PD
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE, build_breakage_dict
    from spectrseqtools_amd.synthetic import make_spectra

    b = make_spectra(400, seed=37)
    bd = build_breakage_dict(555.1294, 455.1491)
    w_full = [k for k, v in bd.items() if "START_END" in v][0]
    su_seq = b.seq_mass - w_full * TOLERANCE
    seq = SequenceInformation(max_len=20, su_mass=float(su_seq[0]), obs_mass=float(b.seq_mass[0]),
                              modification_rate=0.5)
    dp = DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=MATCHING_THRESHOLD,
                                 precision=TOLERANCE, seq=seq, engine=engine)
    max_len = pipeline.max_len_of(su_seq, TOLERANCE, min(m.mass for m in dp.masses[1:]))
    # every other spectrum loses its peaks below 1.6 kDa (missing short
    # fragments): its sides' first bins are whole masses of 3+ nucleotides,
    # off the pair class (the exact replay with binding budgets)
    spec = np.repeat(np.arange(len(b.offsets) - 1), np.diff(b.offsets))
    keep = (spec % 2 == 1) | (b.observed > 1600.0)
    obs = b.observed[keep]
    offsets = np.concatenate([[0], np.cumsum(np.bincount(spec[keep], minlength=len(b.offsets) - 1))])
    rows = PD.classify_device(dp, obs, offsets, su_seq, bd)
    fx = PD.fixpoint_device(dp, rows, max_len)
    plain = PD.bins_device(dp, rows, fx.alpha)
    full = PD.bins_device(dp, rows, fx.alpha, max_len=max_len)
    st0, st1 = plain.status.cpu().numpy(), full.status.cpu().numpy()
    pend = st0 == -10
    assert pend.sum() == full.deferred["queries"] > 100
    assert np.array_equal(st0[~pend], st1[~pend])
    assert not (st1 == -10).any()
    d = full.deferred
    ms_all = [m.mass for m in dp.masses]
    is_mod = [m.is_modification for m in dp.masses]
    rate = [m.modification_rate for m in dp.masses]
    masks = pipeline.mask_rows(fx.alpha, len(ms_all))
    tabs = {}
    n_checked = n_some = 0
    spec_l, mass_l, thr_l = d["spec"], d["mass"], d["thr"]  # list order of the results
    for s0, res in d["results"]:
        for j in range(0, res.n, 5):
            k = s0 + j
            g = int(spec_l[k])
            keep = [0] + [r for r in range(1, len(ms_all)) if masks[g, r]]
            if g not in tabs:
                ms = [ms_all[r] for r in keep]
                tabs[g] = (oracle.build_table(ms, max(ms) * 35, 32),
                           oracle.Alphabet(ms, [is_mod[r] for r in keep],
                                           [round(int(max_len[g]) * rate[r]) for r in keep]))
            tab, alph = tabs[g]
            A = round(dp.seq.modification_rate * int(max_len[g]))
            st, sols, n_e, _ = oracle.explain_table(tab, 32, alph, mass_l[k], thr_l[k], dp.tolerance, A)
            want = [tuple(keep[x] for x in t) for t in sols]
            want_st = (_native.SST_OUT_OF_TABLE if st < 0 else _native.SST_SOME if want else
                       _native.SST_EMPTY if n_e else _native.SST_NONE)
            assert int(res.status[j]) == want_st, (k, g, mass_l[k])
            if want_st == _native.SST_SOME:
                assert res.candidates(j) == want, (k, g)
                n_some += 1
            n_checked += 1
    assert n_checked > 50 and n_some > 10



@pytest.mark.parametrize("tc", SPECTRA)
def test_device_skeleton_walk_vs_reference(tc):
    """Stage 4 on the device (k_skel_walk after classify / fixpoint / bins on
    the device): each side's skeleton, kept fragments, min_end and max_end ==
    the reference's own SkeletonBuilder._predict_skeleton (callers.json.gz),
    under the reference run's hash seed (child process on GPU 0: the lanes
    order explanations as CPython's sets do, from this interpreter's name
    hashes; test_04 / test_08 depend on that order)."""
    import os
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, PYTHONHASHSEED="0")
    p = subprocess.run([sys.executable, os.path.join(here, "_skeleton_check.py"), tc, "device"], env=env,
                       capture_output=True, text=True, timeout=250)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert f"skeleton ok {tc} device" in p.stdout


def _mirror_outcome(obs, su_seq, obs_seq, max_len, engine, mod_rate=0.5):
    """The per-spectrum host mirrors (pinned to the reference on its own test
    spectra): classify_fragments, Predictor.filter_by_explanation,
    SkeletonBuilder._predict_skeleton per side and
    select_sequence_length_with_jaccard with combine_skeleton_sequences."""
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE

    seq = SequenceInformation(max_len=int(max_len), su_mass=float(su_seq), obs_mass=float(obs_seq),
                              modification_rate=mod_rate)
    dp = DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=MATCHING_THRESHOLD,
                                 precision=TOLERANCE, seq=seq, engine=engine)
    try:
        return _mirror_run(dp, obs)
    finally:
        dp.close()  # a table per spectrum: free its HBM now, not at the next full GC pass


def _mirror_run(dp, obs):
    from spectrseqtools_amd import _native
    from spectrseqtools_amd.fragment_classification import classify_fragments
    from spectrseqtools_amd.frame import Frame
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, build_breakage_dict
    from spectrseqtools_amd.prediction import Predictor
    from spectrseqtools_amd.skeleton_building import SkeletonBuilder, combine_skeleton_sequences

    bd = build_breakage_dict(555.1294, 455.1491)
    fr = classify_fragments(Frame({"observed_mass": list(map(float, obs))}), dp, bd)
    f = C.prepared(fr)
    pred = Predictor(dp, EXPLANATION_MASSES)
    frags, expl = pred.filter_by_explanation(f)
    sb = SkeletonBuilder(explanations=expl, dp_table=dp)
    out, sks = {"filter_masses": [m.mass for m in dp.masses], "filter_kept": frags.get_column("index").to_list()}, {}
    # SU differences the final dict's queries hold more than once at different
    # thresholds (the last writer's threshold is the one the walk must use)
    cols = frags.to_dict()
    su_f, ob_f = np.asarray(cols["standard_unit_mass"], np.float64), np.asarray(cols["observed_mass"], np.float64)
    thr_of = {}
    for side in ("START", "END"):
        m = np.array([side in b for b in cols["breakage"]], bool)
        keys, _, thr = pred._side_queries(su_f[m], ob_f[m])
        for k_, t_ in zip(keys, thr.tolist()):
            thr_of.setdefault(k_, set()).add(t_)
    out["dup_thr_keys"] = sum(len(v) > 1 for v in thr_of.values())
    for side in ("START", "END"):
        sub = frags.filter_mask([side in b for b in frags.get_column("breakage").to_list()])
        sk, fs = sb._predict_skeleton(Frame(sub.to_dict()), [set() for _ in range(dp.seq.max_len)])
        out[side] = {"skeleton": [sorted(p) for p in sk], "kept_index": fs.get_column("index").to_list(),
                     "min_end": fs.get_column("min_end").to_list(), "max_end": fs.get_column("max_end").to_list()}
        sks[side] = sk
    try:
        seq_len = sb.select_sequence_length_with_jaccard(start_skeleton=sks["START"], end_skeleton=sks["END"][::-1])
        out["seq_len"] = seq_len
        out["combined"] = [sorted(p) for p in combine_skeleton_sequences(seq_len, sks["START"], sks["END"][::-1])]
    except IndexError:
        out["seq_len"], out["combined"] = "IndexError", None
    except _native.EngineError:
        raise  # the engine failing (out of HBM, say) is not the reference's "no length" exception
    except Exception:  # noqa: BLE001 -- the reference raises a bare Exception when no length fits
        out["seq_len"], out["combined"] = None, None
    out["masses"] = [m.mass for m in dp.masses]
    return out


@pytest.mark.parametrize("variant", ["full_ladders", "short_fragments_missing", "low_modification_rate",
                                     "noise_free", "noise_free_exact"])
def test_device_skeleton_and_length_vs_mirror(engine, variant):
    """Stages 4-5 on the device over synthetic spectra against the
    per-spectrum host mirrors in this process (same interpreter, same hash
    seed): each side's skeleton, kept rows, min_end / max_end, the skeleton
    alphabet, the Jaccard length and the combined skeleton.  Without their
    short fragments, spectra need first bins of whole masses of 3+ nucleotides
    and re-queries against older bins (the masked explain, suspended lanes).
    At --modification_rate 0.05 (cli.py:35) the budgets bind on pair windows
    (max_modifications and caps < 2): every stage runs its spectra in exact
    mode (sst_exact_io: the exact masked replay answers their windows).
    Noise-free spectra repeat SU differences exactly at different observed
    masses, so the final dict's last writer often carries another threshold
    than the bin the walk queries (skeleton_building.py:429-430): the walk
    answers pair-class windows at the dict's threshold, and re-queries
    exact-mode ones instead of taking stage 3's answer."""
    from spectrseqtools_amd import _native, pipeline, pipeline_device as PD
    from spectrseqtools_amd.mass_explanation import MASS_NAMES
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE, build_breakage_dict

    import _synth_cases as SC

    n = 48
    d = SC.variant_inputs(variant, n)  # the inputs of the reference-run fixtures (test_device_synthetic_vs_reference)
    exact, clean, mod_rate = d["exact"], d["clean"], d["mod_rate"]
    obs, offsets, su_seq, max_len = d["obs"], d["offsets"], d["su_seq"], d["max_len"]

    class b:  # noqa: N801 -- the sequence masses under the name the checks below use
        seq_mass = d["seq_mass"]

    bd = build_breakage_dict(*SC.TAGS)
    seq = SequenceInformation(max_len=20, su_mass=float(su_seq[0]), obs_mass=float(b.seq_mass[0]),
                              modification_rate=mod_rate)
    dp = DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=MATCHING_THRESHOLD,
                                 precision=TOLERANCE, seq=seq, engine=engine)
    assert np.array_equal(max_len, pipeline.max_len_of(su_seq, TOLERANCE, min(m.mass for m in dp.masses[1:])))
    if exact:
        assert not PD.budgets_pair_ok(dp, max_len).any()
    rows = PD.classify_device(dp, obs, offsets, su_seq, bd)
    fx = PD.fixpoint_device(dp, rows, max_len)
    bins = PD.bins_device(dp, rows, fx.alpha, max_len=max_len)
    sk = PD.skeleton_device(dp, rows, fx.alpha, max_len, bins=bins)
    ln = PD.length_device(dp, sk, bins.alpha_dev, su_seq, b.seq_mass)
    names = [None] + [MASS_NAMES[m.mass][0] for m in dp.masses[1:]]
    n_len = n_err = n_dup = 0
    for g in range(n):
        want = _mirror_outcome(obs[offsets[g]:offsets[g + 1]], su_seq[g], b.seq_mass[g], max_len[g], engine,
                               mod_rate)
        fm = pipeline.mask_rows(fx.alpha[g:g + 1], len(dp.masses))[0]
        assert [0] + [dp.masses[r].mass for r in range(1, len(dp.masses)) if fm[r]] == want["filter_masses"], g
        o4 = int(rows.peak_off[g].item()) * 4
        al = rows.alive[o4:o4 + int(rows.rows[g].item())].cpu().numpy().astype(bool)
        assert np.flatnonzero(al).tolist() == want["filter_kept"], g
        n_dup += want["dup_thr_keys"] > 0
        assert (sk.status[2 * g:2 * g + 2] == _native.WALK_DONE).all(), (g, sk.status[2 * g:2 * g + 2])
        got = PD.skeleton_frames(dp, rows, sk, g)
        for side in ("START", "END"):
            assert got[side] == want[side], (g, side)
        kept = pipeline.mask_rows(ln.alpha[g:g + 1], len(dp.masses))[0]
        assert [0] + [dp.masses[r].mass for r in range(1, len(dp.masses)) if kept[r]] == want["masses"], g
        if want["seq_len"] is None:
            assert int(ln.status[g]) == _native.JAC_NO_LENGTH, (g, int(ln.status[g]))
            n_err += 1
        elif want["seq_len"] == "IndexError":
            assert int(ln.status[g]) == _native.JAC_INDEX, g
            n_err += 1
        else:
            assert int(ln.status[g]) == _native.JAC_OK and int(ln.seq_len[g]) == want["seq_len"], \
                (g, int(ln.status[g]), int(ln.seq_len[g]), want["seq_len"], int(ln.lower[g]), int(ln.upper[g]))
            L = int(ln.seq_len[g])
            comb = ln.comb[int(ln.comb_off[g]):int(ln.comb_off[g]) + L].cpu().numpy().view(np.uint64)
            got_c = [sorted(names[r] for r in range(1, len(names)) if (int(c[r >> 6]) >> (r & 63)) & 1) for c in comb]
            assert got_c == want["combined"], g
            n_len += 1
    assert n_len >= n // 2
    if clean:
        assert n_dup >= n // 4, n_dup  # the scenario is present, not just allowed
    if variant in ("short_fragments_missing", "low_modification_rate"):
        assert sk.requeries > 0 or bins.deferred["queries"] > 0
        import torch

        # tiny lane capacities: most sides outgrow them and walk again at the
        # big ones (fresh slots), suspended sides resume in either slot kind
        sk2 = PD.skeleton_device(dp, rows, fx.alpha, max_len, bins=bins, caps=(4, 2), big_caps=(64, 32))
        assert sk2.launches > sk.launches
        assert (sk2.status == sk.status).all()
        for x, y in ((sk.skel, sk2.skel), (sk.min_end, sk2.min_end), (sk.max_end, sk2.max_end),
                     (sk.kept, sk2.kept)):
            assert torch.equal(x, y)


@pytest.mark.parametrize("variant", ["full_ladders", "short_fragments_missing", "low_modification_rate",
                                     "noise_free", "noise_free_exact"])
def test_device_synthetic_vs_reference(variant):
    """Stages 2-5 and the skeleton-based reduction on the device over 48
    synthetic spectra per variant against the REFERENCE's own results
    (synth_stages.json.gz, tests/golden/make_synth_golden.py: classify_fragments,
    Predictor.filter_by_explanation, SkeletonBuilder._predict_skeleton per
    side, select_sequence_length_with_jaccard with both
    compute_sequence_length_bound calls, combine_skeleton_sequences, and
    Predictor.predict up to the skeleton-based _reduce_alphabet, all run
    unmodified): final alphabet and kept fragments, each side's skeleton /
    kept fragments / min_end / max_end, the skeleton alphabet, both bounds,
    the length (or its exception), the combined skeleton, build_skeleton's
    fragments and the reduction's alphabet and fragments.  Child process
    under the reference run's hash seed (the walk orders explanations as
    CPython's sets do)."""
    import os
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, PYTHONHASHSEED="0")
    p = subprocess.run([sys.executable, os.path.join(here, "_synth_check.py"), variant, "device"], env=env,
                       capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert f"synth ok {variant} device" in p.stdout


def test_device_pipeline_big_spectra(engine):
    """Spectra of ~3000 peaks (more than 2048 rows: the *_big variants of the
    row kernels in HBM slices, sst_pipe_reserve_rows) batched with ordinary
    ones: classify / fixpoint / bins against the host-driven stages (host
    sliding windows answered by explain_pairs_alpha), and the big spectra's
    skeleton walk, Jaccard length and combined skeleton against the
    per-spectrum host mirrors."""
    from spectrseqtools_amd import _native, pipeline, pipeline_device as PD
    from spectrseqtools_amd.mass_explanation import MASS_NAMES
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE, build_breakage_dict
    from spectrseqtools_amd.synthetic import make_spectra

    small = make_spectra(40, seed=59, len_range=(6, 14))
    # 20-nt sequences with ~2 900 noise peaks each (most of them valid below
    # the sequence mass: > 2 048 rows)
    big = make_spectra(2, seed=61, len_range=(20, 20), noise_frac=24.0)
    parts, seq_mass = [], []
    for i in range(42):  # the big spectra at positions 7 and 30
        src, g = (big, 0) if i == 7 else (big, 1) if i == 30 else (small, i - (i > 7) - (i > 30))
        parts.append(src.observed[src.offsets[g]:src.offsets[g + 1]])
        seq_mass.append(src.seq_mass[g])
    obs = np.concatenate(parts)
    offsets = np.concatenate([[0], np.cumsum([len(x) for x in parts])])
    seq_mass = np.asarray(seq_mass)
    n = len(parts)
    assert max(len(x) for x in parts) > 2500
    bd = build_breakage_dict(555.1294, 455.1491)
    w_full = [k for k, v in bd.items() if "START_END" in v][0]
    su_seq = seq_mass - w_full * TOLERANCE
    seq = SequenceInformation(max_len=20, su_mass=float(su_seq[0]), obs_mass=float(seq_mass[0]),
                              modification_rate=0.5)
    dp = DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=MATCHING_THRESHOLD,
                                 precision=TOLERANCE, seq=seq, engine=engine)
    max_len = pipeline.max_len_of(su_seq, TOLERANCE, min(m.mass for m in dp.masses[1:]))
    c = pipeline.classify(obs, offsets, su_seq, dp, bd)
    rows = PD.classify_device(dp, obs, offsets, su_seq, bd)
    cnt = rows.rows.cpu().numpy()
    assert np.array_equal(cnt, np.diff(c.offsets))
    assert cnt[7] > 2048 and cnt[30] > 2048, cnt[[7, 30]]
    slot = (4 * offsets[:-1])[c.spec] + (np.arange(len(c.spec)) - c.offsets[c.spec])
    assert np.array_equal(rows.su.cpu().numpy()[slot], c.su)
    fx_h = pipeline.filter_fixpoint(c, dp, max_len, EXPLANATION_MASSES)
    fx_d = PD.fixpoint_device(dp, rows, max_len)
    assert np.array_equal(fx_d.alpha, fx_h.alpha)
    assert np.array_equal(fx_d.rounds, fx_h.rounds)
    assert np.array_equal(rows.alive.cpu().numpy()[slot].astype(bool), fx_h.alive)
    c3 = pipeline.subset(c, fx_h.alive)
    q3 = pipeline.bin_queries(c3)
    st3, cnt3, _, _ = dp.device_table.explain_pairs_alpha(q3.diff, q3.thr, q3.spec, fx_h.alpha, dp.tolerance,
                                                          dp.precision)
    order = np.lexsort((q3.side, q3.spec))
    db = PD.bins_device(dp, rows, fx_d.alpha)
    assert np.array_equal(np.diff(db.q_off), np.bincount(q3.spec, minlength=n))
    assert np.array_equal(db.status.cpu().numpy(), st3[order])
    assert np.array_equal(db.count.cpu().numpy().astype(np.int64), cnt3[order].astype(np.int64))
    # stages 4-5 for the big spectra (and a few ordinary ones) against the mirrors
    bins = PD.bins_device(dp, rows, fx_d.alpha, max_len=max_len)
    sk = PD.skeleton_device(dp, rows, fx_d.alpha, max_len, bins=bins)
    ln = PD.length_device(dp, sk, bins.alpha_dev, su_seq, seq_mass)
    names = [None] + [MASS_NAMES[m.mass][0] for m in dp.masses[1:]]
    for g in (7, 30, 0, 41):
        want = _mirror_outcome(obs[offsets[g]:offsets[g + 1]], su_seq[g], seq_mass[g], max_len[g], engine)
        assert (sk.status[2 * g:2 * g + 2] == _native.WALK_DONE).all(), (g, sk.status[2 * g:2 * g + 2])
        got = PD.skeleton_frames(dp, rows, sk, g)
        for side in ("START", "END"):
            assert got[side] == want[side], (g, side)
        kept = pipeline.mask_rows(ln.alpha[g:g + 1], len(dp.masses))[0]
        assert [0] + [dp.masses[r].mass for r in range(1, len(dp.masses)) if kept[r]] == want["masses"], g
        if want["seq_len"] is None:
            assert int(ln.status[g]) == _native.JAC_NO_LENGTH, g
        elif want["seq_len"] == "IndexError":
            assert int(ln.status[g]) == _native.JAC_INDEX, g
        else:
            assert int(ln.status[g]) == _native.JAC_OK and int(ln.seq_len[g]) == want["seq_len"], g
            L = int(ln.seq_len[g])
            comb = ln.comb[int(ln.comb_off[g]):int(ln.comb_off[g]) + L].cpu().numpy().view(np.uint64)
            got_c = [sorted(names[r] for r in range(1, len(names)) if (int(c_[r >> 6]) >> (r & 63)) & 1)
                     for c_ in comb]
            assert got_c == want["combined"], g


def test_device_pipeline_limits(engine):
    """The reference has no peak or length limit (fragment_classification.py:
    17-101, cli.py:161-172): a spectrum of ~6 000 peaks (more than the LDS
    classify kernel's 4 096: k_classify_rows_big in the HBM slices, peaks in
    random order) and one of max_len ~150 (a 140-nt sequence, peaks below
    20 kDa; the walk's positions above 126) batched with ordinary spectra,
    through every stage -- classify / fixpoint / bins against the host-driven
    stages, the walk, the Jaccard stage (the long one's bounds leave the
    reduced table: the reference raises there) and the skeleton-based
    reduction against the per-spectrum host mirrors."""
    from spectrseqtools_amd import _native, pipeline, pipeline_device as PD
    from spectrseqtools_amd.fragment_classification import classify_fragments
    from spectrseqtools_amd.frame import Frame
    from spectrseqtools_amd.mass_explanation import MASS_NAMES
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE, build_breakage_dict
    from spectrseqtools_amd.prediction import Predictor
    from spectrseqtools_amd.synthetic import make_spectra

    rng = np.random.default_rng(83)
    small = make_spectra(10, seed=71, len_range=(6, 14))
    wide = make_spectra(1, seed=73, len_range=(20, 20))
    o_wide = wide.observed[:wide.offsets[1]]
    # 6 000 peaks: mostly light noise (rarely a valid mass below 1.5 kDa), some heavy
    o_wide = np.concatenate([o_wide, rng.uniform(300.0, 1500.0, 5200), rng.uniform(1500.0, 8000.0, 800)])
    o_wide = o_wide[rng.permutation(len(o_wide))]
    long_ = make_spectra(1, seed=79, len_range=(140, 140), internal_per_nt=1)
    o_long = long_.observed[:long_.offsets[1]]
    o_long = o_long[o_long < 20000.0]  # the full table ends at 22.16 kDa: is_valid_mass would raise above
    parts = [small.observed[small.offsets[g]:small.offsets[g + 1]] for g in range(10)]
    seq_mass = list(small.seq_mass)
    parts.insert(3, o_wide)
    seq_mass.insert(3, wide.seq_mass[0])
    parts.insert(8, o_long)
    seq_mass.insert(8, long_.seq_mass[0])
    obs = np.concatenate(parts)
    offsets = np.concatenate([[0], np.cumsum([len(x) for x in parts])])
    seq_mass = np.asarray(seq_mass)
    n = len(parts)
    assert len(parts[3]) > 6000
    bd = build_breakage_dict(555.1294, 455.1491)
    w_full = [k for k, v in bd.items() if "START_END" in v][0]
    su_seq = seq_mass - w_full * TOLERANCE
    seq = SequenceInformation(max_len=20, su_mass=float(su_seq[0]), obs_mass=float(seq_mass[0]),
                              modification_rate=0.5)
    dp = DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=MATCHING_THRESHOLD,
                                 precision=TOLERANCE, seq=seq, engine=engine)
    max_len = pipeline.max_len_of(su_seq, TOLERANCE, min(m.mass for m in dp.masses[1:]))
    assert max_len[8] > 140
    c = pipeline.classify(obs, offsets, su_seq, dp, bd)
    rows = PD.classify_device(dp, obs, offsets, su_seq, bd)
    cnt = rows.rows.cpu().numpy()
    assert np.array_equal(cnt, np.diff(c.offsets))
    slot = (4 * offsets[:-1])[c.spec] + (np.arange(len(c.spec)) - c.offsets[c.spec])
    assert np.array_equal(rows.su.cpu().numpy()[slot], c.su)
    assert np.array_equal(rows.obs.cpu().numpy()[slot], c.obs)
    fx_h = pipeline.filter_fixpoint(c, dp, max_len, EXPLANATION_MASSES)
    fx_d = PD.fixpoint_device(dp, rows, max_len)
    assert np.array_equal(fx_d.alpha, fx_h.alpha)
    assert np.array_equal(rows.alive.cpu().numpy()[slot].astype(bool), fx_h.alive)
    alive_fx = rows.alive.cpu().numpy().copy()
    bins = PD.bins_device(dp, rows, fx_d.alpha, max_len=max_len)
    sk = PD.skeleton_device(dp, rows, fx_d.alpha, max_len, bins=bins)
    ln = PD.length_device(dp, sk, bins.alpha_dev, su_seq, seq_mass)
    post = PD.post_skeleton_device(dp, rows, sk, ln)
    names = [None] + [MASS_NAMES[m.mass][0] for m in dp.masses[1:]]
    for g in (3, 8, 0):
        o = obs[offsets[g]:offsets[g + 1]]
        want = _mirror_outcome(o, su_seq[g], seq_mass[g], max_len[g], engine)
        o4 = int(rows.peak_off[g].item()) * 4
        assert np.flatnonzero(alive_fx[o4:o4 + int(cnt[g])]).tolist() == want["filter_kept"], g
        assert (sk.status[2 * g:2 * g + 2] == _native.WALK_DONE).all(), (g, sk.status[2 * g:2 * g + 2])
        got = PD.skeleton_frames(dp, rows, sk, g)
        for side in ("START", "END"):
            assert got[side] == want[side], (g, side)
        kept = pipeline.mask_rows(ln.alpha[g:g + 1], len(dp.masses))[0]
        assert [0] + [dp.masses[r].mass for r in range(1, len(dp.masses)) if kept[r]] == want["masses"], g
        st = int(ln.status[g])
        if want["seq_len"] is None:  # the reference raised: no length fits, or a bound left the table
            assert st in (_native.JAC_NO_LENGTH, _native.JAC_BOUNDS), (g, st)
            if g == 8:
                assert st == _native.JAC_BOUNDS and int(ln.lb_status[g]) == _native.SST_OUT_OF_TABLE, g
        elif want["seq_len"] == "IndexError":
            assert st == _native.JAC_INDEX, g
        else:
            assert st == _native.JAC_OK and int(ln.seq_len[g]) == want["seq_len"], g
            L = int(ln.seq_len[g])
            comb = ln.comb[int(ln.comb_off[g]):int(ln.comb_off[g]) + L].cpu().numpy().view(np.uint64)
            got_c = [sorted(names[r] for r in range(1, len(names)) if (int(c_[r >> 6]) >> (r & 63)) & 1)
                     for c_ in comb]
            assert got_c == want["combined"], g
        # Predictor.predict up to the skeleton-based reduction (mirror, fresh table)
        seq_g = SequenceInformation(max_len=int(max_len[g]), su_mass=float(su_seq[g]), obs_mass=float(seq_mass[g]),
                                    modification_rate=0.5)
        dp_g = DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=MATCHING_THRESHOLD,
                                       precision=TOLERANCE, seq=seq_g, engine=engine)
        try:
            rec = {}
            fr = classify_fragments(Frame({"observed_mass": list(map(float, o))}), dp_g, bd)
            out = Predictor(dp_g, EXPLANATION_MASSES).predict_skeleton_stage(fr, record=rec)
            if out is None:
                assert int(post.active[g]) == 0, g
                continue
            assert int(post.active[g]) == 1, g
            for key, frame, alive in (("build_skeleton", rec["build_skeleton"], post.alive_skeleton),
                                      ("reduction", out[1], post.alive)):
                idx = np.flatnonzero(alive[o4:o4 + int(cnt[g])].cpu().numpy())
                assert idx.tolist() == frame.get_column("index").to_list(), (g, key)
                assert post.min_end[o4 + idx].cpu().numpy().tolist() == frame.get_column("min_end").to_list()
                assert post.max_end[o4 + idx].cpu().numpy().tolist() == frame.get_column("max_end").to_list()
        finally:
            dp_g.close()


def test_device_fixpoint_rounds_vs_oracle_rebuilt_tables(engine):
    """Every filter_by_explanation round of the device fixpoint (k_fix_round:
    the round's window / singleton answers on the spectrum's alphabet, the
    dict's last-writer semantics, the reduced alphabet; k_valid_alpha: the
    rows is_valid_mass keeps on the reduced table) on 600 synthetic spectra
    against the CPU oracle on each round's REBUILT reduced table
    (set_up_bit_table over the kept rows, mass_table.py:94-121), the queries
    produced by the host-native sliding window (prediction.py:261-329)."""
    from concurrent.futures import ThreadPoolExecutor

    import _oracle as oracle
    from spectrseqtools_amd import pipeline, pipeline_device as PD
    from spectrseqtools_amd._native import su_diff_queries
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation
    from spectrseqtools_amd.masses import (EXPLANATION_MASSES, MATCHING_THRESHOLD, PHOSPHATE_LINK_MASS, TOLERANCE,
                                           build_breakage_dict)
    from spectrseqtools_amd.synthetic import make_spectra

    n = 600
    b = make_spectra(n, seed=53)
    bd = build_breakage_dict(555.1294, 455.1491)
    w_full = [k for k, v in bd.items() if "START_END" in v][0]
    su_seq = b.seq_mass - w_full * TOLERANCE
    seq = SequenceInformation(max_len=20, su_mass=float(su_seq[0]), obs_mass=float(b.seq_mass[0]),
                              modification_rate=0.5)
    dp = DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=MATCHING_THRESHOLD,
                                 precision=TOLERANCE, seq=seq, engine=engine)
    tol = dp.tolerance
    max_len = pipeline.max_len_of(su_seq, TOLERANCE, min(m.mass for m in dp.masses[1:]))
    rows = PD.classify_device(dp, b.observed, b.offsets, su_seq, bd)
    fx = PD.fixpoint_device(dp, rows, max_len, record=True)
    c = PD.to_classified(rows, alive_only=False)  # every classified row, spectrum-major in SU order
    off = rows.peak_off.cpu().numpy()
    slot = 4 * off[:-1][c.spec] + (np.arange(len(c.spec)) - c.offsets[c.spec])
    ms_all = [m.mass for m in dp.masses]
    N = len(ms_all)
    is_mod = np.array([m.is_modification for m in dp.masses])
    rate = [m.modification_rate for m in dp.masses]
    canon = pipeline.row_masks((~is_mod & (np.arange(N) > 0))[None, :])[0]
    max_w = max(EXPLANATION_MASSES.get_column("monoisotopic_mass").to_list()) + PHOSPHATE_LINK_MASS
    side = np.array([("START" in nm) | (("END" in nm) << 1) for nm in c.names], dtype=np.uint8)
    flags = side[c.brk] | (c.singleton.astype(np.uint8) << 2)
    tables = {}

    def table(mask):
        key = (int(mask[0]), int(mask[1]))
        if key not in tables:
            rows_k = pipeline.mask_rows(np.asarray(mask, np.uint64)[None, :], N)[0]
            keep = [0] + [r for r in range(1, N) if rows_k[r]]
            ms = [ms_all[r] for r in keep]
            tables[key] = (keep, oracle.build_table(ms, max(ms) * 35, 32))
        return tables[key]

    def check(task):
        k, g, alpha_in, alive_in, alpha_out, alive_out = task
        keep, tab = table(alpha_in)
        alph = oracle.Alphabet([ms_all[r] for r in keep], [bool(is_mod[r]) for r in keep],
                               [round(int(max_len[g]) * rate[r]) for r in keep])
        A = round(dp.seq.modification_rate * int(max_len[g]))
        idx = np.arange(c.offsets[g], c.offsets[g + 1])[alive_in]
        d, t, _, kind = su_diff_queries(c.su[idx], c.obs[idx], flags[idx], np.array([0, len(idx)]), max_w, tol)
        last = {}  # the dict: key -> last writer's answer (rows of its candidates) or None / []
        for i in range(len(d)):
            st, sols, n_e, _ = oracle.explain_table(tab, 32, alph, d[i], t[i], tol, A)
            assert st >= 0, (k, g, i)
            if kind[i] == 2 or sols:  # singletons always, side pairs with >= 1 explanation
                last[float(d[i])] = [tuple(keep[x] for x in s) for s in sols]
        used = np.zeros(N, bool)
        for v in last.values():
            for s in v:
                used[list(s)] = True
        want = canon | (np.asarray(alpha_in, np.uint64) & pipeline.row_masks(used[None, :])[0])
        assert np.array_equal(want, alpha_out), (k, g)
        changed = pipeline.mask_rows(want[None, :], N).sum() != pipeline.mask_rows(
            np.asarray(alpha_in, np.uint64)[None, :], N).sum()
        exp_alive = alive_in.copy()
        if changed:
            keep2, tab2 = table(want)
            v = oracle.is_valid_batch(tab2, 32, c.su[idx], tol * c.obs[idx], tol)
            assert (v >= 0).all(), (k, g)
            exp_alive[alive_in] = v == 1
        assert np.array_equal(exp_alive, alive_out), (k, g)
        return len(d)

    full = pipeline.row_masks((np.arange(N) > 0)[None, :])[0]
    alpha_prev = np.repeat(full[None, :], n, axis=0)
    alive_prev = np.ones(len(c.spec), bool)
    tasks = []
    for k, (act, alpha_k, alive_k) in enumerate(fx.history):
        alive_now = alive_k[slot]
        for g in np.flatnonzero(act):
            sl = slice(c.offsets[g], c.offsets[g + 1])
            tasks.append((k, int(g), alpha_prev[g].copy(), alive_prev[sl].copy(), alpha_k[g].copy(),
                          alive_now[sl].copy()))
        alpha_prev = alpha_k.copy()
        alive_prev = alive_now.copy()
    table(full)  # shared by every first round
    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 4)) as ex:
        n_q = sum(ex.map(check, tasks))
    assert len(fx.history) >= 3 and n_q > 100_000 and len(tasks) >= 2 * n
