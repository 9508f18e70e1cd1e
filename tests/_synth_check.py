"""Child-process check (run with PYTHONHASHSEED=0, the seed of the reference
run in tests/golden/make_synth_golden.py): config 5's stages on synthetic
spectra (tests/_synth_cases.py) against the REFERENCE's own results
(synth_stages.json.gz) -- filter_by_explanation's alphabet and kept
fragments after every round (device) and at the end, _predict_skeleton per side (skeleton, kept fragments, min_end,
max_end), select_sequence_length_with_jaccard (skeleton alphabet, both
length bounds, the length or its exception, the combined skeleton) and
Predictor.predict's skeleton-based reduction (build_skeleton's fragments,
the alphabet and fragments after _reduce_alphabet).  Explanation lists follow
CPython set order in the reference, the mirrors and the device walk alike.

usage: python tests/_synth_check.py VARIANT device      (the device-resident pipeline, all spectra)
       python tests/_synth_check.py VARIANT cpu [N]     (the host mirrors on the oracle engine, first N)
TEST INFRASTRUCTURE."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE)]

import numpy as np  # noqa: E402


def names_of(dp, mask_row):
    from spectrseqtools_amd.pipeline import mask_rows

    kept = mask_rows(np.asarray(mask_row, dtype=np.uint64).reshape(1, 2), len(dp.masses))[0]
    return [0] + [dp.masses[r].mass for r in range(1, len(dp.masses)) if kept[r]]


def jac_kind(err):
    """The reference's exception -> the device's Jaccard status name."""
    if err is None:
        return "ok"
    return "index" if err.startswith("IndexError") else "no_length"


def check_device(variant, want, d):
    import torch

    from spectrseqtools_amd import _native, pipeline_device as PD
    from spectrseqtools_amd.mass_explanation import MASS_NAMES
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE, build_breakage_dict
    import _synth_cases as SC

    eng = _native.get_engine(0)
    n = len(want)
    seq = SequenceInformation(max_len=20, su_mass=float(d["su_seq"][0]), obs_mass=float(d["seq_mass"][0]),
                              modification_rate=d["mod_rate"])
    dp = DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=MATCHING_THRESHOLD,
                                 precision=TOLERANCE, seq=seq, engine=eng)
    bd = build_breakage_dict(*SC.TAGS)
    ml = d["max_len"]
    rows = PD.classify_device(dp, d["obs"], d["offsets"], d["su_seq"], bd)
    fx = PD.fixpoint_device(dp, rows, ml, record=True)
    alive_fx = rows.alive.cpu().numpy().copy()
    bins = PD.bins_device(dp, rows, fx.alpha, max_len=ml)
    sk = PD.skeleton_device(dp, rows, fx.alpha, ml, bins=bins)
    ln = PD.length_device(dp, sk, bins.alpha_dev, d["su_seq"], d["seq_mass"])
    post = PD.post_skeleton_device(dp, rows, sk, ln)
    names = [None] + [MASS_NAMES[m.mass][0] for m in dp.masses[1:]]
    n_len = n_post = 0
    for g in range(n):
        w = want[g]
        o4 = int(rows.peak_off[g].item()) * 4
        nr = int(rows.rows[g].item())
        # every filter_by_explanation round of this spectrum: the alphabet after
        # _reduce_alphabet and the kept fragments (the reference's rounds)
        mine = [(a_, l_) for act, a_, l_ in fx.history if act[g]]
        assert len(mine) == len(w["filter"]["rounds"]) == int(fx.rounds[g]), (g, len(mine), len(w["filter"]["rounds"]))
        for k, ((a_, l_), rr) in enumerate(zip(mine, w["filter"]["rounds"])):
            assert names_of(dp, a_[g]) == rr["masses"], (g, k, "round alphabet")
            assert np.flatnonzero(l_[o4:o4 + nr]).tolist() == rr["kept_index"], (g, k, "round kept")
        assert names_of(dp, fx.alpha[g]) == w["filter"]["masses"], (g, "filter alphabet")
        assert np.flatnonzero(alive_fx[o4:o4 + nr]).tolist() == w["filter"]["kept_index"], (g, "filter kept")
        assert (sk.status[2 * g:2 * g + 2] == _native.WALK_DONE).all(), (g, sk.status[2 * g:2 * g + 2])
        got = PD.skeleton_frames(dp, rows, sk, g)
        for side in ("START", "END"):
            for key in ("skeleton", "kept_index", "min_end", "max_end"):
                assert got[side][key] == w["skeleton"][side][key], (g, side, key, got[side][key],
                                                                    w["skeleton"][side][key])
        j = w["skeleton"]["jaccard"]
        assert names_of(dp, ln.alpha[g]) == j["masses"], (g, "skeleton alphabet")
        bounds = [["lower", int(ln.lower[g])], ["upper", int(ln.upper[g])]]
        assert bounds[:len(j["bounds"])] == j["bounds"], (g, bounds, j["bounds"])
        st = int(ln.status[g])
        kind = {_native.JAC_OK: "ok", _native.JAC_INDEX: "index", _native.JAC_NO_LENGTH: "no_length"}.get(st, st)
        assert kind == jac_kind(j["error"]), (g, st, j["error"])
        if kind == "ok":
            L = int(ln.seq_len[g])
            assert L == j["seq_len"], (g, L, j["seq_len"])
            comb = ln.comb[int(ln.comb_off[g]):int(ln.comb_off[g]) + L].cpu().numpy().view(np.uint64)
            got_c = [sorted(names[r] for r in range(1, len(names)) if (int(c[r >> 6]) >> (r & 63)) & 1) for c in comb]
            assert got_c == j["combined"], g
            n_len += 1
        p = w["post"]
        if p["default"]:
            assert int(post.active[g]) == 0, (g, "post: predict returns the default")
            continue
        assert int(post.active[g]) == 1, (g, "post active")
        for key, alive in (("build_skeleton", post.alive_skeleton), ("reduction", post.alive)):
            fr = p[key]["fragments"]
            idx = np.flatnonzero(alive[o4:o4 + nr].cpu().numpy())
            assert idx.tolist() == fr["index"], (g, key, idx.tolist(), fr["index"])
            assert post.min_end[o4 + idx].cpu().numpy().tolist() == fr["min_end"], (g, key)
            assert post.max_end[o4 + idx].cpu().numpy().tolist() == fr["max_end"], (g, key)
        assert names_of(dp, post.alpha[g]) == p["reduction"]["masses"], (g, "post alphabet")
        n_post += 1
    torch.cuda.synchronize()
    return n_len, n_post


def check_cpu(variant, want, d, first):
    """The host mirrors (classify_fragments, Predictor.filter_by_explanation,
    SkeletonBuilder._predict_skeleton, select_sequence_length_with_jaccard,
    combine_skeleton_sequences, Predictor.predict_skeleton_stage) with the
    oracle behind DynamicProgrammingTable (tests/_fake_engine.py)."""
    import pytest

    import _callers_checks as C
    import _fake_engine
    from spectrseqtools_amd.fragment_classification import classify_fragments
    from spectrseqtools_amd.frame import Frame
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE, build_breakage_dict
    from spectrseqtools_amd.prediction import Predictor
    from spectrseqtools_amd.skeleton_building import SkeletonBuilder, combine_skeleton_sequences
    import _synth_cases as SC

    mp = pytest.MonkeyPatch()
    _fake_engine.install(mp)
    bd = build_breakage_dict(*SC.TAGS)
    n_len = n_post = 0

    def new_dp(g):
        seq = SequenceInformation(max_len=int(d["max_len"][g]), su_mass=float(d["su_seq"][g]),
                                  obs_mass=float(d["seq_mass"][g]), modification_rate=d["mod_rate"])
        return DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=MATCHING_THRESHOLD,
                                       precision=TOLERANCE, seq=seq)

    for g in range(min(first, len(want))):
        w = want[g]
        obs = d["obs"][d["offsets"][g]:d["offsets"][g + 1]]
        dp = new_dp(g)
        fr = classify_fragments(Frame({"observed_mass": list(map(float, obs))}), dp, bd)
        assert len(fr) == w["n_classified"], g
        pred = Predictor(dp, EXPLANATION_MASSES)
        frags, expl = pred.filter_by_explanation(C.prepared(fr))
        assert [m.mass for m in dp.masses] == w["filter"]["masses"], (g, "filter alphabet")
        assert frags.get_column("index").to_list() == w["filter"]["kept_index"], (g, "filter kept")
        sb = SkeletonBuilder(explanations=expl, dp_table=dp)
        sks = {}
        for side in ("START", "END"):
            sub = frags.filter_mask([side in b for b in frags.get_column("breakage").to_list()])
            sk, fs = sb._predict_skeleton(Frame(sub.to_dict()), [set() for _ in range(dp.seq.max_len)])
            ws = w["skeleton"][side]
            assert [sorted(p) for p in sk] == ws["skeleton"], (g, side)
            assert fs.get_column("index").to_list() == ws["kept_index"], (g, side)
            assert fs.get_column("min_end").to_list() == ws["min_end"], (g, side)
            assert fs.get_column("max_end").to_list() == ws["max_end"], (g, side)
            sks[side] = sk
        j = w["skeleton"]["jaccard"]
        try:
            L = sb.select_sequence_length_with_jaccard(start_skeleton=sks["START"], end_skeleton=sks["END"][::-1])
            assert j["error"] is None and L == j["seq_len"], (g, L, j)
            comb = [sorted(p) for p in combine_skeleton_sequences(L, sks["START"], sks["END"][::-1])]
            assert comb == j["combined"], g
            n_len += 1
        except AssertionError:
            raise
        except IndexError:
            assert jac_kind(j["error"]) == "index", (g, j["error"])
        except Exception:  # noqa: BLE001 -- the reference's bare Exception when no length fits
            assert jac_kind(j["error"]) == "no_length", (g, j["error"])
        assert [m.mass for m in dp.masses] == j["masses"], (g, "skeleton alphabet")
        # Predictor.predict up to the skeleton-based reduction, from a fresh table
        p = w["post"]
        dp2 = new_dp(g)
        rec = {}
        fr2 = classify_fragments(Frame({"observed_mass": list(map(float, obs))}), dp2, bd)
        out = Predictor(dp2, EXPLANATION_MASSES).predict_skeleton_stage(fr2, record=rec)
        if p["default"]:
            assert out is None, g
            continue
        _, frr = out
        for key, frame in (("build_skeleton", rec["build_skeleton"]), ("reduction", frr)):
            wf = p[key]["fragments"]
            assert frame.get_column("index").to_list() == wf["index"], (g, key)
            assert frame.get_column("min_end").to_list() == wf["min_end"], (g, key)
            assert frame.get_column("max_end").to_list() == wf["max_end"], (g, key)
        assert [m.mass for m in dp2.masses] == p["reduction"]["masses"], (g, "post alphabet")
        n_post += 1
    mp.undo()
    return n_len, n_post


def main():
    variant, mode = sys.argv[1], sys.argv[2]
    first = int(sys.argv[3]) if len(sys.argv) > 3 else 10 ** 9
    assert os.environ.get("PYTHONHASHSEED") == "0", "run with PYTHONHASHSEED=0"
    import hashlib

    from conftest import load_golden
    import _synth_cases as SC

    want = load_golden("synth_stages.json.gz")[variant]
    d = SC.variant_inputs(variant, n=len(want["spectra"]))
    assert d["mod_rate"] == want["mod_rate"]
    for g, w in enumerate(want["spectra"]):  # the same inputs the reference ran
        obs = d["obs"][d["offsets"][g]:d["offsets"][g + 1]]
        assert hashlib.sha256(np.ascontiguousarray(obs, dtype=np.float64).tobytes()).hexdigest() == w["obs_sha256"]
        assert (w["su_mass"], w["seq_mass"], w["max_len"]) == (float(d["su_seq"][g]), float(d["seq_mass"][g]),
                                                              int(d["max_len"][g])), g
    if mode == "device":
        n_len, n_post = check_device(variant, want["spectra"], d)
    else:
        n_len, n_post = check_cpu(variant, want["spectra"], d, first)
    print(f"synth ok {variant} {mode} lengths={n_len} post={n_post}")


if __name__ == "__main__":
    main()
