#!/usr/bin/env python3
"""Golden vectors for the config-5 stages on SYNTHETIC spectra, from the
REFERENCE itself (read-only at /root/reference; build container only).

TEST INFRASTRUCTURE.  Same set-up as make_callers_golden.py / make_post_golden.py
(the pandas-backed polars stand-in and the import-only stand-ins; every
reference function runs unmodified, the generator only observes).  The
spectra are tests/_synth_cases.py's (synthetic.make_spectra, 48 per variant:
noise-free ones repeat SU differences exactly at different observed masses;
low-modification-rate ones run with modification_rate 0.05, where budgets bind
on pair windows).  Per spectrum, as cli.py:149-176 sets it up (max_len from the
SU sequence mass, the full alphabet, MATCHING_THRESHOLD):

  filter     classify_fragments (fragment_classification.py:17-101) on the
             observed masses, Predictor.filter_by_explanation
             (prediction.py:170-202): every _reduce_alphabet round's alphabet
             and kept fragment indices
  skeleton   SkeletonBuilder._predict_skeleton per side (skeleton_building.py:
             114-196): skeleton, kept fragments, min_end, max_end; then
             select_sequence_length_with_jaccard (:315-370): the skeleton
             alphabet, both compute_sequence_length_bound results, the chosen
             length, combine_skeleton_sequences (:494-516) at it
  post       Predictor.predict (prediction.py:63-103) from a fresh table up to
             the skeleton-based _reduce_alphabet: build_skeleton's fragments
             and the fragments / alphabet after the reduction (MILP-free: the
             stand-in pulp makes select_sequence_length_with_lp return -1)

Explanation lists follow Python set order (hash-seed dependent in the
reference too): run with PYTHONHASHSEED=0, the seed the tests' child process
uses.

Usage:  PYTHONHASHSEED=0 XDG_CACHE_HOME=/tmp/sst_refcache \\
        python tests/golden/make_synth_golden.py [variant ...] [--jobs 7] [--n 48]
"""
import hashlib
import multiprocessing as mp
import os
import sys
import time
import typing

if not hasattr(typing, "Self"):  # Python 3.10: prediction.py:3 imports it for annotations only
    typing.Self = typing.Any

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE)]
sys.path.append(os.path.dirname(os.path.dirname(HERE)))  # spectrseqtools_amd (the inputs' generator only)

import numpy as np  # noqa: E402

import make_callers_golden as CG  # noqa: E402  (sets sys.path: stand-ins first, then the reference)
import make_golden as G  # noqa: E402
import make_post_golden as PG  # noqa: E402
import polars as pl  # noqa: E402  (the stand-in)
import _synth_cases as SC  # noqa: E402  (the tests' inputs; our synthetic generator, no GPU)

import spectrseqtools.fragment_classification as FC  # noqa: E402

M, MT, EM = G.M, G.MT, G.EM


def obs_digest(obs):
    return hashlib.sha256(np.ascontiguousarray(obs, dtype=np.float64).tobytes()).hexdigest()


def new_dp(su, seq_mass, max_len, mod_rate):
    si = MT.SequenceInformation(max_len=int(max_len), su_mass=float(su), obs_mass=float(seq_mass),
                                modification_rate=mod_rate)
    return MT.DynamicProgrammingTable(EM, compression_rate=32, tolerance=M.MATCHING_THRESHOLD, precision=M.TOLERANCE,
                                      seq=si)


def run_spectrum(job):
    variant, g, obs, su, seq_mass, max_len, mod_rate = job
    t0 = time.time()
    bd = M.build_breakage_dict(*SC.TAGS)
    frame = pl.DataFrame({"observed_mass": [float(x) for x in obs]})
    dp = new_dp(su, seq_mass, max_len, mod_rate)
    classified = FC.classify_fragments(frame, dp, bd)
    prepared = (classified.with_row_index(name="orig_index").sort("standard_unit_mass")
                .with_row_index(name="index"))
    prepared = prepared.with_columns(pl.lit(0, dtype=pl.Int64).alias("min_end"),
                                     pl.lit(-1, dtype=pl.Int64).alias("max_end"))
    frags, expl, rounds = CG.filter_by_explanation(prepared, dp)
    rec = {"n_peaks": len(obs), "obs_sha256": obs_digest(obs), "su_mass": float(su), "seq_mass": float(seq_mass),
           "max_len": int(max_len), "mod_rate": mod_rate, "n_classified": len(classified),
           "filter": {"rounds": rounds, "masses": [int(m.mass) for m in dp.masses],
                      "kept_index": [int(x) for x in frags.get_column("index").to_list()]}}
    sk = CG.skeleton(frags, expl, dp)
    for side in ("START", "END"):
        sk[side].pop("queries")
    rec["skeleton"] = sk
    dp2 = new_dp(su, seq_mass, max_len, mod_rate)
    rec["post"] = PG.predict_to_reduction(FC.classify_fragments(frame, dp2, bd), dp2)
    rec["seconds"] = round(time.time() - t0, 1)
    return variant, g, rec


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    jobs = int(sys.argv[sys.argv.index("--jobs") + 1]) if "--jobs" in sys.argv else 7
    n = int(sys.argv[sys.argv.index("--n") + 1]) if "--n" in sys.argv else 48
    args = [a for a in args if not a.isdigit()]
    variants = args or ["noise_free", "low_modification_rate"]
    assert os.environ.get("PYTHONHASHSEED") == "0", "run with PYTHONHASHSEED=0"
    t0 = time.time()
    work, out = [], {}
    for v in variants:
        d = SC.variant_inputs(v)
        out[v] = {"mod_rate": d["mod_rate"], "spectra": [None] * n}
        for g in range(n):
            o = d["obs"][d["offsets"][g]:d["offsets"][g + 1]]
            work.append((v, g, o, d["su_seq"][g], d["seq_mass"][g], d["max_len"][g], d["mod_rate"]))
    done = 0
    with mp.get_context("fork").Pool(jobs) as pool:
        for v, g, rec in pool.imap_unordered(run_spectrum, work):
            out[v]["spectra"][g] = rec
            done += 1
            print(f"  {v}[{g}]: {rec['n_peaks']} peaks, max_len {rec['max_len']}, "
                  f"seq_len {rec['skeleton']['jaccard']['seq_len']}, {rec['seconds']}s ({done}/{len(work)}, "
                  f"{time.time() - t0:.0f}s)", flush=True)
    out["_meta"] = {"pythonhashseed": os.environ.get("PYTHONHASHSEED"), "n": n, "seconds": round(time.time() - t0)}
    G.dump("synth_stages.json.gz", out, gz=True)


if __name__ == "__main__":
    main()
