#!/usr/bin/env python3
"""Golden vectors for the hot path's CALLERS, from the REFERENCE itself
(read-only at /root/reference; build container only, never the GPU box).

TEST INFRASTRUCTURE.  Uses make_golden.py's set-up (the pandas-backed polars
stand-in in tests/golden/standin/, the reference's own DynamicProgrammingTable,
is_valid_mass and explain_mass_with_table) plus import-only stand-ins for the
modules prediction.py / skeleton_building.py import but never use on these
paths: loguru (logger.warning only), pulp (linear_program.py; every name
raises), ms_deisotope and clr_loader (common.py's RAW reader), and typing.Self
(Python 3.10; annotations only).  Every function below runs UNMODIFIED; the
generator only observes (instance-level wrappers that record what the
reference's own methods return).

  callers.json.gz, per reference test spectrum (tests/testcases/test_0[1-8]):
    classify   the output frame of fragment_classification.classify_fragments
               (:17-101)
    filter     Predictor.filter_by_explanation (prediction.py:170-202) on that
               frame as Predictor.predict prepares it (:68-80): the alphabet and
               the fragment `index` values kept after every _reduce_alphabet
               round (:204-227), and the returned explanation dict (diff ->
               sorted row-index tuples, or None)
    skeleton   SkeletonBuilder._predict_skeleton (skeleton_building.py:114-196)
               per side (START, END) with those explanations on the reduced
               table: the skeleton (sorted names per position), the kept
               fragments' index / min_end / max_end, the explain queries it
               issued; then select_sequence_length_with_jaccard (:315-370) on
               the two skeletons: its alphabet reduction, both
               compute_sequence_length_bound results and the chosen length, and
               combine_skeleton_sequences (:494-516) at that length

Set order: explanation lists follow Python set iteration of name tuples
(hash-seed dependent in the reference); the generator runs with
PYTHONHASHSEED=0 and records whether a second seed changes any skeleton
(`seed_independent`).

Usage:  PYTHONHASHSEED=0 XDG_CACHE_HOME=/tmp/sst_refcache python tests/golden/make_callers_golden.py
"""
import os
import subprocess
import sys
import time
import typing

if not hasattr(typing, "Self"):  # Python 3.10: prediction.py:3 imports it for annotations only
    typing.Self = typing.Any

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden as G  # noqa: E402  (sets sys.path: stand-ins first, then the reference)
import polars as pl  # noqa: E402  (the stand-in)
import yaml  # noqa: E402

import spectrseqtools.fragment_classification as FC  # noqa: E402
import spectrseqtools.prediction as PR  # noqa: E402
import spectrseqtools.skeleton_building as SB  # noqa: E402

M, MT, ME, EM, REF = G.M, G.MT, G.ME, G.EM, G.REF


def _jsonable(v):
    if hasattr(v, "item"):
        v = v.item()
    return v


def frame_dump(df):
    return {"columns": df.columns, "rows": [[_jsonable(x) for x in r] for r in df.rows()]}


def expl_rows(dp, expl):
    """A calculate_explanations list (Explanation objects) or None -> sorted
    row-index tuples of dp's alphabet."""
    return None if expl is None else [list(t) for t in G.rows_of(dp, [tuple(e) for e in expl])]


def skeleton_dump(sk):
    return [sorted(p) for p in sk]


def filter_by_explanation(frame, dp):
    """Predictor.filter_by_explanation, unmodified, with its _reduce_alphabet
    observed per round."""
    pred = PR.Predictor(dp, EM)
    rounds = []
    orig = pred._reduce_alphabet

    def observed(nucleotide_list, fragments):
        out = orig(nucleotide_list, fragments)
        rounds.append({"masses": [int(m.mass) for m in dp.masses],
                       "kept_index": [int(x) for x in out.get_column("index").to_list()]})
        return out

    pred._reduce_alphabet = observed
    frags, expl = pred.filter_by_explanation(frame)
    return frags, expl, rounds


def skeleton(frags, expl, dp):
    """SkeletonBuilder._predict_skeleton per side and the Jaccard length
    selection, unmodified, with explain / length-bound calls observed."""
    sb = SB.SkeletonBuilder(explanations=expl, dp_table=dp)
    queries = []
    orig_calc = SB.calculate_explanations

    def calc(diff, threshold, dp_table):
        r = orig_calc(diff, threshold, dp_table)
        queries.append([diff, threshold, expl_rows(dp_table, r)])
        return r

    bounds = []
    orig_lb = SB.compute_sequence_length_bound

    def lb(dp_table, dir):
        v = orig_lb(dp_table=dp_table, dir=dir)
        bounds.append([dir, int(v)])
        return v

    SB.calculate_explanations, SB.compute_sequence_length_bound = calc, lb
    try:
        out = {}
        for side in ("START", "END"):
            queries.clear()
            n_warn = len(SB.logger.records)
            sk, fr = sb._predict_skeleton(fragments=frags.filter(pl.col("breakage").str.contains(side)),
                                          skeleton_seq=[set() for _ in range(dp.seq.max_len)])
            out[side] = {"skeleton": skeleton_dump(sk), "sk_sets": sk,
                         "kept_index": [int(x) for x in fr.get_column("index").to_list()],
                         "min_end": [int(x) for x in fr.get_column("min_end").to_list()],
                         "max_end": [int(x) for x in fr.get_column("max_end").to_list()],
                         "queries": list(queries), "warnings": len(SB.logger.records) - n_warn}
        start_sk, end_sk = out["START"].pop("sk_sets"), out["END"].pop("sk_sets")[::-1]
        try:
            seq_len = sb.select_sequence_length_with_jaccard(start_skeleton=start_sk, end_skeleton=end_sk)
            combined = skeleton_dump(SB.combine_skeleton_sequences(seq_len, start_sk, end_sk))
            err = None
        except Exception as e:  # the reference raises when no length fits the sequence mass
            seq_len, combined, err = None, None, f"{type(e).__name__}: {e}"
        out["jaccard"] = {"masses": [int(m.mass) for m in dp.masses], "bounds": list(bounds), "seq_len": seq_len,
                          "combined": combined, "error": err}
        return out
    finally:
        SB.calculate_explanations, SB.compute_sequence_length_bound = orig_calc, orig_lb


def main():
    out = {}
    for tc in sorted(os.listdir(f"{REF}/tests/testcases")):
        t0 = time.time()
        base = f"{REF}/tests/testcases/{tc}"
        meta = yaml.safe_load(open(f"{base}/fragments.meta.yaml"))
        frame = pl.read_csv(f"{base}/fragments.tsv", separator="\t")
        bd = M.build_breakage_dict(meta.get("label_mass_5T", 555.1294), meta.get("label_mass_3T", 455.1491))
        su_seq = meta["sequence_mass"] - [k * M.TOLERANCE for k in bd if "START_END" in bd[k]][0]
        max_len = int(su_seq / M.TOLERANCE / G.MIN_INT)
        cutoff = meta.get("intensity_cutoff", M.DEFAULT_INTENSITY_CUTOFF)
        cid = f"callers_{tc}"
        dp = G.make_ctx(cid, max_len, M.MATCHING_THRESHOLD, su=su_seq)
        G.CTX[cid]["obs_mass"] = dp.seq.obs_mass = meta["sequence_mass"]  # cli.py:149-176
        classified = FC.classify_fragments(frame, dp, bd, intensity_cutoff=cutoff)
        rec = {"ctx": G.CTX[cid], "intensity_cutoff": cutoff, "tags": [meta.get("label_mass_5T", 555.1294),
                                                                         meta.get("label_mass_3T", 455.1491)],
               "input": frame_dump(frame), "classify": frame_dump(classified)}
        # Predictor.predict's framing (prediction.py:68-80)
        prepared = (classified.with_row_index(name="orig_index").sort("standard_unit_mass")
                    .with_row_index(name="index"))
        prepared = prepared.with_columns(pl.lit(0, dtype=pl.Int64).alias("min_end"),
                                         pl.lit(-1, dtype=pl.Int64).alias("max_end"))
        frags, expl, rounds = filter_by_explanation(prepared, dp)
        rec["filter"] = {"rounds": rounds, "explanations": {repr(k): expl_rows(dp, v) for k, v in expl.items()}}
        rec["skeleton"] = skeleton(frags, expl, dp)
        out[tc] = rec
        print(f"  {tc}: {len(frame)} fragments -> {len(classified)} classified, "
              f"{len(rec['filter']['rounds'])} reduction rounds, skeleton length "
              f"{rec['skeleton']['jaccard']['seq_len']}, {time.time() - t0:.0f}s", flush=True)
        del dp
    if "--probe-seed" in sys.argv:  # child run under another hash seed: skeletons only
        import json
        print("SKELETONS=" + json.dumps({tc: r["skeleton"] for tc, r in out.items()}))
        return
    # the same skeletons under another PYTHONHASHSEED?
    import json
    env = dict(os.environ, PYTHONHASHSEED="12345")
    probe = subprocess.run([sys.executable, os.path.abspath(__file__), "--probe-seed"], env=env, check=True,
                           capture_output=True, text=True).stdout
    other = json.loads(probe.split("SKELETONS=", 1)[1])
    for tc in out:
        out[tc]["skeleton"]["seed_independent"] = other[tc] == json.loads(json.dumps(out[tc]["skeleton"]))
        print(f"  {tc}: skeleton seed-independent: {out[tc]['skeleton']['seed_independent']}")
    out["_meta"] = {"pythonhashseed": os.environ.get("PYTHONHASHSEED")}
    G.dump("callers.json.gz", out, gz=True)


if __name__ == "__main__":
    main()
