#!/usr/bin/env python3
"""Golden vectors for the hot path's CALLERS, from the REFERENCE itself
(read-only at /root/reference; build container only, never the GPU box).

TEST INFRASTRUCTURE.  Uses make_golden.py's set-up (the pandas-backed polars
stand-in in tests/golden/standin/, the reference's own DynamicProgrammingTable,
is_valid_mass and explain_mass_with_table).

  callers.json.gz, per reference test spectrum (tests/testcases/test_0[1-8]):
    classify   the output frame of the reference's own
               fragment_classification.classify_fragments (:17-101): columns and
               rows, run unmodified through the stand-in
    filter     Predictor.filter_by_explanation (prediction.py:170-202) on that
               frame as Predictor.predict prepares it (:68-80): the alphabet
               after every reduction round, the fragment `index` values kept and
               the last round's explanation dict (diff -> sorted row-index
               tuples, or None).  prediction.py cannot be imported (typing.Self,
               loguru, pulp), so collect_diff_explanations_for_su /
               collect_explanations_per_side / _reduce_alphabet are restated
               here line for line; every explain / is_valid answer and every
               alphabet reduction (table rebuild) is the reference's own code.

Usage:  python tests/golden/make_callers_golden.py
"""
import csv
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden as G  # noqa: E402  (sets sys.path: stand-in first, then the reference)
import polars as pl  # noqa: E402  (the stand-in)
import yaml  # noqa: E402

import spectrseqtools.fragment_classification as FC  # noqa: E402

M, MT, ME, EM, REF = G.M, G.MT, G.ME, G.EM, G.REF


def _jsonable(v):
    if hasattr(v, "item"):
        v = v.item()
    return v


def frame_dump(df):
    return {"columns": df.columns, "rows": [[_jsonable(x) for x in r] for r in df.rows()]}


def wrap_rows(dp, names_set):
    return None if names_set is None else [list(t) for t in G.rows_of(dp, names_set)]


def calculate_explanations(diff, threshold, dp):
    """common.py:47-65 (the module imports ms_deisotope / mono at load)."""
    r = ME.explain_mass_with_table(diff, dp_table=dp,
                                   max_modifications=round(dp.seq.modification_rate * dp.seq.max_len),
                                   threshold=threshold).explanations
    return r  # the name set; list(Explanation) wrapping is order-only


def per_side(rows, dp):
    """prediction.py:286-329 restated (rows: (su, obs) sorted by su)."""
    maxw = max(EM.get_column("monoisotopic_mass").to_list()) + M.PHOSPHATE_LINK_MASS
    su = [r[0] for r in rows]
    obs = [r[1] for r in rows]
    start, end = 0, 1
    out = {}
    while end < len(rows):
        if (end - start) <= 0:
            end += 1
            continue
        diff = su[end] - su[start]
        if diff > maxw:
            start += 1
            end = start + 1
            continue
        thr = dp.tolerance * (obs[start] + obs[end])
        expl = calculate_explanations(diff, thr, dp)
        if expl is not None and len(expl) >= 1:
            out[diff] = expl
        if end == len(rows) - 1:
            start += 1
        else:
            end += 1
    return out


def collect(frags, dp):
    """prediction.py:261-284 restated; frags: dicts in frame order."""
    e = {**per_side([(f["standard_unit_mass"], f["observed_mass"]) for f in frags if "START" in f["breakage"]], dp),
         **per_side([(f["standard_unit_mass"], f["observed_mass"]) for f in frags if "END" in f["breakage"]], dp)}
    for f in frags:
        if f["is_singleton"]:
            e[f["standard_unit_mass"]] = calculate_explanations(f["standard_unit_mass"],
                                                                dp.tolerance * f["observed_mass"], dp)
    return e


def filter_by_explanation(frags, dp):
    """prediction.py:170-227 restated (the reduction and is_valid are the reference's)."""
    rounds = []
    old = -1
    expl = {}
    while old != len(dp.masses):
        old = len(dp.masses)
        expl = collect(frags, dp)
        observed = {nuc for ex in expl.values() if ex is not None for t in ex for nuc in t}
        dp.adapt_individual_modification_rates_by_alphabet_reduction(observed)
        frags = [f for f in frags if ME.is_valid_mass(f["standard_unit_mass"], dp,
                                                       threshold=dp.tolerance * f["observed_mass"])]
        rounds.append({"masses": [int(m.mass) for m in dp.masses], "kept_index": [f["index"] for f in frags]})
    return rounds, {repr(k): wrap_rows(dp, v) for k, v in expl.items()}


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
        G.CTX[cid]["obs_mass"] = meta["sequence_mass"]
        classified = FC.classify_fragments(frame, dp, bd, intensity_cutoff=cutoff)
        rec = {"ctx": G.CTX[cid], "intensity_cutoff": cutoff, "tags": [meta.get("label_mass_5T", 555.1294),
                                                                         meta.get("label_mass_3T", 455.1491)],
               "input": frame_dump(frame), "classify": frame_dump(classified)}
        # Predictor.predict's framing (prediction.py:68-80)
        cols = classified.columns
        rows = [dict(zip(cols, r)) for r in classified.rows()]
        rows = [dict(r, orig_index=i) for i, r in enumerate(rows)]
        rows = sorted(rows, key=lambda r: r["standard_unit_mass"])
        rows = [dict(r, index=i) for i, r in enumerate(rows)]
        rec["filter"] = dict(zip(("rounds", "explanations"), filter_by_explanation(rows, dp)))
        out[tc] = rec
        print(f"  {tc}: {len(frame)} fragments -> {len(classified)} classified, "
              f"{len(rec['filter']['rounds'])} reduction rounds, {time.time() - t0:.0f}s", flush=True)
        del dp
    G.dump("callers.json.gz", out, gz=True)


if __name__ == "__main__":
    main()
