#!/usr/bin/env python3
"""Golden vectors for the prediction pipeline after the skeleton, from the
REFERENCE itself (read-only at /root/reference; build container only).

TEST INFRASTRUCTURE.  Same set-up as make_callers_golden.py (the pandas-backed
polars stand-in and the import-only stand-ins; every reference function runs
unmodified).  Per reference test spectrum (tests/testcases/test_0[1-8]) it
runs Predictor.predict (prediction.py:63-168) on classify_fragments' frame
and observes it up to the skeleton-based alphabet reduction (:99-103):

    build_skeleton   SkeletonBuilder.build_skeleton (skeleton_building.py:26-112)
                     as predict calls it: select_sequence_length_with_lp
                     returns -1 here (pulp is a stand-in whose names raise, so
                     determine_lp_score's try/except gives np.inf for every
                     length, :279-286), which is the path the MILP-free config 5
                     takes -- the Jaccard fallback (:52-57); recorded: the
                     combined skeleton and the returned fragments' index,
                     min_end and max_end (:67-109)
    reduction        the _reduce_alphabet call that follows (:99-103): the
                     alphabet after it and the kept fragments' index, min_end,
                     max_end

predict is stopped right after that call (an exception the generator raises
from its observer), before filter_with_lp.  A spectrum whose build_skeleton
raised (no length fits) records {"default": true}: predict returns
Prediction.default() there (:89-94).

Usage:  PYTHONHASHSEED=0 XDG_CACHE_HOME=/tmp/sst_refcache python tests/golden/make_post_golden.py
"""
import os
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

M, EM, REF = G.M, G.EM, G.REF


class _Stop(Exception):
    pass


def _frame(df):
    return {"index": [int(x) for x in df.get_column("index").to_list()],
            "min_end": [int(x) for x in df.get_column("min_end").to_list()],
            "max_end": [int(x) for x in df.get_column("max_end").to_list()]}


def predict_to_reduction(classified, dp):
    pred = PR.Predictor(dp, EM)
    rec = {}
    orig_reduce = pred._reduce_alphabet
    orig_build = SB.SkeletonBuilder.build_skeleton

    def build(self, fragments, solver_params):
        sk, fr = orig_build(self, fragments=fragments, solver_params=solver_params)
        rec["build_skeleton"] = {"skeleton": [sorted(p) for p in sk], "fragments": _frame(fr),
                                 "masses": [int(m.mass) for m in dp.masses]}
        return sk, fr

    def observed(nucleotide_list, fragments):
        out = orig_reduce(nucleotide_list, fragments)
        if "build_skeleton" in rec:  # the skeleton-based reduction (prediction.py:99-103)
            rec["reduction"] = {"nucleotides": sorted(nucleotide_list), "masses": [int(m.mass) for m in dp.masses],
                                "fragments": _frame(out)}
            raise _Stop
        return out

    pred._reduce_alphabet = observed
    SB.SkeletonBuilder.build_skeleton = build
    try:
        pred.predict(classified, solver_params={})
        rec["default"] = True  # predict returned without reaching the reduction (build_skeleton raised)
    except _Stop:
        rec["default"] = False
    finally:
        SB.SkeletonBuilder.build_skeleton = orig_build
    return rec


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
        dp.seq.obs_mass = meta["sequence_mass"]  # cli.py:149-176
        classified = FC.classify_fragments(frame, dp, bd, intensity_cutoff=cutoff)
        out[tc] = predict_to_reduction(classified, dp)
        r = out[tc]
        print(f"  {tc}: default={r['default']}, "
              f"{len(r.get('build_skeleton', {}).get('fragments', {}).get('index', []))} fragments after the "
              f"skeleton -> {len(r.get('reduction', {}).get('fragments', {}).get('index', []))} after the "
              f"reduction, {time.time() - t0:.0f}s", flush=True)
        del dp
    out["_meta"] = {"pythonhashseed": os.environ.get("PYTHONHASHSEED")}
    G.dump("post_skeleton.json.gz", out, gz=True)


if __name__ == "__main__":
    main()
