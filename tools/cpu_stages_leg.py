#!/usr/bin/env python3
"""CPU baseline of config 5's stages 1-4 (tools/pipeline_bench.py starts it
after its GPU timing, as a child process that never touches the GPU).

The reference runs these stages per spectrum in Python.  This leg runs the
same algorithm on the host: the host mirrors of the reference's callers
(classify_fragments, Predictor.filter_by_explanation with a table rebuild per
alphabet reduction, SkeletonBuilder._predict_skeleton per side) with every
table query answered by the CPU oracle (oracle/sst_oracle.c, the literal
restatement of the reference's DFS; tests/_fake_engine.py puts it behind
DynamicProgrammingTable) -- the "port" kind of cpu_baseline.  One spectrum
per worker process (fork, after the full table is built once), for about
--budget-s seconds, spectra in order; each spectrum's outcome (final
alphabet, kept rows, both sides' skeleton / kept rows / min_end / max_end)
goes back to the bench, which compares it with the device's.

Stage 1's A7 alone is also timed at full size: is_valid_mass (the oracle's
OpenMP batch) on every peak x 4 breakages of the rank's spectra, the exact
queries the device's classify answers.

TEST INFRASTRUCTURE (the oracle is the checker): never imported by the
product path.  Output: one JSON object on stdout.
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]

_STATE = {}


def _install_oracle_engine(full_table):
    """DynamicProgrammingTable's device tables -> the oracle (tests/_fake_engine.py);
    the full alphabet's table built once (shared by the forked workers)."""
    import _fake_engine
    from spectrseqtools_amd import _native

    full_masses = [int(m) for m in full_table.masses]

    def build(cls, masses, max_mass, compression, engine=None):
        if [int(m) for m in masses] == full_masses:
            return full_table
        return _fake_engine.FakeDeviceTable(masses, max_mass, compression)

    _native.DeviceTable.build = classmethod(build)


def _one(g):
    """Spectrum g through stages 1-4 on the host mirrors + oracle."""
    from spectrseqtools_amd.fragment_classification import classify_fragments
    from spectrseqtools_amd.frame import Frame
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE
    from spectrseqtools_amd.prediction import Predictor
    from spectrseqtools_amd.skeleton_building import SkeletonBuilder

    S = _STATE
    o = S["obs"][S["off"][g]:S["off"][g + 1]]
    t0 = time.perf_counter()
    seq = SequenceInformation(max_len=int(S["max_len"][g]), su_mass=float(S["su"][g]),
                              obs_mass=float(S["seq_mass"][g]), modification_rate=0.5)
    dp = DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=MATCHING_THRESHOLD,
                                 precision=TOLERANCE, seq=seq)
    fr = classify_fragments(Frame({"observed_mass": [float(x) for x in o]}), dp, S["bd"])
    t1 = time.perf_counter()
    f = fr.with_row_index("orig_index").sort("standard_unit_mass").with_row_index("index")
    f = f.with_columns(min_end=[0] * len(f), max_end=[-1] * len(f))
    pred = Predictor(dp, EXPLANATION_MASSES)
    frags, expl = pred.filter_by_explanation(f)
    t2 = time.perf_counter()
    out = {"g": int(g), "masses": [int(m.mass) for m in dp.masses], "kept": frags.get_column("index").to_list()}
    sb = SkeletonBuilder(explanations=expl, dp_table=dp)
    for side in ("START", "END"):
        sub = frags.filter_mask([side in b for b in frags.get_column("breakage").to_list()])
        sk, fs = sb._predict_skeleton(Frame(sub.to_dict()), [set() for _ in range(dp.seq.max_len)])
        out[side] = {"skeleton": [sorted(p) for p in sk], "kept_index": fs.get_column("index").to_list(),
                     "min_end": fs.get_column("min_end").to_list(), "max_end": fs.get_column("max_end").to_list()}
    t3 = time.perf_counter()
    out["t"] = [t1 - t0, t2 - t1, t3 - t2]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spectra", type=int, required=True)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--procs", type=int, default=16)
    ap.add_argument("--budget-s", type=float, default=20.0)
    args = ap.parse_args()

    import _oracle as oracle
    import _fake_engine
    from spectrseqtools_amd import pipeline
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE, build_breakage_dict
    from spectrseqtools_amd.synthetic import make_spectra

    batch = make_spectra(args.spectra, seed=args.seed + 1_000_003 * args.rank)  # tools/pipeline_bench.py's spectra
    bd = build_breakage_dict(555.1294, 455.1491)
    w_full = [k for k, v in bd.items() if "START_END" in v][0]
    su_seq = batch.seq_mass - w_full * TOLERANCE
    ints = sorted(set(EXPLANATION_MASSES.get_column("tolerated_integer_masses").to_list()) | {0})
    max_len = pipeline.max_len_of(su_seq, TOLERANCE, min(ints[1:]))
    t0 = time.perf_counter()
    full = _fake_engine.FakeDeviceTable(ints, max(ints) * 35, 32)
    full.close = lambda: None  # shared by every spectrum's DynamicProgrammingTable (a reduction "closes" it)
    build_s = time.perf_counter() - t0
    # stage 1's A7 at full size: every peak x 4 breakages, OpenMP over the procs
    obs = batch.observed
    shifts = np.array([k * TOLERANCE for k in bd.keys()])
    su = np.concatenate([obs - s for s in shifts])
    thr = MATCHING_THRESHOLD * np.tile(obs, len(shifts))
    t0 = time.perf_counter()
    valid = oracle.is_valid_batch(full.table, 32, su, thr, MATCHING_THRESHOLD, nthreads=args.procs,
                                  precision=TOLERANCE)
    a7_s = time.perf_counter() - t0
    res = {"a7": {"kind": "port", "what": "is_valid_mass on every peak x 4 breakages (oracle, OpenMP)",
                  "queries": int(len(su)), "valid": int((valid == 1).sum()), "threads": args.procs,
                  "wall_s": a7_s, "queries_per_s": len(su) / a7_s if a7_s > 0 else 0.0},
           "full_table_build_s": build_s}
    # stages 1-4 per spectrum on the host mirrors (fork: the table is shared)
    _STATE.update(obs=obs, off=batch.offsets, su=su_seq, seq_mass=batch.seq_mass, max_len=max_len, bd=bd)
    _install_oracle_engine(full)
    outs = []
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(args.procs) as pool:
        it = pool.imap(_one, range(args.spectra), chunksize=1)
        for o in it:
            outs.append(o)
            if time.perf_counter() - t0 > args.budget_s:
                break
        pool.terminate()
    wall = time.perf_counter() - t0
    n = len(outs)
    tt = np.array([o.pop("t") for o in outs]) if n else np.zeros((0, 3))
    res["stages1to4"] = {
        "kind": "port", "what": "per spectrum: classify_fragments, filter_by_explanation (a table rebuild per "
                                "alphabet reduction), _predict_skeleton per side -- the host mirrors with the "
                                "oracle answering every query", "threads": args.procs, "spectra": n,
        "sample": f"the first {n} of the rank's {args.spectra} spectra (in order)", "wall_s": wall,
        "spectra_per_s": n / wall if wall > 0 else 0.0, "est_s_all_spectra": args.spectra * wall / n if n else None,
        "thread_s": {"classify": float(tt[:, 0].sum()), "fixpoint": float(tt[:, 1].sum()),
                     "skeleton": float(tt[:, 2].sum())},
        "pythonhashseed": os.environ.get("PYTHONHASHSEED")}
    res["outcomes"] = outs
    print(json.dumps(res))


if __name__ == "__main__":
    main()
