#!/usr/bin/env python3
"""Golden vectors for the reference's out-of-table raises: exception type AND
message of explain_mass_with_table, is_valid_mass and
compute_sequence_length_bound when a window leaves the DP table.

TEST INFRASTRUCTURE -- runs only in the build container, with the REFERENCE
(read-only at /root/reference) imported unmodified through the pandas-backed
polars stand-in (tests/golden/standin, see make_golden.py).

The reference formats the closure variable `value` of the outer window loop
(mass_explanation.py:134-138 + :192; :68-72 in is_valid_mass;
mass_table.py:383-387 + :461): the window value being processed when the DFS
(or the validity scan) first met a mass beyond the table.  To keep the
reference's enumeration below the table end cheap, the table here holds only
two nucleosides (C, G): every reachable mass is a small multiset of two masses.

Output: tests/golden/raise_cases.json
Usage:  python tests/golden/make_raise_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "standin"), "/root/reference"]

import numpy as np  # noqa: E402

import spectrseqtools.masses as M  # noqa: E402
import spectrseqtools.mass_table as MT  # noqa: E402
import spectrseqtools.mass_explanation as ME  # noqa: E402

KEEP = ("C", "G")
MAX_LEN = 40


def make_dp():
    import polars as pl

    frame = M.EXPLANATION_MASSES.filter(pl.col("nucleoside").is_in(list(KEEP)))
    masses = MT.initialize_nucleotide_masses(frame)
    dp = object.__new__(MT.DynamicProgrammingTable)
    dp.compression_per_cell = 32
    dp.tolerance = M.MATCHING_THRESHOLD
    dp.precision = M.TOLERANCE
    dp.seq = MT.SequenceInformation(max_len=MAX_LEN, su_mass=0.0, obs_mass=0.0, modification_rate=0.5)
    dp.masses = masses
    ints = [m.mass for m in masses]
    dp.table = MT.set_up_bit_table(integer_masses=ints, max_mass=max(ints) * MT.MAX_SEQ_LENGTH, compression_rate=32)
    return dp


def outcome(fn):
    try:
        r = fn()
    except Exception as e:  # the raises under test
        return {"status": "raise", "error": type(e).__name__, "message": str(e)}
    if isinstance(r, ME.MassExplanations):
        r = None if r.explanations is None else sorted(list(t) for t in r.explanations)
    elif isinstance(r, (bool, np.bool_)):
        r = bool(r)
    return {"status": "ok", "result": r}


def main():
    dp = make_dp()
    ints = [m.mass for m in dp.masses]
    limit = dp.table.shape[1] * 32
    wC, wG = ints[1], ints[2]
    # windows: wholly beyond the end; straddling it (the raise names the first
    # value >= limit); straddling with a reachable value just below the end
    # (is_valid returns True before it reaches the end); one fully inside
    below = max(a * wC + b * wG for a in range(40) for b in range(40) if a * wC + b * wG < limit)
    windows = [
        ("beyond", limit * 1e-3 + 5.0, 0.01),
        ("straddle_unreachable", (limit - 3) * 1e-3, 0.01),
        ("straddle_reachable_below", (below + 40) * 1e-3, 0.05),
        ("far_beyond_wide", limit * 1e-3 + 900.0, 2.0),
        ("inside", 3 * wC * 1e-3 + 1e-4, 0.002),
    ]
    cases = []
    for tag, mass, thr in windows:
        cases.append({"tag": tag, "fn": "explain", "mass": mass, "threshold": thr,
                      **outcome(lambda: ME.explain_mass_with_table(mass, dp, threshold=thr))})
        cases.append({"tag": tag, "fn": "is_valid", "mass": mass, "threshold": thr,
                      **outcome(lambda: ME.is_valid_mass(mass, dp, threshold=thr))})
        # the length bound's window: round(su/prec) +- ceil(tol * obs / prec)
        obs = thr / dp.tolerance
        dp.seq.su_mass, dp.seq.obs_mass = mass, obs
        for d in ("lower", "upper"):
            cases.append({"tag": tag, "fn": "length_bound", "dir": d, "su_mass": mass, "obs_mass": obs,
                          **outcome(lambda: MT.compute_sequence_length_bound(dp, d))})
    out = {"keep": list(KEEP), "max_len": MAX_LEN, "masses": ints, "limit": limit, "cases": cases}
    with open(os.path.join(HERE, "raise_cases.json"), "w") as f:
        json.dump(out, f, indent=1)
    for c in cases:
        print(c["tag"], c["fn"], c.get("dir", ""), c["status"], c.get("error", ""), c.get("message", c.get("result")))


if __name__ == "__main__":
    main()
