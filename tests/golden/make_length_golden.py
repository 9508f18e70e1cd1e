#!/usr/bin/env python3
"""Golden vectors for compute_sequence_length_bound (mass_table.py:343-487) at
the depth config 5 runs it, from the REFERENCE itself (read-only at
/root/reference; build container only, never the GPU box).

TEST INFRASTRUCTURE.  Same set-up as make_golden.py (the pandas-backed polars
stand-in builds the alphabet frame; everything on the path is the reference's
own code, unmodified).  The reference call sites are skeleton_building.py:
223-224 and 335-336: a DynamicProgrammingTable reduced to the skeleton
alphabet (adapt_individual_modification_rates_by_alphabet_reduction, which
rebuilds the table with set_up_bit_table over the kept rows,
mass_table.py:94-121), then both directions.

Cases (seeded): 40 reduced alphabets -- the 4 canonical rows plus 0..12
modification rows (a few with 20..40) -- times 6 windows each of 6..14
nucleotides of the alphabet's own rows (plus a 2 mDa jitter; alphabets of
<= 8 kept rows two more of 15..20 nucleotides), max_len near the
window's nucleotide count, per-row modification rates from one of three
random rate profiles (caps round(max_len * rate), mass_table.py:416-419,470),
and max_modifications = round(modification_rate * max_len) drawn from
{0, 1, 2, 3, round(0.5 max_len)} (:351), so that budgets bind.  Each alphabet
also has one window past its rebuilt table's end (the reference raises).
Windows whose memo would exceed MAX_NODES entries (MAX_DEEP_NODES for the
15..20-nt ones; estimated with the CPU oracle first, so the reference's Python
finishes) are redrawn.

Output: length_cases.json.gz
  profiles   [3][105] per-row modification rates over the full table's rows
  alphabets  [{rows (full-table row indices, 0 included), masses, table_shape,
              table_sha256 (the reference's rebuilt table)}]
  cases      [{alpha, profile, max_len, max_modifications, modification_rate,
              su_mass, obs_mass, tolerance, caps (per kept row), is_mod,
              nucleotides (the window's sequence length; 0 past the table),
              oracle_nodes (the oracle's memo entries, for sizing only),
              lower, upper (null: the reference raised), seconds}]

Usage:  XDG_CACHE_HOME=/tmp/sst_refcache python tests/golden/make_length_golden.py [--jobs 7]
"""
import hashlib
import multiprocessing as mp
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE)]

import numpy as np  # noqa: E402

import make_golden as G  # noqa: E402  (stand-ins first on sys.path, then the reference)
import _oracle as O  # noqa: E402  (only to size the windows before the reference runs them)

M, MT, ME, EM = G.M, G.MT, G.ME, G.EM
TOL, PREC = M.MATCHING_THRESHOLD, M.TOLERANCE
RATES = (0.02, 0.05, 0.1, 0.25, 0.5)
MAX_NODES = 3_000_000
MAX_DEEP_NODES = 6_000_000
N_ALPHA, PER_ALPHA = 40, 6
CANON = {"A", "C", "G", "U"}


def full_rows():
    si = MT.SequenceInformation(max_len=20, su_mass=0.0, obs_mass=0.0, modification_rate=1.0)
    dp = MT.DynamicProgrammingTable(EM, compression_rate=32, tolerance=TOL, precision=PREC, seq=si)
    return [(int(x.mass), x.names[0] if x.names else None, bool(x.is_modification)) for x in dp.masses]


def plan(rows):
    """Alphabets and windows, sized with the oracle so the reference finishes."""
    rng = np.random.default_rng(606)
    n = len(rows)
    is_mod = np.array([r[2] for r in rows])
    w = np.array([r[0] for r in rows], np.int64)
    canon = [i for i in range(1, n) if not is_mod[i]]
    mods = [i for i in range(1, n) if is_mod[i]]
    profiles = []
    for _ in range(3):
        profiles.append([0.0] + [float(rng.choice(RATES)) if is_mod[i] else 1.0 for i in range(1, n)])
    sizes = [0, 0] + [int(x) for x in rng.integers(1, 5, 12)] + [int(x) for x in rng.integers(5, 9, 12)] + \
        [int(x) for x in rng.integers(9, 13, 10)] + [20, 28, 34, 40]
    alphas, cases = [], []
    for ai, nm in enumerate(sizes[:N_ALPHA]):
        kept = sorted(canon + (rng.choice(mods, nm, replace=False).tolist() if nm else []))
        rws = [0] + kept
        ms = [int(w[r]) for r in rws]
        tab = O.build_table(ms, max(ms) * 35, 32)
        alphas.append({"rows": rws, "masses": ms})
        made = 0
        n_deep = 2 if len(rws) <= 9 else 0  # windows of 15..20 nucleotides, as config 5's longest
        while made < PER_ALPHA + n_deep:
            k = int(rng.integers(6, 15)) if made < PER_ALPHA else int(rng.integers(15, 21))
            p = int(rng.integers(0, 3))
            L = int(np.clip(k + rng.integers(-2, 4), 4, 20))
            a_choice = [0, 1, 2, 3, round(0.5 * L)]
            A = int(a_choice[int(rng.integers(0, len(a_choice)))])
            su = float(w[rng.choice(kept, k)].sum()) * PREC + float(rng.normal(0.0, 0.002))
            ob = su + float(rng.choice([912.303, 537.119, 375.183, 0.0]))
            caps = [round(L * profiles[p][r]) for r in rws]
            alph = O.Alphabet(ms, [bool(is_mod[r]) for r in rws], caps)
            lo, n_lo = O.length_bound_memo(tab, 32, alph, su, ob, TOL, L, A, "lower")
            if n_lo > (MAX_NODES if made < PER_ALPHA else MAX_DEEP_NODES):
                continue
            cases.append({"alpha": ai, "profile": p, "max_len": L, "max_modifications": A,
                          "modification_rate": A / L, "su_mass": su, "obs_mass": ob, "tolerance": TOL,
                          "caps": caps, "is_mod": [bool(is_mod[r]) for r in rws], "oracle_nodes": n_lo,
                          "nucleotides": k})
            made += 1
        # one window past the rebuilt table's end: the reference raises at its first value
        end = tab.shape[1] * 32
        su = (end + 50 + int(rng.integers(0, 5000))) * PREC
        L = 20
        cases.append({"alpha": ai, "profile": 0, "max_len": L, "max_modifications": 10, "modification_rate": 0.5,
                      "su_mass": su, "obs_mass": su, "tolerance": TOL,
                      "caps": [round(L * profiles[0][r]) for r in rws], "is_mod": [bool(is_mod[r]) for r in rws],
                      "oracle_nodes": 0, "nucleotides": 0})
    return profiles, alphas, cases


def run_alpha(job):
    """The reference on one alphabet: rebuild the table, then every window,
    both directions.  Runs in a worker process."""
    ai, alpha, cases, profiles = job
    t0 = time.time()
    si = MT.SequenceInformation(max_len=20, su_mass=0.0, obs_mass=0.0, modification_rate=1.0)
    dp = MT.DynamicProgrammingTable(EM, compression_rate=32, tolerance=TOL, precision=PREC, seq=si)
    keep = set(CANON)
    for x in dp.masses[1:]:
        if x.is_modification and x.mass in alpha["masses"]:
            keep.add(x.names[0])
    dp.adapt_individual_modification_rates_by_alphabet_reduction(keep)
    assert [int(x.mass) for x in dp.masses] == alpha["masses"], ai
    rebuilt = time.time() - t0
    res = {"table_shape": list(dp.table.shape),
           "table_sha256": hashlib.sha256(np.ascontiguousarray(dp.table).tobytes()).hexdigest(), "cases": []}
    for c in cases:
        for i, x in enumerate(dp.masses):
            if x.is_modification:  # the per-row rates the caps come from (mass_table.py:416-419, 470)
                x.modification_rate = profiles[c["profile"]][alpha["rows"][i]]
        assert [round(c["max_len"] * x.modification_rate) for x in dp.masses[1:]] == c["caps"][1:]
        dp.seq = MT.SequenceInformation(max_len=c["max_len"], su_mass=c["su_mass"], obs_mass=c["obs_mass"],
                                        modification_rate=c["modification_rate"])
        assert round(dp.seq.modification_rate * dp.seq.max_len) == c["max_modifications"]
        t = time.time()
        out = {}
        for d in ("lower", "upper"):
            try:
                out[d] = int(MT.compute_sequence_length_bound(dp, d))
            except NotImplementedError:
                out[d] = None
        res["cases"].append(dict(c, lower=out["lower"], upper=out["upper"], seconds=round(time.time() - t, 3)))
    print(f"  alphabet {ai}: {len(alpha['masses'])} rows, rebuild {rebuilt:.0f}s, "
          f"{len(cases)} windows {time.time() - t0 - rebuilt:.0f}s", flush=True)
    return ai, res


def main():
    jobs = int(sys.argv[sys.argv.index("--jobs") + 1]) if "--jobs" in sys.argv else 7
    t0 = time.time()
    rows = full_rows()
    profiles, alphas, cases = plan(rows)
    print(f"planned {len(cases)} windows on {len(alphas)} alphabets "
          f"(oracle memo entries: max {max(c['oracle_nodes'] for c in cases)}, "
          f"sum {sum(c['oracle_nodes'] for c in cases)})", flush=True)
    work = [(ai, a, [c for c in cases if c["alpha"] == ai], profiles) for ai, a in enumerate(alphas)]
    work.sort(key=lambda j: -(len(j[1]["masses"]) * 20 + sum(c["oracle_nodes"] for c in j[2]) * 4e-6))
    out_cases = []
    with mp.get_context("fork").Pool(jobs) as pool:
        for ai, res in pool.imap_unordered(run_alpha, work):
            alphas[ai].update(table_shape=res["table_shape"], table_sha256=res["table_sha256"])
            out_cases += res["cases"]
    out_cases.sort(key=lambda c: (c["alpha"], c["su_mass"]))
    G.dump("length_cases.json.gz", {"profiles": profiles, "alphabets": alphas, "cases": out_cases,
                                    "_meta": {"max_nodes": MAX_NODES, "max_deep_nodes": MAX_DEEP_NODES, "seconds": round(time.time() - t0)}}, gz=True)
    print(f"done in {time.time() - t0:.0f}s")


if __name__ == "__main__":
    main()
