#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ by running the REFERENCE
(spectrseq/spectrseqtools, read-only at /root/reference) unmodified.

TEST INFRASTRUCTURE -- runs only in the build container (the reference never
travels to the GPU box).  `polars` is absent here, so the pandas-backed
stand-in in tests/golden/standin/ is put first on sys.path; it only builds the
alphabet frame (masses.py:53-88) and is cross-checked below against an
independent numpy restatement of that frame.  Everything on the hot path
(set_up_bit_table, is_valid_mass, explain_mass_with_table,
explain_mass_with_recursion, compute_sequence_length_bound) is the reference's
own code.

Outputs (all JSON, floats written with repr so they round-trip exactly):
  alphabet.json        EXPLANATION_MASSES rows, breakage dicts, constants
  tables.json          SHA-256 of reference-built packed tables + tiny tables verbatim
  explain_cases.json.gz explain_mass_with_table / _with_recursion / is_valid_mass /
                       compute_sequence_length_bound known answers
  population.json.gz   A7 (is_valid) and A8 (adjacent-difference explain) query
                       streams of the reference's own test spectra
                       (tests/testcases/test_0[1-8]) with reference answers
  singleton.json.gz    fragment_classification.is_singleton known answers

Usage:  python tests/golden/make_golden.py [--rebuild-full-table]
"""
import csv
import gzip
import hashlib
import json
import math
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path[:0] = [os.path.join(HERE, "standin"), REF]

import numpy as np  # noqa: E402
import yaml  # noqa: E402

import spectrseqtools.masses as M  # noqa: E402
import spectrseqtools.mass_table as MT  # noqa: E402
import spectrseqtools.mass_explanation as ME  # noqa: E402

EM = M.EXPLANATION_MASSES
FULL_CACHE = os.path.join(MT.TABLE_DIR, "tol_1E-03.32_per_cell.npy")
SURVEY_FULL_SHA = "fbbef632442646b71cf69f6a2eca185996c9d34b59f4ea95401ce0ed9a1bc266"


def _rss_gb():
    import resource
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def dump(name, obj, gz=False):
    path = os.path.join(HERE, name)
    data = json.dumps(obj, separators=(",", ":")).encode()
    if gz:
        with gzip.GzipFile(path, "wb", mtime=0) as f:
            f.write(data)
    else:
        with open(path, "wb") as f:
            f.write(data)
    print(f"wrote {name} ({len(data) / 1e6:.2f} MB raw)", flush=True)


# --------------------------------------------------------------------------
# 1. alphabet (+ independent numpy restatement as a stand-in check)
# --------------------------------------------------------------------------
def alphabet():
    rows = EM.rows()
    cols = EM.columns
    recs = [dict(zip(cols, r)) for r in rows]
    for r in recs:
        r["nucleoside_list"] = list(r["nucleoside_list"])
        for k in ("monoisotopic_mass", "modification_rate", "theoretical_mz"):
            r[k] = float(r[k])
        r["tolerated_integer_masses"] = int(r["tolerated_integer_masses"])

    # independent restatement of masses.py:53-88 with the csv module + numpy
    tsv = list(csv.DictReader(open(f"{REF}/spectrseqtools/assets/masses.tsv"), delimiter="\t"))
    groups = {}
    for t in tsv:
        key = float(np.round(float(t["monoisotopic_mass"]), 4))
        g = groups.setdefault(key, {"names": [], "rate": -1.0})
        if t["nucleoside"] not in g["names"]:
            g["names"].append(t["nucleoside"])
        g["rate"] = max(g["rate"], float(t["modification_rate"]))
    indep = [(k, g["names"][0], int(round((k + M.PHOSPHATE_LINK_MASS) / M.TOLERANCE))) for k, g in groups.items()]
    assert [(r["monoisotopic_mass"], r["nucleoside"], r["tolerated_integer_masses"]) for r in recs] == indep
    # half-up decimal rounding of the 5-dp TSV masses gives the same integers
    from decimal import Decimal, ROUND_HALF_UP
    hu = sorted({int(round((float(Decimal(t["monoisotopic_mass"]).quantize(Decimal("0.0001"), ROUND_HALF_UP))
                            + M.PHOSPHATE_LINK_MASS) / M.TOLERANCE)) for t in tsv})
    assert hu == sorted(r["tolerated_integer_masses"] for r in recs), "rounding-mode sensitive alphabet"

    tags = [(555.1294, 455.1491)]
    for tc in sorted(os.listdir(f"{REF}/tests/testcases")):
        meta = yaml.safe_load(open(f"{REF}/tests/testcases/{tc}/fragments.meta.yaml"))
        tags.append((meta.get("label_mass_5T", 555.1294), meta.get("label_mass_3T", 455.1491)))
    brk = [{"mass_5_prime": a, "mass_3_prime": b,
            "dict": [[k, v] for k, v in M.build_breakage_dict(a, b).items()]} for a, b in sorted(set(tags))]
    out = {
        "rows": recs,
        "element_masses": M.ELEMENT_MASSES,
        "phosphate_link_mass": M.PHOSPHATE_LINK_MASS,
        "tolerance": M.TOLERANCE,
        "matching_threshold": M.MATCHING_THRESHOLD,
        "compression_rate": M.COMPRESSION_RATE,
        "unmodified_bases": M.UNMODIFIED_BASES,
        "nuc_reps": M.NUC_REPS,
        "breakage_dicts": brk,
        "mass_names": {str(k): v for k, v in ME.MASS_NAMES.items()},
        "is_mod": {str(k): v for k, v in ME.IS_MOD.items()},
    }
    dump("alphabet.json", out)
    return recs


# --------------------------------------------------------------------------
# contexts: a DynamicProgrammingTable plus how it was made
# --------------------------------------------------------------------------
MIN_INT = min(EM.get_column("tolerated_integer_masses").to_list())
CTX = {}


def make_ctx(cid, max_len, tolerance, mod_rate=0.5, keep=None, su=None):
    si = MT.SequenceInformation(max_len=max_len, su_mass=su if su is not None else 0.0,
                                obs_mass=su if su is not None else 0.0, modification_rate=mod_rate)
    dp = MT.DynamicProgrammingTable(EM, compression_rate=32, tolerance=tolerance, precision=M.TOLERANCE, seq=si)
    if keep is not None:
        dp.adapt_individual_modification_rates_by_alphabet_reduction(keep)
    CTX[cid] = {
        "id": cid,
        "max_len": max_len,
        "mod_rate": mod_rate,
        "tolerance": tolerance,
        "precision": M.TOLERANCE,
        "su_mass": si.su_mass,
        "obs_mass": si.obs_mass,
        "masses": [int(x.mass) for x in dp.masses],
        "names": [list(x.names) for x in dp.masses],
        "is_mod": [bool(x.is_modification) for x in dp.masses],
        "rates": [float(x.modification_rate) for x in dp.masses],
        "caps": [round(max_len * x.modification_rate) for x in dp.masses],
        "table_shape": list(dp.table.shape),
        "table_sha256": sha(dp.table),
    }
    return dp


def rows_of(dp, names_set):
    """reference name tuple -> ascending row-index tuple (each int mass has one
    representative, masses.py:67-71; MASS_NAMES is keyed by int mass)."""
    idx = {}
    for i, x in enumerate(dp.masses):
        for n in ME.MASS_NAMES.get(x.mass, []):
            idx[n] = i
    return sorted(tuple(sorted(idx[n] for n in t)) for t in names_set)


def run_explain(dp, cid, mass, threshold, A, with_memo=True, fn="table", names_limit=500):
    rec = {"ctx": cid, "fn": fn, "mass": mass, "threshold": threshold,
           "max_modifications": "inf" if A == np.inf else int(A), "with_memo": with_memo}
    t0 = time.perf_counter()
    try:
        if fn == "table":
            r = ME.explain_mass_with_table(mass, dp, max_modifications=A, threshold=threshold,
                                           with_memo=with_memo).explanations
        else:
            r = ME.explain_mass_with_recursion(mass, dp, max_modifications=A, threshold=threshold).explanations
    except MemoryError:
        return None  # sample skipped: the reference's solution-list memo outgrew the generator's memory cap
    except Exception as e:  # reference raises NameError / NotImplementedError
        rec.update(status="raise", error=type(e).__name__)
        return rec
    rec["seconds"] = round(time.perf_counter() - t0, 6)
    if r is None:
        rec["status"] = "none"
    else:
        rec["status"] = "set"
        if names_limit is None or len(r) <= names_limit:  # big sets: names follow from rows via MASS_NAMES
            rec["names"] = sorted(list(t) for t in r)
        rec["rows"] = [list(t) for t in rows_of(dp, r)]
    return rec


def run_valid(dp, cid, mass, threshold):
    rec = {"ctx": cid, "fn": "is_valid", "mass": mass, "threshold": threshold}
    try:
        rec["result"] = bool(ME.is_valid_mass(mass, dp, threshold=threshold))
    except Exception as e:
        rec["result"] = "raise"
        rec["error"] = type(e).__name__
    return rec


def get_seq_weight(seq):
    # tests/test_explain_masses.py:16-31 restated (map_elements is not in the stand-in)
    mono = {r[1]: r[0] for r in EM.rows()}
    return round(len(seq) * M.PHOSPHATE_LINK_MASS + sum(mono[x] for x in seq), 5)


# --------------------------------------------------------------------------
# 2. tables
# --------------------------------------------------------------------------
def tables(rebuild_full):
    out = {"packed": [], "tiny": []}
    full = np.load(FULL_CACHE)
    s = sha(full)
    assert s == SURVEY_FULL_SHA, s
    if rebuild_full:
        t0 = time.time()
        ints = sorted(set(EM.get_column("tolerated_integer_masses").to_list() + [0]))
        again = MT.set_up_bit_table(ints, max(ints) * MT.MAX_SEQ_LENGTH, 32)
        assert sha(again) == s
        print(f"full table rebuilt by reference in {time.time() - t0:.0f}s, sha ok", flush=True)
    out["packed"].append({"what": "full alphabet (load_dp_table cache, reference-built)",
                          "masses": sorted(set(EM.get_column("tolerated_integer_masses").to_list() + [0])),
                          "max_mass": 633169 * 35, "compression": 32, "shape": list(full.shape),
                          "sha256": s, "last_word_last_row": int(full[-1, -1]),
                          "rows_first_words": [[int(v) for v in full[r, :4]] for r in range(full.shape[0])],
                          "checksums_per_row": [int(np.bitwise_xor.reduce(full[r])) for r in range(full.shape[0])]})
    del full
    rng = random.Random(11)
    ints = sorted(EM.get_column("tolerated_integer_masses").to_list())
    subsets = [("canonical", [0, 305042, 306026, 329053, 345048])]
    for k in (3, 7, 12):
        subsets.append((f"random{k}", sorted([0] + rng.sample(ints, k))))
    for what, ms in subsets:
        t0 = time.time()
        tab = MT.set_up_bit_table(ms, max(ms) * MT.MAX_SEQ_LENGTH, 32)
        out["packed"].append({"what": what, "masses": ms, "max_mass": max(ms) * 35, "compression": 32,
                              "shape": list(tab.shape), "sha256": sha(tab),
                              "checksums_per_row": [int(np.bitwise_xor.reduce(tab[r])) for r in range(tab.shape[0])]})
        print(f"table {what} {tab.shape} {time.time() - t0:.1f}s", flush=True)
    # tiny synthetic alphabets, every compression, incl. the last-column mask quirk
    # (mass_table.py:246: shift >= width when (max_mass+1) % max_col == 0)
    for C in (4, 8, 16, 32):
        for ms, mm in (([0, 3, 5], 60), ([0, 7], 2 * C - 1), ([0, 2, 9, 11], 101), ([0, 5, 6], 3 * C - 1),
                       ([0, 1], 13), ([0, 4, 13, 31, 37], 250)):
            tab = MT.set_up_bit_table(ms, mm, C)
            out["tiny"].append({"masses": ms, "max_mass": mm, "compression": C, "shape": list(tab.shape),
                                "words": [[int(v) for v in row] for row in tab]})
    dump("tables.json", out)


# --------------------------------------------------------------------------
# 3. known answers for the per-mass functions
# --------------------------------------------------------------------------
def cases():
    out = []
    # (a) tests/test_explain_masses.py:34-136, both enumerators, full candidate sets
    seqs = [("A",), ("A", "A"), ("G", "G"), ("C", "C"), ("U", "U"), ("C", "U", "A", "G"), ("C", "C", "U", "A", "G", "G")]
    for thr in (10e-6, 5e-6, 2e-6):
        for seq in seqs:
            m = get_seq_weight(seq)
            cid = f"tem_{''.join(seq)}_{thr:g}"
            dp = make_ctx(cid, int(m / M.TOLERANCE / MIN_INT), thr, su=m)
            A = round(0.5 * len(seq))
            r = run_explain(dp, cid, m, None, A, names_limit=None)
            assert tuple(seq) in {tuple(x) for x in r["names"]}
            r["tag"] = "test_explain_masses/table"
            out.append(r)
            r = run_explain(dp, cid, m, None, A, fn="recursion", names_limit=None)
            r["tag"] = "test_explain_masses/recursion"
            out.append(r)
            out.append(dict(run_valid(dp, cid, m, None), tag="test_explain_masses/is_valid"))
            if len(seq) <= 2:
                for d in ("lower", "upper"):
                    out.append({"ctx": cid, "fn": "length_bound", "dir": d, "tag": "test_explain_masses/length",
                                "result": MT.compute_sequence_length_bound(dp, d)})
            del dp
            print(f"  tem {''.join(seq)} {thr:g} n={len(out)}", flush=True)

    # (b) full alphabet, random adjacent-difference-like and whole masses, all budget regimes
    rng = random.Random(5)
    for max_len in (2, 3, 4, 20):
        cid = f"full_L{max_len}"
        dp = make_ctx(cid, max_len, M.MATCHING_THRESHOLD, su=1000.0)
        ints = [x.mass for x in dp.masses[1:]]
        n_q = 160 if max_len != 20 else 240
        t_ctx = time.time()
        for qi in range(n_q):
            if qi % 40 == 0:
                print(f"    {cid} q{qi} {time.time() - t_ctx:.0f}s rss={_rss_gb():.1f}GB", flush=True)
            k = rng.choice([1, 1, 2, 2, 3, 3, 4])
            m = sum(rng.choice(ints) for _ in range(k)) * 1e-3 + rng.uniform(-0.02, 0.02)
            thr = 1e-5 * rng.uniform(600, 14000)
            A = rng.choice([0, 1, 2, 3, 10, np.inf, round(0.5 * max_len)])
            r = run_explain(dp, cid, m, thr, A)
            if r is not None:
                out.append(dict(r, tag="random/table"))
            if k <= 2 and rng.random() < 0.4:  # no-memo DFS is exponential in the item count
                r = run_explain(dp, cid, m, thr, A, with_memo=False)
                if r is not None:
                    out.append(dict(r, tag="random/nomemo"))
            out.append(dict(run_valid(dp, cid, m, thr), tag="random/is_valid"))
        # edge windows: around zero, negative, straddling and beyond the table end
        limit = dp.table.shape[1] * 32
        for m, thr in ((0.0, 0.05), (0.0004, 0.01), (-0.5, 0.2), (-3.0, 0.01), (0.3, 0.01),
                       (limit * 1e-3 - 0.01, 0.05), (limit * 1e-3 + 5, 0.01), (limit * 1e-3 - 0.5, 0.1),
                       (305.042, 0.0), (305.042, 1e-9), (633.169, 0.0005)):
            # windows reaching values just below the table end would make the
            # reference enumerate ~70-mers before it raises: is_valid only
            if not (limit * 1e-3 - 1 < m < limit * 1e-3):
                out.append(dict(run_explain(dp, cid, m, thr, np.inf), tag="edge/table"))
            out.append(dict(run_valid(dp, cid, m, thr), tag="edge/is_valid"))
        if max_len in (3, 4):
            for _ in range(6):
                k = rng.choice([1, 2])
                su = sum(rng.choice(ints) for _ in range(k)) * 1e-3
                dp.seq.su_mass = su
                dp.seq.obs_mass = su + rng.uniform(0, 1000)
                for d in ("lower", "upper"):
                    out.append({"ctx": cid, "fn": "length_bound", "dir": d, "tag": "random/length",
                                "su_mass": dp.seq.su_mass, "obs_mass": dp.seq.obs_mass,
                                "result": MT.compute_sequence_length_bound(dp, d)})
        del dp
        print(f"  {cid} n={len(out)}", flush=True)

    # (c) config 1: canonical alphabet, random canonical 1..8-mers, seed 1
    rng = random.Random(1)
    cid = "canonical_L20"
    dp = make_ctx(cid, 20, M.MATCHING_THRESHOLD, keep={"A", "C", "G", "U"}, su=1000.0)
    for _ in range(1000):
        seq = tuple(rng.choice("ACGU") for _ in range(rng.randint(1, 8)))
        m = get_seq_weight(seq)
        r = run_explain(dp, cid, m, None, round(0.5 * len(seq)))
        r["tag"] = "config1/table"
        r["seq"] = "".join(seq)
        out.append(r)
        out.append(dict(run_valid(dp, cid, m, None), tag="config1/is_valid"))
    del dp
    print(f"  config1 n={len(out)}", flush=True)
    dump("explain_cases.json.gz", {"contexts": CTX, "cases": out}, gz=True)


# --------------------------------------------------------------------------
# 4. the reference pipeline's own query population on its own test spectra
# --------------------------------------------------------------------------
def population():
    """classify_fragments (fragment_classification.py:39-101) and
    collect_explanations_per_side (prediction.py:286-329) restated as query
    generators; answers come from the reference's is_valid_mass /
    explain_mass_with_table (via calculate_explanations, common.py:47-57)."""
    ctxs = {}
    a7, a8 = [], []
    maxw = max(EM.get_column("monoisotopic_mass").to_list()) + M.PHOSPHATE_LINK_MASS
    for tc in sorted(os.listdir(f"{REF}/tests/testcases")):
        base = f"{REF}/tests/testcases/{tc}"
        meta = yaml.safe_load(open(f"{base}/fragments.meta.yaml"))
        rows = list(csv.DictReader(open(f"{base}/fragments.tsv"), delimiter="\t"))
        col = "observed_mass" if "observed_mass" in rows[0] else "neutral_mass"
        obs = [float(r[col]) for r in rows]
        inten = [float(r["intensity"]) if "intensity" in r else None for r in rows]
        bd = M.build_breakage_dict(meta.get("label_mass_5T", 555.1294), meta.get("label_mass_3T", 455.1491))
        su_seq = meta["sequence_mass"] - [k * M.TOLERANCE for k in bd if "START_END" in bd[k]][0]
        max_len = int(su_seq / M.TOLERANCE / MIN_INT)
        cid = f"pop_{tc}"
        dp = make_ctx(cid, max_len, M.MATCHING_THRESHOLD, su=su_seq)
        CTX[cid]["obs_mass"] = meta["sequence_mass"]
        cutoff = meta.get("intensity_cutoff", M.DEFAULT_INTENSITY_CUTOFF)
        kept = []
        t0 = time.perf_counter()
        for k, b in bd.items():
            for o, it in zip(obs, inten):
                su = o - (k * dp.precision)
                thr = dp.tolerance * o
                v = bool(ME.is_valid_mass(su, dp, threshold=thr))
                a7.append([cid, su, thr, v])
                if v:
                    kept.append((su, o, b[0], it if it is not None else cutoff * 1.1))
        t7 = time.perf_counter() - t0
        kept = sorted(kept, key=lambda c: c[0])
        kept = [c for c in kept if c[3] > cutoff and c[1] < 50000]
        kept = [c for c in kept if c[0] < su_seq + 1 and (c[0] > su_seq - 1 or not ("START" in c[2] and "END" in c[2]))]
        A = round(dp.seq.modification_rate * dp.seq.max_len)
        t0 = time.perf_counter()
        n8 = 0
        for side in ("START", "END"):
            fr = [c for c in kept if side in c[2]]
            s, e = 0, 1
            while e < len(fr):
                if e - s <= 0:
                    e += 1
                    continue
                d = fr[e][0] - fr[s][0]
                if d > maxw:
                    s += 1
                    e = s + 1
                    continue
                thr = dp.tolerance * (fr[s][1] + fr[e][1])
                r = ME.explain_mass_with_table(d, dp, max_modifications=A, threshold=thr).explanations
                rec = [cid, d, thr, A, None if r is None else [list(t) for t in rows_of(dp, r)]]
                a8.append(rec)
                n8 += 1
                if e == len(fr) - 1:
                    s += 1
                else:
                    e += 1
        t8 = time.perf_counter() - t0
        ctxs[cid] = CTX[cid]
        # the spectrum itself (data of the reference's tests/testcases) so the
        # producer chain can be replayed: observed masses, intensities, meta
        ctxs[cid]["spectrum"] = {"observed": obs, "intensity": inten, "sequence_mass": meta["sequence_mass"],
                                 "intensity_cutoff": cutoff, "su_seq": su_seq,
                                 "tags": [meta.get("label_mass_5T", 555.1294), meta.get("label_mass_3T", 455.1491)]}
        print(f"  {tc}: max_len={max_len} A7={len(obs) * len(bd)} ({t7:.2f}s) A8={n8} ({t8:.2f}s)", flush=True)
        del dp
    dump("population.json.gz", {"contexts": ctxs, "a7": a7, "a8": a8}, gz=True)


# --------------------------------------------------------------------------
# 5. is_singleton (fragment_classification.py:104-119) known answers
# --------------------------------------------------------------------------
def singleton():
    """The reference's own is_singleton on (a) every A7 query of its test
    spectra (the valid fragments classify_fragments would test) and (b)
    windows placed on / next to every row mass and the sentinel 0, with
    thresholds from 0 to several units.  Full-alphabet table, integer_masses =
    the table's rows as classify_fragments passes them (:73-80)."""
    import spectrseqtools.fragment_classification as FC

    dp = make_ctx("singleton_full", 20, M.MATCHING_THRESHOLD)
    rows = [m.mass for m in dp.masses]
    pop = json.loads(gzip.open(os.path.join(HERE, "population.json.gz")).read())
    qs = [(q[1], q[2]) for q in pop["a7"]]
    rng = random.Random(7)
    for w in rows:
        for d in (-3, -2, -1, 0, 1, 2, 3):
            for thr_units in (0, 1, 2, 4):
                m = (w + d) * dp.precision + rng.uniform(-0.0004, 0.0004)
                qs.append((m, thr_units * dp.precision + rng.choice([0.0, 1e-7, -1e-7])))
    for m in (0.0, 0.0004, -0.0004, -0.5, 0.5):
        qs.append((m, 0.001))
    out = []
    t0 = time.perf_counter()
    for m, thr in qs:
        thr = max(thr, 0.0)
        out.append([m, thr, bool(FC.is_singleton(m, rows, dp, threshold=thr))])
    print(f"  is_singleton: {len(out)} queries ({time.perf_counter() - t0:.1f}s), "
          f"{sum(o[2] for o in out)} true", flush=True)
    dump("singleton.json.gz", {"context": CTX["singleton_full"], "queries": out}, gz=True)


if __name__ == "__main__":
    t = time.time()
    parts = [a for a in sys.argv[1:] if not a.startswith("--")] or ["alphabet", "tables", "cases", "population"]
    if "alphabet" in parts:
        alphabet()
    if "tables" in parts:
        tables("--rebuild-full-table" in sys.argv)
    if "cases" in parts:
        cases()
    if "population" in parts:
        population()
    if "singleton" in parts:
        singleton()
    print(f"done in {time.time() - t:.0f}s")
