#!/usr/bin/env python3
"""One compute_sequence_length_bound call (A11, mass_table.py:343-487) on the
full 105-row alphabet, as the mirror's compute_sequence_length_bound issues
it: the first-visit frontier (the default for budget-binding windows), the
round-4 DFS replay (SST_LB_REPLAY) and the C oracle on one host thread (the
checker, timed beside it).  Sequence masses of whole 5-, 8- and 10-mers
(the 10-mer: the reference's 72 s call in BASELINE.md), max_len 20,
budgets round(0.5 * 20) = 10 and caps round(20 * 0.5)."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
import _oracle as oracle  # noqa: E402  (the CPU baseline / checker)
from conftest import load_golden  # noqa: E402
from spectrseqtools_amd import _native  # noqa: E402

CANON = (305042, 306026, 329053, 345048)


def main():
    g = load_golden("alphabet.json")
    rows = sorted({r["tolerated_integer_masses"] for r in g["rows"]} | {0})
    is_mod = [m not in CANON and m != 0 for m in rows]
    max_len = 20
    caps = [round(max_len * (0.5 if md else (1.0 if m else 0.0))) for m, md in zip(rows, is_mod)]
    eng = _native.get_engine(0)
    dev = _native.DeviceTable.build(rows, max(rows) * 35, 32, engine=eng)
    dev.set_budgets(is_mod, caps)
    table = oracle.build_table(rows, max(rows) * 35, 32)
    alph = oracle.Alphabet(rows, is_mod, caps)
    rng = np.random.default_rng(10)
    out = []
    for k in (5, 8, 10):
        su = float(rng.choice(rows[1:], k).sum()) * 1e-3
        rec = {"nt": k, "su_mass": su}
        for d in ("lower", "upper"):
            for name, kw in (("frontier", {}), ("replay", {"replay": True})):
                dev.length_bound([su], [su], 1e-5, 1e-3, max_len, 10, d, exact_only=True, **kw)  # warm
                t0 = time.perf_counter()
                v, st = dev.length_bound([su], [su], 1e-5, 1e-3, max_len, 10, d, exact_only=True, **kw)
                rec[f"{name}_{d}_s"] = time.perf_counter() - t0
                rec[f"{name}_{d}"] = int(v[0]) if int(st[0]) == 0 else f"status {int(st[0])}"
            t0 = time.perf_counter()
            w, memo = oracle.length_bound_memo(table, 32, alph, su, su, 1e-5, max_len, 10, d)
            rec[f"oracle_{d}_s"] = time.perf_counter() - t0
            rec[f"oracle_{d}"] = w
            rec["memo_entries"] = memo
            assert rec[f"frontier_{d}"] == w == rec[f"replay_{d}"], rec
        out.append(rec)
        print(json.dumps(rec), file=sys.stderr, flush=True)
    print(json.dumps({"workload": "compute_sequence_length_bound, one call, full alphabet", "calls": out}))


if __name__ == "__main__":
    main()
