#!/usr/bin/env python3
"""Batched compute_sequence_length_bound (A11) throughput: the bounds the
reference computes after alphabet reduction (skeleton_building.py:223-224,
335-336: lower and upper per spectrum), for many spectra at once on one
reduced alphabet, against the C oracle on one thread (a bounded sample of
the same queries).  Alphabets: canonical, and canonical + 4 modifications
(budgets can bind).  Sequence masses of random 10..20-mers over the
alphabet, obs = su (seq_info in skeleton building carries both)."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
import _oracle as oracle  # noqa: E402  (the CPU baseline / checker)
from spectrseqtools_amd import _native  # noqa: E402

CANON = (305042, 306026, 329053, 345048)
MODS4 = (308042, 319058, 330037, 345037)  # 8U, 0C, 9A, 55U (rows of the full alphabet)


def run(rows, n, seed, tol=1e-5, prec=1e-3):
    rows = sorted({0, *rows})
    is_mod = [m not in CANON and m != 0 for m in rows]
    eng = _native.get_engine(0)
    dev = _native.DeviceTable.build(rows, max(rows) * 35, 32, engine=eng)
    rng = np.random.default_rng(seed)
    L = rng.integers(10, 21, n)
    su = np.array([rng.choice(rows[1:], k).sum() for k in L]) * prec + rng.normal(0, 0.002, n)
    max_len = 20
    caps = [round(max_len * (0.5 if md else (1.0 if m else 0.0))) for m, md in zip(rows, is_mod)]
    dev.set_budgets(is_mod, caps)
    A = round(0.5 * max_len)
    out = {"alphabet_rows": len(rows), "queries": n}
    table = oracle.build_table(rows, max(rows) * 35, 32)
    alph = oracle.Alphabet(rows, is_mod, caps)
    for d in ("lower", "upper"):
        dev.length_bound(su[:4], su[:4], tol, prec, max_len, A, d)  # warm-up
        t0 = time.perf_counter()
        v, st = dev.length_bound(su, su, tol, prec, max_len, A, d)
        gpu = time.perf_counter() - t0
        k = min(n, 64)
        t0 = time.perf_counter()
        want = [oracle.length_bound(table, 32, alph, su[i], su[i], tol, max_len, A, d) for i in range(k)]
        cpu = time.perf_counter() - t0
        ok = all(int(v[i]) == want[i] for i in range(k) if want[i] is not None and st[i] == 0)
        out[d] = {"gpu_s": gpu, "gpu_queries_per_s": n / gpu, "oracle_1thread_queries_per_s": k / cpu,
                  "oracle_sample": k, "agree_on_sample": ok, "statuses": np.unique(st).tolist()}
    dev.close()
    return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    res = {"canonical": run(CANON, n, 1), "canonical+4mods": run(CANON + MODS4, n, 2)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
