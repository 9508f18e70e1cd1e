#!/usr/bin/env python3
"""Time compute_sequence_length_bound on the GPU for growing full-alphabet
sequences (the reference quotes 5.2 s / 72 s; the C oracle 3 / 20 / 70 s for
10 / 15 / 20-mers on this host)."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from spectrseqtools_amd import _native  # noqa: E402
from spectrseqtools_amd.masses import EXPLANATION_MASSES  # noqa: E402
from spectrseqtools_amd.mass_table import initialize_nucleotide_masses  # noqa: E402

CANON = (305042, 306026, 329053, 345048)
ms = [m.mass for m in initialize_nucleotide_masses(EXPLANATION_MASSES)]
eng = _native.get_engine(0)
dev = _native.DeviceTable.build(ms, max(ms) * 35, 32, engine=eng)
res = []
for L in [int(x) for x in (sys.argv[1:] or ["5", "10", "15", "20"])]:
    is_mod = [m not in CANON and m != 0 for m in ms]
    caps = [round(L * (0.5 if md else (1.0 if m else 0.0))) for m, md in zip(ms, is_mod)]
    dev.set_budgets(is_mod, caps)
    rng = np.random.default_rng(L)
    su = rng.choice(CANON, L).sum() * 1e-3
    for d in ("lower", "upper"):
        t0 = time.perf_counter()
        v, st = dev.length_bound([su], [su], 1e-5, 1e-3, L, round(0.5 * L), d)
        dt = time.perf_counter() - t0
        r = {"L": L, "su": su, "dir": d, "bound": int(v[0]), "status": int(st[0]), "seconds": dt}
        print(json.dumps(r), flush=True)
        res.append(r)

# explain_mass_with_recursion on the reference's own 6-mer (tests/test_explain_masses.py: CCUAGG)
for tol in (1e-5, 5e-6, 2e-6):
    is_mod = [m not in CANON and m != 0 for m in ms]
    caps = [round(6 * (0.5 if md else (1.0 if m else 0.0))) for m, md in zip(ms, is_mod)]
    dev.set_budgets(is_mod, caps)
    t0 = time.perf_counter()
    r = dev.explain_recursion([1935.25876], None, tol, 1e-3, 3)
    dt = time.perf_counter() - t0
    print(json.dumps({"recursion": "CCUAGG", "tol": tol, "status": int(r.status[0]), "count": int(r.count[0]),
                      "seconds": dt}), flush=True)
