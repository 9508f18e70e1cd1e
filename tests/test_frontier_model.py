"""The first-visit frontier (sst_frontier.hip) restated in plain
Python on a rebuilt table's pair bits, against the CPU oracle's literal
compute_sequence_length_bound (mass_table.py:343-487): the theorem the GPU
engine rests on, checked on the CPU.

The reference's memo is keyed by (mass, row) and ignores the budgets, so each
node's value is fixed by its first visit.  The DFS explores up before left
and window values ascending, and expands a node only at its first visit, so
that visit is the lexicographically smallest (root index, c_{K-1}, ..., c_r)
path over the node's two possible parents, each taken at ITS first visit:
    FV(m, r) = lexmin(FV(m, r + 1) . up, FV(m + w_r, r) . left)
a recurrence over descending masses.  The values are then a DP over
ascending masses.  TEST INFRASTRUCTURE: a model of the kernel's algorithm,
not part of the product."""
import heapq
import math

import numpy as np
import pytest

import _oracle as oracle
from conftest import load_golden

TOL, PREC = 1e-5, 1e-3
CANONICAL = (305042, 306026, 329053, 345048)
RATES = (0.02, 0.05, 0.1, 0.25, 0.5)


def frontier_bounds(tab, C, w, is_mod, cap, su, obs, max_len, A0):
    """(lower, upper, memo entries), or (None, None, 0) where the reference raises."""
    K = len(w)
    limit = tab.shape[1] * C

    def pair(r, m):
        return (int(tab[r, m // C]) >> (2 * (C - 1 - m % C))) & 3

    target = int(round(su / PREC))
    thr = int(math.ceil(TOL * obs / PREC))
    lo_w, hi_w = target - thr, target + thr
    if hi_w >= limit:
        return None, None, 0
    cand = {}  # mass -> {row: (key, A, B)}: the left candidate of (mass, row)
    heap = []
    for i, v in enumerate(range(lo_w, hi_w + 1)):
        if v >= 1 and pair(K - 1, v):
            cand.setdefault(v, {})[K - 1] = ((i,) + (0,) * (K - 1), A0, cap[K - 1])
            heapq.heappush(heap, -v)
    nodes = {}  # (mass, row) -> left move attempted
    done = set()
    while heap:  # descending masses
        m = -heapq.heappop(heap)
        if m in done:
            continue
        done.add(m)
        up = None
        for r in range(max(cand[m]), 0, -1):
            left = cand[m].get(r)
            if up is None and left is None:
                break
            p = pair(r, m)
            if p == 0:
                up = None
                continue
            key, A, B = up if (up is not None and (left is None or up[0] < left[0])) else left
            latt = bool((p >> 1) & 1) and (not is_mod[r] or (A > 0 and B > 0))
            if latt and m - w[r] >= 1:
                k2 = list(key)
                k2[K - r] += 1
                assert r not in cand.setdefault(m - w[r], {})  # one left parent per node
                cand[m - w[r]][r] = (tuple(k2), A - is_mod[r], B - is_mod[r])
                heapq.heappush(heap, -(m - w[r]))
            nodes[(m, r)] = latt
            up = (key, A, cap[r - 1]) if p & 1 else None
    out = []
    for d in (0, 1):
        dflt = -1 if d else max_len + 1
        comb = max if d else min
        val = {}

        def get(m, r):
            if m < 0:
                return dflt
            if m == 0:
                return 0
            return val.get((m, r), dflt)  # absent: pair == 0

        for (m, r) in sorted(nodes):  # ascending masses
            b = dflt
            if pair(r, m) & 1:
                b = comb(b, get(m, r - 1))
            if nodes[(m, r)]:
                b = comb(b, get(m - w[r], r) + 1)
            val[(m, r)] = b
        best = comb(get(v, K - 1) if (v <= 0 or pair(K - 1, v)) else dflt for v in range(lo_w, hi_w + 1))
        out.append((max_len if d else 1) if best == dflt else best)
    return out[0], out[1], len(nodes)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_frontier_model_equals_oracle(seed):
    g = load_golden("alphabet.json")
    rows = sorted({r["tolerated_integer_masses"] for r in g["rows"]} | {0})
    rng = np.random.default_rng(seed)
    canon = [i for i, m in enumerate(rows) if m in CANONICAL]
    mods = [i for i, m in enumerate(rows) if i > 0 and m not in CANONICAL]
    n_ok = n_nodes = n_bind = 0
    for _ in range(70):
        max_len = int(rng.integers(3, 21))
        a = sorted(set(canon + rng.choice(mods, size=int(rng.integers(0, 12)), replace=False).tolist()))
        ms = [rows[r] for r in [0] + a]
        is_mod = [m not in CANONICAL and m != 0 for m in ms]
        rate = [float(rng.choice(RATES)) if md else (1.0 if m else 0.0) for m, md in zip(ms, is_mod)]
        cap = [round(max_len * r) for r in rate]
        A0 = int(rng.choice([0, 1, 2, 3, round(0.5 * max_len)]))
        tab = oracle.build_table(ms, max(ms) * 35, 32)
        alph = oracle.Alphabet(ms, is_mod, cap)
        wv = np.array(ms[1:])
        su = float(wv[rng.integers(0, len(wv), int(rng.integers(2, 12)))].sum()) * PREC + rng.normal(0, 0.002)
        obs = su + 912.303
        (w_lo, n_memo), (w_up, _) = (oracle.length_bound_memo(tab, 32, alph, su, obs, TOL, max_len, A0, d)
                                     for d in ("lower", "upper"))
        want = [w_lo, w_up]
        lo, up, nn = frontier_bounds(tab, 32, ms, is_mod, cap, su, obs, max_len, A0)
        if want[0] is None:
            assert lo is None
            continue
        assert [lo, up] == want, (lo, up, want, A0, max_len)
        assert nn == n_memo, (nn, n_memo)  # the same (mass, row) nodes as the reference's memo
        free = [oracle.length_bound(tab, 32, oracle.Alphabet(ms, is_mod, [99] * len(ms)), su, obs, TOL, max_len, 99, d)
                for d in ("lower", "upper")]
        n_bind += free != want
        n_ok += 1
        n_nodes += nn
    assert n_ok >= 60 and n_nodes > 5000 and n_bind >= 3
