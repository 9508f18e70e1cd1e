"""Columnar, many-spectrum form of the prediction pipeline's explanation
stages (SURVEY config 5), on the GPU engine.

The reference runs its pipeline one spectrum at a time and one query at a
time (cli.py:192-207 -> classify_fragments, Predictor.predict).  Here the
stages that issue hot-path queries run over a whole batch of spectra at once,
in flat arrays (spectrum id per row) instead of per-spectrum frames:

  1. classify   (fragment_classification.py:17-101): every peak x breakage
                 weight -> one is_valid batch, valid rows -> one is_singleton
                 batch, then the intensity / mass / sequence-mass filters and
                 the per-spectrum SU-mass sort (sst_sort_rows, host-native);
  2. su_diffs   (prediction.py:261-329, the first filter_by_explanation
                 round): every side's sliding-window pairs (sst_su_diff_queries,
                 host-native) and the singleton masses -> one explain batch;
  3. bins       (skeleton_building.py:114-196, 372-421): every side's bins
                 (neighbouring SU differences within tolerance) and the
                 speculative bin-pair queries -> one explain batch; the first
                 bin of a side explains whole fragment masses (deep windows:
                 the engine's deferred DFS kernels).

  4. fixpoint   (prediction.py:170-227, filter_by_explanation): every round
                 of every spectrum at once -- the pair-class explains of all
                 spectra against their own reduced alphabets (one
                 sst_explain_pairs_alpha call: the reduced tables are never
                 built), the explanation dicts' surviving entries and observed
                 rows (sst_dict_union, host-native), the alphabet reduction as
                 row-mask arithmetic, and is_valid of every remaining fragment
                 against its spectrum's reduced table (one sst_is_valid_alpha
                 call); spectra whose alphabet stopped shrinking drop out.

Every stage's rows equal what the per-spectrum mirrors produce
(tests/test_pipeline.py); the fixpoint's rounds equal the reference's own
(tests/golden/callers.json.gz).  Budgets follow each spectrum's max_len (the
cli derives it from the sequence mass, cli.py:158-177): spectra are grouped
by max_len and each group is one engine call with that group's row caps.
The MILP is not a batched stage.
"""
from dataclasses import dataclass

import numpy as np

from ._native import sort_rows, su_diff_queries as _su_diff_queries
from .masses import MATCHING_THRESHOLD, PHOSPHATE_LINK_MASS, TOLERANCE

MAX_VARIANCE = 1  # fragment_classification.py:8


@dataclass
class Classified:
    """classify_fragments' rows of all spectra, spectrum-major, each spectrum
    sorted by SU mass (its frame's row order)."""
    spec: np.ndarray        # spectrum id
    su: np.ndarray          # standard_unit_mass
    obs: np.ndarray         # observed_mass
    frag: np.ndarray        # fragment_index (peak position within its spectrum)
    brk: np.ndarray         # breakage code: index into `names`
    singleton: np.ndarray   # is_singleton
    names: list             # breakage label per code
    offsets: np.ndarray     # [S+1] row ranges per spectrum
    n_valid_queries: int    # is_valid queries issued
    n_singleton_queries: int


def max_len_of(su_seq, precision=TOLERANCE, min_int_mass=None):
    """cli.py:158-170: int(su_mass / precision / min(integer masses with rate > 0))."""
    return (np.asarray(su_seq, dtype=np.float64) / precision / min_int_mass).astype(np.int64)


def classify(obs, offsets, su_seq, dp_table, breakage_dict, intensity=None, intensity_cutoff=0.5e6,
             mass_cutoff=50000):
    """Stage 1 over S spectra: obs[offsets[s]:offsets[s+1]] are spectrum s's
    observed masses; su_seq[s] its SU sequence mass (dp_table.seq.su_mass of
    its own pipeline run)."""
    from .fragment_classification import is_singletons, valid_peaks

    obs = np.asarray(obs, dtype=np.float64)
    offsets = np.asarray(offsets, dtype=np.int64)
    S = len(offsets) - 1
    n_peaks = np.diff(offsets)
    spec_p = np.repeat(np.arange(S), n_peaks)
    frag_p = np.arange(len(obs)) - offsets[spec_p]
    inten = (np.full(len(obs), intensity_cutoff * 1.1) if intensity is None
             else np.asarray(intensity, dtype=np.float64))
    weights = list(breakage_dict.keys())
    names = [breakage_dict[w][0] for w in weights]
    B = len(weights)
    # breakage-major within each spectrum (the reference's pl.concat order)
    spec = np.tile(spec_p, B)
    frag = np.tile(frag_p, B)
    brk = np.repeat(np.arange(B), len(obs))
    ob = np.tile(obs, B)
    su = ob - np.repeat(np.asarray(weights, dtype=np.float64) * dp_table.precision, len(obs))
    valid = valid_peaks(obs, breakage_dict, dp_table)  # one lane per peak, breakage-major like `su`
    keep = np.flatnonzero(valid)
    sing = is_singletons(su[keep], [m.mass for m in dp_table.masses], dp_table,
                         thresholds=dp_table.tolerance * ob[keep]) if len(keep) else np.zeros(0, bool)
    # filters (:84-95), then per spectrum: SU order, ties in concat order
    it = np.tile(inten, B)[keep]
    full = np.array([("START" in n) and ("END" in n) for n in names], dtype=bool)[brk[keep]]
    seq = np.asarray(su_seq, dtype=np.float64)[spec[keep]]
    ok = (it > intensity_cutoff) & (ob[keep] < mass_cutoff) & (su[keep] < seq + MAX_VARIANCE) & \
         ((su[keep] > seq - MAX_VARIANCE) | ~full)
    rows, sing = keep[ok], sing[ok]
    # the expanded position orders each spectrum's rows as its own concat (breakage,
    # fragment): per spectrum by SU mass, ties in that order (host-native sort)
    order = sort_rows(spec[rows], su[rows], S)
    rows, sing = rows[order], sing[order]
    off = np.searchsorted(spec[rows], np.arange(S + 1))
    return Classified(spec[rows], su[rows], ob[rows], frag[rows], brk[rows], sing, names, off, len(su), len(keep))


def subset(c: Classified, keep):
    """The rows of c where keep is set (e.g. a fixpoint's surviving rows)."""
    idx = np.flatnonzero(np.asarray(keep, dtype=bool))
    off = np.searchsorted(c.spec[idx], np.arange(len(c.offsets)))
    return Classified(c.spec[idx], c.su[idx], c.obs[idx], c.frag[idx], c.brk[idx], c.singleton[idx], c.names, off,
                      c.n_valid_queries, c.n_singleton_queries)


def _sides(c: Classified, side):
    """Rows of one side per spectrum (SU order kept): row ids and offsets."""
    m = np.array([side in n for n in c.names], dtype=bool)[c.brk]
    rows = np.flatnonzero(m)
    return rows, np.searchsorted(c.spec[rows], np.arange(len(c.offsets)))


@dataclass
class Queries:
    diff: np.ndarray
    thr: np.ndarray
    spec: np.ndarray
    kind: np.ndarray  # stage-specific tag (su_diffs: 0 START pair, 1 END pair, 2 singleton; bins: bin id)
    side: np.ndarray = None  # bins: 0 START, 1 END


def su_diff_queries(c: Classified, explanation_masses, tolerance=MATCHING_THRESHOLD):
    """Stage 2's queries: per spectrum the START-side pairs, the END-side
    pairs, then the singletons (collect_diff_explanations_for_su's order),
    produced by host-native code in one pass (sst_su_diff_queries)."""
    max_w = max(explanation_masses.get_column("monoisotopic_mass").to_list()) + PHOSPHATE_LINK_MASS
    side = np.array([("START" in n) | (("END" in n) << 1) for n in c.names], dtype=np.uint8)
    flags = side[c.brk] | (np.asarray(c.singleton, dtype=np.uint8) << 2)
    d, t, g, k = _su_diff_queries(c.su, c.obs, flags, c.offsets, max_w, tolerance)
    return Queries(d, t, g, k)


def bin_queries(c: Classified, tolerance=MATCHING_THRESHOLD):
    """Stage 3's speculative queries: per side, its bins as
    SkeletonBuilder._predict_skeleton forms them, the first bin's whole
    masses and every later bin against the bin before it (kind = the bin's
    global id; bins of a spectrum's START side, then END side)."""
    d_all, t_all, s_all, k_all, sd_all = [], [], [], [], []
    bin_base = 0
    for side_k, side in enumerate(("START", "END")):
        rows, off = _sides(c, side)
        su, ob = c.su[rows], c.obs[rows]
        n = len(rows)
        if n == 0:
            continue
        first = np.zeros(n, dtype=bool)
        first[off[:-1][np.diff(off) > 0]] = True  # first row of each side
        joins = np.zeros(n, dtype=bool)  # row i joins row i-1's bin
        joins[1:] = (su[1:] - su[:-1]) <= tolerance * (ob[:-1] + ob[1:])
        joins &= ~first
        bin_id = np.cumsum(~joins) - 1  # a bin per run
        nb = int(bin_id[-1]) + 1 if n else 0
        # a bin is explained when a later row of its side closes it, or its last
        # row is the side's last row and joined it (:150-153); the side's own
        # first bin has no predecessor
        last_of_side = np.zeros(n, dtype=bool)
        last_of_side[off[1:][np.diff(off) > 0] - 1] = True
        bstart = np.flatnonzero(~joins)
        bend = np.append(bstart[1:], n)  # exclusive
        closed = ~last_of_side[bend - 1] | (joins[bend - 1] & (bend - bstart > 1))
        side_first = first[bstart]
        # first bins: whole masses against 0.0
        fb = np.flatnonzero(side_first & closed)
        mem = np.concatenate([np.arange(bstart[b], bend[b]) for b in fb]) if len(fb) else np.zeros(0, np.int64)
        d_all.append(su[mem])
        t_all.append(tolerance * (0.0 + ob[mem]))
        s_all.append(c.spec[rows[mem]])
        k_all.append(bin_base + bin_id[mem])
        sd_all.append(np.full(len(mem), side_k))
        # later bins against their predecessor: |prev| x |cur| pairs
        lb = np.flatnonzero(~side_first & closed)
        if len(lb):
            psz = (bend - bstart)[lb - 1]
            csz = (bend - bstart)[lb]
            reps = psz * csz
            tot = int(reps.sum())
            grp = np.repeat(np.arange(len(lb)), reps)
            local = np.arange(tot) - np.repeat(np.cumsum(reps) - reps, reps)
            p = bstart[lb - 1][grp] + local // csz[grp]
            q = bstart[lb][grp] + local % csz[grp]
            d_all.append(su[q] - su[p])
            t_all.append(tolerance * (ob[p] + ob[q]))
            s_all.append(c.spec[rows[q]])
            k_all.append(bin_base + bin_id[q])
            sd_all.append(np.full(len(q), side_k))
        bin_base += nb
    cat = (lambda x: np.concatenate(x)) if d_all else (lambda x: np.zeros(0))
    return Queries(cat(d_all), cat(t_all), cat(s_all).astype(np.int64), cat(k_all).astype(np.int64),
                   cat(sd_all).astype(np.int8))


def row_masks(rows_bool):
    """[S, N] bool row membership -> [S, 2] u64 masks (rows 0..63, 64..119)."""
    b = np.asarray(rows_bool, dtype=bool)
    S, N = b.shape
    out = np.zeros((S, 2), np.uint64)
    for r in range(N):
        if b[:, r].any():
            out[b[:, r], r >> 6] |= np.uint64(1) << np.uint64(r & 63)
    return out


def mask_rows(masks, n_rows):
    """[S, 2] u64 masks -> [S, n_rows] bool."""
    m = np.asarray(masks, dtype=np.uint64).reshape(-1, 2)
    r = np.arange(n_rows)
    return ((m[:, r >> 6] >> (r & 63).astype(np.uint64)) & np.uint64(1)).astype(bool)


@dataclass
class Fixpoint:
    """filter_by_explanation over many spectra: final alphabets (row masks of
    the full table), the surviving rows of the Classified frame, the rounds
    each spectrum ran, and the last round's queries / answers (the
    explanation dict the skeleton stage reads: keep marks its entries)."""
    alpha: np.ndarray        # [S, 2] u64
    alive: np.ndarray        # [rows] bool
    rounds: np.ndarray       # [S]
    history: list            # per round: (active spectra [S] bool, alpha [S, 2], alive [rows]) when recorded
    last: dict               # spectrum-major arrays of the final round: diff, thr, spec, kind, status, count,
    #                          rowmask, range, keep
    queries: list = None     # per round: (explain queries, is_valid queries)


def filter_fixpoint(c: Classified, dp_table, max_len, explanation_masses, tolerance=None,
                    record=False):
    """Predictor.filter_by_explanation (prediction.py:170-202) for every
    spectrum of `c` at once.  dp_table: the full alphabet's table (its rows
    are the mask bits); max_len[s]: spectrum s's SequenceInformation.max_len
    (its budgets).  Per round and spectrum, as the reference: explain every
    sliding-window pair of both sides and every singleton (the dict
    collect_diff_explanations_for_su builds), reduce the alphabet to the
    canonical rows plus the modifications the dict's explanations name
    (adapt_individual_modification_rates_by_alphabet_reduction,
    mass_table.py:94-100), keep the fragments is_valid_mass accepts on the
    reduced table (:204-227); repeat while the alphabet shrank.  Every window
    of these rounds is pair-class (a difference below the heaviest nucleotide,
    or a singleton's mass); budgets cannot bind once max_modifications and the
    modification rows' caps are >= 2, which is checked (smaller budgets raise
    NotImplementedError: the per-spectrum mirror handles them)."""
    tolerance = dp_table.tolerance if tolerance is None else tolerance  # prediction.py:219, :280, :315
    dev = dp_table.device_table
    masses = dp_table.masses
    N = len(masses)
    S = len(c.offsets) - 1
    max_len = np.broadcast_to(np.asarray(max_len, dtype=np.int64), (S,))
    is_mod = np.array([m.is_modification for m in masses])
    rows_all = np.zeros((1, N), bool)
    rows_all[0, 1:] = True
    alpha = np.repeat(row_masks(rows_all), S, axis=0)
    canon = row_masks((~is_mod & (np.arange(N) > 0))[None, :])[0]
    # budgets: max_modifications = round(0.5 max_len) (common.py:55) and the
    # modification rows' caps round(max_len * rate) (mass_explanation.py:158-172)
    from .pipeline_device import budgets_pair_ok

    pair_ok = budgets_pair_ok(dp_table, max_len)  # else: the exact masked explain answers the spectrum's windows
    max_w = max(explanation_masses.get_column("monoisotopic_mass").to_list()) + PHOSPHATE_LINK_MASS
    side = np.array([("START" in n) | (("END" in n) << 1) for n in c.names], dtype=np.uint8)
    flags = side[c.brk] | (np.asarray(c.singleton, dtype=np.uint8) << 2)
    alive = np.ones(len(c.su), bool)
    active = np.ones(S, bool)
    rounds = np.zeros(S, np.int64)
    history = []
    parts = []  # (spectra active in the round, the round's queries and answers)
    n_queries = []
    pop = lambda m: np.bitwise_count(np.asarray(m, dtype=np.uint64)).sum(axis=1)  # noqa: E731
    while active.any():
        rows = np.flatnonzero(alive & active[c.spec])
        off = np.searchsorted(c.spec[rows], np.arange(S + 1))
        d, t, g, k = _su_diff_queries(c.su[rows], c.obs[rows], flags[rows], off, max_w, tolerance)
        st, cnt, rm, rg = dev.explain_pairs_alpha(d, t, g, alpha, tolerance, dp_table.precision)
        ex = ~pair_ok[g]
        if ex.any():  # budgets can bind: the exact replay on each spectrum's alphabet
            st[ex], cnt[ex], rm[ex] = _exact_answers(dp_table, d[ex], t[ex], g[ex], alpha, max_len, tolerance)
        if (st == -10).any():
            raise NotImplementedError("filter_fixpoint: a window outside the pair class")
        q_off = np.searchsorted(g, np.arange(S + 1))
        from ._native import dict_union

        keep, union = dict_union(q_off, d, k, st, rm)
        new_alpha = alpha.copy()
        new_alpha[active] = canon[None, :] | (alpha[active] & union[active])
        changed = pop(new_alpha) != pop(alpha)
        parts.append((active.copy(), {"diff": d, "thr": t, "spec": g, "kind": k, "status": st, "count": cnt, "rowmask": rm,
                      "range": rg, "keep": keep}))
        alpha = new_alpha
        rounds[active] += 1
        # _reduce_alphabet's is_valid_mass filter on the reduced tables (:211-227)
        v = dev.is_valid_alpha(c.su[rows], tolerance * c.obs[rows], off, alpha, tolerance, dp_table.precision)
        if (v < 0).any():
            raise NotImplementedError("is_valid_mass raised on a reduced table (window past its extent)")
        alive[rows[v != 1]] = False
        n_queries.append((len(d), len(rows)))
        if record:
            history.append((active.copy(), alpha.copy(), alive.copy()))
        active &= changed
    return Fixpoint(alpha, alive, rounds, history, _final_round(parts, S), n_queries)


def _exact_answers(dp_table, diff, thr, spec, alpha, max_len, tolerance):
    """Windows of budget-binding spectra through the exact masked explain
    (sst_explain_alpha_batch_device, one pass per max_len group): status,
    candidate count and the union of the candidates' rows."""
    dev = dp_table.device_table
    masses = dp_table.masses
    is_mod = [m.is_modification for m in masses]
    st = np.zeros(len(diff), np.int8)
    cnt = np.zeros(len(diff), np.uint32)
    rm = np.zeros((len(diff), 2), np.uint64)
    ml = np.asarray(max_len, dtype=np.int64)[spec]
    for L in np.unique(ml):
        sel = np.flatnonzero(ml == L)
        dev.set_budgets(is_mod, [round(int(L) * m.modification_rate) for m in masses])
        res = dev.explain_alpha(diff[sel], thr[sel], spec[sel].astype(np.int32), alpha, tolerance,
                                dp_table.precision, round(dp_table.seq.modification_rate * int(L)))
        st[sel] = res.status
        cnt[sel] = res.count
        for j, i in enumerate(sel):
            for c in res.candidates(j):
                for r in c:
                    rm[i, r >> 6] |= np.uint64(1) << np.uint64(r & 63)
    return st, cnt, rm


def _final_round(parts, S):
    """Each spectrum's queries and answers of its last round, spectrum-major."""
    if not parts:
        return {}
    final_part = np.full(S, -1, np.int64)
    for j, (act, _) in enumerate(parts):
        final_part[act] = j
    out = {}
    keys = parts[0][1].keys()
    sel = []
    for j, (_, rd) in enumerate(parts):
        sel.append(final_part[rd["spec"]] == j)
    for kk in keys:
        out[kk] = np.concatenate([rd[kk][m] for (_, rd), m in zip(parts, sel)])
    order = np.argsort(out["spec"], kind="stable")
    return {kk: v[order] for kk, v in out.items()}
