"""Config 5 with every stage's arrays in HBM: classify_fragments,
the filter_by_explanation fixpoint and the skeleton's speculative bin
queries over many spectra, driven from the host one launch per stage / round
(sst_classify_rows_device, sst_fix_round_device, sst_valid_rows_alpha_device,
sst_bins_count_device / sst_bins_emit_device; kernels in csrc/sst_pipe.hip
and csrc/sst_alpha.hip).  The host only loops the rounds (one 4-byte read per
round: how many spectra are still reducing) and sizes the bin answers (one
8-byte read).

Rows of spectrum g sit in slots 4 * peak_off[g] + i (i < rows[g]), in the
SU order of its classify_fragments frame, so a row's slot offset is the
`index` Predictor.predict gives it (prediction.py:68-72).  PyTorch provides
the device memory only; every computation is the library's.
"""
from dataclasses import dataclass

import numpy as np

from . import _native
from .masses import PHOSPHATE_LINK_MASS
from .pipeline import mask_rows, row_masks

ERR_BITS = {1: "a spectrum has more than 1024 peaks", 2: "a spectrum has more than 2048 rows",
            4: "a window outside the pair class", 8: "is_valid_mass raised (a window past a table's end)",
            16: "an explanation dict too large for the LDS hash", 32: "rows out of mass order"}


def _check_err(err):
    e = int(err.item())
    if e:
        raise _native.EngineError("device pipeline: " + "; ".join(v for k, v in ERR_BITS.items() if e & k))


@dataclass
class DeviceRows:
    """classify_fragments' frames of a batch, on the device."""
    peak_off: object   # torch int64 [S + 1]
    su: object         # torch f64 [4 P] row slots
    obs: object
    meta: object       # torch int32: breakage | sides << 2 | singleton << 4 | peak << 8
    alive: object      # torch uint8
    rows: object       # torch int32 [S]
    valid: object      # torch int8 [4 P] A7 codes (breakage-major) or None
    names: list        # breakage label per code


def classify_device(dp_table, obs, offsets, su_seq, breakage_dict, intensity=None, intensity_cutoff=0.5e6,
                    mass_cutoff=50000, keep_valid=False, device=None):
    """Stage 1 on the device.  obs: every spectrum's peaks (spectrum g:
    obs[offsets[g]:offsets[g+1]]), su_seq[g] its SequenceInformation.su_mass.
    Peaks may come in any order: the kernel ranks each spectrum's peaks by
    mass in LDS (equal masses keep their order, so the rows' SU order and its
    ties are the reference's); the rows' peak positions are the caller's."""
    import torch

    dev = device or torch.device("cuda", dp_table.device_table.engine.device)
    obs_t = torch.as_tensor(np.ascontiguousarray(obs, dtype=np.float64), device=dev)
    off_t = torch.as_tensor(np.ascontiguousarray(offsets, dtype=np.int64), device=dev)
    su_t = torch.as_tensor(np.ascontiguousarray(su_seq, dtype=np.float64), device=dev)
    int_t = None if intensity is None else torch.as_tensor(np.ascontiguousarray(intensity, dtype=np.float64),
                                                           device=dev)
    P, S = len(obs), len(offsets) - 1
    weights = list(breakage_dict.keys())
    names = [breakage_dict[w][0] for w in weights]
    shifts = np.array([w * dp_table.precision for w in weights], dtype=np.float64)
    sides = np.array([("START" in n) | (("END" in n) << 1) for n in names], dtype=np.uint8)
    max_w = _max_weight()
    su = torch.empty(max(1, 4 * P), dtype=torch.float64, device=dev)
    ob = torch.empty_like(su)
    meta = torch.empty(max(1, 4 * P), dtype=torch.int32, device=dev)
    alive = torch.zeros(max(1, 4 * P), dtype=torch.uint8, device=dev)
    rows = torch.zeros(max(1, S), dtype=torch.int32, device=dev)
    valid = torch.empty(max(1, len(weights) * P), dtype=torch.int8, device=dev) if keep_valid else None
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    eng = dp_table.device_table.engine
    torch.cuda.synchronize(dev)
    eng.check(eng._lib.sst_classify_rows_device(
        dp_table.device_table.handle, obs_t.data_ptr(), off_t.data_ptr(), S, P,
        None if int_t is None else int_t.data_ptr(), float(intensity_cutoff), float(mass_cutoff), su_t.data_ptr(),
        _native._ptr(shifts), _native._ptr(sides), len(shifts), float(max_w), float(dp_table.tolerance),
        float(dp_table.precision), None if valid is None else valid.data_ptr(), su.data_ptr(), ob.data_ptr(),
        meta.data_ptr(), alive.data_ptr(), rows.data_ptr(), err.data_ptr()), "sst_classify_rows_device")
    eng.synchronize()
    _check_err(err)
    return DeviceRows(off_t, su, ob, meta, alive, rows, valid, names)


def _max_weight(explanation_masses=None):
    from .masses import EXPLANATION_MASSES

    em = explanation_masses if explanation_masses is not None else EXPLANATION_MASSES
    return max(em.get_column("monoisotopic_mass").to_list()) + PHOSPHATE_LINK_MASS


@dataclass
class DeviceFixpoint:
    alpha: np.ndarray     # [S, 2] u64 final alphabets (row masks of the full table)
    rounds: np.ndarray    # [S]
    queries: np.ndarray   # [S] explain queries over all rounds
    history: list         # per round (recorded): (active [S] bool, alpha [S, 2], alive slots)
    n_rounds: int


def fixpoint_device(dp_table, rows: DeviceRows, max_len, tolerance=None, record=False):
    """Stage 2 on the device: Predictor.filter_by_explanation (prediction.py:
    170-202) for every spectrum, one sst_fix_round_device + one
    sst_valid_rows_alpha_device launch per round, until no alphabet shrinks.
    max_len[s] bounds the budgets (checked as in pipeline.filter_fixpoint)."""
    tolerance = dp_table.tolerance if tolerance is None else tolerance  # prediction.py:219, :280, :315
    import torch

    masses = dp_table.masses
    N = len(masses)
    S = len(rows.rows)
    dev = rows.su.device
    is_mod = np.array([m.is_modification for m in masses])
    rate = np.array([m.modification_rate for m in masses], dtype=np.float64)
    max_len = np.broadcast_to(np.asarray(max_len, dtype=np.int64), (S,))
    # round() on the same f64 products, ties to even like Python's round (vectorised over spectra)
    A = np.round(dp_table.seq.modification_rate * max_len.astype(np.float64)).astype(np.int64)
    cap_min = (np.round(np.outer(max_len.astype(np.float64), rate[is_mod])).min(axis=1).astype(np.int64)
               if is_mod.any() else np.full(S, 2, dtype=np.int64))
    if (A < 2).any() or (cap_min < 2).any():
        raise NotImplementedError("fixpoint_device: budgets that can bind on pair windows (max_len too small)")
    full = np.zeros((1, N), bool)
    full[0, 1:] = True
    alpha = torch.as_tensor(np.repeat(row_masks(full), S, axis=0).view(np.int64), device=dev).contiguous()
    alpha_next = torch.empty_like(alpha)
    active = torch.ones(S, dtype=torch.uint8, device=dev)
    active_next = torch.empty_like(active)
    rounds = torch.zeros(S, dtype=torch.int32, device=dev)
    queries = torch.zeros(S, dtype=torch.int32, device=dev)
    ctl = torch.zeros(2, dtype=torch.int32, device=dev)  # [0] spectra whose alphabet shrank, [1] error bits
    n_active, err = ctl[0:1], ctl[1:2]
    eng = dp_table.device_table.engine
    L = eng._lib
    h = dp_table.device_table.handle
    history = []
    n_rounds = 0
    max_w = _max_weight()
    torch.cuda.synchronize(dev)
    while True:  # per round: two launches, one synchronize, one 8-byte read
        eng.check(L.sst_fix_round_device(h, rows.peak_off.data_ptr(), S, rows.su.data_ptr(), rows.obs.data_ptr(),
                                         rows.meta.data_ptr(), rows.alive.data_ptr(), rows.rows.data_ptr(),
                                         alpha.data_ptr(), alpha_next.data_ptr(), active.data_ptr(),
                                         active_next.data_ptr(), rounds.data_ptr(), queries.data_ptr(),
                                         n_active.data_ptr(), float(max_w), float(tolerance),
                                         float(dp_table.precision), err.data_ptr()), "sst_fix_round_device")
        # re-filter only the spectra whose alphabet shrank: an unchanged alphabet is
        # the table the rows already passed (round 1: classify's full table)
        eng.check(L.sst_valid_rows_alpha_device(h, rows.peak_off.data_ptr(), S, rows.su.data_ptr(),
                                                rows.obs.data_ptr(), rows.rows.data_ptr(), alpha_next.data_ptr(),
                                                active_next.data_ptr(), rows.alive.data_ptr(), float(tolerance),
                                                float(dp_table.precision), err.data_ptr()),
                  "sst_valid_rows_alpha_device")
        eng.synchronize()
        n_rounds += 1
        if record:
            history.append((active.cpu().numpy().astype(bool), alpha_next.cpu().numpy().view(np.uint64).copy(),
                            rows.alive.cpu().numpy().astype(bool)))
        n_act, e = (int(x) for x in ctl.cpu().tolist())
        if e:
            _check_err(err)
        alpha, alpha_next = alpha_next, alpha
        active, active_next = active_next, active
        if n_act == 0:
            break
    return DeviceFixpoint(alpha.cpu().numpy().view(np.uint64).copy(), rounds.cpu().numpy(),
                          queries.cpu().numpy(), history, n_rounds)


def to_classified(rows: DeviceRows, alive_only=True):
    """The device rows back on the host as pipeline.Classified (spectrum-major,
    each spectrum's rows in SU order; with alive_only the rows the fixpoint
    kept) -- the input of the host stages after the fixpoint (bin queries)."""
    from .pipeline import Classified

    off = rows.peak_off.cpu().numpy()
    cnt = rows.rows.cpu().numpy().astype(np.int64)[:len(off) - 1]
    S = len(cnt)
    spec = np.repeat(np.arange(S), cnt)
    local = np.arange(int(cnt.sum())) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    slot = 4 * off[:-1][spec] + local
    su, ob = rows.su.cpu().numpy()[slot], rows.obs.cpu().numpy()[slot]
    meta = rows.meta.cpu().numpy()[slot]
    keep = rows.alive.cpu().numpy()[slot].astype(bool) if alive_only else np.ones(len(slot), bool)
    spec, su, ob, meta = spec[keep], su[keep], ob[keep], meta[keep]
    offsets = np.searchsorted(spec, np.arange(S + 1))
    return Classified(spec, su, ob, (meta >> 8).astype(np.int64), (meta & 3).astype(np.int64),
                      ((meta >> 4) & 1).astype(bool), rows.names, offsets, 0, 0)


@dataclass
class DeviceBins:
    """The skeleton's speculative bin queries of every spectrum, answered on
    its alphabet (spectrum-major: START side, then END; bins in order)."""
    q_off: np.ndarray     # [S + 1] query offsets per spectrum
    status: object        # torch int8 [Q]: SST_NONE / EMPTY / SOME (-10 off the pair class when not answered)
    count: object         # torch int32 [Q] candidates
    deferred: dict = None  # the off-pair-class queries' masked explain: n, per max_len group results, tallies


def bins_device(dp_table, rows: DeviceRows, alpha, tolerance=None, max_len=None):
    """Stage 3 on the device (SkeletonBuilder._predict_skeleton's bins,
    skeleton_building.py:114-160) over the rows the fixpoint kept
    (rows.alive) and the final alphabets `alpha` ([S, 2] u64 row masks).
    Pair-class windows are answered by k_bins_emit; with max_len (per
    spectrum) the others -- the sides' first bins' whole masses and wide bin
    differences -- are listed by it and answered by the masked explain
    (sst_explain_alpha_batch_device, the DFS roles on each spectrum's
    alphabet), one pass per max_len group (its budgets: round(0.5 max_len),
    caps round(max_len * rate), common.py:55, mass_explanation.py:158-172)."""
    tolerance = dp_table.tolerance if tolerance is None else tolerance  # prediction.py:219, :280, :315
    import torch

    S = len(rows.rows)
    dev = rows.su.device
    a = torch.as_tensor(np.ascontiguousarray(alpha, dtype=np.uint64).view(np.int64), device=dev)
    n_q = torch.zeros(max(1, S), dtype=torch.int32, device=dev)
    q_off = torch.zeros(S + 1, dtype=torch.int64, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    eng = dp_table.device_table.engine
    L = eng._lib
    h = dp_table.device_table.handle
    torch.cuda.synchronize(dev)
    eng.check(L.sst_bins_count_device(h, rows.peak_off.data_ptr(), S, rows.su.data_ptr(), rows.obs.data_ptr(),
                                      rows.meta.data_ptr(), rows.alive.data_ptr(), rows.rows.data_ptr(),
                                      float(tolerance), n_q.data_ptr(), q_off.data_ptr(), err.data_ptr()),
              "sst_bins_count_device")
    eng.synchronize()
    _check_err(err)
    total = int(q_off[S].item())
    status = torch.empty(max(1, total), dtype=torch.int8, device=dev)
    count = torch.empty(max(1, total), dtype=torch.int32, device=dev)
    defer = max_len is not None
    if defer:
        d_mass = torch.empty(max(1, total), dtype=torch.float64, device=dev)
        d_thr = torch.empty_like(d_mass)
        d_spec = torch.empty(max(1, total), dtype=torch.int32, device=dev)
        d_q = torch.empty(max(1, total), dtype=torch.int64, device=dev)
        n_def = torch.zeros(1, dtype=torch.int32, device=dev)
    ptr = (lambda x: x.data_ptr()) if defer else (lambda x: None)
    eng.check(L.sst_bins_emit_device(h, rows.peak_off.data_ptr(), S, rows.su.data_ptr(), rows.obs.data_ptr(),
                                     rows.meta.data_ptr(), rows.alive.data_ptr(), rows.rows.data_ptr(), a.data_ptr(),
                                     float(tolerance), float(dp_table.precision), q_off.data_ptr(),
                                     status.data_ptr(), count.data_ptr(), ptr(d_mass) if defer else None,
                                     ptr(d_thr) if defer else None, ptr(d_spec) if defer else None,
                                     ptr(d_q) if defer else None, ptr(n_def) if defer else None, err.data_ptr()),
              "sst_bins_emit_device")
    eng.synchronize()
    _check_err(err)
    out = DeviceBins(q_off.cpu().numpy(), status[:total], count[:total])
    if defer:
        out.deferred = answer_deferred(dp_table, a, d_mass, d_thr, d_spec, d_q, int(n_def.item()), max_len,
                                       status, count)
    return out


def answer_deferred(dp_table, alpha, d_mass, d_thr, d_spec, d_q, n, max_len, status, count):
    """The listed off-pair-class windows through the masked explain, one pass
    per max_len group (the rows' caps follow max_len); statuses and counts
    scattered into the bin-query arrays.  Returns the per-group results."""
    import torch

    dt = dp_table.device_table
    eng = dt.engine
    info = {"queries": n, "groups": [], "results": []}
    if n == 0:
        return info
    spec = d_spec[:n].cpu().numpy()
    ml = np.asarray(max_len, dtype=np.int64)[spec]
    order = np.argsort(ml, kind="stable")
    o = torch.as_tensor(order, device=d_mass.device)
    mass, thr = d_mass[:n][o].contiguous(), d_thr[:n][o].contiguous()
    sp, qi = d_spec[:n][o].contiguous(), d_q[:n][o].contiguous()
    ml_s = ml[order]
    info["spec"], info["mass"], info["thr"] = sp.cpu().numpy(), mass.cpu().numpy(), thr.cpu().numpy()
    bounds = np.flatnonzero(np.diff(ml_s)) + 1
    starts = np.concatenate([[0], bounds])
    ends = np.concatenate([bounds, [n]])
    masses = dp_table.masses
    is_mod = [m.is_modification for m in masses]
    A_rate = dp_table.seq.modification_rate
    for s0, s1 in zip(starts.tolist(), ends.tolist()):
        L = int(ml_s[s0])
        dt.set_budgets(is_mod, [round(L * m.modification_rate) for m in masses])
        k = int(s1 - s0)
        res = dt.explain_alpha_device(mass.data_ptr() + 8 * s0, thr.data_ptr() + 8 * s0, sp.data_ptr() + 4 * s0,
                                      alpha.data_ptr(), k, dp_table.tolerance, dp_table.precision,
                                      round(A_rate * L))
        res.fetch_device()
        idx = qi[s0:s1]
        status[idx] = torch.as_tensor(res.status, device=status.device)
        count[idx] = torch.as_tensor(res.count.astype(np.int32), device=count.device)
        info["groups"].append((L, k))
        info["results"].append((int(s0), res))
    info["order"] = order
    return info
