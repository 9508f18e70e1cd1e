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
the device memory, plus the index gathers that set up a masked-explain pass's
per-query budget rows (_lens_pass); every stage's computation -- the rounds'
re-query merge included (sst_requery_merge_device) -- is the library's.
"""
import ctypes
import os
import sys
import time
from dataclasses import dataclass

import numpy as np

from . import _native
from .masses import PHOSPHATE_LINK_MASS
from .pipeline import mask_rows, row_masks

_PROGRESS = os.environ.get("SST_PIPE_PROGRESS") == "1"  # per-launch lines of the long stages on stderr

# Stage 5's one device buffer per GPU for a pass's reach bitsets and
# lowest-rank bytes (tens of GB at 100 k spectra): kept between length passes
# unless the pass trims (allocating and releasing it per call put up to a few
# seconds of hipMalloc / hipFree into the stage, from run to run).
_LEN_BUF = {}


def _length_buffer(dev, nbytes):
    import torch

    key = dev.index if dev.index is not None else 0
    b = _LEN_BUF.get(key)
    if b is None or b.numel() < nbytes:
        _LEN_BUF.pop(key, None)
        b = None
        torch.cuda.empty_cache()
        b = torch.empty(max(256, int(nbytes)), dtype=torch.uint8, device=dev)
        _LEN_BUF[key] = b
    return b


def reserve_length_buffer(dev, nbytes=64 << 30):
    """Allocate stage 5's reach buffer ahead (a serving process's warm-up):
    passes whose batches fit it (length_device's reach_budget_bytes is the
    default size) then allocate nothing.  At most half of the device's free
    memory (ranks sharing a GPU; the frontier's own workspace is allocated in
    the warm-up's pass before this); a pass that needs more allocates it
    then, as without a reservation."""
    import torch

    free, _ = torch.cuda.mem_get_info(dev)
    try:
        _length_buffer(dev, min(int(nbytes), int(free) // 2))
    except torch.OutOfMemoryError:
        release_length_buffer(dev)


def release_length_buffer(dev=None):
    """Free stage 5's reach buffer (every GPU's when dev is None)."""
    import torch

    if dev is None:
        _LEN_BUF.clear()
    else:
        _LEN_BUF.pop(dev.index if dev.index is not None else 0, None)
    torch.cuda.empty_cache()
LB_NOT_RUN = -6  # length_device(spectra=...): the bounds of a spectrum outside the sample
MAX_PEAKS = 16383  # peaks per spectrum (sst_internal.h kPipeMaxPeaksBig: above 4096 in HBM slices)
ERR_BITS = {1: f"a spectrum has more than {MAX_PEAKS} peaks", 2: "a spectrum has more rows than the reserved slices hold",
            4: "a window outside the pair class", 8: "is_valid_mass raised (a window past a table's end)",
            16: "an explanation dict too large for the LDS hash", 32: "rows out of mass order",
            64: "an exact-mode query list overflowed", 128: "an exact-mode answer raised or was capped"}


def _one_stream(fn):
    """Run a stage with the engine and PyTorch on one stream.  The stages mix
    engine launches (the ctx's stream) with PyTorch uploads, fills and reads
    (the caller's current stream); on two streams a kernel could read an
    input before its upload lands, or a read see a buffer before the kernel
    that fills it has run.  The stage runs on a private stream that first
    waits for the caller's, with the engine queued on it
    (sst_ctx_set_stream); the caller's stream waits for it at the end."""
    import functools

    @functools.wraps(fn)
    def run(dp_table, *args, **kw):
        import torch

        eng = dp_table.device_table.engine
        dev = torch.device("cuda", eng.device)
        st = _STREAMS.get(eng.device)
        if st is None:
            st = _STREAMS[eng.device] = torch.cuda.Stream(device=dev)
        caller = torch.cuda.current_stream(dev)
        prev = getattr(eng, "_stage_stream", None)  # an enclosing stage's (stages nest)
        st.wait_stream(caller)
        try:
            with torch.cuda.stream(st):
                eng.set_stream(st.cuda_stream)
                eng._stage_stream = st.cuda_stream
                return fn(dp_table, *args, **kw)
        finally:
            eng.set_stream(prev)
            eng._stage_stream = prev
            caller.wait_stream(st)
    return run


_STREAMS = {}


class _Heartbeat:
    """Prints `what` every `period` seconds on stderr until stop() (a long
    device call holds no Python lock, so a watcher sees the run is alive)."""

    def __init__(self, what, period):
        import threading
        import time

        self._stop = threading.Event()
        t0 = time.perf_counter()

        def run():
            while not self._stop.wait(period):
                print(f"{what}: {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)

        self._t = threading.Thread(target=run, daemon=True)
        self._t.start()

    def stop(self):
        self._stop.set()
        self._t.join()


def _check_err(err):
    e = int(err.item())
    if e:
        known = [v for k, v in ERR_BITS.items() if e & k]
        rest = e & ~sum(ERR_BITS)
        if rest:
            known.append(f"unknown error bits {rest:#x}")
        raise _native.EngineError("device pipeline: " + "; ".join(known))


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


@_one_stream
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
    eng = dp_table.device_table.engine
    # spectra of more than 2048 rows run in the context's HBM slices (sst_pipe_reserve_rows)
    peaks = np.diff(np.asarray(offsets, dtype=np.int64))
    if len(peaks):
        eng.check(eng._lib.sst_pipe_reserve_rows(dp_table.device_table.handle,
                                                 min(int(peaks.max()), MAX_PEAKS) * len(shifts)),
                  "sst_pipe_reserve_rows")
    su = torch.empty(max(1, 4 * P), dtype=torch.float64, device=dev)
    ob = torch.empty_like(su)
    meta = torch.empty(max(1, 4 * P), dtype=torch.int32, device=dev)
    alive = torch.zeros(max(1, 4 * P), dtype=torch.uint8, device=dev)
    rows = torch.zeros(max(1, S), dtype=torch.int32, device=dev)
    valid = torch.empty(max(1, len(weights) * P), dtype=torch.int8, device=dev) if keep_valid else None
    err = torch.zeros(1, dtype=torch.int32, device=dev)
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


class _ExactLists:
    """Exact-mode (budget-binding) spectra's query lists and their answers
    (sst_exact_io): capacity for a round's queries, the masked explain per
    max_len group, the answers' references."""

    def __init__(self, dp_table, rows, pair_ok, max_len, cap=None):
        import torch

        self.dp = dp_table
        self.rows = rows
        self.max_len = np.asarray(max_len, dtype=np.int64)
        self.dev = rows.su.device
        S = len(rows.rows)
        self.ok = torch.as_tensor(np.asarray(pair_ok, dtype=np.uint8), device=self.dev)
        self.exact = torch.as_tensor(~np.asarray(pair_ok, bool), device=self.dev)
        self.block = torch.zeros(max(1, S), dtype=torch.int64, device=self.dev)
        self.count = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.cap = 0
        self.results = []
        self.io = _native.ExactIO()
        self.io.pair_ok = self.ok.data_ptr()
        self.io.xq_count = self.count.data_ptr()
        self.io.xq_block = self.block.data_ptr()
        self._alloc(max(1024, int(cap or 0)))

    def _alloc(self, cap):
        import torch

        self.cap = cap
        self.mass = torch.empty(cap, dtype=torch.float64, device=self.dev)
        self.thr = torch.empty(cap, dtype=torch.float64, device=self.dev)
        self.spec = torch.empty(cap, dtype=torch.int32, device=self.dev)
        self.single = torch.empty(cap, dtype=torch.uint8, device=self.dev)
        self.st = torch.empty(cap, dtype=torch.int8, device=self.dev)
        self.n = torch.empty(cap, dtype=torch.int32, device=self.dev)
        self.ptr = torch.empty(cap, dtype=torch.int64, device=self.dev)
        io = self.io
        io.xq_mass, io.xq_thr, io.xq_spec = self.mass.data_ptr(), self.thr.data_ptr(), self.spec.data_ptr()
        io.xq_single, io.xq_cap = self.single.data_ptr(), cap
        io.xa_st, io.xa_n, io.xa_ptr = self.st.data_ptr(), self.n.data_ptr(), self.ptr.data_ptr()

    def reset(self):
        self.count.zero_()
        self.results = []

    def prepare(self, active):
        """Before a fixpoint round: room for the exact-mode active spectra's
        queries (their count from sst_dict_count_device on the current rows)."""
        import torch

        dp, r = self.dp, self.rows
        eng = dp.device_table.engine
        S = len(r.rows)
        n_q = torch.zeros(max(1, S), dtype=torch.int32, device=self.dev)
        off = torch.zeros(S + 1, dtype=torch.int64, device=self.dev)
        err = torch.zeros(1, dtype=torch.int32, device=self.dev)
        eng.check(eng._lib.sst_dict_count_device(dp.device_table.handle, r.peak_off.data_ptr(), S, r.su.data_ptr(),
                                                 r.obs.data_ptr(), r.meta.data_ptr(), r.alive.data_ptr(),
                                                 r.rows.data_ptr(), float(_max_weight()), float(dp.tolerance),
                                                 n_q.data_ptr(), off.data_ptr(), err.data_ptr()),
                  "sst_dict_count_device")
        need = int((n_q[:S].to(torch.int64) * (active[:S].to(torch.bool) & self.exact[:S])).sum().item())
        if need > self.cap:
            self._alloc(need)
        self.reset()

    def answer(self, alpha_dev):
        """The listed queries through the exact masked explain (one pass per
        max_len group), their references into xa_*."""
        import torch

        n = int(self.count.item())
        if n > self.cap:
            raise _native.EngineError("exact-mode query list overflow")
        if n == 0:
            return
        self.st[:n].fill_(-10)
        dst = torch.arange(n, dtype=torch.int64, device=self.dev)
        self.results = _masked_explain_refs(self.dp, alpha_dev, self.mass, self.thr, self.spec, n, self.max_len, dst,
                                            self.ptr, self.n, self.st)


@dataclass
class DeviceFixpoint:
    alpha: np.ndarray     # [S, 2] u64 final alphabets (row masks of the full table)
    rounds: np.ndarray    # [S]
    queries: np.ndarray   # [S] explain queries over all rounds
    history: list         # per round (recorded): (active [S] bool, alpha [S, 2], alive slots)
    n_rounds: int


@_one_stream
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
    max_len = np.ascontiguousarray(np.broadcast_to(np.asarray(max_len, dtype=np.int64), (S,)))
    # spectra whose budgets can bind on pair windows run in exact mode: their
    # queries go to the exact masked explain (sst_exact_io)
    ok = budgets_pair_ok(dp_table, max_len)
    xio = None if ok.all() else _ExactLists(dp_table, rows, ok, max_len)
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
        xp = None
        if xio is not None:  # list capacity: the round's queries of the exact-mode spectra
            xio.prepare(active)
            xp = ctypes.byref(xio.io)
        eng.check(L.sst_fix_round_device(h, rows.peak_off.data_ptr(), S, rows.su.data_ptr(), rows.obs.data_ptr(),
                                         rows.meta.data_ptr(), rows.alive.data_ptr(), rows.rows.data_ptr(),
                                         alpha.data_ptr(), alpha_next.data_ptr(), active.data_ptr(),
                                         active_next.data_ptr(), rounds.data_ptr(), queries.data_ptr(),
                                         n_active.data_ptr(), float(max_w), float(tolerance),
                                         float(dp_table.precision), err.data_ptr(), xp), "sst_fix_round_device")
        if xio is not None:  # the listed queries answered exactly, then the exact-mode half of the round
            xio.answer(alpha)
            eng.check(L.sst_fix_finish_device(h, S, rows.rows.data_ptr(), alpha.data_ptr(), alpha_next.data_ptr(), active.data_ptr(),
                                              active_next.data_ptr(), rounds.data_ptr(), queries.data_ptr(),
                                              n_active.data_ptr(), err.data_ptr(), xp), "sst_fix_finish_device")
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
    q_off_dev: object = None  # torch int64 [S + 1] (the walk's view of the speculative queries)
    q0_dev: object = None     # torch int32 [S] the START side's count
    alpha_dev: object = None  # torch int64 [S, 2] the alphabets they were answered on


@_one_stream
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
    n_q0 = torch.zeros(max(1, S), dtype=torch.int32, device=dev)
    q_off = torch.zeros(S + 1, dtype=torch.int64, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    eng = dp_table.device_table.engine
    L = eng._lib
    h = dp_table.device_table.handle
    torch.cuda.synchronize(dev)
    eng.check(L.sst_bins_count_device(h, rows.peak_off.data_ptr(), S, rows.su.data_ptr(), rows.obs.data_ptr(),
                                      rows.meta.data_ptr(), rows.alive.data_ptr(), rows.rows.data_ptr(),
                                      float(tolerance), n_q.data_ptr(), q_off.data_ptr(), err.data_ptr(),
                                      n_q0.data_ptr()),
              "sst_bins_count_device")
    eng.synchronize()
    _check_err(err)
    total = int(q_off[S].item())
    status = torch.empty(max(1, total), dtype=torch.int8, device=dev)
    count = torch.empty(max(1, total), dtype=torch.int32, device=dev)
    defer = max_len is not None
    pok = None
    if defer:
        ok = budgets_pair_ok(dp_table, np.broadcast_to(np.asarray(max_len, dtype=np.int64), (S,)))
        if not ok.all():  # exact-mode spectra: every window to the masked explain
            pok = torch.as_tensor(ok.astype(np.uint8), device=dev)
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
                                     ptr(d_q) if defer else None, ptr(n_def) if defer else None, err.data_ptr(),
                                     pok.data_ptr() if pok is not None else None),
              "sst_bins_emit_device")
    eng.synchronize()
    _check_err(err)
    out = DeviceBins(q_off.cpu().numpy(), status[:total], count[:total], q_off_dev=q_off, q0_dev=n_q0,
                     alpha_dev=a)
    if defer:
        out.deferred = answer_deferred(dp_table, a, d_mass, d_thr, d_spec, d_q, int(n_def.item()), max_len,
                                       status, count)
    return out


def answer_deferred(dp_table, alpha, d_mass, d_thr, d_spec, d_q, n, max_len, status, count):
    """The listed off-pair-class windows through the masked explain with
    their spectra's budgets (one pass, per-query budgets: the rows' caps
    follow max_len); statuses and counts scattered into the bin-query
    arrays.  Returns the pass's result and the list (in its order)."""
    import torch

    info = {"queries": n, "groups": [], "results": []}
    if n == 0:
        return info
    spec = d_spec[:n].cpu().numpy()
    ml = np.asarray(max_len, dtype=np.int64)[spec]
    info["spec"], info["mass"], info["thr"] = spec, d_mass[:n].cpu().numpy(), d_thr[:n].cpu().numpy()
    res = _lens_pass(dp_table, alpha, d_mass, d_thr, d_spec, n, max_len)
    res.fetch_device()
    idx = d_q[:n]
    status[idx] = torch.as_tensor(res.status, device=status.device)
    count[idx] = torch.as_tensor(res.count.astype(np.int32), device=count.device)
    Ls, ks = np.unique(ml, return_counts=True)
    info["groups"] = [(int(L), int(k)) for L, k in zip(Ls, ks)]
    info["results"].append((0, res))
    info["order"] = np.arange(n)
    info["dst"] = idx.contiguous()  # list position -> bin-query index
    return info


# ---------------------------------------------------------------------------
# Stage 4: SkeletonBuilder._predict_skeleton's walk on the device
# (skeleton_building.py:114-196, 372-482; kernels in csrc/sst_skel.hip)
# ---------------------------------------------------------------------------
def budgets_pair_ok(dp_table, max_len):
    """Per spectrum: budgets cannot bind on a pair-class window (<= 2 items):
    max_modifications = round(0.5 max_len) (common.py:55) and every
    modification row's cap round(max_len * rate) (mass_explanation.py:158-172)
    are >= 2 -- the fast-path theorem for the lane's pair-list answers."""
    masses = dp_table.masses
    is_mod = np.array([m.is_modification for m in masses])
    rate = np.array([m.modification_rate for m in masses], dtype=np.float64)
    ml = np.asarray(max_len, dtype=np.int64).astype(np.float64)
    A = np.round(dp_table.seq.modification_rate * ml).astype(np.int64)
    cap_min = (np.round(np.outer(ml, rate[is_mod])).min(axis=1).astype(np.int64) if is_mod.any()
               else np.full(len(ml), 2, dtype=np.int64))
    return (A >= 2) & (cap_min >= 2)


def name_hashes(dp_table):
    """hash() of each table row's nucleoside name in this interpreter (the
    set order the reference's explanation lists follow, common.py:60-65)."""
    from .mass_explanation import MASS_NAMES

    out = np.zeros(len(dp_table.masses), np.int64)
    for r, m in enumerate(dp_table.masses):
        if r == 0:
            continue
        names = MASS_NAMES[m.mass]
        if len(names) != 1:  # mass_explanation.py:302-318 would expand the product of equal-mass names
            raise NotImplementedError("skeleton walk: an integer mass with several nucleoside names")
        out[r] = hash(names[0])
    return out


@dataclass
class DeviceDict:
    off: object    # torch int64 [S + 1]
    n: object      # torch int32 [S]
    key: object    # torch int64 (double bits, ascending per spectrum)
    thr: object    # torch f64


@_one_stream
def final_dict_device(dp_table, rows: DeviceRows, alpha_dev, tolerance=None, max_len=None):
    """filter_by_explanation's final explanation dict of every spectrum
    (prediction.py:261-329 over the fixpoint's rows and alphabets), as
    sorted (key, last writer's threshold) lists on the device."""
    import torch

    tolerance = dp_table.tolerance if tolerance is None else tolerance
    S = len(rows.rows)
    dev = rows.su.device
    eng = dp_table.device_table.engine
    L = eng._lib
    h = dp_table.device_table.handle
    n_q = torch.zeros(max(1, S), dtype=torch.int32, device=dev)
    off = torch.zeros(S + 1, dtype=torch.int64, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    max_w = _max_weight()
    args = (h, rows.peak_off.data_ptr(), S, rows.su.data_ptr(), rows.obs.data_ptr(), rows.meta.data_ptr(),
            rows.alive.data_ptr(), rows.rows.data_ptr())
    torch.cuda.synchronize(dev)
    eng.check(L.sst_dict_count_device(*args, float(max_w), float(tolerance), n_q.data_ptr(), off.data_ptr(),
                                      err.data_ptr()), "sst_dict_count_device")
    eng.synchronize()
    total = int(off[S].item())
    key = torch.empty(max(1, total), dtype=torch.int64, device=dev)
    thr = torch.empty(max(1, total), dtype=torch.float64, device=dev)
    n_ent = torch.zeros(max(1, S), dtype=torch.int32, device=dev)
    xp = None
    if max_len is not None:
        ok = budgets_pair_ok(dp_table, np.broadcast_to(np.asarray(max_len, dtype=np.int64), (S,)))
        if not ok.all():  # exact-mode spectra: their final-round queries answered by the exact masked explain
            xio = _ExactLists(dp_table, rows, ok, max_len, cap=total)
            xio.reset()
            xp = ctypes.byref(xio.io)
            eng.check(L.sst_dict_list_device(*args, float(max_w), float(tolerance), err.data_ptr(), xp),
                      "sst_dict_list_device")
            xio.answer(alpha_dev)
    eng.check(L.sst_dict_build_device(*args, alpha_dev.data_ptr(), float(max_w), float(tolerance),
                                      float(dp_table.precision), off.data_ptr(), key.data_ptr(), thr.data_ptr(),
                                      n_ent.data_ptr(), err.data_ptr(), xp), "sst_dict_build_device")
    eng.synchronize()
    _check_err(err)
    return DeviceDict(off, n_ent, key, thr)


def _lens_pass(dp_table, alpha_dev, mass, thr, spec, n, max_len):
    """The masked explain of windows [0, n) on their spectra's alphabets with
    their spectra's budgets (round(max_len * rate) per row,
    round(seq.modification_rate * max_len) modifications: the budgets the
    rebuilt table of skeleton_building.py:212 / prediction.py:207 carries),
    in one pass (sst_explain_alpha_lens_batch_device)."""
    import torch

    dt = dp_table.device_table
    dev = mass.device
    masses = dp_table.masses
    lens = np.unique(np.asarray(max_len, dtype=np.int64))
    caps = np.array([[round(int(L) * m.modification_rate) for m in masses] for L in lens], dtype=np.int64)
    mods_l = torch.as_tensor(np.array([round(dp_table.seq.modification_rate * int(L)) for L in lens], np.int64),
                             device=dev)
    ml_q = torch.as_tensor(np.asarray(max_len, dtype=np.int64), device=dev)[spec[:n].long()]
    qlen = torch.searchsorted(torch.as_tensor(lens, device=dev), ml_q).to(torch.int32).contiguous()
    mods = mods_l[qlen.long()].contiguous()
    res = dt.explain_alpha_lens_device(mass.data_ptr(), thr.data_ptr(), spec.data_ptr(), alpha_dev.data_ptr(),
                                       qlen.data_ptr(), caps, n, dp_table.tolerance, dp_table.precision,
                                       mods.data_ptr())
    res.keep_alive = (qlen, mods)  # read by the pass until it settles
    return res


def _masked_explain_refs(dp_table, alpha_dev, mass, thr, spec, n, max_len, dst, ptr, cnt, st):
    """Windows answered by the masked explain (_lens_pass); each window's
    candidate reference lands at dst[i] of (ptr, cnt, st).  Returns the
    results (their payload backs the references)."""
    if n == 0:
        return []
    res = _lens_pass(dp_table, alpha_dev, mass, thr, spec, n, max_len)
    eng = dp_table.device_table.engine
    eng.check(eng._lib.sst_result_refs_device(res.handle, dst.data_ptr(), ptr.data_ptr(), cnt.data_ptr(),
                                              st.data_ptr()), "sst_result_refs_device")
    return [res]


def merge_requery_round(dp_table, merged, n_merged, block, p_, n_, s_, n_sides):
    """Append one re-query round's answers to the merged per-side lists the
    walk reads as a single round (sst_requery_merge_device: per side the
    earlier rounds' entries, then this round's; sides in order).  merged:
    the previous view (block, ptr, n, st) or None; n_merged its entries;
    block[sid] = start << 32 | count: side sid's entries of this round in p_
    / n_ / s_.  Returns the new view (start << 32 | count per side, ptr, n,
    st) and its entry count -- known on the host, so no device read-back."""
    import torch

    dev = block.device
    n_new = n_merged + len(p_)
    m_block = torch.empty(max(1, n_sides), dtype=torch.int64, device=dev)
    m_ptr = torch.empty(max(1, n_new), dtype=torch.int64, device=dev)
    m_n = torch.empty(max(1, n_new), dtype=torch.int32, device=dev)
    m_st = torch.empty(max(1, n_new), dtype=torch.int8, device=dev)
    tot = torch.empty(max(1, n_sides), dtype=torch.int32, device=dev)
    off = torch.empty(n_sides + 1, dtype=torch.int64, device=dev)
    a = _native.RequeryMergeArgs()
    if merged is not None:
        a.o_block, a.o_ptr, a.o_n, a.o_st = (t.data_ptr() for t in merged)
    a.block, a.ptr, a.n, a.st = block.data_ptr(), p_.data_ptr(), n_.data_ptr(), s_.data_ptr()
    a.n_sides = n_sides
    a.m_block, a.m_ptr, a.m_n, a.m_st = m_block.data_ptr(), m_ptr.data_ptr(), m_n.data_ptr(), m_st.data_ptr()
    dt = dp_table.device_table
    dt.engine.check(dt.engine._lib.sst_requery_merge_device(dt.handle, ctypes.byref(a), tot.data_ptr(),
                                                            off.data_ptr()), "sst_requery_merge_device")
    return (m_block, m_ptr, m_n, m_st), n_new


@dataclass
class DeviceSkeleton:
    """_predict_skeleton of both sides of every spectrum (device arrays)."""
    max_len: np.ndarray   # [S]
    skel_off: np.ndarray  # [S + 1] exclusive prefix of 2 max_len (positions)
    skel: object          # torch int64 [2 total, 2]: spectrum g, side sd, position i at skel_off[g] + sd max_len + i
    min_end: object       # torch int32 [2, slots] (row slots; side 0 START, 1 END)
    max_end: object
    kept: object          # torch uint8 [2, slots]: rows the walk did not reject (alive rows of the side)
    status: np.ndarray    # [2 S] SST_WALK_* per side
    launches: int         # walk launches (re-query rounds + 1, and big-capacity reruns)
    requeries: int        # re-query windows the masked explain answered
    dict_entries: int
    results: list         # the masked explain results the references point into


@_one_stream
def skeleton_device(dp_table, rows: DeviceRows, alpha, max_len, bins=None, tolerance=None, caps=(64, 32),
                    big_caps=(8192, 8192), max_rounds=4096, name_hash=None):
    """Stage 4 on the device: SkeletonBuilder._predict_skeleton for the START
    and END rows of every spectrum (the rows the fixpoint kept, its final
    alphabets `alpha` [S, 2] u64), with filter_by_explanation's final dict.
    `bins`: stage 3's bins_device(..., max_len=max_len) result (computed here
    when None).  caps = (explanations per bin, candidates per query) of the
    lanes' scratch; sides that outgrow them are walked again with big_caps.
    max_rounds bounds the re-query rounds (each answers every suspended side's
    next re-query bin).  name_hash: hash() of each row's nucleoside name (the
    reference's set order, common.py:60-65); None = this interpreter's
    (name_hashes).  A sharded run passes rank 0's to every rank, so that
    every spectrum's walk follows one interpreter's order."""
    import torch

    tolerance = dp_table.tolerance if tolerance is None else tolerance
    S = len(rows.rows)
    dev = rows.su.device
    eng = dp_table.device_table.engine
    L = eng._lib
    h = dp_table.device_table.handle
    max_len = np.ascontiguousarray(np.broadcast_to(np.asarray(max_len, dtype=np.int64), (S,)))
    if bins is None:
        bins = bins_device(dp_table, rows, alpha, tolerance=tolerance, max_len=max_len)
    alpha_dev = bins.alpha_dev
    dct = final_dict_device(dp_table, rows, alpha_dev, tolerance, max_len=max_len)
    Q = int(bins.q_off[-1])
    s_ptr = torch.zeros(max(1, Q), dtype=torch.int64, device=dev)
    s_n = torch.zeros(max(1, Q), dtype=torch.int32, device=dev)
    s_st = torch.full((max(1, Q),), -10, dtype=torch.int8, device=dev)
    results = []
    if bins.deferred is not None and bins.deferred["queries"]:
        d = bins.deferred
        dst = d["dst"]
        for s0, res in d["results"]:
            eng.check(L.sst_result_refs_device(res.handle, dst.data_ptr() + 8 * s0, s_ptr.data_ptr(), s_n.data_ptr(),
                                               s_st.data_ptr()), "sst_result_refs_device")
            results.append(res)
    elif bins.deferred is None:
        raise ValueError("skeleton_device: stage 3 must answer its off-pair-class queries (bins_device(max_len=...))")
    ml_t = torch.as_tensor(max_len.astype(np.int32), device=dev)
    pair_ok = torch.as_tensor(budgets_pair_ok(dp_table, max_len).astype(np.uint8), device=dev)
    skel_off = np.concatenate([[0], np.cumsum(2 * max_len)]).astype(np.int64)
    skel = torch.zeros((max(1, int(skel_off[-1])), 2), dtype=torch.int64, device=dev)
    skel_off_t = torch.as_tensor(skel_off, device=dev)
    slots = int(rows.su.numel())
    min_end = torch.zeros((2, slots), dtype=torch.int32, device=dev)
    max_end = torch.full((2, slots), -1, dtype=torch.int32, device=dev)
    kept = torch.zeros((2, slots), dtype=torch.uint8, device=dev)
    side_rows = torch.zeros(2 * slots, dtype=torch.int16, device=dev)
    status = torch.zeros(max(1, 2 * S), dtype=torch.uint8, device=dev)
    ctl = torch.zeros(3, dtype=torch.int32, device=dev)  # suspended, big, request count
    # the names' str hashes fix the explanation sets' iteration order: this
    # interpreter's, or the caller's (a sharded run uses rank 0's on every rank)
    nh = torch.as_tensor(name_hashes(dp_table) if name_hash is None else np.asarray(name_hash, np.int64), device=dev)
    ml_max = int(max_len.max()) if S else 1
    len_cap = ml_max + 2
    if len_cap > 255:
        raise NotImplementedError("skeleton walk: max_len above 253")
    pos_cap = _native.pyset_table_size(ml_max + 1)
    req_cap = max(1 << 16, Q)
    req_mass = torch.empty(req_cap, dtype=torch.float64, device=dev)
    req_thr = torch.empty_like(req_mass)
    req_spec = torch.empty(req_cap, dtype=torch.int32, device=dev)
    a = _native.WalkArgs()
    a.peak_off, a.cnt, a.r_su, a.r_ob = (rows.peak_off.data_ptr(), rows.rows.data_ptr(), rows.su.data_ptr(),
                                         rows.obs.data_ptr())
    a.r_meta, a.alive, a.alpha, a.max_len = rows.meta.data_ptr(), rows.alive.data_ptr(), alpha_dev.data_ptr(), \
        ml_t.data_ptr()
    a.pair_ok, a.n_spec, a.slots = pair_ok.data_ptr(), S, slots
    a.tol, a.prec, a.rprec = float(tolerance), float(dp_table.precision), 1.0 / float(dp_table.precision)
    a.d_off, a.d_n, a.d_key, a.d_thr = dct.off.data_ptr(), dct.n.data_ptr(), dct.key.data_ptr(), dct.thr.data_ptr()
    a.q_off, a.q0 = bins.q_off_dev.data_ptr(), bins.q0_dev.data_ptr()
    a.s_ptr, a.s_n, a.s_st = s_ptr.data_ptr(), s_n.data_ptr(), s_st.data_ptr()
    a.req_mass, a.req_thr, a.req_spec = req_mass.data_ptr(), req_thr.data_ptr(), req_spec.data_ptr()
    a.req_count, a.req_cap = ctl.data_ptr() + 8, req_cap
    a.name_hash = nh.data_ptr()
    a.side_rows, a.skel_off, a.skel = side_rows.data_ptr(), skel_off_t.data_ptr(), skel.data_ptr()
    a.min_end, a.max_end, a.kept = min_end.data_ptr(), max_end.data_ptr(), kept.data_ptr()
    a.side_status, a.n_suspended, a.n_big = status.data_ptr(), ctl.data_ptr(), ctl.data_ptr() + 4
    a.pos_cap, a.len_cap = pos_cap, len_cap
    # every re-query answer so far, merged per side in round order (block =
    # start << 32 | count per side, then ptr / n / st): the lanes see one
    # round, so the number of re-query rounds is not bounded by the ABI's
    # SST_WALK_MAX_ROUNDS (exact-mode spectra re-query every bin whose
    # predecessor had no explanations through the host)
    merged, n_merged = None, 0
    keep_alive = []
    n_rounds = 0
    run = np.arange(2 * S, dtype=np.int32)
    big = np.zeros(0, np.int32)
    launches = 0
    n_req_total = 0
    # scratch slots: every side's at the small caps (slot = side id), the
    # sides that outgrew them at the big caps (slots in the order they did);
    # a suspended side's state stays in its slot and the relaunch resumes it
    t_small, t_big = _native.pyset_table_size(caps[1]), _native.pyset_table_size(big_caps[1])
    stride_small = _native.walk_scratch_bytes(pos_cap, len_cap, caps[0], caps[1], t_small)
    stride_big = _native.walk_scratch_bytes(pos_cap, len_cap, big_caps[0], big_caps[1], t_big)
    scratch_small = torch.empty(max(1, 2 * S) * stride_small, dtype=torch.uint8, device=dev)
    scratch_big = torch.zeros(0, dtype=torch.uint8, device=dev)  # zeroed: a new slot holds no state
    big_slot = {}
    torch.cuda.synchronize(dev)
    while len(run) or len(big):
        req_block = torch.zeros(max(1, 2 * S), dtype=torch.int64, device=dev)
        a.req_block = req_block.data_ptr()
        a.n_rounds = 0 if merged is None else 1
        if merged is not None:
            a.rq_block[0], a.rq_ptr[0], a.rq_n[0], a.rq_st[0] = (t.data_ptr() for t in merged)
        ctl.zero_()
        for b in big.tolist():
            big_slot.setdefault(b, len(big_slot))
        need = len(big_slot) * stride_big
        if need > scratch_big.numel():
            grown = torch.zeros(max(need, 2 * scratch_big.numel()), dtype=torch.uint8, device=dev)
            grown[:scratch_big.numel()].copy_(scratch_big)
            scratch_big = grown
        for sides, (e_cap, c_cap), t_cap, stride, scr in ((run, caps, t_small, stride_small, scratch_small),
                                                          (big, big_caps, t_big, stride_big, scratch_big)):
            if not len(sides):
                continue
            sides_t = torch.as_tensor(sides, device=dev)
            slots_t = sides_t if scr is scratch_small else torch.as_tensor(
                np.array([big_slot[b] for b in sides.tolist()], np.int32), device=dev)
            a.sides, a.n_sides = sides_t.data_ptr(), len(sides)
            a.slot, a.resume = slots_t.data_ptr(), int(launches > 0)
            a.scratch, a.scratch_stride = scr.data_ptr(), stride
            a.expl_cap, a.cand_cap, a.tset_cap = e_cap, c_cap, t_cap
            eng.check(L.sst_skel_walk_device(h, ctypes.byref(a)), "sst_skel_walk_device")
            keep_alive.append((sides_t, slots_t))
            launches += 1
        eng.synchronize()
        keep_alive.clear()
        n_susp, n_big, n_req = (int(x) for x in ctl.cpu().tolist())
        if _PROGRESS:
            print(f"[skeleton walk] launch {launches}: {n_susp} suspended, {n_big} big, {n_req} re-queries",
                  file=sys.stderr, flush=True)
        st_h = status.cpu().numpy()
        was_big = np.zeros(2 * S, bool)
        was_big[big] = True
        new_big = np.flatnonzero((st_h == _native.WALK_BIG) & ~was_big).astype(np.int32)
        st_h[big[st_h[big] == _native.WALK_BIG]] = _native.WALK_LIMIT  # outgrew the big capacities too
        if len(big):
            status[torch.as_tensor(big.astype(np.int64), device=dev)] = torch.as_tensor(st_h[big], device=dev)
        susp = np.flatnonzero(st_h == _native.WALK_SUSPENDED).astype(np.int32)
        run = susp[~was_big[susp]]
        big = np.concatenate([susp[was_big[susp]], new_big]).astype(np.int32)
        if n_req:
            if n_rounds >= max_rounds:
                break  # the sides still suspended keep SST_WALK_SUSPENDED
            if n_req > req_cap:
                raise _native.EngineError("skeleton walk: re-query list overflow")
            p_ = torch.zeros(n_req, dtype=torch.int64, device=dev)
            n_ = torch.zeros(n_req, dtype=torch.int32, device=dev)
            s_ = torch.full((n_req,), -10, dtype=torch.int8, device=dev)
            dst = torch.arange(n_req, dtype=torch.int64, device=dev)
            res = _masked_explain_refs(dp_table, alpha_dev, req_mass, req_thr, req_spec, n_req, max_len, dst, p_, n_,
                                       s_)
            results.extend(res)
            merged, n_merged = merge_requery_round(dp_table, merged, n_merged, req_block[:2 * S], p_, n_, s_, 2 * S)
            n_rounds += 1
            n_req_total += n_req
    return DeviceSkeleton(max_len, skel_off, skel, min_end, max_end, kept, status.cpu().numpy()[:2 * S], launches,
                          n_req_total, int(dct.n.sum().item()), results)


def skeleton_frames(dp_table, rows: DeviceRows, sk: DeviceSkeleton, g):
    """Spectrum g's walk as the reference's values: per side (START, END) the
    skeleton (sorted names per position), the kept rows' `index` (their place
    among the spectrum's rows: Predictor.predict's SU-order index), min_end
    and max_end -- the fields tests/golden/callers.json.gz records."""
    from .mass_explanation import MASS_NAMES

    ml = int(sk.max_len[g])
    off = int(rows.peak_off[g].item()) * 4
    n = int(rows.rows[g].item())
    alive = rows.alive[off:off + n].cpu().numpy().astype(bool)
    meta = rows.meta[off:off + n].cpu().numpy().astype(np.int64)
    out = {}
    skel = sk.skel[int(sk.skel_off[g]):int(sk.skel_off[g]) + 2 * ml].cpu().numpy().view(np.uint64)
    names = [None] + [MASS_NAMES[m.mass][0] for m in dp_table.masses[1:]]
    for sd, side in enumerate(("START", "END")):
        pos = []
        for i in range(ml):
            m0, m1 = int(skel[sd * ml + i, 0]), int(skel[sd * ml + i, 1])
            rows_i = [r for r in range(len(names)) if (m0 >> r) & 1 or (r >= 64 and (m1 >> (r - 64)) & 1)]
            pos.append(sorted(names[r] for r in rows_i))
        on = alive & (((meta >> (2 + sd)) & 1) == 1)
        kp = sk.kept[sd, off:off + n].cpu().numpy().astype(bool) & on
        idx = np.flatnonzero(kp)
        out[side] = {"skeleton": pos, "kept_index": idx.tolist(),
                     "min_end": sk.min_end[sd, off + idx].cpu().numpy().tolist() if len(idx) else [],
                     "max_end": sk.max_end[sd, off + idx].cpu().numpy().tolist() if len(idx) else []}
    return out


# ---------------------------------------------------------------------------
# Stage 5: select_sequence_length_with_jaccard on the device (its two length
# bounds on each spectrum's skeleton alphabet) and combine_skeleton_sequences
# (skeleton_building.py:315-370, 494-516; mass_table.py:343-487)
# ---------------------------------------------------------------------------
@dataclass
class DeviceLength:
    alpha: np.ndarray     # [S, 2] u64 the skeleton's alphabets
    lower: np.ndarray     # [S] compute_sequence_length_bound(dir="lower")
    upper: np.ndarray     # [S] (dir="upper")
    lb_status: np.ndarray  # [S] 0 ok, else the bound raised (SST_OUT_OF_TABLE / ABORTED / -5)
    seq_len: np.ndarray   # [S] the chosen length
    status: np.ndarray    # [S] SST_JAC_*
    comb_off: np.ndarray  # [S + 1]
    comb: object          # torch int64 [total, 2] the combined skeleton (masks)
    reach_batches: int
    distinct_alphabets: int = 0  # skeleton alphabets (each one's row bitsets built once)
    replay_nodes: object = None  # [S] frontier: memo entries of the bounds' DFS; replay: phase-1 nodes over attempts
    engine: str = "frontier"
    frontier: dict = None  # sst_lbf_stats summed over the batches (frontier engine)


@_one_stream
def length_bounds_alpha_device(dp_table, alpha_sk, su, ob, max_len, caps_len, a0_len, sel=None, engine="frontier",
                               reach_budget_bytes=64 << 30, share_alphabets=True, length_chunk=1 << 30,
                               soft_nodes=1 << 20, heavy_memo=1 << 22, frontier_workspace=0, keep_buffers=False):
    """compute_sequence_length_bound(dir="lower") and (dir="upper")
    (mass_table.py:343-487) for spectra on reduced alphabets (alpha_sk [S, 2]
    u64 row masks; su / ob the SequenceInformation masses; max_len [S]), with
    the budgets per max_len: caps_len[L, r] = round(L * rate_r) (row stride
    MAX_ROWS) and a0_len[L] = round(modification_rate * L).  Only spectra
    `sel` are computed (the others keep lb_status LB_NOT_RUN).  engine:
    "frontier" (the first-visit frontier) or "replay" (the round-4
    per-spectrum DFS replay).  Returns (lower, upper, lb_status, nodes, stats)."""
    import torch

    dt = dp_table.device_table
    eng = dt.engine
    L = eng._lib
    h = dt.handle
    S = len(alpha_sk)
    dev = torch.device("cuda", eng.device) if hasattr(eng, "device") else torch.device("cuda")
    su = np.asarray(su, dtype=np.float64)
    ob = np.asarray(ob, dtype=np.float64)
    ml = np.asarray(max_len, dtype=np.int64)
    prec, tol = dp_table.precision, dp_table.tolerance
    hi = np.rint(su / prec) + np.ceil(tol * ob / prec)  # the window's top (mass_table.py:354-359)
    words = (np.maximum(hi, 0).astype(np.int64) >> 5) + 2
    from .pipeline import mask_rows

    n_rows = len(dp_table.masses)
    # spectra with one skeleton alphabet share its rows' bitsets (built up to
    # the heaviest of their windows): few distinct alphabets among many spectra
    sel = np.arange(S) if sel is None else np.asarray(sel, dtype=np.int64)
    lower = np.zeros(S, np.int64)
    upper = np.zeros(S, np.int64)
    lb_st = np.full(S, LB_NOT_RUN, np.int8)
    lb_st[sel] = 0
    nodes = np.zeros(S, np.int64)
    masses = dp_table.masses
    is_mod = [m.is_modification for m in masses]
    caps_len = np.ascontiguousarray(caps_len, dtype=np.int32)
    a0_len = [int(x) for x in a0_len]
    ml_hi = int(ml[sel].max()) if len(sel) else 1
    if caps_len.shape[0] <= ml_hi or len(a0_len) <= ml_hi or caps_len.shape[1] != _native.MAX_ROWS:
        raise ValueError("length bounds: caps_len / a0_len must cover every max_len")
    # value ranges: the replay's int8 value slots hold max_len + 1 for max_len <= 120 (sst_api.cpp), the
    # frontier's u8 lower values max_len + 1 <= 254
    if ml_hi > (120 if engine == "replay" else 253):
        raise NotImplementedError(f"length bounds ({engine}): max_len {ml_hi} above the engine's limit")
    caps_t = torch.as_tensor(caps_len, device=dev)
    a0_t = torch.as_tensor(np.asarray(a0_len, np.int32), device=dev)
    dt.set_budgets(is_mod, [int(c) for c in caps_len[ml_hi, :len(masses)]])  # the rows' modification flags
    stats = {"batches": 0, "distinct": 0, "frontier": {}}

    def bounds_pass(sel, soft_nodes, memo_first):
        """Both bounds of spectra `sel`, in batches whose row bitsets fit
        the budget; returns the spectra left SST_LB_HEAVY (over soft_nodes)."""
        # spectra with one skeleton alphabet share its rows' bitsets (built up
        # to the heaviest of their windows)
        if share_alphabets:
            uniq, inv = np.unique(alpha_sk[sel], axis=0, return_inverse=True)
            inv = inv.reshape(-1)
        else:
            uniq, inv = alpha_sk[sel], np.arange(len(sel))
        U = len(uniq)
        stats["distinct"] = max(stats["distinct"], U)
        words_u = np.zeros(U, np.int64)
        np.maximum.at(words_u, inv, words[sel])
        K_u = mask_rows(uniq, n_rows)[:, 1:].sum(axis=1).astype(np.int64)
        need_u = 4 * K_u * words_u
        by_u = np.argsort(inv, kind="stable")  # spectra grouped by alphabet
        u_first = np.concatenate([[0], np.cumsum(np.bincount(inv, minlength=U))])
        u0 = 0
        while u0 < U:
            u1, tot = u0, 0
            while u1 < U and (u1 == u0 or tot + need_u[u1] <= reach_budget_bytes):
                tot += int(need_u[u1])
                u1 += 1
            nu = u1 - u0
            off_u = np.concatenate([[0], np.cumsum(need_u[u0:u1] // 4)[:-1]]).astype(np.int64)
            bits = torch.empty(max(1, int(tot // 4)), dtype=torch.int32, device=dev)
            # (every device array stays referenced until the batch is done: a
            # temporary's block can be handed to the next allocation at once)
            alu_t = torch.as_tensor(uniq[u0:u1].view(np.int64), device=dev).contiguous()
            wu_t = torch.as_tensor(words_u[u0:u1], device=dev)
            ou_t = torch.as_tensor(off_u, device=dev)
            eng.check(L.sst_reach_rows_device(h, alu_t.data_ptr(), wu_t.data_ptr(), ou_t.data_ptr(), nu,
                                              bits.data_ptr()), "sst_reach_rows_device")
            lu_src = by_u[u_first[u0]:u_first[u1]]
            members = sel[lu_src]  # this batch's spectra
            n = len(members)
            if _PROGRESS:
                eng.synchronize()
                print(f"[length] batch {stats['batches']}: {n} spectra, {nu} alphabets, {tot / 2**20:.1f} MiB of row "
                      f"bitsets, soft node budget {soft_nodes}", file=sys.stderr, flush=True)
            lu = inv[lu_src] - u0  # their alphabets within the batch
            al_t = torch.as_tensor(uniq[u0:u1][lu].view(np.int64), device=dev).contiguous()
            w_t = torch.as_tensor(words_u[u0:u1][lu], device=dev)
            o_t = torch.as_tensor(off_u[lu], device=dev)
            order = np.argsort(ml[members], kind="stable")
            su_t = torch.as_tensor(su[members][order], device=dev)
            ob_t = torch.as_tensor(ob[members][order], device=dev)
            sp_t = torch.as_tensor(order.astype(np.int32), device=dev)
            ql_t = torch.as_tensor(ml[members][order].astype(np.int32), device=dev)
            lo_t = torch.zeros(n, dtype=torch.int64, device=dev)
            up_t = torch.zeros(n, dtype=torch.int64, device=dev)
            st_t = torch.zeros(n, dtype=torch.int8, device=dev)
            nd_t = torch.zeros(n, dtype=torch.int64, device=dev)
            # every max_len in one launch (per-query budgets); a heartbeat line
            # every 30 s while a long replay runs (the call releases the GIL)
            beat = _Heartbeat("[length] replay running", 30.0) if _PROGRESS else None
            for s0 in range(0, n, length_chunk):
                s1 = min(n, s0 + length_chunk)
                eng.check(L.sst_length_bounds_reach_device(
                    h, su_t.data_ptr() + 8 * s0, ob_t.data_ptr() + 8 * s0, sp_t.data_ptr() + 4 * s0, al_t.data_ptr(),
                    bits.data_ptr(), o_t.data_ptr(), w_t.data_ptr(), s1 - s0, float(tol), float(prec), ml_hi,
                    a0_len[ml_hi], lo_t.data_ptr() + 8 * s0, up_t.data_ptr() + 8 * s0, st_t.data_ptr() + s0,
                    ql_t.data_ptr() + 4 * s0, caps_t.data_ptr(), a0_t.data_ptr(), nd_t.data_ptr() + 8 * s0,
                    int(soft_nodes), int(memo_first), int(K_u.max() <= 64)), "sst_length_bounds_reach_device")
            if beat is not None:
                beat.stop()
            idx = members[order]
            lower[idx] = lo_t.cpu().numpy()
            upper[idx] = up_t.cpu().numpy()
            lb_st[idx] = st_t.cpu().numpy()
            nodes[idx] += nd_t.cpu().numpy()
            del bits
            stats["batches"] += 1
            u0 = u1
        return sel[lb_st[sel] == _native.LB_HEAVY]

    def frontier_pass(sel):
        """Both bounds of spectra `sel` by the first-visit frontier
        (sst_length_bounds_frontier_device): per batch of alphabets, the row
        bitsets, then one byte per mass (the lowest kept rank reaching it),
        then every spectrum of the batch in one call."""
        if share_alphabets:
            uniq, inv = np.unique(alpha_sk[sel], axis=0, return_inverse=True)
            inv = inv.reshape(-1)
        else:
            uniq, inv = alpha_sk[sel], np.arange(len(sel))
        U = len(uniq)
        stats["distinct"] = max(stats["distinct"], U)
        words_u = np.zeros(U, np.int64)
        np.maximum.at(words_u, inv, words[sel])
        K_u = mask_rows(uniq, n_rows)[:, 1:].sum(axis=1).astype(np.int64)
        need_u = 4 * K_u * words_u + 32 * words_u
        by_u = np.argsort(inv, kind="stable")
        u_first = np.concatenate([[0], np.cumsum(np.bincount(inv, minlength=U))])
        batches, u0 = [], 0
        while u0 < U:
            u1, tot = u0, 0
            while u1 < U and (u1 == u0 or tot + need_u[u1] <= reach_budget_bytes):
                tot += int(need_u[u1])
                u1 += 1
            batches.append((u0, u1))
            u0 = u1
        # one buffer for every batch's row bitsets and lowest-rank bytes, sized
        # to the largest (a fresh allocation of tens of GB per batch, and its
        # release, idled the GPU for 0.1 s each), kept across passes unless
        # keep_buffers is False (_length_buffer)
        kw_b = [int((K_u[b0:b1] * words_u[b0:b1]).sum()) for b0, b1 in batches]
        lw_b = [int(32 * words_u[b0:b1].sum()) for b0, b1 in batches]
        lr_at = [(4 * max(1, kw) + 255) // 256 * 256 for kw in kw_b]  # the lowest-rank bytes after the bitsets
        buf = _length_buffer(dev, max([256] + [a_ + max(1, lw) for a_, lw in zip(lr_at, lw_b)]))
        bits = lr = None
        for bi, (u0, u1) in enumerate(batches):
            nu = u1 - u0
            wb = words_u[u0:u1]
            off_u = np.concatenate([[0], np.cumsum(K_u[u0:u1] * wb)[:-1]]).astype(np.int64)
            lr_off = np.concatenate([[0], np.cumsum(32 * wb)[:-1]]).astype(np.int64)
            bits = buf[:4 * max(1, kw_b[bi])].view(torch.int32)
            lr = buf[lr_at[bi]:lr_at[bi] + max(1, lw_b[bi])]
            alu_t = torch.as_tensor(uniq[u0:u1].view(np.int64), device=dev).contiguous()
            wu_t = torch.as_tensor(wb, device=dev)
            ou_t = torch.as_tensor(off_u, device=dev)
            lo_u_t = torch.as_tensor(lr_off, device=dev)
            t_batch = time.perf_counter()
            eng.check(L.sst_reach_rows_device(h, alu_t.data_ptr(), wu_t.data_ptr(), ou_t.data_ptr(), nu,
                                              bits.data_ptr()), "sst_reach_rows_device")
            eng.check(L.sst_reach_lowest_device(h, alu_t.data_ptr(), wu_t.data_ptr(), ou_t.data_ptr(), nu,
                                                bits.data_ptr(), lo_u_t.data_ptr(), lr.data_ptr()),
                      "sst_reach_lowest_device")
            if _PROGRESS:
                eng.synchronize()
            t_reach = time.perf_counter() - t_batch
            lu_src = by_u[u_first[u0]:u_first[u1]]
            members = sel[lu_src]
            n = len(members)
            lu = (inv[lu_src] - u0).astype(np.int32)
            su_t = torch.as_tensor(su[members], device=dev)
            ob_t = torch.as_tensor(ob[members], device=dev)
            sp_t = torch.as_tensor(lu, device=dev)
            ql_t = torch.as_tensor(ml[members].astype(np.int32), device=dev)
            lo_t = torch.zeros(n, dtype=torch.int64, device=dev)
            up_t = torch.zeros(n, dtype=torch.int64, device=dev)
            st_t = torch.zeros(n, dtype=torch.int8, device=dev)
            nd_t = torch.zeros(n, dtype=torch.int64, device=dev)
            fs = _native.LbfStats()
            beat = _Heartbeat("[length] frontier running", 30.0) if _PROGRESS else None
            eng.check(L.sst_length_bounds_frontier_device(
                h, su_t.data_ptr(), ob_t.data_ptr(), sp_t.data_ptr(), alu_t.data_ptr(), lr.data_ptr(),
                lo_u_t.data_ptr(), n, float(tol), float(prec), ml_hi, a0_len[ml_hi], lo_t.data_ptr(), up_t.data_ptr(),
                st_t.data_ptr(), ql_t.data_ptr(), caps_t.data_ptr(), a0_t.data_ptr(), nd_t.data_ptr(),
                int(frontier_workspace), ctypes.byref(fs)), "sst_length_bounds_frontier_device")
            if beat is not None:
                beat.stop()
            lower[members] = lo_t.cpu().numpy()
            upper[members] = up_t.cpu().numpy()
            lb_st[members] = st_t.cpu().numpy()
            nodes[members] += nd_t.cpu().numpy()
            fd = fs.as_dict()
            for k_, v_ in fd.items():
                if k_ in ("bands", "key_words", "max_band_groups", "max_band_nodes", "table_slots", "node_cap"):
                    stats["frontier"][k_] = max(stats["frontier"].get(k_, 0), v_)
                elif k_ == "overflow_bits":
                    stats["frontier"][k_] = stats["frontier"].get(k_, 0) | v_
                else:
                    stats["frontier"][k_] = stats["frontier"].get(k_, 0) + v_
            if _PROGRESS:
                print(f"[length] frontier batch {stats['batches']}: {n} spectra, {nu} alphabets, reach "
                      f"{t_reach:.3f}s, batch {time.perf_counter() - t_batch:.3f}s: {fd}", file=sys.stderr, flush=True)
            stats["batches"] += 1
        buf = bits = lr = None  # (views of the cached buffer)
        if not keep_buffers:
            release_length_buffer(dev)

    if engine == "frontier":
        frontier_pass(sel)
        heavy = []
    elif engine == "replay":
        # light spectra first, under a soft node budget, so that no batch waits
        # for its few heavy spectra; then the heavy ones together, with a larger
        # first memo
        heavy = bounds_pass(sel, soft_nodes, 0) if soft_nodes else sel
    else:
        raise ValueError(f"length_device: engine {engine!r}")
    if len(heavy):
        if _PROGRESS:
            print(f"[length] {len(heavy)} spectra over {soft_nodes} nodes: replayed together", file=sys.stderr,
                  flush=True)
        bounds_pass(heavy, 0, heavy_memo if soft_nodes else 0)
    return lower, upper, lb_st, nodes, stats


@_one_stream
def length_device(dp_table, sk: DeviceSkeleton, alpha_dev, su_seq, obs_seq, reach_budget_bytes=64 << 30,
                  share_alphabets=True, length_chunk=1 << 30, spectra=None, soft_nodes=1 << 20,
                  heavy_memo=1 << 22, engine="frontier", frontier_workspace=0, trim=True):
    """Stage 5: each spectrum's skeleton alphabet (the canonical rows and the
    modifications its START / END skeletons name), both length bounds on it,
    then the Jaccard selection and the combined skeleton (k_jaccard).
    engine="frontier" (default): sst_reach_rows_device + sst_reach_lowest_device
    + sst_length_bounds_frontier_device -- the reduced table's pairs from its
    rows' reachability, every node's first visit computed band by band over
    descending masses, no DFS replay; batches of alphabets whose
    bitsets fit `reach_budget_bytes`, every max_len in one call
    (frontier_workspace: the call's device workspace, 0 = its default).
    engine="replay": sst_length_bounds_reach_device, one replay of the
    reference's DFS per spectrum (the round-4 engine, kept for comparison).
    spectra: the bounds for these spectra only (indices; the others get
    lb_status LB_NOT_RUN and Jaccard status SST_JAC_BOUNDS) -- a bounded
    sample where the reference's DFS is too large to replay for all.
    trim: release the frontier's cached workspace (sst_ctx_trim) and the
    reach buffer once the bounds are done, so later stages and other
    allocators get that HBM (trim=False keeps both for the next call, as a
    serving process would; reserve_length_buffer sizes the reach buffer
    ahead)."""
    import torch

    dt = dp_table.device_table
    eng = dt.engine
    L = eng._lib
    h = dt.handle
    S = len(sk.max_len)
    dev = sk.skel.device
    ml = sk.max_len.astype(np.int64)
    ml_t = torch.as_tensor(ml.astype(np.int32), device=dev)
    skel_off_t = torch.as_tensor(sk.skel_off, device=dev)
    a_sk = torch.empty((max(1, S), 2), dtype=torch.int64, device=dev)
    eng.check(L.sst_skeleton_alpha_device(h, S, ml_t.data_ptr(), skel_off_t.data_ptr(), sk.skel.data_ptr(),
                                          alpha_dev.data_ptr(), a_sk.data_ptr()), "sst_skeleton_alpha_device")
    alpha_sk = a_sk.cpu().numpy().view(np.uint64)[:S].copy()
    su = np.asarray(su_seq, dtype=np.float64)
    ob = np.asarray(obs_seq, dtype=np.float64)
    prec = dp_table.precision
    sel = np.arange(S) if spectra is None else np.unique(np.asarray(spectra, dtype=np.int64))
    masses = dp_table.masses
    # budgets by max_len (mass_explanation.py:158-172 as set_budgets): caps
    # round(L * rate) per row, max_modifications round(modification_rate * L)
    ml_hi = int(ml[sel].max()) if len(sel) else 1
    caps_len = np.zeros((ml_hi + 1, _native.MAX_ROWS), np.int32)
    for Lm in range(ml_hi + 1):
        caps_len[Lm, :len(masses)] = [min(round(Lm * m.modification_rate), 1 << 30) for m in masses]
    a0_len = [min(round(dp_table.seq.modification_rate * Lm), 1 << 30) for Lm in range(ml_hi + 1)]
    lower, upper, lb_st, nodes, stats = length_bounds_alpha_device(
        dp_table, alpha_sk, su, ob, ml, caps_len, a0_len, sel=sel, engine=engine,
        reach_budget_bytes=reach_budget_bytes, share_alphabets=share_alphabets, length_chunk=length_chunk,
        soft_nodes=soft_nodes, heavy_memo=heavy_memo, frontier_workspace=frontier_workspace, keep_buffers=not trim)
    if trim:
        eng.trim()
    n_batches, U = stats["batches"], stats["distinct"]
    # Jaccard + combine
    comb_off = np.concatenate([[0], np.cumsum(ml)]).astype(np.int64)
    comb = torch.zeros((max(1, int(comb_off[-1])), 2), dtype=torch.int64, device=dev)
    lo_d = torch.as_tensor(lower, device=dev)
    up_d = torch.as_tensor(upper, device=dev)
    st_d = torch.as_tensor(lb_st, device=dev)
    su_d = torch.as_tensor(su, device=dev)
    rm = torch.as_tensor(np.array([m.mass * prec for m in masses], dtype=np.float64), device=dev)
    co_d = torch.as_tensor(comb_off, device=dev)
    seq_len = torch.zeros(max(1, S), dtype=torch.int32, device=dev)
    jst = torch.zeros(max(1, S), dtype=torch.int8, device=dev)
    from .fragment_classification import MAX_VARIANCE

    ja = _native.JaccardArgs(S, ml_t.data_ptr(), skel_off_t.data_ptr(), sk.skel.data_ptr(), lo_d.data_ptr(),
                             up_d.data_ptr(), st_d.data_ptr(), su_d.data_ptr(), rm.data_ptr(), co_d.data_ptr(),
                             comb.data_ptr(), seq_len.data_ptr(), jst.data_ptr(), float(MAX_VARIANCE))
    eng.check(L.sst_jaccard_device(h, ctypes.byref(ja)), "sst_jaccard_device")
    eng.synchronize()
    return DeviceLength(alpha_sk, lower, upper, lb_st, seq_len.cpu().numpy()[:S], jst.cpu().numpy()[:S], comb_off,
                        comb, n_batches, U, nodes, engine, stats["frontier"])


# ---------------------------------------------------------------------------
# After the skeleton: build_skeleton's fragments and the skeleton-based
# alphabet reduction (prediction.py:88-103, skeleton_building.py:67-109)
# ---------------------------------------------------------------------------
@dataclass
class DevicePost:
    alpha: np.ndarray   # [S, 2] u64 the alphabet after _reduce_alphabet(skeleton nucleotides)
    active: np.ndarray  # [S] 1: the spectrum reached the reduction (its Jaccard length stands)
    alive: object       # torch uint8 row slots: the fragments after the reduction's is_valid filter
    alive_skeleton: object  # torch uint8 row slots: build_skeleton's fragments (before the filter)
    min_end: object     # torch int32 row slots (build_skeleton's, clamped to [0, len))
    max_end: object
    rows_before: int    # fragments build_skeleton returned (all spectra)
    rows_after: int     # after the is_valid filter


@_one_stream
def post_skeleton_device(dp_table, rows: DeviceRows, sk: DeviceSkeleton, ln: DeviceLength, tolerance=None):
    """Predictor.predict after build_skeleton (prediction.py:88-103), every
    spectrum at once: build_skeleton's fragments -- the START walk's kept
    rows, the END walk's kept rows START did not keep, the internal rows no
    kept terminal row shares a peak with, min_end / max_end as
    skeleton_building.py:67-109 sets them (sst_post_skeleton_device) -- then
    _reduce_alphabet on the combined skeleton's nucleotides: the alphabet
    without the modifications the skeleton does not name, and is_valid_mass of
    every remaining fragment on it (sst_valid_rows_alpha_device, :204-227)."""
    import torch

    dt = dp_table.device_table
    eng = dt.engine
    L = eng._lib
    h = dt.handle
    S = len(sk.max_len)
    dev = sk.skel.device
    tol = dp_table.tolerance if tolerance is None else tolerance
    slots = int(rows.alive.numel())
    i32 = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.int32), device=dev)  # noqa: E731
    seq_len = i32(ln.seq_len)
    # build_skeleton first runs select_sequence_length_with_lp (skeleton_building.py:
    # 45-57, 198-251): without a solver it only combines the skeletons at every
    # candidate length in [lower, upper], which raises IndexError past max_len
    # (:494-512) -- build_skeleton raises and predict returns its default
    jac_post = np.array(ln.status, dtype=np.int8, copy=True)
    lp_raises = (ln.lb_status == 0) & (ln.lower <= ln.upper) & (ln.upper > np.asarray(sk.max_len, np.int64))
    jac_post[lp_raises & (jac_post == _native.JAC_OK)] = _native.JAC_INDEX
    jst = torch.as_tensor(jac_post, device=dev)
    comb_off = torch.as_tensor(np.ascontiguousarray(ln.comb_off[:-1] if len(ln.comb_off) > S else ln.comb_off,
                                                    dtype=np.int64), device=dev)
    alpha = torch.as_tensor(np.ascontiguousarray(ln.alpha).view(np.int64), device=dev)
    alpha_out = torch.empty_like(alpha)
    active = torch.zeros(max(1, S), dtype=torch.uint8, device=dev)
    alive_out = torch.zeros_like(rows.alive)
    min_out = torch.zeros(slots, dtype=torch.int32, device=dev)
    max_out = torch.zeros(slots, dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    a = _native.PostArgs(S, rows.peak_off.data_ptr(), rows.rows.data_ptr(), rows.meta.data_ptr(),
                         rows.alive.data_ptr(), sk.kept.data_ptr(), sk.min_end.data_ptr(), sk.max_end.data_ptr(), slots,
                         seq_len.data_ptr(), jst.data_ptr(), comb_off.data_ptr(), ln.comb.data_ptr(), alpha.data_ptr(),
                         alpha_out.data_ptr(), active.data_ptr(), alive_out.data_ptr(), min_out.data_ptr(),
                         max_out.data_ptr(), err.data_ptr())
    eng.check(L.sst_post_skeleton_device(h, ctypes.byref(a)), "sst_post_skeleton_device")
    alive_skel = alive_out.clone()
    before = int(alive_out.sum().item())
    err2 = torch.zeros(1, dtype=torch.int32, device=dev)
    eng.check(L.sst_valid_rows_alpha_device(h, rows.peak_off.data_ptr(), S, rows.su.data_ptr(), rows.obs.data_ptr(),
                                            rows.rows.data_ptr(), alpha_out.data_ptr(), active.data_ptr(),
                                            alive_out.data_ptr(), float(tol), float(dp_table.precision),
                                            err2.data_ptr()), "sst_valid_rows_alpha_device")
    eng.synchronize()
    if int(err.item()):
        raise _native.EngineError(f"post-skeleton stage: a spectrum of more than {MAX_PEAKS} peaks")
    _check_err(err2)
    return DevicePost(alpha_out.cpu().numpy().view(np.uint64)[:S].copy(), active.cpu().numpy()[:S].copy(),
                      alive_out, alive_skel, min_out, max_out, before, int(alive_out.sum().item()))


# ---------------------------------------------------------------------------
# Per-spectrum outcomes, packed for the gather to rank 0 (config 5 on N GPUs)
# ---------------------------------------------------------------------------
OUTCOME_MAGIC = 0x35435453  # "STC5"


def pack_outcomes(rows: DeviceRows, fx, sk: DeviceSkeleton, ln: DeviceLength, post=None):
    """One rank's config-5 outcome per spectrum as one uint8 device tensor:
    the fixpoint's and the skeleton's alphabets, both length bounds and their
    status, the Jaccard length and status, the walk's per-side status, the
    rows each side's walk kept (a bit per row slot), the combined skeleton
    (max_len positions reserved per spectrum, seq_len used), and with `post`
    (post_skeleton_device) the alphabet after the skeleton-based reduction
    and the fragments that survive it (a bit per row slot)."""
    import torch

    dev = sk.skel.device
    S = len(sk.max_len)
    u8 = lambda t: t.contiguous().view(torch.uint8).reshape(-1)  # noqa: E731
    host = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
    kept = (sk.kept & rows.alive.view(1, -1)).reshape(-1)
    pad = (-kept.numel()) % 8
    if pad:
        kept = torch.cat([kept, torch.zeros(pad, dtype=torch.uint8, device=dev)])
    weights = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.int32, device=dev)
    kept_bits = (kept.view(-1, 8).to(torch.int32) * weights).sum(dim=1).to(torch.uint8)
    def bits(flags):
        f = flags.reshape(-1)
        pad = (-f.numel()) % 8
        if pad:
            f = torch.cat([f, torch.zeros(pad, dtype=torch.uint8, device=dev)])
        return (f.view(-1, 8).to(torch.int32) * weights).sum(dim=1).to(torch.uint8)

    post_bits = bits(post.alive & rows.alive) if post is not None else None
    head = np.array([OUTCOME_MAGIC, S, int(rows.su.numel()), int(sk.skel_off[-1]), int(ln.comb_off[-1]),
                     int(kept_bits.numel()), 0 if post is None else int(post_bits.numel()), 0], dtype=np.int64)
    parts = [host(head), host(np.asarray(fx.alpha, dtype=np.uint64).view(np.int64)),
             host(ln.alpha.view(np.int64)), host(ln.lower), host(ln.upper), host(ln.lb_status),
             host(ln.seq_len.astype(np.int32)), host(ln.status), host(sk.status), host(sk.max_len.astype(np.int32)),
             ln.comb[:int(ln.comb_off[-1])], kept_bits]
    if post is not None:
        parts += [host(post.alpha.view(np.int64)), host(post.active.astype(np.uint8)), post_bits]
    return torch.cat([u8(p) for p in parts])


def unpack_outcomes(buf):
    """pack_outcomes' bytes (host numpy uint8) -> dict of numpy arrays."""
    b = np.asarray(buf, dtype=np.uint8)
    head = b[:64].view(np.int64)
    if int(head[0]) != OUTCOME_MAGIC:
        raise ValueError("not a config-5 outcome buffer")
    S, slots, _, n_comb, n_kept, n_post = (int(x) for x in head[1:7])
    o = 64
    out = {}

    def take(name, dtype, count):
        nonlocal o
        nb = np.dtype(dtype).itemsize * count
        out[name] = b[o:o + nb].view(dtype).copy()
        o += nb

    take("alpha", np.uint64, 2 * S)
    take("alpha_skeleton", np.uint64, 2 * S)
    take("lower", np.int64, S)
    take("upper", np.int64, S)
    take("lb_status", np.int8, S)
    take("seq_len", np.int32, S)
    take("status", np.int8, S)
    take("walk_status", np.uint8, 2 * S)
    take("max_len", np.int32, S)
    take("combined", np.uint64, 2 * n_comb)
    take("kept_bits", np.uint8, n_kept)
    out["kept"] = np.unpackbits(out.pop("kept_bits"), bitorder="little")[:2 * slots].reshape(2, slots)
    if n_post:
        take("alpha_post", np.uint64, 2 * S)
        take("post_active", np.uint8, S)
        take("post_bits", np.uint8, n_post)
        out["alpha_post"] = out["alpha_post"].reshape(S, 2)
        out["post_alive"] = np.unpackbits(out.pop("post_bits"), bitorder="little")[:slots]
    out["alpha"] = out["alpha"].reshape(S, 2)
    out["alpha_skeleton"] = out["alpha_skeleton"].reshape(S, 2)
    out["combined"] = out["combined"].reshape(-1, 2)
    if o != len(b):
        raise ValueError("outcome buffer size mismatch")
    return out
