"""Full-size parity at the benchmark's workload (10 000
synthetic spectra, full alphabet, <= 20-mer; 4.3 M A7 + 10.7 M A8 queries):
is_valid and explain statuses / candidate counts against the OpenMP C
oracle, bit-exact, and every returned candidate checked by size-independent
properties (a distinct multiset of table rows, in the reference's order,
whose mass sum lies in the query's quantised window)."""
import os
import sys

import numpy as np
import pytest

import _oracle as oracle

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def fullsize():
    sys.path.insert(0, REPO)
    import bench
    from spectrseqtools_amd import _native
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation

    seq = SequenceInformation(max_len=20, su_mass=6500.0, obs_mass=6500.0, modification_rate=0.5)
    dp = DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=MATCHING_THRESHOLD,
                                 precision=TOLERANCE, seq=seq, engine=_native.get_engine(0))
    wl = bench.build_workload(10000, 1000, dp)
    return dp, wl


@pytest.fixture(scope="module")
def oracle_a8(fullsize):
    """The C oracle's statuses / counts for all A8 queries (OpenMP), mapped
    to the engine's status codes; computed once for the module."""
    from spectrseqtools_amd import _native

    dp, wl = fullsize
    ms = [m.mass for m in dp.masses]
    host = oracle.build_table(ms, max(ms) * 35, 32)
    alph = oracle.Alphabet(ms, [m.is_modification for m in dp.masses],
                           [round(dp.seq.max_len * m.modification_rate) for m in dp.masses])
    A = round(dp.seq.modification_rate * dp.seq.max_len)
    ost, ocnt, _ = oracle.explain_batch(host, 32, alph, wl["a8_mass"], wl["a8_thr"], A, dp.tolerance, nthreads=16)
    want = np.where(ost < 0, _native.SST_OUT_OF_TABLE,
                    np.where(ost == 0, _native.SST_NONE, np.where(ocnt > 0, _native.SST_SOME, _native.SST_EMPTY)))
    return host, alph, want, ocnt


def _check_candidates(res, masses, thr, ms, prec):
    """Every candidate of every SOME query: rows ascending, sum inside the
    quantised window, distinct within its query, and in the reference's order
    (ascending sum, then top row)."""
    from spectrseqtools_amd import _native

    some = res.status == _native.SST_SOME
    target = np.rint(masses / prec)
    th = np.ceil(thr / prec)
    lo, hi = (target - th)[some], (target + th)[some]
    pos = res.offset[some].astype(np.int64)
    cnt = res.count[some].astype(np.int64)
    pay = res.payload
    prev_key = np.full(len(pos), -1, np.int64)
    for j in range(int(cnt.max())):
        act = j < cnt
        p = pos[act]
        k = pay[p].astype(np.int64)
        assert ((k >= 1) & (k <= 3)).all()
        r0 = pay[p + 1].astype(np.int64)
        r1 = np.where(k >= 2, pay[np.minimum(p + 2, len(pay) - 1)], 0).astype(np.int64)
        r2 = np.where(k >= 3, pay[np.minimum(p + 3, len(pay) - 1)], 0).astype(np.int64)
        assert (r0 >= 1).all() and ((k < 2) | (r1 >= r0)).all() and ((k < 3) | (r2 >= r1)).all()
        total = ms[r0] + np.where(k >= 2, ms[r1], 0) + np.where(k >= 3, ms[r2], 0)
        assert ((total >= lo[act]) & (total <= hi[act])).all()
        top = np.where(k == 1, r0, np.where(k == 2, r1, r2))
        key = total * 128 + top
        assert (key > prev_key[act]).all()  # strictly increasing: distinct and ordered
        prev_key[act] = key
        pos[act] = p + 1 + k


def test_fullsize_is_valid_vs_oracle(fullsize):
    dp, wl = fullsize
    ms = [m.mass for m in dp.masses]
    host = oracle.build_table(ms, max(ms) * 35, 32)
    got = dp.device_table.is_valid(wl["a7_mass"], wl["a7_thr"], dp.tolerance, dp.precision)
    want = oracle.is_valid_batch(host, 32, wl["a7_mass"], wl["a7_thr"], dp.tolerance, nthreads=16)
    assert len(got) > 4_000_000
    assert np.array_equal(got, want)


def test_fullsize_explain_vs_oracle_and_properties(fullsize, oracle_a8):
    from spectrseqtools_amd import _native

    dp, wl = fullsize
    host, alph, want, ocnt = oracle_a8
    ms = np.array([m.mass for m in dp.masses], dtype=np.int64)
    A = round(dp.seq.modification_rate * dp.seq.max_len)
    masses, thr = wl["a8_mass"], wl["a8_thr"]
    res = dp.device_table.explain(masses, thr, dp.tolerance, dp.precision, A)
    assert res.n > 10_000_000
    # statuses and counts: the C oracle (literal restatement), all queries
    assert np.array_equal(res.status.astype(np.int64), want)
    some = res.status == _native.SST_SOME
    assert np.array_equal(res.count[some].astype(np.int64), ocnt[some])
    _check_candidates(res, masses, thr, ms, dp.precision)


def test_fullsize_device_path_reused_vs_oracle(fullsize, oracle_a8):
    """The path bench.py times, at its full size: explain_device on HBM inputs
    into one result object reused over two passes (the pass packs its own
    dense result; the host settles it by polling the header), then fetched.
    Statuses and counts equal the oracle's for all 10.7 M queries, the dense
    hit list decodes to the same per-query counts and offsets, and both passes
    are bit-identical."""
    torch = pytest.importorskip("torch")
    from spectrseqtools_amd import _native
    from spectrseqtools_amd.parallel import device_bytes

    dp, wl = fullsize
    ms = np.array([m.mass for m in dp.masses], dtype=np.int64)
    A = round(dp.seq.modification_rate * dp.seq.max_len)
    masses, thr = wl["a8_mass"], wl["a8_thr"]
    n = len(masses)
    dev = torch.device("cuda", 0)
    dm = torch.from_numpy(masses).to(dev)
    dt = torch.from_numpy(thr).to(dev)
    torch.cuda.synchronize()
    tdev = dp.device_table
    res = None
    digests = []
    for _ in range(2):
        res = tdev.explain_device(dm.data_ptr(), dt.data_ptr(), n, dp.tolerance, dp.precision, A, reuse=res)
        n_hits, n_bytes = res.settle()
        ptr, nh = res.hit_list_device()
        assert nh == n_hits
        recs = device_bytes(ptr, 16 * nh, dev).cpu().numpy().view(np.uint32).reshape(-1, 4)
        res.fetch_device()
        assert len(res.payload) == n_bytes
        digests.append((res.status.tobytes(), recs.tobytes(), res.payload.tobytes()))
    assert digests[0] == digests[1]
    host, alph, want, ocnt = oracle_a8
    assert np.array_equal(res.status.astype(np.int64), want)
    some = res.status == _native.SST_SOME
    assert np.array_equal(res.count[some].astype(np.int64), ocnt[some])
    # the hit list: one record per query with candidates, decoding to the
    # fetched count / offset arrays; payloads in hit order, back to back
    q = recs[:, 0].astype(np.int64)
    assert len(q) == int(np.isin(res.status, (_native.SST_SOME, _native.SST_OVERFLOW)).sum())
    assert len(np.unique(q)) == len(q)
    assert np.array_equal(recs[:, 1].astype(np.int64), res.count[q].astype(np.int64))
    off = recs[:, 2].astype(np.int64) | (recs[:, 3].astype(np.int64) << 32)
    assert np.array_equal(off[some[q]], res.offset[q][some[q]].astype(np.int64))
    assert (np.diff(off[some[q]]) > 0).all()  # all-pair workload: payload pieces back to back in hit order
    # candidates decode inside their window (first candidate of every query)
    target = np.rint(masses / dp.precision)
    th = np.ceil(thr / dp.precision)
    qs = q[some[q]]
    p = off[some[q]]
    k = res.payload[p].astype(np.int64)
    r0 = res.payload[p + 1].astype(np.int64)
    r1 = np.where(k >= 2, res.payload[np.minimum(p + 2, len(res.payload) - 1)], 0).astype(np.int64)
    total = ms[r0] + np.where(k >= 2, ms[r1], 0)
    assert ((k >= 1) & (k <= 2)).all()
    assert ((total >= target[qs] - th[qs]) & (total <= target[qs] + th[qs])).all()


def test_fullsize_step_device_vs_oracle(fullsize, oracle_a8):
    """The exact launch bench.py times: sst_step_device --
    k_step, one scan workgroup per CU, ~41 tile rounds per scan wave, the
    is_valid workgroups beside it -- on the full config-3 workload, twice into
    one reused result.  Against the oracle: the A7 byte of every (peak x
    breakage) pair, every A8 status and count, the exact candidate lists of a
    sample, the candidates' properties for all queries, the dense hit list and
    the wire-v5 decode of the pass (scan order, pair refs)."""
    torch = pytest.importorskip("torch")
    from spectrseqtools_amd import _native
    from spectrseqtools_amd.parallel import canonical_digest, decode_hits, device_bytes, scan_order_key, wire_unpack

    dp, wl = fullsize
    host, alph, want, ocnt = oracle_a8
    ms = np.array([m.mass for m in dp.masses], dtype=np.int64)
    A = round(dp.seq.modification_rate * dp.seq.max_len)
    masses, thr = wl["a8_mass"], wl["a8_thr"]
    n, P = len(masses), len(wl["obs"])
    dev = torch.device("cuda", 0)
    dm, dt, do = (torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (masses, thr, wl["obs"]))
    out7 = torch.full((4 * P,), 9, dtype=torch.int8, device=dev)
    torch.cuda.synchronize()
    tdev = dp.device_table
    res, digests = None, []
    for _ in range(2):
        out7.fill_(9)
        torch.cuda.synchronize()
        res = tdev.step_device(do.data_ptr(), P, wl["shifts"], out7.data_ptr(), dm.data_ptr(), dt.data_ptr(), n,
                               dp.tolerance, dp.precision, A, reuse=res)
        n_hits, n_bytes = res.settle()
        ptr, nh = res.hit_list_device()
        assert nh == n_hits
        recs = device_bytes(ptr, 16 * nh, dev).cpu().numpy().view(np.uint32).reshape(-1, 4)
        res.fetch_device()
        digests.append((res.status.tobytes(), recs.tobytes(), res.payload.tobytes()))
    assert digests[0] == digests[1]
    # the timed grid: one scan workgroup per CU, many tile rounds per wave
    refs_p, n_pair, pair_bytes, n_wg = res.pair_hits_device()
    assert n_wg >= 64 and -(-((n + 63) // 64) // (16 * n_wg)) >= 8, n_wg
    # A7: every (breakage, peak) byte against the oracle
    engine_sync = _native.get_engine(0)
    engine_sync.synchronize()
    a7 = out7.cpu().numpy()
    assert len(a7) == len(wl["a7_mass"]) > 4_000_000
    assert np.array_equal(a7, oracle.is_valid_batch(host, 32, wl["a7_mass"], wl["a7_thr"], dp.tolerance, nthreads=16))
    # A8: all statuses and counts
    assert np.array_equal(res.status.astype(np.int64), want)
    some = res.status == _native.SST_SOME
    assert np.array_equal(res.count[some].astype(np.int64), ocnt[some])
    _check_candidates(res, masses, thr, ms, dp.precision)
    # exact candidate lists (reference order) of a sample of the hits
    rng = np.random.default_rng(31)
    for i in rng.choice(np.flatnonzero(some), 3000, replace=False):
        st, sols, _, _ = oracle.explain_table(host, 32, alph, masses[i], thr[i], dp.tolerance, A)
        assert res.candidates(int(i)) == sols, i
    # the dense hit list: pair-path hits first, in the scan's order
    q = recs[:, 0].astype(np.int64)
    assert len(q) == int(np.isin(res.status, (_native.SST_SOME, _native.SST_OVERFLOW)).sum())
    assert len(np.unique(q)) == len(q)
    assert np.array_equal(recs[:, 1].astype(np.int64), res.count[q].astype(np.int64))
    off = recs[:, 2].astype(np.int64) | (recs[:, 3].astype(np.int64) << 32)
    assert np.array_equal(off[some[q]], res.offset[q][some[q]].astype(np.int64))
    assert 0 < n_pair <= len(q)
    assert (np.diff(scan_order_key(q[:n_pair], n, n_wg)) > 0).all()
    # wire v5 of this pass decodes to the same result
    precs = tdev.pair_records()
    fixed = res.wire_pack(out7.data_ptr(), 4 * P)
    wbuf = torch.zeros(fixed + 8 * (4 * P + n + n_pair), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    res.wire_pack(out7.data_ptr(), 4 * P, wbuf.data_ptr(), wbuf.numel())
    engine_sync.synchronize()
    v_, st_, hits_, pay_ = wire_unpack(wbuf.cpu().numpy(), precs)
    cnt_, off_ = decode_hits(st_, hits_)
    assert np.array_equal(v_, a7) and np.array_equal(st_, res.status)
    assert canonical_digest(st_, cnt_, off_, pay_) == canonical_digest(res.status, res.count, res.offset, res.payload)


def test_fullsize_rows_step_vs_oracle(fullsize, oracle_a8):
    """The step from the peaks (bench.py --a8-source rows: sst_step_rows_device,
    A7, the classification filters, per-side SU order and the sliding window's
    pairs formed on the device) on the full config-3 workload, twice into one
    reused result.  Its queries are the host producers' in the same order, so
    against the oracle: the A7 byte of every (peak x breakage) pair, every A8
    status and count, the candidates' properties, the exact candidate lists of
    a sample and the dense hit list (query order, payload back to back)."""
    torch = pytest.importorskip("torch")
    from spectrseqtools_amd import _native
    from spectrseqtools_amd.parallel import device_bytes

    dp, wl = fullsize
    host, alph, want, ocnt = oracle_a8
    ms = np.array([m.mass for m in dp.masses], dtype=np.int64)
    A = round(dp.seq.modification_rate * dp.seq.max_len)
    masses, thr = wl["a8_mass"], wl["a8_thr"]
    n, P, S = len(masses), len(wl["obs"]), len(wl["peak_off"]) - 1
    dev = torch.device("cuda", 0)
    do, dpo, ds = (torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (wl["obs"], wl["peak_off"], wl["su_seq"]))
    out7 = torch.full((4 * P,), 9, dtype=torch.int8, device=dev)
    torch.cuda.synchronize()
    tdev = dp.device_table
    res, digests = None, []
    for _ in range(2):
        out7.fill_(9)
        torch.cuda.synchronize()
        res = tdev.step_rows_device(do.data_ptr(), dpo.data_ptr(), S, P, ds.data_ptr(), wl["shifts"], wl["sides"],
                                    out7.data_ptr(), wl["max_weight"], dp.tolerance, dp.precision, A,
                                    int(n * 1.1) + 64, reuse=res)
        n_hits, n_bytes = res.settle()
        ptr, nh = res.hit_list_device()
        assert nh == n_hits
        recs = device_bytes(ptr, 16 * nh, dev).cpu().numpy().view(np.uint32).reshape(-1, 4)
        res.fetch_device()
        assert res.n == n and len(res.payload) == n_bytes
        digests.append((res.status.tobytes(), recs.tobytes(), res.payload.tobytes()))
    assert digests[0] == digests[1]
    _native.get_engine(0).synchronize()
    a7 = out7.cpu().numpy()
    assert len(a7) == len(wl["a7_mass"]) > 4_000_000
    assert np.array_equal(a7, oracle.is_valid_batch(host, 32, wl["a7_mass"], wl["a7_thr"], dp.tolerance, nthreads=16))
    assert np.array_equal(res.status.astype(np.int64), want)
    some = res.status == _native.SST_SOME
    assert np.array_equal(res.count[some].astype(np.int64), ocnt[some])
    _check_candidates(res, masses, thr, ms, dp.precision)
    rng = np.random.default_rng(37)
    for i in rng.choice(np.flatnonzero(some), 3000, replace=False):
        st, sols, _, _ = oracle.explain_table(host, 32, alph, masses[i], thr[i], dp.tolerance, A)
        assert res.candidates(int(i)) == sols, i
    q = recs[:, 0].astype(np.int64)
    assert len(q) == int(np.isin(res.status, (_native.SST_SOME, _native.SST_OVERFLOW)).sum())
    assert (np.diff(q) > 0).all()  # query order
    assert np.array_equal(recs[:, 1].astype(np.int64), res.count[q].astype(np.int64))
    off = recs[:, 2].astype(np.int64) | (recs[:, 3].astype(np.int64) << 32)
    assert np.array_equal(off[some[q]], res.offset[q][some[q]].astype(np.int64))
    assert (np.diff(off[some[q]]) > 0).all()
