"""GPU tests of the result path (through the C ABI): candidate caps (SST_OVERFLOW
with the exact count), the device entry points with result reuse (the pair
scan's hit lists are rebuilt every pass and scattered into count/offset at the
first view), and queueing on a caller's stream (sst_ctx_set_stream).
Checked against the CPU oracle and against the host-buffer entry points."""
import numpy as np
import pytest

import _oracle as oracle
from conftest import load_golden
from spectrseqtools_amd import _native

pytestmark = pytest.mark.gpu

TOL, PREC = 1e-5, 1e-3
CANONICAL = (305042, 306026, 329053, 345048)


@pytest.fixture(scope="module")
def engine():
    return _native.get_engine(0)


@pytest.fixture(scope="module")
def rows():
    g = load_golden("alphabet.json")
    return sorted({r["tolerated_integer_masses"] for r in g["rows"]} | {0})


@pytest.fixture(scope="module")
def dev(engine, rows):
    t = _native.DeviceTable.build(rows, max(rows) * 35, 32, engine=engine)
    is_mod = [m not in CANONICAL and m != 0 for m in rows]
    t.set_budgets(is_mod, [round(20 * (0.5 if md else (1.0 if m else 0.0))) for m, md in zip(rows, is_mod)])
    return t


@pytest.fixture(scope="module")
def host(rows):
    return oracle.build_table(rows, max(rows) * 35, 32)


def _queries(rng, rows, n, kmax, thr_hi=14000, noise=0.004):
    ints = np.array(rows[1:])
    k = rng.integers(1, kmax + 1, n)
    masses = np.array([ints[rng.integers(0, len(ints), kk)].sum() for kk in k]) * 1e-3
    return masses + rng.normal(0, noise, n), 1e-5 * rng.uniform(300, thr_hi, n)


def _same(a, b, n):
    """Two ExplainResults hold the same answers (status, counts, candidates)."""
    assert np.array_equal(a.status[:n], b.status[:n])
    for i in range(n):
        if int(a.status[i]) in (_native.SST_SOME, _native.SST_OVERFLOW):
            assert int(a.count[i]) == int(b.count[i]), i
        if int(a.status[i]) == _native.SST_SOME:
            assert a.candidates(i) == b.candidates(i), i


def test_explain_cap_overflow(dev, host, rows):
    """cap_per_query: sets larger than the cap report OVERFLOW with the exact
    count and no payload, on the pair path (<= 2 items) and beyond it."""
    rng = np.random.default_rng(11)
    m2, t2 = _queries(rng, rows, 400, 2)
    m3, t3 = _queries(rng, rows, 80, 3)
    masses, thr = np.concatenate([m2, m3]), np.concatenate([t2, t3])
    is_mod = [m not in CANONICAL and m != 0 for m in rows]
    alph = oracle.Alphabet(rows, is_mod, [round(20 * (0.5 if md else (1.0 if m else 0.0)))
                                          for m, md in zip(rows, is_mod)])
    want = [oracle.explain_table(host, 32, alph, masses[i], thr[i], TOL, 10) for i in range(len(masses))]
    for cap in (1, 2, 3):
        res = dev.explain(masses, thr, TOL, PREC, 10, cap=cap)
        n_over = n_some = 0
        for i, (st, sols, n_empty, _) in enumerate(want):
            if st < 0:
                assert int(res.status[i]) == _native.SST_OUT_OF_TABLE, i
            elif len(sols) > cap:
                assert int(res.status[i]) == _native.SST_OVERFLOW, (cap, i, int(res.status[i]), len(sols))
                assert int(res.count[i]) == len(sols), (cap, i)
                n_over += 1
            else:
                ws = _native.SST_SOME if sols else (_native.SST_EMPTY if n_empty else _native.SST_NONE)
                assert int(res.status[i]) == ws, (cap, i)
                if sols:
                    assert res.candidates(i) == sols, (cap, i)
                    n_some += 1
        assert n_over > 0 and n_some > 0, (cap, n_over, n_some)


def test_device_entry_points_with_reuse(engine, dev, rows):
    """explain_device / is_valid_device on HBM inputs, one result object reused
    over passes with many, few and many hits again: every pass matches the
    host-buffer entry points (stale hit lists or offsets would not)."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(12)
    n = 3000
    many = _queries(rng, rows, n, 2)
    few = (rng.uniform(0.2, 0.9, n), 1e-5 * rng.uniform(300, 2000, n))  # masses below the first reachable one
    mixed = _queries(rng, rows, n, 3)
    dev_t = torch.device("cuda", engine.device)
    res = None
    out = torch.empty(n, dtype=torch.int8, device=dev_t)
    for masses, thr in (many, few, many, mixed):
        dm = torch.from_numpy(np.ascontiguousarray(masses)).to(dev_t)
        dt = torch.from_numpy(np.ascontiguousarray(thr)).to(dev_t)
        torch.cuda.synchronize()  # the engine queues on its own stream
        res = dev.explain_device(dm.data_ptr(), dt.data_ptr(), n, TOL, PREC, 10, reuse=res)
        dev.is_valid_device(dm.data_ptr(), dt.data_ptr(), n, TOL, PREC, out.data_ptr())
        res.fetch_device()
        _same(res, dev.explain(masses, thr, TOL, PREC, 10), n)
        engine.synchronize()
        assert np.array_equal(out.cpu().numpy(), dev.is_valid(masses, thr, TOL, PREC))


def test_side_stream(engine, dev, rows):
    """sst_ctx_set_stream: A7 on a caller's stream beside A8 on the engine
    stream; results equal the one-stream results."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(13)
    n = 5000
    masses, thr = _queries(rng, rows, n, 2)
    dev_t = torch.device("cuda", engine.device)
    dm = torch.from_numpy(masses).to(dev_t)
    dt = torch.from_numpy(thr).to(dev_t)
    out = torch.full((n,), 7, dtype=torch.int8, device=dev_t)
    side = torch.cuda.Stream(device=dev_t)
    torch.cuda.synchronize()
    res = dev.explain_device(dm.data_ptr(), dt.data_ptr(), n, TOL, PREC, 10)
    try:
        engine.set_stream(side.cuda_stream)
        dev.is_valid_device(dm.data_ptr(), dt.data_ptr(), n, TOL, PREC, out.data_ptr())
    finally:
        engine.set_stream(None)
    torch.cuda.synchronize()
    res.fetch_device()
    assert np.array_equal(out.cpu().numpy(), dev.is_valid(masses, thr, TOL, PREC))
    _same(res, dev.explain(masses, thr, TOL, PREC, 10), n)


def test_hit_list_matches_result_arrays(engine, dev, rows):
    """sst_result_hit_list: one {query, count, offset} record per query with
    candidates, equal to the compacted count / offset arrays (the --gather
    wire format)."""
    torch = pytest.importorskip("torch")
    from spectrseqtools_amd.parallel import device_bytes

    rng = np.random.default_rng(14)
    n = 4000
    masses, thr = _queries(rng, rows, n, 3)
    dev_t = torch.device("cuda", engine.device)
    dm = torch.from_numpy(masses).to(dev_t)
    dt = torch.from_numpy(thr).to(dev_t)
    torch.cuda.synchronize()
    res = dev.explain_device(dm.data_ptr(), dt.data_ptr(), n, TOL, PREC, 10, cap=50)
    ptr, n_hits = res.hit_list_device()
    recs = device_bytes(ptr, 16 * n_hits, dev_t).cpu().numpy().view(np.uint32).reshape(-1, 4)
    res.fetch_device()
    has = np.isin(res.status, (_native.SST_SOME, _native.SST_OVERFLOW, _native.SST_ABORTED))
    assert n_hits == int(has.sum()) and n_hits > 0
    q = recs[:, 0].astype(np.int64)
    assert len(np.unique(q)) == n_hits and has[q].all()
    assert np.array_equal(recs[:, 1].astype(np.uint64), res.count[q])
    st = res.status[q]
    some = st == _native.SST_SOME
    off = recs[:, 2].astype(np.uint64) | (recs[:, 3].astype(np.uint64) << np.uint64(32))
    assert np.array_equal(off[some], res.offset[q][some])
    assert (st == _native.SST_OVERFLOW).any()  # cap=50 leaves some queries over the cap


def test_wire_pair_hits_roundtrip(engine, dev, rows):
    """sst_result_pair_hits + sst_wire_pack / parallel.wire_unpack (the N>1
    gather's wire format v5) on a real device pass: the pair-path hits come
    in the documented scan order (several tile rounds per wave), their refs
    name the pair-list entries of their candidates (SOME and OVERFLOW), the
    device packer writes the bytes of the numpy statement (wire_pack_host;
    list entries in any order), and the decoded wire holds exactly the
    result's answers (canonical digest: status, counts, every query's
    candidate bytes) and the is_valid codes.  A buffer too small for the list
    is refused by the receiver."""
    torch = pytest.importorskip("torch")
    from spectrseqtools_amd.parallel import (canonical_digest, decode_hits, device_bytes, scan_order_key,
                                             wire_pack_host, wire_unpack, wire_used_bytes)

    rng = np.random.default_rng(15)
    m2, t2 = _queries(rng, rows, 600_000, 2)
    m3, t3 = _queries(rng, rows, 3000, 3)
    masses, thr = np.concatenate([m2, m3, np.full(7, 1e7)]), np.concatenate([t2, t3, np.full(7, 0.01)])
    perm = rng.permutation(len(masses))
    masses, thr = masses[perm], thr[perm]
    n = len(masses)
    dev_t = torch.device("cuda", engine.device)
    dm = torch.from_numpy(masses).to(dev_t)
    dt = torch.from_numpy(thr).to(dev_t)
    valid = rng.integers(-1, 2, 100_003).astype(np.int8)
    dv = torch.from_numpy(valid).to(dev_t)
    torch.cuda.synchronize()
    res = dev.explain_device(dm.data_ptr(), dt.data_ptr(), n, TOL, PREC, 10, cap=3)
    hits_p, n_hits = res.hit_list_device()
    refs_p, n_pair, pair_bytes, n_wg = res.pair_hits_device()
    assert 0 < n_pair < n_hits and n_wg > 1
    assert -(-((n + 63) // 64) // (16 * n_wg)) > 1  # several tile rounds per scan wave
    hits = device_bytes(hits_p, 16 * n_hits, dev_t)
    recs = dev.pair_records()
    fixed = res.wire_pack(dv.data_ptr(), len(valid))  # sizing only
    cap = fixed + 8 * (len(valid) + n + n_pair)
    wbuf = torch.zeros(cap, dtype=torch.uint8, device=dev_t)
    torch.cuda.synchronize()  # the engine stream packs into it
    assert res.wire_pack(dv.data_ptr(), len(valid), wbuf.data_ptr(), cap) == fixed
    torch.cuda.synchronize()
    engine.synchronize()
    wire = wbuf.cpu().numpy()
    res.fetch_device()
    h = hits.cpu().numpy().view(np.uint32).reshape(-1, 4)
    q = h[:n_pair, 0].astype(np.int64)
    key = scan_order_key(q, n, n_wg)
    assert (np.diff(key) > 0).all()  # the scan's order
    refs = device_bytes(refs_p, 2 * n_pair, dev_t).cpu().numpy().view(np.uint16)
    ovf = (refs >> 15).astype(bool)
    assert np.array_equal(ovf, res.status[q] == _native.SST_OVERFLOW) and ovf.any()
    for j in np.flatnonzero(~ovf)[:200]:  # refs name the candidates' pair-list entries
        first, cnt = int(refs[j] & 0x7FFF), int(h[j, 1])
        want = [tuple((int(r) >> (8 * (k + 1))) & 0xFF for k in range(int(r) & 0xFF)) for r in recs[first:first + cnt]]
        assert res.candidates(int(q[j])) == want, j
    # the device packer's bytes = the numpy statement's
    used = wire_used_bytes(wire)
    want = wire_pack_host(valid, res.status, h, res.payload, refs, n_pair, pair_bytes, n_wg, recs)
    assert used == len(want) and used > fixed  # raises, OUT_OF_TABLE / OVERFLOW statuses, counts > 7 listed
    hw, hh = wire[:128].view(np.uint64).copy(), want[:128].view(np.uint64).copy()
    hw[10] = hh[10] = 0  # list capacity: the buffer's, not the result's
    assert np.array_equal(hw, hh)
    assert np.array_equal(wire[128:fixed], want[128:fixed])
    srt = lambda b: np.sort(b[fixed:used].view(np.uint64))  # list entries: in any order
    assert np.array_equal(srt(wire), srt(want))
    types = set((wire[fixed:used].view(np.uint32)[0::2] >> 30).tolist())
    assert types == {0, 1, 2}, types
    v_, st_, hits_, pay_ = wire_unpack(wire, recs)
    cnt_, off_ = decode_hits(st_, hits_)
    assert np.array_equal(v_, valid)
    assert np.array_equal(st_, res.status)
    assert canonical_digest(st_, cnt_, off_, pay_) == canonical_digest(res.status, res.count, res.offset, res.payload)
    # no room for the list: the receiver refuses the buffer
    small = torch.zeros(fixed, dtype=torch.uint8, device=dev_t)
    torch.cuda.synchronize()
    res.wire_pack(dv.data_ptr(), len(valid), small.data_ptr(), fixed)
    torch.cuda.synchronize()
    engine.synchronize()
    with pytest.raises(ValueError, match="list entries"):
        wire_unpack(small.cpu().numpy(), recs)


def test_step_device_equals_separate_calls(engine, dev, rows):
    """sst_step_device (is_valid over peaks and the explain pass in one
    launch) gives the same is_valid bytes and the same answers as
    sst_is_valid_peaks_device + sst_explain_batch_device, over result reuse;
    and with 3 breakage weights (two launches)."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(16)
    n = 40_000
    masses, thr = _queries(rng, rows, n, 2)
    obs = np.sort(rng.uniform(150.0, 9000.0, 25_000))
    dev_t = torch.device("cuda", engine.device)
    dm, dt, do = (torch.from_numpy(np.ascontiguousarray(x)).to(dev_t) for x in (masses, thr, obs))
    for shifts in (np.array([0.0, 375.183, 537.119, 912.303]), np.array([0.0, 375.183, 537.119])):
        out_a = torch.full((len(shifts) * len(obs),), 9, dtype=torch.int8, device=dev_t)
        out_b = torch.full_like(out_a, 7)
        torch.cuda.synchronize()
        res = None
        for _ in range(2):
            res = dev.step_device(do.data_ptr(), len(obs), shifts, out_a.data_ptr(), dm.data_ptr(), dt.data_ptr(), n,
                                  TOL, PREC, 10, reuse=res)
            res.fetch_device()
        dev.is_valid_peaks_device(do.data_ptr(), len(obs), shifts, TOL, PREC, out_b.data_ptr())
        ref = dev.explain_device(dm.data_ptr(), dt.data_ptr(), n, TOL, PREC, 10)
        ref.fetch_device()
        engine.synchronize()
        assert np.array_equal(out_a.cpu().numpy(), out_b.cpu().numpy())
        _same(res, ref, n)


def test_empty_batches(engine, dev, rows):
    """Zero-length batches on every entry point: empty results (no launch
    faults), a result reused from full to empty and back, and the step entry
    point with no peaks or no explain queries."""
    torch = pytest.importorskip("torch")
    e = np.zeros(0)
    assert len(dev.is_valid(e, e, TOL, PREC)) == 0
    r0 = dev.explain(e, e, TOL, PREC, 10)
    assert r0.n == 0 and len(r0.status) == 0
    dev_t = torch.device("cuda", engine.device)
    rng = np.random.default_rng(17)
    masses, thr = _queries(rng, rows, 1000, 2)
    dm = torch.from_numpy(masses).to(dev_t)
    dt = torch.from_numpy(thr).to(dev_t)
    obs = torch.from_numpy(np.sort(rng.uniform(200.0, 5000.0, 300))).to(dev_t)
    out = torch.full((4 * 300,), 9, dtype=torch.int8, device=dev_t)
    shifts = np.array([0.0, 375.183, 537.119, 912.303])
    torch.cuda.synchronize()
    res = None
    for n in (1000, 0, 1000, 0):  # a result has the capacity of its first pass
        res = dev.explain_device(dm.data_ptr(), dt.data_ptr(), n, TOL, PREC, 10, reuse=res)
        nh, nb = res.settle()
        res.fetch_device()
        if n == 0:
            assert nh == 0 and nb == 0 and len(res.status) == 0
        else:
            _same(res, dev.explain(masses, thr, TOL, PREC, 10), n)
    ref = dev.is_valid_peaks(obs.cpu().numpy(), shifts, TOL, PREC)
    s0 = dev.step_device(obs.data_ptr(), 300, shifts, out.data_ptr(), dm.data_ptr(), dt.data_ptr(), 0, TOL, PREC, 10)
    s0.fetch_device()
    engine.synchronize()
    assert len(s0.status) == 0 and np.array_equal(out.cpu().numpy(), ref)
    s1 = dev.step_device(obs.data_ptr(), 0, shifts, out.data_ptr(), dm.data_ptr(), dt.data_ptr(), 1000, TOL, PREC, 10)
    s1.fetch_device()
    _same(s1, dev.explain(masses, thr, TOL, PREC, 10), 1000)
    ptr, nh = s1.hit_list_device()
    assert nh == int(np.isin(s1.status, (_native.SST_SOME, _native.SST_OVERFLOW)).sum())


def test_reuse_across_empty_pass_with_lookback(engine, dev, rows):
    """A result reused big -> empty -> a different big batch, with enough
    queries for several scan workgroups (the fused scan's decoupled look-back
    runs): after the empty pass the next pass's dense result, pair-path part
    and wire pack equal a fresh result's (an empty pass must zero the
    look-back aggregates and the scan header the next pass reads)."""
    torch = pytest.importorskip("torch")
    from spectrseqtools_amd.parallel import canonical_digest, decode_hits, wire_unpack

    rng = np.random.default_rng(18)
    n = 150_000
    batches = [_queries(rng, rows, n, 2), _queries(rng, rows, n, 2, thr_hi=9000)]
    dev_t = torch.device("cuda", engine.device)
    dd = [tuple(torch.from_numpy(np.ascontiguousarray(x)).to(dev_t) for x in b) for b in batches]
    valid = np.zeros(16, np.int8)
    dv = torch.from_numpy(valid).to(dev_t)
    torch.cuda.synchronize()
    recs = dev.pair_records()
    res = None
    for b, nn in ((0, n), (0, 0), (1, n), (1, 0), (0, n), (1, n)):
        dm, dt = dd[b]
        res = dev.explain_device(dm.data_ptr(), dt.data_ptr(), nn, TOL, PREC, 10, reuse=res)
        res.fetch_device()
        if nn == 0:
            assert res.settle() == (0, 0)
            continue
        # the reference: a result that never saw an empty pass.  Whether a pass
        # keeps its pair-path part depends on the arena it finds (a pass that
        # outgrows it re-runs unfused, reporting no pair-path part), so the
        # comparison is of the decoded results, not of that split
        fresh = dev.explain_device(dm.data_ptr(), dt.data_ptr(), nn, TOL, PREC, 10)
        fresh.fetch_device()
        _, n_pair, pair_bytes, n_wg = res.pair_hits_device()
        assert n_wg > 1
        assert res.settle()[0] == fresh.settle()[0]  # hits (the payload's pad bytes follow the layout)
        assert canonical_digest(res.status, res.count, res.offset, res.payload) == \
            canonical_digest(fresh.status, fresh.count, fresh.offset, fresh.payload)
        fixed = res.wire_pack(dv.data_ptr(), len(valid))
        wbuf = torch.zeros(fixed + 8 * (len(valid) + nn + n_pair), dtype=torch.uint8, device=dev_t)
        torch.cuda.synchronize()
        res.wire_pack(dv.data_ptr(), len(valid), wbuf.data_ptr(), wbuf.numel())
        engine.synchronize()
        v_, st_, hits_, pay_ = wire_unpack(wbuf.cpu().numpy(), recs)
        cnt_, off_ = decode_hits(st_, hits_)
        assert canonical_digest(st_, cnt_, off_, pay_) == \
            canonical_digest(fresh.status, fresh.count, fresh.offset, fresh.payload)
