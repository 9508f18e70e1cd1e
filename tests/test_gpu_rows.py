"""GPU tests of the step from the peaks (sst_step_rows_device: A7,
classify_fragments' filters, per-side SU order and the sliding window's pairs
formed on the device) against the host producers (bench.workload_from:
classify_queries + is_valid + filters + sst_su_diff_queries, the chain the
CPU suite pins to the reference) and the CPU oracle: A7 codes, the query
count, every answer (canonical digest against the explain pass over the
host-built queries), statuses and exact candidate lists of a sample against
the oracle; edge spectra (no peaks, one peak, duplicate peaks, heavy peaks,
spectra over 160 peaks, peaks not in mass order, intensities below the
cutoff, a mass cutoff that drops peaks)."""
import os
import sys

import numpy as np
import pytest

import _oracle as oracle

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dp():
    sys.path.insert(0, REPO)
    from spectrseqtools_amd import _native
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation

    seq = SequenceInformation(max_len=20, su_mass=6500.0, obs_mass=6500.0, modification_rate=0.5)
    return DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=MATCHING_THRESHOLD,
                                   precision=TOLERANCE, seq=seq, engine=_native.get_engine(0))


def _run(dp, wl, intensity=None, cutoff=0.5e6, mass_cutoff=50000.0, reuse=None, max_q=None):
    import torch

    dev = torch.device("cuda", 0)
    do = torch.from_numpy(wl["obs"]).to(dev)
    dpo = torch.from_numpy(wl["peak_off"]).to(dev)
    ds = torch.from_numpy(wl["su_seq"]).to(dev)
    di = None if intensity is None else torch.from_numpy(np.ascontiguousarray(intensity, dtype=np.float64)).to(dev)
    out7 = torch.full((4 * len(wl["obs"]),), 9, dtype=torch.int8, device=dev)
    torch.cuda.synchronize()
    A = round(dp.seq.modification_rate * dp.seq.max_len)
    res = dp.device_table.step_rows_device(do.data_ptr(), dpo.data_ptr(), len(wl["peak_off"]) - 1, len(wl["obs"]),
                                           ds.data_ptr(), wl["shifts"], wl["sides"], out7.data_ptr(),
                                           wl["max_weight"], dp.tolerance, dp.precision, A,
                                           max_q or max(1, int(len(wl["a8_mass"]) * 1.1) + 64),
                                           d_intensity=None if di is None else di.data_ptr(),
                                           intensity_cutoff=cutoff, mass_cutoff=mass_cutoff, reuse=reuse)
    res.fetch_device()
    dp.device_table.engine.synchronize()
    return res, out7.cpu().numpy()


def _check(dp, wl, res, a7, sample=800, seed=0):
    import torch
    from spectrseqtools_amd import _native
    from spectrseqtools_amd.parallel import canonical_digest

    assert np.array_equal(a7, wl["a7_valid"])
    n = len(wl["a8_mass"])
    assert res.n == n
    A = round(dp.seq.modification_rate * dp.seq.max_len)
    if n == 0:
        return
    dev = torch.device("cuda", 0)
    dm = torch.from_numpy(wl["a8_mass"]).to(dev)
    dt = torch.from_numpy(wl["a8_thr"]).to(dev)
    torch.cuda.synchronize()
    hq = dp.device_table.explain_device(dm.data_ptr(), dt.data_ptr(), n, dp.tolerance, dp.precision, A)
    hq.fetch_device()
    assert np.array_equal(res.status, hq.status)
    assert canonical_digest(res.status, res.count, res.offset, res.payload) == \
        canonical_digest(hq.status, hq.count, hq.offset, hq.payload)
    ms = [m.mass for m in dp.masses]
    host = oracle.build_table(ms, max(ms) * 35, 32)
    alph = oracle.Alphabet(ms, [m.is_modification for m in dp.masses],
                           [round(dp.seq.max_len * m.modification_rate) for m in dp.masses])
    rng = np.random.default_rng(seed)
    some = np.flatnonzero(res.status == _native.SST_SOME)
    pick = np.concatenate([rng.choice(some, min(sample, len(some)), replace=False),
                           rng.integers(0, n, min(sample, n))])
    for i in pick:
        st, sols, n_e, _ = oracle.explain_table(host, 32, alph, wl["a8_mass"][i], wl["a8_thr"][i], dp.tolerance, A)
        want = _native.SST_SOME if sols else (_native.SST_EMPTY if n_e else _native.SST_NONE)
        assert int(res.status[i]) == want, i
        assert res.candidates(int(i)) == sols, i


def test_rows_step_config3_sample(dp):
    import bench

    wl = bench.build_workload(2500, 4242, dp)
    res, a7 = _run(dp, wl)
    _check(dp, wl, res, a7)
    # reused result, another batch
    wl2 = bench.build_workload(1500, 4243, dp)
    res2, a72 = _run(dp, wl2, reuse=res)
    _check(dp, wl2, res2, a72, seed=1)


def test_rows_step_edge_spectra(dp):
    import bench
    from spectrseqtools_amd.synthetic import make_spectra

    b = make_spectra(40, seed=77)
    rng = np.random.default_rng(5)
    obs, offs, seqm, inten = [], [0], [], []
    for s in range(40):
        o = b.observed[b.offsets[s]:b.offsets[s + 1]]
        if s % 10 == 0:
            o = o[:0]  # no peaks
        elif s % 10 == 1:
            o = o[:1]  # one peak
        elif s % 10 == 2:
            o = np.concatenate([o, o[: len(o) // 2]])  # duplicate peaks: ties between rows
        elif s % 10 == 3:
            o = np.concatenate([o, rng.uniform(15000.0, 21000.0, 3)])  # heavy peaks (near the table's end)
        elif s % 10 == 4:  # over 160 peaks: the workgroup-per-spectrum kernels
            o = np.concatenate([o] + [b.observed[b.offsets[t]:b.offsets[t + 1]] for t in (s + 1, s + 2)])
        elif s % 10 == 6:  # every peak within max_weight of the others: more pairs than a side's answer slots
            o = rng.uniform(3000.0, 3250.0, 40)
        o = np.sort(o)
        if s % 10 == 5:
            o = np.concatenate([o, o[:3]])[rng.permutation(len(o) + 3)]  # unsorted, with ties: ranked on the device
        obs.append(o)
        offs.append(offs[-1] + len(o))
        seqm.append(b.seq_mass[s])
        inten.append(np.where(rng.random(len(o)) < 0.15, 1e5, 1e7))  # some below the cutoff
    obs, seqm, inten = np.concatenate(obs), np.array(seqm), np.concatenate(inten)
    for with_int, cut in ((False, 50000.0), (True, 50000.0), (True, 3000.0)):
        wl = bench.workload_from(obs, offs, seqm, dp, intensity=inten if with_int else None, mass_cutoff=cut)
        res, a7 = _run(dp, wl, intensity=inten if with_int else None, mass_cutoff=cut)
        _check(dp, wl, res, a7, sample=300, seed=2)


def test_rows_step_chunked(dp):
    """More spectra than the wave kernels' chunk arrays hold one per wave (64
    per CU: 16 384 on MI355X), so each wave takes a contiguous chunk of two
    spectra: the chunk totals, the 64-chunk tile sums and each spectrum's
    offsets within its chunk."""
    import bench

    wl = bench.build_workload(17000, 4711, dp)
    res, a7 = _run(dp, wl)
    _check(dp, wl, res, a7, sample=200, seed=4)


def test_rows_step_capacity_overflow(dp):
    """A result too small for the step's queries is reported, not overrun
    (each chunk checks its own end against the result's capacity after its
    look-back), and the next step on the same engine is answered in full."""
    import bench
    from spectrseqtools_amd import _native

    wl = bench.build_workload(600, 31, dp)
    with pytest.raises(_native.EngineError, match="more queries"):
        _run(dp, wl, max_q=len(wl["a8_mass"]) // 2)
    res, a7 = _run(dp, wl)
    _check(dp, wl, res, a7, sample=200, seed=3)


def test_rows_step_refuses_binding_budgets(dp):
    """Windows whose budgets could bind are refused, not answered wrongly."""
    import bench
    from spectrseqtools_amd import _native

    wl = bench.build_workload(20, 9, dp)
    import torch

    dev = torch.device("cuda", 0)
    do = torch.from_numpy(wl["obs"]).to(dev)
    dpo = torch.from_numpy(wl["peak_off"]).to(dev)
    ds = torch.from_numpy(wl["su_seq"]).to(dev)
    out7 = torch.empty(4 * len(wl["obs"]), dtype=torch.int8, device=dev)
    torch.cuda.synchronize()
    with pytest.raises(_native.EngineError, match="max_modifications"):
        dp.device_table.step_rows_device(do.data_ptr(), dpo.data_ptr(), 20, len(wl["obs"]), ds.data_ptr(),
                                         wl["shifts"], wl["sides"], out7.data_ptr(), wl["max_weight"], dp.tolerance,
                                         dp.precision, 1, 100000)
