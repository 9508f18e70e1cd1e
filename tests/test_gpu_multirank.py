"""SURVEY 8(d) config 4 on the HIP engine: bench.py's sharded, gathered step
(spectra sharded by rank, every step's complete result packed on the device
in the wire format and gathered to rank 0 while the next step computes) run
as two ranks on GPU 0 (torch.distributed gloo, SST_DEVICE=0: one card on the
test box; the driver's 8-GPU run uses RCCL).  Rank 0's received buffers of the
last step are decoded here (wire_unpack + decode_hits) and EVERY query of both
ranks is checked against the CPU oracle: is_valid codes, explain statuses and
counts, candidate properties, and the exact candidate lists of a sample."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import _oracle as oracle

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_gathered_step_vs_oracle(tmp_path):
    from spectrseqtools_amd import _native
    from spectrseqtools_amd.masses import EXPLANATION_MASSES
    from spectrseqtools_amd.mass_table import initialize_nucleotide_masses
    from spectrseqtools_amd.parallel import candidates, decode_hits, wire_unpack

    dump = str(tmp_path / "gathered")
    env = dict(os.environ, SST_DEVICE="0", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"), "--gpus", "2",
           "--backend", "gloo", "--spectra", "1200", "--steps", "4", "--warmup", "1", "--batches", "2",
           "--no-cpu-baseline", "--dump-gathered", dump]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280, cwd=REPO)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-5000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    assert '"n_gpus": 2' in line and "gathered to rank 0" in line
    g = np.load(os.path.join(dump, "gathered.npz"))
    precs = g["precs"]
    masses = initialize_nucleotide_masses(EXPLANATION_MASSES)
    ms = [m.mass for m in masses]
    host = oracle.build_table(ms, max(ms) * 35, 32)
    caps = [round(20 * min(m.modification_rate, 0.5)) if m.is_modification else round(20 * m.modification_rate)
            for m in masses]
    alph = oracle.Alphabet(ms, [m.is_modification for m in masses], caps)
    rng = np.random.default_rng(41)
    for r in range(2):
        inp = np.load(os.path.join(dump, f"inputs_rank{r}.npz"))
        A = int(inp["max_mods"])
        valid, st, hits, pay = wire_unpack(g[f"rank{r}"], precs)
        cnt, off = decode_hits(st, hits)
        assert len(valid) == len(inp["a7_mass"]) > 100_000 and len(st) == len(inp["a8_mass"]) > 1_000_000
        want7 = oracle.is_valid_batch(host, 32, inp["a7_mass"], inp["a7_thr"], 1e-5, nthreads=16)
        assert np.array_equal(valid, want7), r
        ost, ocnt, _ = oracle.explain_batch(host, 32, alph, inp["a8_mass"], inp["a8_thr"], A, 1e-5, nthreads=16)
        want = np.where(ost < 0, _native.SST_OUT_OF_TABLE,
                        np.where(ost == 0, _native.SST_NONE, np.where(ocnt > 0, _native.SST_SOME, _native.SST_EMPTY)))
        assert np.array_equal(st.astype(np.int64), want), r
        some = st == _native.SST_SOME
        assert np.array_equal(cnt[some].astype(np.int64), ocnt[some]), r
        # every candidate decodes to a distinct multiset inside its window, in the reference's order
        target, th = np.rint(inp["a8_mass"] / 1e-3), np.ceil(inp["a8_thr"] / 1e-3)
        for i in np.flatnonzero(some)[::97]:
            c = candidates(pay, cnt, off, i)
            sums = [sum(ms[x] for x in t) for t in c]
            assert all(target[i] - th[i] <= v <= target[i] + th[i] for v in sums), i
            assert [(v, t[-1]) for v, t in zip(sums, c)] == sorted(set((v, t[-1]) for v, t in zip(sums, c))), i
        for i in rng.choice(np.flatnonzero(some), 1500, replace=False):
            _, sols, _, _ = oracle.explain_table(host, 32, alph, inp["a8_mass"][i], inp["a8_thr"][i], 1e-5, A)
            assert candidates(pay, cnt, off, i) == sols, (r, i)


@pytest.mark.timeout(600)  # three pipeline runs (two ranks, then each rank alone)
def test_two_rank_pipeline_outcomes_vs_single_rank(tmp_path):
    """Config 5 sharded: tools/pipeline_bench.py as two ranks on GPU 0 (gloo),
    every stage device-resident through the skeleton walk and the length
    selection, each rank's per-spectrum outcomes gathered to rank 0; each
    rank's gathered bytes equal a single-process run on that rank's spectra.
    The ranks run with PYTHONHASHSEED unset (each interpreter its own str
    hashes): the walk must follow rank 0's name hashes on both ranks, and the
    single-rank runs are given those (--name-hashes)."""
    from spectrseqtools_amd import _native
    from spectrseqtools_amd.pipeline_device import unpack_outcomes

    multi, single = str(tmp_path / "multi"), str(tmp_path / "single")
    env = dict(os.environ, SST_DEVICE="0", MASTER_ADDR="127.0.0.1")
    env.pop("PYTHONHASHSEED", None)  # random per interpreter: rank 0's name hashes must rule
    bench = os.path.join(REPO, "tools", "pipeline_bench.py")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), bench, "--spectra", "400", "--warmup-spectra", "16", "--length-spectra", "48", "--backend", "gloo", "--cpu-baseline-s", "0",
           "--dump-outcomes", multi]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280, cwd=REPO)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-5000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    assert '"n_gpus": 2' in line and '"gather"' in line
    for r in range(2):
        p = subprocess.run([sys.executable, bench, "--spectra", "400", "--warmup-spectra", "16", "--length-spectra", "48",
                            "--cpu-baseline-s", "0", "--as-rank", str(r), "--dump-outcomes", single, "--name-hashes",
                            os.path.join(multi, "name_hashes.npy")],
                           env=env, capture_output=True, text=True, timeout=250,
                           cwd=REPO)
        assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-5000:]
        got = np.load(os.path.join(multi, f"outcome_rank{r}.npy"))
        want = np.load(os.path.join(single, f"outcome_rank{r}.npy"))
        assert np.array_equal(got, want), r
        o = unpack_outcomes(got)
        # stage 5 ran on each rank's first 48 spectra (--length-spectra): the
        # others carry SST_JAC_BOUNDS (their bounds not run)
        assert len(o["seq_len"]) == 400 and (o["walk_status"] == 0).all()
        assert (o["status"][:48] == 0).sum() > 24 and (o["status"][48:] == _native.JAC_BOUNDS).all()
