#!/usr/bin/env python3
"""bench.py -- peaks explained/sec on MI355X (BASELINE.json metric).

One step = the reference pipeline's hot path over one batch of synthetic
spectra (10k spectra, ~1M peaks, full 104-mass /
105-row alphabet, <=20-mer) with every input already resident in HBM:
  * A7: is_valid_mass for every peak x 4 breakage weights
        (fragment_classification.py:52-67)  -> k_is_valid_peaks (one lane per
        peak, the peak's mass read once for its 4 windows)
  * A8: explain_mass_with_table for every adjacent SU-mass difference the
        reference's sliding window emits (prediction.py:286-329), budget
        round(0.5*max_len)                  -> k_explain_main (+ deferred kernels)
  * N>1: spectra shard by rank (weak scaling: `--spectra` per GPU); each
        step's complete result of every rank (wire format v5, sst_wire_pack:
        1-bit A7 / A8 codes, ~16 bits per pair-path hit, the deferred hits'
        records and payload; ~5.4 MB per rank per config-3 step) is packed on
        the device and gathered to rank 0 over RCCL on other streams while the
        next step computes (--no-gather: results stay in each rank's HBM).
value = peaks of all ranks / step time (max over ranks).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--spectra S]
       (N>1 under torch.distributed.run, one rank per GPU)
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "peaks explained/sec (full 148-nt alphabet, <=20-mer) at 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def windows(masses, thr, prec, limit):
    """Scan range [max(lo,1), hi] of each query (the same IEEE quantisation as
    the kernels / mass_explanation.py:107-114) and the bitset words it spans
    (0 for windows that are empty or leave the table)."""
    target = np.rint(masses / prec).astype(np.int64)
    th = np.ceil(thr / prec).astype(np.int64)
    lo = np.maximum(target - th, 1)
    hi = target + th
    ok = (hi >= lo) & (hi < limit)
    return lo, hi, np.where(ok, (hi >> 6) - (lo >> 6) + 1, 0)


def result_digest(r):
    """SHA-256 of a fetched result's answers: status bytes, per-query counts
    and every query's candidate bytes (parallel.canonical_digest: a result
    object reused across batches keeps stale pad bytes between payload
    records, which are layout, not answers)."""
    from spectrseqtools_amd.parallel import canonical_digest

    return canonical_digest(r.status, r.count, r.offset, r.payload)


def build_workload(n_spectra, seed, dp):
    """SURVEY 8(d) config 3's queries for `n_spectra` synthetic spectra (see
    workload_from)."""
    from spectrseqtools_amd.synthetic import make_spectra

    batch = make_spectra(n_spectra, seed=seed)
    # a peak list comes sorted by mass (the rows step merges the breakages'
    # sorted streams); fragment_index = the position in this list
    obs = batch.observed[np.lexsort((batch.observed, batch.spectrum))]
    return workload_from(obs, batch.offsets, batch.seq_mass, dp)


def workload_from(obs, offsets, seq_mass, dp, intensity=None, intensity_cutoff=0.5e6, mass_cutoff=50000.0):
    """A7 on every peak x breakage weight (classify_fragments' form); A8 on
    every sliding-window pair of each spectrum's START and END side after the
    is_valid, intensity / mass and sequence-mass filters (the first
    filter_by_explanation round without singletons), produced on the host by
    the library's host-native sliding window (sst_su_diff_queries).  Rows are
    ordered per spectrum by SU mass, ties in breakage-major then peak order
    (the reference's stable sort), whatever the peaks' order."""
    from spectrseqtools_amd._native import su_diff_queries
    from spectrseqtools_amd.masses import build_breakage_dict
    from spectrseqtools_amd.producers import MAX_VARIANCE, classify_queries, max_nucleotide_weight

    tol, prec = dp.tolerance, dp.precision
    obs = np.ascontiguousarray(obs, dtype=np.float64)
    offsets = np.asarray(offsets, dtype=np.int64)
    n_spectra = len(offsets) - 1
    spectrum = np.repeat(np.arange(n_spectra), np.diff(offsets))
    brk = build_breakage_dict(555.1294, 455.1491)
    cq = classify_queries(obs, brk, prec, tol)
    valid = dp.device_table.is_valid(cq.su_mass, cq.threshold, tol, prec)  # setup pass: selects the window inputs
    if (valid < 0).any():
        raise RuntimeError("synthetic peak outside the DP table")
    n_brk = len(brk)
    P = len(obs)
    spec = np.tile(spectrum, n_brk)
    names = [v[0] for v in brk.values()]
    code = np.repeat(np.arange(n_brk), P)
    is_start = np.array(["START" in n for n in names])[code]
    is_end = np.array(["END" in n for n in names])[code]
    se_w = [k for k, v in brk.items() if "START_END" in v][0]
    # per spectrum by SU mass, ties in breakage-major order (classify_fragments' sort)
    order = np.lexsort((cq.su_mass, spec))
    inten = np.ones(P, bool) if intensity is None else np.asarray(intensity) > intensity_cutoff
    keep = (valid == 1) & np.tile(inten & (obs < mass_cutoff), n_brk)
    order = order[keep[order]]
    su, sp = cq.su_mass[order], spec[order]
    # filter_by_sequence_mass (fragment_classification.py:122-139)
    su_seq = (np.asarray(seq_mass) - se_w * prec)[sp]
    full = is_start[order] & is_end[order]
    ok = (su < su_seq + MAX_VARIANCE) & ((su > su_seq - MAX_VARIANCE) | ~full)
    rows = order[ok]
    flags = (is_start[rows].astype(np.uint8) | (is_end[rows].astype(np.uint8) << 1))
    offs = np.searchsorted(spec[rows], np.arange(n_spectra + 1))
    diffs, dthr, _, _ = su_diff_queries(cq.su_mass[rows], cq.observed[rows], flags, offs,
                                        max_nucleotide_weight(), tol)
    return {
        "peaks": P, "a7_mass": cq.su_mass, "a7_thr": cq.threshold, "a8_mass": diffs, "a8_thr": dthr,
        "spectra": n_spectra, "a7_valid": valid, "obs": obs,
        "shifts": np.array([w * prec for w in brk], dtype=np.float64),  # classify_fragments' su = obs - w * prec
        # the rows step's inputs: peak ranges per spectrum, SU sequence masses,
        # each breakage's sides (bit 0 START, bit 1 END)
        "peak_off": np.ascontiguousarray(offsets, dtype=np.int64),
        "su_seq": np.ascontiguousarray(np.asarray(seq_mass) - se_w * prec, dtype=np.float64),
        "sides": np.array([("START" in v[0]) | (("END" in v[0]) << 1) for v in brk.values()], dtype=np.uint8),
        "max_weight": max_nucleotide_weight(),
        "side_rows": int((flags & 1).astype(bool).sum() + (flags & 2).astype(bool).sum()),
    }


def cpu_baseline(wl_fn, dp, budget_s=10.0, single_budget_s=8.0):
    """The CPU oracle (literal C restatement of is_valid_mass /
    explain_mass_with_table) on a bounded sample of the same workload, with
    OpenMP over all the host threads the box grants, and single-threaded
    (per-core parity against BASELINE.md's reference-Python rates)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import _oracle as oracle

    ms = [m.mass for m in dp.masses]
    table = oracle.build_table(ms, max(ms) * 35, 32)
    alph = oracle.Alphabet(ms, [m.is_modification for m in dp.masses],
                           [round(dp.seq.max_len * m.modification_rate) for m in dp.masses])
    A = round(dp.seq.modification_rate * dp.seq.max_len)
    all_threads = oracle.LIB.ora_num_threads()

    lookups = []

    def leg(threads, budget, n_max):
        def run(wl):
            t0 = time.perf_counter()
            oracle.is_valid_batch(table, 32, wl["a7_mass"], wl["a7_thr"], dp.tolerance, nthreads=threads)
            _, _, lk = oracle.explain_batch(table, 32, alph, wl["a8_mass"], wl["a8_thr"], A, dp.tolerance,
                                            nthreads=threads)
            dt = time.perf_counter() - t0
            lookups.append(float(lk.mean()) if len(lk) else 0.0)
            return dt

        # size the sample from a small probe, then repeat it until ~budget s of
        # CPU work has been timed (the same sample each time: identical results)
        n = 100
        t = run(wl_fn(n))
        n = int(min(n_max, max(n, n * budget / 4 / max(t, 1e-3))))
        wl = wl_fn(n)
        reps, total = 0, 0.0
        while total < budget:
            total += run(wl)
            reps += 1
        return {"value": reps * wl["peaks"] / total, "unit": "peaks/s", "cores": threads, "kind": "port",
                "sample": f"{n} synthetic spectra ({wl['peaks']} peaks, {len(wl['a7_mass'])} A7 + "
                          f"{len(wl['a8_mass'])} A8 queries) x {reps} repetitions, oracle/sst_oracle.c with "
                          f"{threads} OpenMP thread{'s' if threads > 1 else ''}, {total:.1f} s"}

    out = leg(all_threads, budget_s, 20000)
    # table cells the reference DFS reads per A8 query (S of SURVEY 8(d)'s
    # byte model), counted by the literal restatement on the sample
    out["survey_lookups_per_a8_query"] = lookups[-1]
    out["single_core"] = leg(1, single_budget_s, 2000)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--spectra", type=int, default=10000, help="spectra per GPU")
    ap.add_argument("--seed", type=int, default=1000)
    ap.add_argument("--batches", type=int, default=3,
                    help="distinct config-3 batches cycled over the steps (>= 3: more inputs than the Infinity "
                         "Cache holds, so every step streams its inputs from HBM)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="torch.distributed backend for N>1 (nccl = RCCL over xGMI; gloo: rehearsal of the "
                         "multi-rank path, e.g. several ranks on one GPU with SST_DEVICE=0)")
    ap.add_argument("--no-gather", action="store_true",
                    help="N>1: keep every rank's results in its own HBM (default: each step's complete result of "
                         "every rank is gathered to rank 0 over RCCL, overlapped with the next step)")
    ap.add_argument("--event-every", type=int, default=0,
                    help="bracket every n-th launch of the roofline kernel with HIP events (0: about five "
                         "brackets over the timed steps, at least every 4th launch)")
    ap.add_argument("--a7-stream", type=int, default=0,
                    help="1: queue the A7 batch on a second HIP stream, concurrent with the A8 chain "
                         "(sst_ctx_set_stream); 0: both on the engine stream, one after the other")
    ap.add_argument("--fused-step", type=int, default=1,
                    help="1 (default): A7 and A8 in one launch (sst_step_device: the is_valid workgroups "
                         "behind the pair scan's grid, filling its tail); 0: two launches (then the roofline "
                         "kernel is the scan alone)")
    ap.add_argument("--dump-gathered", default=None,
                    help="test hook (tests/test_gpu_multirank.py): write the last step's gathered wire buffers "
                         "(rank 0) and every rank's inputs of that step into this directory")
    ap.add_argument("--a8-source", default="queries", choices=("rows", "queries"),
                    help="queries (default, the headline line): the A8 (mass, threshold) pairs are produced on "
                         "the host before timing (sst_step_device); rows: each step starts from the peaks -- A7, "
                         "the classification filters, the per-side SU order and the sliding window's pairs on "
                         "the device (sst_step_rows_device, the second config-3 line)")
    ap.add_argument("--no-validate", action="store_true",
                    help="diagnostic builds only: skip the result checks after the timed region")
    ap.add_argument("--no-events", action="store_true",
                    help="diagnostic: time the steps without the per-kernel HIP events (no roofline)")
    ap.add_argument("--workload", default="config3", choices=("config3", "config1"),
                    help="config3 (default): the headline A7 + A8 step; config1: whole-mass explain of random "
                         "canonical <=8-mers on the canonical table (the deferred DFS kernels, SURVEY 8(d))")
    ap.add_argument("--queries", type=int, default=200000, help="config1: queries per step per GPU")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per launch (profiles/), reported as roofline.traffic")
    args = ap.parse_args()
    if args.a7_stream:
        args.fused_step = 0  # A7 on its own stream: two launches

    import torch

    from spectrseqtools_amd import _native
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation
    from spectrseqtools_amd.parallel import (WIRE_HEADER, Gatherer, canonical_digest, decode_hits, dist_env,
                                             wire_unpack, wire_used_bytes)

    rank, world, local = dist_env()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    gpu = int(os.environ.get("SST_DEVICE", local))  # one GPU per rank (override: rehearsal on one card)
    torch.cuda.set_device(gpu)
    dev_t = torch.device("cuda", gpu)
    dist = None
    if world > 1:
        import torch.distributed as dist

        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev_t)
        else:
            dist.init_process_group("gloo")

    engine = _native.get_engine(gpu)
    if args.workload == "config1":
        return main_config1(args, engine, dist, rank, world, dev_t)
    seq = SequenceInformation(max_len=20, su_mass=6500.0, obs_mass=6500.0, modification_rate=0.5)
    dp = DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=MATCHING_THRESHOLD,
                                 precision=TOLERANCE, seq=seq, engine=engine)
    A = round(seq.modification_rate * seq.max_len)  # calculate_explanations (common.py:55)
    tdev = dp.device_table
    R = max(1, args.batches)
    # R distinct batches, cycled step by step: with R >= 3 their inputs (~180
    # MB each) and one step's outputs exceed the 256 MB Infinity Cache, so no
    # step's inputs are still on-die from their previous use
    wls = [build_workload(args.spectra, args.seed + 7919 * b + rank * 1_000_003, dp) for b in range(R)]
    wl = wls[0]
    n7s = [len(w["a7_mass"]) for w in wls]
    n8s = [len(w["a8_mass"]) for w in wls]
    rows_mode = args.a8_source == "rows"
    if rows_mode:
        args.fused_step = 1
    dev_in = []
    for w in wls:
        d = {"obs": torch.from_numpy(w["obs"]).to(dev_t), "P": len(w["obs"]), "shifts": w["shifts"],
             "n7": len(w["a7_mass"]), "n8": len(w["a8_mass"])}
        if rows_mode:
            d.update(poff=torch.from_numpy(w["peak_off"]).to(dev_t), su_seq=torch.from_numpy(w["su_seq"]).to(dev_t))
        else:
            d.update(a8m=torch.from_numpy(w["a8_mass"]).to(dev_t), a8t=torch.from_numpy(w["a8_thr"]).to(dev_t))
        dev_in.append(d)
    cap8 = int(max(n8s) * 1.05) + 1024  # the rows step's query capacity
    # two result sets used in turn: while step k runs on the GPU, the host
    # settles step k-1 (waits for its pass, reads its header, runs any routed
    # deferred windows or retries) -- the pipelined consumer loop of a serving
    # deployment; every step's result is complete and checked inside the
    # timed region
    outs7 = [torch.empty(max(n7s), dtype=torch.int8, device=dev_t) for _ in range(2)]
    torch.cuda.synchronize()
    ext = torch.cuda.ExternalStream(engine.stream, device=dev_t)

    results = [None, None]
    batch_of = [None, None]  # which batch the result set last computed
    gath = Gatherer(dist, dev_t) if (dist and not args.no_gather) else None
    side = torch.cuda.Stream(device=dev_t) if args.a7_stream else None
    settled = {"n": 0, "sent": 0}
    # N>1 delivery: step j's result goes to rank 0 while step j+1 computes.
    # pass_done[j&1]: step j's kernels (engine stream); the pack stream packs
    # it (sst_wire_pack, one kernel) into wire buffer j&1 once the gather of
    # step j-2 has read that buffer (gathered[j&1]); copied[j&1]: that pack,
    # which the engine stream waits for before step j+2 reuses the same
    # result buffers; the comm stream gathers the packed buffer (sst_wire_pack
    # itself waits for any work settling queued on the engine stream)
    comm = torch.cuda.Stream(device=dev_t) if gath is not None else None
    packer = torch.cuda.Stream(device=dev_t) if gath is not None else None
    pass_done = [torch.cuda.Event(), torch.cuda.Event()]
    copied = [None, None]
    gathered = [None, None]
    wbuf = [None, None]
    expect = [None] * R  # per batch: (n_hits, payload bytes) of its reference pass
    wire_sizes = []  # per delivered step: every rank's agreed wire bytes
    hdr_host = None

    def settle(r, b):
        nh, nb = r.settle()
        if (nh, nb) != expect[b]:
            raise RuntimeError(f"step result differs from the reference pass: {nh} hits / {nb} B vs {expect[b]}")
        settled["n"] += 1

    def send(j):
        """Step j's complete result of this rank -> rank 0 in the wire format
        v5 (sst_wire_pack, include/sst.h: 1-bit is_valid codes and hit flags,
        per pair-path hit its first pair-list entry in w bits and a 3-bit
        count, which rank 0 expands from its own copy of the table's pair
        list; records + payload of the deferred paths' hits; a list of the
        rare rest)."""
        r, b = results[j & 1], batch_of[j & 1]
        settle(r, b)  # host: the pass's header (routed windows / retries handled)
        packer.wait_event(pass_done[j & 1])
        if side is not None:
            packer.wait_stream(side)
        if gathered[j & 1] is not None:
            packer.wait_event(gathered[j & 1])
        engine.set_stream(packer.cuda_stream)
        r.wire_pack(outs7[j & 1].data_ptr(), n7s[b], wbuf[j & 1].data_ptr(), wbuf[j & 1].numel())
        engine.set_stream(None)
        # this step's wire size (the packed header: fixed part + its list),
        # agreed with one all_gather of an int64 per rank inside the timed loop
        # (RCCL has no gatherv: the gather then moves the largest rank's size);
        # the event follows the header's copy, so the host reads this step's
        # header, not the previous one's
        with torch.cuda.stream(packer):
            hdr_host.copy_(wbuf[j & 1][:WIRE_HEADER], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(packer)
        copied[j & 1] = ev
        ev.synchronize()
        sizes = gath.agree(wire_used_bytes(hdr_host.numpy()), capacity=wbuf[j & 1].numel())
        wire_sizes.append(sizes)
        with torch.cuda.stream(comm):
            comm.wait_event(ev)
            gath.gather(wbuf[j & 1])
            ev2 = torch.cuda.Event()
            ev2.record(comm)
            gathered[j & 1] = ev2
        settled["sent"] += 1

    def launch(b, out7, reuse):
        d = dev_in[b]
        if rows_mode:  # everything from the peaks on the device (sst_step_rows_device)
            w = wls[b]
            return tdev.step_rows_device(d["obs"].data_ptr(), d["poff"].data_ptr(), len(w["peak_off"]) - 1, d["P"],
                                         d["su_seq"].data_ptr(), d["shifts"], w["sides"], out7.data_ptr(),
                                         w["max_weight"], dp.tolerance, dp.precision, A, cap8, reuse=reuse)
        if args.fused_step:  # A7 and A8 in one launch (sst_step_device)
            return tdev.step_device(d["obs"].data_ptr(), d["P"], d["shifts"], out7.data_ptr(), d["a8m"].data_ptr(),
                                    d["a8t"].data_ptr(), d["n8"], dp.tolerance, dp.precision, A, reuse=reuse)
        res = reuse
        if args.a7_stream != 2:
            res = tdev.explain_device(d["a8m"].data_ptr(), d["a8t"].data_ptr(), d["n8"], dp.tolerance, dp.precision,
                                      A, reuse=res)
        if side is not None:
            engine.set_stream(side.cuda_stream)
        tdev.is_valid_peaks_device(d["obs"].data_ptr(), d["P"], d["shifts"], dp.tolerance, dp.precision,
                                   out7.data_ptr())
        if side is not None:
            engine.set_stream(None)
        if args.a7_stream == 2:
            res = tdev.explain_device(d["a8m"].data_ptr(), d["a8t"].data_ptr(), d["n8"], dp.tolerance, dp.precision,
                                      A, reuse=res)
        return res

    def step(k):
        cur = k & 1
        if copied[cur] is not None:  # step k-2's wire copy read these buffers
            ext.wait_event(copied[cur])
        b = k % R
        results[cur] = launch(b, outs7[cur], results[cur])
        batch_of[cur] = b
        if gath is not None:
            pass_done[cur].record(ext)
        if k > 0:  # the previous step's result, while this one runs: settled, and delivered for N>1
            if gath is not None:
                send(k - 1)
            else:
                settle(results[cur ^ 1], batch_of[cur ^ 1])

    def drain(k_last):
        if results[k_last & 1] is not None:
            if gath is not None:
                send(k_last)
            else:
                settle(results[k_last & 1], batch_of[k_last & 1])

    # untimed reference pass of every batch (the same entry point as the timed
    # steps: the dense layout follows the scan's grid, which the fused step
    # sizes for itself): sizes for the gather and each batch's expected result
    refs = []
    for b in range(R):
        rr = launch(b, outs7[0], None)
        rr.fetch_device()
        engine.synchronize()
        a7_ok = np.array_equal(outs7[0][:n7s[b]].cpu().numpy(), wls[b]["a7_valid"])
        if not a7_ok:
            raise RuntimeError(f"batch {b}: is_valid bytes differ from the setup pass")
        expect[b] = rr.settle()
        if rows_mode:
            # the device producers must issue exactly the host producers' queries:
            # the same answers as the explain pass over the host-built (mass,
            # threshold) pairs (which tests/test_gpu_fullsize.py checks against the oracle)
            if rr.n != n8s[b]:
                raise RuntimeError(f"batch {b}: the rows step issued {rr.n} queries, the host producers {n8s[b]}")
            dm_ = torch.from_numpy(wls[b]["a8_mass"]).to(dev_t)
            dt_ = torch.from_numpy(wls[b]["a8_thr"]).to(dev_t)
            torch.cuda.synchronize()
            hq = tdev.explain_device(dm_.data_ptr(), dt_.data_ptr(), n8s[b], dp.tolerance, dp.precision, A)
            hq.fetch_device()
            if canonical_digest(hq.status, hq.count, hq.offset, hq.payload) != \
                    canonical_digest(rr.status, rr.count, rr.offset, rr.payload):
                raise RuntimeError(f"batch {b}: the rows step's answers differ from the host-produced queries'")
            hq.close()
            del dm_, dt_
        refs.append({"digest": result_digest(rr), "stats": rr.stats(), "status": rr.status.copy(),
                     "canon": canonical_digest(rr.status, rr.count, rr.offset, rr.payload) if gath is not None
                     else None, "n_hits": expect[b][0],
                     "pair_hits": rr.pair_hits_device()[1] if args.fused_step else 0,
                     "cap": None})
        if gath is not None:
            # the wire buffer's capacity: the fixed part (host-known from the
            # result's sizes) + a list slot for every query and hit (the bound
            # sst_wire_pack accepts); each timed step agrees its used size
            fixed = rr.wire_pack(outs7[0].data_ptr(), n7s[b])
            refs[b]["cap"] = fixed + 8 * (n7s[b] + n8s[b] + expect[b][0])
        if b == int(np.argmax(n8s)):
            results[0] = rr  # the result sets get the capacity of the largest batch
        else:
            rr.close()
    results[1] = launch(int(np.argmax(n8s)), outs7[1], None)
    results[1].settle()
    if gath is not None:
        precs = tdev.pair_records()
        cap_w = max(rf["cap"] for rf in refs)
        wbuf = [torch.empty(cap_w, dtype=torch.uint8, device=dev_t) for _ in range(2)]
        hdr_host = torch.empty(WIRE_HEADER, dtype=torch.uint8).pin_memory()
        torch.cuda.synchronize()
    for k in range(args.warmup):
        step(k)
    drain(args.warmup - 1)
    torch.cuda.synchronize()
    engine.synchronize()

    # events bracket only the kernel the roofline reports, and only every
    # --event-every-th launch of it: each bracket costs two event records
    # (~6 us each on the stream), which would otherwise inflate every step;
    # the other kernels' times are in the rocprofv3 summaries under profiles/
    every = args.event_every if args.event_every > 0 else max(4, args.steps // 5)
    engine.profile(not args.no_events, kernels=(_native.K_EXPLAIN_SCAN, _native.K_RESULT_PACK), every=every)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    settled["n"] = settled["sent"] = 0
    wire_sizes.clear()  # the timed steps' agreed sizes
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    drain(args.steps - 1)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    prof = engine.profile_read() if not args.no_events else {}
    engine.profile(False)
    timed_batches = [k % R for k in range(args.steps)]
    peaks_mine = sum(dev_in[b]["P"] for b in timed_batches) / args.steps  # peaks per step (mean over the cycle)
    n7_mine = sum(n7s[b] for b in timed_batches) / args.steps
    n8_mine = sum(n8s[b] for b in timed_batches) / args.steps
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev_t)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        pk = torch.tensor([peaks_mine, n7_mine, n8_mine], dtype=torch.float64, device=dev_t)
        dist.all_reduce(pk)
        peaks_all, n7_all, n8_all = (float(x) for x in pk.tolist())
    else:
        peaks_all, n7_all, n8_all = peaks_mine, n7_mine, n8_mine

    # every timed step was settled in the loop; the last two steps' results
    # must equal their batch's reference pass bit for bit (status bytes, hit
    # list, payload), and A7 the setup pass
    if settled["n"] != args.steps and not args.no_validate:
        raise RuntimeError(f"{settled['n']} of {args.steps} steps settled")
    if gath is not None and settled["sent"] != args.steps:
        raise RuntimeError(f"{settled['sent']} of {args.steps} steps delivered to rank 0")
    for r, b in zip(results, batch_of):
        if r is not None:
            r.fetch_device()
            if result_digest(r) != refs[b]["digest"] and not args.no_validate:
                raise RuntimeError(f"a timed step's result (batch {b}) differs from the reference pass")
    engine.synchronize()
    for o, b in zip(outs7, batch_of):
        assert np.array_equal(o[:n7s[b]].cpu().numpy(), wls[b]["a7_valid"]), \
            "is_valid results changed between setup and timed runs"
    if gath is not None:
        # rank 0 decodes what it received from every rank in the last step:
        # each rank's result digest must match (and its A7 bytes)
        last_b = (args.steps - 1) % R
        mine = torch.tensor(np.frombuffer(bytes.fromhex(refs[last_b]["canon"]), dtype=np.uint8).copy(), device=dev_t)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        if rank == 0 and not args.no_validate:
            for r_, (buf, want) in enumerate(zip(gath.last, allr)):
                v_, st_, hits_, pay_ = wire_unpack(buf.cpu().numpy(), precs)
                cnt_, off_ = decode_hits(st_, hits_)
                if bytes.fromhex(canonical_digest(st_, cnt_, off_, pay_)) != bytes(want.cpu().numpy()):
                    raise RuntimeError(f"rank {r_}'s gathered result does not decode to its own result")
    if args.dump_gathered:
        os.makedirs(args.dump_gathered, exist_ok=True)
        last_b = (args.steps - 1) % R
        w_ = wls[last_b]
        np.savez(os.path.join(args.dump_gathered, f"inputs_rank{rank}.npz"), a7_mass=w_["a7_mass"],
                 a7_thr=w_["a7_thr"], a8_mass=w_["a8_mass"], a8_thr=w_["a8_thr"], obs=w_["obs"],
                 shifts=w_["shifts"], max_mods=np.int64(A))
        if rank == 0 and gath is not None:
            np.savez(os.path.join(args.dump_gathered, "gathered.npz"), precs=precs,
                     **{f"rank{r_}": b_.cpu().numpy() for r_, b_ in enumerate(gath.last)})
    for rf in refs:
        st = rf["status"]
        if (st < -2).any() and not args.no_validate:
            raise RuntimeError(f"internal statuses in results: {np.unique(st[st < -2])}")

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    limit = tdev.n_cols * tdev.compression
    w_min = min(m.mass for m in dp.masses if m.mass > 0)
    # the device path's pair scan packs its own result (fused: no k_result_pack
    # launch): its algorithmic bytes are then the inputs, the status bytes and
    # the dense result (16-B hit record + candidate bytes per query with
    # candidates, 2-B pair-list ref per pair hit); the wave-local records and
    # payload it re-reads are not
    fused = _native.K_RESULT_PACK not in prof

    def batch_bytes(b):
        """Algorithmic bytes per launch of each kernel for batch b (DESIGN.md
        section 4), and the part of them that is L2-resident bitset words."""
        w_, rf = wls[b], refs[b]
        stats, st = rf["stats"], rf["status"]
        _, _, w7 = windows(w_["a7_mass"], w_["a7_thr"], dp.precision, limit)
        _, hi8, w8 = windows(w_["a8_mass"], w_["a8_thr"], dp.precision, limit)
        # queries the scan answers from the LDS pair list: non-empty windows
        # below 3 * w_min (budgets never bind there for this config; checked
        # against the engine's own counter)
        pair = (w8 > 0) & (hi8 < 3 * w_min)
        n_pair, n_work, nodes = int(stats[6]), int(stats[0]), int(stats[4])
        if int(pair.sum()) != n_pair and not args.no_validate:
            raise RuntimeError(f"pair-path partition {int(pair.sum())} != engine counter {n_pair}")
        some = (st == 2) | (st == -2)
        n7, n8, P = n7s[b], n8s[b], dev_in[b]["P"]
        # algorithmic HBM bytes per launch; the LDS pair list is on-chip and
        # the 2.8 MB is_valid bitset L2-resident, both counted at 8 B per
        # bitset word touched (bitset_l2 below: that part):
        #   k_is_valid:       the peak's mass (8, once for its 4 windows) + result (1 per window) + the
        #                     window's bitset words (8 each)
        #   k_explain_scan:   mass+thr (16) + status (1) of every query it resolves;
        #                     pair path: dense hit record + payload of each SOME / OVERFLOW;
        #                     other windows: bitset words (8 each); 16 B worklist item per queued query
        #   k_explain_expand: worklist item (16) + status/count/offset (17) + 16 B per
        #                     index record expanded + payload (its bitset words are not counted)
        #   k_result_pack:    8-B hit record in + 16-B dense record out per hit, the
        #                     candidate payload read and written once (pad bytes not counted)
        n_some_pair = int(((st == 2) & pair).sum())
        cand_bytes = int(stats[7]) - 2 * n_some_pair + int(stats[5])
        bits7, bits8 = 8 * int(w7.sum()), 8 * int(w8[~pair].sum())
        bk = {
            "k_is_valid": float(8 * P + n7 + bits7),
            # (stats[7] counts the 2 pad bytes per SOME query of the dword record stores: not algorithmic)
            "k_explain_scan": float(n8 * 16 + (n8 - n_work) +
                                    (16 * rf["n_hits"] + cand_bytes + 2 * rf["pair_hits"] if fused else
                                     8 * int((some & pair).sum()) + int(stats[7]) - 2 * n_some_pair)
                                    + bits8 + 16 * n_work),
            "k_result_pack": float(24 * rf["n_hits"] + 2 * cand_bytes),
            "k_explain_expand": float(n_work * (16 + 17) + 16 * nodes + int(stats[5])),
        }
        l2 = {"k_is_valid": float(bits7), "k_explain_scan": float(bits8)}
        if rows_mode:
            # the step from the peaks: each peak (8) read once, its A7 codes and
            # bitset words, every side row written to scratch and read back
            # (16 + 16: the round-3 model, kept so that fractions compare
            # across rounds -- the kernels now keep the rows in LDS and move
            # the compact answer scratch instead), then
            # per query its status byte and per hit the dense record (16), the
            # pair-list ref (2) and the candidate bytes; the queries themselves
            # never touch HBM
            bk["k_explain_scan"] = float(8 * P + n7 + bits7 + 32 * w_["side_rows"] + n8 +
                                         18 * rf["n_hits"] + cand_bytes)
            l2["k_explain_scan"] = float(bits7)
        elif args.fused_step:  # the scan's launch also ran A7 (k_step): its bytes are both predicates'
            bk["k_explain_scan"] += bk["k_is_valid"]
            l2["k_explain_scan"] += l2["k_is_valid"]
        # SURVEY 8(d)'s literal per-query model: 16 B in + 8 B per window word
        # for every A7 and A8 query, 16 B out and the payload per A8 query, and
        # 8 B per table cell the reference DFS looks up (S, from the oracle on
        # the CPU sample: cpu_baseline)
        lit = float(16 * n7 + 8 * int(w7.sum()) + 32 * n8 + 8 * int(w8.sum()) + cand_bytes)
        return bk, l2, lit, n8

    per = [batch_bytes(b) for b in range(R)]
    bytes_k = {k: sum(per[b][0][k] for b in timed_batches) / args.steps for k in per[0][0]}
    l2_k = {k: sum(per[b][1][k] for b in timed_batches) / args.steps for k in per[0][1]}
    lit_bytes = sum(per[b][2] for b in timed_batches) / args.steps
    kern = {}
    for kid, (ms, cnt) in prof.items():
        name = _native.KERNEL_NAMES[kid]
        kern[name] = {"avg_us": 1e3 * ms / cnt, "launches": cnt}
        if name in bytes_k:
            kern[name]["algorithmic_bytes"] = bytes_k[name]
            kern[name]["achieved_GBps"] = bytes_k[name] / (1e3 * ms / cnt * 1e-6) / 1e9
    dom = max(bytes_k, key=lambda k: kern.get(k, {"avg_us": 0.0})["avg_us"])
    dbytes, dus = bytes_k[dom], kern.get(dom, {"avg_us": float("nan")})["avg_us"]
    achieved = dbytes / (dus * 1e-6) / 1e9
    hbm_only = (dbytes - l2_k.get(dom, 0.0)) / (dus * 1e-6) / 1e9
    traffic, traffic_src = None, None
    tkey = ("k_rows" if rows_mode else "k_step" if args.fused_step and dom == "k_explain_scan" else dom) + \
        (f"_rot{R}" if R > 1 else "")
    if args.spectra == 10000 and args.seed == 1000:  # the workload the PMC passes in profiles/ measured
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            traffic = tj.get(tkey)
            traffic_src = tj.get("_source", {}).get(tkey)
        except (OSError, ValueError):
            pass
    st = refs[timed_batches[-1]]["status"]
    stats = refs[timed_batches[-1]]["stats"]
    res = results[(args.steps - 1) & 1]
    some = (st == 2) | (st == -2)
    n_hits0 = refs[timed_batches[-1]]["n_hits"]
    ws_arr = np.asarray(wire_sizes, dtype=np.int64) if wire_sizes else None  # [delivered steps, ranks]
    ms_step = 1e3 * elapsed / args.steps
    value = peaks_all / (elapsed / args.steps)

    cpu = None
    lit_frac = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(lambda n: build_workload(n, args.seed, dp), dp)
        if dom == "k_explain_scan":
            lit_bytes += 8.0 * cpu["survey_lookups_per_a8_query"] * sum(n8s[b] for b in timed_batches) / args.steps
            lit_frac = lit_bytes / (dus * 1e-6) / 1e9 / HBM_PEAK_GBPS

    line = {
        "metric": METRIC,
        "value": value,
        "unit": "peaks/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic",
        "config": {
            "workload": "config3: synthetic spectra (SURVEY 8(d)), full 104-mass/105-row alphabet, <=20-mer, "
                        "A7 (4 breakages/peak) + A8 (sliding-window differences) per step",
            "a8_source": ("rows: A7, classification filters, per-side SU order and sliding-window pairs formed on "
                          "the device from the peaks inside each step (sst_step_rows_device)" if rows_mode else
                          "queries: A8 (mass, threshold) pairs produced on the host before timing"),
            "spectra_per_gpu": args.spectra,
            "batches": (f"{R} distinct batches of {args.spectra} spectra (seeds {args.seed} + 7919 b), cycled "
                        f"step by step, {sum(w['obs'].nbytes + w['a8_mass'].nbytes + w['a8_thr'].nbytes for w in wls) / 1e6:.0f} MB "
                        f"of inputs: no step's inputs are still in the 256 MB Infinity Cache" if R > 1 else "1 batch"),
            "peaks": peaks_all,
            "a7_queries": n7_all,
            "a8_queries": n8_all,
            "max_len": seq.max_len,
            "max_modifications": A,
            "a7_stream": ("side stream, concurrent with the A8 chain" if args.a7_stream else "engine stream"),
            "parallelism": ((f"spectra sharded over {world} GPUs; every step's complete result of every rank "
                             f"gathered to rank 0 ({'RCCL' if args.backend == 'nccl' else 'gloo'}, wire format "
                             f"v5, sst_wire_pack), overlapped with the next step"
                             if gath is not None else f"spectra sharded over {world} GPUs, results kept per rank")
                            if world > 1 else "1 GPU"),
            "wire_bytes_per_rank_step": ({"mean": ws_arr.mean(axis=0).tolist(), "max": ws_arr.max(axis=0).tolist(),
                                          "steps": int(len(ws_arr)),
                                          "agreed": "per timed step: all_gather of each rank's packed size"}
                                         if ws_arr is not None else None),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": ("k_rows_count_w + k_rows_emit_w (+ k_rows_count / k_rows_emit for spectra over 160 peaks: "
                       "the step from the peaks)" if rows_mode else
                       "k_step (k_is_valid_peaks + k_explain_scan in one launch)" if args.fused_step and
                       dom == "k_explain_scan" else dom),
            "achieved": achieved,
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "algorithmic_bytes_per_launch": dbytes,
            # the same minus the bitset words (8 B per word touched), which
            # the 2.8 MB L2-resident bitset serves: bytes that cross HBM
            "frac_hbm_resident": hbm_only / HBM_PEAK_GBPS,
            "hbm_resident_bytes_per_launch": dbytes - l2_k.get(dom, 0.0),
            # SURVEY 8(d)'s literal model (16 B in + 8 B per window word per
            # query, + 8 B per table cell the reference DFS reads, S from the
            # oracle on the CPU sample); > 1 is possible: the LDS pair list
            # answers windows without the table reads the model charges
            "frac_survey_literal": lit_frac,
            "survey_literal_bytes_per_launch": lit_bytes if lit_frac is not None else None,
            "avg_launch_us": dus,
            "event_timed_launches": kern.get(dom, {}).get("launches", 0),  # every --event-every-th step
        },
        "kernels": kern,
        "engine_stats": {"pair": int(stats[6]), "shallow": int(stats[0]), "deep": int(stats[1]), "exact": int(stats[2]),
                         "nomemo": int(stats[3]), "index_loads": int(stats[4]),
                         "candidates": int(res.count[some].sum()), "payload_bytes": int(stats[5] + stats[7]),
                         "hits": n_hits0, "dense_payload_bytes": int(len(res.payload))},
        "step": ("k_rows_count_w + k_rows_count + k_rows_emit_w + k_rows_emit (from the peaks)" if rows_mode else
                 "k_is_valid + k_explain_scan (packing its own dense result)" if fused else
                 "k_is_valid + k_explain_scan + k_result_pack") +
                " per step: status bytes, dense hit list and dense payload of every query (the complete "
                "result); the host settles step k-1 while step k runs",
        "queries_per_s": (n7_all + n8_all) / (elapsed / args.steps),
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


CONFIG1_TEST_SEQ = ["A", "AA", "GG", "CC", "UU", "CUAG", "CCUAGG"]  # tests/test_explain_masses.py:34-42
CONFIG1_PPM = (10e-6, 5e-6, 2e-6)  # :51


def config1_queries(n, seed):
    """the reference test's 7 masses x 3 tolerances, then
    random canonical 1..8-mers (masses as get_seq_weight, test_explain_masses.py:
    16-31: round(len * PHOSPHATE_LINK_MASS + sum of monoisotopic masses, 5)),
    tolerance cycling over the test's three; budget round(0.5 * len) (:92)."""
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, PHOSPHATE_LINK_MASS

    mono = dict(zip(EXPLANATION_MASSES.get_column("nucleoside").to_list(),
                    EXPLANATION_MASSES.get_column("monoisotopic_mass").to_list()))
    seqs = [s for s in CONFIG1_TEST_SEQ for _ in CONFIG1_PPM]
    ppm = [p for _ in CONFIG1_TEST_SEQ for p in CONFIG1_PPM]
    rng = np.random.default_rng(seed)
    lens = rng.integers(1, 9, max(0, n - len(seqs)))
    letters = np.array(list("ACGU"))
    seqs += ["".join(letters[rng.integers(0, 4, L)]) for L in lens]
    ppm += [CONFIG1_PPM[k % 3] for k in range(len(lens))]
    mass = np.array([round(len(q) * PHOSPHATE_LINK_MASS + sum(mono[c] for c in q), 5) for q in seqs])
    return mass, np.asarray(ppm) * mass, np.array([round(0.5 * len(q)) for q in seqs], dtype=np.int64)


def main_config1(args, engine, dist, rank, world, dev_t):
    """Config 1 step: one explain pass over whole canonical masses (windows of
    up to 8 items: the scan routes them to the deferred DFS kernel), settled
    inside the step (deferred launch + result pack), with inputs in HBM."""
    import torch

    from spectrseqtools_amd import _native
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, TOLERANCE, UNMODIFIED_BASES

    seq = SequenceInformation(max_len=8, su_mass=0.0, obs_mass=0.0, modification_rate=0.5)
    dp = DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=10e-6, precision=TOLERANCE,
                                 seq=seq, engine=engine)
    dp.adapt_individual_modification_rates_by_alphabet_reduction(set(UNMODIFIED_BASES))  # 5 x 377 397 table
    tdev = dp.device_table
    mass, thr, mods = config1_queries(args.queries, args.seed + rank * 1_000_003)
    n = len(mass)
    dm = torch.from_numpy(mass).to(dev_t)
    dt = torch.from_numpy(thr).to(dev_t)
    dmods = torch.from_numpy(mods).to(dev_t)
    torch.cuda.synchronize()

    def step(res):
        res = tdev.explain_device(dm.data_ptr(), dt.data_ptr(), n, dp.tolerance, dp.precision, 0,
                                  d_mods=dmods.data_ptr(), reuse=res)
        res.settle()  # routed windows: the deferred DFS launch and the result pack, inside the step
        return res

    res = step(None)
    res.fetch_device()
    ref_st, ref_cnt = res.status.copy(), res.count.copy()
    for k in range(args.warmup):
        res = step(res)
    engine.synchronize()
    engine.profile(not args.no_events, kernels=(_native.K_EXPLAIN_SCAN, _native.K_EXPLAIN_DEEP,
                                                 _native.K_RESULT_PACK), every=1)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        res = step(res)
    engine.synchronize()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    prof = engine.profile_read() if not args.no_events else {}
    engine.profile(False)
    res.fetch_device()
    if not (np.array_equal(res.status, ref_st) and np.array_equal(res.count, ref_cnt)):
        raise RuntimeError("a timed config-1 step's result differs from the reference pass")
    # parity sample against the CPU oracle (the checker, outside the timed region)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import _oracle as oracle

    ms = [m.mass for m in dp.masses]
    table = oracle.build_table(ms, max(ms) * 35, 32)
    alph = oracle.Alphabet(ms, [m.is_modification for m in dp.masses],
                           [round(seq.max_len * m.modification_rate) for m in dp.masses])
    sample = np.unique(np.concatenate([np.arange(min(n, 21)), np.random.default_rng(3).integers(0, n, 400)]))
    for i in sample:
        st, sols, n_empty, _ = oracle.explain_table(table, 32, alph, mass[i], thr[i], dp.tolerance, int(mods[i]))
        if sorted(res.candidates(i)) != sorted(sols) and not args.no_validate:
            raise RuntimeError(f"config-1 query {i} differs from the oracle")
    stats = res.stats()
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev_t)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    n_def = int(stats[1] + stats[2] + stats[3])
    nodes = int(stats[4])
    some = res.status == _native.SST_SOME
    # algorithmic bytes of the deferred launch: each routed query's window
    # bounds (16) and status byte, 16 B per index record the DFS loads, its
    # payload and 16-B hit record per query with candidates
    limit = tdev.n_cols * tdev.compression
    _, hi, w = windows(mass, thr, dp.precision, limit)
    pair = (w > 0) & (hi < 3 * min(m.mass for m in dp.masses if m.mass > 0))  # answered by the scan
    if int(pair.sum()) != int(stats[6]):
        raise RuntimeError(f"pair-path partition {int(pair.sum())} != engine counter {int(stats[6])}")
    n_hit_def = int((some & ~pair).sum())
    bytes_def = float(n_def * 17 + 16 * nodes + int(stats[5]) + 16 * n_hit_def)
    traffic, traffic_src = None, None  # PMC-derived HBM bytes per launch (tools/pmc_c1.sh -> profiles/traffic.json)
    try:
        with open(args.traffic_json) as f:
            tj = json.load(f)
        traffic = tj.get("k_explain_deferred_c1")
        traffic_src = tj.get("_source", {}).get("k_explain_deferred_c1")
    except (OSError, ValueError):
        pass
    kern = {}
    for kid, (ms_, cnt) in prof.items():
        kern[_native.KERNEL_NAMES[kid]] = {"avg_us": 1e3 * ms_ / cnt, "launches": cnt}
    dus = kern.get("k_explain_deferred", {"avg_us": float("nan")})["avg_us"]
    achieved = bytes_def / (dus * 1e-6) / 1e9
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        sub = np.arange(min(n, 20000))
        out = {}
        for threads in (oracle.LIB.ora_num_threads(), 1):
            k = len(sub) if threads > 1 else min(len(sub), 4000)
            t1 = time.perf_counter()
            oracle.explain_batch(table, 32, alph, mass[:k], thr[:k], mods[:k], dp.tolerance, nthreads=threads)
            dt_ = time.perf_counter() - t1
            out[threads] = {"value": k / dt_, "unit": "peaks/s", "cores": threads, "kind": "port",
                            "sample": f"first {k} config-1 queries, oracle/sst_oracle.c, {threads} thread(s), "
                                      f"{dt_:.1f} s"}
        cpu = out[max(out)]
        cpu["single_core"] = out[1]
        cpu["reference_python_single_core"] = {"value": 904.0, "unit": "peaks/s", "source": "BASELINE.md config 1"}
    print(json.dumps({
        "metric": METRIC, "value": n * world / (elapsed / args.steps), "unit": "peaks/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
        "config": {"workload": "config1: whole masses of random canonical 1..8-mers (+ the reference test's 7 x 3), "
                               "canonical 5-row table, budget round(0.5 len) per query", "queries_per_gpu": n},
        "roofline": {"bound": "hbm", "kernel": "k_explain_deferred", "achieved": achieved, "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
                     "traffic_source": traffic_src, "algorithmic_bytes_per_launch": bytes_def, "avg_launch_us": dus,
                     "random_line_fetches_per_launch": nodes,
                     "random_line_rate_note": "the DFS fetches one index record per node: "
                                              f"{nodes / (dus * 1e-6) / 1e9:.1f} G fetches/s against the ~50 G/s "
                                              "a dependent random chase reaches (profiles/r3_chase_probe.txt)"},
        "kernels": kern,
        "engine_stats": {"pair": int(stats[6]), "deep": int(stats[1]), "exact": int(stats[2]),
                         "nomemo": int(stats[3]), "index_loads": nodes, "candidates": int(res.count[some].sum()),
                         "payload_bytes": int(stats[5] + stats[7])},
        "step": "explain pass (scan routes deep windows) + settle: deferred DFS launch + result pack",
        "cpu_baseline": cpu,
    }), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
