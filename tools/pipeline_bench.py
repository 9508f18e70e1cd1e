#!/usr/bin/env python3
"""Config-5 harness: the prediction pipeline's explanation
stages over many synthetic spectra, batched on the GPU engine
(spectrseqtools_amd/pipeline.py):

  stage 1  classify_fragments      is_valid (peaks x 4 breakages) + is_singleton
  stage 2  first filter_by_explanation round: sliding-window SU differences of
           both sides + singleton masses -> explain
  stage 3  skeleton bins: each side's bins, first bin's whole masses and every
           later bin against its predecessor -> explain (deep windows: the
           deferred DFS kernels)

One process per GPU (torch.distributed.run for N > 1, spectra sharded by
rank, no collective in the data path); every stage is timed over all of this
rank's spectra with barriers around it, max over ranks.  The full alphabet's
table serves every spectrum (the reference's per-spectrum alphabet reduction
is a table rebuild, timed separately: `reduction_rebuild_ms`); each explain
call covers the spectra of one max_len (their row caps and budget).  Results
come back to the host (status, counts, payload: PCIe included).  The
reference Python cannot run on the GPU box; `reference_estimate_s` prices the
same query counts at its measured single-core rates (is_valid
70 k/s, sliding-window explain 3.6-4.5 k/s).

Usage: python tools/pipeline_bench.py [--spectra 100000] [--seed 7]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spectra", type=int, default=100000, help="spectra per GPU")
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--cap", type=int, default=1 << 16, help="candidate cap per query (OVERFLOW beyond)")
    args = ap.parse_args()

    import torch

    from spectrseqtools_amd import _native, pipeline
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE, build_breakage_dict
    from spectrseqtools_amd.parallel import dist_env
    from spectrseqtools_amd.synthetic import make_spectra

    rank, world, local = dist_env()
    gpu = int(os.environ.get("SST_DEVICE", local))
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(gpu)
        dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
    engine = _native.get_engine(gpu)

    def barrier():
        if dist:
            dist.barrier()

    def tmax(x):
        if not dist:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=torch.device("cuda", gpu))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    t0 = time.perf_counter()
    batch = make_spectra(args.spectra, seed=args.seed + 1_000_003 * rank)
    gen_s = time.perf_counter() - t0
    bd = build_breakage_dict(555.1294, 455.1491)
    w_full = [k for k, v in bd.items() if "START_END" in v][0]
    su_seq = batch.seq_mass - w_full * TOLERANCE  # cli.py:149-156
    seq0 = SequenceInformation(max_len=20, su_mass=float(su_seq[0]), obs_mass=float(batch.seq_mass[0]),
                               modification_rate=0.5)
    dp = DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=MATCHING_THRESHOLD,
                                 precision=TOLERANCE, seq=seq0, engine=engine)
    min_int = min(m.mass for m in dp.masses[1:])
    max_len = pipeline.max_len_of(su_seq, TOLERANCE, min_int)  # cli.py:158-170

    def explain_grouped(q):
        """One engine call per max_len group; returns statuses, counts, timing.
        Groups from the spectra's max_len (one radix sort of the queries' small
        group ids, not one full scan of the queries per group)."""
        st = np.zeros(len(q.diff), np.int8)
        cnt = np.zeros(len(q.diff), np.uint64)
        lens_u, spec_gid = np.unique(max_len, return_inverse=True)
        if len(q.spec) and (np.diff(q.spec) >= 0).all():  # spectrum-major: a group is its spectra's ranges
            qoff = np.searchsorted(q.spec, np.arange(len(max_len) + 1))
            groups = []
            for gi in range(len(lens_u)):
                sp = np.flatnonzero(spec_gid == gi)
                ln = qoff[sp + 1] - qoff[sp]
                groups.append(np.repeat(qoff[sp] - (np.cumsum(ln) - ln), ln) + np.arange(int(ln.sum())))
        else:
            gid = spec_gid.astype(np.uint16)[q.spec]
            order = np.argsort(gid, kind="stable")  # radix sort (16-bit keys)
            cuts = np.concatenate([[0], np.cumsum(np.bincount(gid, minlength=len(lens_u)))])
            groups = [order[cuts[gi]:cuts[gi + 1]] for gi in range(len(lens_u))]
        calls = 0
        for gi, L in enumerate(lens_u):
            m = groups[gi]
            if len(m) == 0:
                continue
            dp.seq = SequenceInformation(max_len=int(L), su_mass=0.0, obs_mass=0.0, modification_rate=0.5)
            A = round(dp.seq.modification_rate * dp.seq.max_len)  # common.py:55
            r = dp.device_table.explain(q.diff[m], q.thr[m], dp.tolerance, dp.precision, A, cap=args.cap)
            st[m] = r.status
            cnt[m] = r.count
            calls += 1
        return st, cnt, calls

    stages = {}
    engine.profile(True)
    barrier()
    t0 = time.perf_counter()
    c = pipeline.classify(batch.observed, batch.offsets, su_seq, dp, bd)
    barrier()
    stages["classify"] = {"s": tmax(time.perf_counter() - t0), "is_valid_queries": c.n_valid_queries,
                          "is_singleton_queries": c.n_singleton_queries, "rows_kept": int(c.offsets[-1])}
    stages["classify"]["kernels"] = {_native.KERNEL_NAMES.get(k, str(k)): v for k, v in engine.profile_read().items()}

    barrier()
    t0 = time.perf_counter()
    q2 = pipeline.su_diff_queries(c, EXPLANATION_MASSES)
    st2, cnt2, calls2 = explain_grouped(q2)
    barrier()
    stages["su_diffs"] = {"s": tmax(time.perf_counter() - t0), "queries": len(q2.diff), "engine_calls": calls2,
                          "with_candidates": int(((st2 == 2) | (st2 == -2)).sum()),
                          "candidates": int(cnt2[st2 == 2].sum())}
    stages["su_diffs"]["kernels"] = {_native.KERNEL_NAMES.get(k, str(k)): v for k, v in engine.profile_read().items()}

    barrier()
    t0 = time.perf_counter()
    q3 = pipeline.bin_queries(c)
    st3, cnt3, calls3 = explain_grouped(q3)
    barrier()
    stages["bins"] = {"s": tmax(time.perf_counter() - t0), "queries": len(q3.diff), "engine_calls": calls3,
                      "with_candidates": int(((st3 == 2) | (st3 == -2)).sum()),
                      "overflow": int((st3 == -2).sum()), "candidates": int(cnt3[st3 == 2].sum())}
    stages["bins"]["kernels"] = {_native.KERNEL_NAMES.get(k, str(k)): v for k, v in engine.profile_read().items()}
    engine.profile(False)

    # per-spectrum alphabet reduction = a table rebuild (canonical + 3 mods)
    keep = {m.names[0] for m in dp.masses[1:5]} | {m.names[0] for m in dp.masses[-3:]}
    from spectrseqtools_amd.masses import EXPLANATION_MASSES as EM

    dp2 = DynamicProgrammingTable(EM, compression_rate=32, tolerance=MATCHING_THRESHOLD, precision=TOLERANCE,
                                  seq=seq0, engine=engine)
    t0 = time.perf_counter()
    dp2.adapt_individual_modification_rates_by_alphabet_reduction(keep)
    engine.synchronize()
    rebuild_ms = 1e3 * (time.perf_counter() - t0)

    peaks = len(batch.observed)
    total_s = sum(v["s"] for v in stages.values())
    if dist:
        t = torch.tensor([peaks, args.spectra], dtype=torch.int64, device=torch.device("cuda", gpu))
        dist.all_reduce(t)
        peaks_all, spectra_all = (int(x) for x in t.tolist())
    else:
        peaks_all, spectra_all = peaks, args.spectra
    ref_est = (stages["classify"]["is_valid_queries"] / 70e3 +
               (stages["su_diffs"]["queries"] + stages["bins"]["queries"]) / 4.0e3)
    if rank == 0:
        print(json.dumps({
            "workload": "config5: explanation stages of the prediction pipeline (classify_fragments, first "
                        "filter_by_explanation round, skeleton bin queries) over synthetic spectra, full alphabet",
            "n_gpus": world, "spectra": spectra_all, "peaks": peaks_all,
            "stages": stages, "total_s": total_s,
            "spectra_per_s": spectra_all / total_s, "peaks_per_s": peaks_all / total_s,
            "reduction_rebuild_ms": rebuild_ms, "generation_s": gen_s,
            "reference_estimate_s_per_gpu_share": ref_est,
            "reference_estimate_basis": "BASELINE.md single-core rates: is_valid 70k/s, explain 4.0k/s "
                                        "(queries of one GPU's share; 1 core)",
        }), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
