"""Debug: the mirror test's three variants in one process (as pytest runs
them), then mismatches of the last one with the bounds of both sides."""
import os
import sys

import numpy as np

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import test_gpu_pipeline_device as T  # noqa: E402
from spectrseqtools_amd import _native, pipeline, pipeline_device as PD  # noqa: E402
from spectrseqtools_amd.mass_table import (DynamicProgrammingTable, SequenceInformation,  # noqa: E402
                                           compute_sequence_length_bound)
from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE, build_breakage_dict  # noqa
from spectrseqtools_amd.synthetic import make_spectra  # noqa: E402

engine = _native.get_engine(0)


def scenario(variant):
    n = 48
    mod_rate = 0.05 if variant == "low_modification_rate" else 0.5
    b = make_spectra(n, seed={"full_ladders": 41, "short_fragments_missing": 43}.get(variant, 47), len_range=(6, 14),
                     mod_rate=0.3 if variant == "low_modification_rate" else 0.5)
    spec = np.repeat(np.arange(n), np.diff(b.offsets))
    keep = np.ones(len(b.observed), bool)
    if variant != "full_ladders":
        keep = (spec % 3 == 0) | (b.observed > 1300.0)
    obs = b.observed[keep]
    offsets = np.concatenate([[0], np.cumsum(np.bincount(spec[keep], minlength=n))])
    bd = build_breakage_dict(555.1294, 455.1491)
    w_full = [k for k, v in bd.items() if "START_END" in v][0]
    su_seq = b.seq_mass - w_full * TOLERANCE
    seq = SequenceInformation(max_len=20, su_mass=float(su_seq[0]), obs_mass=float(b.seq_mass[0]),
                              modification_rate=mod_rate)
    dp = DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=MATCHING_THRESHOLD,
                                 precision=TOLERANCE, seq=seq, engine=engine)
    max_len = pipeline.max_len_of(su_seq, TOLERANCE, min(m.mass for m in dp.masses[1:]))
    rows = PD.classify_device(dp, obs, offsets, su_seq, bd)
    fx = PD.fixpoint_device(dp, rows, max_len)
    bins = PD.bins_device(dp, rows, fx.alpha, max_len=max_len)
    sk = PD.skeleton_device(dp, rows, fx.alpha, max_len, bins=bins)
    ln = PD.length_device(dp, sk, bins.alpha_dev, su_seq, b.seq_mass)
    bad = 0
    import torch
    def mem(tag):
        f, t = torch.cuda.mem_get_info(0)
        print(f"[mem] {variant} {tag}: free {f / 2**30:.1f} GiB of {t / 2**30:.1f}; torch reserved "
              f"{torch.cuda.memory_reserved(0) / 2**30:.1f} GiB, allocated {torch.cuda.memory_allocated(0) / 2**30:.1f}",
              flush=True)
    mem("after device stages")
    for g in range(n):
        if g % 12 == 0:
            mem(f"mirror {g}")
        o = T._mirror_outcome(obs[offsets[g]:offsets[g + 1]], su_seq[g], b.seq_mass[g], max_len[g], engine, mod_rate)
        got_sk = PD.skeleton_frames(dp, rows, sk, g)
        sk_ok = all(got_sk[sd] == o[sd] for sd in ("START", "END"))
        want = o["seq_len"]
        dev = (int(ln.status[g]), int(ln.seq_len[g]))
        ok = (want is None and dev[0] == _native.JAC_NO_LENGTH) or (want == "IndexError" and dev[0] == _native.JAC_INDEX) \
            or (isinstance(want, int) and dev == (0, want))
        if not (ok and sk_ok):
            bad += 1
            seq_g = SequenceInformation(max_len=int(max_len[g]), su_mass=float(su_seq[g]), obs_mass=float(b.seq_mass[g]),
                                        modification_rate=mod_rate)
            dpg = DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=MATCHING_THRESHOLD,
                                          precision=TOLERANCE, seq=seq_g, engine=engine)
            names = {m.mass: m.names[0] for m in dpg.masses[1:]}
            dpg.adapt_individual_modification_rates_by_alphabet_reduction({names[m] for m in o["masses"][1:]})
            import gc; gc.collect()
            lo_h = compute_sequence_length_bound(dpg, "lower")
            up_h = compute_sequence_length_bound(dpg, "upper")
            print("seed", os.environ.get("PYTHONHASHSEED"), variant, "g", g, "skeleton_ok", sk_ok, "mirror", lo_h, up_h,
                  want, "device", int(ln.lower[g]), int(ln.upper[g]), dev, "lb_status", int(ln.lb_status[g]),
                  flush=True)
            print("  START", o["START"]["skeleton"], "\n  END", o["END"]["skeleton"], flush=True)
    print("seed", os.environ.get("PYTHONHASHSEED"), variant, "mismatches", bad, flush=True)
    del rows, fx, bins, sk, ln, dp
    import gc
    gc.collect()
    mem("end")


for v in sys.argv[1:] or ["full_ladders", "short_fragments_missing", "low_modification_rate"]:
    scenario(v)
