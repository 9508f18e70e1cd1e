"""The synthetic spectra of the config-5 stage tests (one definition, so the
reference-run fixtures of tests/golden/make_synth_golden.py and the GPU / CPU
tests read the same inputs).  TEST INFRASTRUCTURE.

variant -> 48 spectra of 6..14 nucleotides from synthetic.make_spectra:
  full_ladders             every ladder and internal peak, 3 ppm, 20 % noise
  short_fragments_missing  two thirds of the spectra lose their peaks below
                           1300 Da (first bins of 3+ nucleotides, re-queries)
  low_modification_rate    as above at --modification_rate 0.05 (cli.py:35):
                           budgets bind on pair windows (exact mode)
  noise_free               no mass error, no noise peaks: SU differences repeat
                           exactly at different observed masses
  noise_free_exact         noise-free at modification rate 0.05
"""
import numpy as np

VARIANTS = ("full_ladders", "short_fragments_missing", "low_modification_rate", "noise_free", "noise_free_exact")
SEEDS = {"full_ladders": 41, "short_fragments_missing": 43, "noise_free": 53, "noise_free_exact": 59,
         "low_modification_rate": 47}
TAGS = (555.1294, 455.1491)


def variant_inputs(variant, n=48):
    """-> dict(obs, offsets, su_seq, seq_mass, max_len, mod_rate, exact, clean)."""
    from spectrseqtools_amd import pipeline
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, TOLERANCE, build_breakage_dict
    from spectrseqtools_amd.synthetic import make_spectra

    exact = variant in ("low_modification_rate", "noise_free_exact")
    clean = variant.startswith("noise_free")
    b = make_spectra(n, seed=SEEDS[variant], len_range=(6, 14), mod_rate=0.3 if exact else 0.5,
                     ppm=0.0 if clean else 3.0, noise_frac=0.0 if clean else 0.2)
    spec = np.repeat(np.arange(n), np.diff(b.offsets))
    keep = np.ones(len(b.observed), bool)
    if variant in ("short_fragments_missing", "low_modification_rate"):
        keep = (spec % 3 == 0) | (b.observed > 1300.0)
    obs = b.observed[keep]
    offsets = np.concatenate([[0], np.cumsum(np.bincount(spec[keep], minlength=n))])
    bd = build_breakage_dict(*TAGS)
    w_full = [k for k, v in bd.items() if "START_END" in v][0]
    su_seq = b.seq_mass - w_full * TOLERANCE
    min_int = min(EXPLANATION_MASSES.get_column("tolerated_integer_masses").to_list())
    max_len = pipeline.max_len_of(su_seq, TOLERANCE, min_int)  # cli.py:158-170 (every rate > 0)
    return {"obs": obs, "offsets": offsets, "su_seq": su_seq, "seq_mass": b.seq_mass, "max_len": max_len,
            "mod_rate": 0.05 if exact else 0.5, "exact": exact, "clean": clean}
