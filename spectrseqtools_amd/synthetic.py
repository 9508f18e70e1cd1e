"""Synthetic MS2 spectra for benchmarks and scale tests (SURVEY.md 8(d),
configs 2-4): random RNA sequences over the full alphabet, their terminal
ladders and internal fragments shifted by the breakage weights of
build_breakage_dict, 3 ppm Gaussian mass error and 20 % uniform noise peaks.
There is no public dataset for this path; everything here is seeded.
"""
from dataclasses import dataclass

import numpy as np

from .masses import EXPLANATION_MASSES, PHOSPHATE_LINK_MASS, TOLERANCE, UNMODIFIED_BASES, build_breakage_dict


@dataclass
class SpectrumBatch:
    observed: np.ndarray      # [P] observed neutral masses, spectrum-major
    spectrum: np.ndarray      # [P] spectrum id of each peak
    offsets: np.ndarray       # [S+1] peak ranges per spectrum
    seq_mass: np.ndarray      # [S] observed full-sequence mass (meta sequence_mass)
    lengths: np.ndarray       # [S]


def _nucleotide_masses():
    names = EXPLANATION_MASSES.get_column("nucleoside").to_list()
    mono = np.asarray(EXPLANATION_MASSES.get_column("monoisotopic_mass").to_list(), dtype=np.float64)
    canon = np.array([n in UNMODIFIED_BASES for n in names])
    return mono + PHOSPHATE_LINK_MASS, canon


def make_spectra(n_spectra, seed=1000, len_range=(10, 20), mod_rate=0.5, ppm=3.0, noise_frac=0.2,
                 internal_per_nt=4, tags=(555.1294, 455.1491)):
    rng = np.random.default_rng(seed)
    nt_mass, canon = _nucleotide_masses()
    canon_idx = np.nonzero(canon)[0]
    mod_idx = np.nonzero(~canon)[0]
    brk = build_breakage_dict(*tags)
    w_of = {names[0]: k * TOLERANCE for k, names in brk.items()}
    w_start, w_end, w_full, w_int = w_of["START_c/y"], w_of["c/y_END"], w_of["START_END"], w_of["c/y_c/y"]
    obs_all, spec_all, offsets, seq_masses, lens = [], [], [0], [], []
    for s in range(n_spectra):
        L = int(rng.integers(len_range[0], len_range[1] + 1))
        n_mod = int(rng.integers(0, round(mod_rate * L) + 1))
        seq = rng.choice(canon_idx, L)
        if n_mod:
            seq[rng.choice(L, n_mod, replace=False)] = rng.choice(mod_idx, n_mod)
        m = nt_mass[seq]
        cs = np.concatenate([[0.0], np.cumsum(m)])
        total = cs[-1]
        prefix = cs[1:L] + w_start                       # START-side ladder
        suffix = (total - cs[1:L]) + w_end               # END-side ladder
        full = np.array([total + w_full])
        n_int = internal_per_nt * L
        a = rng.integers(1, L - 1, n_int)
        b = np.minimum(a + rng.integers(1, 8, n_int), L - 1)
        internal = (cs[b] - cs[a]) + w_int
        peaks = np.concatenate([prefix, suffix, full, internal])
        peaks = peaks * (1.0 + rng.normal(0.0, ppm * 1e-6, len(peaks)))
        noise = rng.uniform(300.0, 8000.0, int(noise_frac * len(peaks)))
        peaks = np.concatenate([peaks, noise])
        obs_all.append(peaks)
        spec_all.append(np.full(len(peaks), s, dtype=np.int64))
        offsets.append(offsets[-1] + len(peaks))
        seq_masses.append(float(full[0]))
        lens.append(L)
    return SpectrumBatch(np.concatenate(obs_all), np.concatenate(spec_all), np.asarray(offsets, dtype=np.int64),
                         np.asarray(seq_masses), np.asarray(lens))
