"""Fragment classification on the GPU engine.

Mirror of spectrseqtools/fragment_classification.py (reference v0.1.2).
classify_fragments (:17-101) keeps the reference's signature, columns, row
order and filters; its two per-row `map_elements` predicates (is_valid_mass
over every fragment x breakage weight, :52-67, and is_singleton over the
valid rows, :70-82) become one engine call each.  classify_fragments_batch
classifies many spectra that share one DP table with one call per predicate
for all of them (the config-5 pipeline harness, tools/pipeline_bench.py).
"""
import numpy as np

from .frame import as_columns, like
from .mass_table import DynamicProgrammingTable

MAX_VARIANCE = 1  # fragment_classification.py:8


def is_singleton(mass, integer_masses, dp_table: DynamicProgrammingTable, threshold=None) -> bool:
    """fragment_classification.py:104-119: some value of the quantised window
    (target = round(mass / precision), threshold default tolerance * mass) is one
    of integer_masses."""
    return bool(is_singletons([mass], integer_masses, dp_table, None if threshold is None else [threshold])[0])


def is_singletons(masses, integer_masses, dp_table: DynamicProgrammingTable, thresholds=None):
    """Batched is_singleton: bool per mass (one engine call)."""
    eng = dp_table.device_table.engine
    out = eng.is_singleton(integer_masses, masses, thresholds, dp_table.tolerance, dp_table.precision)
    return np.asarray(out).astype(bool)


def valid_peaks(observed, breakage_dict, dp_table: DynamicProgrammingTable):
    """is_valid_mass over every peak x breakage weight (:52-67) in one engine
    call reading each peak once (sst_is_valid_peaks): bool[len(dict) * n],
    breakage-major.  Raises the reference's NotImplementedError for the first
    row whose window leaves the table."""
    from .mass_explanation import _not_in_table, first_value_beyond

    obs = np.ascontiguousarray(observed, dtype=np.float64)
    shifts = np.array([w * dp_table.precision for w in breakage_dict], dtype=np.float64)
    out = dp_table.device_table.is_valid_peaks(obs, shifts, dp_table.tolerance, dp_table.precision)
    bad = np.flatnonzero(out < 0)
    if len(bad):
        k, p = divmod(int(bad[0]), len(obs))
        raise NotImplementedError(_not_in_table(first_value_beyond(float(obs[p] - shifts[k]),
                                                                   float(dp_table.tolerance * obs[p]), dp_table)))
    return out.astype(bool)


def _expand(fragment_masses, breakage_dict, precision, intensity_cutoff):
    """Columns of the reference's pl.concat over breakage weights (:26-49):
    fragment_index first, the input columns (intensity added when missing,
    neutral_mass renamed to observed_mass in place), then standard_unit_mass and
    breakage; breakage-major row order."""
    cols = as_columns(fragment_masses)
    n = len(next(iter(cols.values()), []))
    if "intensity" not in cols:
        cols["intensity"] = [intensity_cutoff * 1.1] * n
    if "neutral_mass" in cols:
        cols = {("observed_mass" if k == "neutral_mass" else k): v for k, v in cols.items()}
    cols = {"fragment_index": list(range(n)), **cols}
    obs = np.asarray(cols["observed_mass"], dtype=np.float64)
    out = {k: [] for k in cols}
    su, brk = [], []
    for weight, names in breakage_dict.items():
        for k, v in cols.items():
            out[k] += v
        su.append(obs - (weight * precision))
        brk += [names[0]] * n
    out["standard_unit_mass"] = np.concatenate(su) if su else np.zeros(0)
    out["breakage"] = brk
    return out


def _finish(cols, valid, singleton, dp_table, intensity_cutoff, mass_cutoff):
    """The valid rows with is_singleton, sorted by SU mass, then the intensity,
    mass and sequence-mass filters (:50-95)."""
    keep = np.flatnonzero(valid)
    su = np.asarray(cols["standard_unit_mass"], dtype=np.float64)[keep]
    order = keep[np.argsort(su, kind="stable")]
    sing = np.zeros(len(valid), dtype=bool)
    sing[keep] = singleton
    inten = np.asarray(cols["intensity"], dtype=np.float64)
    obs = np.asarray(cols["observed_mass"], dtype=np.float64)
    order = order[(inten[order] > intensity_cutoff) & (obs[order] < mass_cutoff)]
    su_all = np.asarray(cols["standard_unit_mass"], dtype=np.float64)
    order = order[_sequence_mass_mask(dp_table.seq.su_mass, su_all[order], [cols["breakage"][i] for i in order])]
    out = {}
    for k, v in cols.items():
        vv = v.tolist() if isinstance(v, np.ndarray) else v
        out[k] = [vv[i] for i in order]
    out["is_singleton"] = [bool(sing[i]) for i in order]
    return out


def _sequence_mass_mask(mass_cutoff, su, breakage):
    """filter_by_sequence_mass (:122-139) as a row mask."""
    su = np.asarray(su, dtype=np.float64)
    full = np.array([("START" in b) and ("END" in b) for b in breakage], dtype=bool)
    return (su < mass_cutoff + MAX_VARIANCE) & ((su > mass_cutoff - MAX_VARIANCE) | ~full)


def classify_fragments(fragment_masses, dp_table: DynamicProgrammingTable, breakage_dict: dict, output_file_path=None,
                       intensity_cutoff=0.5e6, mass_cutoff=50000):
    """fragment_classification.py:17-101.  Returns a frame of the input's kind
    (polars, pandas or spectrseqtools_amd.frame.Frame) with the reference's
    columns: fragment_index, the input columns, standard_unit_mass, breakage,
    is_singleton.  Rows whose SU window leaves the DP table raise the
    reference's NotImplementedError (first offending row in frame order)."""
    cols = _expand(fragment_masses, breakage_dict, dp_table.precision, intensity_cutoff)
    su = cols["standard_unit_mass"]
    obs = np.asarray(cols["observed_mass"], dtype=np.float64)
    n = len(obs) // max(1, len(breakage_dict))
    valid = valid_peaks(obs[:n], breakage_dict, dp_table)  # the concat repeats the peaks per weight
    keep = np.flatnonzero(valid)
    singleton = is_singletons(su[keep], [m.mass for m in dp_table.masses], dp_table,
                              thresholds=dp_table.tolerance * obs[keep]) if len(keep) else np.zeros(0, bool)
    out = _finish(cols, valid, singleton, dp_table, intensity_cutoff, mass_cutoff)
    frame = like(fragment_masses, out)
    if output_file_path is not None:
        frame.write_csv(output_file_path, separator="\t")
    return frame


def classify_fragments_batch(spectra, dp_table: DynamicProgrammingTable, breakage_dict: dict, intensity_cutoff=0.5e6,
                             mass_cutoff=50000):
    """classify_fragments over many spectra (fragment frames) that share
    dp_table: one is_valid and one is_singleton engine call for all of them.
    Returns one frame per spectrum, each equal to classify_fragments' output.
    intensity_cutoff may be one value per spectrum."""
    cuts = np.broadcast_to(np.asarray(intensity_cutoff, dtype=np.float64), (len(spectra),))
    parts = [_expand(f, breakage_dict, dp_table.precision, float(c)) for f, c in zip(spectra, cuts)]
    su = np.concatenate([p["standard_unit_mass"] for p in parts]) if parts else np.zeros(0)
    obs = np.concatenate([np.asarray(p["observed_mass"], dtype=np.float64) for p in parts]) if parts else np.zeros(0)
    # one engine call for every spectrum's peaks (each spectrum's rows are
    # breakage-major over its own peaks: regroup the peaks-major answers)
    B = len(breakage_dict)
    peaks = [np.asarray(p["observed_mass"][:len(p["observed_mass"]) // max(1, B)], dtype=np.float64) for p in parts]
    allp = np.concatenate(peaks) if peaks else np.zeros(0)
    v = valid_peaks(allp, breakage_dict, dp_table).reshape(B, len(allp)) if len(allp) else np.zeros((B, 0), bool)
    cuts_p = np.concatenate([[0], np.cumsum([len(x) for x in peaks])]).astype(np.int64)
    valid = np.concatenate([v[:, cuts_p[j]:cuts_p[j + 1]].ravel() for j in range(len(peaks))]) if peaks else \
        np.zeros(0, bool)
    keep = np.flatnonzero(valid)
    singleton = is_singletons(su[keep], [m.mass for m in dp_table.masses], dp_table,
                              thresholds=dp_table.tolerance * obs[keep]) if len(keep) else np.zeros(0, bool)
    sing_all = np.zeros(len(su), dtype=bool)
    sing_all[keep] = singleton
    out, o = [], 0
    for f, p, c in zip(spectra, parts, cuts):
        k = len(p["standard_unit_mass"])
        v = valid[o:o + k]
        out.append(like(f, _finish(p, v, sing_all[o:o + k][v], dp_table, float(c), mass_cutoff)))
        o += k
    return out


def filter_by_sequence_mass(mass_cutoff: float, fragments):
    """fragment_classification.py:122-139."""
    cols = as_columns(fragments)
    mask = _sequence_mass_mask(mass_cutoff, cols["standard_unit_mass"], cols["breakage"])
    idx = np.flatnonzero(mask)
    return like(fragments, {k: [v[i] for i in idx] for k, v in cols.items()})
