"""The explanation-collection half of the predictor, on the GPU engine.

Mirror of spectrseqtools/prediction.py (reference v0.1.2), Predictor
(:54-329) restricted to the stages on the mass-explanation hot path:
collect_explanations_per_side (:286-329), collect_diff_explanations_for_su
(:261-284), filter_by_explanation (:170-202) and _reduce_alphabet
(:204-227).  The reference issues one explain_mass_with_table call per
sliding-window pair and one is_valid_mass call per fragment row; here every
stage is one batched engine call (the window pairs of both sides and the
singletons together).  The dict each stage returns has the reference's keys,
insertion order and overwrite semantics; each value is the list
calculate_explanations returns (its order is the reference's set iteration
order, i.e. hash-seed dependent in the reference too).

predict()'s MILP stages -- filter_with_lp() and the final
LinearProgramInstance (linear_program.py: pulp/CBC) -- are outside the hot
path and absent from this image; predict_skeleton_stage() runs predict up to
them (:63-103).
"""
import numpy as np

from .common import calculate_explanations_batch
from .frame import Frame, as_columns, like
from .mass_explanation import is_valid_masses
from .masses import PHOSPHATE_LINK_MASS
from ._native import window_pairs


def _side_mask(breakage, side):
    return np.array([side in b for b in breakage], dtype=bool)


class Predictor:
    def __init__(self, dp_table, explanation_masses):
        self.explanation_masses = explanation_masses
        self.dp_table = dp_table

    # -- query generation ----------------------------------------------------
    def _max_weight(self):
        """prediction.py:287-290."""
        return max(self.explanation_masses.get_column("monoisotopic_mass").to_list()) + PHOSPHATE_LINK_MASS

    def _side_queries(self, su, obs):
        """The sliding window of one side (prediction.py:293-328): (diff,
        threshold) of every pair the reference explains, in its order."""
        su_a = np.asarray(su, dtype=np.float64)
        s, e = window_pairs(su_a, [0, len(su_a)], self._max_weight())  # host-native producer (sst_window_pairs)
        if not len(s):
            return [], np.zeros(0), np.zeros(0)
        ob_a = np.asarray(obs, dtype=np.float64)
        # calculate_error_threshold (common.py:37-44, l1_norm): tolerance * (m1 + m2)
        return [float(x) for x in su_a[e] - su_a[s]], su_a[e] - su_a[s], self.dp_table.tolerance * (ob_a[s] + ob_a[e])

    @staticmethod
    def _fill_side(explanations, keys, results):
        for d, expl in zip(keys, results):  # :322-323
            if expl is not None and len(expl) >= 1:
                explanations[d] = expl
        return explanations

    # -- reference stages ----------------------------------------------------
    def collect_explanations_per_side(self, fragments) -> dict:
        """prediction.py:286-329, one engine call for all window pairs."""
        cols = as_columns(fragments)
        keys, diffs, thr = self._side_queries(cols["standard_unit_mass"], cols["observed_mass"])
        res = calculate_explanations_batch(diffs, thr, self.dp_table) if len(keys) else []
        return self._fill_side({}, keys, res)

    def collect_diff_explanations_for_su(self, fragments) -> dict:
        """prediction.py:261-284: START-side and END-side window pairs and the
        singleton masses in one engine call."""
        cols = as_columns(fragments)
        su = np.asarray(cols["standard_unit_mass"], dtype=np.float64)
        obs = np.asarray(cols["observed_mass"], dtype=np.float64)
        parts = []
        for side in ("START", "END"):
            m = _side_mask(cols["breakage"], side)
            parts.append(self._side_queries(su[m], obs[m]))
        sing = np.flatnonzero(np.asarray(cols["is_singleton"], dtype=bool))
        diffs = np.concatenate([p[1] for p in parts] + [su[sing]])
        thr = np.concatenate([p[2] for p in parts] + [self.dp_table.tolerance * obs[sing]])
        res = calculate_explanations_batch(diffs, thr, self.dp_table) if len(diffs) else []
        n0, n1 = len(parts[0][0]), len(parts[1][0])
        explanations = {**self._fill_side({}, parts[0][0], res[:n0]),
                        **self._fill_side({}, parts[1][0], res[n0:n0 + n1])}
        for k, expl in zip(su[sing].tolist(), res[n0 + n1:]):  # :276-282 (None kept)
            explanations[k] = expl
        return explanations

    def filter_by_explanation(self, fragments):
        """prediction.py:170-202: explain, reduce the alphabet to the observed
        nucleosides, drop fragments that became invalid; until the alphabet is
        stable."""
        old_alphabet_size = -1
        explanations = {}
        while old_alphabet_size != len(self.dp_table.masses):
            old_alphabet_size = len(self.dp_table.masses)
            explanations = self.collect_diff_explanations_for_su(fragments=fragments)
            observed_nucleotides = {
                nuc for expls in explanations.values() if expls is not None for expl in expls for nuc in expl
            }
            fragments = self._reduce_alphabet(observed_nucleotides, fragments)
        return fragments, explanations

    def predict_skeleton_stage(self, fragments, solver_params=None, record=None):
        """Predictor.predict up to its MILP stages (prediction.py:63-103): the
        framing (index, min_end 0, max_end -1), filter_by_explanation,
        SkeletonBuilder.build_skeleton (the MILP-free path, see
        skeleton_building), then _reduce_alphabet on the combined skeleton's
        nucleotides.  Returns (skeleton_seq, fragments), or None where predict
        returns Prediction.default() because build_skeleton raised (:89-94).
        filter_with_lp and the final LinearProgramInstance need pulp/CBC.
        record (a dict, optional) receives build_skeleton's fragments."""
        from .skeleton_building import SkeletonBuilder

        f = Frame(as_columns(fragments)).with_row_index("orig_index").sort("standard_unit_mass")
        f = f.with_row_index("index")
        f = f.with_columns(min_end=[0] * len(f), max_end=[-1] * len(f))
        f, explanations = self.filter_by_explanation(f)
        try:
            skeleton_seq, f = SkeletonBuilder(explanations=explanations, dp_table=self.dp_table).build_skeleton(
                f, solver_params)
        except Exception:  # noqa: BLE001 -- prediction.py:93-94
            return None
        if record is not None:
            record["build_skeleton"] = f
        nucleotides = {nuc for skeleton_pos in skeleton_seq for nuc in skeleton_pos}
        return skeleton_seq, self._reduce_alphabet(nucleotide_list=nucleotides, fragments=f)

    def _reduce_alphabet(self, nucleotide_list, fragments):
        """prediction.py:204-227: alphabet reduction (a GPU table rebuild when
        rows drop) and one is_valid call over the fragment rows."""
        self.dp_table.adapt_individual_modification_rates_by_alphabet_reduction(nucleotide_list)
        cols = as_columns(fragments)
        if not len(cols.get("standard_unit_mass", [])):
            return fragments
        obs = np.asarray(cols["observed_mass"], dtype=np.float64)
        ok = is_valid_masses(cols["standard_unit_mass"], self.dp_table, thresholds=self.dp_table.tolerance * obs)
        idx = np.flatnonzero(ok)
        return like(fragments, {k: [v[i] for i in idx] for k, v in cols.items()})


def collect_diff_explanations_batch(spectra, dp_table, explanation_masses, max_mods=None):
    """collect_diff_explanations_for_su over many spectra (classified fragment
    frames) that share dp_table, in one engine call.  max_mods: the budget per
    spectrum (default round(modification_rate * max_len) of dp_table.seq, as
    calculate_explanations); one dict per spectrum."""
    from .common import _wrap
    from .mass_explanation import explain_masses

    pred = Predictor(dp_table, explanation_masses)
    per, diffs, thrs, budgets = [], [], [], []
    A0 = round(dp_table.seq.modification_rate * dp_table.seq.max_len)
    for j, f in enumerate(spectra):
        cols = as_columns(f)
        su = np.asarray(cols["standard_unit_mass"], dtype=np.float64)
        obs = np.asarray(cols["observed_mass"], dtype=np.float64)
        parts = [pred._side_queries(su[m], obs[m]) for m in
                 (_side_mask(cols["breakage"], "START"), _side_mask(cols["breakage"], "END"))]
        sing = np.flatnonzero(np.asarray(cols["is_singleton"], dtype=bool))
        per.append((parts[0][0], parts[1][0], su[sing].tolist()))
        d = np.concatenate([parts[0][1], parts[1][1], su[sing]])
        diffs.append(d)
        thrs.append(np.concatenate([parts[0][2], parts[1][2], dp_table.tolerance * obs[sing]]))
        budgets.append(np.full(len(d), A0 if max_mods is None else max_mods[j], dtype=np.int64))
    if not per:
        return []
    res = explain_masses(np.concatenate(diffs), dp_table, max_modifications=np.concatenate(budgets),
                         thresholds=np.concatenate(thrs))
    out, o = [], 0
    for k0, k1, ks in per:
        r = [_wrap(x.explanations) for x in res[o:o + len(k0) + len(k1) + len(ks)]]
        o += len(k0) + len(k1) + len(ks)
        e = {**Predictor._fill_side({}, k0, r[:len(k0)]), **Predictor._fill_side({}, k1, r[len(k0):len(k0) + len(k1)])}
        for k, expl in zip(ks, r[len(k0) + len(k1):]):
            e[k] = expl
        out.append(e)
    return out
