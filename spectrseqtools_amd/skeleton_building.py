"""Skeleton building's mass-explanation queries, on the GPU engine.

Mirror of spectrseqtools/skeleton_building.py (reference v0.1.2),
SkeletonBuilder restricted to the parts on the hot path: _predict_skeleton
(:114-196) with explain_bin_differences (:372-421) / explain_mass_difference
(:423-440), update_skeleton_for_given_explanations (:442-482), the length
helpers (validate_sequence_length_by_mass :291-313,
select_sequence_length_with_jaccard :315-370 -- its two length bounds are
GPU calls) and the module functions jaccard_index / combine_skeleton_sequences
(:485-520).

The reference explains each bin against the last bin that had explanations,
one explain_mass_with_table call per fragment pair.  Bins depend only on
neighbouring SU-mass differences, so _predict_skeleton computes every bin
first and explains, in one engine call, each bin against the bin before it
(the first bin against mass 0); the sequential walk then uses those answers
and issues another batch only for a bin whose previous bin had no
explanation (the reference then pairs it with an older bin).  Whole-fragment
masses of the first bin and wide differences leave the LDS pair path: these
are the engine's deferred DFS kernels (k_explain_deferred).

select_sequence_length_with_lp / determine_lp_score need the MILP (pulp/CBC),
outside the hot path and absent from this image.  build_skeleton (:26-112)
is mirrored with the length the reference selects when no LP instance can be
built -- determine_lp_score's `except Exception: return np.inf` (:279-286)
for every candidate length, so select_sequence_length_with_lp returns -1 and
the Jaccard selection decides (:52-57) -- which is config 5's MILP-free path.
That path still runs select_sequence_length_with_lp's own steps before the LP
(:198-251): the alphabet reduction, both length bounds, and
combine_skeleton_sequences for every candidate length in [lower, upper],
which raises IndexError for a length above the skeletons' max_len
(:494-512); build_skeleton then raises and predict returns its default.
"""
from dataclasses import dataclass, field
from itertools import chain, groupby
from typing import List, Optional, Set

from .common import Explanation, _wrap, calculate_error_threshold, calculate_explanations
from .fragment_classification import MAX_VARIANCE
from .frame import Frame, as_columns, like
from .mass_explanation import explain_masses
from .mass_table import DynamicProgrammingTable, compute_sequence_length_bound


@dataclass
class SkeletonBuilder:
    explanations: dict  # diff -> explanation list (Predictor.filter_by_explanation); the reference's cache
    dp_table: DynamicProgrammingTable
    engine_calls: int = field(default=0, repr=False)  # batched explain calls made (measurement)

    def build_skeleton(self, fragments, solver_params=None):
        """skeleton_building.py:26-112 on the MILP-free path (module note):
        both sides' skeletons, the Jaccard length, the combined skeleton, and
        the fragments: the START walk's kept rows (min_end / max_end - 1), the
        END walk's kept rows START did not keep (len - min_end / len -
        max_end), the internal rows whose fragment_index no kept terminal row
        has, end indices outside [0, len) clamped to len - 1, sorted by index.
        Raises as the reference does when no length fits (predict then returns
        its default prediction)."""
        if not isinstance(fragments, Frame):
            sk, fr = self.build_skeleton(Frame(as_columns(fragments)), solver_params)
            return sk, like(fragments, fr.to_dict())
        brk = fragments["breakage"]
        start_sk, start_fr = self._predict_skeleton(
            fragments.filter_mask(["START" in b for b in brk]),
            skeleton_seq=[set() for _ in range(self.dp_table.seq.max_len)])
        end_sk, end_fr = self._predict_skeleton(
            fragments.filter_mask(["END" in b for b in brk]),
            skeleton_seq=[set() for _ in range(self.dp_table.seq.max_len)])
        end_sk = end_sk[::-1]
        self._lp_candidates_without_solver(start_skeleton=start_sk, end_skeleton=end_sk)
        seq_len = self.select_sequence_length_with_jaccard(start_skeleton=start_sk, end_skeleton=end_sk)
        skeleton_seq = combine_skeleton_sequences(seq_len=seq_len, start_skeleton=start_sk, end_skeleton=end_sk)
        n = len(skeleton_seq)
        start_idx = set(start_fr["index"])
        end_fr = end_fr.filter_mask([i not in start_idx for i in end_fr["index"]])
        start_fr = start_fr.with_columns(min_end=[x - 1 for x in start_fr["min_end"]],
                                         max_end=[x - 1 for x in start_fr["max_end"]])
        end_fr = end_fr.with_columns(min_end=[n - x for x in end_fr["min_end"]],
                                     max_end=[n - x for x in end_fr["max_end"]])
        terminal = {k: start_fr[k].to_list() + end_fr[k].to_list() for k in fragments.columns}
        term_peaks = set(terminal["fragment_index"])
        internal = fragments.filter_mask([("START" not in b and "END" not in b) and fi not in term_peaks
                                          for b, fi in zip(brk, fragments["fragment_index"])])
        merged = Frame({k: internal[k].to_list() + terminal[k] for k in fragments.columns}).sort("index")

        def clamp(v):
            return [n - 1 if (x < 0 or x >= n) else x for x in v]

        merged = merged.with_columns(min_end=clamp(merged["min_end"]), max_end=clamp(merged["max_end"]))
        return skeleton_seq, merged

    # -- single queries, as the reference -----------------------------------
    def explain_mass_difference(self, diff: float, prev_mass: float, current_mass: float) -> List[Explanation]:
        """skeleton_building.py:423-440."""
        if diff in self.explanations:
            return self.explanations.get(diff, [])
        threshold = calculate_error_threshold(prev_mass, current_mass, self.dp_table.tolerance)
        return calculate_explanations(diff, threshold, self.dp_table)

    def explain_bin_differences(self, prev_bin: list, current_bin: list, fragments) -> List[Explanation]:
        """skeleton_building.py:372-421 (one engine call for the bin pair)."""
        q = self._bin_queries(prev_bin, current_bin, fragments)
        return self._merge_bin(self._answer([q])[0])

    # -- batched queries ----------------------------------------------------
    @staticmethod
    def _bin_queries(prev_bin, current_bin, fragments):
        """The (diff, prev_mass, current_mass) triples of one bin pair, in the
        reference's order (:378-398)."""
        su = fragments["standard_unit_mass"]
        obs = fragments["observed_mass"]
        if prev_bin is None:
            return [(su[i], 0.0, obs[i]) for i in current_bin]
        return [(su[c] - su[p], obs[p], obs[c]) for p in prev_bin for c in current_bin]

    def _answer(self, query_lists):
        """explain_mass_difference for lists of triples: cache hits from
        self.explanations, everything else in one engine call."""
        todo = [(d, calculate_error_threshold(pm, cm, self.dp_table.tolerance))
                for ql in query_lists for (d, pm, cm) in ql if d not in self.explanations]
        res = []
        if todo:
            A = round(self.dp_table.seq.modification_rate * self.dp_table.seq.max_len)  # common.py:55
            res = [_wrap(r.explanations) for r in
                   explain_masses([t[0] for t in todo], self.dp_table, max_modifications=A,
                                  thresholds=[t[1] for t in todo])]
            self.engine_calls += 1
        out, k = [], 0
        for ql in query_lists:
            ans = []
            for (d, _pm, _cm) in ql:
                if d in self.explanations:
                    ans.append(self.explanations.get(d, []))
                else:
                    ans.append(res[k])
                    k += 1
            out.append(ans)
        return out

    @staticmethod
    def _merge_bin(explanations):
        """:400-421: None if every query has none, else the flattened list
        without duplicates (first occurrence kept)."""
        if all(expl is None for expl in explanations):
            return None
        flat = [expl for expl_list in explanations if expl_list is not None for expl in expl_list if expl is not None]
        unique = []
        for expl in flat:
            if expl not in unique:
                unique.append(expl)
        return unique

    def _predict_skeleton(self, fragments, skeleton_seq: Optional[List[Set[str]]] = None):
        """skeleton_building.py:114-196.  `fragments` is sorted by SU mass and
        carries index, standard_unit_mass, observed_mass, min_end, max_end (as
        in Predictor.predict); it is updated in place (min_end / max_end) and
        returned without the rejected rows."""
        if skeleton_seq is None:
            skeleton_seq = [set() for _ in range(self.dp_table.seq.max_len)]
        if not isinstance(fragments, Frame):  # polars / pandas in, the same kind out
            sk, fr = self._predict_skeleton(Frame(as_columns(fragments)), skeleton_seq)
            return sk, like(fragments, fr.to_dict())
        n = len(fragments)
        events, qs = self.speculative_bin_queries(fragments)
        spec = {}
        for b, ans in enumerate(self._answer(qs)):
            spec[(b - 1 if b else None, b)] = ans
        pos = {0}
        last_valid = None  # event id of the last bin with explanations
        invalid = []
        idx_col = fragments["index"]
        e = 0
        for i in range(1, n):
            if len(pos) == 0:  # :132-135
                invalid.append(idx_col[i])
                continue
            if e >= len(events) or events[e][1] != i:
                continue  # fragment i joined the open bin
            members = events[e][0]
            key = (last_valid, e)
            if key not in spec:  # the previous bin had no explanation: pair with an older one
                prev = None if last_valid is None else events[last_valid][0]
                spec[key] = self._answer([self._bin_queries(prev, members, fragments)])[0]
            explanations = self._merge_bin(spec[key])
            if explanations is None:
                invalid.extend(idx_col[k] for k in members)
            else:
                pos, skeleton_seq = self.update_skeleton_for_given_explanations(explanations, pos, skeleton_seq)
                for k in members:
                    fragments[k, "min_end"] = min(pos, default=1)
                    fragments[k, "max_end"] = max(pos, default=0)
                last_valid = e
            e += 1
        bad = set(invalid)
        keep = [k for k in range(n) if idx_col[k] not in bad]
        return skeleton_seq, fragments.take(keep)

    def speculative_bin_queries(self, fragments):
        """The bins _predict_skeleton's loop forms (:131-153) -- they depend on
        neighbouring differences only -- as events (bin members, the fragment
        that closes the bin; a bin never closed is never explained), and each
        bin's queries against the bin before it (the first bin against mass 0)."""
        n = len(fragments)
        su = fragments["standard_unit_mass"]
        obs = fragments["observed_mass"]
        events = []
        current = [0]
        for i in range(1, n):
            diff = su[i] - su[i - 1]
            thr = calculate_error_threshold(obs[i - 1], obs[i], self.dp_table.tolerance)
            if diff <= thr:
                current.append(i)
                if i + 1 < n:
                    continue
            events.append((list(current), i))
            current = [i]
        qs = [self._bin_queries(None if b == 0 else events[b - 1][0], events[b][0], fragments)
              for b in range(len(events))]
        return events, qs

    def update_skeleton_for_given_explanations(self, explanations, pos, skeleton_seq):
        """skeleton_building.py:442-482 (host set logic, unchanged)."""
        next_pos = set()
        for p in pos:
            alphabet_per_expl_len = {
                expl_len: set(chain(*expls))
                for expl_len, expls in groupby(
                    [expl for expl in explanations if 0 <= p + len(expl) - 1 < self.dp_table.seq.max_len], len)
            }
            for expl_len, alphabet in alphabet_per_expl_len.items():
                for i in range(expl_len):
                    possible_nucleotides = skeleton_seq[p + i]
                    if possible_nucleotides.issuperset(alphabet):
                        possible_nucleotides.clear()
                    for j in alphabet:
                        possible_nucleotides.add(j)
            next_pos.update(p + expl_len for expl_len in alphabet_per_expl_len)
        return next_pos, skeleton_seq

    def validate_sequence_length_by_mass(self, start_skeleton, end_skeleton, nuc_masses) -> bool:
        """skeleton_building.py:291-313."""
        min_mass = 0
        max_mass = 0
        for start_nucs, end_nucs in zip(start_skeleton, end_skeleton):
            min_mass += min([nuc_masses[nuc] for nuc in (start_nucs | end_nucs)], default=0)
            max_mass += max([nuc_masses[nuc] for nuc in (start_nucs | end_nucs)], default=0)
        return min_mass - MAX_VARIANCE <= self.dp_table.seq.su_mass <= max_mass + MAX_VARIANCE

    def _lp_candidates_without_solver(self, start_skeleton, end_skeleton):
        """select_sequence_length_with_lp (skeleton_building.py:198-251) where
        no LP instance can be built (determine_lp_score -> np.inf, so it
        returns -1): its alphabet reduction, both bounds, and
        combine_skeleton_sequences per candidate length -- the only step
        that can raise (IndexError past the skeletons' length)."""
        nucleotides = {nuc for skeleton_pos in start_skeleton + end_skeleton for nuc in skeleton_pos}
        self.dp_table.adapt_individual_modification_rates_by_alphabet_reduction(nucleotides)
        min_len = compute_sequence_length_bound(dp_table=self.dp_table, dir="lower")
        max_len = compute_sequence_length_bound(dp_table=self.dp_table, dir="upper")
        for len_cand in range(min_len, max_len + 1):
            combine_skeleton_sequences(seq_len=len_cand, start_skeleton=start_skeleton, end_skeleton=end_skeleton)
        return -1

    def select_sequence_length_with_jaccard(self, start_skeleton, end_skeleton) -> int:
        """skeleton_building.py:315-370 (the two length bounds on the GPU)."""
        nucleotides = {nuc for skeleton_pos in start_skeleton + end_skeleton for nuc in skeleton_pos}
        self.dp_table.adapt_individual_modification_rates_by_alphabet_reduction(nucleotides)
        nucleoside_masses = {mass.names[0]: mass.mass * self.dp_table.precision for mass in self.dp_table.masses[1:]}
        min_len = compute_sequence_length_bound(dp_table=self.dp_table, dir="lower")
        max_len = compute_sequence_length_bound(dp_table=self.dp_table, dir="upper")
        best_len = min_len
        best_val = -1
        for len_cand in range(min_len, max_len + 1):
            value = sum(map(jaccard_index, zip(start_skeleton[:len_cand],
                                               end_skeleton[len(end_skeleton) - len_cand:]))) / len_cand
            if value > best_val and self.validate_sequence_length_by_mass(
                    start_skeleton=start_skeleton[:len_cand], end_skeleton=end_skeleton[len(end_skeleton) - len_cand:],
                    nuc_masses=nucleoside_masses):
                best_val = value
                best_len = len_cand
        if best_val < 0:
            raise Exception("No sequence length fitting the given sequence mass could be estimated.")
        return best_len


def jaccard_index(input) -> float:
    """skeleton_building.py:485-491."""
    if len(input[0]) == 0 or len(input[1]) == 0:
        return 1
    return len(input[0].intersection(input[1])) / len(input[0].union(input[1]))


def combine_skeleton_sequences(seq_len: int, start_skeleton, end_skeleton):
    """skeleton_building.py:494-520."""
    start_skeleton = start_skeleton[:seq_len]
    end_skeleton = end_skeleton[len(end_skeleton) - seq_len:]
    skeleton_seq = [set() for _ in range(seq_len)]
    for i in range(seq_len):
        skeleton_seq[i] = start_skeleton[i].intersection(end_skeleton[i])
        if not skeleton_seq[i]:
            skeleton_seq[i] = start_skeleton[i].union(end_skeleton[i])
    return skeleton_seq
