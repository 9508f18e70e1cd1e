"""TEST INFRASTRUCTURE: a CPU stand-in for _native.DeviceTable backed by the
oracle (oracle/sst_oracle.c), so that the host-side mirrors of the
reference's callers (classify_fragments, Predictor, SkeletonBuilder) run in
the CPU suite.  Installed only by tests (monkeypatch of DeviceTable.build);
the product path has no CPU fallback (tests/test_boundary.py)."""
import numpy as np

import _oracle as oracle
from spectrseqtools_amd import _native


class FakeResult:
    def __init__(self, status, sols):
        self.n = len(status)
        self.status = np.asarray(status, dtype=np.int8)
        self.count = np.array([len(s) for s in sols], dtype=np.uint64)
        self._sols = sols

    def candidates(self, i):
        return list(self._sols[i])


class FakeEngine:
    device = -1

    @staticmethod
    def is_singleton(integer_masses, masses, thresholds, tolerance, precision):
        return oracle.is_singleton_batch(masses, thresholds, integer_masses, tolerance, precision).astype(np.int8)


class FakeDeviceTable:
    compression = 32

    def __init__(self, masses, max_mass, compression):
        assert compression == 32
        self.masses = [int(m) for m in masses]
        self.table = oracle.build_table(self.masses, int(max_mass), compression)
        self.n_cols = self.table.shape[1]
        self.engine = FakeEngine()
        self.alph = None
        self.calls = 0

    def set_budgets(self, is_mod, caps):
        self.alph = oracle.Alphabet(self.masses, is_mod, caps)

    def close(self):
        self.table = None

    def is_valid(self, masses, thresholds, tolerance, precision):
        self.calls += 1
        return oracle.is_valid_batch(self.table, 32, masses, thresholds, tolerance, precision=precision)

    def is_valid_peaks(self, observed, shifts, tolerance, precision):
        self.calls += 1
        o = np.asarray(observed, dtype=np.float64)
        su = np.concatenate([o - s for s in shifts]) if len(shifts) else np.zeros(0)
        return oracle.is_valid_batch(self.table, 32, su, tolerance * np.tile(o, len(shifts)), tolerance,
                                     precision=precision)

    # -- per-spectrum reduced alphabets: the oracle on each alphabet's own table
    def _alpha_table(self, mask_row):
        rows = [r for r in range(len(self.masses)) if r == 0 or (int(mask_row[r >> 6]) >> (r & 63)) & 1]
        key = tuple(rows)
        cache = self.__dict__.setdefault("_alpha_cache", {})
        if key not in cache:
            ms = [self.masses[r] for r in rows]
            tab = oracle.build_table(ms, max(ms) * 35, 32)
            caps = None if self.alph is None else [int(self.alph.cap[r]) for r in rows]
            mods = None if self.alph is None else [int(self.alph.is_mod[r]) for r in rows]
            cache[key] = (rows, tab, oracle.Alphabet(ms, mods or [0] * len(ms), caps or [0] * len(ms)))
        return cache[key]

    def pair_records(self):
        """The pair list (sst_table_pair_records' encoding): 1- and 2-item sums
        below 3 w_min by (sum, top row)."""
        ms = self.masses
        wmin = min(m for m in ms if m > 0)
        e = []
        for r1 in range(1, len(ms)):
            e.append((ms[r1], r1, 1 | (r1 << 8)))
            for r2 in range(1, r1 + 1):
                if ms[r1] + ms[r2] < 3 * wmin:
                    e.append((ms[r1] + ms[r2], r1, 2 | (r2 << 8) | (r1 << 16)))
        e.sort(key=lambda x: (x[0], x[1]))
        self._pair_sums = np.array([x[0] for x in e], dtype=np.int64)
        return np.array([x[2] for x in e], dtype=np.uint32)

    def explain_pairs_alpha(self, masses, thresholds, spec, masks, tolerance, precision):
        recs = self.pair_records()
        sums = self._pair_sums
        wmin = min(m for m in self.masses if m > 0)
        n = len(masses)
        st, cnt = np.zeros(n, np.int8), np.zeros(n, np.uint32)
        rm, rg = np.zeros((n, 2), np.uint64), np.zeros((n, 2), np.uint32)
        masks = np.asarray(masks, dtype=np.uint64).reshape(-1, 2)
        for i in range(n):
            rows, tab, alph = self._alpha_table(masks[spec[i]])
            target = int(np.rint(masses[i] / precision))
            th = int(np.ceil(thresholds[i] / precision))
            if target + th >= 3 * wmin:
                st[i] = -10
                continue
            A = round(0.5 * 20)  # pair windows: budgets cannot bind (filter_fixpoint checks)
            s_, sols, n_empty, _ = oracle.explain_table(tab, 32, alph, float(masses[i]), float(thresholds[i]),
                                                        tolerance, A, precision=precision)
            full = [tuple(rows[x] for x in t) for t in sols]
            st[i] = _native.SST_SOME if full else (_native.SST_EMPTY if n_empty else _native.SST_NONE)
            cnt[i] = len(full)
            for t in full:
                for r in t:
                    rm[i, r >> 6] |= np.uint64(1) << np.uint64(r & 63)
            a = max(target - th, 1)
            rg[i] = (np.searchsorted(sums, a), np.searchsorted(sums, target + th, side="right"))
        return st, cnt, rm, rg

    def is_valid_alpha(self, masses, thresholds, offsets, masks, tolerance, precision):
        masks = np.asarray(masks, dtype=np.uint64).reshape(-1, 2)
        out = np.zeros(len(masses), np.int8)
        for g in range(len(offsets) - 1):
            a, b = int(offsets[g]), int(offsets[g + 1])
            if a == b:
                continue
            rows, tab, _ = self._alpha_table(masks[g])
            out[a:b] = oracle.is_valid_batch(tab, 32, masses[a:b], thresholds[a:b], tolerance, precision=precision)
        return out

    def length_bound(self, su_masses, obs_masses, tolerance, precision, max_len, max_mods, direction,
                     exact_only=False):
        out = np.zeros(len(su_masses), np.int64)
        st = np.zeros(len(su_masses), np.int8)
        for i, (su, ob) in enumerate(zip(su_masses, obs_masses)):
            v = oracle.length_bound(self.table, 32, self.alph, su, ob, tolerance, int(max_len), int(max_mods),
                                    direction, precision=precision)
            if v is None:
                st[i] = _native.SST_OUT_OF_TABLE
            else:
                out[i] = v
        return out, st

    def explain(self, masses, thresholds, tolerance, precision, max_mods, with_memo=True, cap=2 ** 32):
        self.calls += 1
        masses = np.asarray(masses, dtype=np.float64)
        A = np.broadcast_to(np.asarray(max_mods, dtype=np.float64), masses.shape)
        st, sols = [], []
        for i, m in enumerate(masses):
            a = "inf" if not np.isfinite(A[i]) else int(A[i])
            t = None if thresholds is None else float(thresholds[i])
            s, rows, n_empty, _ = oracle.explain_table(self.table, 32, self.alph, float(m), t, tolerance, a,
                                                       with_memo=with_memo, precision=precision)
            if s == -1:
                st.append(_native.SST_OUT_OF_TABLE)
                sols.append([])
            elif s == 0:
                st.append(_native.SST_NONE)
                sols.append([])
            elif rows:
                st.append(_native.SST_SOME)
                sols.append(rows)
            else:
                st.append(_native.SST_EMPTY)
                sols.append([])
        return FakeResult(st, sols)


def install(monkeypatch):
    """Route DynamicProgrammingTable's device tables to the oracle."""
    monkeypatch.setattr(_native.DeviceTable, "build",
                        classmethod(lambda cls, masses, max_mass, compression, engine=None:
                                    FakeDeviceTable(masses, max_mass, compression)))
